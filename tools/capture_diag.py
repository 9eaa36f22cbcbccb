"""Where does a captured RCCL exchange stop?  (capture_full hangs on a one-rank
communicator.)  Runs one variant per child process with a stack-dumping timeout, printing a marker
before and after every host call, so the log shows whether the host blocks inside the call
(ncclGroupEnd / all_to_all_single), inside capture_end (graph instantiate), or on the device
(replay + synchronize never returns).  The parent stops at the first variant that does not finish.

    python tools/capture_diag.py OUTDIR variant[,variant...]

variants: abi-eager, abi-op[:mode], torch-op[:mode], abi-step[:mode], torch-step[:mode], abi-step2, torch-step2,
abi-step2m, torch-step2m, abi-step2raw[:mode], torch-step2raw[:mode] (raw HIP capture, graph inspected + dumped)
(mode = torch.cuda.graph capture_error_mode: global (default) | thread_local | relaxed)
"""
import faulthandler
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def mark(s):
    print(f"[{time.perf_counter():.3f}] {s}", flush=True)


def child(variant):
    import numpy as np
    import torch
    import torch.distributed as dist
    import dlrm_pkg
    pkg = dlrm_pkg.load()
    name, _, mode = variant.partition(":")
    mode = mode or "global"
    faulthandler.dump_traceback_later(40, exit=False)
    gpu = torch.device("cuda:0")
    torch.cuda.set_device(gpu)
    kind, what = name.split("-")
    if kind == "torch":
        import socket
        sk = socket.socket()
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
        sk.close()
        dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1, device_id=gpu)
        mark("torch pg up")
    T, B, D = 5, 128, 32
    if what in ("eager", "op"):
        send = torch.randn((T * B * D,), device=gpu)
        recv = torch.empty_like(send)
        if kind == "abi":
            from dlrm_jl_amd.comm import CommExchange
            comm = CommExchange(0, 1, gpu)
            mark("comm up")

            def op():
                comm.alltoall_fwd(send, recv, D, B, [T])
        else:
            def op():
                dist.all_to_all_single(recv, send, [T * B * D], [T * B * D])
        op()
        torch.cuda.synchronize()
        mark(f"eager exchange ok: {torch.equal(recv, send)}")
        if what == "eager":
            return
        recv.zero_()
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        g = torch.cuda.CUDAGraph()
        with torch.cuda.stream(s):
            mark(f"capture_begin (mode {mode})")
            g.capture_begin(capture_error_mode=mode)
            mark("in capture: calling the exchange")
            op()
            mark("in capture: exchange call returned")
            g.capture_end()
            mark("capture_end returned (graph instantiated)")
        torch.cuda.current_stream().wait_stream(s)
        torch.cuda.synchronize()
        mark("synced after capture")
        g.replay()
        mark("replay launched")
        torch.cuda.synchronize()
        mark(f"replay synced: equal={torch.equal(recv, send)}")
        return
    # the whole sharded step (tests/test_gpu_parity.py::test_sharded_whole_step_graph_world1)
    from helpers import rand_indices, rand_tables
    from dlrm_jl_amd.sharded import HipShardOps, ShardedHotPath, TablePartition
    rows, D, B, L = [3, 5000, 70, 100000, 11], 32, 128, 1
    T = len(rows)
    rng = np.random.default_rng(23)
    tabs = rand_tables(rng, rows, D)
    idx = pkg.PackedIndices(torch.from_numpy(rand_indices(rng, rows, B, L)).to(torch.int32).reshape(T, B, L).to(gpu))
    x = torch.from_numpy(rng.standard_normal((B, D)).astype(np.float32)).to(gpu)
    F = T + 1
    dout = torch.from_numpy(rng.standard_normal((B, D + F * (F - 1) // 2)).astype(np.float32) * 1e-2).to(gpu)
    ops = HipShardOps([torch.from_numpy(t).to(gpu) for t in tabs], B, L, 0.25, device=gpu)
    micro = 2 if what == "step2" else 1
    if what not in ("step2m", "step2raw", "step2bigstack", "step2fresh"):
        eng = ShardedHotPath(ops, TablePartition(T, 1), 0, B, D, L, torch.float32, gpu, exchange=kind, micro=micro)
        eng.step(x, idx, dout)
        torch.cuda.synchronize()
        mark("eager step ok")
    if what == "step2raw":  # the M = 2 schedule that segfaulted, captured with raw HIP calls
        raw_capture_m2(pkg, eng_args=(ops, TablePartition(T, 1), B, D, L, gpu, kind), x=x, idx=idx, dout=dout,
                       mode=mode)
        return
    if what == "step2fresh":  # exchanges on the second stream(s), one fresh stream per exchange
        raw_capture_m2(pkg, eng_args=(ops, TablePartition(T, 1), B, D, L, gpu, kind), x=x, idx=idx, dout=dout,
                       mode=mode, fresh=True)
        return
    if what == "step2bigstack":  # the same in a thread with a 1 GiB stack (is it a stack overflow?)
        import threading
        threading.stack_size(1 << 30)
        err = []

        def body():
            try:
                raw_capture_m2(pkg, eng_args=(ops, TablePartition(T, 1), B, D, L, gpu, kind), x=x, idx=idx,
                               dout=dout, mode=mode)
            except Exception as e:  # noqa: BLE001
                err.append(e)
        th = threading.Thread(target=body)
        th.start()
        th.join()
        mark(f"big-stack thread done: {err}")
        return
    if what == "step2m":  # M = 2 schedule written out, a marker after every host call
        eng = ShardedHotPath(ops, TablePartition(T, 1), 0, B, D, L, torch.float32, gpu, exchange=kind, micro=2)
        eng.step(x, idx, dout)
        torch.cuda.synchronize()
        mark("eager M=2 step ok")
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        g = torch.cuda.CUDAGraph()
        with torch.cuda.stream(s):
            g.capture_begin(capture_error_mode=mode)
            main, cs = torch.cuda.current_stream(), eng._cstream
            ev_look, ev_recv, ev_bwd, _ = eng._ev
            for m in range(2):
                eng.seg_lookup(idx, m)
                ev_look[m].record(main)
                cs.wait_event(ev_look[m])
                with torch.cuda.stream(cs):
                    mark(f"in capture: exchange_fwd({m}) on the comm stream")
                    eng.exchange_fwd(m)
                    mark(f"in capture: exchange_fwd({m}) returned")
                    ev_recv[m].record(cs)
            for m in range(2):
                main.wait_event(ev_recv[m])
                eng.seg_interact(x, dout, m)
                ev_bwd[m].record(main)
                cs.wait_event(ev_bwd[m])
                with torch.cuda.stream(cs):
                    mark(f"in capture: exchange_bwd({m})")
                    eng.exchange_bwd(m)
                    mark(f"in capture: exchange_bwd({m}) returned")
            main.wait_stream(cs)
            eng.seg_update(idx)
            mark("in capture: all recorded; capture_end")
            g.capture_end()
            mark("capture_end returned")
        torch.cuda.current_stream().wait_stream(s)
        g.replay()
        torch.cuda.synchronize()
        mark("replay synced")
        return
    if micro > 1:  # the engine's own capture, markers around it
        mark(f"capture_full (M = {micro}) begin")
        eng.capture_full(x, [idx], dout)
        mark("capture_full returned")
        eng.step_graphed(0)
        torch.cuda.synchronize()
        mark("replay synced")
        eng.close()
        mark("closed")
        return
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(s):
        mark(f"capture_begin (mode {mode})")
        g.capture_begin(capture_error_mode=mode)
        eng._side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(eng._side):
            eng.seg_index(idx)
            eng._ix_done.record(eng._side)
        mark("in capture: side-stream index build recorded")
        eng.seg_lookup(idx, 0)
        mark("in capture: lookup recorded")
        eng.exchange_fwd(0)
        mark("in capture: forward exchange returned")
        eng.seg_interact(x, dout, 0)
        mark("in capture: interaction recorded")
        eng.exchange_bwd(0)
        mark("in capture: backward exchange returned")
        torch.cuda.current_stream().wait_event(eng._ix_done)
        eng.seg_update(idx)
        mark("in capture: update recorded")
        g.capture_end()
        mark("capture_end returned")
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g.replay()
    mark("replay launched")
    torch.cuda.synchronize()
    mark("replay synced")


NODE_TYPES = {0: "kernel", 1: "memcpy", 2: "memset", 3: "host", 4: "child-graph", 5: "empty", 6: "wait-event",
              7: "event-record", 8: "ext-sem-signal", 9: "ext-sem-wait", 10: "mem-alloc", 11: "mem-free",
              12: "memcpy-from-symbol", 13: "memcpy-to-symbol"}


def raw_capture_m2(pkg, eng_args, x, idx, dout, mode, fresh=False):
    """the M = 2 step with both exchanges on the SECOND (comm) stream, captured with
    hipStreamBeginCapture / hipStreamEndCapture through ctypes instead of torch.cuda.graph, so the
    captured graph can be inspected before it is instantiated: its node types, the nodes with no
    dependency (roots) and no dependent (leaves), which stream each exchange's nodes joined from,
    and a Graphviz dump (hipGraphDebugDotPrint).  Then hipGraphInstantiate, with the library's
    native fatal-signal backtrace armed (dlrm_debug_fatal_trace), so a crash names its frame."""
    import ctypes
    import torch
    from dlrm_jl_amd.sharded import ShardedHotPath
    ops, part, B, D, L, gpu, kind = eng_args
    hip = ctypes.CDLL("libamdhip64.so")
    vp = ctypes.c_void_p
    lib = pkg._lib.load()
    lib.dlrm_debug_fatal_trace(1)
    mark("native fatal-signal backtrace armed")
    eng = ShardedHotPath(ops, part, 0, B, D, L, torch.float32, gpu, exchange=kind, micro=2)
    eng.step(x, idx, dout)
    torch.cuda.synchronize()
    mark("eager M=2 step ok")
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    cmode = {"global": 0, "thread_local": 1, "relaxed": 2}[mode]
    graph = vp()
    with torch.cuda.stream(s):
        main, cs = torch.cuda.current_stream(), eng._cstream
        rc = hip.hipStreamBeginCapture(vp(main.cuda_stream), ctypes.c_int(cmode))
        mark(f"hipStreamBeginCapture rc={rc}")
        ev_look, ev_recv, ev_bwd, _ = eng._ev
        # fresh: every exchange on a stream of its own, forked from the origin stream once and joined
        # once (no stream both waits on the origin and is waited on by it more than one time)
        xs = [torch.cuda.Stream() for _ in range(4)] if fresh else [cs] * 4
        ev_done = [torch.cuda.Event() for _ in range(4)]
        for m in range(2):
            eng.seg_lookup(idx, m)
            ev_look[m].record(main)
            xs[m].wait_event(ev_look[m])
            with torch.cuda.stream(xs[m]):
                eng.exchange_fwd(m)
                ev_recv[m].record(xs[m])
        mark("forward exchanges recorded on the comm stream(s)")
        for m in range(2):
            main.wait_event(ev_recv[m])
            eng.seg_interact(x, dout, m)
            ev_bwd[m].record(main)
            xs[2 + m].wait_event(ev_bwd[m])
            with torch.cuda.stream(xs[2 + m]):
                eng.exchange_bwd(m)
                ev_done[2 + m].record(xs[2 + m])
        mark("backward exchanges recorded on the comm stream(s)")
        if fresh:
            for m in range(2):
                main.wait_event(ev_done[2 + m])
        else:
            main.wait_stream(cs)
        eng.seg_update(idx)
        st = ctypes.c_int(-1)
        hip.hipStreamIsCapturing(vp(cs.cuda_stream), ctypes.byref(st))
        mark(f"comm stream capture status before end: {st.value} (1 = active)")
        lib.dlrm_debug_fatal_trace(2)  # (re-armed last: RCCL / the runtime may have replaced it)
        mark("handlers re-armed; hipStreamEndCapture ...")
        rc = hip.hipStreamEndCapture(vp(main.cuda_stream), ctypes.byref(graph))
        mark(f"hipStreamEndCapture rc={rc} graph={graph.value}")
    n = ctypes.c_size_t(0)
    hip.hipGraphGetNodes(graph, None, ctypes.byref(n))
    nodes = (vp * n.value)()
    hip.hipGraphGetNodes(graph, nodes, ctypes.byref(n))
    hist, roots, leaves = {}, 0, 0
    for i in range(n.value):
        t = ctypes.c_int(-1)
        hip.hipGraphNodeGetType(vp(nodes[i]), ctypes.byref(t))
        name = NODE_TYPES.get(t.value, f"type{t.value}")
        hist[name] = hist.get(name, 0) + 1
        nd = ctypes.c_size_t(0)
        hip.hipGraphNodeGetDependencies(vp(nodes[i]), None, ctypes.byref(nd))
        ndp = ctypes.c_size_t(0)
        hip.hipGraphNodeGetDependentNodes(vp(nodes[i]), None, ctypes.byref(ndp))
        roots += nd.value == 0
        leaves += ndp.value == 0
    mark(f"captured graph: {n.value} nodes {hist}; roots {roots}, leaves {leaves}")
    out = os.environ.get("DIAG_DOT", "/tmp/m2_graph.dot")
    rc = hip.hipGraphDebugDotPrint(graph, out.encode(), ctypes.c_uint(0xffff))
    mark(f"hipGraphDebugDotPrint rc={rc} -> {out}")
    ex = vp()
    mark("hipGraphInstantiate ...")
    rc = hip.hipGraphInstantiate(ctypes.byref(ex), graph, None, None, ctypes.c_size_t(0))
    mark(f"hipGraphInstantiate rc={rc}")
    if rc == 0:
        rc = hip.hipGraphLaunch(ex, vp(torch.cuda.current_stream().cuda_stream))
        torch.cuda.synchronize()
        mark(f"replay rc={rc} synced")
        hip.hipGraphExecDestroy(ex)
    hip.hipGraphDestroy(graph)
    eng.close()
    mark("closed")


def proc_state(pid):
    out = []
    try:
        for tid in sorted(os.listdir(f"/proc/{pid}/task"), key=int):
            def rd(f):
                try:
                    with open(f"/proc/{pid}/task/{tid}/{f}") as fh:
                        return fh.read().strip()
                except Exception as e:
                    return f"?{e.__class__.__name__}"
            comm = rd("comm")
            out.append(f"  tid {tid} {comm:16s} wchan={rd('wchan')} syscall={rd('syscall').split(' ')[0]}")
    except Exception as e:
        out.append(f"  ({e!r})")
    return "\n".join(out)


def main():
    outdir, variants = sys.argv[1], sys.argv[2].split(",")
    os.makedirs(outdir, exist_ok=True)
    for v in variants:
        log = os.path.join(outdir, f"diag_{v.replace(':', '_')}.log")
        env = dict(os.environ, NCCL_DEBUG=os.environ.get("NCCL_DEBUG", "INFO"))
        with open(log, "w") as fh:
            p = subprocess.Popen([sys.executable, "-u", __file__, "--child", v], stdout=fh, stderr=subprocess.STDOUT,
                                 env=env)
            t0 = time.time()
            while p.poll() is None and time.time() - t0 < 60:
                time.sleep(0.5)
            if p.poll() is None:
                st = proc_state(p.pid)
                p.kill()
                p.wait()
                fh.write("\n== TIMEOUT at 60 s; thread states before the kill:\n" + st + "\n")
                print(f"{v}: TIMEOUT (log {log})", flush=True)
                print(st, flush=True)
                sys.exit(3)
            print(f"{v}: rc={p.returncode} ({time.time() - t0:.1f} s)", flush=True)
            if p.returncode != 0:
                sys.exit(4)


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[1] == "--child":
        child(sys.argv[2])
    else:
        main()
