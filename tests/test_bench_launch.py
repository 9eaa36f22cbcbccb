"""bench.py --gpus N without an outside launcher (CPU): one fresh process per rank with
torchrun's environment, started before the parent touches the GPU; the job's exit code is the
first failing rank's."""
import os
import sys
import time

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def test_rank_env_is_torchruns():
    env = bench.rank_env({"KEEP": "1", "RANK": "9"}, 3, 8, 29123)
    assert env["KEEP"] == "1"
    assert (env["RANK"], env["LOCAL_RANK"], env["WORLD_SIZE"], env["LOCAL_WORLD_SIZE"]) == ("3", "3", "8", "8")
    assert (env["MASTER_ADDR"], env["MASTER_PORT"]) == ("127.0.0.1", "29123")


def test_spawn_ranks_gives_each_rank_its_environment(tmp_path):
    code = ("import os, sys; open(os.path.join(sys.argv[1], os.environ['RANK']), 'w').write("
            "' '.join(os.environ[k] for k in ('LOCAL_RANK', 'WORLD_SIZE', 'MASTER_ADDR', 'MASTER_PORT')))")
    rc = bench.spawn_ranks(4, [sys.executable, "-c", code, str(tmp_path)], port=29555)
    assert rc == 0
    got = {p.name: p.read_text().split() for p in tmp_path.iterdir()}
    assert sorted(got) == ["0", "1", "2", "3"]
    for r, (lr, ws, addr, port) in got.items():
        assert (lr, ws, addr, port) == (r, "4", "127.0.0.1", "29555")


def test_spawn_ranks_stops_the_job_when_a_rank_fails():
    # rank 1 fails at once; the others would wait 60 s (as peers blocked in a collective do)
    code = "import os, sys, time; r = int(os.environ['RANK']); sys.exit(3) if r == 1 else time.sleep(60)"
    t0 = time.time()
    rc = bench.spawn_ranks(3, [sys.executable, "-c", code])
    assert rc == 3
    assert time.time() - t0 < 30


def test_main_launches_ranks_before_loading_the_library(monkeypatch):
    calls = []
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    monkeypatch.setenv("DLRM_DIST_BACKEND", "gloo")  # (no GPU count check)
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "2", "--steps", "4"])
    monkeypatch.setattr(bench, "spawn_ranks", lambda n, cmd: calls.append((n, cmd)) or 0)
    monkeypatch.setattr(bench.dlrm_pkg, "load", lambda: calls.append("load"))
    with pytest.raises(SystemExit) as e:
        bench.main()
    assert e.value.code == 0
    assert calls and calls[0][0] == 2 and "load" not in calls
    n, cmd = calls[0]
    assert cmd[-4:] == ["--gpus", "2", "--steps", "4"] and cmd[0] == sys.executable


def test_main_refuses_more_rccl_ranks_than_gpus(monkeypatch):
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    monkeypatch.delenv("DLRM_DIST_BACKEND", raising=False)
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "8"])
    monkeypatch.setattr(bench.torch.cuda, "device_count", lambda: 1)
    monkeypatch.setattr(bench, "spawn_ranks", lambda n, cmd: pytest.fail("must not launch"))
    with pytest.raises(SystemExit) as e:
        bench.main()
    assert "RCCL needs one GPU per rank" in str(e.value.code)
