# HIP graph runtime knobs: does the side-stream branch of a replayed graph overlap?
set -o pipefail
O=gpurun_out/r6p; mkdir -p $O
run() {  # name, env..., workload
  local n=$1; shift; local wl=$1; shift
  env "$@" timeout -k 10 240 python bench.py --no-cpu-baseline --chain 0 --workload $wl > $O/$n.json 2> $O/$n.err || { tail $O/$n.err; return 1; }
  python -c "import json; d=json.load(open('$O/$n.json')); print('$n', round(d['value']/1e6,2), d['ms_per_step'], {k: v['us'] for k, v in d['roofline']['stages'].items()})"
}
run bf16_base kaggle-d128-b8192-bf16 X=1 &&
run bf16_nopc kaggle-d128-b8192-bf16 DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 &&
run bf16_q2 kaggle-d128-b8192-bf16 DEBUG_HIP_FORCE_GRAPH_QUEUES=2 &&
run bf16_nopc_q2 kaggle-d128-b8192-bf16 DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 DEBUG_HIP_FORCE_GRAPH_QUEUES=2 &&
run d128_base kaggle-d128-b2048 X=1 &&
run d128_nopc kaggle-d128-b2048 DEBUG_CLR_GRAPH_PACKET_CAPTURE=0
