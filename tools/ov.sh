set -o pipefail
for mode in graph eager; do for ov in 0 1; do
  timeout -k 10 60 python3 bench.py --steps 400 --warmup 20 --no-cpu-baseline --stage-timing 0 --mode $mode --overlap-indexer $ov | python3 -c "import json,sys; d=json.load(sys.stdin); print('$mode ov=$ov', d['ms_per_step'], d['value'])" || exit 1
done; done
export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace -d gpurun_out/tl_ov -o run --output-format csv -- python3 bench.py --steps 30 --warmup 3 --no-cpu-baseline --stage-timing 0 --mode eager --overlap-indexer 1 > /dev/null 2>&1 && python3 tools/timeline.py gpurun_out/tl_ov --steps 2
