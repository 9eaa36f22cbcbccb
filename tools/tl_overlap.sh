set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for mode in graph eager; do for ov in 0 1; do
  timeout -k 10 120 rocprofv3 --kernel-trace -d gpurun_out/tl_${mode}_${ov} -o run --output-format csv -- python3 bench.py --steps 30 --warmup 3 --no-cpu-baseline --stage-timing 0 --mode $mode --overlap-indexer $ov > gpurun_out/tl_${mode}_${ov}.log 2>&1 || exit 1
  echo "== $mode overlap=$ov"; python3 tools/timeline.py gpurun_out/tl_${mode}_${ov} --steps 2
  timeout -k 10 60 python3 bench.py --steps 200 --warmup 10 --no-cpu-baseline --stage-timing 0 --mode $mode --overlap-indexer $ov | python3 -c "import json,sys; d=json.load(sys.stdin); print('untraced', d['ms_per_step'])" || exit 1
done; done
