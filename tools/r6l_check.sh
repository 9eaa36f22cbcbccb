# sharded step schedule: M=1 on one stream (plus the side-stream index build); sim step + host time
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r6l}
mkdir -p $O
for m in 1 2; do
  timeout -k 10 120 python tools/shard_sim.py --micro $m > $O/ss_m$m.json 2> $O/ss_m$m.err || { tail $O/ss_m$m.err; exit 1; }
  cat $O/ss_m$m.json
done
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "sharded or comm" > $O/gpu_tests.txt 2>&1 || { tail -40 $O/gpu_tests.txt; exit 1; }
tail -2 $O/gpu_tests.txt
