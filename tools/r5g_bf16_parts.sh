# configs[2] (bf16, B=8192): side-stream parts build at 4 vs 8 parts per table, same box
set -e
O=gpurun_out/r5g
mkdir -p $O
for p in 4 8; do
  DLRM_BUILD_PARTS=$p timeout -k 10 300 python -u bench.py --no-cpu-baseline --workload kaggle-d128-b8192-bf16 > $O/bf16_parts$p.json 2> $O/bf16_parts$p.err
done
