# Terabyte rows (bf16, B=2048), in-apply indexer build: parts per table 2 / 4 / 8, same box
set -e
O=gpurun_out/r5d
mkdir -p $O
for p in 4 8 2; do
  DLRM_STEP_PARTS=$p timeout -k 10 420 python -u bench.py --no-cpu-baseline --workload terabyte-d128-bf16-zipf --pipeline 2 > $O/tb_parts$p.json 2> $O/tb_parts$p.err
done
