# Terabyte rows (bf16, B=2048): indexer in the forward (0) vs in the previous apply (2), same box
set -e
O=gpurun_out/r5c
mkdir -p $O
for p in 2 0; do
  timeout -k 10 420 python -u bench.py --no-cpu-baseline --workload terabyte-d128-bf16-zipf --pipeline $p > $O/tb_p$p.json 2> $O/tb_p$p.err
done
