# BASELINE configs at HEAD, one MI355X (no CPU baseline: the metric config's is in r5_bench_kaggle-d128-b2048.json)
set -e
O=gpurun_out/r5b
mkdir -p $O
for w in kaggle-d16-b2048 kaggle-d128-b8192-bf16 pooled-64x256-l10 terabyte-d128-bf16-zipf; do
  timeout -k 10 420 python -u bench.py --no-cpu-baseline --workload $w > $O/bench_$w.json 2> $O/bench_$w.err
done
