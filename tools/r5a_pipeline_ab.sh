set -e
mkdir -p gpurun_out/r5a
for p in 0 1; do timeout -k 10 240 python bench.py --no-cpu-baseline --pipeline $p > gpurun_out/r5a/d128_p$p.json 2> gpurun_out/r5a/d128_p$p.err; done
for p in 2 1; do timeout -k 10 240 python bench.py --no-cpu-baseline --workload kaggle-d16-b2048 --pipeline $p > gpurun_out/r5a/d16_p$p.json 2> gpurun_out/r5a/d16_p$p.err; done
