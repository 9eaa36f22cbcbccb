# 8-part in-apply build for <= 256-B rows: GPU suite, then Terabyte-rows and metric bench at the new defaults
set -e
O=gpurun_out/r5e
mkdir -p $O
timeout -k 10 480 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.txt 2>&1
timeout -k 10 300 python -u bench.py --no-cpu-baseline --workload terabyte-d128-bf16-zipf > $O/tb.json 2> $O/tb.err
timeout -k 10 300 python -u bench.py --no-cpu-baseline --workload kaggle-d16-b2048 > $O/d16.json 2> $O/d16.err
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $O/d128.json 2> $O/d128.err
