# round-2 re-entry check at HEAD: GPU parity suite, smoke, indexer-pipeline A/B, default bench, rocprof summary
set -e
export TMPDIR=/tmp
O=gpurun_out/r5
mkdir -p $O
timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.txt 2>&1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.txt 2>&1
for p in 0 1; do timeout -k 10 180 python bench.py --no-cpu-baseline --pipeline $p > $O/d128_p$p.json 2> $O/d128_p$p.err; done
for p in 2 1; do timeout -k 10 180 python bench.py --no-cpu-baseline --workload kaggle-d16-b2048 --pipeline $p > $O/d16_p$p.json 2> $O/d16_p$p.err; done
timeout -k 10 240 python bench.py > $O/bench_default.json 2> $O/bench_default.err
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 bench.py --no-cpu-baseline > $O/bench_prof.json 2> $O/bench_prof.err
