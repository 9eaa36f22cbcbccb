# round-3: GPU suite, stage times, default bench lines (metric + D=16), kernel trace of the metric bench
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r6i}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1 || { tail -40 $O/gpu_tests.txt; exit 1; }
tail -2 $O/gpu_tests.txt
timeout -k 10 120 python tools/stage_times.py > $O/stage_d128.txt 2>&1 || { tail -20 $O/stage_d128.txt; exit 1; }
grep -v "^{" $O/stage_d128.txt
timeout -k 10 180 python bench.py --no-cpu-baseline > $O/d128.json 2> $O/d128.err || exit 1
python -c "import json; d=json.load(open('$O/d128.json')); print('d128', d['value'], d['sustained']['value'], d['drop_in_chain']['value'], {k: v['us'] for k, v in d['roofline']['stages'].items()})"
timeout -k 10 180 python bench.py --no-cpu-baseline --chain 0 --workload kaggle-d16-b2048 > $O/d16.json 2> $O/d16.err || exit 1
python -c "import json; d=json.load(open('$O/d16.json')); print('d16', d['value'], d['sustained']['value'], {k: v['us'] for k, v in d['roofline']['stages'].items()})"
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/kt -o run --output-format csv -- python3 bench.py --no-cpu-baseline --chain 0 --steps 40 --sustain 0 > $O/kt.log 2>&1 || { tail $O/kt.log; exit 1; }
python3 tools/prof_summary.py --kt $O/kt --workload kaggle-d128-b2048 --out $O/kt_summary > /dev/null && cat $O/kt_summary.md
