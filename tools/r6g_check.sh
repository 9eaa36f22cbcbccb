# round-3: forward probe (TabPtrs / defer knobs), GPU suite, stage times, bench at both indexer placements
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r6g}
mkdir -p $O
timeout -k 10 200 tools/bin/fwd_probe > $O/fwd_probe.txt 2>&1 || { tail -20 $O/fwd_probe.txt; exit 1; }
grep -i "body\|LIBRARY" $O/fwd_probe.txt
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1 || { tail -40 $O/gpu_tests.txt; exit 1; }
tail -2 $O/gpu_tests.txt
timeout -k 10 120 python tools/stage_times.py > $O/stage_d128.txt 2>&1 || { tail -20 $O/stage_d128.txt; exit 1; }
grep -v "^{" $O/stage_d128.txt
for p in 0 2; do timeout -k 10 180 python bench.py --no-cpu-baseline --chain 0 --pipeline $p > $O/d128_p$p.json 2> $O/d128_p$p.err || exit 1; python -c "import json; d=json.load(open('$O/d128_p$p.json')); print($p, d['value'], d['sustained']['value'], {k: v['us'] for k, v in d['roofline']['stages'].items()})"; done
for p in 2; do timeout -k 10 180 python bench.py --no-cpu-baseline --chain 0 --workload kaggle-d16-b2048 --pipeline $p > $O/d16_p$p.json 2> $O/d16_p$p.err || exit 1; python -c "import json; d=json.load(open('$O/d16_p$p.json')); print('d16', $p, d['value'], d['sustained']['value'], {k: v['us'] for k, v in d['roofline']['stages'].items()})"; done
