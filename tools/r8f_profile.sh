# rocprofv3 kernel-trace + FETCH/WRITE/MFMA passes of the metric config at HEAD (16-B forward output
# stores), then the default bench line (CPU baseline + drop-in chain)
set -o pipefail
export TMPDIR=/tmp
DLRM_HEAD=766126d bash tools/profile.sh r8f kaggle-d128-b2048 --chain 0 || exit 1
cat gpurun_out/prof_r8f_kaggle-d128-b2048/r8f_kaggle-d128-b2048.md
timeout -k 10 400 python bench.py > gpurun_out/r8f_bench.json 2> gpurun_out/r8f_bench.err || { tail gpurun_out/r8f_bench.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/r8f_bench.json')); print(round(d['value']/1e6,3), d['ms_per_step'], d.get('sustained',{}).get('value'), {k: v['us'] for k, v in d['roofline']['stages'].items()}, d.get('drop_in_chain',{}).get('value'), d['cpu_baseline'])"
