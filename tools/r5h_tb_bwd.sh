# Terabyte rows (bf16 x 128, B=2048): backward shape sweep (samples per block; split vs one wave per sample)
set -e
O=gpurun_out/r5h
mkdir -p $O
for v in "DLRM_BWD_SPB=4" "DLRM_BWD_SPB=2" "DLRM_BWD_SPB=8" "DLRM_BWD_SPLIT=0"; do
  env $v timeout -k 10 300 python -u bench.py --no-cpu-baseline --workload terabyte-d128-bf16-zipf > $O/tb_$v.json 2> $O/tb_$v.err
done
