# rocprofv3 kernel-trace + FETCH/WRITE/MFMA passes at d704747: bf16 B=8192 (plain dt stores), pooled, Terabyte rows
set -o pipefail
for WL in kaggle-d128-b8192-bf16 pooled-64x256-l10 terabyte-d128-bf16-zipf; do
  DLRM_HEAD=d704747 bash tools/profile.sh r7b $WL --chain 0 || exit 1
  echo "== $WL"; cat gpurun_out/prof_r7b_$WL/r7b_$WL.md
done
