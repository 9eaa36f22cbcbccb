# rocprofv3 kernel-trace + FETCH/WRITE/MFMA passes of four bench workloads at one HEAD
set -o pipefail
for WL in kaggle-d128-b2048 kaggle-d16-b2048 kaggle-d128-b8192-bf16 pooled-64x256-l10; do
  DLRM_HEAD=c5f4fff bash tools/profile.sh r6n $WL --chain 0 || exit 1
  echo "== $WL"; cat gpurun_out/prof_r6n_$WL/r6n_$WL.md
done
