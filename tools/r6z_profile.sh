# rocprofv3 kernel-trace + FETCH/WRITE/MFMA passes of the BASELINE configs at one HEAD (part $1: a / b)
set -o pipefail
case "$1" in
  a) WLS="kaggle-d128-b2048 kaggle-d16-b2048 kaggle-d128-b8192-bf16" ;;
  b) WLS="pooled-64x256-l10 terabyte-d128-bf16-zipf" ;;
esac
for WL in $WLS; do
  DLRM_HEAD=d714b6c bash tools/profile.sh r6z $WL --chain 0 || exit 1
  echo "== $WL"; cat gpurun_out/prof_r6z_$WL/r6z_$WL.md
done
