#!/bin/bash
# rocprofv3 evidence for one workload (run on the GPU box from the repo root):
#   pass 1: --kernel-trace --stats  (per-kernel average duration)
#   pass 2: --pmc FETCH_SIZE        (own run, per MI355X_MICROARCH.md §HBM)
#   pass 3: --pmc WRITE_SIZE        (own run)
#   pass 4: --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE  (own run: MFMA busy fraction)
# then tools/prof_summary.py -> profiles/<tag>_<workload>.{json,md} and profiles/pmc_<workload>.json
# (the latter feeds bench.py's roofline.traffic).
#   usage: tools/profile.sh TAG WORKLOAD [extra bench args]
set -o pipefail
TAG=${1:?tag}; WL=${2:?workload}; shift 2
export TMPDIR=/tmp
O=gpurun_out/prof_${TAG}_${WL}
rm -rf "$O"; mkdir -p "$O"
B="--workload $WL --steps 40 --warmup 5 --no-cpu-baseline --sustain 0 $*"
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$O/kt" -o run --output-format csv -- python3 bench.py $B > "$O/kt.log" 2>&1 || { echo "kt pass failed"; tail -n 20 "$O/kt.log"; exit 1; }
timeout -k 10 240 rocprofv3 --pmc FETCH_SIZE -d "$O/fetch" -o run --output-format csv -- python3 bench.py $B > "$O/fetch.log" 2>&1 || { echo "fetch pass failed"; tail -n 20 "$O/fetch.log"; exit 1; }
timeout -k 10 240 rocprofv3 --pmc WRITE_SIZE -d "$O/write" -o run --output-format csv -- python3 bench.py $B > "$O/write.log" 2>&1 || { echo "write pass failed"; tail -n 20 "$O/write.log"; exit 1; }
timeout -k 10 240 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE -d "$O/mfma" -o run --output-format csv -- python3 bench.py $B > "$O/mfma.log" 2>&1 || { echo "mfma pass failed"; tail -n 20 "$O/mfma.log"; exit 1; }
python3 tools/prof_summary.py --kt "$O/kt" --fetch "$O/fetch" --write "$O/write" --mfma "$O/mfma" --workload "$WL" --head "${DLRM_HEAD:-unknown}" --out "$O/${TAG}_${WL}" || exit 1
cp "$(find "$O/kt" -name '*kernel_stats.csv' | head -n 1)" "$O/${TAG}_${WL}_kernel_stats.csv"
cp "$O/${TAG}_${WL}.json" "$O/pmc_${WL}.json"
# the raw traces stay on the box (gpurun copies back at most 64 MiB)
rm -rf "$O/kt" "$O/fetch" "$O/write" "$O/mfma"
