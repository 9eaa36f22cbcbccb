set -o pipefail
echo "== 256-thread indexer, block 2"; DLRM_IX256=1 timeout -k 10 120 bash tools/phase_indexer.sh 2 2>&1 | grep -v warning | tail -4
echo "== 256-thread indexer, block 8 (3 rows)"; DLRM_IX256=1 timeout -k 10 120 bash tools/phase_indexer.sh 8 2>&1 | tail -4
