# forward probe only
set -o pipefail
O=gpurun_out/${1:-r8b}; mkdir -p $O
timeout -k 10 200 tools/bin/fwd_probe > $O/fwd_probe.txt 2>&1 || { tail -20 $O/fwd_probe.txt; exit 1; }
cat $O/fwd_probe.txt
