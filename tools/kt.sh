#!/bin/bash
# Quick per-kernel stats (rocprofv3 --kernel-trace --stats) of one bench run.
#   usage: tools/kt.sh NAME [bench args]
set -o pipefail
export TMPDIR=/tmp
N=${1:?name}; shift
O=gpurun_out/kt_$N
rm -rf "$O"; mkdir -p "$O"
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$O" -o run --output-format csv -- python3 bench.py --steps 40 --warmup 5 --no-cpu-baseline "$@" > "$O/log" 2>&1 || { tail -n 20 "$O/log"; exit 1; }
python3 tools/prof_summary.py --kt "$O" --out "$O/sum" > /dev/null && cat "$O/sum.md"
