#!/bin/bash
# Builds the phase-timestamped library variant (-DDLRM_PHASE=<block>) into /tmp and runs
# tools/phase_indexer.py with it.  usage: tools/phase_indexer.sh [block]
set -e
BLK=${1:-2}
D=dlrm.jl_amd/csrc
mkdir -p /tmp/dlrm_phase
for f in abi.cpp lookup.hip interact.hip update.hip hashindex.hip; do
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=fast -DDLRM_PHASE=$BLK -x hip -c $D/$f -o /tmp/dlrm_phase/$f.o &
done
wait
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o /tmp/dlrm_phase/libdlrm_hip.so /tmp/dlrm_phase/*.o
DLRM_HIP_LIB=/tmp/dlrm_phase/libdlrm_hip.so python3 tools/${PHASE_SCRIPT:-phase_indexer.py}
