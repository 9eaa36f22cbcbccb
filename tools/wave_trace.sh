#!/bin/bash
# Builds the wave-timestamped library variant (-DDLRM_WTRACE) into /tmp and runs
# tools/wave_trace.py with it.  usage: tools/wave_trace.sh [args for wave_trace.py]
set -e
D=dlrm.jl_amd/csrc
mkdir -p /tmp/dlrm_wt
for f in abi.cpp lookup.hip interact.hip update.hip hashindex.hip; do
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=fast -DDLRM_WTRACE -x hip -c $D/$f -o /tmp/dlrm_wt/$f.o &
done
wait
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o /tmp/dlrm_wt/libdlrm_hip.so /tmp/dlrm_wt/*.o
DLRM_HIP_LIB=/tmp/dlrm_wt/libdlrm_hip.so python3 tools/wave_trace.py "$@"
