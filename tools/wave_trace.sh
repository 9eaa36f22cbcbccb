#!/bin/bash
# Builds the wave-timestamped library variant (-DDLRM_WTRACE) into /tmp and runs
# tools/wave_trace.py with it.  usage: [DLRM_WT_D=16] tools/wave_trace.sh [args for wave_trace.py]
set -e
D=dlrm.jl_amd/csrc
SRCS=$(sed -n 's/^SRCS := //p' $D/Makefile)
mkdir -p /tmp/dlrm_wt
for f in $SRCS; do
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=fast -DDLRM_WTRACE -x hip -c $D/$f -o /tmp/dlrm_wt/$f.o &
done
wait
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o /tmp/dlrm_wt/libdlrm_hip.so /tmp/dlrm_wt/*.o \
  -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
DLRM_HIP_LIB=/tmp/dlrm_wt/libdlrm_hip.so python3 tools/wave_trace.py "$@"
