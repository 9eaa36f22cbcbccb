#!/bin/bash
# Builds a variant of libdlrm_hip.so with extra compile flags (e.g. -DDLRM_WTRACE, -DDLRM_PHASE=3)
# into DIR (in-tree, so it travels to the GPU box).  usage: tools/build_variant.sh DIR FLAGS...
set -e
DIR=${1:?dir}; shift
D=dlrm.jl_amd/csrc
mkdir -p "$DIR"
SRCS="abi.cpp lookup.hip interact.hip update.hip hashindex.hip dense.hip dac.hip slice.hip comm.cpp"
for f in $SRCS; do
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=fast "$@" -x hip -c $D/$f -o "$DIR/$f.o" &
done
wait
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o "$DIR/libdlrm_hip.so" "$DIR"/*.o -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
rm -f "$DIR"/*.o
