#!/bin/bash
# Builds libdlrm_hip.so from a git revision's sources into DIR, for A/B timing against the working
# tree (DLRM_HIP_LIB=DIR/libdlrm_hip.so python tools/stage_times.py).  usage: tools/ab_build.sh REV DIR
set -e
REV=${1:?rev}; DIR=${2:?dir}
rm -rf "$DIR"; mkdir -p "$DIR/r/pkg/csrc" "$DIR/r/include"
for f in abi.cpp lookup.hip interact.hip update.hip hashindex.hip common.hpp indexer.hpp; do
  git show "$REV:dlrm.jl_amd/csrc/$f" > "$DIR/r/pkg/csrc/$f" 2>/dev/null || rm -f "$DIR/r/pkg/csrc/$f"
done
git show "$REV:include/dlrm_hip.h" > "$DIR/r/include/dlrm_hip.h"
cd "$DIR/r/pkg/csrc"
for f in abi.cpp lookup.hip interact.hip update.hip hashindex.hip; do
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=fast -x hip -c $f -o $f.o &
done
wait
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o "$DIR/libdlrm_hip.so" *.o
