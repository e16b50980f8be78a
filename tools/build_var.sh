#!/bin/bash
# diagnostic build of libneo_hip.so with extra -D flags for upols_levels.hip: tools/ab/<name>/
# usage: tools/build_var.sh <name> -DFLAG ...
set -e
N=$1; shift
cd "$(dirname "$0")/../neo-dsp_amd"
make -s -j8
F="-O3 -std=c++20 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-result -fvisibility=hidden"
mkdir -p ../tools/ab/$N
/opt/rocm/bin/hipcc $F "$@" -c csrc/upols_levels.hip -o ../tools/ab/$N/upols_levels.o
/opt/rocm/bin/hipcc $F -shared -o ../tools/ab/$N/libneo_hip.so $(ls build/*.o | grep -v upols_levels) ../tools/ab/$N/upols_levels.o
