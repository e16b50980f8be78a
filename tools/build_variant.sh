#!/bin/bash
# A variant build of libneo_hip.so: tools/ab/<name>/libneo_hip.so with extra hipcc flags on one
# source (SRC, default upols_levels; e.g. -DNEO_STEP_WPE=3, SRC=upols_group -DNEO_GROUP_PROBE),
# the other objects from the current build.
set -e
N=$1; shift
S=${SRC:-upols_levels}
cd "$(dirname "$0")/../neo-dsp_amd"
make -s -j8
F="-O3 -std=c++20 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-result -fvisibility=hidden -ffp-contract=on"
mkdir -p ../tools/ab/$N
/opt/rocm/bin/hipcc $F "$@" -c csrc/$S.hip -o ../tools/ab/$N/$S.o
objs=$(ls build/*.o | grep -v "/$S.o")
/opt/rocm/bin/hipcc $F -shared -o ../tools/ab/$N/libneo_hip.so $objs ../tools/ab/$N/$S.o
rm -f ../tools/ab/$N/$S.o
