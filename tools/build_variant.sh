#!/bin/bash
# A variant build of libneo_hip.so: tools/ab/<name>/libneo_hip.so with extra hipcc flags on
# upols_levels.hip (e.g. -DNEO_STEP_WPE=3), the other objects from the current build.
set -e
N=$1; shift
cd "$(dirname "$0")/../neo-dsp_amd"
make -s -j8
F="-O3 -std=c++20 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-result -fvisibility=hidden"
mkdir -p ../tools/ab/$N
/opt/rocm/bin/hipcc $F "$@" -c csrc/upols_levels.hip -o ../tools/ab/$N/upols_levels.o
objs=$(ls build/*.o | grep -v upols_levels)
/opt/rocm/bin/hipcc $F -shared -o ../tools/ab/$N/libneo_hip.so $objs ../tools/ab/$N/upols_levels.o
rm -f ../tools/ab/$N/upols_levels.o
