#!/bin/bash
# Diagnostic build with per-workgroup timeline records in the step kernel (NEO_TIMELINE;
# tools/timeline.py reads them): tools/ab/tl/libneo_hip.so. Extra flags in $@ (e.g. -DNEO_ROLES=...).
set -e
cd "$(dirname "$0")/../neo-dsp_amd"
make -s -j8
F="-O3 -std=c++20 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-result -fvisibility=hidden -ffp-contract=on"
D=../tools/ab/${TL_NAME:-tl}
mkdir -p $D
/opt/rocm/bin/hipcc $F -DNEO_TIMELINE "$@" -c csrc/upols_levels.hip -o $D/upols_levels.o
objs=$(ls build/*.o | grep -v upols_levels)
/opt/rocm/bin/hipcc $F -shared -o $D/libneo_hip.so $objs $D/upols_levels.o
