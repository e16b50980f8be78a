#!/bin/bash
# Diagnostic builds of libneo_hip.so with only some roles of the step kernel (k_lvl_step)
# enabled (NEO_ROLES bit mask: 1 block, 2 Toeplitz T <= 16, 4 Toeplitz 32, 8 far phase 1, 16 far phase 2), for timing the
# roles apart on the GPU (results of a partial build are wrong): tools/ab/<mask>/libneo_hip.so
set -e
cd "$(dirname "$0")/../neo-dsp_amd"
make -s -j8
F="-O3 -std=c++20 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-result -fvisibility=hidden"
for R in "$@"; do
  mkdir -p ../tools/ab/$R
  /opt/rocm/bin/hipcc $F -DNEO_ROLES=$R -c csrc/upols_levels.hip -o ../tools/ab/$R/upols_levels.o &
done
wait
for R in "$@"; do
  objs=$(ls build/*.o | grep -v upols_levels)
  /opt/rocm/bin/hipcc $F -shared -o ../tools/ab/$R/libneo_hip.so $objs ../tools/ab/$R/upols_levels.o
done
