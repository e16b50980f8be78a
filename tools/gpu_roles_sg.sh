#!/bin/bash
# Role-masked builds (tools/build_roles.sh <masks>) under step groups: the bench's per-kernel
# HIP-event times (block launch, background slice launch) per build at workload $W (default c5)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=$R/gpurun_out
T=${1:-rsg}; shift
W=${W:-c5}
F="--no-cpu-baseline --no-fft --no-offline --no-host-io --no-parity --steps 128 --warmup 5"
for M in full "$@"; do
  if [ "$M" = full ]; then L=""; else L=$R/tools/ab/$M/libneo_hip.so; fi
  NEO_BENCH_NO_CHECK=1 NEO_HIP_LIBRARY=$L timeout -k 10 200 python bench.py --workload $W $F > $O/rsg_${W}_${M}_$T.json 2> $O/rsg_${W}_${M}_$T.err || { tail -3 $O/rsg_${W}_${M}_$T.err; exit 1; }
  python3 - $O/rsg_${W}_${M}_$T.json $M <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d["roofline"]
ks = " ".join("%s %.2f us" % (k["kernel"], k.get("ms_per_launch", k.get("ms_per_step", 0)) * 1e3) for k in r.get("kernels", []))
print(sys.argv[2], "step %.2f us" % (d["ms_per_step"] * 1e3), ks)
PY
done
