#!/bin/bash
# repeated short benches (the driver's flags): wall vs GPU-event time per step and the host's
# enqueue time, spin-wait on / off
set -o pipefail
show() { python -c "import json,sys;r=json.load(open('gpurun_out/rep.json'));print(sys.argv[1], round(r['value']), r['ms_per_step'], r['gpu_ms_per_step'], r['host_launch_ms'])" "$1"; }
for v in 1 0 1 0; do
  NEO_BENCH_SPIN=$v timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-fft --no-offline > gpurun_out/rep.json 2> gpurun_out/rep.err || { tail -5 gpurun_out/rep.err; exit 1; }
  show "spin=$v"
done
timeout -k 10 200 python bench.py --steps 128 --warmup 5 --no-cpu-baseline --no-fft --no-offline > gpurun_out/rep.json 2> gpurun_out/rep.err && show "steps128"
