#!/bin/bash
# repeated short benches (the driver's flags): wall vs GPU-event time per step
set -o pipefail
for i in 1 2 3; do
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-fft --no-offline > gpurun_out/rep_$i.json 2> gpurun_out/rep_$i.err || exit 1
  python -c "import json;r=json.load(open('gpurun_out/rep_$i.json'));print('$i', r['value'], r['ms_per_step'], r['gpu_ms_per_step'])"
done
