set -o pipefail
R0=$(pwd)
WL=c4 LIBS="tl tl0" bash tools/gpu_timeline.sh r3c && \
cd /tmp && export TMPDIR=/tmp && \
NEO_HIP_LIBRARY=$R0/tools/ab/tl0/libneo_hip.so timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R0/gpurun_out/prof_tl0 -o run -- python3 $R0/tools/timeline.py --workload c4 --steps 100 > $R0/gpurun_out/prof_tl0.log 2>&1 && \
NEO_HIP_LIBRARY=$R0/tools/ab/tl/libneo_hip.so timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R0/gpurun_out/prof_tl -o run -- python3 $R0/tools/timeline.py --workload c4 --steps 100 > $R0/gpurun_out/prof_tl.log 2>&1 && \
for d in prof_tl0 prof_tl; do f=$(find $R0/gpurun_out/$d -name "*kernel_stats.csv" | head -1); echo "== $d"; grep -i "lvl_step" $f | cut -c1-300; done
