for R in 4 8 2; do TAG=role$R LIB=$(pwd)/tools/ab/$R/libneo_hip.so bash tools/gpu_pmc_step.sh > gpurun_out/pmcrole_$R.txt 2>&1 || exit 1; done
TAG=full bash tools/gpu_pmc_step.sh > gpurun_out/pmcrole_full.txt 2>&1
