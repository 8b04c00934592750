# Round 2: host time per HIP runtime call in the kernel broker (served path)
source tools/gpu_steps.sh
export TMPDIR=/tmp
PROF_FLAGS="--hip-runtime-trace --marker-trace" PROF_DIR=gpurun_out/prof_api step prof_api 300 bash tools/prof_served.sh 300
