source tools/gpu_steps.sh
export TMPDIR=/tmp
step kt35 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider
step pk35 120 rocprofv3 --kernel-trace --stats -d gpurun_out/pk35 -o run -- python tools/payload_kernels.py --reps 30
PROF_DIR=gpurun_out/prof35 step prof35 300 bash tools/prof_served.sh 300
step b35_short1 300 python bench.py --gpus 1 --steps 20 --warmup 5
step b35_short2 300 python bench.py --gpus 1 --steps 20 --warmup 5
