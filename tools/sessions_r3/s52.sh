source tools/gpu_steps.sh
export TMPDIR=/tmp
step kt52 400 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider
step pk52 150 rocprofv3 --kernel-trace --stats -d gpurun_out/pk52 -o run -- python tools/payload_kernels.py --reps 30
BK_REDUCE_BLOCKS=4096 step pk52_r4096 150 rocprofv3 --kernel-trace --stats -d gpurun_out/pk52_r4096 -o run -- python tools/payload_kernels.py --reps 30
BK_REDUCE_BLOCKS=16384 step pk52_r16384 150 rocprofv3 --kernel-trace --stats -d gpurun_out/pk52_r16384 -o run -- python tools/payload_kernels.py --reps 30
step b52_short1 300 python bench.py --gpus 1 --steps 20 --warmup 5
step b52_short2 300 python bench.py --gpus 1 --steps 20 --warmup 5
