source tools/gpu_steps.sh
export TMPDIR=/tmp
step rr40_1024 120 rocprofv3 --kernel-trace --stats -d gpurun_out/rr40_1024 -o run -- python tools/payload_kernels.py --reps 20
BK_RANDRED_BLOCKS=2048 step rr40_2048 120 rocprofv3 --kernel-trace --stats -d gpurun_out/rr40_2048 -o run -- python tools/payload_kernels.py --reps 20
BK_RANDRED_BLOCKS=4096 step rr40_4096 120 rocprofv3 --kernel-trace --stats -d gpurun_out/rr40_4096 -o run -- python tools/payload_kernels.py --reps 20
BK_RANDRED_BLOCKS=512 step rr40_512 120 rocprofv3 --kernel-trace --stats -d gpurun_out/rr40_512 -o run -- python tools/payload_kernels.py --reps 20
step kt40 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider
