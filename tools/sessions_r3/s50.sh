source tools/gpu_steps.sh
export TMPDIR=/tmp
step kt50 400 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider
step pk50 150 rocprofv3 --kernel-trace --stats -d gpurun_out/pk50 -o run -- python tools/payload_kernels.py --reps 30
BK_STREAM_BLOCKS_PER_CU=16 step pk50_s16 150 rocprofv3 --kernel-trace --stats -d gpurun_out/pk50_s16 -o run -- python tools/payload_kernels.py --reps 30
BK_STREAM_BLOCKS_PER_CU=32 step pk50_s32 150 rocprofv3 --kernel-trace --stats -d gpurun_out/pk50_s32 -o run -- python tools/payload_kernels.py --reps 30
BK_STREAM_BLOCKS_PER_CU=128 step pk50_s128 150 rocprofv3 --kernel-trace --stats -d gpurun_out/pk50_s128 -o run -- python tools/payload_kernels.py --reps 30
