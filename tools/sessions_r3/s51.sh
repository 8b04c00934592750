source tools/gpu_steps.sh
export TMPDIR=/tmp
step kt51 400 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider
for b in 4096 8192 16384 32768; do
BK_REDUCE_BLOCKS=$b step pk51_r$b 150 rocprofv3 --kernel-trace --stats -d gpurun_out/pk51_r$b -o run -- python tools/payload_kernels.py --reps 30
done
for s in 64 128 256 512; do
BK_STREAM_BLOCKS_PER_CU=$s step pk51_s$s 150 rocprofv3 --kernel-trace --stats -d gpurun_out/pk51_s$s -o run -- python tools/payload_kernels.py --reps 30
done
