source tools/gpu_steps.sh
export TMPDIR=/tmp
step kt49 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider
step pk49 150 rocprofv3 --kernel-trace --stats -d gpurun_out/pk49 -o run -- python tools/payload_kernels.py --reps 30
step b49_short1 300 python bench.py --gpus 1 --steps 20 --warmup 5
step b49_short2 300 python bench.py --gpus 1 --steps 20 --warmup 5
