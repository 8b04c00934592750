source tools/gpu_steps.sh
export TMPDIR=/tmp
step gputests37 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider
step smoke37 300 python -c "import __graft_entry__ as g; g.smoke()"
step pk37 120 rocprofv3 --kernel-trace --stats -d gpurun_out/pk37 -o run -- python tools/payload_kernels.py --reps 30
step b37_short1 300 python bench.py --gpus 1 --steps 20 --warmup 5
step b37_short2 300 python bench.py --gpus 1 --steps 20 --warmup 5
step b37_short3 300 python bench.py --gpus 1 --steps 20 --warmup 5
step b37_600 300 python bench.py --gpus 1
