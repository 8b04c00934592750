source tools/gpu_steps.sh
export TMPDIR=/tmp
step kbench 300 python tools/bench_kernels.py
step prof_kbench 240 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_transpose -o run -- python3 tools/bench_kernels.py
