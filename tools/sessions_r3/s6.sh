source tools/gpu_steps.sh
step cgroup 30 bash -c 'cat /proc/self/cgroup; echo ---; stat -fc %T /sys/fs/cgroup; cat /sys/fs/cgroup/cgroup.controllers 2>&1; g=$(sed -n "s/^0:://p" /proc/self/cgroup); echo "own=$g"; ls -ld /sys/fs/cgroup$g 2>&1; cat /sys/fs/cgroup$g/cgroup.subtree_control 2>&1; cat /sys/fs/cgroup$g/cgroup.controllers 2>&1; mkdir /sys/fs/cgroup$g/bee-probe 2>&1 && echo MKDIR_OK && rmdir /sys/fs/cgroup$g/bee-probe; id'
step gputests 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider
BEE_BENCH_TRACE=gpurun_out/trace_short1.json step b_short1 240 python bench.py --gpus 1 --steps 20 --warmup 5
step b_default 300 python bench.py --gpus 1
BEE_BENCH_TRACE=gpurun_out/trace_short2.json step b_short2 240 python bench.py --gpus 1 --steps 20 --warmup 5
step blaslt 120 rocprofv3 --kernel-trace --stats -d gpurun_out/blaslt -o run -- python tools/probe/blaslt_kernel_probe.py
step gemm_ab 300 python tools/gemm_ab.py --rounds 5
