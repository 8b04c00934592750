source tools/gpu_steps.sh
step autogroup 10 bash -c 'cat /proc/sys/kernel/sched_autogroup_enabled; nproc; cat /sys/fs/cgroup/cpu.max 2>/dev/null; cat /proc/self/autogroup'
for i in 1 2 3; do
  step pg_$i 300 python bench.py --gpus 1 --steps 300 --warmup 30
  BEE_SANDBOX_SETSID=1 step ss_$i 300 python bench.py --gpus 1 --steps 300 --warmup 30
done
