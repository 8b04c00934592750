source tools/gpu_steps.sh
step cpufreq 300 bash tools/probe/cpufreq_probe.sh --gpus 1 --steps 20 --warmup 5
