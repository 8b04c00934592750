# CPU cost per request by process role on the GPU box (headline payload)
source tools/gpu_steps.sh
export CPU_BD_DELAY=6 CPU_BD_WINDOW=4
step cpu_bd 300 python tools/cpu_breakdown.py --steps 3000 --warmup 3
step cpu_bd_hello 300 python tools/cpu_breakdown.py --steps 3000 --warmup 3 --workload hello
