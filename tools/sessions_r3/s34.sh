source tools/gpu_steps.sh
step pk34 120 python tools/payload_kernels.py --reps 50
step prof34 300 bash tools/prof_served.sh 300
