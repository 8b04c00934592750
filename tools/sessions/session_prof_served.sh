source tools/gpu_steps.sh
step prof_served 300 bash tools/prof_served.sh 200
