# Round 2 session 3: every BASELINE config on the 1-GPU box with the current build + served-path kernel profile
source tools/gpu_steps.sh
export TMPDIR=/tmp
step suite 900 python tools/bench_suite.py --out gpurun_out/r2_s3_bench_suite.jsonl
step prof_served 300 bash tools/prof_served.sh 200
