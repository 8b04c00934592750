source tools/gpu_steps.sh
step suite 900 python tools/bench_suite.py --out gpurun_out/bench_suite_final.jsonl
