# Round-end validation on one MI355X: GPU suite, smoke, the driver's bench
# command, longer headline runs, kernel microbench, served-path profile
source tools/gpu_steps.sh
step gputests 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench_default 400 python bench.py
step bench_np600a 300 python bench.py --steps 600
step bench_he600 300 python bench.py --workload hello --steps 600
step bench_np600b 300 python bench.py --steps 600
step kbench 300 python tools/bench_kernels.py
step prof_served 300 bash tools/prof_served.sh 300
