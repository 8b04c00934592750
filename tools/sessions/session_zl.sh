source tools/gpu_steps.sh
step gputests 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider
step bench_native 300 python bench.py --steps 100
step bench_pyloop 300 env BEE_ZYGOTE_PYLOOP=1 python bench.py --steps 100
step bench_native2 300 python bench.py --steps 100
export CPU_BD_DELAY=6 CPU_BD_WINDOW=4
step cpu_bd 300 python tools/cpu_breakdown.py --steps 3000 --warmup 3
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
