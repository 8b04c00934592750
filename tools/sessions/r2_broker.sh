# Round 2: new broker core + client handles + jail + latched interposer on MI355X; KFD VRAM sysfs probe
source tools/gpu_steps.sh
export TMPDIR=/tmp
step kfdprobe 120 python tools/probe/kfd_vram_probe.py
step gputests 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider
step isotests 300 python -u -m pytest tests/test_isolation_cpu.py tests/test_broker_fuzz_cpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench_np600 300 python bench.py --steps 600
step gemm_edge 300 python tools/gemm_edge_bench.py
