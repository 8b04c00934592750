# Round 2: GPU suite + smoke + bench with the sandbox jail on (box runs unprivileged: Landlock/seccomp level)
source tools/gpu_steps.sh
export TMPDIR=/tmp
step isoprobe 60 python tools/probe/isolation_probe.py
step gputests 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider
step isotests 300 python -u -m pytest tests/test_isolation_cpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench_default 400 python bench.py
step bench_np600 300 python bench.py --steps 600
