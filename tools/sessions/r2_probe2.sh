source tools/gpu_steps.sh
export TMPDIR=/tmp
step kfdprobe 120 python tools/probe/kfd_vram_probe.py
step gputests 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider
step bench_np600 300 python bench.py --steps 600
