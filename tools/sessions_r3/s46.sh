source tools/gpu_steps.sh
export TMPDIR=/tmp
step gputests46 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider
step smoke46 300 python -c "import __graft_entry__ as g; g.smoke()"
step b46_short1 300 python bench.py --gpus 1 --steps 20 --warmup 5
step b46_short2 300 python bench.py --gpus 1 --steps 20 --warmup 5
step b46_short3 300 python bench.py --gpus 1 --steps 20 --warmup 5
step b46_600 300 python bench.py --gpus 1
PROF_DIR=gpurun_out/prof46 step prof46 300 bash tools/prof_served.sh 300
