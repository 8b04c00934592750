# Round 2: THP zygote heap + native sandbox bootstrap + coalesced broker frames, measured on MI355X
source tools/gpu_steps.sh
export TMPDIR=/tmp
step gputests 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench_np600 300 python bench.py --steps 600
step bench_default 400 python bench.py
step bench_np600_noboot 300 env BEE_NATIVE_BOOT=0 BEE_ZYGOTE_THP=0 python bench.py --steps 600 --materialized-steps 0
