source tools/gpu_steps.sh
step compile_cost 60 python tools/probe/compile_cost.py
