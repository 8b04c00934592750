# headline payload kernels under rocprofv3 (lazy fused draw, and materialised),
# plus the sandbox lifecycle CPU probe on the GPU box's cores
source tools/gpu_steps.sh
export TMPDIR=/tmp
step payload_direct 120 python tools/payload_direct.py --iters 20
step prof_payload 180 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_payload -o run -- python3 tools/payload_direct.py --iters 20
export BEE_LAZY_RANDOM=0
step prof_payload_mat 180 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_payload_mat -o run -- python3 tools/payload_direct.py --iters 20
unset BEE_LAZY_RANDOM
step worker_cost 180 python tools/probe/worker_cost.py --n 300
