# Round 2 session 3: [K][N] GEMM kernel vs transpose+TN vs hipBLASLt over K (where should matmul(a, b) read B in place?)
source tools/gpu_steps.sh
export TMPDIR=/tmp
step nnsweep 300 python tools/gemm_nn_bench.py '[[4096,4096,512],[4096,4096,1024],[4096,4096,2048],[4096,4096,3072],[4096,4096,4096],[8192,8192,1024],[8192,8192,2048],[8192,8192,4096],[8192,8192,8192],[8192,4096,2048],[2048,8192,2048],[16384,4096,1024]]'
