# Round 2 session 3: Philox round keys hoisted into SGPRs for the fused rand->reduce loop; A/B vs the previous build (same box), RNG tests
source tools/gpu_steps.sh
export TMPDIR=/tmp
step rngtests 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "uniform or philox or rand or normal or reduc" --timeout 120 --timeout-method thread -p no:cacheprovider
step rr_new_1 120 python tools/probe/rand_reduce_bench.py
step rr_old_1 120 env BEE_KERNEL_LIB=abtmp/libbeekern_prev.so python tools/probe/rand_reduce_bench.py
step rr_new_2 120 python tools/probe/rand_reduce_bench.py
step rr_old_2 120 env BEE_KERNEL_LIB=abtmp/libbeekern_prev.so python tools/probe/rand_reduce_bench.py
