# Round 2 session 3: Philox three-input XORs as v_bitop3_b32; kernel A/B vs the two-XOR build (same box), bitwise RNG tests
source tools/gpu_steps.sh
export TMPDIR=/tmp
step rngtests 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "uniform or philox or rand or normal" --timeout 120 --timeout-method thread -p no:cacheprovider
step rr_new_1 120 python tools/probe/rand_reduce_bench.py
step rr_old_1 120 env BEE_KERNEL_LIB=abtmp/libbeekern_xor2.so python tools/probe/rand_reduce_bench.py
step rr_new_2 120 python tools/probe/rand_reduce_bench.py
step rr_old_2 120 env BEE_KERNEL_LIB=abtmp/libbeekern_xor2.so python tools/probe/rand_reduce_bench.py
step kbench 300 python tools/bench_kernels.py
