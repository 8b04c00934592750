source tools/gpu_steps.sh
export TMPDIR=/tmp
step ax39_def 120 rocprofv3 --kernel-trace --stats -d gpurun_out/ax39_def -o run -- python tools/probe/axis_shapes.py
BK_COLSUM_BLOCKS=512 BK_COLSUM_MIN_ROWS=256 step ax39_512 120 rocprofv3 --kernel-trace --stats -d gpurun_out/ax39_512 -o run -- python tools/probe/axis_shapes.py
BK_COLSUM_BLOCKS=1024 BK_COLSUM_MIN_ROWS=128 step ax39_1024 120 rocprofv3 --kernel-trace --stats -d gpurun_out/ax39_1024 -o run -- python tools/probe/axis_shapes.py
BK_COLSUM_BLOCKS=128 BK_COLSUM_MIN_ROWS=1024 step ax39_128 120 rocprofv3 --kernel-trace --stats -d gpurun_out/ax39_128 -o run -- python tools/probe/axis_shapes.py
step kt39 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "axis"
