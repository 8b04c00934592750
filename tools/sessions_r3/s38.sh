source tools/gpu_steps.sh
export TMPDIR=/tmp
step ax38 120 rocprofv3 --kernel-trace --stats -d gpurun_out/ax38 -o run -- python tools/probe/axis_shapes.py
