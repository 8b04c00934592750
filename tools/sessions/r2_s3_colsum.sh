# Round 2 session 3: column-sum kernels with independent load chains; axis tests + served-path profile
source tools/gpu_steps.sh
export TMPDIR=/tmp
step axistests 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "axis or reduc or sum" --timeout 120 --timeout-method thread -p no:cacheprovider
step prof_served 300 bash tools/prof_served.sh 200
