# Round 2 session 3: served-path kernel + marker profile of the final build
source tools/gpu_steps.sh
export TMPDIR=/tmp
step prof_served 300 bash tools/prof_served.sh 300
