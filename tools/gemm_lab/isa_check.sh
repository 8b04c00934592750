#!/bin/bash
# Compile the GEMM lab with resource remarks + assembly and summarise each
# kernel: VGPR/AGPR/scratch, instruction mix, waterfall loops.
#   bash tools/gemm_lab/isa_check.sh [kernel-name-substring]
set -e
ROOT=$(cd "$(dirname "$0")/../.." && pwd)
OUT=${TMPDIR:-/tmp}/gemmlab_isa
mkdir -p "$OUT"
cd "$OUT"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -c "$ROOT/tools/gemm_lab/gemm_lab.hip" --save-temps \
  -o lab.o -Rpass-analysis=kernel-resource-usage > res.txt 2>&1 || { grep error res.txt | head; exit 1; }
grep -E "Function Name|VGPRs:|AGPRs|ScratchSize|Occupancy" res.txt | sed 's/.*remark: //; s/.*hpp:[0-9]*:[0-9]*: //; s/ \[-Rpass.*//' \
  | paste - - - - - | grep "${1:-.}" | sed 's/Function Name: _ZN2bk//'
python3 "$ROOT/tools/gemm_lab/isa_stats.py" gemm_lab-hip-amdgcn-amd-amdhsa-gfx950.s "${1:-gemm}"
