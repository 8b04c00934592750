#!/bin/bash
# Instruction histogram of the main K-loop of one lab kernel (after isa_check.sh)
#   bash tools/gemm_lab/loop_hist.sh <mangled-name-prefix>
S=${TMPDIR:-/tmp}/gemmlab_isa/gemm_lab-hip-amdgcn-amd-amdhsa-gfx950.s
L=$(grep -n "^$1.*:" $S | head -1 | cut -d: -f1)
awk -v s=$L 'NR>=s' $S | awk '/s_endpgm/{exit} {print}' > ${TMPDIR:-/tmp}/kern.s
A=$(grep -n "Loop Header" ${TMPDIR:-/tmp}/kern.s | head -1 | cut -d: -f1)
B=$(awk -v a=$A 'NR>a && /s_cbranch_scc/ {print NR; exit}' ${TMPDIR:-/tmp}/kern.s)
echo "loop lines $A-$B"
sed -n "${A},${B}p" ${TMPDIR:-/tmp}/kern.s | grep -v "^\s*;" | awk '{print $1}' | sort | uniq -c | sort -rn | head -${2:-14}
