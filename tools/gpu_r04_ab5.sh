#!/bin/bash
# tools/gpu_r04_ab3.sh, then the fused-path stamps of a steady-state step (STEP=10) on the hexapod and spider
set -o pipefail
R=$GRAFT_REPO_ROOT; TAG=${TAG:-r04_ab5}; OUT=$R/gpurun_out/$TAG; mkdir -p $OUT; cd $R
TAG=$TAG bash $R/tools/gpu_r04_ab3.sh || exit 1
STEP=10 FUSED=1 timeout -k 10 120 python tools/stamps.py > $OUT/stamps_step10.txt 2>&1 || { echo stamps failed; tail -5 $OUT/stamps_step10.txt; exit 1; }
grep -vE "amdgpu.ids|histogram" $OUT/stamps_step10.txt
echo "call done"
