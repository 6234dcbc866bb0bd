#!/bin/bash
# tools/gpu_r04_ab3.sh, then the fused-path stamps of a call queued behind another (B2B=1): the
# preparation pass's wave-start spread without the host's enqueue in front of it
set -o pipefail
R=$GRAFT_REPO_ROOT; TAG=${TAG:-r04_ab4}; OUT=$R/gpurun_out/$TAG; mkdir -p $OUT; cd $R
TAG=$TAG bash $R/tools/gpu_r04_ab3.sh || exit 1
B2B=1 FUSED=1 timeout -k 10 120 python tools/stamps.py > $OUT/stamps_b2b.txt 2>&1 || { echo stamps failed; tail -5 $OUT/stamps_b2b.txt; exit 1; }
grep -E "^p:|TOTAL|entry|wave start" $OUT/stamps_b2b.txt
echo "call done"
