#!/bin/bash
# Round-4 counters on the product library: the traffic set and the stall set (tools/gpu_pmc.sh), then
# the solve_forces bench line with its CPU baseline.   TAG=<dir>
set -o pipefail
R=$GRAFT_REPO_ROOT; TAG=${TAG:-r04_pmc}; OUT=$R/gpurun_out/$TAG; mkdir -p $OUT; cd $R
PMC_OUT=$TAG/traffic bash $R/tools/gpu_pmc.sh || exit 1
PMC_SET=diag PMC_OUT=$TAG/diag bash $R/tools/gpu_pmc.sh || exit 1
if [ -n "$FORCES" ]; then
  timeout -k 10 200 python bench.py --forces --steps 20 --warmup 5 --cpu-seconds 8 > $OUT/forces.json 2> $OUT/forces.err || { tail -5 $OUT/forces.err; exit 1; }
  cat $OUT/forces.json
fi
echo "call done"
