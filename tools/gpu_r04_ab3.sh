#!/bin/bash
# GPU tests, an interleaved A/B (tools/gpu_r04_ab.sh) with the fused-path stamps, per-variant kernel
# averages (tools/gpu_kstats_sweep.sh).   VARIANTS, TAG, ARGSETS
set -o pipefail
R=$GRAFT_REPO_ROOT; TAG=${TAG:-r04_ab3}; OUT=$R/gpurun_out/$TAG; mkdir -p $OUT; cd $R
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|assert" $OUT/tests.log | head -30; tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
SKIP_TESTS=1 STAMPS=1 TAG=$TAG/ab bash $R/tools/gpu_r04_ab.sh > $OUT/ab.log 2>&1 || { tail -20 $OUT/ab.log; exit 1; }
cat $OUT/ab/ab.txt; grep -E "^(kin|k:|contact|outputs|particular|TOTAL|entry|p:)" $OUT/ab/stamps_fused.txt
TAG=$TAG/ks bash $R/tools/gpu_kstats_sweep.sh > $OUT/ks.log 2>&1 || { tail -20 $OUT/ks.log; exit 1; }
cat $OUT/ks/summary.txt
echo "call done"
