#!/bin/bash
# Round-4 traffic evidence: FETCH_SIZE / WRITE_SIZE calibration on known byte counts (tools/fetch_calib.hip),
# then the product library's traffic PMC set on the driver command.   TAG=<dir>  TESTS=1: the GPU suite first
set -o pipefail
R=$GRAFT_REPO_ROOT; TAG=${TAG:-r04_traffic}; OUT=$R/gpurun_out/$TAG; mkdir -p $OUT; cd $R
if [ -n "$TESTS" ]; then
  timeout -k 10 1100 python -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|assert" $OUT/tests.log | head -30; tail -30 $OUT/tests.log; exit 1; }
  tail -1 $OUT/tests.log
fi
cd /tmp && export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 60 rocprofv3 --pmc $c --output-format csv -d $OUT/calib/$c -o run -- $R/tools/_build/fetch_calib > $OUT/calib_$c.log 2>&1 || { echo "calib $c failed"; tail -5 $OUT/calib_$c.log; exit 1; }
done
python3 $R/tools/pmc_calib.py $OUT/calib | tee $OUT/calib.txt
PMC_OUT=$TAG/traffic bash $R/tools/gpu_pmc.sh || exit 1
echo "call done"
