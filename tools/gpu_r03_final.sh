#!/bin/bash
# Round-3 evidence call (run under gpurun): tools/gpu_r03.sh (GPU tests, smoke, driver bench + repeats,
# K = 200, control-step stamps, solve_forces bench, kernel trace), solve_forces stamps and kernel trace,
# PMC passes for the control step and for solve_forces, and the same-box A/B against the round-2 tree
# (_r02/, when present). Stops at the first failure.   TAG=<outputs dir>
set -o pipefail
R=$GRAFT_REPO_ROOT; TAG=${TAG:-r03_final}; OUT=$R/gpurun_out/$TAG; mkdir -p $OUT
cd $R
TAG=$TAG STAMPS="libhslabs_stamps.so" bash tools/gpu_r03.sh || exit 1
timeout -k 10 120 python tools/forces_stamps.py > $OUT/forces_stamps.txt 2>&1 || { echo "forces stamps failed"; tail -5 $OUT/forces_stamps.txt; exit 1; }
cat $OUT/forces_stamps.txt
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_forces -o run -- python3 $R/bench.py --forces --steps 20 --warmup 5 --no-cpu > $OUT/prof_forces.log 2>&1 ) || { echo "forces prof failed"; tail -20 $OUT/prof_forces.log; exit 1; }
PMC_OUT=$TAG/pmc bash tools/gpu_pmc.sh || exit 1
PMC_OUT=$TAG/pmc_forces BENCH_ARGS="--forces --steps 20 --warmup 5" bash tools/gpu_pmc.sh || exit 1
if [ -d _r02 ]; then TAG=$TAG/r02ab VARIANTS=base REPS=2 bash tools/gpu_r02ab.sh || exit 1; fi
echo "r03 final call done"
