#!/bin/bash
# One gpurun call: GPU tests, smoke, the driver's bench command, and a rocprofv3 kernel trace of
# that same command. Every GPU step has its own time limit; the script stops at the first failure.
#   TESTS=<pytest args> (default: all -m gpu tests)  TAG=<name for the outputs>
#   SKIP_TESTS=1: bench and trace only;  EXTRA=1: also K=200, --forces and the other workloads
set -o pipefail
R=$GRAFT_REPO_ROOT; TAG=${TAG:-run}; OUT=$R/gpurun_out/$TAG; mkdir -p $OUT
cd $R
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  timeout -k 10 900 python -u -m pytest ${TESTS:-tests} -m gpu -x -v --timeout 300 --timeout-method thread \
    > $OUT/tests.log 2>&1 || { echo "tests failed"; tail -40 $OUT/tests.log; exit 1; }
  tail -3 $OUT/tests.log
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo smoke failed; cat $OUT/smoke.log; exit 1; }
  cat $OUT/smoke.log
fi
DRIVER="--gpus 1 --steps 20 --warmup 5"
timeout -k 10 300 python bench.py $DRIVER > $OUT/bench_driver.json 2> $OUT/bench_driver.err || { echo bench failed; tail -20 $OUT/bench_driver.err; exit 1; }
cat $OUT/bench_driver.json
for i in 1 2 3; do
  timeout -k 10 120 python bench.py $DRIVER --no-cpu >> $OUT/bench_driver_repeats.jsonl 2>> $OUT/bench_driver.err || { echo bench repeat failed; exit 1; }
done
python -c "import json;print('driver repeats', [round(json.loads(l)['value']/1e6,1) for l in open('$OUT/bench_driver_repeats.jsonl')])"
if [ "${EXTRA:-0}" = 1 ]; then
  timeout -k 10 300 python bench.py --steps 200 --warmup 20 --no-cpu > $OUT/bench_200.json 2> $OUT/bench_200.err || { echo bench200 failed; tail -20 $OUT/bench_200.err; exit 1; }
  cat $OUT/bench_200.json
  timeout -k 10 300 python bench.py --forces --steps 20 --warmup 5 > $OUT/bench_forces.json 2> $OUT/bench_forces.err || { echo forces failed; tail -20 $OUT/bench_forces.err; exit 1; }
  cat $OUT/bench_forces.json
  O=$OUT/other_workloads.jsonl; : > $O
  for a in "--model spider --rollouts 16384 --horizon 32 --fp32" "--model spider --rollouts 16384 --horizon 32" \
           "--mixed" "--model myant" "--rollouts 32768" "--curved"; do
    timeout -k 10 120 python -u bench.py --no-cpu $DRIVER $a >> $O 2>> $OUT/other.err || { echo "other $a failed"; exit 1; }
  done
  python -c "import json;[print(json.loads(l)['config']['workload'], round(json.loads(l)['value']/1e6,1)) for l in open('$O')]"
fi
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 $R/bench.py $DRIVER --no-cpu > $OUT/prof.log 2>&1 || { echo prof failed; tail -20 $OUT/prof.log; exit 1; }
for f in $(find $OUT/prof -name "*kernel_stats.csv"); do cat $f; done
