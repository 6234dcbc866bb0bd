#!/bin/bash
# Round-3 measurement call (run under gpurun): tests, smoke, driver bench + repeats, interleaved A/B
# of tuning variants, per-phase stamps, solve_forces bench, kernel trace. Stops at the first failure.
#   TAG=<outputs dir>  VARIANTS="base v1 ..."  STAMPS="libhslabs_stamps.so ..."  SKIP_TESTS=1
set -o pipefail
R=$GRAFT_REPO_ROOT; TAG=${TAG:-r03}; OUT=$R/gpurun_out/$TAG; mkdir -p $OUT
cd $R
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  timeout -k 10 600 python -u -m pytest ${TESTS:-tests} -m gpu -x -q --timeout 300 --timeout-method thread \
    > $OUT/tests.log 2>&1 || { echo "tests failed"; tail -40 $OUT/tests.log; exit 1; }
  tail -3 $OUT/tests.log
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo smoke failed; cat $OUT/smoke.log; exit 1; }
  tail -1 $OUT/smoke.log
fi
DRIVER="--gpus 1 --steps 20 --warmup 5"
timeout -k 10 300 python bench.py $DRIVER > $OUT/bench_driver.json 2> $OUT/bench_driver.err || { echo bench failed; tail -20 $OUT/bench_driver.err; exit 1; }
python -c "import json;d=json.load(open('$OUT/bench_driver.json'));print('driver', round(d['value']/1e6,2), 'M; kernel us/step', round(d['roofline']['kernel_ms']*1e3,3), 'cpu', d['cpu_baseline']['value'])"
for v in ${VARIANTS:-}; do :; done
for i in 1 2 3; do
  for v in ${VARIANTS:-base}; do
    if [ $v = base ]; then unset HSLABS_VARIANT; else export HSLABS_VARIANT=$v; fi
    for a in "$DRIVER" "--steps 200 --warmup 20"; do
      timeout -k 10 120 python bench.py --no-cpu $a > $OUT/ab.json 2>>$OUT/ab.err || { tail -5 $OUT/ab.err; exit 1; }
      python -c "import json;d=json.load(open('$OUT/ab.json'));print('$v', d['steps'], round(d['value']/1e6,2), 'M; kernel us/step', round(d['roofline']['kernel_ms']*1e3,3))" | tee -a $OUT/ab.txt
    done
  done
done
unset HSLABS_VARIANT
for s in ${STAMPS:-}; do
  STAMPS_LIB=$s timeout -k 10 120 python tools/stamps.py > $OUT/stamps_$s.txt 2>&1 || { echo "stamps $s failed"; tail -5 $OUT/stamps_$s.txt; exit 1; }
  echo "== $s"; cat $OUT/stamps_$s.txt
done
if [ "${FORCES:-1}" = 1 ]; then
  timeout -k 10 300 python bench.py --forces --steps 20 --warmup 5 > $OUT/bench_forces.json 2> $OUT/bench_forces.err || { echo forces failed; tail -20 $OUT/bench_forces.err; exit 1; }
  cat $OUT/bench_forces.json
  for i in 1 2; do
    for v in ${FVARIANTS:-}; do
      if [ $v = base ]; then unset HSLABS_VARIANT; else export HSLABS_VARIANT=$v; fi
      timeout -k 10 120 python bench.py --forces --no-cpu --steps 20 --warmup 5 > $OUT/fab.json 2>>$OUT/fab.err || { tail -5 $OUT/fab.err; exit 1; }
      python -c "import json;d=json.load(open('$OUT/fab.json'));print('forces $v', round(d['value']/1e6,2), 'M; kernel us/step', round(d['roofline']['kernel_ms']*1e3,3), d['check'])" | tee -a $OUT/fab.txt
    done
  done
  unset HSLABS_VARIANT
fi
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 $R/bench.py $DRIVER --no-cpu > $OUT/prof.log 2>&1 || { echo prof failed; tail -20 $OUT/prof.log; exit 1; }
for f in $(find $OUT/prof -name "*kernel_stats.csv"); do cat $f; done
echo "r03 call done"
