#!/bin/bash
# GPU tests on the product library, then an interleaved A/B of tuning builds at the
# driver command and at K = 200, then the driver job's kernel trace.   VARIANTS="base v1 ..."  TAG=...
set -o pipefail
R=$GRAFT_REPO_ROOT; TAG=${TAG:-ab}; OUT=$R/gpurun_out/$TAG; mkdir -p $OUT; cd $R
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 1100 python -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|assert" $OUT/tests.log | head -30; tail -30 $OUT/tests.log; exit 1; }
  tail -1 $OUT/tests.log
fi
# ARGSETS: bench argument sets separated by ';' (default: the driver command and K = 200)
IFS=';' read -ra SETS <<< "${ARGSETS:---steps 20 --warmup 5;--steps 200 --warmup 20}"
for args in "${SETS[@]}"; do
  echo "== $args" | tee -a $OUT/ab.txt
  for i in 1 2; do
  for v in ${VARIANTS:-base}; do
    if [ $v = base ]; then unset HSLABS_VARIANT; else export HSLABS_VARIANT=$v; fi
    timeout -k 10 180 python bench.py --no-cpu $args > $OUT/${v}.json 2>$OUT/${v}.err || { tail -5 $OUT/${v}.err; exit 1; }
    python -c "import json;d=json.load(open('$OUT/${v}.json'));print('$v', round(d['value']/1e6,2), 'M steps/s; kernel us/step', round(d['roofline']['kernel_ms']*1e3,3))" | tee -a $OUT/ab.txt
  done; done
done
unset HSLABS_VARIANT
if [ -n "$STAMPS" ]; then
  FUSED=1 timeout -k 10 120 python tools/stamps.py > $OUT/stamps_fused.txt 2>&1 || { echo stamps failed; tail -5 $OUT/stamps_fused.txt; exit 1; }
  grep -vE "amdgpu.ids" $OUT/stamps_fused.txt
fi
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu > $OUT/prof.log 2>&1 || { echo prof failed; tail -20 $OUT/prof.log; exit 1; }
python3 $R/tools/trace_tail.py $OUT/prof/run_kernel_trace.csv 4 > $OUT/trace_tail.txt; cat $OUT/trace_tail.txt
if [ -n "$STEPS_TRACE" ]; then  # the online-loop shape: one hs_run_steps launch per control period
  timeout -k 10 120 python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 --launch steps --no-cpu > $OUT/steps.json 2>$OUT/steps.err || { tail -5 $OUT/steps.err; exit 1; }
  cat $OUT/steps.json
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/steps_prof -o run -- python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 --launch steps --no-cpu > $OUT/steps_prof.log 2>&1 || { echo steps prof failed; tail -20 $OUT/steps_prof.log; exit 1; }
  python3 $R/tools/trace_tail.py $OUT/steps_prof/run_kernel_trace.csv 25 > $OUT/steps_trace_tail.txt; tail -8 $OUT/steps_trace_tail.txt
fi
echo "call done"
