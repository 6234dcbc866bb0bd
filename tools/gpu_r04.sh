#!/bin/bash
# Round-4 GPU call (run under gpurun): the GPU test suite, smoke, the driver's bench command and
# repeats, the online-loop shape (--launch steps), kernel traces of both. Stops at the first failure.
#   TAG=<outputs dir>  SKIP_TESTS=1 (measurements only)  PMC=1 (also the PMC passes)
set -o pipefail
R=$GRAFT_REPO_ROOT; TAG=${TAG:-r04}; OUT=$R/gpurun_out/$TAG; mkdir -p $OUT; cd $R
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 1100 python -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|assert" $OUT/tests.log | head -30; tail -30 $OUT/tests.log; exit 1; }
  tail -1 $OUT/tests.log
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo smoke failed; cat $OUT/smoke.log; exit 1; }
  tail -1 $OUT/smoke.log
fi
for i in 1 2 3; do
  timeout -k 10 120 python bench.py --no-cpu --steps 20 --warmup 5 > $OUT/rep.json 2>>$OUT/rep.err || { tail -5 $OUT/rep.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/rep.json'));print('driver', round(d['value']/1e6,2), 'M; kernel us/step', round(d['roofline']['kernel_ms']*1e3,3))" | tee -a $OUT/repeats.txt
  timeout -k 10 120 python bench.py --no-cpu --launch steps --steps 20 --warmup 5 > $OUT/steps.json 2>>$OUT/rep.err || { tail -5 $OUT/rep.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/steps.json'));print('launch steps', round(d['value']/1e6,2), 'M; kernel us/step', round(d['roofline']['kernel_ms']*1e3,3))" | tee -a $OUT/repeats.txt
done
timeout -k 10 120 python bench.py --no-cpu --steps 200 --warmup 20 > $OUT/k200.json 2>>$OUT/rep.err || { tail -5 $OUT/rep.err; exit 1; }
python -c "import json;d=json.load(open('$OUT/k200.json'));print('K=200', round(d['value']/1e6,2), 'M; kernel us/step', round(d['roofline']['kernel_ms']*1e3,3))" | tee -a $OUT/repeats.txt
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu > $OUT/prof.log 2>&1 || { echo prof failed; tail -20 $OUT/prof.log; exit 1; }
python3 $R/tools/trace_tail.py $OUT/prof/run_kernel_trace.csv 5 > $OUT/trace_tail.txt; cat $OUT/trace_tail.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_steps -o run -- python3 $R/bench.py --gpus 1 --launch steps --steps 20 --warmup 5 --no-cpu > $OUT/prof_steps.log 2>&1 || { echo prof steps failed; tail -20 $OUT/prof_steps.log; exit 1; }
python3 $R/tools/trace_tail.py $OUT/prof_steps/run_kernel_trace.csv 22 > $OUT/trace_tail_steps.txt; tail -4 $OUT/trace_tail_steps.txt
if [ -n "$PMC" ]; then PMC_OUT=$TAG/pmc bash $R/tools/gpu_pmc.sh || exit 1; fi
echo "call done"
