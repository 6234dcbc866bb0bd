#!/bin/bash
# The round's evidence call (run under gpurun) on the product library: GPU tests, smoke, the driver's bench
# command (with the CPU baseline) and repeats, K = 200, solve_forces, a kernel trace with stats, the PMC
# traffic passes and the fused-path phase stamps. Stops at the first failure.   TAG=<outputs dir>
set -o pipefail
R=$GRAFT_REPO_ROOT; TAG=${TAG:-evidence}; OUT=$R/gpurun_out/$TAG; mkdir -p $OUT; cd $R
# ONLY_PMC=1: the counter passes alone (a second call: the whole set does not fit one call's time limit)
if [ -z "$ONLY_PMC" ]; then
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { echo "tests failed"; tail -40 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo smoke failed; cat $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_driver.json 2> $OUT/bench_driver.err || { echo bench failed; tail -20 $OUT/bench_driver.err; exit 1; }
python -c "import json;d=json.load(open('$OUT/bench_driver.json'));print('driver', round(d['value']/1e6,2), 'M; kernel us/step', round(d['roofline']['kernel_ms']*1e3,3), 'cpu', d['cpu_baseline']['value'])"
for i in 1 2 3; do
  timeout -k 10 120 python bench.py --no-cpu --steps 20 --warmup 5 > $OUT/rep.json 2>>$OUT/rep.err || { tail -5 $OUT/rep.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/rep.json'));print('driver repeat', round(d['value']/1e6,2), 'M; kernel us/step', round(d['roofline']['kernel_ms']*1e3,3))" | tee -a $OUT/repeats.txt
done
for i in 1 2; do
  timeout -k 10 120 python bench.py --no-cpu --steps 200 --warmup 20 > $OUT/k200.json 2>>$OUT/rep.err || { tail -5 $OUT/rep.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/k200.json'));print('K=200', round(d['value']/1e6,2), 'M; kernel us/step', round(d['roofline']['kernel_ms']*1e3,3))" | tee -a $OUT/repeats.txt
done
timeout -k 10 300 python bench.py --forces --steps 20 --warmup 5 > $OUT/bench_forces.json 2> $OUT/bench_forces.err || { echo forces failed; tail -20 $OUT/bench_forces.err; exit 1; }
python -c "import json;d=json.load(open('$OUT/bench_forces.json'));print('forces', round(d['value']/1e6,2), 'M; kernel us/step', round(d['roofline']['kernel_ms']*1e3,3))"
for w in "--model spider --rollouts 16384 --horizon 32 --fp32" "--model spider --rollouts 16384 --horizon 32" "--mixed" "--model myant" "--rollouts 32768" "--curved" "--sim" "--sim --fp32 --model spider --rollouts 16384"; do
  timeout -k 10 180 python -u bench.py --no-cpu $w >> $OUT/other_workloads.jsonl 2>>$OUT/other.err || { echo "other workload failed: $w"; tail -5 $OUT/other.err; exit 1; }
  tail -1 $OUT/other_workloads.jsonl | python -c "import json,sys;d=json.loads(sys.stdin.read());print('$w', round(d['value']/1e6,3), 'M', d['unit'])"
done
# the limb-lane step kernel's phase stamps (libhslabs_stamps.so, built beforehand: tools/limb_stamps.py --build-only)
timeout -k 10 120 python tools/limb_stamps.py > $OUT/stamps_limb.txt 2>&1 || { echo stamps failed; tail -5 $OUT/stamps_limb.txt; exit 1; }
STEP=10 timeout -k 10 120 python tools/limb_stamps.py > $OUT/stamps_limb_step10.txt 2>&1 || { echo stamps failed; tail -5 $OUT/stamps_limb_step10.txt; exit 1; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu > $OUT/prof.log 2>&1 || { echo prof failed; tail -20 $OUT/prof.log; exit 1; }
python3 $R/tools/trace_tail.py $OUT/prof/run_kernel_trace.csv 5 > $OUT/trace_tail.txt; cat $OUT/trace_tail.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_steps -o run -- python3 $R/bench.py --gpus 1 --launch steps --steps 20 --warmup 5 --no-cpu > $OUT/prof_steps.log 2>&1 || { echo prof steps failed; tail -20 $OUT/prof_steps.log; exit 1; }
python3 $R/tools/trace_tail.py $OUT/prof_steps/run_kernel_trace.csv 25 > $OUT/trace_tail_steps.txt; tail -4 $OUT/trace_tail_steps.txt
timeout -k 10 120 python3 $R/bench.py --gpus 1 --launch steps --steps 20 --warmup 5 --no-cpu > $OUT/bench_steps.json 2>>$OUT/rep.err || { tail -5 $OUT/rep.err; exit 1; }
fi
[ -n "$SKIP_PMC" ] && { echo "evidence call done (no PMC)"; exit 0; }
cd /tmp && export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 60 rocprofv3 --pmc $c --output-format csv -d $OUT/calib/$c -o run -- $R/tools/_build/fetch_calib > $OUT/calib_$c.log 2>&1 || { echo "calib $c failed"; tail -5 $OUT/calib_$c.log; exit 1; }
done
python3 $R/tools/pmc_calib.py $OUT/calib > $OUT/calib.txt; cat $OUT/calib.txt
PMC_OUT=$TAG/pmc bash $R/tools/gpu_pmc.sh || exit 1
PMC_SET=diag PMC_OUT=$TAG/pmc_diag bash $R/tools/gpu_pmc.sh || exit 1
PMC_OUT=$TAG/pmc_forces BENCH_ARGS="--forces --steps 20 --warmup 5" bash $R/tools/gpu_pmc.sh || exit 1
# configs[2] and configs[4]: the traffic passes on their own bench commands
PMC_OUT=$TAG/pmc_c2 BENCH_ARGS="--model spider --rollouts 16384 --horizon 32 --fp32 --steps 20 --warmup 5" bash $R/tools/gpu_pmc.sh || exit 1
PMC_OUT=$TAG/pmc_c4 BENCH_ARGS="--mixed --steps 20 --warmup 5" bash $R/tools/gpu_pmc.sh || exit 1
if [ -n "$SPREAD" ]; then N=$SPREAD TAG=$TAG/spread bash $R/tools/gpu_spread_probe.sh || exit 1; fi
echo "evidence call done"
