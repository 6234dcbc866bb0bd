#!/bin/bash
# Round-4 baseline on the round-3 library (run under gpurun): the driver's bench command and repeats,
# the online-loop shape (--launch steps, one launch per control period) with its kernel trace, the
# driver command's kernel trace, PMC passes over every kernel of the driver job (setup pass and IK table
# included) and the fused-path phase stamps. Stops at the first failure.   TAG=<outputs dir>
set -o pipefail
R=$GRAFT_REPO_ROOT; TAG=${TAG:-r04_base}; OUT=$R/gpurun_out/$TAG; mkdir -p $OUT; cd $R
for i in 1 2 3; do
  timeout -k 10 120 python bench.py --no-cpu --steps 20 --warmup 5 > $OUT/rep.json 2>>$OUT/rep.err || { tail -5 $OUT/rep.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/rep.json'));print('driver', round(d['value']/1e6,2), 'M; kernel us/step', round(d['roofline']['kernel_ms']*1e3,3))" | tee -a $OUT/repeats.txt
  timeout -k 10 120 python bench.py --no-cpu --launch steps --steps 20 --warmup 5 > $OUT/steps.json 2>>$OUT/rep.err || { tail -5 $OUT/rep.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/steps.json'));print('launch steps', round(d['value']/1e6,2), 'M; kernel us/step', round(d['roofline']['kernel_ms']*1e3,3))" | tee -a $OUT/repeats.txt
done
FUSED=1 timeout -k 10 120 python tools/stamps.py > $OUT/stamps_fused.txt 2>&1 || { echo stamps failed; tail -5 $OUT/stamps_fused.txt; exit 1; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu > $OUT/prof.log 2>&1 || { echo prof failed; tail -20 $OUT/prof.log; exit 1; }
python3 $R/tools/trace_tail.py $OUT/prof/run_kernel_trace.csv 5 > $OUT/trace_tail.txt; cat $OUT/trace_tail.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_steps -o run -- python3 $R/bench.py --gpus 1 --launch steps --steps 20 --warmup 5 --no-cpu > $OUT/prof_steps.log 2>&1 || { echo prof steps failed; tail -20 $OUT/prof_steps.log; exit 1; }
python3 $R/tools/trace_tail.py $OUT/prof_steps/run_kernel_trace.csv 22 > $OUT/trace_tail_steps.txt; cat $OUT/trace_tail_steps.txt
PMC_OUT=$TAG/pmc bash $R/tools/gpu_pmc.sh || exit 1
echo "baseline call done"
