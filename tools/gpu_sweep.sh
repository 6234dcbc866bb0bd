#!/bin/bash
# GPU parity suite + bench sweep over tuning variants (run under gpurun).
#   VARIANTS="w2 w3 w4" bash tools/gpu_sweep.sh
set -o pipefail
R=$GRAFT_REPO_ROOT; OUT=$R/gpurun_out; mkdir -p $OUT
cd $R
timeout -k 10 600 python -m pytest tests -m gpu -x -q > $OUT/pytest_gpu.log 2>&1 || { echo "gpu tests failed"; tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
ARGS="${BENCH_ARGS:---steps 200 --warmup 20 --no-cpu}"
timeout -k 10 200 python bench.py $ARGS > $OUT/bench_base.json 2> $OUT/bench_base.err || { echo "bench failed"; tail -20 $OUT/bench_base.err; exit 1; }
echo "base: $(python -c "import json;d=json.load(open('$OUT/bench_base.json'));print(d['value'], d['roofline']['kernel_ms'])")"
for v in $VARIANTS; do
  HSLABS_LIB=$R/hslabs_amd/_build/libhslabs_$v.so timeout -k 10 200 python bench.py $ARGS > $OUT/bench_$v.json 2> $OUT/bench_$v.err || { echo "bench $v failed"; tail -20 $OUT/bench_$v.err; exit 1; }
  echo "$v: $(python -c "import json;d=json.load(open('$OUT/bench_$v.json'));print(d['value'], d['roofline']['kernel_ms'])")"
done
if [ -f hslabs_amd/_build/libhslabs_stamps.so ]; then
  timeout -k 10 200 python tools/stamps.py > $OUT/stamps.log 2>&1 || { echo "stamps failed"; tail -20 $OUT/stamps.log; exit 1; }
  cat $OUT/stamps.log
fi
