#!/bin/bash
# Interleaved A/B timing of the product library ("base") and tuning builds
# (hslabs_amd/_build/variants/libhslabs_<name>.so, build.build_variant) in one gpurun call.
#   VARIANTS="base v1 v2"  REPS=2  BENCH_ARGS="--steps 200 --warmup 20"  TAG=ab
set -o pipefail
R=$GRAFT_REPO_ROOT; OUT=$R/gpurun_out/${TAG:-ab}; mkdir -p $OUT; cd $R
for i in $(seq ${REPS:-2}); do
for v in ${VARIANTS:-base}; do
  if [ $v = base ]; then unset HSLABS_VARIANT; else export HSLABS_VARIANT=$v; fi
  timeout -k 10 120 python bench.py --no-cpu ${BENCH_ARGS:---steps 200 --warmup 20} > $OUT/${v}_$i.json 2>$OUT/${v}_$i.err || { tail -5 $OUT/${v}_$i.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/${v}_$i.json'));print('$v', round(d['value']/1e6,2), 'M steps/s; kernel us/step', round(d['roofline']['kernel_ms']*1e3,3))"
done; done
