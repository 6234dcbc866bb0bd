#!/bin/bash
# fp32 accuracy per guard variant (myant rows) and configs[2] throughput per occupancy variant.
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
lib() { [ -n "$1" ] && echo $R/hslabs_amd/_build/libhslabs_$1.so; }
for v in "" ${GUARDS:-g1e-3 g1e-5}; do
  echo "== guard variant ${v:-default}"
  HSLABS_LIB=$(lib $v) timeout -k 10 300 python tools/fp32_probe.py > gpurun_out/probe.log 2>&1 || { tail -5 gpurun_out/probe.log; exit 1; }
  grep myant gpurun_out/probe.log
done
for v in "" ${OCC:-f32w3 f32w4}; do
  HSLABS_LIB=$(lib $v) timeout -k 10 200 python bench.py --model spider --rollouts 16384 --horizon 32 --fp32 --steps 20 --warmup 3 --no-cpu > gpurun_out/c3.json || exit 1
  echo "occupancy variant ${v:-default}: $(python -c "import json;d=json.load(open('gpurun_out/c3.json'));print(d['value'], d['roofline']['kernel_ms'])")"
done
