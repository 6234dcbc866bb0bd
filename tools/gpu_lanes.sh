#!/bin/bash
# Lane activity per phase (tools/lane_activity.py): one PMC pass per build, the product library and
# the timing-only variants xnokin / xnosolve / xnoschur (build them first:
#   python -c "from hslabs_amd import build as b; b.SRC_FLAGS = {}; \
#     b.build_variant('xnokin', ['HS_EXP_KIN_FIRST=5']); b.build_variant('xnosolve', ['HS_EXP_NO_SOLVE']); \
#     b.build_variant('xnoschur', ['HS_EXP_NO_SCHUR'])")
set -o pipefail
R=$GRAFT_REPO_ROOT; OUT=$R/gpurun_out/${LANES_OUT:-lanes}; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for v in base xnokin xnosolve xnoschur; do
  if [ $v = base ]; then unset HSLABS_VARIANT; else export HSLABS_VARIANT=$v; fi
  mkdir -p $OUT/$v
  timeout -k 10 120 rocprofv3 --pmc SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAVES --output-format csv \
    -d $OUT/$v/p1 -o run -- python3 $R/bench.py --steps 20 --warmup 5 --no-cpu > $OUT/$v/p1.log 2>&1 || { echo "$v failed"; tail -5 $OUT/$v/p1.log; exit 1; }
done
python3 $R/tools/lane_activity.py $OUT $OUT/summary.txt --rollouts 4096
