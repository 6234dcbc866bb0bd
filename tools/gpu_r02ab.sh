#!/bin/bash
# Same-box A/B of the round-2 final tree (_r02/, git archive of c775ac1 with its own built library)
# against the current library and its tuning variants: control loop (driver config and K = 200)
# and solve_forces (tools/forces_probe.py). VARIANTS="base noguard ..."  REPS=3  TAG=r02ab
set -o pipefail
R=$GRAFT_REPO_ROOT; OUT=$R/gpurun_out/${TAG:-r02ab}; mkdir -p $OUT; cd $R
for i in $(seq ${REPS:-3}); do
  for a in "--gpus 1 --steps 20 --warmup 5" "--steps 200 --warmup 20"; do
    (cd _r02 && timeout -k 10 120 python bench.py --no-cpu $a > $OUT/r02.json 2>>$OUT/r02.err) || { tail -5 $OUT/r02.err; exit 1; }
    python -c "import json;d=json.load(open('$OUT/r02.json'));print('r02', d['steps'], round(d['value']/1e6,2), 'M; kernel us/step', round(d['roofline']['kernel_ms']*1e3,3))" | tee -a $OUT/ab.txt
    for v in ${VARIANTS:-base}; do
      if [ $v = base ]; then unset HSLABS_VARIANT; else export HSLABS_VARIANT=$v; fi
      timeout -k 10 120 python bench.py --no-cpu $a > $OUT/cur.json 2>>$OUT/cur.err || { tail -5 $OUT/cur.err; exit 1; }
      python -c "import json;d=json.load(open('$OUT/cur.json'));print('$v', d['steps'], round(d['value']/1e6,2), 'M; kernel us/step', round(d['roofline']['kernel_ms']*1e3,3))" | tee -a $OUT/ab.txt
    done
    unset HSLABS_VARIANT
  done
  if [ "${FORCES:-1}" = 1 ]; then
    (cd _r02 && timeout -k 10 120 python tools/forces_probe.py 2>>$OUT/r02.err | sed 's/^/r02 forces /') | tee -a $OUT/ab.txt || exit 1
    timeout -k 10 120 python tools/forces_probe.py 2>>$OUT/cur.err | sed 's/^/cur forces /' | tee -a $OUT/ab.txt || exit 1
  fi
done
echo "r02ab done"
