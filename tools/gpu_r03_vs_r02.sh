#!/bin/bash
# Same-box comparison of the round-2 final tree (_r02/: git archive of c775ac1 with its own library,
# gitignored) and the current library, interleaved: the driver command, K = 200, configs[2] (spider
# fp32, H = 32) and configs[4] (mixed).   REPS=2  TAG=r03_vs_r02
set -o pipefail
R=$GRAFT_REPO_ROOT; OUT=$R/gpurun_out/${TAG:-r03_vs_r02}; mkdir -p $OUT; cd $R
for i in $(seq ${REPS:-2}); do
  for a in "--gpus 1 --steps 20 --warmup 5" "--steps 200 --warmup 20" "--model spider --rollouts 16384 --horizon 32 --fp32" "--mixed"; do
    (cd _r02 && timeout -k 10 180 python bench.py --no-cpu $a > $OUT/r02.json 2>>$OUT/r02.err) || { tail -5 $OUT/r02.err; exit 1; }
    python -c "import json;d=json.load(open('$OUT/r02.json'));print('r02 | $a |', round(d['value']/1e6,2), 'M; kernel us/step', round(d['roofline']['kernel_ms']*1e3,3))" | tee -a $OUT/ab.txt
    timeout -k 10 180 python bench.py --no-cpu $a > $OUT/cur.json 2>>$OUT/cur.err || { tail -5 $OUT/cur.err; exit 1; }
    python -c "import json;d=json.load(open('$OUT/cur.json'));print('r03 | $a |', round(d['value']/1e6,2), 'M; kernel us/step', round(d['roofline']['kernel_ms']*1e3,3))" | tee -a $OUT/ab.txt
  done
done
echo "r03 vs r02 done"
