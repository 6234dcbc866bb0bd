#!/bin/bash
# Run-to-run spread of the driver command on one box: N back-to-back runs, each
# with the GPU's shader-clock state read from sysfs before and after (the level marked '*' in
# pp_dpm_sclk) and the power/temperature rocm-smi reports, to see whether slow runs follow the clock.
set -o pipefail
R=$GRAFT_REPO_ROOT; OUT=$R/gpurun_out/${TAG:-r04_spread}; mkdir -p $OUT; cd $R
dev=$(ls -d /sys/class/drm/card*/device 2>/dev/null | while read d; do [ -r $d/pp_dpm_sclk ] && echo $d && break; done)
sclk() { if [ -n "$dev" ]; then grep '\*' $dev/pp_dpm_sclk | tr -s ' ' | tr '\n' ' '; else echo "n/a"; fi; }
timeout -k 10 30 rocm-smi --showclocks --showpower --showtemp > $OUT/smi_before.txt 2>&1 || true
for i in $(seq 1 ${N:-12}); do
  a=$(sclk)
  timeout -k 10 120 python bench.py --no-cpu --steps 20 --warmup 5 > $OUT/run.json 2>>$OUT/run.err || { tail -5 $OUT/run.err; exit 1; }
  b=$(sclk)
  python3 -c "import json;d=json.load(open('$OUT/run.json'));print('run $i', round(d['value']/1e6,2), 'M steps/s; kernel us/step', round(d['roofline']['kernel_ms']*1e3,3), '| sclk before: $a | after: $b')" | tee -a $OUT/spread.txt
  [ -n "$SLEEP" ] && sleep $SLEEP
done
timeout -k 10 30 rocm-smi --showclocks --showpower --showtemp > $OUT/smi_after.txt 2>&1 || true
grep -iE "sclk|power|temp" $OUT/smi_after.txt | head -8
echo "call done"
