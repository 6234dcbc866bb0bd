#!/bin/bash
# Per-variant kernel averages (rocprofv3 --kernel-trace --stats) of one bench command: VARIANTS="base v1 ..."
# ARGS="<bench args>" TAG=...   Prints each variant's hs_* kernel rows (calls, average ns).
set -o pipefail
R=$GRAFT_REPO_ROOT; TAG=${TAG:-kstats}; OUT=$R/gpurun_out/$TAG; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for i in 1 2; do
for v in ${VARIANTS:-base}; do
  if [ $v = base ]; then unset HSLABS_VARIANT; else export HSLABS_VARIANT=$v; fi
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$v.$i -o run -- python3 $R/bench.py --gpus 1 --no-cpu ${ARGS:---steps 20 --warmup 5} > $OUT/$v.$i.log 2>&1 || { echo "$v failed"; tail -20 $OUT/$v.$i.log; exit 1; }
  python3 - "$OUT/$v.$i/run_kernel_stats.csv" "$v" <<'PY' | tee -a $OUT/summary.txt
import csv, sys
rows = [r for r in csv.DictReader(open(sys.argv[1])) if 'hs_' in r['Name']]
print(sys.argv[2], ' | '.join(f"{r['Name'].split('(')[0].split('::')[-1][:28]} x{r['Calls']} {float(r['AverageNs'])/1e3:.2f}us" for r in rows))
PY
done; done
echo "call done"
