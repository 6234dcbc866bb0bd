#!/bin/bash
# bench + rocprofv3 kernel-trace/stats on one MI355X (run under gpurun)
set -o pipefail
R=$GRAFT_REPO_ROOT; OUT=$R/gpurun_out; mkdir -p $OUT
cd $R
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo smoke failed; cat $OUT/smoke.log; exit 1; }
cat $OUT/smoke.log
timeout -k 10 400 python bench.py ${BENCH_ARGS:---steps 200 --warmup 20} > $OUT/bench.json 2> $OUT/bench.err || { echo bench failed; tail -20 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 $R/bench.py ${BENCH_ARGS:---steps 200 --warmup 20} --no-cpu > $OUT/prof.log 2>&1 || { echo prof failed; tail -20 $OUT/prof.log; exit 1; }
find $OUT/prof -name "*stats*" | head; for f in $(find $OUT/prof -name "*kernel_stats.csv"); do cat $f; done
