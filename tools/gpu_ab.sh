# A/B timing helper: product library vs a tuning variant (HSLABS_LIB), interleaved runs.
#   [BENCH_ARGS="..."] [TAG=name] bash tools/gpu_ab.sh [variant.so]
set -e
mkdir -p gpurun_out
T=${TAG:-ab}
for i in 1 2; do
  timeout -k 10 120 python -u bench.py --no-cpu $BENCH_ARGS > gpurun_out/${T}_base_$i.json 2>&1
  if [ -n "$1" ]; then HSLABS_LIB=$1 timeout -k 10 120 python -u bench.py --no-cpu $BENCH_ARGS > gpurun_out/${T}_var_$i.json 2>&1; fi
done
