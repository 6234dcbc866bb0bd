# Interleaved timing of the product library and tuning variants (HSLABS_LIB):
#   [BENCH_ARGS="..."] [TAG=name] bash tools/gpu_sweep_libs.sh name1 name2 ...
# (variant name -> hslabs_amd/_build/libhslabs_<name>.so; "base" = the product library)
set -e
mkdir -p gpurun_out
T=${TAG:-sw}
for i in 1 2; do
  for v in base "$@"; do
    if [ "$v" = base ]; then L=""; else L=hslabs_amd/_build/libhslabs_$v.so; fi
    HSLABS_LIB=$L timeout -k 10 120 python -u bench.py --no-cpu $BENCH_ARGS > gpurun_out/${T}_${v}_$i.json 2>&1
  done
done
