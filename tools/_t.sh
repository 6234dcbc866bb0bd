cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/pv2; mkdir -p $O
for v in base straight; do
  if [ $v = base ]; then unset HSLABS_VARIANT; else export HSLABS_VARIANT=$v; fi
  timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 --output-format csv -d $O/$v -o run -- python3 $R/bench.py --steps 20 --warmup 5 --no-cpu > $O/$v.log 2>&1 || { echo "$v failed"; tail -3 $O/$v.log; exit 1; }
done
cd $R && VARIANTS="base straight" REPS=2 TAG=ab8 bash tools/gpu_ab.sh
cd $GRAFT_REPO_ROOT && VARIANTS="base f5 f6" REPS=2 TAG=ab9 BENCH_ARGS="--model spider --rollouts 16384 --horizon 32 --fp32 --steps 10 --warmup 3" bash tools/gpu_ab.sh
