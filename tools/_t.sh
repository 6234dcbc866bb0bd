set -o pipefail
cd $GRAFT_REPO_ROOT; O=gpurun_out/t6; mkdir -p $O
timeout -k 10 120 python tools/variant_dump.py $O/base.npz > $O/d1.log 2>&1 || { tail $O/d1.log; exit 1; }
timeout -k 10 120 env HSLABS_VARIANT=rl python tools/variant_dump.py $O/rl.npz > $O/d2.log 2>&1 || { tail $O/d2.log; exit 1; }
python tools/variant_dump.py --compare $O/base.npz $O/rl.npz | head -5; rm -f $O/*.npz
VARIANTS="base rl" REPS=3 TAG=ab6 bash tools/gpu_ab.sh
