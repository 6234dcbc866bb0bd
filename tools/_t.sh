set -o pipefail
cd $GRAFT_REPO_ROOT; O=gpurun_out/t7; mkdir -p $O
timeout -k 10 120 python tools/variant_dump.py $O/base.npz > $O/d1.log 2>&1 || { tail $O/d1.log; exit 1; }
timeout -k 10 120 env HSLABS_VARIANT=new python tools/variant_dump.py $O/new.npz > $O/d2.log 2>&1 || { tail $O/d2.log; exit 1; }
python tools/variant_dump.py --compare $O/base.npz $O/new.npz | head -8; rm -f $O/*.npz
VARIANTS="base new" REPS=3 TAG=ab7 bash tools/gpu_ab.sh
