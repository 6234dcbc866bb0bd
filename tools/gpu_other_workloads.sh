set -o pipefail
O=gpurun_out/ow.jsonl; : > $O
timeout -k 10 120 python -u bench.py --no-cpu --model spider --rollouts 16384 --horizon 32 --fp32 >> $O &&
timeout -k 10 120 python -u bench.py --no-cpu --model spider --rollouts 16384 --horizon 32 >> $O &&
timeout -k 10 120 python -u bench.py --no-cpu --mixed >> $O &&
timeout -k 10 120 python -u bench.py --no-cpu --model myant >> $O &&
timeout -k 10 120 python -u bench.py --no-cpu --rollouts 32768 >> $O
