set -o pipefail
O=gpurun_out/sweep8k; mkdir -p $O
for cfg in "8 auto" "8 0" "12 auto" "12 0" "16 0" "6 0"; do
  set -- $cfg
  if [ "$2" = "auto" ]; then unset ZG_LINES_FCHAIN; else export ZG_LINES_FCHAIN=$2; fi
  timeout -k 10 200 python -u bench.py --no-cpu --no-configs --no-iso --proofs 8192 --inflight $1 --steps 40 > $O/b_$1_$2.json 2> $O/b_$1_$2.err || { echo "fail $cfg"; tail -5 $O/b_$1_$2.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/b_$1_$2.json')); print('inflight $1 fuse $2', round(d['ms_per_step'],3), 'ms/batch', round(d['value']), 'proofs/s', d['context_stats']['fused_launches'])"
done
