# in-flight x fusion sweep on 8k-proof shards: CFGS="6:auto 6:0 ..." (inflight:ZG_LINES_FCHAIN)
set -o pipefail
O=gpurun_out/sweep8k; mkdir -p $O
for cfg in ${CFGS:-3:auto 3:0 4:auto 4:0 5:0 6:auto 6:0}; do
  inf=${cfg%%:*}; fu=${cfg##*:}
  if [ "$fu" = "auto" ]; then unset ZG_LINES_FCHAIN; else export ZG_LINES_FCHAIN=$fu; fi
  timeout -k 10 200 python -u bench.py --no-cpu --no-configs --no-iso --proofs 8192 --inflight $inf --steps 40 > $O/b_${inf}_$fu.json 2> $O/b_${inf}_$fu.err || { echo "fail $cfg"; tail -5 $O/b_${inf}_$fu.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/b_${inf}_$fu.json')); print('inflight $inf fuse $fu', round(d['ms_per_step'],3), 'ms/batch', round(d['value']), 'proofs/s', d['context_stats']['fused_launches'])"
done
