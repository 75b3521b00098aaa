#!/bin/bash
# 64k-shard bench (default in-flight depth) under alternative knobs, alternating repeats:
# ENVS="A=1,B=2 C=3 ..." (comma = same run), REPS="1 2"
set -o pipefail
O=gpurun_out/${TAG:-r04env64}; mkdir -p $O
for rep in ${REPS:-1 2}; do for cfg in default ${ENVS:-}; do
  envs=""; [ "$cfg" != default ] && envs=$(echo $cfg | tr ',' ' ')
  env $envs timeout -k 10 200 python3 -u bench.py --no-cpu --no-configs --no-iso --steps 20 > $O/b64_${cfg}_$rep.json 2> $O/b64_${cfg}_$rep.err || { echo "bench 64k $cfg failed"; tail -20 $O/b64_${cfg}_$rep.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/b64_${cfg}_$rep.json')); print('64k $cfg rep $rep', round(d['ms_per_step'],3), 'ms/step', round(d['value']), 'proofs/s')"
done; done
