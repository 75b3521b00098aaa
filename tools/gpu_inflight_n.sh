#!/bin/bash
# bench at a given shard size (PROOFS) and in-flight depths (DEPTHS), alternating repeats (REPS)
set -o pipefail
O=gpurun_out/${TAG:-r04inf}; mkdir -p $O
for rep in ${REPS:-1 2 3}; do for inf in ${DEPTHS:-4 6}; do
  timeout -k 10 200 python3 -u bench.py --no-cpu --no-configs --no-iso --proofs ${PROOFS:-32768} --inflight $inf --steps ${STEPS:-30} > $O/b_${PROOFS}_if${inf}_$rep.json 2> $O/b_${PROOFS}_if${inf}_$rep.err || { echo "bench $inf failed"; tail -20 $O/b_${PROOFS}_if${inf}_$rep.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/b_${PROOFS}_if${inf}_$rep.json')); print('${PROOFS} inflight $inf rep $rep', round(d['ms_per_step'],3), 'ms/batch', round(d['value']), 'proofs/s')"
done; done
