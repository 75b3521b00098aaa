#!/bin/bash
# bench at the per-rank shard sizes of 1/2/4/8 GPUs for 1..3 batches in flight (no CPU leg)
set -o pipefail
TAG=${1:-inflight}
O=gpurun_out/$TAG
mkdir -p $O
for n in ${SIZES:-65536 32768 16384 8192}; do
  for f in ${INFLIGHT:-1 2 3}; do
    timeout -k 10 150 python -u bench.py --no-cpu --no-configs --n $n --inflight $f --steps ${STEPS:-8} > $O/b_${n}_$f.json 2> $O/b_${n}_$f.err || { echo "bench $n $f failed"; tail -20 $O/b_${n}_$f.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], sys.argv[3], round(d['ms_per_step'],3), 'ms', round(d['value']), 'proofs/s', round(d['phase_ms']['device_pipeline'],2))" $O/b_${n}_$f.json $n $f
  done
done
