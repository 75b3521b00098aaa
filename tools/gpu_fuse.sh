#!/bin/bash
# fused R-chain + f-chain launch vs split launches with batches in flight (deferred verdicts),
# plus the one-rank RCCL rehearsal of the multi-GPU protocol. Usage: bash tools/gpu_fuse.sh TAG
set -o pipefail
TAG=${1:-fuse}
O=gpurun_out/$TAG
mkdir -p $O
show() { python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], round(d['ms_per_step'],3), 'ms', round(d['value']), 'proofs/s', d['config']['batches_in_flight_per_gpu'], {k: round(v,3) for k,v in d['phase_ms'].items()})" $1 $2; }
for n in 8192 16384; do
  for f in auto 0; do
    if [ $f = auto ]; then unset ZG_LINES_FCHAIN; else export ZG_LINES_FCHAIN=$f; fi
    timeout -k 10 150 python -u bench.py --no-cpu --no-configs --no-iso --n $n > $O/b_${n}_$f.json 2> $O/b_${n}_$f.err || { echo "bench $n $f failed"; tail -20 $O/b_${n}_$f.err; exit 1; }
    show $O/b_${n}_$f.json "$n fuse=$f"
  done
done
unset ZG_LINES_FCHAIN
timeout -k 10 180 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29517 bench.py --no-cpu --no-configs --no-iso --dist --proofs 8192 > $O/b_8192_dist.json 2> $O/b_8192_dist.err || { echo "bench dist failed"; tail -20 $O/b_8192_dist.err; exit 1; }
show $O/b_8192_dist.json "8192 dist"
