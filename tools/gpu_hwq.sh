#!/bin/bash
# hardware-queue count vs the one-rank RCCL rehearsal at the 8-GPU shard. Usage: bash tools/gpu_hwq.sh TAG
set -o pipefail
TAG=${1:-hwq}
O=gpurun_out/$TAG
mkdir -p $O
show() { python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], round(d['ms_per_step'],3), 'ms', round(d['value']), 'proofs/s', {k: (round(v,3) if isinstance(v,float) else v) for k,v in d['host_ms_per_batch'].items()})" $1 $2; }
P=29517
for q in ${QUEUES:-16 20}; do
  export GPU_MAX_HW_QUEUES=$q
  timeout -k 10 150 python -u bench.py --no-cpu --no-configs --no-iso --proofs 8192 > $O/b_$q.json 2> $O/b_$q.err || { echo "bench $q failed"; tail -20 $O/b_$q.err; exit 1; }
  show $O/b_$q.json "8192 q=$q"
  P=$((P+1))
  timeout -k 10 180 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port $P bench.py --no-cpu --no-configs --no-iso --dist --proofs 8192 > $O/b_${q}_dist.json 2> $O/b_${q}_dist.err || { echo "bench $q dist failed"; tail -20 $O/b_${q}_dist.err; exit 1; }
  show $O/b_${q}_dist.json "8192_dist q=$q"
done
