#!/bin/bash
# high-priority checker/RCCL streams vs default, with and without the RCCL path (one rank).
# Usage: bash tools/gpu_prio.sh TAG
set -o pipefail
TAG=${1:-prio}
O=gpurun_out/$TAG
mkdir -p $O
show() { python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], round(d['ms_per_step'],3), 'ms', round(d['value']), 'proofs/s', {k: (round(v,3) if isinstance(v,float) else v) for k,v in d['host_ms_per_batch'].items()})" $1 $2; }
P=29517
for n in 8192 65536; do
  for pr in "" "--no-priority"; do
    tag=${n}${pr:+_noprio}
    timeout -k 10 150 python -u bench.py --no-cpu --no-configs --no-iso --proofs $n $pr > $O/b_$tag.json 2> $O/b_$tag.err || { echo "bench $tag failed"; tail -20 $O/b_$tag.err; exit 1; }
    show $O/b_$tag.json "$tag"
    P=$((P+1))
    timeout -k 10 180 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port $P bench.py --no-cpu --no-configs --no-iso --dist --proofs $n $pr > $O/b_${tag}_dist.json 2> $O/b_${tag}_dist.err || { echo "bench $tag dist failed"; tail -20 $O/b_${tag}_dist.err; exit 1; }
    show $O/b_${tag}_dist.json "${tag}_dist"
  done
done
