#!/bin/bash
# deferred vs synchronous verdicts: bench at the per-rank shard sizes, plus the RCCL rehearsal
# (--dist, world size 1) at the 8-GPU shard. Usage: bash tools/gpu_verdict.sh TAG
set -o pipefail
TAG=${1:-verdict}
O=gpurun_out/$TAG
mkdir -p $O
show() { python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], round(d['ms_per_step'],3), 'ms', round(d['value']), 'proofs/s', {k: (round(v,3) if isinstance(v,float) else v) for k,v in d['host_ms_per_batch'].items()})" $1 $2; }
for n in 8192 65536; do
  for mode in sync deferred deferred4; do
    flag=""; [ $mode = sync ] && flag="--sync-verdict"
    [ $mode = deferred4 ] && flag="--inflight 4"
    [ $mode = deferred4 ] && [ $n = 8192 ] && continue
    timeout -k 10 150 python -u bench.py --no-cpu --no-configs --no-iso --proofs $n $flag > $O/b_${n}_$mode.json 2> $O/b_${n}_$mode.err || { echo "bench $n $mode failed"; tail -20 $O/b_${n}_$mode.err; exit 1; }
    show $O/b_${n}_$mode.json "$n $mode"
  done
done
timeout -k 10 180 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29517 bench.py --no-cpu --no-configs --no-iso --dist --proofs 8192 > $O/b_8192_dist.json 2> $O/b_8192_dist.err || { echo "bench dist failed"; tail -20 $O/b_8192_dist.err; exit 1; }
show $O/b_8192_dist.json "8192 dist-deferred"
