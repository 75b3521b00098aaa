#!/bin/bash
# 64k batches in flight sweep + RCCL (--dist, world 1) rehearsal of bench.py. Usage: bash tools/gpu_sweep_inflight.sh TAG
set -o pipefail
O=$(pwd)/gpurun_out/${1:-sweep}
mkdir -p $O
for k in 3 4 5 6; do
  timeout -k 10 200 python3 -u bench.py --no-cpu --no-configs --no-iso --inflight $k --steps 24 --warmup 4 > $O/if$k.json 2> $O/if$k.err || { echo "inflight $k failed"; tail -20 $O/if$k.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/if$k.json')); print('inflight $k', round(d['value']), round(d['ms_per_step'],3))"
done
timeout -k 10 300 python3 -u bench.py --dist --no-cpu --no-configs --steps 10 --warmup 3 > $O/bench_dist.json 2> $O/bench_dist.err || { echo "dist failed"; tail -20 $O/bench_dist.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench_dist.json')); print('dist 64k', round(d['value']), round(d['ms_per_step'],3), d['config']['collective'])"
timeout -k 10 300 python3 -u bench.py --dist --no-cpu --no-configs --no-iso --proofs 8192 --steps 30 --warmup 6 > $O/bench_dist_8k.json 2> $O/bench_dist_8k.err || { echo "dist 8k failed"; tail -20 $O/bench_dist_8k.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench_dist_8k.json')); print('dist 8k', round(d['value']), round(d['ms_per_step'],3))"
