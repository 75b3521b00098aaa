#!/bin/bash
# gpu_round.sh TAG plus the bench at the 8-GPU per-rank shard (8,192 proofs) on one GPU.
set -o pipefail
TAG=${1:-run}
bash tools/gpu_round.sh $TAG || exit 1
timeout -k 10 120 python -u bench.py --no-cpu --no-configs --n 8192 > gpurun_out/$TAG/bench_8192.json 2> gpurun_out/$TAG/bench_8192.err || { echo "bench 8192 failed"; exit 1; }
cat gpurun_out/$TAG/bench_8192.json
