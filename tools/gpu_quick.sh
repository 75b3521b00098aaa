#!/bin/bash
# Quick GPU-box pass: gpu tests, then the bench (no CPU leg, no side configs) at the 1/2/4/8-GPU
# per-rank shard sizes. Usage (repo root on the box): bash tools/gpu_quick.sh TAG
set -o pipefail
TAG=${1:-quick}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 420 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -30 $O/gpu_tests.log; exit 1; }
tail -3 $O/gpu_tests.log
for n in 65536 32768 16384 8192; do
  timeout -k 10 120 python -u bench.py --no-cpu --no-configs --n $n > $O/bench_$n.json 2> $O/bench_$n.err || { echo "bench $n failed"; tail -20 $O/bench_$n.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], round(d['ms_per_step'],3), 'ms', round(d['value']), 'proofs/s', {k: round(v,3) for k,v in d['phase_ms'].items()})" $O/bench_$n.json $n
done
