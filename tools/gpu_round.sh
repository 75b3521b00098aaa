#!/bin/bash
# One GPU-box pass: gpu parity tests, bench (with cpu baseline), rocprofv3 kernel stats of the bench.
# Usage (from the repo root on the box): bash tools/gpu_round.sh TAG
set -o pipefail
TAG=${1:-run}
R=$(pwd)
O=$R/gpurun_out/$TAG
mkdir -p $O
timeout -k 10 420 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -30 $O/gpu_tests.log; exit 1; }
tail -3 $O/gpu_tests.log
timeout -k 10 300 python -u bench.py > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -30 $O/bench.err; exit 1; }
cat $O/bench.json
cd /tmp && export TMPDIR=/tmp
# the bench as run (batches in flight: kernel durations include sharing the GPU) and with one
# batch in flight (the isolated durations of roofline_isolated); no side configs, no CPU leg
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 $R/bench.py --no-cpu --no-configs --no-iso --steps 9 --warmup 0 > $O/prof_bench.json 2> $O/prof_bench.err || { echo "rocprof failed"; tail -30 $O/prof_bench.err; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_iso -o run -- python3 $R/bench.py --no-cpu --no-configs --no-iso --steps 6 --warmup 0 --inflight 1 --sync-verdict > $O/prof_bench_iso.json 2> $O/prof_bench_iso.err || { echo "rocprof iso failed"; tail -30 $O/prof_bench_iso.err; exit 1; }
cd $R && python3 tools/rocpd_stats.py $O/prof/run_results.db $O/kernel_stats.csv && python3 tools/rocpd_stats.py $O/prof_iso/run_results.db $O/kernel_stats_isolated.csv
