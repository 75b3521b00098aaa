#!/bin/bash
# Round-2 GPU pass: gpu tests; the driver's bench command, timed; the configuration that used to
# abort (8,192-proof shards, 8 batches in flight + the checker = 9 slots); rocprofv3 kernel stats.
# Usage (repo root on the box): bash tools/gpu_r02.sh TAG [skip_tests]
set -o pipefail
TAG=${1:-r02}
R=$(pwd)
O=$R/gpurun_out/$TAG
mkdir -p $O
nproc > $O/host.txt; grep -m1 "model name" /proc/cpuinfo >> $O/host.txt; echo "OMP=$OMP_NUM_THREADS" >> $O/host.txt
if [ -z "$2" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -40 $O/gpu_tests.log; exit 1; }
  tail -3 $O/gpu_tests.log
  timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $O/smoke.log; exit 1; }
  tail -1 $O/smoke.log
fi
t0=$(date +%s.%N)
timeout -k 10 500 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -30 $O/bench.err; exit 1; }
t1=$(date +%s.%N)
echo "driver bench wall s: $(python3 -c "print($t1-$t0)")" | tee $O/bench_wall.txt
cat $O/bench.json
timeout -k 10 200 python -u bench.py --no-cpu --no-configs --proofs 8192 --inflight 8 > $O/bench_8192_if8.json 2> $O/bench_8192_if8.err || { echo "bench 8192 x8 failed"; tail -30 $O/bench_8192_if8.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench_8192_if8.json')); print('8192 x8 in flight', round(d['ms_per_step'],3), 'ms/batch', round(d['value']), 'proofs/s', d['context_stats'])"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 $R/bench.py --no-cpu --no-configs --no-iso --steps 9 --warmup 0 > $O/prof_bench.json 2> $O/prof_bench.err || { echo "rocprof failed"; tail -30 $O/prof_bench.err; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_iso -o run -- python3 $R/bench.py --no-cpu --no-configs --no-iso --steps 6 --warmup 0 --inflight 1 --sync-verdict > $O/prof_bench_iso.json 2> $O/prof_bench_iso.err || { echo "rocprof iso failed"; tail -30 $O/prof_bench_iso.err; exit 1; }
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof_tree -o run -- python3 $R/tools/bench_tree.py --no-cpu --reps 5 > $O/prof_tree.json 2> $O/prof_tree.err || { echo "rocprof trees failed"; tail -30 $O/prof_tree.err; exit 1; }
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof_pghr -o run -- python3 $R/tools/bench_pghr13.py --no-cpu --reps 2 > $O/prof_pghr.json 2> $O/prof_pghr.err || { echo "rocprof pghr13 failed"; tail -30 $O/prof_pghr.err; exit 1; }
cd $R && for k in prof prof_iso prof_tree prof_pghr; do python3 tools/rocpd_stats.py $O/$k/run_results.db $O/kernel_stats_${k#prof}.csv; done
