#!/bin/bash
# gpu tests, then config 4 vs a clean 4,096 batch (tools/bisect_bench.py) plain and under rocprofv3.
# Usage (repo root on the box): bash tools/gpu_bisect.sh TAG [skip_tests]
set -o pipefail
TAG=${1:-bisect}
R=$(pwd)
O=$R/gpurun_out/$TAG
mkdir -p $O
if [ -z "$2" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -40 $O/gpu_tests.log; exit 1; }
  tail -3 $O/gpu_tests.log
fi
timeout -k 10 200 python -u tools/bisect_bench.py 5 > $O/bisect.json 2> $O/bisect.err || { echo "bisect bench failed"; tail -30 $O/bisect.err; exit 1; }
cat $O/bisect.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 $R/tools/bisect_bench.py 2 > $O/prof_bisect.json 2> $O/prof_bisect.err || { echo "rocprof failed"; tail -30 $O/prof_bisect.err; exit 1; }
cd $R && python3 tools/rocpd_stats.py $O/prof/run_results.db $O/kernel_stats_bisect.csv && head -20 $O/kernel_stats_bisect.csv | cut -c1-150
