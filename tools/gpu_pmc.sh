#!/bin/bash
# PMC passes over a short bench run (one pass per counter group, each under its own timeout).
# Usage (repo root on the box): bash tools/gpu_pmc.sh TAG
set -o pipefail
TAG=${1:-pmc}
R=$(pwd)
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY" \
           "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_WAIT_INST_LDS SQ_INSTS_BRANCH SQ_ACTIVE_INST_LDS" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d $O/p$i -o run -- python3 $R/bench.py --no-cpu --no-configs --steps 1 --warmup 0 --inflight 1 > $O/p$i.out 2> $O/p$i.err || { echo "pass $i failed"; tail -5 $O/p$i.err; exit 1; }
done
python3 $R/tools/pmc_summary.py $O/p1 $O/p2 $O/p3 $O/p4 > $O/pmc_summary.txt && python3 $R/tools/pmc_traffic.py $O/p3 $O/p4 > $O/pmc_traffic.json && echo ok
