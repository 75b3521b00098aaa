#!/bin/bash
# A/B HBM traffic (FETCH_SIZE, WRITE_SIZE passes) of the main library, a variant and the split decode.
set -o pipefail
R=$(pwd); O=$R/gpurun_out/${TAG:-r04o}; mkdir -p $O; cd /tmp && export TMPDIR=/tmp
for v in ${VARS:-main split}; do
  lv=$v; sp=0
  if [ $v = main ]; then lv=""; fi
  if [ $v = split ]; then lv=""; sp=1; fi
  ZG_DECODE_SPLIT=$sp ZG_LIB_VARIANT=$lv timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/f_$v -o run -- python3 $R/bench.py --no-cpu --no-configs --steps ${STEPS:-1} --warmup 0 --inflight ${INFL:-1} > $O/f_$v.out 2> $O/f_$v.err || { echo "pass $v failed"; tail -5 $O/f_$v.err; exit 1; }
  ZG_DECODE_SPLIT=$sp ZG_LIB_VARIANT=$lv timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/w_$v -o run -- python3 $R/bench.py --no-cpu --no-configs --steps ${STEPS:-1} --warmup 0 --inflight ${INFL:-1} > $O/w_$v.out 2> $O/w_$v.err || { echo "pass w $v failed"; tail -5 $O/w_$v.err; exit 1; }
  python3 $R/tools/pmc_traffic.py $O/f_$v $O/w_$v > $O/traffic_$v.json || exit 1
done
echo ok
