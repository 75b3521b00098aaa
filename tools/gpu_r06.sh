#!/bin/bash
# Round-6 GPU pass: gpu tests, smoke, the driver's bench command (timed), optionally rocprofv3
# kernel stats of the bench. Usage (repo root on the box): bash tools/gpu_r06.sh TAG [tests|bench|prof]...
set -o pipefail
TAG=${1:-r06}
shift
STEPS=${*:-tests bench}
R=$(pwd)
O=$R/gpurun_out/$TAG
mkdir -p $O
nproc > $O/host.txt; grep -m1 "model name" /proc/cpuinfo >> $O/host.txt; echo "OMP=$OMP_NUM_THREADS" >> $O/host.txt
for s in $STEPS; do
  case $s in
  tests)
    timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -60 $O/gpu_tests.log; exit 1; }
    tail -3 $O/gpu_tests.log
    timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $O/smoke.log; exit 1; }
    tail -1 $O/smoke.log ;;
  bench)
    t0=$(date +%s.%N)
    timeout -k 10 500 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -30 $O/bench.err; exit 1; }
    t1=$(date +%s.%N)
    echo "driver bench wall s: $(python3 -c "print($t1-$t0)")" | tee $O/bench_wall.txt
    python3 -c "import json; d=json.load(open('$O/bench.json')); print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['phase_ms'])" ;;
  mb)
    # f-chain microbenchmark variants (tools/mb_fchain.hip, built on the CPU side): same hash = same nodes
    for v in tools/mb_fchain tools/mb_fchain_*; do
      [ -x "$v" ] || continue
      case "$v" in *.hip) continue ;; esac
      echo "== $v" >> $O/mb.txt
      timeout -k 10 60 ./$v 65536 3 >> $O/mb.txt 2>&1 || { echo "mb $v failed"; tail -20 $O/mb.txt; exit 1; }
    done
    cat $O/mb.txt ;;
  lanetest)
    timeout -k 10 400 python -u -m pytest tests/test_gpu_fused.py tests/test_gpu_parity.py -m gpu -x -v --timeout 200 --timeout-method thread > $O/lanetest.log 2>&1 || { echo "lane tests failed"; tail -40 $O/lanetest.log; exit 1; }
    tail -3 $O/lanetest.log ;;
  wave8k)
    # 8k shards (the 8-GPU per-rank size), 6 batches in flight: kernel trace -> wave-time shares
    cd /tmp && export TMPDIR=/tmp
    timeout -k 10 300 rocprofv3 --kernel-trace -d $O/prof8k -o run -- python3 $R/bench.py --no-cpu --no-configs --no-iso --proofs 8192 --steps 36 --warmup 6 > $O/prof8k.json 2> $O/prof8k.err || { echo "rocprof 8k failed"; tail -30 $O/prof8k.err; exit 1; }
    cd $R && python3 tools/wavetime.py $O/prof8k/run_results.db $O/wavetime_8k.txt > /dev/null && rm -f $O/prof8k/run_results.db && head -30 $O/wavetime_8k.txt ;;
  configs)
    # the driver's default bench line incl. config 2 / config 4 side lines (no CPU leg)
    timeout -k 10 400 python3 -u bench.py --no-cpu > $O/bench_configs.json 2> $O/bench_configs.err || { echo "bench configs failed"; tail -30 $O/bench_configs.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/bench_configs.json')); print({k: d[k] for k in d if 'config' in k.lower() or k in ('value','ms_per_step')})" ;;
  env8k)
    # 8k-shard bench (6 in flight) under alternative knobs: ENVS="A=1,B=2 C=3 ..." (comma = same run)
    for cfg in default ${ENVS:-}; do
      envs=""; [ "$cfg" != default ] && envs=$(echo $cfg | tr ',' ' ')
      env $envs timeout -k 10 200 python3 -u bench.py --no-cpu --no-configs --no-iso --proofs 8192 --steps 40 > $O/b8k_$cfg.json 2> $O/b8k_$cfg.err || { echo "bench 8k $cfg failed"; tail -20 $O/b8k_$cfg.err; exit 1; }
      python3 -c "import json; d=json.load(open('$O/b8k_$cfg.json')); print('8k $cfg', round(d['ms_per_step'],3), 'ms/batch', round(d['value']), 'proofs/s')"
    done ;;
  envab)
    # A/B of knobs over shard sizes, back to back: ENVS as env8k, SHARDS="65536 8192"
    for n in ${SHARDS:-65536 8192}; do for cfg in default ${ENVS:-}; do
      envs=""; [ "$cfg" != default ] && envs=$(echo $cfg | tr ',' ' ')
      env $envs timeout -k 10 200 python3 -u bench.py --no-cpu --no-configs --no-iso --proofs $n --steps 40 > $O/ab_${n}_$cfg.json 2> $O/ab_${n}_$cfg.err || { echo "bench ab $n $cfg failed"; tail -20 $O/ab_${n}_$cfg.err; exit 1; }
      python3 -c "import json; d=json.load(open('$O/ab_${n}_$cfg.json')); print('$cfg shard $n', round(d['ms_per_step'],3), 'ms/batch', round(d['value']), 'proofs/s', {k: round(v,3) for k,v in d.get('phase_ms', {}).items()})"
    done; done ;;
  inflight8k)
    # 8k shards at several batches-in-flight depths
    for inf in ${DEPTHS:-4 6 8 10}; do
      timeout -k 10 200 python3 -u bench.py --no-cpu --no-configs --no-iso --proofs 8192 --inflight $inf --steps 40 > $O/b8k_if$inf.json 2> $O/b8k_if$inf.err || { echo "bench 8k inflight $inf failed"; tail -20 $O/b8k_if$inf.err; exit 1; }
      python3 -c "import json; d=json.load(open('$O/b8k_if$inf.json')); print('8k inflight $inf', round(d['ms_per_step'],3), 'ms/batch', round(d['value']), 'proofs/s')"
    done ;;
  pmcsize)
    # VALU instructions per batch by kernel, 64k (4 in flight) and 8k (6 in flight), one --pmc pass each
    cd /tmp && export TMPDIR=/tmp
    for cfg in "65536 4 8" "8192 6 36"; do
      set -- $cfg
      timeout -s KILL 200 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES --output-format csv -d $O/pmc_$1 -o run -- python3 $R/bench.py --no-cpu --no-configs --no-iso --proofs $1 --inflight $2 --steps $3 --warmup 0 > $O/pmc_$1.out 2> $O/pmc_$1.err || { echo "pmc $1 failed"; tail -5 $O/pmc_$1.err; exit 1; }
      # batches verified = timed steps + the warmup-free pipeline's own checks (steps + inflight drained)
      python3 $R/tools/pmc_per_batch.py $O/pmc_$1 $3 > $O/pmc_per_batch_$1.txt && head -16 $O/pmc_per_batch_$1.txt
    done
    cd $R ;;
  quick)
    timeout -k 10 200 python3 -u bench.py --no-cpu --no-configs > $O/bench_quick.json 2> $O/bench_quick.err || { echo "bench quick failed"; tail -30 $O/bench_quick.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/bench_quick.json')); print('64k', d['value'], d['ms_per_step'], d['roofline']['frac'], {k: round(v,3) for k,v in d['roofline']['phase_ms'].items()})"
    timeout -k 10 200 python -u bench.py --no-cpu --no-configs --proofs 8192 > $O/bench_8192.json 2> $O/bench_8192.err || { echo "bench 8192 failed"; tail -30 $O/bench_8192.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/bench_8192.json')); print('8k', round(d['ms_per_step'],3), 'ms/batch', round(d['value']), 'proofs/s')" ;;
  lanes)
    for v in 0 1 2; do
      ZG_LINES_LANE=$v timeout -k 10 200 python3 -u bench.py --no-cpu --no-configs > $O/bench_lanes$v.json 2> $O/bench_lanes$v.err || { echo "bench lanes $v failed"; tail -30 $O/bench_lanes$v.err; exit 1; }
      python3 -c "import json; d=json.load(open('$O/bench_lanes$v.json')); print('lines_lane $v', round(d['value']), round(d['ms_per_step'],3), {k: round(v,3) for k,v in d['roofline']['phase_ms'].items()})"
    done ;;
  lanes8k)
    for n in 8192 16384; do for v in 0 1; do
      ZG_LINES_LANE=$v timeout -k 10 200 python3 -u bench.py --no-cpu --no-configs --no-iso --proofs $n > $O/bench_l$v_$n.json 2> $O/bench_l$v_$n.err || { echo "bench lanes $v $n failed"; tail -30 $O/bench_l$v_$n.err; exit 1; }
      python3 -c "import json; d=json.load(open('$O/bench_l$v_$n.json')); print('n $n lines_lane $v', round(d['value']), round(d['ms_per_step'],3), {k: round(v,3) for k,v in d['phase_ms'].items()})"
    done; done ;;
  prof)
    cd /tmp && export TMPDIR=/tmp
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 $R/bench.py --no-cpu --no-configs --no-iso --steps 9 --warmup 0 > $O/prof_bench.json 2> $O/prof_bench.err || { echo "rocprof failed"; tail -30 $O/prof_bench.err; exit 1; }
    ZG_SERIAL_SIDE=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_iso -o run -- python3 $R/bench.py --no-cpu --no-configs --no-iso --steps 6 --warmup 0 --inflight 1 --sync-verdict > $O/prof_bench_iso.json 2> $O/prof_bench_iso.err || { echo "rocprof iso failed"; tail -30 $O/prof_bench_iso.err; exit 1; }
    cd $R && for k in prof prof_iso; do python3 tools/rocpd_stats.py $O/$k/run_results.db $O/kernel_stats_${k#prof}.csv; done ;;
  variants)
    for v in $VARIANTS; do
      ZG_LIB_VARIANT=$v timeout -k 10 200 python3 -u bench.py --no-cpu --no-configs > $O/bench_$v.json 2> $O/bench_$v.err || { echo "bench $v failed"; tail -30 $O/bench_$v.err; exit 1; }
      python3 -c "import json; d=json.load(open('$O/bench_$v.json')); print('$v 64k', round(d['value']), round(d['ms_per_step'],3), {k: round(v,3) for k,v in d['roofline']['phase_ms'].items()})"
    done ;;
  pghr)
    for n in 65536 8192; do
      timeout -k 10 200 python3 -u tools/bench_pghr13.py --no-cpu --n $n > $O/pghr_$n.json 2> $O/pghr_$n.err || { echo "pghr bench failed"; tail -30 $O/pghr_$n.err; exit 1; }
      cat $O/pghr_$n.json
    done
    cd /tmp && export TMPDIR=/tmp
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_pghr -o run -- python3 $R/tools/bench_pghr13.py --no-cpu --reps 2 > /dev/null 2> $O/prof_pghr.err || { echo "rocprof pghr failed"; tail -30 $O/prof_pghr.err; exit 1; }
    cd $R && python3 tools/rocpd_stats.py $O/prof_pghr/run_results.db $O/kernel_stats_pghr.csv && python3 tools/timeline.py $O/prof_pghr/run_results.db k_pghr_decode_g1 $O/pghr_timeline.txt > /dev/null && rm -f $O/prof_pghr/run_results.db ;;
  pghrvar)
    for v in $VARIANTS; do for n in 65536 8192; do
      ZG_LIB_VARIANT=$v timeout -k 10 200 python3 -u tools/bench_pghr13.py --no-cpu --n $n > $O/pghr_${v}_$n.json 2> $O/pghr_${v}_$n.err || { echo "pghr bench $v failed"; tail -30 $O/pghr_${v}_$n.err; exit 1; }
      echo "$v $(cat $O/pghr_${v}_$n.json)"
    done; done ;;
  pghrk)
    for v in main $VARIANTS; do for k in ${KS:-1 2 4 8}; do
      lv=$v; [ $v = main ] && lv=
      ZG_LIB_VARIANT=$lv ZG_BSEG_K=$k timeout -k 10 200 python3 -u tools/bench_pghr13.py --no-cpu --n 65536 > $O/pghrk_${v}_$k.json 2> $O/pghrk_${v}_$k.err || { echo "pghr bench $v $k failed"; tail -30 $O/pghrk_${v}_$k.err; exit 1; }
      echo "$v K=$k $(cat $O/pghrk_${v}_$k.json)"
    done; done ;;
  pghrb)
    for b in 1 2 4; do for n in 65536 8192; do
      ZG_STRAUS_B=$b timeout -k 10 200 python3 -u tools/bench_pghr13.py --no-cpu --n $n > $O/pghrb_${b}_$n.json 2> $O/pghrb_${b}_$n.err || { echo "pghr bench B=$b failed"; tail -30 $O/pghrb_${b}_$n.err; exit 1; }
      echo "B=$b $(cat $O/pghrb_${b}_$n.json)"
    done; done ;;
  pghr8k)
    cd /tmp && export TMPDIR=/tmp
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_pghr8k -o run -- python3 $R/tools/bench_pghr13.py --no-cpu --n 8192 --reps 2 > /dev/null 2> $O/prof_pghr8k.err || { echo "rocprof pghr 8k failed"; tail -30 $O/prof_pghr8k.err; exit 1; }
    cd $R && python3 tools/timeline.py $O/prof_pghr8k/run_results.db k_pghr_decode_g1 $O/pghr8k_timeline.txt > /dev/null && rm -f $O/prof_pghr8k/run_results.db ;;
  pghrtests)
    timeout -k 10 600 python -u -m pytest tests/test_gpu_pghr13.py tests/test_collector.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests_pghr.log 2>&1 || { echo "gpu pghr tests failed"; tail -60 $O/gpu_tests_pghr.log; exit 1; }
    tail -3 $O/gpu_tests_pghr.log ;;
  c2trace)
    timeout -k 10 200 python3 -u tools/config2_trace.py > $O/c2.json 2> $O/c2.err || { echo "config2 failed"; tail -30 $O/c2.err; exit 1; }
    cat $O/c2.json
    cd /tmp && export TMPDIR=/tmp
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_c2 -o run -- python3 $R/tools/config2_trace.py > $O/prof_c2.json 2> $O/prof_c2.err || { echo "rocprof c2 failed"; tail -30 $O/prof_c2.err; exit 1; }
    cd $R && python3 tools/timeline.py $O/prof_c2/run_results.db k_chacha20 $O/c2_timeline.txt > /dev/null && python3 tools/rocpd_stats.py $O/prof_c2/run_results.db $O/kernel_stats_c2.csv && rm -f $O/prof_c2/run_results.db ;;
  bisect)
    for B in 512 1024 2048; do
      ZG_BISECT_BUDGET=$B timeout -k 10 300 python3 -u tools/small_batch.py 3 > $O/small_b$B.json 2> $O/small_b$B.err || { echo "small batch $B failed"; tail -30 $O/small_b$B.err; exit 1; }
      python3 -c "import json; d=[json.loads(l) for l in open('$O/small_b$B.json') if l.startswith('{')]; print('budget $B', [(r['cap'], round(r['config2_1024_spends']['ms_per_batch'],2), round(r['config4_4096_1pct_corrupted']['ms_per_batch'],2), r['config4_4096_1pct_corrupted']['exact_reject_set'], r['stats']['bisect_nodes']) for r in d])"
    done ;;
  prof8k)
    cd /tmp && export TMPDIR=/tmp
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof8k -o run -- python3 $R/bench.py --no-cpu --no-configs --no-iso --proofs 8192 --steps 36 --warmup 0 > $O/prof8k_bench.json 2> $O/prof8k_bench.err || { echo "rocprof 8k failed"; tail -30 $O/prof8k_bench.err; exit 1; }
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof8k_iso -o run -- python3 $R/bench.py --no-cpu --no-configs --no-iso --proofs 8192 --steps 6 --warmup 0 --inflight 1 --sync-verdict > $O/prof8k_bench_iso.json 2> $O/prof8k_bench_iso.err || { echo "rocprof 8k iso failed"; tail -30 $O/prof8k_bench_iso.err; exit 1; }
    cd $R && for k in prof8k prof8k_iso; do python3 tools/rocpd_stats.py $O/$k/run_results.db $O/kernel_stats_${k}.csv; done ;;
  shards)
    # per-rank shard sizes of the 1/2/4/8-GPU curve (default batches in flight), one run each
    for n in ${SHARDS:-8192 16384 32768}; do
      timeout -k 10 200 python3 -u bench.py --no-cpu --no-configs --no-iso --proofs $n --steps 40 > $O/b_$n.json 2> $O/b_$n.err || { echo "bench $n failed"; tail -20 $O/b_$n.err; exit 1; }
      python3 -c "import json; d=json.load(open('$O/b_$n.json')); print('shard $n', round(d['ms_per_step'],3), 'ms/batch', round(d['value']), 'proofs/s', d['config'].get('batches_in_flight_per_gpu'))"
    done ;;
  hwq8k)
    # 8k shards (6 in flight) at several hardware-queue counts x stream-pair pools: "Q:P ..."
    for cfg in ${HWQ:-24:8 16:8 12:6 8:4 32:8}; do
      q=${cfg%%:*}; pp=${cfg##*:}
      GPU_MAX_HW_QUEUES=$q ZG_STREAM_PAIRS=$pp ZG_BENCH_HWQ=$q timeout -k 10 200 python3 -u bench.py --no-cpu --no-configs --no-iso --proofs ${HWQN:-8192} --steps 40 > $O/hwq_$q_$pp.json 2> $O/hwq_$q_$pp.err || { echo "bench hwq $cfg failed"; tail -20 $O/hwq_$q_$pp.err; exit 1; }
      python3 -c "import json; d=json.load(open('$O/hwq_$q_$pp.json')); print('hwq $cfg', round(d['ms_per_step'],3), 'ms/batch', round(d['value']), 'proofs/s')"
    done ;;
  pipetest)
    timeout -k 10 600 python -u -m pytest tests/test_gpu_pipeline.py tests/test_gpu_multiproc.py tests/test_gpu_rccl.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/pipetest.log 2>&1 || { echo "pipeline tests failed"; tail -60 $O/pipetest.log; exit 1; }
    tail -3 $O/pipetest.log ;;
  mbaff)
    # affine vs projective R-chain step cost (tools/mb_affine.hip, built on the CPU side)
    timeout -k 10 120 ./tools/mb_affine 65536 16 > $O/mb_affine.txt 2>&1 || { echo "mb_affine failed"; cat $O/mb_affine.txt; exit 1; }
    cat $O/mb_affine.txt ;;
  k4tests)
    timeout -k 10 600 python -u -m pytest tests/test_gpu_csum.py tests/test_gpu_configs.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/k4tests.log 2>&1 || { echo "k4 tests failed"; tail -60 $O/k4tests.log; exit 1; }
    tail -3 $O/k4tests.log ;;
  occ8k)
    # 8k shards in flight: wave-time by kernel, resident waves over time, per-stream gaps (tools/occupancy.py)
    cd /tmp && export TMPDIR=/tmp
    timeout -k 10 300 rocprofv3 --kernel-trace ${PROFARGS:-} -d $O/occ8k -o run -- python3 $R/bench.py --no-cpu --no-configs --no-iso --proofs ${OCCN:-8192} --steps 36 --warmup 6 ${OCCARGS:-} > $O/occ8k.json 2> $O/occ8k.err || { echo "rocprof occ failed"; tail -30 $O/occ8k.err; exit 1; }
    cd $R && python3 tools/wavetime.py $O/occ8k/run_results.db $O/wavetime_occ.txt > /dev/null && python3 tools/occupancy.py $O/occ8k/run_results.db $O/occupancy.txt > $O/occupancy_stdout.txt && python3 tools/batch_path.py $O/occ8k/run_results.db $O/batch_path.txt > /dev/null && head -12 $O/occupancy.txt && head -40 $O/batch_path.txt && head -12 $O/wavetime_occ.txt && { [ -z "${PROFARGS:-}" ] || python3 tools/host_api.py $O/occ8k/run_results.db $O/host_api.txt > /dev/null; } && { [ -n "${KEEPDB:-}" ] || rm -f $O/occ8k/run_results.db; } ;;
  abiso)
    # A/B of knobs with the isolated pass (the kernels alone after the timed region): ENVS as envab, SHARDS
    for n in ${SHARDS:-65536}; do for cfg in default ${ENVS:-}; do
      envs=""; [ "$cfg" != default ] && envs=$(echo $cfg | tr ',' ' ')
      env $envs timeout -k 10 240 python3 -u bench.py --no-cpu --no-configs --proofs $n --steps 30 > $O/abiso_${n}_$cfg.json 2> $O/abiso_${n}_$cfg.err || { echo "bench abiso $n $cfg failed"; tail -20 $O/abiso_${n}_$cfg.err; exit 1; }
      python3 -c "import json; d=json.load(open('$O/abiso_${n}_$cfg.json')); r=d['roofline']; print('$cfg shard $n', round(d['ms_per_step'],3), 'ms/batch', round(d['value']), 'proofs/s; iso', {k: round(v,3) for k,v in r['phase_ms'].items()})"
    done; done ;;
  afftest)
    timeout -k 10 600 python -u -m pytest tests/test_gpu_affine.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/afftest.log 2>&1 || { echo "affine tests failed"; tail -60 $O/afftest.log; exit 1; }
    tail -3 $O/afftest.log ;;
  benchcfg)
    # the driver's default command plus the side lines (config 2 / 4 / clean 4,096 / config 5, f3, f4, CPU legs)
    timeout -k 10 600 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_full.json 2> $O/bench_full.err || { echo "bench full failed"; tail -30 $O/bench_full.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/bench_full.json')); print(d['value'], d['ms_per_step']); oc=d['other_configs']; print({k: (round(v['ms_per_batch'],3) if isinstance(v, dict) and 'ms_per_batch' in v else v) for k, v in oc.items() if k != 'config5_replay'}); print(json.dumps(oc['config5_replay']))" ;;
  ckab)
    # verdict threads (bench.py --checkers) at 8k and 64k shards, and the K4 / latency-priority variants (isolated K4)
    for n in ${SHARDS:-8192 65536}; do for ck in 1 2; do
      timeout -k 10 240 python3 -u bench.py --no-cpu --no-configs --proofs $n --steps 40 --checkers $ck > $O/ck_${n}_$ck.json 2> $O/ck_${n}_$ck.err || { echo "bench ck $n $ck failed"; tail -20 $O/ck_${n}_$ck.err; exit 1; }
      python3 -c "import json; d=json.load(open('$O/ck_${n}_$ck.json')); print('checkers $ck shard $n', round(d['ms_per_step'],3), 'ms/batch', round(d['value']), 'verdict ms', round(d['host_ms_per_batch']['exchange_and_final_exp'],3), 'k4 iso', round(d['k4_msm_bucket_phase']['k4_total_ms'],3))"
    done; done ;;
  varab)
    # library variants (ZG_LIB_VARIANT, tools/build_variant.py) against the default, in flight + isolated K4
    for n in ${SHARDS:-8192 65536}; do for v in default $VARIANTS; do
      lv=$v; [ $v = default ] && lv=
      ZG_LIB_VARIANT=$lv timeout -k 10 240 python3 -u bench.py --no-cpu --no-configs --proofs $n --steps 40 > $O/var_${n}_$v.json 2> $O/var_${n}_$v.err || { echo "bench var $n $v failed"; tail -20 $O/var_${n}_$v.err; exit 1; }
      python3 -c "import json; d=json.load(open('$O/var_${n}_$v.json')); r=d['roofline']; print('$v shard $n', round(d['ms_per_step'],3), 'ms/batch', round(d['value']), 'verdict ms', round(d['host_ms_per_batch']['exchange_and_final_exp'],3), 'k4 iso', round(d['k4_msm_bucket_phase']['k4_total_ms'],3), 'iso', {k: round(v,3) for k,v in r['phase_ms'].items()})"
    done; done ;;
  depths)
    # batches in flight by shard size: DEPTHS_<n>="6 8 ..." (default "6 8")
    for n in ${SHARDS:-8192 65536}; do
      eval ds=\${DEPTHS_$n:-"6 8"}
      for inf in $ds; do
        timeout -k 10 200 python3 -u bench.py --no-cpu --no-configs --no-iso --proofs $n --inflight $inf --steps 40 > $O/d_${n}_$inf.json 2> $O/d_${n}_$inf.err || { echo "bench depth $n $inf failed"; tail -20 $O/d_${n}_$inf.err; exit 1; }
        python3 -c "import json; d=json.load(open('$O/d_${n}_$inf.json')); print('shard $n inflight $inf', round(d['ms_per_step'],3), 'ms/batch', round(d['value']), 'proofs/s hwq', d['config']['hw_queues'])"
      done
    done ;;
  preptest)
    timeout -k 10 600 python -u -m pytest tests/test_gpu_prep_batch.py tests/test_collector.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/preptest.log 2>&1 || { echo "prep tests failed"; tail -60 $O/preptest.log; exit 1; }
    tail -3 $O/preptest.log ;;
  config5)
    timeout -k 10 300 python3 -u tools/run_config5.py ${C5ARGS:-} > $O/config5.json 2> $O/config5.err || { echo "config5 failed"; tail -30 $O/config5.err; exit 1; }
    cat $O/config5.json ;;
  distq)
    # the RCCL path at world size 1 (bench.py --dist) by hardware-queue count: "N:Q ..." (shard N, queues Q; 0 = bench default)
    for cfg in ${DISTQ:-8192:0 8192:28 8192:32 65536:0}; do
      n=${cfg%%:*}; q=${cfg##*:}; ex=""; [ "$q" != 0 ] && ex="ZG_BENCH_HWQ=$q"
      env $ex timeout -k 10 240 python3 -u bench.py --dist --no-cpu --no-configs --no-iso --proofs $n --steps 40 > $O/dq_${n}_$q.json 2> $O/dq_${n}_$q.err || { echo "bench dist $cfg failed"; tail -20 $O/dq_${n}_$q.err; exit 1; }
      python3 -c "import json; d=json.load(open('$O/dq_${n}_$q.json')); print('dist shard $n hwq', d['config']['hw_queues'], round(d['ms_per_step'],3), 'ms/batch', round(d['value']), 'proofs/s', d['config']['batches_in_flight_per_gpu'], 'in flight; verdict ms', round(d['host_ms_per_batch']['exchange_and_final_exp'],3))"
    done ;;
  distx)
    # the per-batch exchange at world size 1 under --dist: RCCL (with / without priority streams) vs no --dist
    for n in ${SHARDS:-8192 65536}; do for x in nodist rccl rcclnp; do
      case $x in nodist) a="";; rccl) a="--dist";; rcclnp) a="--dist --no-priority";; esac
      timeout -k 10 240 python3 -u bench.py $a --no-cpu --no-configs --no-iso --proofs $n --steps 40 > $O/dx_${n}_$x.json 2> $O/dx_${n}_$x.err || { echo "bench distx $n $x failed"; tail -20 $O/dx_${n}_$x.err; exit 1; }
      python3 -c "import json; d=json.load(open('$O/dx_${n}_$x.json')); print('$x shard $n', round(d['ms_per_step'],3), 'ms/batch', round(d['value']), 'proofs/s; verdict ms', round(d['host_ms_per_batch']['exchange_and_final_exp'],3), d['config']['collective'][:40])"
    done; done ;;
  distcpu)
    # CPUs the bench process keeps busy in the timed region, --dist vs not
    for n in ${SHARDS:-8192}; do for x in nodist rccl; do
      a=""; [ $x = rccl ] && a="--dist"
      timeout -k 10 240 python3 -u bench.py $a --no-cpu --no-configs --no-iso --proofs $n --steps 100 > $O/dc_${n}_$x.json 2> $O/dc_${n}_$x.err || { echo "bench distcpu $n $x failed"; tail -20 $O/dc_${n}_$x.err; exit 1; }
      python3 -c "import json; d=json.load(open('$O/dc_${n}_$x.json')); print('$x shard $n', round(d['ms_per_step'],3), 'ms/batch; CPUs busy', round(d['host_ms_per_batch']['process_cpus_busy'],2))"
    done; done ;;
  distp)
    # stream priorities under --dist (world 1), repeated: nodist / RCCL+checkers high / RCCL normal / all normal
    for rep in 1 2; do for n in ${SHARDS:-8192 65536}; do for x in nodist hi rnorm allnorm; do
      case $x in nodist) a="";; hi) a="--dist";; rnorm) a="--dist --rccl-priority normal";; allnorm) a="--dist --no-priority";; esac
      timeout -k 10 240 python3 -u bench.py $a --no-cpu --no-configs --no-iso --proofs $n --steps 60 > $O/dp_${n}_${x}_$rep.json 2> $O/dp_${n}_${x}_$rep.err || { echo "bench distp $n $x failed"; tail -20 $O/dp_${n}_${x}_$rep.err; exit 1; }
      python3 -c "import json; d=json.load(open('$O/dp_${n}_${x}_$rep.json')); print('rep $rep $x shard $n', round(d['ms_per_step'],3), 'ms/batch; verdict ms', round(d['host_ms_per_batch']['exchange_and_final_exp'],3))"
    done; done; done ;;
  distp2)
    # under --dist (world 1), repeated: default / one checker / default-priority exchange stream / 32 queues / all normal + 1 checker
    for rep in 1 2; do for n in ${SHARDS:-8192 32768}; do for x in hi ck1 xnorm q32 norm1; do
      e=""; a="--dist"
      case $x in ck1) a="--dist --checkers 1";; xnorm) e="ZG_XSTREAM_PRIO=0";; q32) e="ZG_BENCH_HWQ=32";; norm1) a="--dist --no-priority --checkers 1";; esac
      env $e timeout -k 10 240 python3 -u bench.py $a --no-cpu --no-configs --no-iso --proofs $n --steps 60 > $O/dq_${n}_${x}_$rep.json 2> $O/dq_${n}_${x}_$rep.err || { echo "bench distp2 $n $x failed"; tail -20 $O/dq_${n}_${x}_$rep.err; exit 1; }
      python3 -c "import json; d=json.load(open('$O/dq_${n}_${x}_$rep.json')); print('rep $rep $x shard $n', round(d['ms_per_step'],3), 'ms/batch; verdict ms', round(d['host_ms_per_batch']['exchange_and_final_exp'],3))"
    done; done; done ;;
  ck8k)
    # checkers 1 vs 2, with and without --dist, repeated (same box)
    for rep in 1 2 3; do for n in ${SHARDS:-8192}; do for x in n1 n2 d1 d2; do
      case $x in n1) a="--checkers 1";; n2) a="--checkers 2";; d1) a="--dist --checkers 1";; d2) a="--dist --checkers 2";; esac
      timeout -k 10 240 python3 -u bench.py $a --no-cpu --no-configs --no-iso --proofs $n --steps 60 > $O/ck_${n}_${x}_$rep.json 2> $O/ck_${n}_${x}_$rep.err || { echo "bench ck8k $n $x failed"; tail -20 $O/ck_${n}_${x}_$rep.err; exit 1; }
      python3 -c "import json; d=json.load(open('$O/ck_${n}_${x}_$rep.json')); print('rep $rep $x shard $n', round(d['ms_per_step'],3), 'ms/batch; verdict ms', round(d['host_ms_per_batch']['exchange_and_final_exp'],3))"
    done; done; done ;;
  coal)
    # the coalescing checker (--coalesce on: gt_check_many) against the checker pool, single process and
    # under --dist, alternating on one box
    for rep in 1 2 3; do for n in ${SHARDS:-8192 65536}; do for x in n2 nc d1 dc; do
      case $x in n2) a="--checkers 2";; nc) a="--coalesce on";; d1) a="--dist --checkers 1";; dc) a="--dist --coalesce on";; esac
      timeout -k 10 240 python3 -u bench.py $a --no-cpu --no-configs --no-iso --proofs $n --steps 60 > $O/co_${n}_${x}_$rep.json 2> $O/co_${n}_${x}_$rep.err || { echo "bench coal $n $x failed"; tail -20 $O/co_${n}_${x}_$rep.err; exit 1; }
      python3 -c "import json; d=json.load(open('$O/co_${n}_${x}_$rep.json')); print('rep $rep $x shard $n', round(d['ms_per_step'],3), 'ms/batch; verdict ms', round(d['host_ms_per_batch']['exchange_and_final_exp'],3), '|', d['config']['verdict'])"
    done; done; done ;;
  coprio)
    # the coalescing checker at the default stream priority (--no-priority) vs high, single process and --dist
    for rep in 1 2 3; do for n in ${SHARDS:-8192 65536}; do for x in n2 nc ncl dc dcl; do
      case $x in n2) a="--checkers 2";; nc) a="--coalesce on";; ncl) a="--coalesce on --no-priority";; dc) a="--dist";; dcl) a="--dist --no-priority";; esac
      timeout -k 10 240 python3 -u bench.py $a --no-cpu --no-configs --no-iso --proofs $n --steps 60 > $O/cp_${n}_${x}_$rep.json 2> $O/cp_${n}_${x}_$rep.err || { echo "bench coprio $n $x failed"; tail -20 $O/cp_${n}_${x}_$rep.err; exit 1; }
      python3 -c "import json; d=json.load(open('$O/cp_${n}_${x}_$rep.json')); print('rep $rep $x shard $n', round(d['ms_per_step'],3), 'ms/batch')"
    done; done; done ;;
  depthco)
    # batches in flight with the coalescing checker under --dist (and 64k single process), two repeats
    for rep in 1 2; do for cfg in "8192 6" "8192 8" "8192 10" "16384 6" "16384 8" "65536 5" "65536 6" "65536 7"; do
      set -- $cfg; n=$1; d=$2
      for x in rccl nodist; do
        [ $x = nodist ] && [ $n != 65536 ] && continue
        a=""; [ $x = rccl ] && a="--dist"
        timeout -k 10 240 python3 -u bench.py $a --inflight $d --no-cpu --no-configs --no-iso --proofs $n --steps 60 > $O/dc_${n}_${d}_${x}_$rep.json 2> $O/dc_${n}_${d}_${x}_$rep.err || { echo "bench depthco $n $d $x failed"; tail -20 $O/dc_${n}_${d}_${x}_$rep.err; exit 1; }
        python3 -c "import json; d=json.load(open('$O/dc_${n}_${d}_${x}_$rep.json')); print('rep $rep $x shard $n inflight $d', round(d['ms_per_step'],3), 'ms/batch')"
      done
    done; done ;;
  distshards)
    # per-rank shard sizes of the 2/4/8-GPU line under --dist (world 1) against the single-process run, two repeats
    for rep in 1 2; do for n in ${SHARDS:-8192 16384 32768}; do for x in nodist rccl; do
      a=""; [ $x = rccl ] && a="--dist"
      timeout -k 10 240 python3 -u bench.py $a --no-cpu --no-configs --no-iso --proofs $n --steps 60 > $O/ds_${n}_${x}_$rep.json 2> $O/ds_${n}_${x}_$rep.err || { echo "bench distshards $n $x failed"; tail -20 $O/ds_${n}_${x}_$rep.err; exit 1; }
      python3 -c "import json; d=json.load(open('$O/ds_${n}_${x}_$rep.json')); print('rep $rep $x shard $n', round(d['ms_per_step'],3), 'ms/batch', round(d['value']), 'proofs/s;', d['config']['batches_in_flight_per_gpu'], 'in flight')"
    done; done; done ;;
  esac
done
