set -o pipefail
O=gpurun_out/r04y; mkdir -p $O
for rep in ${REPS:-1 2}; do for inf in ${DEPTHS:-3 4 5 6}; do
  timeout -k 10 200 python3 -u bench.py --no-cpu --no-configs --no-iso --inflight $inf --steps 20 > $O/b64_if${inf}_$rep.json 2> $O/b64_if${inf}_$rep.err || { echo "bench $inf failed"; tail -20 $O/b64_if${inf}_$rep.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/b64_if${inf}_$rep.json')); print('64k inflight $inf rep $rep', round(d['ms_per_step'],3), 'ms/step', round(d['value']), 'proofs/s')"
done; done
