#!/bin/bash
# Staged-words parity boundaries; the bench in the driver's form twice and the default form once
# (compute block: poison before the warmup).
set -o pipefail
TAG=${1:-r3zd}
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -q --timeout 150 --timeout-method thread \
    -p no:cacheprovider -k "staged or held or overlapped_compute" > gpurun_out/${TAG}_parity.txt 2>&1
rc=$?; echo "parity rc=$rc"; tail -2 gpurun_out/${TAG}_parity.txt
[ $rc -eq 0 ] || { grep -E "FAIL|Error" gpurun_out/${TAG}_parity.txt | head; exit $rc; }
for i in 1 2; do
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/${TAG}_bench_k20_$i.json 2> gpurun_out/${TAG}_bench_k20_$i.err \
    || { echo "bench k20 failed"; tail -20 gpurun_out/${TAG}_bench_k20_$i.err; exit 1; }
done
timeout -k 10 300 python3 bench.py --no-pmc > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err \
    || { echo "bench failed"; tail -20 gpurun_out/${TAG}_bench.err; exit 1; }
for f in bench_k20_1 bench_k20_2 bench; do
python3 -c "import json,sys; j=json.load(open(sys.argv[1])); r=j['roofline']; b=j['barriered']; c=j['compute']; print(sys.argv[1], j['value'], r['avg_launch_us'], r['frac'], r.get('frac_of_achievable_per_block'), r.get('frac_of_achievable_same_form'), 'bar', b['frac'], b.get('frac_of_achievable_per_block'), 'batched', j['batched']['frac'], 'cmp', c['overlapped']['frac'], c['overlapped'].get('frac_vs_verify'), c['barriered']['frac'], c['barriered'].get('frac_vs_verify'), 'cpu', j['cpu_baseline']['value'], 'traffic', r.get('traffic'))" gpurun_out/${TAG}_$f.json
done
