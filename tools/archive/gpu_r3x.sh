#!/bin/bash
# Parity of lab variant 115 (s_setprio by rounds left), its A/B in both launch modes and at 1 GiB,
# and the bench in the driver's form and the default form (polling settle, precomputed pointers).
set -o pipefail
TAG=${1:-r3x}
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -q --timeout 150 --timeout-method thread \
    -p no:cacheprovider -k "variant" > gpurun_out/${TAG}_parity.txt 2>&1
rc=$?; echo "parity rc=$rc"; tail -2 gpurun_out/${TAG}_parity.txt
[ $rc -eq 0 ] || exit $rc
V=0,115
timeout -k 10 200 python3 tools/ab.py --variants $V --bpc 512,4096 --rounds 9 --overlap > gpurun_out/${TAG}_ab_ovl.jsonl 2> gpurun_out/${TAG}_ab_ovl.err || exit 1
timeout -k 10 200 python3 tools/ab.py --variants $V --bpc 512,4096 --rounds 9 > gpurun_out/${TAG}_ab_bar.jsonl 2> gpurun_out/${TAG}_ab_bar.err || exit 1
timeout -k 10 200 python3 tools/ab.py --variants $V --bpc 512 --rounds 7 --block-mib 1024 --blocks 2 --reps 6 > gpurun_out/${TAG}_ab_1g.jsonl 2> gpurun_out/${TAG}_ab_1g.err || exit 1
timeout -k 10 200 python3 tools/ab.py --variants $V --bpc 512 --rounds 9 --overlap --mode compute > gpurun_out/${TAG}_ab_cmp_ovl.jsonl 2> gpurun_out/${TAG}_ab_cmp_ovl.err || exit 1
for f in ovl bar 1g cmp_ovl; do echo "== $f"; python3 -c "
import json,sys
for l in open(sys.argv[1]):
    j=json.loads(l); print(j['bpc'], j['case'], j['us_med'], j['us_min'], j['results_ok'])" gpurun_out/${TAG}_ab_$f.jsonl; done
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/${TAG}_bench_k20.json 2> gpurun_out/${TAG}_bench_k20.err \
    || { echo "bench k20 failed"; tail -20 gpurun_out/${TAG}_bench_k20.err; exit 1; }
timeout -k 10 300 python3 bench.py --no-pmc > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err \
    || { echo "bench failed"; tail -20 gpurun_out/${TAG}_bench.err; exit 1; }
for f in bench_k20 bench; do
python3 -c "import json,sys; j=json.load(open(sys.argv[1])); r=j['roofline']; b=j['barriered']; c=j['compute']; print(sys.argv[1], j['value'], r['avg_launch_us'], r['frac'], r.get('frac_of_achievable_per_block'), 'bar', b['frac'], b.get('frac_of_achievable_per_block'), 'batched', j['batched']['frac'], 'cmp', c['overlapped']['frac'], c['overlapped'].get('frac_vs_verify'), c['barriered']['frac'], c['barriered'].get('frac_vs_verify'), 'cpu', j['cpu_baseline']['value'], 'traffic', r.get('traffic'))" gpurun_out/${TAG}_$f.json
done
