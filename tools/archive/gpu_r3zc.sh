#!/bin/bash
# Staged compute words (production for compute at bpc 512 over contiguous blocks of <= 32 rounds per
# wave): the whole -m gpu suite, A/B against held stores (lab 122), the bench in both forms.
set -o pipefail
TAG=${1:-r3zc}
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 480 python -u -m pytest tests -m gpu -q --timeout 150 --timeout-method thread \
    -p no:cacheprovider > gpurun_out/${TAG}_gpu_tests.txt 2>&1
rc=$?; echo "gpu tests rc=$rc"; tail -2 gpurun_out/${TAG}_gpu_tests.txt
[ $rc -eq 0 ] || { grep -E "FAIL|Error" gpurun_out/${TAG}_gpu_tests.txt | head -20; exit $rc; }
ab() { # name args...
    local n=$1; shift
    timeout -k 10 200 python3 tools/ab.py "$@" > gpurun_out/${TAG}_$n.jsonl 2> gpurun_out/${TAG}_$n.err || { echo "ab $n failed"; tail -3 gpurun_out/${TAG}_$n.err; exit 1; }
    echo "== $n"; python3 -c "
import json,sys
for l in open(sys.argv[1]):
    j=json.loads(l); print(j['bpc'], j['mode'], j['case'], j['us_med'], j['us_min'], j['results_ok'])" gpurun_out/${TAG}_$n.jsonl
}
ab c128_ovl --variants 0,122 --mode compute --rounds 11 --overlap || exit 1
ab c128_bar --variants 0,122 --mode compute --rounds 11 || exit 1
ab c256_ovl --variants 0,122 --mode compute --block-mib 256 --blocks 4 --reps 12 --rounds 7 --overlap || exit 1
ab v128_ovl --variants 0 --rounds 11 --overlap || exit 1
ab v128_bar --variants 0 --rounds 11 || exit 1
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/${TAG}_bench_k20.json 2> gpurun_out/${TAG}_bench_k20.err \
    || { echo "bench k20 failed"; tail -20 gpurun_out/${TAG}_bench_k20.err; exit 1; }
timeout -k 10 300 python3 bench.py --no-pmc > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err \
    || { echo "bench failed"; tail -20 gpurun_out/${TAG}_bench.err; exit 1; }
for f in bench_k20 bench; do
python3 -c "import json,sys; j=json.load(open(sys.argv[1])); r=j['roofline']; b=j['barriered']; c=j['compute']; print(sys.argv[1], j['value'], r['avg_launch_us'], r['frac'], r.get('frac_of_achievable_per_block'), r.get('frac_of_achievable_same_form'), 'bar', b['frac'], b.get('frac_of_achievable_per_block'), 'batched', j['batched']['frac'], 'cmp', c['overlapped']['frac'], c['overlapped'].get('frac_vs_verify'), c['barriered']['frac'], c['barriered'].get('frac_vs_verify'), 'cpu', j['cpu_baseline']['value'], 'traffic', r.get('traffic'))" gpurun_out/${TAG}_$f.json
done
