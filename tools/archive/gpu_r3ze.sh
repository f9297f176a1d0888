#!/bin/bash
# The bench in both forms with the paired compute/verify regions.
set -o pipefail
TAG=${1:-r3ze}
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/${TAG}_bench_k20.json 2> gpurun_out/${TAG}_bench_k20.err \
    || { echo "bench k20 failed"; tail -20 gpurun_out/${TAG}_bench_k20.err; exit 1; }
timeout -k 10 300 python3 bench.py --no-pmc > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err \
    || { echo "bench failed"; tail -20 gpurun_out/${TAG}_bench.err; exit 1; }
for f in bench_k20 bench; do
python3 -c "import json,sys; j=json.load(open(sys.argv[1])); r=j['roofline']; b=j['barriered']; c=j['compute']; print(sys.argv[1], j['value'], r['avg_launch_us'], r['frac'], r.get('frac_of_achievable_per_block'), r.get('frac_of_achievable_same_form'), 'bar', b['frac'], 'cmp', c['overlapped']['frac'], c['overlapped'].get('frac_vs_verify'), c['overlapped']['paired'], c['barriered']['frac'], c['barriered'].get('frac_vs_verify'), c['barriered']['paired'])" gpurun_out/${TAG}_$f.json
done
