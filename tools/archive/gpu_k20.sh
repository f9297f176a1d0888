#!/bin/bash
# The driver's bench command (K=20, W=5) against the default K=2000, with and without the
# lead-in spin ahead of the start event (bench.py --lead-us). Usage (gpurun): bash tools/gpu_k20.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
run() {  # tag, args...
  local tag=$1; shift
  timeout -k 10 200 python3 bench.py "$@" --no-pmc --no-cpu-baseline > gpurun_out/k_$tag.json 2> gpurun_out/k_$tag.err || exit 1
  python3 -c "
import json; d=json.load(open('gpurun_out/k_$tag.json')); r=d['roofline']
print('$tag', d['value'], d['ms_per_step'], d['host_ms_per_step'], r['avg_launch_us'], r['frac'], d.get('lead_in_us'))"
}
for i in 1 2 3; do
  run lead_k20_$i --gpus 1 --steps 20 --warmup 5
  run nolead_k20_$i --gpus 1 --steps 20 --warmup 5 --lead-us 0
done
run lead_k2000 --gpus 1 --steps 2000 --warmup 1000
run nolead_k2000 --gpus 1 --steps 2000 --warmup 1000 --lead-us 0
