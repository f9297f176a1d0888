#!/bin/bash
# Host issue timeline of the driver-form timed regions (tools/launch_host_probe.py).
set -o pipefail
TAG=${1:-r3v}
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 200 python3 tools/launch_host_probe.py > gpurun_out/${TAG}_host_probe.jsonl 2> gpurun_out/${TAG}_host_probe.err \
    || { echo "probe failed"; tail -5 gpurun_out/${TAG}_host_probe.err; exit 1; }
python3 -c "
import json,sys,statistics as S
from collections import defaultdict
d=defaultdict(list); f=defaultdict(list)
for l in open(sys.argv[1]):
    j=json.loads(l); k=(j['case'],j['overlap'],j['mode']); d[k].append(j['gpu_us_per_launch']); f[k].append(j['issue_us'][0])
for k in d: print(k, 'gpu med %.2f min %.2f max %.2f' % (S.median(d[k]), min(d[k]), max(d[k])), 'first issue', f[k])" gpurun_out/${TAG}_host_probe.jsonl
