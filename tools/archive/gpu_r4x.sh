#!/bin/bash
# Round 4, VERDICT r3 item 1's question: do the driver region's first launches have a longer head
# (fill done, first data) than launches after 1000 overlapped ones? Per-launch rows, lab 146.
set -o pipefail
TAG=${1:-r4x}
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
for rep in 1 2; do
timeout -k 10 300 python -u tools/wave_spread.py --form bench --k 20 --variant 146 --mid >> gpurun_out/${TAG}_form.jsonl \
    2>> gpurun_out/${TAG}_form.err || { tail gpurun_out/${TAG}_form.err; exit 1; }
done
python3 -c "
import json
for l in open('gpurun_out/${TAG}_form.jsonl'):
    d = json.loads(l); print(d['form'], d['us_per_launch_events'])
    for r in d['launches']: print('  ', r['launch'], r['start_us'], r['span_us'], r['wave_end_p10_p90_us'], r.get('fill_done_p50_us'), r.get('first_data_p50_us'))"
