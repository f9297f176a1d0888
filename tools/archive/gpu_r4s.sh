#!/bin/bash
# Round 4: the head of a 128 MiB launch: kernel arguments landed / fill done / first data, per wave,
# production (146) and without table loads (147).
set -o pipefail
TAG=${1:-r4s}
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in 146 147; do
timeout -k 10 300 python -u tools/wave_spread.py --k 40 --kinds crc --variant $v --mid > gpurun_out/${TAG}_spread$v.jsonl \
    2> gpurun_out/${TAG}_spread$v.err || { tail gpurun_out/${TAG}_spread$v.err; exit 1; }
cat gpurun_out/${TAG}_spread$v.jsonl
done
