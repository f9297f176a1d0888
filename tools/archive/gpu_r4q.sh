#!/bin/bash
# Round 4: the head of a 128 MiB launch, wave by wave (lab 146: fill-done and first-data times),
# barriered and overlapped, and the read's spread for comparison.
set -o pipefail
TAG=${1:-r4q}
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/wave_spread.py --k 40 --kinds crc --variant 146 --mid > gpurun_out/${TAG}_spread146.jsonl \
    2> gpurun_out/${TAG}_spread146.err; rc=$?; cat gpurun_out/${TAG}_spread146.jsonl; [ $rc -eq 0 ] || { tail gpurun_out/${TAG}_spread146.err; exit 1; }
