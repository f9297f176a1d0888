#!/bin/bash
# Kernel trace of the driver's bench command (K=20, W=5): per-dispatch durations of the timed region.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
for i in 1 2; do
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/k20tr_$i -o run \
    -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-pmc --no-cpu-baseline > gpurun_out/k20tr_$i.json 2> gpurun_out/k20tr_$i.err || exit 1
done
