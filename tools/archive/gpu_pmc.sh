#!/bin/bash
# PMC passes of the production verify kernel in the bench's timed mode (overlapped launches:
# the solo-tail kernel) and in barriered mode. Usage (gpurun): bash tools/gpu_pmc.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
bash tools/pmc.sh gpurun_out/pmc_ovl --launches 16 --overlap || exit 1
bash tools/pmc.sh gpurun_out/pmc_bar --launches 16 || exit 1
python3 tools/pmc_summary.py gpurun_out/pmc_ovl > gpurun_out/pmc_ovl_summary.json
python3 tools/pmc_summary.py gpurun_out/pmc_bar > gpurun_out/pmc_bar_summary.json
cat gpurun_out/pmc_ovl_summary.json gpurun_out/pmc_bar_summary.json
