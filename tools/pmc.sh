#!/bin/bash
# PMC passes for the verify kernel (one rocprofv3 invocation per counter group, as
# MI355X_MICROARCH.md's rocprofv3 section prescribes; never combined with tracing).
# Usage (on the GPU box): tools/pmc.sh <out_dir> [extra args for tools/pmc_driver.py]
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$(mkdir -p "$1" && cd "$1" && pwd); shift
mkdir -p "$OUT"
cd /tmp
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE" \
           "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INST_CYCLES_VMEM_RD" \
           "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  rc=0
  timeout -k 10 240 rocprofv3 --pmc $grp --output-format csv -d "$OUT/p$i" -o run -- \
      python3 "$R/tools/pmc_driver.py" "$@" > "$OUT/p$i.log" 2>&1 || rc=$?
  if [ $rc -ne 0 ]; then
    echo "pass $i ($grp) rc=$rc"; tail -5 "$OUT/p$i.log"
    # a timeout / abort / segfault ends the GPU work of this call
    case $rc in 124|134|137|139) exit $rc;; esac
  fi
done
