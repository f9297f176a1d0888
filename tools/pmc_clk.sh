#!/bin/bash
# clock/activity counters for kernel variants (one rocprofv3 pass per group, no tracing mix)
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/pmc_clk
mkdir -p $OUT
cd /tmp
for v in 0 77; do
  timeout -k 10 120 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAVES --output-format csv -d $OUT/v${v}_a -o run -- python3 $R/tools/pmc_driver.py --variant $v --launches 24 > $OUT/v${v}_a.log 2>&1 || exit 1
  timeout -k 10 120 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD --output-format csv -d $OUT/v${v}_b -o run -- python3 $R/tools/pmc_driver.py --variant $v --launches 24 > $OUT/v${v}_b.log 2>&1 || exit 1
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/v${v}_t -o run -- python3 $R/tools/pmc_driver.py --variant $v --launches 24 > $OUT/v${v}_t.log 2>&1 || exit 1
done
