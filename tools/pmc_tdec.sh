#!/bin/bash
# PMC passes (each its own rocprofv3 run, --pmc only) over tools/tdec_kernels.py: identical launches of one
# decoder kernel, so every dispatch's counters describe the same work.
# Usage: tools/pmc_tdec.sh TAG [tdec_kernels.py args]
set -o pipefail
TAG=${1:-pmc}; shift
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
i=0
for P in "SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU" \
         "SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE" \
         "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $P --output-format csv -d $OUT/p$i -o pmc -- python3 $GRAFT_REPO_ROOT/tools/tdec_kernels.py "$@" > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $OUT/p$i.log; exit 1; }
done
cd $GRAFT_REPO_ROOT && python tools/pmc_summary.py gpurun_out/$TAG tdec gpurun_out/$TAG/summary.json
