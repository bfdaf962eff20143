#!/bin/bash
# Two SQ counter passes (rocprofv3 --pmc, kernel trace only) over one bench workload.
# Usage: tools/pmc_sq.sh TAG WORKLOAD [extra bench args]
set -o pipefail
TAG=${1:-pmc}; WL=${2:-k6144}; shift 2
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
i=2
for P in "SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU" \
         "SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $P --output-format csv -d $OUT/p$i -o pmc -- python3 $GRAFT_REPO_ROOT/bench.py --workload $WL --steps 2 --warmup 1 --cpu-seconds 0 --pdsch-steps 0 "$@" > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $OUT/p$i.log; exit 1; }
done
cd $GRAFT_REPO_ROOT && python tools/pmc_summary.py gpurun_out/$TAG $WL gpurun_out/$TAG/summary.json
