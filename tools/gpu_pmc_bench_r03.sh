#!/bin/bash
# round 3 PMC passes (tools/pmc.sh: FETCH_SIZE, WRITE_SIZE, SQ counters) over the bench workloads at HEAD
set -o pipefail
for W in dlsch ulsch pusch pdsch ldpc nrsch; do
  bash $GRAFT_REPO_ROOT/tools/pmc.sh r03_pmc_$W $W || exit 1
  (cd $GRAFT_REPO_ROOT && python tools/pmc_summary.py gpurun_out/r03_pmc_$W $W gpurun_out/r03_pmc_$W/summary.json) || exit 1
done
echo done
