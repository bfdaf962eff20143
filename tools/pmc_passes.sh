#!/bin/bash
# Custom PMC passes (each its own rocprofv3 --pmc run, killed after 60 s) over tools/tdec_kernels.py.
# Usage: PASSES="CTR CTR ...;CTR ..." tools/pmc_passes.sh TAG [tdec_kernels.py args]
set -o pipefail
TAG=${1:-pmc}; shift
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
i=0
IFS=';' read -ra PS <<< "$PASSES"
for P in "${PS[@]}"; do
  i=$((i+1))
  timeout -s KILL 60 rocprofv3 --pmc $P --output-format csv -d $OUT/p$i -o pmc -- python3 $GRAFT_REPO_ROOT/tools/tdec_kernels.py "$@" > $OUT/p$i.log 2>&1 || { echo "pass $i ($P) failed"; tail -5 $OUT/p$i.log; exit 1; }
done
cd $GRAFT_REPO_ROOT && python tools/pmc_summary.py gpurun_out/$TAG tdec gpurun_out/$TAG/summary.json
