#!/bin/bash
# round 3 PMC at HEAD: counter calibration per access width, then the decoder kernels' passes
set -o pipefail
bash $GRAFT_REPO_ROOT/tools/gpu_calib.sh || exit 1
for W in all188 k6144 class8; do
  bash $GRAFT_REPO_ROOT/tools/pmc_tdec.sh r03_pmc_$W --kernel single --workload $W --launches 3 || exit 1
done
echo done
