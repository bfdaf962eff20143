#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
for k in single pair; do
  timeout -k 10 120 python tools/tdec_kernels.py --kernel $k --workload k6144 --batch 2048 || exit 1
  timeout -k 10 120 python tools/tdec_kernels.py --kernel $k --workload k6144 --batch 1024 || exit 1
  timeout -k 10 120 python tools/tdec_kernels.py --kernel $k --workload all188 --batch 1024 --launches 3 || exit 1
done
bash tools/pmc_tdec.sh pmc_s2048 --kernel single --workload k6144 --batch 2048 || exit 1
bash tools/pmc_tdec.sh pmc_s188 --kernel single --workload all188 --launches 2 || exit 1
