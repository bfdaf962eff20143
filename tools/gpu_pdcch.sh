#!/bin/bash
# PDCCH / PCFICH GPU parity run.  Usage: tools/gpu_pdcch.sh TAG [pytest -k expr]
set -o pipefail
TAG=${1:-pdcch}; K=${2:-"pdcch"}; OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v -k "$K" --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; tail -40 $OUT/pytest.log; exit $rc
