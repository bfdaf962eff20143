#!/bin/bash
# round 3: eNB control-channel TX tests, then counter calibration + decoder PMC passes
set -o pipefail
OUT=gpurun_out/r03f
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_enb_ctrl_gpu.py tests/test_enb_dl_gpu.py -m gpu -x -v --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -30 $OUT/pytest.log
# an ordinary test failure (rc 1) lets the profiling run; a crash, abort or time limit ends the call
[ $rc -le 1 ] || exit 1
bash tools/gpu_pmc_r03.sh
