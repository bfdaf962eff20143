#!/bin/bash
# round 3: software-pipelined phase 2 of the single-lane decoder -- parity, then A/B timings against the
# previous build (srsran_4g_amd/lib/ab/libsrsran_4g_amd_base.so) on the same box
set -o pipefail
OUT=gpurun_out/r03o
mkdir -p $OUT
export TMPDIR=/tmp
BASE=srsran_4g_amd/lib/ab/libsrsran_4g_amd_base.so
timeout -k 10 600 python -u -m pytest tests/test_tdec16_gpu.py tests/test_tdec8s_gpu.py tests/test_tdec_w8_gpu.py tests/test_tdec_fullsize_gpu.py tests/test_tdec_gpu.py tests/test_sch_gpu.py -m gpu -q -x --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAIL|Error|passed|failed" $OUT/pytest.log | head -20; [ $rc -eq 0 ] || exit 1
for L in "" "--lib $BASE"; do
  for w in 0 6144; do
    for b in 1024 2048; do
      timeout -k 10 120 python tools/tdec_kernels.py --kernel single --workload k6144 --batch $b --launches 5 --w8 $w $L || exit 1
    done
  done
  timeout -k 10 200 python tools/tdec_kernels.py --kernel single --workload all188 --launches 3 $L || exit 1
  timeout -k 10 120 python tools/tdec_kernels.py --kernel single --workload class8 --batch 1024 --launches 3 --w8 800 $L || exit 1
done
echo done
