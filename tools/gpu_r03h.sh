#!/bin/bash
# round 3: single-lane split variant (helper waves): parity, then timing against the other decoders
set -o pipefail
OUT=gpurun_out/r03h
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_tdec16_gpu.py tests/test_tdec8s_gpu.py tests/test_tdec_fullsize_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -6 $OUT/pytest.log; [ $rc -eq 0 ] || exit 1
for b in 256 512 1024; do
  for k in split single pair quad; do
    timeout -k 10 120 python tools/tdec_kernels.py --kernel $k --workload k6144 --batch $b --launches 3 || exit 1
  done
done
for K in 512 800; do
  for b in 512 1024 2048; do
    for k in split quad; do
      timeout -k 10 120 python tools/tdec_kernels.py --kernel $k --K $K --batch $b --launches 3 || exit 1
    done
  done
done
