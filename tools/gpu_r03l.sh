#!/bin/bash
# round 3: the 8-step-window build of the single-lane decoder (parity + timing against W=16),
# the PDSCH chain at NFFT 1536, the H2D loop with its warm pass, PDSCH PMC
set -o pipefail
OUT=gpurun_out/r03l
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_tdec_w8_gpu.py tests/test_tdec16_gpu.py tests/test_tdec8s_gpu.py tests/test_tdec_fullsize_gpu.py -m gpu -v --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAIL|Error|passed|failed" $OUT/pytest.log | head -30; [ $rc -le 1 ] || exit 1
for w in 0 6144; do
  timeout -k 10 120 python tools/tdec_kernels.py --kernel single --workload class8 --batch 1024 --launches 3 --w8 $w || exit 1
  timeout -k 10 120 python tools/tdec_kernels.py --kernel single --workload class8 --batch 4096 --launches 3 --w8 $w || exit 1
  for K in 1024 2048 4096 6144; do
    timeout -k 10 120 python tools/tdec_kernels.py --kernel single --workload k6144 --K $K --batch 2048 --launches 3 --w8 $w || exit 1
  done
  timeout -k 10 200 python tools/tdec_kernels.py --kernel single --workload all188 --launches 3 --w8 $w || exit 1
done
timeout -k 10 300 python bench.py --workload pdsch --steps 5 --warmup 2 --cpu-seconds 0 > $OUT/pdsch_2048.json 2> $OUT/pdsch_2048.err || { tail -5 $OUT/pdsch_2048.err; exit 1; }
cat $OUT/pdsch_2048.json
timeout -k 10 300 python bench.py --workload pdsch --nfft 1536 --steps 5 --warmup 2 --cpu-seconds 0 > $OUT/pdsch_1536.json 2> $OUT/pdsch_1536.err || { tail -5 $OUT/pdsch_1536.err; exit 1; }
cat $OUT/pdsch_1536.json
bash tools/pmc.sh r03_pmc_pdsch pdsch || exit 1
python tools/pmc_summary.py gpurun_out/r03_pmc_pdsch pdsch gpurun_out/r03_pmc_pdsch/summary.json || exit 1
echo done
