#!/bin/bash
# round 3: two-window prefetch in the single-lane decoder (parity + timing), eNB -> UE loop, PCIe probe, PMC
set -o pipefail
OUT=gpurun_out/r03k
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_tdec16_gpu.py tests/test_tdec8s_gpu.py tests/test_tdec_fullsize_gpu.py tests/test_enb_ue_loop_gpu.py -m gpu -v --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAIL|Error|passed|failed" $OUT/pytest.log | head -30; [ $rc -le 1 ] || exit 1
for b in 1024 2048; do
  timeout -k 10 120 python tools/tdec_kernels.py --kernel single --workload k6144 --batch $b --launches 3 || exit 1
done
timeout -k 10 200 python tools/tdec_kernels.py --kernel single --workload all188 --launches 3 || exit 1
timeout -k 10 120 python tools/tdec_kernels.py --kernel single --workload class8 --batch 256 --launches 3 || exit 1
timeout -k 10 240 python tools/h2d_probe.py > $OUT/h2d_probe.jsonl 2> $OUT/h2d_probe.err || { tail -5 $OUT/h2d_probe.err; exit 1; }
cat $OUT/h2d_probe.jsonl
for W in pusch pdsch ldpc nrsch; do
  bash tools/pmc.sh r03_pmc_$W $W || exit 1
  python tools/pmc_summary.py gpurun_out/r03_pmc_$W $W gpurun_out/r03_pmc_$W/summary.json || exit 1
done
echo done
