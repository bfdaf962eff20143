#!/bin/bash
# round 3: eNB -> UE loop through the PDCCH, full-size decoder defaults, PCIe loop probe, remaining PMC
set -o pipefail
OUT=gpurun_out/r03j
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_enb_ue_loop_gpu.py tests/test_tdec_fullsize_gpu.py -m gpu -v --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "PASS|FAIL|Error|assert" $OUT/pytest.log | head -40; [ $rc -le 1 ] || exit 1
timeout -k 10 240 python tools/h2d_probe.py > $OUT/h2d_probe.jsonl 2> $OUT/h2d_probe.err || { tail -5 $OUT/h2d_probe.err; exit 1; }
cat $OUT/h2d_probe.jsonl
for W in pusch pdsch ldpc nrsch; do
  bash tools/pmc.sh r03_pmc_$W $W || exit 1
  python tools/pmc_summary.py gpurun_out/r03_pmc_$W $W gpurun_out/r03_pmc_$W/summary.json || exit 1
done
echo done
