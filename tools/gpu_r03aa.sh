#!/bin/bash
# round 3: the 16-sub-block class's fused-launch cut onto 8-step windows -- parity, then the cut sweep
set -o pipefail
OUT=gpurun_out/r03aa
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_tdec_w8_gpu.py tests/test_tdec16_gpu.py tests/test_tdec8s_gpu.py tests/test_tdec_fullsize_gpu.py tests/test_tdec_gpu.py -m gpu -q -x --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAIL|Error|passed|failed" $OUT/pytest.log | head -20; [ $rc -eq 0 ] || exit 1
for w in 0 1280 1536 1792 2048 1536 1280; do
  timeout -k 10 300 python bench.py --w8-fused-max-k $w --cpu-seconds 0 --pdsch-steps 0 > $OUT/all188_c$w.json 2> $OUT/all188_c$w.err || { tail -5 $OUT/all188_c$w.err; exit 1; }
  python -c "import json; d=json.load(open('$OUT/all188_c$w.json')); print('cut $w', d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'], d['mbps_16_half_its'], d['output_check']['mismatched'])" || exit 1
done
