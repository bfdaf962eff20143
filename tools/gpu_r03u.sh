#!/bin/bash
# round 3: the fused class launches cut into LDS-sized parts on their own pool streams -- parity, then the
# all-188 step A/B against the previous build on the same box
set -o pipefail
OUT=gpurun_out/r03u
mkdir -p $OUT
export TMPDIR=/tmp
BASE=$GRAFT_REPO_ROOT/srsran_4g_amd/lib/ab/libsrsran_4g_amd_base.so
timeout -k 10 600 python -u -m pytest tests/test_tdec16_gpu.py tests/test_tdec8s_gpu.py tests/test_tdec_w8_gpu.py tests/test_tdec_fullsize_gpu.py tests/test_tdec_gpu.py -m gpu -q -x --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAIL|Error|passed|failed" $OUT/pytest.log | head -20; [ $rc -eq 0 ] || exit 1
for r in 1 2; do
  for L in new base; do
    if [ $L = base ]; then export SRSRAN_AMD_LIB=$BASE; else unset SRSRAN_AMD_LIB; fi
    timeout -k 10 300 python bench.py --cpu-seconds 0 --pdsch-steps 0 > $OUT/all188_$L$r.json 2> $OUT/all188_$L$r.err || { tail -5 $OUT/all188_$L$r.err; exit 1; }
    python -c "import json; d=json.load(open('$OUT/all188_$L$r.json')); print('$L', d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'], d['mbps_16_half_its'], d['output_check'])" || exit 1
  done
done
unset SRSRAN_AMD_LIB
echo done
