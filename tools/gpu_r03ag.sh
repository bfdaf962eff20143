#!/bin/bash
# round 3: single-lane threshold 576 -- parity of the affected paths, PUSCH line and its PMC
set -o pipefail
OUT=gpurun_out/r03ag
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_tdec16_gpu.py tests/test_tdec_fullsize_gpu.py tests/test_pusch_gpu.py tests/test_uci_gpu.py tests/test_sch_gpu.py tests/test_ulsch.py -m gpu -q -x --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAIL|Error|passed|failed|no tests ran" $OUT/pytest.log | head -20; [ $rc -le 1 ] || exit 1
timeout -k 10 300 python bench.py --workload pusch --steps 5 --warmup 2 --cpu-seconds 6 > $OUT/pusch.json 2> $OUT/pusch.err || { tail -5 $OUT/pusch.err; exit 1; }
python -c "import json; d=json.load(open('$OUT/pusch.json')); print('pusch', d['value'], d['ms_per_step'], d['roofline']['kernel'], d['roofline']['avg_launch_ms'], d['config'].get('ue_subframes_per_s'))" || exit 1
bash tools/pmc.sh r03_pmc_pusch pusch || exit 1
python tools/pmc_summary.py gpurun_out/r03_pmc_pusch pusch gpurun_out/r03_pmc_pusch/summary.json || exit 1
echo done
