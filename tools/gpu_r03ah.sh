#!/bin/bash
# round 3: descriptor uploads of the PDSCH / DL-SCH batch path on copy streams -- parity, then A/B
set -o pipefail
OUT=gpurun_out/r03ai
mkdir -p $OUT
export TMPDIR=/tmp
BASE=$GRAFT_REPO_ROOT/srsran_4g_amd/lib/ab/libsrsran_4g_amd_base.so
timeout -k 10 600 python -u -m pytest tests/test_pdsch_gpu.py tests/test_sch_gpu.py tests/test_extcp_gpu.py tests/test_uci_gpu.py tests/test_pusch_gpu.py tests/test_ulsch.py tests/test_enb_ue_loop_gpu.py tests/test_threads_gpu.py -m gpu -q -x --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAIL|Error|passed|failed|no tests" $OUT/pytest.log | head -20; [ $rc -eq 0 ] || exit 1
for r in 1 2; do
  for L in new base; do
    if [ $L = base ]; then export SRSRAN_AMD_LIB=$BASE; else unset SRSRAN_AMD_LIB; fi
    for W in pdsch dlsch pusch; do
      timeout -k 10 300 python bench.py --workload $W --steps 10 --warmup 3 --cpu-seconds 0 > $OUT/${W}_$L$r.json 2> $OUT/${W}_$L$r.err || { tail -5 $OUT/${W}_$L$r.err; exit 1; }
      python -c "import json; d=json.load(open('$OUT/${W}_$L$r.json')); c=d['config']; print('$W $L', d['value'], d['ms_per_step'], c.get('subframes_per_s'), c.get('tb_ok_fraction', c.get('tbs_ok')))" || exit 1
    done
  done
done
