#!/bin/bash
# round 3: PDSCH transmit symbols against the reference's building blocks; remaining clean secondary lines
set -o pipefail
OUT=gpurun_out/r03v
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_pdsch_tx_ref_gpu.py tests/test_enb_dl_gpu.py -m gpu -v --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "PASS|FAIL|Error|passed|failed" $OUT/pytest.log | head -30; [ $rc -le 1 ] || exit 1
OUTN=gpurun_out/r03n
mkdir -p $OUTN
run() {
  local n=$1; shift
  timeout -k 10 300 python bench.py "$@" --steps 5 --warmup 2 > $OUTN/$n.json 2> $OUTN/$n.err || { echo "$n failed"; tail -5 $OUTN/$n.err; return 1; }
  python -c "import json; d=json.load(open('$OUTN/$n.json')); print('$n', d['value'], d['unit'], d['ms_per_step'], (d.get('roofline') or {}).get('kernel'), (d.get('cpu_baseline') or {}).get('value'))"
}
run dlloop --workload dlloop --cpu-seconds 0 &&
run ldpc_bg1 --workload ldpc --cpu-seconds 6 &&
run ldpc_bg2 --workload ldpc --bg 2 --cpu-seconds 0 &&
run nrsch --workload nrsch --cpu-seconds 6 &&
run pdsch_low --workload pdsch --snr 17 --cpu-seconds 0 &&
echo done
