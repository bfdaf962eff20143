#!/bin/bash
# One GPU session: turbo / DL-SCH parity tests, then the two turbo bench workloads.
# Usage: tools/gpu_check.sh TAG [pytest -k expr]
set -o pipefail
TAG=${1:-run}; K=${2:-"tdec or sch or threads"}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q -k "$K" --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; tail -15 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python bench.py --workload k6144 --steps 10 --warmup 2 --cpu-seconds 0 > $OUT/k6144.json 2> $OUT/k6144.err || exit 1
python -c "import json;d=json.load(open('$OUT/k6144.json'));print('k6144', d['value'], d['roofline']['avg_launch_ms'], d.get('output_check'))"
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --cpu-seconds 0 --pdsch-steps 0 > $OUT/all188.json 2> $OUT/all188.err || exit 1
python -c "import json;d=json.load(open('$OUT/all188.json'));print('all188', d['value'], d['roofline']['avg_launch_ms'], d['mbps_16_half_its'], d.get('output_check'))"
