#!/bin/bash
# Turbo-decoder check on one GPU box: lane-pair parity tests, DL-SCH / PDSCH parity, then the
# turbo bench lines (all-188 default, k6144 with both kernels) and the PDSCH chain.
# Usage: tools/gpu_t16.sh TAG
set -o pipefail
TAG=${1:-t16}; OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q -k "tdec or sch or pdsch or threads or ue_dl" --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python bench.py --steps 5 --warmup 2 --cpu-seconds 0 --pdsch-steps 10 > $OUT/all188.json 2> $OUT/all188.err || exit 1
timeout -k 10 100 python bench.py --workload k6144 --steps 10 --warmup 2 --cpu-seconds 0 > $OUT/k6144_quad.json 2> $OUT/k6144_quad.err || exit 1
SRSRAN_TDEC16_MIN_CB=1 timeout -k 10 100 python bench.py --workload k6144 --steps 10 --warmup 2 --cpu-seconds 0 > $OUT/k6144_pair.json 2> $OUT/k6144_pair.err || exit 1
timeout -k 10 100 python bench.py --workload dlsch --steps 10 --warmup 2 --cpu-seconds 0 > $OUT/dlsch.json 2> $OUT/dlsch.err || exit 1
python - <<PY
import json
d=json.load(open("$OUT/all188.json")); print("all188", d["value"], d["roofline"]["avg_launch_ms"], "16hi", d.get("mbps_16_half_its"), d.get("output_check"), "pdsch", d.get("pdsch_subframes_per_s"))
for f in ("k6144_quad","k6144_pair","dlsch"):
    d=json.load(open("$OUT/%s.json"%f)); print(f, d["value"], d["roofline"]["avg_launch_ms"], d.get("output_check"))
PY
