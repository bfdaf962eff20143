#!/bin/bash
# Timing ablation of the decoder phases (results are NOT valid decodes in ablation modes).
set -o pipefail
for F in 0 1 2 3; do
  SRSRAN_TDEC_ABLATE=$F timeout -k 10 120 python bench.py --workload k6144 --steps 20 --warmup 3 --cpu-seconds 0 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('ablate=$F', d['roofline']['avg_launch_ms'], 'ms/launch')" || exit 1
done
