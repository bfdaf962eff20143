#!/bin/bash
# Occupancy probe of the lane-pair turbo kernel: K = 6144 at 1024 / 2048 / 4096 blocks a launch,
# then the SQ / traffic counters of the all-188 launch.
set -o pipefail
TAG=${1:-occ}; OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
for B in 1024 2048 4096; do
  timeout -k 10 100 python bench.py --workload k6144 --batch $B --steps 10 --warmup 2 --cpu-seconds 0 > $OUT/k6144_$B.json 2> $OUT/k6144_$B.err || exit 1
  python -c "import json;d=json.load(open('$OUT/k6144_$B.json'));print($B, d['value'], d['roofline']['avg_launch_ms'])"
done
bash tools/pmc.sh $TAG/pmc all188 --pdsch-steps 0 || exit 1
python tools/pmc_summary.py gpurun_out/$TAG/pmc all188 gpurun_out/$TAG/pmc_summary.json
