#!/bin/bash
# round 3: PCIe loop of the PDSCH chain -- hardware-queue count A/B (HIP multiplexes streams over
# GPU_MAX_HW_QUEUES queues), and the standalone probe on the same box
set -o pipefail
OUT=gpurun_out/r03q
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 240 python tools/h2d_probe.py > $OUT/h2d_probe.jsonl 2> $OUT/h2d_probe.err || { tail -5 $OUT/h2d_probe.err; exit 1; }
cat $OUT/h2d_probe.jsonl
for q in 4 8 16; do
  GPU_MAX_HW_QUEUES=$q timeout -k 10 300 python bench.py --workload pdsch --steps 5 --warmup 2 --cpu-seconds 0 > $OUT/pdsch_q$q.json 2> $OUT/pdsch_q$q.err || { tail -5 $OUT/pdsch_q$q.err; exit 1; }
  python -c "import json; d=json.load(open('$OUT/pdsch_q$q.json')); c=d['config']; print('hwq $q', c['subframes_per_s'], c['subframes_per_s_h2d_inclusive'], c['h2d_copy_only_subframes_per_s'])" || exit 1
done
echo done
