#!/bin/bash
# round 3: single-lane vs lane-pair 16-class decoder between 512 and 1024 blocks (threshold), PUSCH at both
set -o pipefail
OUT=gpurun_out/r03af
mkdir -p $OUT
export TMPDIR=/tmp
for b in 640 768 896 1014; do
  for k in single pair; do
    timeout -k 10 120 python tools/tdec_kernels.py --kernel $k --workload k6144 --batch $b --launches 5 || exit 1
  done
done
for t in single pair; do
  timeout -k 10 300 python bench.py --workload pusch --tdec16 $t --steps 5 --warmup 2 --cpu-seconds 0 > $OUT/pusch_$t.json 2> $OUT/pusch_$t.err || { tail -5 $OUT/pusch_$t.err; exit 1; }
  python -c "import json; d=json.load(open('$OUT/pusch_$t.json')); print('pusch $t', d['value'], d['ms_per_step'], d['roofline']['kernel'], d['roofline']['avg_launch_ms'])" || exit 1
done
