#!/bin/bash
# round 3: the 16-sub-block class cut at w8_max_k (small sizes on 8-step windows as their own fused launch)
set -o pipefail
OUT=gpurun_out/r03z
mkdir -p $OUT
export TMPDIR=/tmp
for w in 800 1536 2368 3136 800 2368; do
  timeout -k 10 300 python bench.py --w8-max-k $w --cpu-seconds 0 --pdsch-steps 0 > $OUT/all188_w$w.json 2> $OUT/all188_w$w.err || { tail -5 $OUT/all188_w$w.err; exit 1; }
  python -c "import json; d=json.load(open('$OUT/all188_w$w.json')); print('w8 $w', d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'], d['mbps_16_half_its'], d['output_check']['mismatched'])" || exit 1
done
