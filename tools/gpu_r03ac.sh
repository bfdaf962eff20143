#!/bin/bash
# round 3: fused-launch cut sweep around 2048, then PMC of the all-188 16-class at the default cut
set -o pipefail
OUT=gpurun_out/r03ac
mkdir -p $OUT
export TMPDIR=/tmp
for w in 1920 2048 2176 2304 2048 1920 2304; do
  timeout -k 10 300 python bench.py --w8-fused-max-k $w --cpu-seconds 0 --pdsch-steps 0 > $OUT/all188_c$w.json 2> $OUT/all188_c$w.err || { tail -5 $OUT/all188_c$w.err; exit 1; }
  python -c "import json; d=json.load(open('$OUT/all188_c$w.json')); print('cut $w', d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'], d['mbps_16_half_its'], d['output_check']['mismatched'])" || exit 1
done
bash tools/pmc_tdec.sh r03_pmc_all188b --kernel single --workload all188 --launches 3 || exit 1
echo done
