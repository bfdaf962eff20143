#!/bin/bash
# round 3: wave priority for the large-size part of the cut all-188 class (A/B against the previous build)
set -o pipefail
OUT=gpurun_out/r03ae
mkdir -p $OUT
export TMPDIR=/tmp
BASE=$GRAFT_REPO_ROOT/srsran_4g_amd/lib/ab/libsrsran_4g_amd_prio2.so
for r in 1 2 3; do
  for L in new base; do
    if [ $L = base ]; then export SRSRAN_AMD_LIB=$BASE; else unset SRSRAN_AMD_LIB; fi
    timeout -k 10 300 python bench.py --cpu-seconds 0 --pdsch-steps 0 > $OUT/all188_$L$r.json 2> $OUT/all188_$L$r.err || { tail -5 $OUT/all188_$L$r.err; exit 1; }
    python -c "import json; d=json.load(open('$OUT/all188_$L$r.json')); print('$L', d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'], d['mbps_16_half_its'], d['output_check']['mismatched'])" || exit 1
  done
done
unset SRSRAN_AMD_LIB
for w in 2560 3072 2048 2560; do
  timeout -k 10 300 python bench.py --w8-fused-max-k $w --cpu-seconds 0 --pdsch-steps 0 > $OUT/all188_c$w.json 2> $OUT/all188_c$w.err || { tail -5 $OUT/all188_c$w.err; exit 1; }
  python -c "import json; d=json.load(open('$OUT/all188_c$w.json')); print('cut $w', d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'], d['output_check']['mismatched'])" || exit 1
done
