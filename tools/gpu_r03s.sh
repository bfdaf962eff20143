#!/bin/bash
# round 3: PCIe loop with the host-side buffer wait (priority A/B), the default bench line, then one clean
# line per secondary workload
set -o pipefail
OUT=gpurun_out/r03s
mkdir -p $OUT
export TMPDIR=/tmp
for pr in 0 -1; do
  timeout -k 10 300 python bench.py --workload pdsch --h2d-priority $pr --steps 5 --warmup 2 --cpu-seconds 0 > $OUT/pdsch_pr$pr.json 2> $OUT/pdsch_pr$pr.err || { tail -5 $OUT/pdsch_pr$pr.err; exit 1; }
  python -c "import json; d=json.load(open('$OUT/pdsch_pr$pr.json')); c=d['config']; print('prio $pr', c['subframes_per_s'], c['subframes_per_s_h2d_inclusive'], c['h2d_copy_only_subframes_per_s'], d['host_phases_us_per_call'])" || exit 1
done
timeout -k 10 600 python bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err || { tail -5 $OUT/bench_default.err; exit 1; }
cat $OUT/bench_default.json
bash tools/gpu_r03n.sh
