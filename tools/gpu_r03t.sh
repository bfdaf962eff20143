#!/bin/bash
# round 3: PCIe loop (copy-first ordering), all-188 step with the 8-class on 16- / 8-step windows (same box),
# then the remaining clean secondary lines
set -o pipefail
OUT=gpurun_out/r03t
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --workload pdsch --steps 5 --warmup 2 --cpu-seconds 0 > $OUT/pdsch.json 2> $OUT/pdsch.err || { tail -5 $OUT/pdsch.err; exit 1; }
python -c "import json; d=json.load(open('$OUT/pdsch.json')); c=d['config']; print('pdsch', c['subframes_per_s'], c['subframes_per_s_h2d_inclusive'], c['h2d_copy_only_subframes_per_s'])" || exit 1
for w in 0 800 0 800; do
  timeout -k 10 300 python bench.py --w8-max-k $w --cpu-seconds 0 --pdsch-steps 0 > $OUT/all188_w$w.json 2> $OUT/all188_w$w.err || { tail -5 $OUT/all188_w$w.err; exit 1; }
  python -c "import json; d=json.load(open('$OUT/all188_w$w.json')); print('w8 $w', d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'], d['per_kernel_mbps'])" || exit 1
done
OUTN=gpurun_out/r03n
run() {
  local n=$1; shift
  timeout -k 10 300 python bench.py "$@" --steps 5 --warmup 2 > $OUTN/$n.json 2> $OUTN/$n.err || { echo "$n failed"; tail -5 $OUTN/$n.err; return 1; }
  python -c "import json; d=json.load(open('$OUTN/$n.json')); print('$n', d['value'], d['unit'], d['ms_per_step'], (d.get('roofline') or {}).get('kernel'), (d.get('cpu_baseline') or {}).get('value'))"
}
run dlloop --workload dlloop --cpu-seconds 0 &&
run ldpc_bg1 --workload ldpc --cpu-seconds 6 &&
run ldpc_bg2 --workload ldpc --bg 2 --cpu-seconds 0 &&
run nrsch --workload nrsch --cpu-seconds 6 &&
run pdsch_low --workload pdsch --snr 17 --cpu-seconds 0 &&
echo done
