#!/bin/bash
# round 3: one clean bench line per secondary workload at HEAD (no profiler attached)
set -o pipefail
OUT=gpurun_out/r03n
mkdir -p $OUT
export TMPDIR=/tmp
run() {  # name, bench args...
  local n=$1; shift
  timeout -k 10 300 python bench.py "$@" --steps 5 --warmup 2 > $OUT/$n.json 2> $OUT/$n.err || { echo "$n failed"; tail -5 $OUT/$n.err; return 1; }
  python -c "import json; d=json.load(open('$OUT/$n.json')); print('$n', d['value'], d['unit'], d['ms_per_step'], (d.get('roofline') or {}).get('kernel'), (d.get('roofline') or {}).get('frac'), (d.get('cpu_baseline') or {}).get('value'))"
}
run k6144 --workload k6144 --cpu-seconds 6 &&
run dlsch --workload dlsch --cpu-seconds 6 &&
run ulsch --workload ulsch --cpu-seconds 6 &&
run pusch --workload pusch --cpu-seconds 6 &&
run dlenc --workload dlenc --cpu-seconds 6 &&
run dlloop --workload dlloop --cpu-seconds 0 &&
run ldpc_bg1 --workload ldpc --cpu-seconds 6 &&
run ldpc_bg2 --workload ldpc --bg 2 --cpu-seconds 0 &&
run nrsch --workload nrsch --cpu-seconds 6 &&
run pdsch_low --workload pdsch --snr 17 --cpu-seconds 0 &&
echo done
