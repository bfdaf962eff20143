#!/bin/bash
# round 3: cycles per trellis step with and without the window loads (diagnostic builds)
set -o pipefail
OUT=gpurun_out/r03x
mkdir -p $OUT
export TMPDIR=/tmp
: > $OUT/stamps.jsonl
for lib in stamps stamps_fake; do
  for args in "--K 6144 --batch 1024" "--K 2048 --batch 2048"; do
    timeout -k 10 120 python tools/tdec_stamps.py --lib $lib $args >> $OUT/stamps.jsonl 2> $OUT/stamps.err || { tail -5 $OUT/stamps.err; exit 1; }
  done
done
python - <<'PY'
import json
for l in open("gpurun_out/r03x/stamps.jsonl"):
    d = json.loads(l)
    print(d["lib"], d["kernel"], d["K"], d["batch"], "ms", d["launch_ms"], "GHz", d["clock_ghz_implied"], "half-it", d["half_it_cycles"],
          " ".join(f"{k}={d[k]['cycles_per_step']}" for k in d if isinstance(d[k], dict) and "cycles_per_step" in d[k]))
PY
