#!/bin/bash
# round 3: cycles per trellis step of the single-lane decoder from in-kernel clock stamps (diagnostic build)
set -o pipefail
OUT=gpurun_out/r03w
mkdir -p $OUT
export TMPDIR=/tmp
: > $OUT/stamps.jsonl
for args in "--K 6144 --batch 1024" "--K 6144 --batch 1024 --w8 6144" "--K 6144 --batch 2048" "--K 1024 --batch 2048" "--K 512 --batch 4096 --w8 800" "--K 512 --batch 4096"; do
  timeout -k 10 120 python tools/tdec_stamps.py $args >> $OUT/stamps.jsonl 2> $OUT/stamps.err || { tail -5 $OUT/stamps.err; exit 1; }
done
cat $OUT/stamps.jsonl
