#!/bin/bash
set -o pipefail
OUT=gpurun_out/r03r
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 240 python tools/h2d_probe.py > $OUT/h2d_probe.jsonl 2> $OUT/h2d_probe.err || { tail -5 $OUT/h2d_probe.err; exit 1; }
cat $OUT/h2d_probe.jsonl
