#!/bin/bash
# round 3: VALU issue cost / dependent latency of the turbo decoder's instruction forms (micro-benchmark)
set -o pipefail
OUT=gpurun_out/r03y
mkdir -p $OUT
timeout -k 10 60 ./tools/valu_issue > $OUT/valu_issue.jsonl 2> $OUT/valu_issue.err || { tail -5 $OUT/valu_issue.err; exit 1; }
cat $OUT/valu_issue.jsonl
