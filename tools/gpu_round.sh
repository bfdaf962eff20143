#!/bin/bash
# One GPU session: parity tests, both bench workloads, rocprofv3 kernel trace of the k6144 bench.
# Usage: tools/gpu_round.sh TAG
set -o pipefail
TAG=${1:-run}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 500 python -m pytest tests -m gpu -q > $OUT/pytest_gpu.log 2>&1; echo "pytest rc=$?"; tail -2 $OUT/pytest_gpu.log
grep -q " passed" $OUT/pytest_gpu.log || exit 1
grep -q "failed" $OUT/pytest_gpu.log && exit 1
timeout -k 10 300 python bench.py --workload k6144 --steps 20 --warmup 3 --cpu-seconds 10 > $OUT/bench_k6144.json 2> $OUT/bench_k6144.err || exit 1
cat $OUT/bench_k6144.json
timeout -k 10 400 python bench.py --steps 5 --warmup 2 --cpu-seconds 10 > $OUT/bench_all188.json 2> $OUT/bench_all188.err || exit 1
cat $OUT/bench_all188.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o k6144 -- python3 bench.py --workload k6144 --steps 20 --warmup 3 --cpu-seconds 0 > $OUT/prof_stdout.log 2>&1 || exit 1
find $OUT/prof -name "*stats*" | head; 
