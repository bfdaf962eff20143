#!/bin/bash
# One GPU session at HEAD: full -m gpu suite, default bench line, rocprof kernel stats of the default bench,
# and the PDSCH bench with its own rocprof summary.
# Usage: tools/gpu_r02.sh TAG [skip-tests]
set -o pipefail
TAG=${1:-run}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
if [ "$2" != "skip-tests" ]; then
  timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
  rc=$?; tail -4 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
fi
timeout -k 10 300 python bench.py > $OUT/bench.json 2> $OUT/bench.err || exit 1
cat $OUT/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_all188 -o all188 -- \
  python3 bench.py --steps 5 --warmup 2 --cpu-seconds 0 --pdsch-steps 0 > $OUT/prof_all188.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_pdsch -o pdsch -- \
  python3 bench.py --workload pdsch --steps 5 --warmup 2 --cpu-seconds 0 > $OUT/prof_pdsch.log 2>&1 || exit 1
find $OUT -name "*kernel_stats*"
