#!/bin/bash
# Round-3 GPU session: full -m gpu suite, the default bench line, rocprofv3 stats of the default bench.
# Usage: tools/gpu_r03.sh TAG [skip-tests]
set -o pipefail
TAG=${1:-r03}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
if [ "$2" != "skip-tests" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/pytest_gpu.log
  [ $rc -eq 0 ] || exit 1
fi
timeout -k 10 400 python bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err || { echo bench failed; tail -20 $OUT/bench_default.err; exit 1; }
cat $OUT/bench_default.json
cd /tmp && cd - > /dev/null
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o default -- python3 bench.py --steps 5 --warmup 2 --cpu-seconds 0 --pdsch-cpu-seconds 0 > $OUT/prof_stdout.log 2>&1 || { echo prof failed; exit 1; }
find $OUT/prof -name "*stats*"
