#!/bin/bash
# GPU parity run: the whole -m gpu suite (or the given test files), one process, per-test timeout.
# Usage: tools/gpu_tests.sh TAG [pytest args...]
set -o pipefail
TAG=${1:-t}
shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest ${@:-tests} -m gpu -x -v --timeout 300 --timeout-method thread -rs > $OUT/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"
tail -15 $OUT/pytest_gpu.log
exit $rc
