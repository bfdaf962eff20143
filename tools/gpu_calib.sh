#!/bin/bash
# FETCH_SIZE / WRITE_SIZE calibration per access width (tools/fetch_calib.hip), one --pmc pass each
set -o pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/calib
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pf -o pmc -- $GRAFT_REPO_ROOT/tools/fetch_calib > $OUT/fetch.log 2> $OUT/fetch.err || { echo "fetch pass failed"; tail -5 $OUT/fetch.err; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pw -o pmc -- $GRAFT_REPO_ROOT/tools/fetch_calib > $OUT/write.log 2> $OUT/write.err || { echo "write pass failed"; tail -5 $OUT/write.err; exit 1; }
cd $GRAFT_REPO_ROOT && python tools/fetch_calib.py gpurun_out/calib
