#!/bin/bash
# round 3 closing run (5): the whole -m gpu suite, smoke(), the default bench line, rocprofv3 kernel stats of it
set -o pipefail
OUT=gpurun_out/r03_final5
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1 || { tail -5 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 600 python bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err || { tail -5 $OUT/bench_default.err; exit 1; }
python -c "import json; d=json.load(open('$OUT/bench_default.json')); print(d['value'], d['ms_per_step'], d['roofline'], d['pdsch_subframes_per_s'], d['pdsch']['subframes_per_s_h2d_inclusive'])"
R=$GRAFT_REPO_ROOT
cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$OUT/prof -o run -- python3 $R/bench.py --steps 5 --warmup 2 --cpu-seconds 0 --pdsch-cpu-seconds 0 > $R/$OUT/bench_prof.json 2> $R/$OUT/bench_prof.err || { tail -5 $R/$OUT/bench_prof.err; exit 1; }
echo done
