#!/bin/bash
# round 3 closing run: the whole -m gpu suite, smoke(), the default bench line, rocprofv3 kernel stats of it
set -o pipefail
OUT=gpurun_out/r03_final
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1 || { tail -5 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 600 python bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err || { tail -5 $OUT/bench_default.err; exit 1; }
cat $OUT/bench_default.json
cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$OUT/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 2 --cpu-seconds 0 --pdsch-cpu-seconds 0 > $GRAFT_REPO_ROOT/$OUT/bench_prof.json 2> $GRAFT_REPO_ROOT/$OUT/bench_prof.err || { tail -5 $GRAFT_REPO_ROOT/$OUT/bench_prof.err; exit 1; }
timeout -k 10 300 python bench.py --workload pdsch --nfft 1536 --steps 5 --warmup 2 --cpu-seconds 0 > $OUT/pdsch_1536.json 2> $OUT/pdsch_1536.err || { tail -5 $OUT/pdsch_1536.err; exit 1; }
echo bench-done
bash tools/pmc.sh r03_pmc_pdsch pdsch || exit 1
python tools/pmc_summary.py gpurun_out/r03_pmc_pdsch pdsch gpurun_out/r03_pmc_pdsch/summary.json || exit 1
echo done2
