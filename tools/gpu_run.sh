#!/bin/bash
# One GPU lease (gpurun), parameterised: runs the named steps in order, each under its own time limit,
# and stops at the first failure (no GPU step after a fault, abort or timeout).
#
# Usage: tools/gpu_run.sh TAG STEP [STEP ...]      output under gpurun_out/TAG/
#   tests[:PYTEST_SELECTION]   pytest -m gpu (default: tests), e.g. tests:tests/test_pusch_gpu.py
#   testse:ENV:SELECTION       the same with ENV (VAR=VAL[,VAR=VAL]) in the environment
#   smoke                      __graft_entry__.smoke()
#   bench:NAME[:ARGS]          python bench.py ARGS > bench_NAME.json (ARGS space-separated, e.g. "--steps 10")
#   benche:NAME:ENV:ARGS       the same with ENV (VAR=VAL[,VAR=VAL]) in the environment
#   prof:NAME[:ARGS]           rocprofv3 --kernel-trace --stats of bench.py ARGS -> prof_NAME/
#   pmc:NAME[:ARGS]            tools/pmc_tdec.sh passes over tools/tdec_kernels.py ARGS -> NAME/
#   pmcb:NAME:WORKLOAD[ ARGS]  tools/pmc.sh passes over bench.py --workload WORKLOAD ARGS -> NAME/summary.json
#   py:NAME:SCRIPT[ ARGS]      python SCRIPT ARGS > NAME.log
set -o pipefail
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
for STEP in "$@"; do
  KIND=${STEP%%:*}; REST=${STEP#*:}; [ "$REST" = "$STEP" ] && REST=""
  NAME=${REST%%:*}; ARGS=${REST#*:}; [ "$ARGS" = "$REST" ] && ARGS=""
  echo "== $STEP"
  case $KIND in
    tests)
      SEL=${REST:-tests}; SEL=${SEL//,/ }
      timeout -k 10 900 python -u -m pytest $SEL -m gpu -q -x --timeout 300 --timeout-method thread \
        > $OUT/pytest_gpu.log 2>&1
      rc=$?; tail -3 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || { echo "pytest rc=$rc"; exit 1; } ;;
    testse)  # testse:VAR=VAL[,VAR=VAL]:SELECTION -- pytest -m gpu with environment settings
      ENVS=${REST%%:*}; SEL=${REST#*:}
      timeout -k 10 900 env ${ENVS//,/ } python -u -m pytest $SEL -m gpu -q -x --timeout 300 --timeout-method thread \
        > $OUT/pytest_gpu_env.log 2>&1
      rc=$?; tail -3 $OUT/pytest_gpu_env.log; [ $rc -eq 0 ] || { echo "pytest rc=$rc"; exit 1; } ;;
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 \
        || { tail -5 $OUT/smoke.log; exit 1; }
      tail -2 $OUT/smoke.log ;;
    bench)
      timeout -k 10 900 python bench.py $ARGS > $OUT/bench_$NAME.json 2> $OUT/bench_$NAME.err \
        || { tail -5 $OUT/bench_$NAME.err; exit 1; }
      python tools/bench_brief.py $OUT/bench_$NAME.json ;;
    benche)  # benche:NAME:VAR=VAL[,VAR=VAL]:ARGS -- bench with environment settings
      ENVS=${ARGS%%:*}; BARGS=${ARGS#*:}; [ "$BARGS" = "$ARGS" ] && BARGS=""
      timeout -k 10 900 env ${ENVS//,/ } python bench.py $BARGS > $OUT/bench_$NAME.json 2> $OUT/bench_$NAME.err \
        || { tail -5 $OUT/bench_$NAME.err; exit 1; }
      python tools/bench_brief.py $OUT/bench_$NAME.json ;;
    prof)
      (cd /tmp && timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$NAME -o run \
        -- python3 $R/bench.py $ARGS > $OUT/prof_$NAME.json 2> $OUT/prof_$NAME.err) \
        || { tail -5 $OUT/prof_$NAME.err; exit 1; }
      python tools/bench_brief.py $OUT/prof_$NAME.json ;;
    pmc)
      bash $R/tools/pmc_tdec.sh $TAG/$NAME $ARGS || exit 1 ;;
    pmcb)
      bash $R/tools/pmc.sh $TAG/$NAME $ARGS || exit 1
      (cd $R && python tools/pmc_summary.py gpurun_out/$TAG/$NAME ${ARGS%% *} gpurun_out/$TAG/$NAME/summary.json) ;;
    py)
      timeout -k 10 600 python $ARGS > $OUT/$NAME.log 2>&1 || { tail -8 $OUT/$NAME.log; exit 1; }
      tail -4 $OUT/$NAME.log ;;
    *) echo "unknown step $STEP"; exit 2 ;;
  esac
done
echo "all steps done"
