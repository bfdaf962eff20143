#!/bin/bash
# round 3: 8-step windows as the 8-sub-block class default (parity + class timings against the quad
# decoder), the default bench line, the PCIe loop with a high- / normal-priority copy stream
set -o pipefail
OUT=gpurun_out/r03m
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_tdec_w8_gpu.py tests/test_tdec8s_gpu.py tests/test_tdec_fullsize_gpu.py tests/test_tdec_gpu.py tests/test_sch_gpu.py -m gpu -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAIL|Error|passed|failed" $OUT/pytest.log | head -30; [ $rc -le 1 ] || exit 1
for K in 512 800; do
  for b in 512 1024 2048 4096; do
    timeout -k 10 120 python tools/tdec_kernels.py --kernel quad --K $K --batch $b --launches 3 || exit 1
    timeout -k 10 120 python tools/tdec_kernels.py --kernel single --K $K --batch $b --launches 3 --w8 800 || exit 1
  done
done
timeout -k 10 120 python tools/tdec_kernels.py --kernel quad --workload class8 --batch 1024 --launches 3 || exit 1
timeout -k 10 120 python tools/tdec_kernels.py --kernel single --workload class8 --batch 1024 --launches 3 --w8 800 || exit 1
for pr in 0 -1; do
  timeout -k 10 300 python bench.py --workload pdsch --h2d-priority $pr --steps 5 --warmup 2 --cpu-seconds 0 > $OUT/pdsch_pr$pr.json 2> $OUT/pdsch_pr$pr.err || { tail -5 $OUT/pdsch_pr$pr.err; exit 1; }
  python -c "import json; d=json.load(open('$OUT/pdsch_pr$pr.json')); c=d['config']; print('prio $pr', c['subframes_per_s'], c['subframes_per_s_h2d_inclusive'], c['h2d_copy_only_subframes_per_s'], d['host_enqueue_ms_per_step'], d['host_phases_us_per_call'])" || exit 1
done
timeout -k 10 600 python bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err || { tail -5 $OUT/bench_default.err; exit 1; }
cat $OUT/bench_default.json
echo done
