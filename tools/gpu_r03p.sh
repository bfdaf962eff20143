#!/bin/bash
# round 3: (1) branch-free software-pipelined phase 2 -- parity + A/B against the previous build;
# (2) 8-class thresholds with 8-step windows; (3) PCIe loop copy-stream priority A/B with host phases
set -o pipefail
OUT=gpurun_out/r03p
mkdir -p $OUT
export TMPDIR=/tmp
BASE=srsran_4g_amd/lib/ab/libsrsran_4g_amd_base.so
timeout -k 10 600 python -u -m pytest tests/test_tdec16_gpu.py tests/test_tdec8s_gpu.py tests/test_tdec_w8_gpu.py tests/test_tdec_fullsize_gpu.py -m gpu -q -x --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAIL|Error|passed|failed" $OUT/pytest.log | head -20; [ $rc -eq 0 ] || exit 1
for L in "" "--lib $BASE"; do
  timeout -k 10 120 python tools/tdec_kernels.py --kernel single --workload k6144 --batch 1024 --launches 5 $L || exit 1
  timeout -k 10 200 python tools/tdec_kernels.py --kernel single --workload all188 --launches 3 $L || exit 1
done
for K in 512 800; do
  for b in 512 1024 2048 4096; do
    timeout -k 10 120 python tools/tdec_kernels.py --kernel quad --K $K --batch $b --launches 3 --lib $BASE || exit 1
    timeout -k 10 120 python tools/tdec_kernels.py --kernel single --K $K --batch $b --launches 3 --w8 800 --lib $BASE || exit 1
  done
done
for pr in 0 -1; do
  timeout -k 10 300 python bench.py --workload pdsch --h2d-priority $pr --steps 5 --warmup 2 --cpu-seconds 0 > $OUT/pdsch_pr$pr.json 2> $OUT/pdsch_pr$pr.err || { tail -5 $OUT/pdsch_pr$pr.err; exit 1; }
  python -c "import json; d=json.load(open('$OUT/pdsch_pr$pr.json')); c=d['config']; print('prio $pr', c['subframes_per_s'], c['subframes_per_s_h2d_inclusive'], c['h2d_copy_only_subframes_per_s'], d['host_enqueue_ms_per_step'], d['host_phases_us_per_call'])" || exit 1
done
echo done
