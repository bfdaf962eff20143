#!/bin/bash
# round 3: batched UCI PUSCH path, retuned decoder thresholds
set -o pipefail
OUT=gpurun_out/r03e
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_pusch_gpu.py tests/test_uci_gpu.py tests/test_sch_gpu.py tests/test_tdec16_gpu.py tests/test_tdec8s_gpu.py tests/test_tdec_fullsize_gpu.py tests/test_tdec_gpu.py tests/test_pdsch_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 $OUT/pytest.log; [ $rc -eq 0 ] || exit 1
for K in 408 512 800; do
  for b in 256 512 1024; do
    for k in single quad; do
      timeout -k 10 120 python tools/tdec_kernels.py --kernel $k --K $K --batch $b --launches 3 || exit 1
    done
  done
done
timeout -k 10 300 python bench.py --workload pusch --steps 5 --warmup 2 --cpu-seconds 0 > $OUT/pusch.json 2> $OUT/pusch.err || { tail -5 $OUT/pusch.err; exit 1; }
python -c "import json; d=json.load(open('$OUT/pusch.json')); print('pusch', d['value'], d['ms_per_step'], d['config']['tb_ok_fraction'])"
timeout -k 10 400 python bench.py --steps 5 --warmup 2 --cpu-seconds 0 --pdsch-cpu-seconds 0 --pdsch-low-snr 17 > $OUT/bench_default.json 2> $OUT/bench_default.err || { tail -5 $OUT/bench_default.err; exit 1; }
python -c "
import json; d=json.load(open('$OUT/bench_default.json'))
print('all188', d['value'], d['ms_per_step'], d['roofline']['kernel'], d['roofline']['avg_launch_ms'], d['per_kernel_mbps'], d['output_check'])
p=d['pdsch']; print('pdsch', p['subframes_per_s'], p['subframes_per_s_h2d_inclusive'], p['roofline']['kernel'], p['avg_half_iterations'])
print('low', d.get('pdsch_low_snr'))"
