#!/bin/bash
set -o pipefail
OUT=gpurun_out/r03c
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_tdec1s_gpu.py tests/test_tdec8s_gpu.py tests/test_tdec16_gpu.py tests/test_tdec_fullsize_gpu.py tests/test_pdcch_gpu.py tests/test_tdec_gpu.py tests/test_sch_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 $OUT/pytest.log; [ $rc -eq 0 ] || exit 1
for k in single quad; do
  timeout -k 10 120 python tools/tdec_kernels.py --kernel $k --workload class8 --launches 3 || exit 1
  timeout -k 10 120 python tools/tdec_kernels.py --kernel $k --workload class1 --launches 3 || exit 1
done
timeout -k 10 400 python bench.py --steps 5 --warmup 2 --cpu-seconds 0 --pdsch-cpu-seconds 0 > $OUT/bench_default.json 2> $OUT/bench_default.err || { tail -5 $OUT/bench_default.err; exit 1; }
python -c "
import json; d=json.load(open('$OUT/bench_default.json'))
print('all188', d['value'], d['ms_per_step'], d['roofline']['kernel'], d['roofline']['avg_launch_ms'], d['per_kernel_mbps'], d['output_check'])
p=d['pdsch']; print('pdsch', p['subframes_per_s'], p['subframes_per_s_h2d_inclusive'], p['h2d_copy_only_subframes_per_s'], p['roofline']['kernel'], p['avg_half_iterations'])
print('low', d.get('pdsch_low_snr'))"
for snr in 16 18 19 20 22; do
  timeout -k 10 200 python bench.py --workload pdsch --snr $snr --steps 5 --warmup 2 --cpu-seconds 0 > $OUT/pdsch_$snr.json 2> $OUT/pdsch_$snr.err || { tail -5 $OUT/pdsch_$snr.err; exit 1; }
  python -c "import json; d=json.load(open('$OUT/pdsch_$snr.json'))['config']; print('snr $snr', d['subframes_per_s'], d['avg_half_iterations'], d['tb_ok_fraction'])"
done
