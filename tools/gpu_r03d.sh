#!/bin/bash
# round 3: generic-class threshold, single vs pair at the PDSCH chain's batch sizes, low-SNR operating point
set -o pipefail
OUT=gpurun_out/r03d
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_tdec1s_gpu.py tests/test_tdec_fullsize_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 $OUT/pytest.log; [ $rc -eq 0 ] || exit 1
for b in 256 512 1024 2048; do
  for k in single pair quad; do
    timeout -k 10 120 python tools/tdec_kernels.py --kernel $k --workload k6144 --batch $b --launches 3 || exit 1
  done
done
for k in single quad; do
  timeout -k 10 120 python tools/tdec_kernels.py --kernel $k --workload class8 --batch 256 --launches 3 || exit 1
done
for t in single pair; do
  for snr in 17 17.5; do
    timeout -k 10 200 python bench.py --workload pdsch --snr $snr --tdec16 $t --steps 5 --warmup 2 --cpu-seconds 0 > $OUT/pdsch_${t}_$snr.json 2> $OUT/pdsch_${t}_$snr.err || { tail -5 $OUT/pdsch_${t}_$snr.err; exit 1; }
    python -c "import json; d=json.load(open('$OUT/pdsch_${t}_$snr.json')); c=d['config']; print('pdsch $t $snr', c['subframes_per_s'], c['avg_half_iterations'], c['tb_ok_fraction'], d['roofline']['kernel'], d['roofline']['avg_launch_ms'])"
  done
done
timeout -k 10 400 python bench.py --steps 5 --warmup 2 --cpu-seconds 0 --pdsch-cpu-seconds 0 > $OUT/bench_default.json 2> $OUT/bench_default.err || { tail -5 $OUT/bench_default.err; exit 1; }
python -c "
import json; d=json.load(open('$OUT/bench_default.json'))
print('all188', d['value'], d['ms_per_step'], d['roofline']['kernel'], d['roofline']['avg_launch_ms'], d['per_kernel_mbps'], d['output_check'])"
