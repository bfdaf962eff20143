#!/bin/bash
# single-lane decoder bring-up: parity of both 16-class kernels, then all188 / k6144 with each kernel.
set -o pipefail
OUT=gpurun_out/${1:-e8}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_tdec16_gpu.py tests/test_tdec_fullsize_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 $OUT/pytest.log; [ $rc -eq 0 ] || exit 1
for k in single pair; do
  timeout -k 10 300 python bench.py --workload all188 --steps 5 --warmup 2 --cpu-seconds 0 --pdsch-steps 0 --tdec16 $k > $OUT/all188_$k.json 2> $OUT/all188_$k.err || { echo "bench all188 $k failed"; tail -5 $OUT/all188_$k.err; exit 1; }
  python -c "import json; d=json.load(open('$OUT/all188_$k.json')); print('all188 $k', d['value'], d['roofline']['kernel'], d['roofline']['avg_launch_ms'], d['k6144_mbps'], d['output_check'])"
done
for k in single pair quad; do
  for b in 1024 2048 4096; do
    timeout -k 10 200 python bench.py --workload k6144 --batch $b --steps 10 --warmup 2 --cpu-seconds 0 --tdec16 $k > $OUT/k6144_${k}_$b.json 2> $OUT/k6144_${k}_$b.err || { echo "bench k6144 $k $b failed"; tail -5 $OUT/k6144_${k}_$b.err; exit 1; }
    python -c "import json; d=json.load(open('$OUT/k6144_${k}_$b.json')); print('k6144 $k $b', d['value'], d['roofline']['kernel'], d['roofline']['avg_launch_ms'], d['output_check']['mismatched'])"
  done
done
