# 8-bit decoder as two waves a workgroup (alpha / beta meeting in the middle): parity, then K = 6144 x 1024 timing
set -o pipefail
bash tools/gpu_run.sh r06ag "tests:tests/test_tdec8bit.py,tests/test_llr8_gpu.py" \
  bench:k:"--steps 3 --cpu-seconds 0 --pdsch-steps 0 --pdsch-low-snr 0"
