# DL-SCH-mode decoder vs the plain kernel, both K = 6144 x 2028 blocks at 2 half-iterations (the C3 batch)
set -o pipefail
bash tools/gpu_run.sh r06t "py:plain2:tools/tdec_kernels.py --workload k6144 --batch 2028 --iters 2 --launches 10" \
  "py:plain8:tools/tdec_kernels.py --workload k6144 --batch 2028 --iters 8 --launches 5" \
  "prof:chain1:--workload pdsch --pdsch-workers 1 --steps 30 --cpu-seconds 0"
