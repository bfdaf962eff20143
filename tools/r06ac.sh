# decoder time against half-iterations at the C3 batch (K = 6144 x 2028): the fixed part of a launch
set -o pipefail
bash tools/gpu_run.sh r06ac "py:i1:tools/tdec_kernels.py --workload k6144 --batch 2028 --iters 1 --launches 10" \
  "py:i2:tools/tdec_kernels.py --workload k6144 --batch 2028 --iters 2 --launches 10" \
  "py:i3:tools/tdec_kernels.py --workload k6144 --batch 2028 --iters 3 --launches 10" \
  "py:i4:tools/tdec_kernels.py --workload k6144 --batch 2028 --iters 4 --launches 10" \
  "py:j2:tools/tdec_kernels.py --workload k6144 --batch 1024 --iters 2 --launches 10" \
  "py:j1:tools/tdec_kernels.py --workload k6144 --batch 1024 --iters 1 --launches 10"
