set -o pipefail
bash tools/gpu_run.sh r06e \
 "py:k2048_w16:tools/tdec_kernels.py --K 2048 --batch 65536 --w8 0 --launches 3" \
 "py:k2048_w8:tools/tdec_kernels.py --K 2048 --batch 65536 --w8 2048 --launches 3" \
 "py:k1024_w16:tools/tdec_kernels.py --K 1024 --batch 65536 --w8 0 --launches 3" \
 "py:k1024_w8:tools/tdec_kernels.py --K 1024 --batch 65536 --w8 1024 --launches 3" \
 "py:k3072_w16:tools/tdec_kernels.py --K 3072 --batch 32768 --w8 0 --launches 3" \
 "py:k3072_w8:tools/tdec_kernels.py --K 3072 --batch 32768 --w8 3072 --launches 3"
