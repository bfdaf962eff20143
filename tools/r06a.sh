set -o pipefail
bash tools/gpu_run.sh r06a \
 "bench:def:" \
 "py:k3072_w16:tools/tdec_kernels.py --K 3072 --batch 8192 --w8 0" \
 "py:k3072_w8:tools/tdec_kernels.py --K 3072 --batch 8192 --w8 3072" \
 "py:k2048_w16:tools/tdec_kernels.py --K 2048 --batch 8192 --w8 0" \
 "py:k2048_w8:tools/tdec_kernels.py --K 2048 --batch 8192 --w8 2048" \
 "py:k4096_w16:tools/tdec_kernels.py --K 4096 --batch 8192 --w8 0" \
 "py:k4096_w8:tools/tdec_kernels.py --K 4096 --batch 8192 --w8 4096" \
 "py:k6144_w16:tools/tdec_kernels.py --K 6144 --batch 4096 --w8 0"
