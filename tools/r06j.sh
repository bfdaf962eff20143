set -o pipefail
bash tools/gpu_run.sh r06j \
 "tests:tests/test_tdec_gpu.py,tests/test_tdec_w8_gpu.py,tests/test_tdec8s_gpu.py,tests/test_tdec16_gpu.py,tests/test_tdec1s_gpu.py,tests/test_sch_gpu.py,tests/test_pdsch_gpu.py,tests/test_tdec_fullsize_gpu.py" \
 "bench:def:"
