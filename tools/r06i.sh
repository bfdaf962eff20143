set -o pipefail
bash tools/gpu_run.sh r06i \
 "tests:tests/test_pdcch_gpu.py,tests/test_tdd_gpu.py,tests/test_chest_gpu.py,tests/test_enb_ue_loop_gpu.py,tests/test_tdec8bit.py,tests/test_llr8_gpu.py,tests/test_pdsch_gpu.py::test_pdsch_fused_matches_two_kernel_path,tests/test_tdec_fullsize_gpu.py" \
 "bench:def:"
