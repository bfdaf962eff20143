set -o pipefail
bash tools/gpu_run.sh r06m "tests:tests/test_enb_dl_ref_api_gpu.py,tests/test_tx_ref_api_gpu.py,tests/test_pdsch_tx_ref_gpu.py,tests/test_enb_dl_gpu.py,tests/test_enb_ctrl_gpu.py,tests/test_enb_ue_loop_gpu.py,tests/test_enc_gpu.py,tests/test_sch_gpu.py"
