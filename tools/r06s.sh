# OFDM options (keep_dc, freq shift, window offset, phase compensation) + the OFDM / MBSFN / ext-CP suites
set -o pipefail
bash tools/gpu_run.sh r06s "tests:tests/test_ofdm_opts_gpu.py,tests/test_ofdm_gpu.py,tests/test_extcp_gpu.py,tests/test_mbsfn_gpu.py,tests/test_chest_gpu.py,tests/test_enb_dl_gpu.py"
