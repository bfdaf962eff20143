set -o pipefail
mkdir -p gpurun_out/r06l
timeout -k 10 300 python tools/chain_stamps.py --snr 17 > gpurun_out/r06l/chain17.json 2> gpurun_out/r06l/chain.err && \
timeout -k 10 300 python tools/chain_stamps.py --snr 30 > gpurun_out/r06l/chain30.json 2>> gpurun_out/r06l/chain.err && \
cat gpurun_out/r06l/chain17.json gpurun_out/r06l/chain30.json && \
bash tools/gpu_run.sh r06l "tests:tests/test_enb_dl_ref_api_gpu.py,tests/test_pdsch_tx_ref_gpu.py,tests/test_enb_dl_gpu.py,tests/test_enb_ctrl_gpu.py,tests/test_enb_ue_loop_gpu.py"
