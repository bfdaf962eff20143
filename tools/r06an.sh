# int16 I/Q input (srsran_ofdm_rx_gpu_sc16, srsran_ue_dl_gpu_decode_batch_sc16): parity, then the PCIe-inclusive rates
set -o pipefail
bash tools/gpu_run.sh r06an "tests:tests/test_ofdm_opts_gpu.py,tests/test_pdsch_gpu.py" \
  bench:pd:"--workload pdsch --steps 30 --cpu-seconds 0"
python3 - <<'PY'
import json
d = json.loads(open("gpurun_out/r06an/bench_pd.json").read().strip().splitlines()[-1])
c = d["config"]
print({k: c[k] for k in c if "h2d" in k or "sc16" in k or k == "subframes_per_s"})
PY
