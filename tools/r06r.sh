# bit layout by launch kind (natural for plain launches, slot for DL-SCH batches): decoder tests + A/B vs previous commit
set -o pipefail
A="--steps 30 --cpu-seconds 0 --pdsch-steps 0 --pdsch-low-snr 0"
bash tools/gpu_run.sh r06r "tests:tests/test_tdec_gpu.py,tests/test_tdec16_gpu.py,tests/test_tdec8s_gpu.py,tests/test_tdec_w8_gpu.py,tests/test_tdec_fullsize_gpu.py,tests/test_sch_gpu.py,tests/test_pdsch_gpu.py" \
  benche:old1:SRSRAN_AMD_LIB=srsran_4g_amd/lib/ab_old.so:"$A" bench:new1:"$A" \
  benche:old2:SRSRAN_AMD_LIB=srsran_4g_amd/lib/ab_old.so:"$A" bench:new2:"$A"
