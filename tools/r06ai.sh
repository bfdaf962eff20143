# same-box A/B: HEAD library (ab_old.so) vs this tree (persistent-capable multi kernel) at cap 0 and 2 a CU
set -o pipefail
A="--steps 30 --cpu-seconds 0 --pdsch-steps 0 --pdsch-low-snr 0"
O=SRSRAN_AMD_LIB=srsran_4g_amd/lib/ab_old.so
bash tools/gpu_run.sh r06ai bench:warm:"--steps 10 --cpu-seconds 0 --pdsch-steps 0 --pdsch-low-snr 0" \
  benche:old1:$O:"$A" bench:new1:"$A" benche:p2a:SRSRAN_AMD_TDEC_MID_PERSIST=2:"$A" \
  benche:old2:$O:"$A" bench:new2:"$A" benche:p2b:SRSRAN_AMD_TDEC_MID_PERSIST=2:"$A"
