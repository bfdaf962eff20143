# A/B of the decoder library: the previous commit's (ab_old.so) and this tree's, alternating, headline only
set -o pipefail
A="--steps 30 --cpu-seconds 0 --pdsch-steps 0 --pdsch-low-snr 0"
bash tools/gpu_run.sh r06o benche:old1:SRSRAN_AMD_LIB=srsran_4g_amd/lib/ab_old.so:"$A" bench:new1:"$A" \
  benche:old2:SRSRAN_AMD_LIB=srsran_4g_amd/lib/ab_old.so:"$A" bench:new2:"$A"
