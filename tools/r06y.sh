# all-188 step: class streams at equal priority (default) vs the first class's stream at the highest priority
set -o pipefail
A="--steps 30 --cpu-seconds 0 --pdsch-steps 0 --pdsch-low-snr 0"
bash tools/gpu_run.sh r06y bench:warm:"--steps 10 --cpu-seconds 0 --pdsch-steps 0 --pdsch-low-snr 0" bench:def1:"$A" \
  benche:prio1:SRSRAN_AMD_TDEC_MULTI=priority:"$A" bench:def2:"$A" benche:prio2:SRSRAN_AMD_TDEC_MULTI=priority:"$A" \
  benche:serial:SRSRAN_AMD_TDEC_MULTI=serial:"$A"
