# all-188 step with the 16-step kernels compiled under other machine-scheduler strategies (-amdgpu-sched-strategy)
set -o pipefail
A="--steps 30 --cpu-seconds 0 --pdsch-steps 0 --pdsch-low-snr 0"
L=SRSRAN_AMD_LIB=srsran_4g_amd/lib/ab
bash tools/gpu_run.sh r06aj bench:warm:"--steps 10 --cpu-seconds 0 --pdsch-steps 0 --pdsch-low-snr 0" bench:def1:"$A" \
  benche:ilp:$L/lib_max-ilp.so:"$A" benche:itilp:$L/lib_iterative-ilp.so:"$A" benche:mem:$L/lib_max-memory-clause.so:"$A" \
  bench:def2:"$A" benche:ilp2:$L/lib_max-ilp.so:"$A"
