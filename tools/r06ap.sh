# HIP hardware queues a process (GPU_MAX_HW_QUEUES, HIP default 4) against 8: the all-188 step's class streams, the
# 3-worker PDSCH chain, the PUSCH workers
set -o pipefail
A="--steps 30 --cpu-seconds 0 --pdsch-steps 0 --pdsch-low-snr 0"
bash tools/gpu_run.sh r06ap bench:warm:"--steps 10 --cpu-seconds 0 --pdsch-steps 0 --pdsch-low-snr 0" \
  bench:a4:"$A" benche:a8:GPU_MAX_HW_QUEUES=8:"$A" bench:a4b:"$A" benche:a8b:GPU_MAX_HW_QUEUES=8:"$A" \
  bench:p4:"--workload pdsch --steps 30 --cpu-seconds 0" benche:p8:GPU_MAX_HW_QUEUES=8:"--workload pdsch --steps 30 --cpu-seconds 0" \
  benche:p8w4:GPU_MAX_HW_QUEUES=8:"--workload pdsch --steps 30 --cpu-seconds 0 --pdsch-workers 4" \
  benche:u8w3:GPU_MAX_HW_QUEUES=8:"--workload pusch --steps 30 --cpu-seconds 0 --pusch-workers 3" \
  benche:u8w2:GPU_MAX_HW_QUEUES=8:"--workload pusch --steps 30 --cpu-seconds 0 --pusch-workers 2"
for f in p4 p8 p8w4; do python3 -c "
import json; d=json.loads(open('gpurun_out/r06ap/bench_$f.json').read().strip().splitlines()[-1]); print('$f', d['config']['subframes_per_s'], d['ms_per_step'])"; done
for f in u8w3 u8w2; do python3 -c "
import json; d=json.loads(open('gpurun_out/r06ap/bench_$f.json').read().strip().splitlines()[-1]); print('$f', d['config']['ue_subframes_per_s'], d['ms_per_step'])"; done
