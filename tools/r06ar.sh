# PUSCH workers: run-to-run spread of 1 and 2 workers, 20 and 60 steps
set -o pipefail
bash tools/gpu_run.sh r06ar bench:w1:"--workload pusch --steps 20 --cpu-seconds 0 --pusch-workers 1" \
  bench:w2a:"--workload pusch --steps 20 --cpu-seconds 0 --pusch-workers 2" \
  bench:w2b:"--workload pusch --steps 20 --cpu-seconds 0 --pusch-workers 2" \
  bench:w2c:"--workload pusch --steps 60 --cpu-seconds 0 --pusch-workers 2" \
  bench:w1b:"--workload pusch --steps 60 --cpu-seconds 0 --pusch-workers 1"
for f in w1 w2a w2b w2c w1b; do python3 -c "
import json; d=json.loads(open('gpurun_out/r06ar/bench_$f.json').read().strip().splitlines()[-1]); c=d['config']
print('$f', c['ue_subframes_per_s'], d['ms_per_step'], c['batch_workers'])"; done
