# PUSCH chain with 1 / 2 / 3 / 4 PHY workers on host threads (srsENB's nof_phy_threads)
set -o pipefail
bash tools/gpu_run.sh r06ao "tests:tests/test_pusch_gpu.py" \
  bench:w1:"--workload pusch --steps 30 --cpu-seconds 0 --pusch-workers 1" \
  bench:w2:"--workload pusch --steps 30 --cpu-seconds 0 --pusch-workers 2" \
  bench:w3:"--workload pusch --steps 30 --cpu-seconds 0 --pusch-workers 3" \
  bench:w4:"--workload pusch --steps 30 --cpu-seconds 0 --pusch-workers 4"
for f in w1 w2 w3 w4; do python3 -c "
import json; d=json.loads(open('gpurun_out/r06ao/bench_$f.json').read().strip().splitlines()[-1]); c=d['config']
print('$f', c['ue_subframes_per_s'], d['ms_per_step'], c['tb_ok_fraction'], c['batch_workers'])"; done
