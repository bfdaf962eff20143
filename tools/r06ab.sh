# branch-free single-period de-matcher: parity (DL-SCH, UL-SCH, PDSCH, PUSCH) and the chain
set -o pipefail
bash tools/gpu_run.sh r06ab "tests:tests/test_sch_gpu.py,tests/test_pdsch_gpu.py,tests/test_pusch_gpu.py,tests/test_tdd_gpu.py" \
  bench:pd1:"--workload pdsch --steps 30 --cpu-seconds 0" bench:pd2:"--workload pdsch --steps 30 --cpu-seconds 0" \
  "pmcb:pdsch:pdsch --pdsch-workers 1"
