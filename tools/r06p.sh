# PMC A/B of the 16-sub-block decoder at K = 6144 (8 half-iterations): previous commit's library vs this tree's
set -o pipefail
bash tools/gpu_run.sh r06p "pmc:old:--workload k6144 --lib /root/repo/srsran_4g_amd/lib/ab_old.so" "pmc:new:--workload k6144" \
  "py:t_old:tools/tdec_kernels.py --workload k6144 --lib /root/repo/srsran_4g_amd/lib/ab_old.so --launches 10" \
  "py:t_new:tools/tdec_kernels.py --workload k6144 --launches 10" \
  "py:a_old:tools/tdec_kernels.py --workload all188 --lib /root/repo/srsran_4g_amd/lib/ab_old.so --launches 10" \
  "py:a_new:tools/tdec_kernels.py --workload all188 --launches 10"
