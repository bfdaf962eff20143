# PMC A/B of the 16-sub-block class of the all-188 step (both multi kernels): previous commit's library vs this tree's
set -o pipefail
bash tools/gpu_run.sh r06q "pmc:old:--workload all188 --lib /root/repo/srsran_4g_amd/lib/ab_old.so --launches 3" "pmc:new:--workload all188 --launches 3"
