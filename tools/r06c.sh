set -o pipefail
P1="SQC_ICACHE_HITS SQC_ICACHE_MISSES SQ_IFETCH SQ_INSTS SQ_WAVES GRBM_GUI_ACTIVE SQ_INSTS_VALU"
P2="SQC_ICACHE_REQ SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH_LEVEL SQ_INSTS_BRANCH SQ_INSTS_SMEM SQ_WAVES"
P3="SQC_TC_INST_REQ SQC_TC_STALL SQ_WAVES SQ_INST_CYCLES_SALU"
export PASSES="$P1;$P2;$P3"
bash tools/pmc_passes.sh r06c/k2048_w16 --K 2048 --batch 8192 --w8 0 --launches 3 && \
bash tools/pmc_passes.sh r06c/k2048_w8 --K 2048 --batch 8192 --w8 2048 --launches 3 && \
bash tools/pmc_passes.sh r06c/k6144_w16 --K 6144 --batch 4096 --w8 0 --launches 3
