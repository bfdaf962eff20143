set -o pipefail
mkdir -p gpurun_out/r06b
(cd /tmp && timeout -s KILL 90 rocprofv3 -L > $GRAFT_REPO_ROOT/gpurun_out/r06b/counters.txt 2>&1) || true
grep -o 'SQC_[A-Z_0-9]*\|SQ_IFETCH[A-Z_]*\|SQ_INST[A-Z_]*\|SQ_WAIT[A-Z_]*' gpurun_out/r06b/counters.txt | sort -u > gpurun_out/r06b/sq_names.txt || true
A="SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU"
B="SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE"
export PASSES="$A;$B"
bash tools/pmc_passes.sh r06b/k2048_w16 --K 2048 --batch 8192 --w8 0 --launches 3 && \
bash tools/pmc_passes.sh r06b/k2048_w8 --K 2048 --batch 8192 --w8 2048 --launches 3 && \
bash tools/pmc_passes.sh r06b/k6144_w16 --K 6144 --batch 4096 --w8 0 --launches 3
