# rocprofv3 PMC passes of one A/B check binary (scripts/ubench/sib_check.hip):
#   bash scripts/ubench/pmc_sib.sh TAG BIN
set -e -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
tag=$1; bin=$2
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_SALU \
    --output-format csv -d "$R/gpurun_out/pmcs_${tag}_1" -o p -- "$R/$bin" 1916284264916 1000000000 1 > "$R/gpurun_out/pmcs_${tag}_1.log" 2>&1 || [ $? -eq 1 ]
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_INSTS_SMEM SQ_WAVES \
    --output-format csv -d "$R/gpurun_out/pmcs_${tag}_2" -o p -- "$R/$bin" 1916284264916 1000000000 1 > "$R/gpurun_out/pmcs_${tag}_2.log" 2>&1 || [ $? -eq 1 ]
