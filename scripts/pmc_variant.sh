# Two rocprofv3 --pmc passes of one probe-build knob value of
# scripts/knob_sweep.py (LDS and issue/wait groups), each under its own limit:
#   bash scripts/pmc_variant.sh TAG KNOB VALUE FIELD
# -> gpurun_out/pmcv_TAG_{lds,wait}/ ; summarise with scripts/pmc_summary.py
set -e -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
tag=$1; knob=$2; val=$3; field=$4
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT \
    SQ_LDS_ADDR_CONFLICT SQ_WAVES GRBM_GUI_ACTIVE \
    --output-format csv -d "$R/gpurun_out/pmcv_${tag}_lds" -o p -- \
    python3 "$R/scripts/knob_sweep.py" "$knob" "$val" "$field" > "$R/gpurun_out/pmcv_${tag}_lds.log" 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY \
    SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_WAIT_ANY GRBM_GUI_ACTIVE \
    --output-format csv -d "$R/gpurun_out/pmcv_${tag}_wait" -o p -- \
    python3 "$R/scripts/knob_sweep.py" "$knob" "$val" "$field" > "$R/gpurun_out/pmcv_${tag}_wait.log" 2>&1
