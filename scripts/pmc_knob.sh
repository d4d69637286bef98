# PMC passes of one knob value of scripts/knob_sweep.py (probe build), one
# rocprofv3 run per counter group, each under its own time limit:
#   bash scripts/pmc_knob.sh TAG KNOB VALUE FIELD
# -> gpurun_out/pmck_TAG_{lds,busy}/ (counter_collection.csv)
set -e -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
tag=$1; knob=$2; val=$3; field=$4
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_WAVES \
    --output-format csv -d "$R/gpurun_out/pmck_${tag}_lds" -o p -- \
    python3 "$R/scripts/knob_sweep.py" "$knob" "$val" "$field" > "$R/gpurun_out/pmck_${tag}_lds.log" 2>&1
timeout -s KILL 120 rocprofv3 --pmc VALUBusy GRBM_GUI_ACTIVE \
    --output-format csv -d "$R/gpurun_out/pmck_${tag}_busy" -o p -- \
    python3 "$R/scripts/knob_sweep.py" "$knob" "$val" "$field" > "$R/gpurun_out/pmck_${tag}_busy.log" 2>&1
