# PMC passes over the detailed b40 1e9 field (prof_detailed.py, 2 reps), one
# counter group per rocprofv3 run; output under gpurun_out/pmc_<tag>_<n>.
set -e
tag=${1:-x}
cd /tmp && export TMPDIR=/tmp
R=/root/repo
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES" \
           "SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES SQ_INSTS_SALU GRBM_GUI_ACTIVE GRBM_COUNT" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $grp --output-format csv -d $R/gpurun_out/pmc_${tag}_$i -o p -- python3 $R/scripts/prof_detailed.py 2 > $R/gpurun_out/pmc_${tag}_$i.log 2>&1
done
