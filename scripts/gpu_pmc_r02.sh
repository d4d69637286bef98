# Round-2 PMC passes over the production fd2 kernel: b80 (2e8 field at the
# range start) and b40 (1e9), 2 reps each; one rocprofv3 --pmc run per group.
set -e
cd /tmp && export TMPDIR=/tmp
R=/root/repo
for cfg in "b80 80 2e8" "b40 40 1e9"; do
  set -- $cfg
  tag=$1; base=$2; size=$3
  i=0
  for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES" \
             "SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES SQ_INSTS_SALU GRBM_GUI_ACTIVE GRBM_COUNT" \
             "VALUBusy"; do
    i=$((i+1))
    timeout -s KILL 90 rocprofv3 --pmc $grp --output-format csv -d $R/gpurun_out/pmc_r02_${tag}_$i -o p -- python3 $R/scripts/prof_detailed.py 2 detailed $base $size > $R/gpurun_out/pmc_r02_${tag}_$i.log 2>&1
  done
done
