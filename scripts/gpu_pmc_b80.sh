# PMC passes over the b80 detailed kernel (2e8 field, 2 reps): LDS activity and
# bank conflicts vs VALU issue, to tell an LDS-bound kernel from a latency-
# bound one at its 2 waves/SIMD.  One rocprofv3 --pmc run per group.
set -e
tag=${1:-b80}
cd /tmp && export TMPDIR=/tmp
R=/root/repo
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES" \
           "SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES SQ_INSTS_SALU GRBM_GUI_ACTIVE GRBM_COUNT" \
           "VALUBusy"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $grp --output-format csv -d $R/gpurun_out/pmc_${tag}_$i -o p -- python3 $R/scripts/prof_detailed.py 2 detailed 80 2e8 > $R/gpurun_out/pmc_${tag}_$i.log 2>&1
done
