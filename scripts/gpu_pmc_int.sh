# Integer-issue evidence for the detailed b40 kernel (north star: "rocprof
# VALU-busy and integer-instruction-issue counters"): raw INT32/INT64 VALU
# instruction counts and the tool's own derived VALUBusy / VALUUtilization,
# one rocprofv3 --pmc run per group over scripts/prof_detailed.py (2 reps of
# the 1e9 @ base 40 field).  Summary: scripts/pmc_int_summary.py.
set -e
tag=${1:-int}
cd /tmp && export TMPDIR=/tmp
R=/root/repo
i=0
for grp in "SQ_INSTS_VALU SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_WAVES GRBM_GUI_ACTIVE" \
           "VALUBusy" "VALUUtilization"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $grp --output-format csv -d $R/gpurun_out/pmc_${tag}_$i -o p -- python3 $R/scripts/prof_detailed.py 2 > $R/gpurun_out/pmc_${tag}_$i.log 2>&1
done
