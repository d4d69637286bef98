# Kernel-trace summary and PMC passes of the massive field (b50 1e13 niceonly,
# one GPU): which kernels take the time, and the niceonly kernel's VALU / LDS
# / memory counters.  The per-dispatch CSVs are summarised on the box and
# removed (thousands of launches).
set -e
cd /tmp && export TMPDIR=/tmp
R=/root/repo
O=$R/gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_massive -o run -- python3 $R/scripts/massive_1gpu.py 10 > $O/prof_massive.log 2>&1
rm -f $O/prof_massive/run_kernel_trace.csv
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_BUSY_CYCLES SQ_WAVE_CYCLES" \
           "VALUBusy" "GRBM_GUI_ACTIVE GRBM_COUNT SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d $O/pmc_massive_$i -o p -- python3 $R/scripts/massive_1gpu.py 10 > $O/pmc_massive_$i.log 2>&1
  for k in niceonly_kernel msd_level_kernel msd_fused_kernel msd_wave_kernel; do
    python3 $R/scripts/pmc_sum_all.py $k $O/pmc_massive_$i/p_counter_collection.csv >> $O/pmc_massive_summary.txt
  done
  rm -f $O/pmc_massive_$i/p_counter_collection.csv
done
