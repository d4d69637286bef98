# PMC over the niceonly pipeline of the b40 1e9 field (per-dispatch counters).
set -e
cd /tmp && export TMPDIR=/tmp
R=/root/repo
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY --output-format csv -d $R/gpurun_out/pmc_nice -o p -- python3 $R/scripts/prof_detailed.py 2 niceonly > $R/gpurun_out/pmc_nice.log 2>&1
