set -e
cd /tmp && export TMPDIR=/tmp
R=/root/repo
for pr in 0 1 2 3; do
NICE_PROBE_LIB=1 NICE_MSD_PROBE=$pr timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/msdp$pr -o p -- python3 $R/scripts/prof_detailed.py 2 niceonly > $R/gpurun_out/msdp$pr.log 2>&1
done
