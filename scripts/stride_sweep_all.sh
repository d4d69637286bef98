# Pipelined sibling-stride sweep (scripts/ubench/stride_sweep_pipe.py) over
# the sibling-lane bases, every odd L in [61, 255], 1e9 and 1.25e8 fields.
#   gpurun -- bash scripts/stride_sweep_all.sh "40 42 ..." [log]
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
log=${2:-gpurun_out/sweep_all.log}
for b in $1; do
  timeout -k 10 300 python3 scripts/ubench/stride_sweep_pipe.py --base $b --sizes 1e9,1.25e8 --lo 61 --hi 255 \
      --reps ${REPS:-3} --numbers ${NUMBERS:-6e9} >> $log 2>> $log.err
done
