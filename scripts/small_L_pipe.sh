# Sibling-lane stride sweep, pipelined (scripts/shard_pipelined.py at world
# 1 over the bench field's first FS numbers, forced L; 0 = the pick).
#   gpurun -- bash scripts/small_L_pipe.sh "FS ..." "L ..." [log]
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
log=${3:-gpurun_out/small_L_pipe.log}
for fs in $1; do
  for L in $2; do
    timeout -k 10 120 python3 scripts/shard_pipelined.py --worlds 1 --field-size $fs --force-L $L --steps ${STEPS:-200} >> $log 2>> $log.err
  done
done
