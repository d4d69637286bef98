# Exchange-backend A/B for the N = 8 shard step (1/8 of the 1e9 b40 field) on
# one GPU: host time per step by phase (scripts/ubench/step_phases.py, a
# world-1 process group from the environment), then bench.py plain and under
# a 1-rank torchrun with the exchange in shared memory (4 and 8 HW queues)
# and over RCCL.
#   gpurun -- bash scripts/exch_ab2.sh
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
A="--field-size 1.25e8 --steps 200 --warmup 20 --no-cpu-baseline"
timeout -k 10 200 python3 scripts/ubench/step_phases.py > gpurun_out/phases.log 2>&1
export WORLD_SIZE=1 RANK=0 LOCAL_RANK=0 MASTER_ADDR=127.0.0.1
for x in nccl gloo shm; do
  MASTER_PORT=$((29500 + RANDOM % 400)) timeout -k 10 200 python3 scripts/ubench/step_phases.py --exchange $x >> gpurun_out/phases.log 2>&1
done
unset WORLD_SIZE RANK LOCAL_RANK
timeout -k 10 300 python3 bench.py $A > gpurun_out/ex_plain.json 2> gpurun_out/ex_plain.err
bash scripts/gpu.sh torchrun 1 ex_shm1 $A
bash scripts/gpu.sh torchrun 1 ex_shm2 $A --exchange-lag 2
bash scripts/gpu.sh torchrun 1 ex_shm1q8 $A --hw-queues 8
bash scripts/gpu.sh torchrun 1 ex_nccl1 $A --exchange-backend nccl
timeout -k 10 300 python3 bench.py $A > gpurun_out/ex_plain2.json 2> gpurun_out/ex_plain2.err
