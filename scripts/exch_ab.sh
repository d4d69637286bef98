# The N = 8 shard step (1/8 of the 1e9 b40 field) on one GPU under a 1-rank
# process group: exchange lag 1 / 2 / 3 (PipelinedExchange), then a kernel +
# memory-copy trace of the lag-1 step with the process group set up from the
# environment (no launcher, so the profiler sits directly on python3).
#   gpurun -- bash scripts/exch_ab.sh
set -e -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
A="--field-size 1.25e8 --steps 200 --warmup 20 --no-cpu-baseline"
timeout -k 10 300 python3 bench.py $A > gpurun_out/ex_plain.json 2> gpurun_out/ex_plain.err
for lag in 1 2 3; do
    bash scripts/gpu.sh torchrun 1 ex_lag$lag $A --exchange-lag $lag
done
export WORLD_SIZE=1 RANK=0 LOCAL_RANK=0 MASTER_ADDR=127.0.0.1 MASTER_PORT=$((29500 + RANDOM % 400))
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv \
    -d "$R/gpurun_out/prof_ex" -o run -- python3 "$R/bench.py" --gpus 1 $A --steps 50 --mode both \
    > "$R/gpurun_out/prof_ex.json" 2> "$R/gpurun_out/prof_ex.err"
