# Kernel + memory-copy trace of the 8-way shard step in a 1-rank process group
# (environment, no launcher) with the default shared-memory exchange: the
# field kernels only, no copy or collective kernels per step.
#   gpurun -- bash scripts/exch_trace.sh
set -e -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
export WORLD_SIZE=1 RANK=0 LOCAL_RANK=0 LOCAL_WORLD_SIZE=1 MASTER_ADDR=127.0.0.1 MASTER_PORT=$((29500 + RANDOM % 400))
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv \
    -d "$R/gpurun_out/prof_shm" -o run -- python3 "$R/bench.py" --gpus 1 --field-size 1.25e8 --steps 50 \
    --warmup 20 --no-cpu-baseline > "$R/gpurun_out/prof_shm.json" 2> "$R/gpurun_out/prof_shm.err"
