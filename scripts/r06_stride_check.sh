# After a launcher change: GPU tests, the default bench line twice, the 8-way
# shard step plain and under a 1-rank torchrun, the pipelined per-rank
# projection.
#   gpurun -- bash scripts/r06_stride_check.sh TAG
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
tag=${1:-x}
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/tests_$tag.log 2>&1
bash scripts/gpu.sh bench ${tag}_a
bash scripts/gpu.sh bench ${tag}_b
A="--field-size 1.25e8 --steps 200 --warmup 20 --no-cpu-baseline"
bash scripts/gpu.sh bench ${tag}_s8 $A
bash scripts/gpu.sh torchrun 1 ${tag}_s8tr $A
timeout -k 10 300 python3 scripts/shard_pipelined.py > gpurun_out/shard_pipelined_$tag.log 2> gpurun_out/shard_pipelined_$tag.err
