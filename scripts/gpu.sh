# GPU-box runner (run through gpurun from the repo root):
#   bash scripts/gpu.sh tests                      # pytest -m gpu  -> gpurun_out/tests.log
#   bash scripts/gpu.sh bench TAG [bench args]     # one bench line -> gpurun_out/bench_TAG.json
#   bash scripts/gpu.sh torchrun N TAG [args]      # bench under torchrun, N ranks on device(s)
#   bash scripts/gpu.sh prof TAG [bench args]      # rocprofv3 kernel trace + stats of that bench
#   bash scripts/gpu.sh pmc TAG "COUNTERS" [bench args]   # one rocprofv3 --pmc pass of that bench
#   bash scripts/gpu.sh configs                    # every BASELINE config on one GPU
#   bash scripts/gpu.sh massive                    # whole massive field, dealt 8 ways
# Every GPU step runs under its own time limit; the script stops at the first
# failure (set -e), so nothing runs on the GPU after a fault or a timeout.
set -e -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
mkdir -p gpurun_out
task=$1
shift
case "$task" in
tests)
    timeout -k 10 700 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
        > gpurun_out/tests.log 2>&1 ;;
bench)
    tag=$1; shift
    timeout -k 10 400 python3 bench.py "$@" > gpurun_out/bench_$tag.json 2> gpurun_out/bench_$tag.err ;;
torchrun)
    n=$1; tag=$2; shift 2
    timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node "$n" \
        --master-addr 127.0.0.1 --master-port $((29500 + RANDOM % 400)) bench.py --gpus "$n" "$@" \
        > gpurun_out/tr_$tag.json 2> gpurun_out/tr_$tag.err ;;
prof)
    tag=$1; shift
    cd /tmp && export TMPDIR=/tmp
    timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_$tag" \
        -o run -- python3 "$R/bench.py" --no-cpu-baseline "$@" > "$R/gpurun_out/prof_$tag.json" \
        2> "$R/gpurun_out/prof_$tag.err" ;;
pmc)
    tag=$1; counters=$2; shift 2
    cd /tmp && export TMPDIR=/tmp
    timeout -s KILL 240 rocprofv3 --pmc $counters --output-format csv -d "$R/gpurun_out/pmc_$tag" \
        -o p -- python3 "$R/bench.py" --no-cpu-baseline "$@" > "$R/gpurun_out/pmc_$tag.json" \
        2> "$R/gpurun_out/pmc_$tag.err" ;;
configs)
    timeout -k 10 400 python3 -u scripts/bench_configs.py > gpurun_out/configs.jsonl 2> gpurun_out/configs.err ;;
massive)
    timeout -k 10 300 python3 -u scripts/massive_deal.py 8 3 > gpurun_out/massive_deal_8.log 2>&1 ;;
*)
    echo "unknown task $task" >&2; exit 2 ;;
esac
