# Round-6 lane init from host-supplied start digits (bases whose n passes 64
# bits): GPU tests, then every config and the per-base 1e9 fields.
set -e -o pipefail
bash scripts/gpu.sh tests
timeout -k 10 500 python3 -u scripts/bench_configs.py --bases all > gpurun_out/configs_init.jsonl 2> gpurun_out/configs_init.err
