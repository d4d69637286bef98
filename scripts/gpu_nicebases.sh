set -e
cd /root/repo
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "niceonly" > gpurun_out/t_nice.log 2>&1
timeout -k 10 300 python3 scripts/bench_configs.py --nice-bases 50,52,53,54,55 --only-bases --reps 3 > gpurun_out/configs_nice.jsonl 2> gpurun_out/configs_nice.err
