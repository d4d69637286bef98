# Round-2 (second session) refresh: all GPU tests, the bench line, every
# BASELINE config, the massive field whole and dealt 8 ways.
set -e
cd /root/repo
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t_all.log 2>&1
timeout -k 10 300 python3 bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err
timeout -k 10 300 python3 -u scripts/bench_configs.py > gpurun_out/configs.jsonl 2> gpurun_out/configs.err
timeout -k 10 300 python3 -u scripts/massive_deal.py 8 3 > gpurun_out/massive_deal_8.log 2>&1
