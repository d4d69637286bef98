# GPU tests + small-field configs + pipeline at full and 8-way shard size.
set -e
cd /root/repo
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t_all.log 2>&1
timeout -k 10 300 python3 -u scripts/bench_configs.py > gpurun_out/configs.jsonl 2> gpurun_out/configs.err
B="timeout -k 10 200 python3 bench.py --no-cpu-baseline"
TR="timeout -k 10 200 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1"
$B > gpurun_out/b_pipe.json
$TR --master-port 29512 bench.py --steps 40 --field-size 1.25e8 > gpurun_out/b_tr1_shard8.json 2> gpurun_out/b_tr1_shard8.err
$B --steps 40 --field-size 1.25e8 > gpurun_out/b_shard8.json
