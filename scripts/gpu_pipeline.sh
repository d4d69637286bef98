# Pipelined bench: GPU tests, bench at N=1 (pipelined depth 1/2 and --sync),
# torchrun 1 rank, and the per-rank load of an 8-way strong split (1.25e8
# shard of the field; plain and torchrun 1 rank).
set -e
cd /root/repo
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
B="timeout -k 10 200 python3 bench.py --no-cpu-baseline"
TR="timeout -k 10 200 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1"
$B --steps 20 --warmup 5 > gpurun_out/b_pipe.json
$B --steps 20 --warmup 5 --depth 1 > gpurun_out/b_pipe_d1.json
$B --steps 20 --warmup 5 --sync > gpurun_out/b_sync.json
$TR --master-port 29511 bench.py --steps 20 --warmup 5 > gpurun_out/b_tr1.json 2> gpurun_out/b_tr1.err
$TR --master-port 29512 bench.py --steps 40 --warmup 5 --field-size 1.25e8 > gpurun_out/b_tr1_shard8.json 2> gpurun_out/b_tr1_shard8.err
$TR --master-port 29513 bench.py --steps 40 --warmup 5 --field-size 1.25e8 --depth 1 > gpurun_out/b_tr1_shard8_d1.json 2> gpurun_out/b_tr1_shard8_d1.err
$B --steps 40 --warmup 5 --field-size 1.25e8 > gpurun_out/b_shard8.json
$B --steps 40 --warmup 5 --field-size 1.25e8 --depth 1 > gpurun_out/b_shard8_d1.json
