# Per-rank load of the 8-way strong split (a 1.25e8 shard of the field with
# its share of niceonly chunks): plain and under torchrun 1 rank (RCCL
# exchange on), 40 and 200 steps.
set -e
cd /root/repo
mkdir -p gpurun_out
B="timeout -k 10 200 python3 bench.py --no-cpu-baseline"
TR="timeout -k 10 200 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1"
$B --steps 40 --warmup 5 --field-size 1.25e8 > gpurun_out/b_shard8.json
$B --steps 200 --warmup 10 --field-size 1.25e8 > gpurun_out/b_shard8_200.json
$TR --master-port 29512 bench.py --steps 40 --warmup 5 --field-size 1.25e8 > gpurun_out/b_tr1_shard8.json 2> gpurun_out/b_tr1_shard8.err
$TR --master-port 29514 bench.py --steps 200 --warmup 10 --field-size 1.25e8 > gpurun_out/b_tr1_shard8_200.json 2> gpurun_out/b_tr1_shard8_200.err
