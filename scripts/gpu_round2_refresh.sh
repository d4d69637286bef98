# Round-2 refresh: GPU tests, the bench line (with the CPU baseline), torchrun
# 1 rank, rocprofv3 kernel-trace summaries (default pipelined command and
# --sync), the PMC traffic passes of the detailed kernel, all BASELINE configs.
set -e
cd /root/repo
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t_all.log 2>&1
timeout -k 10 300 python3 bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err
timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 1 --no-cpu-baseline > gpurun_out/bench_tr1.json 2> gpurun_out/bench_tr1.err
bash scripts/gpu_prof.sh prof_default --steps 20 --warmup 5
bash scripts/gpu_prof.sh prof_sync --steps 20 --warmup 5 --sync
cd /tmp && export TMPDIR=/tmp
R=/root/repo
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/pmc_fetch -o p -- python3 $R/scripts/prof_detailed.py 2 > $R/gpurun_out/pmc_fetch.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/gpurun_out/pmc_write -o p -- python3 $R/scripts/prof_detailed.py 2 > $R/gpurun_out/pmc_write.log 2>&1
cd $R
timeout -k 10 300 python3 -u scripts/bench_configs.py > gpurun_out/configs.jsonl 2> gpurun_out/configs.err
timeout -k 10 300 python3 -u scripts/massive_deal.py 8 3 > gpurun_out/massive_deal_8.log 2>&1
