set -e
cd /root/repo
mkdir -p gpurun_out
timeout -k 10 120 python3 scripts/pipeline_phases.py 1.25e8 60 1 > gpurun_out/phases_shard8.log 2>&1
timeout -k 10 120 python3 scripts/pipeline_phases.py 1.25e8 60 2 >> gpurun_out/phases_shard8.log 2>&1
