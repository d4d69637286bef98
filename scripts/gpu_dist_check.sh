# Dist-path timing: phase medians (plain / torchrun) + bench plain and torchrun 1 rank.
set -e
cd /root/repo
mkdir -p gpurun_out
bash scripts/dop.sh
bash scripts/quick_check.sh
