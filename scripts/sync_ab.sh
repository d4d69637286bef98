# Bench-step A/B (alternating, 20 steps each, no CPU baseline): detailed
# workgroup size (NICE_FD2_WG512=1 vs the 1024-thread default) and the two
# modes at once vs in sequence (--sequential), printed as ms/step, both-modes
# wall median and detailed kernel ms.
set -e
cd /root/repo
for i in 1 2; do
  # (the workgroup-size leg needs the probe build: scripts/wg_ab.sh)
  timeout -k 10 120 python bench.py --no-cpu-baseline --steps 20 > gpurun_out/ab_default_$i.json
  timeout -k 10 120 python bench.py --no-cpu-baseline --steps 20 --sequential > gpurun_out/ab_seq_$i.json
done
for f in gpurun_out/ab_*.json; do
  python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], round(d['ms_per_step'],4), round(d.get('both_wall_ms_median',0),4), round(d['roofline']['kernel_ms'],4))" $f
done
