# b40 sibling-kernel variants (probe NICE_FD2_SIB: 142 = the product's VALU-
# decoded C2 + pipelined walk, 132 = pipelined walk without the decode, 141 /
# 131 = per-sibling lookup groups with / without it) on the pipelined bench
# step with round 6's stride picks, probe library, two passes.
#   gpurun -- bash scripts/sib_variant_ab.sh
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
out=gpurun_out/sib_variant.log
for pass in 1 2; do
  for v in 142 132 141 131; do
    for fs in 1e9 1.25e8; do
      NICE_FD2_SIB=$v timeout -k 10 120 python3 bench.py --probe-lib --field-size $fs --steps 60 --warmup 10 \
          --no-cpu-baseline > gpurun_out/sv.json 2> gpurun_out/sv.err
      python3 -c "import json; d=json.loads(open('gpurun_out/sv.json').readline()); print('sib', $v, '$fs', round(d['ms_per_step'],4), round(d['detailed_ms_per_step'],4))" >> $out
    done
  done
done
