# Same-box A/B of library builds (scripts/lib_ab.py), interleaved processes.
set -e -o pipefail
for i in 1 2; do
  for d in ab_old ab_b583c6d ab_4b8c21e ab_6cd8e0c .; do
    timeout -k 10 120 python3 scripts/lib_ab.py $d 80:1e9 60:1e9 >> gpurun_out/lib_ab4.log 2>&1
  done
done
