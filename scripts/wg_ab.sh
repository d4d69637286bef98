# Detailed kernel ms, 1024- vs 512-thread workgroups (NICE_FD2_WG512=1) under
# the short-chunk launch, b40 / b50 / b80 1e9 fields, alternating.
set -e
cd /root/repo
for i in 1 2; do
  for wg in 1024 512; do
    if [ $wg = 512 ]; then export NICE_FD2_WG512=1; else unset NICE_FD2_WG512; fi
    echo "wg $wg: $(bash scripts/gridx_probe.sh "40 80" "50 160" "80 240" | awk '{printf "%s %s ms  ", $1, $4}')"
  done
done
