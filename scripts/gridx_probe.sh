# Detailed kernel time vs the target chunk (NICE_FD2_TCHUNK, numbers per lane;
# one chunk per lane, as many workgroup rounds as needed) on the b40 / b50 1e9
# and b80 1e9 benchmark fields: "base tchunk -> median kernel ms, result hash".
# Usage: bash scripts/gridx_probe.sh "40 60" "40 100" ...
set -e
cd /root/repo
for cfg in "$@"; do
  set -- $cfg
  NICE_FD2_TCHUNK=$2 timeout -k 10 90 python -c "
import sys, statistics; sys.path.insert(0, '.'); sys.path.insert(0, 'scripts'); import probe_lib
import nice_amd as N
ctx = N.GpuContext(0); s = N.get_base_range_u128($1).range_start
h, l = ctx.detailed_raw(s, s + 10**9, $1); ref = (list(h), sorted(l))
ks = []
for _ in range(5):
    h, l = ctx.detailed_raw(s, s + 10**9, $1); ks.append(ctx.kernel_stats().kernel_ms)
    assert sum(h) == 10**9
print('b$1 tchunk', $2, round(statistics.median(ks), 4), 'ms', hash(str(ref)))
"
done
