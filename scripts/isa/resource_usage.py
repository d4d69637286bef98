"""Per-kernel VGPRs / AGPRs / scratch / occupancy / LDS from hipcc's
-Rpass-analysis=kernel-resource-usage remarks (stderr of the build).

    python scripts/isa/resource_usage.py BUILD.log [NAME_SUBSTRING]"""
import re
import sys

cur, rows = None, {}
for ln in open(sys.argv[1]):
    m = re.search(r"Function Name: (\S+)", ln)
    if m:
        cur = m.group(1)
        rows.setdefault(cur, {})
        continue
    m = re.search(r"remark:.*?\s+(VGPRs|AGPRs|ScratchSize \[bytes/lane\]|Occupancy \[waves/SIMD\]|LDS Size \[bytes/block\]): (\d+)", ln)
    if m and cur:
        rows[cur][m.group(1).split()[0]] = int(m.group(2))
sub = sys.argv[2] if len(sys.argv) > 2 else "fd2_kernel"
for k, v in rows.items():
    if sub in k:
        cfg = re.search(r"CfgILi(.*?)EEEE", k)
        name = cfg.group(1).replace("ELi", ",").replace("Li", "") if cfg else k
        print(f"Cfg<{name}>  VGPR {v.get('VGPRs')} AGPR {v.get('AGPRs')} scratch {v.get('ScratchSize')} B/lane  "
              f"occupancy {v.get('Occupancy')} waves/SIMD  LDS {v.get('LDS')} B")
