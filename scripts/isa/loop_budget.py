"""Issue budget of a kernel's hot loop by line range of a --save-temps .s
extract, leaving out the exec-skipped sub-blocks that a list of
`s_cbranch_execz .LBBx_y` targets opens (rare paths inside the loop).

    python scripts/isa/loop_budget.py FILE.s FIRST LAST NUMBERS_PER_ITER [SKIP_TARGET ...]

Lines FIRST..LAST (1-based, inclusive) are the loop's blocks, latch
included; each SKIP_TARGET (e.g. .LBB2_22) drops the lines from the branch
to it up to its label.  Prices VALU opcodes as issue_budget.py does."""
import collections
import re
import sys

sys.path.insert(0, __file__.rsplit("/", 1)[0])
from issue_budget import cost  # noqa: E402

path, first, last, per = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), float(sys.argv[4])
skips = set(sys.argv[5:])
lines = open(path).read().splitlines()[first - 1:last]
c = collections.Counter()
skip = None
for ln in lines:
    s = ln.strip()
    if skip:
        if s.startswith(skip + ":"):
            skip = None
        continue
    m = re.match(r"^s_cbranch_execz (\.LBB\d+_\d+)$", s)
    if m and m.group(1) in skips:
        skip = m.group(1)
        continue
    if not s or s.startswith(";") or s.startswith(".") or s.endswith(":"):
        continue
    c[s.split()[0]] += 1
v = {k: n for k, n in c.items() if k.startswith("v_")}
cyc = sum(n * cost(k) for k, n in v.items())
ds = sum(n for k, n in c.items() if k.startswith("ds_"))
sa = sum(n for k, n in c.items() if k.startswith("s_"))
for k, n in sorted(v.items(), key=lambda x: -x[1]):
    print(f"{n:4d} {k}  ({cost(k)} cyc)")
print(f"per iteration: VALU {sum(v.values())} instr, {cyc} issue cycles; LDS {ds}; SALU/branch {sa}")
print(f"per number ({per:g} per iteration): VALU {sum(v.values()) / per:.1f} instr, {cyc / per:.1f} cycles "
      f"per wave-step; LDS {ds / per:.2f}")
