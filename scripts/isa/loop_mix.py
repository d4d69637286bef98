"""Count the instruction mix of a kernel's hot loop in a hipcc --save-temps .s
file: every instruction of the blocks belonging to the innermost loop named by
its header label, excluding blocks listed as rare (by label).  Classes follow
the measured gfx950 issue costs (profiles/r01/isa_issue_rates_gfx950.log)."""
import re
import sys
from collections import Counter

FAST = {"v_add_u32", "v_sub_u32", "v_or_b32", "v_and_b32", "v_xor_b32", "v_lshrrev_b32",
        "v_mov_b32", "v_add_f32", "v_fma_f32", "v_subrev_u32"}


def blocks(lines):
    cur, out = None, {}
    for ln in lines:
        m = re.match(r"^(\.LBB\d+_\d+|; %bb\.\d+):?", ln)
        if m:
            cur = m.group(1).replace("; %bb.", "bb")
            out.setdefault(cur, [])
            continue
        s = ln.strip()
        if cur and s and not s.startswith(";") and not s.startswith("."):
            out[cur].append(s.split()[0])
    return out


def main(path, kernel, first, last, skip):
    text = open(path).read().splitlines()
    i = next(k for k, l in enumerate(text) if l.startswith(kernel + ":"))
    j = next(k for k in range(i + 1, len(text)) if text[k].startswith(".Lfunc_end"))
    bl = blocks(text[i:j])
    names = list(bl)
    a, b = names.index(first), names.index(last)
    c = Counter()
    for n in names[a:b + 1]:
        if n in skip:
            continue
        for op in bl[n]:
            c[op] += 1
    v = {k: n for k, n in c.items() if k.startswith("v_")}
    fast = sum(n for k, n in v.items() if k.split("_e32")[0].split("_e64")[0] in FAST)
    slow = sum(v.values()) - fast
    ds = sum(n for k, n in c.items() if k.startswith("ds_"))
    for k, n in sorted(c.items(), key=lambda x: -x[1]):
        print(f"{n:4d} {k}")
    print(f"VALU {sum(v.values())} (fast {fast}, slow {slow}), est cycles {fast * 2.5 + slow * 4.4:.0f}; LDS {ds}")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], sys.argv[3], sys.argv[4], set(sys.argv[5:]))
