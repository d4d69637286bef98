"""VALU / LDS issue budget of a kernel's hot loop, from a hipcc --save-temps
.s file: the instructions of the listed basic blocks (the loop's common path,
rare blocks left out), each VALU opcode priced at its measured gfx950 issue
cost per wave64 instruction on one SIMD (profiles/r01/isa_issue_rates_gfx950.log:
2 cycles for the full-rate forms, 4 for the half-rate ones -- the table's
2.3-2.9 and 4.2-4.7 at its nominal 2.4 GHz; unmeasured v_cmp / v_cndmask /
v_mov forms taken as full rate, any other unmeasured opcode as half rate).

    python scripts/isa/issue_budget.py FILE.s KERNEL_SYMBOL NUMBERS_PER_ITER LABEL...

Prints per number (a wave-step = 64 numbers): VALU instructions, VALU issue
cycles, LDS instructions, and the opcode histogram."""
import re
import sys
from collections import Counter

FULL = {"v_add_u32", "v_sub_u32", "v_subrev_u32", "v_or_b32", "v_and_b32", "v_xor_b32", "v_lshrrev_b32",
        "v_mov_b32", "v_add_f32", "v_fma_f32", "v_cndmask_b32", "v_readfirstlane_b32"}


def base_op(op):
    op = re.sub(r"_(e32|e64|sdwa|dpp)$", "", op)
    return op


def cost(op):
    b = base_op(op)
    if b in FULL or b.startswith("v_cmp"):
        return 2
    return 4


def main(path, kernel, per_iter, labels):
    text = open(path).read().splitlines()
    i = next(k for k, l in enumerate(text) if l.startswith(kernel + ":"))
    j = next(k for k in range(i + 1, len(text)) if text[k].startswith(".Lfunc_end"))
    blocks, cur = {}, None
    for ln in text[i:j]:
        m = re.match(r"^(\.LBB\d+_\d+|; %bb\.\d+):?", ln)
        if m:
            cur = m.group(1).replace("; %bb.", "bb")
            blocks[cur] = []
            continue
        s = ln.strip()
        if cur and s and not s.startswith(";") and not s.startswith("."):
            blocks[cur].append(s.split()[0])
    c = Counter()
    for lb in labels:
        c.update(blocks[lb.replace("%bb.", "bb")])
    v = {k: n for k, n in c.items() if k.startswith("v_")}
    cyc = sum(n * cost(k) for k, n in v.items())
    ds = sum(n for k, n in c.items() if k.startswith("ds_"))
    for k, n in sorted(c.items(), key=lambda x: -x[1]):
        print(f"{n:4d} {k}{'' if not k.startswith('v_') else f'  ({cost(k)} cyc)'}")
    nv = sum(v.values())
    print(f"per iteration ({per_iter} numbers per lane): VALU {nv} instr, {cyc} issue cycles; LDS {ds}")
    print(f"per number: VALU {nv / per_iter:.1f} instr, {cyc / per_iter:.1f} issue cycles per wave-step; "
          f"LDS {ds / per_iter:.2f} instr")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], float(sys.argv[3]), sys.argv[4:])
