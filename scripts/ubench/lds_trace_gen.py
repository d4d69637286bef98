"""Index traces of the FD kernel's data-random LDS lookups, for
scripts/ubench/lds_trace.hip (a bank swizzle of the
16-byte pair table, measured on the kernel's real index pattern).

Per wave w (WAVES of them), a random n0 inside the base's valid range and a
random step i of the chunk; lane k holds n = n0 + k * chunk + i (the
production lane layout: a wave's lanes sit `chunk` numbers apart).  For every
looked-up limb (S = n^2 limbs 1..S_HI, C = n^3 limbs 1..C_HI, radix b^2) the
limb value is the table index.  For each layout the file holds the stored
POSITION of that index (layouts permute entries within 16-entry blocks), as
u16 [layout][wave][limb][lane], so the kernel measures what the layout costs.
The model column is what a bank-quad count predicts: per 16-lane group of a
ds_read_b128, the largest number of DISTINCT entries sharing a bank quad
(position mod 16), averaged over lookups.

    python3 scripts/ubench/lds_trace_gen.py 80 245 8 16 gpurun_out/trace80.bin
"""
import os
import random
import struct
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from nice_amd.api import get_base_range_u128  # noqa: E402  (host helper, no device)

WAVES = 4096


def h(x, bits):
    return (x * 0x9E3779B1 & 0xffffffff) >> (32 - bits)


# Entry e's stored position: the identity, or e with its low 4 / 5 bits XORed
# by a hash of the bits above them (a permutation within aligned blocks of
# 16 / 32 entries: 16-byte entries put a block on the 64 banks once, 8-byte
# entries twice).
LAYOUTS = {
    "identity": lambda e: e,
    "xor4_hi": lambda e: e ^ ((e >> 4) & 15),
    "xor4_hash": lambda e: e ^ h(e >> 4, 4),
    "xor5_hash": lambda e: e ^ h(e >> 5, 5),
}


def main():
    base, chunk, s_hi, c_hi, path = (int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3]),
                                     int(sys.argv[4]), sys.argv[5])
    B = base * base
    r = get_base_range_u128(base)
    rng = random.Random(base * 1000 + chunk)
    idx = []  # [wave][limb][lane]
    for _ in range(WAVES):
        n0 = r.range_start + rng.randrange(r.range_end - r.range_start - 64 * chunk - 1)
        i = rng.randrange(chunk)
        ns = [n0 + lane * chunk + i for lane in range(64)]
        S = [n * n for n in ns]
        C = [s * n for s, n in zip(S, ns)]
        rows = [[(v // B ** q) % B for v in S] for q in range(1, s_hi + 1)]
        rows += [[(v // B ** q) % B for v in C] for q in range(1, c_hi + 1)]
        idx.append(rows)
    nl = s_hi + c_hi
    with open(path, "wb") as f:
        f.write(struct.pack("<6I", len(LAYOUTS), WAVES, nl, B, base, chunk))
        for name, fn in LAYOUTS.items():
            f.write(name.encode().ljust(16, b"\0"))
            model = 0.0
            for rows in idx:
                for row in rows:
                    pos = [fn(e) for e in row]
                    f.write(struct.pack(f"<{len(pos)}H", *pos))
                    for g in range(4):
                        load = {}
                        for p in set(pos[16 * g:16 * g + 16]):
                            load[p % 16] = load.get(p % 16, 0) + 1
                        model += max(load.values())
            print(f"{name:12s} model max-quad-load per 16-lane group: "
                  f"{model / (WAVES * nl * 4):.3f}", flush=True)


if __name__ == "__main__":
    main()
