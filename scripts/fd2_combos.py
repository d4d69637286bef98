"""Limb-count combos of the production FD kernel (fd2_detailed.hip) per base:
for each base with a valid range, the (ND, NE, NE2) = radix-b^2 limb counts of
D1 = 2e+1, E1 = 3e^2+3e+1, E2 = 6e+6 at a segment end e, for every distinct
value over the range (the host splits launches where they change;
fd2::thresholds does the same walk with bignums at run time).  Prints the
FD2_COMBOS X-macro entries and the per-base layout facts.

    python scripts/fd2_combos.py [bases...]     (default: 40..80 with a range)
"""
import sys


def base_range(b):
    """get_base_range_u128 (base_range.rs:43-54) through the product library's
    host helper (no device needed)."""
    sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(
        __import__("os").path.abspath(__file__))))
    import nice_amd as N
    try:
        r = N.get_base_range_u128(b)
    except OverflowError:
        return None
    return (r.range_start, r.range_end) if r else None


def limbs(x, B):
    k = 0
    while x >= B ** k:
        k += 1
    return k


def combo(e, B):
    return (limbs(2 * e + 1, B), limbs(3 * e * e + 3 * e + 1, B), limbs(6 * e + 6, B))


def combos(b):
    r = base_range(b)
    if r is None:
        return []
    s, e = r
    B = b * b
    out = [combo(s + 1, B)]
    a = s
    while combo(a + 1, B) != combo(e, B):
        lo, hi, cur = a + 1, e, combo(a + 1, B)
        while lo < hi:
            mid = (lo + hi) // 2
            if combo(mid, B) == cur:
                lo = mid + 1
            else:
                hi = mid
        a = lo - 1
        out.append(combo(lo, B))
    return out


if __name__ == "__main__":
    bases = [int(x) for x in sys.argv[1:]] or [b for b in range(40, 81) if base_range(b)]
    items = []
    for b in bases:
        for c in combos(b):
            items.append(f"X({b}, {c[0]}, {c[1]}, {c[2]})")
        print(b, base_range(b), combos(b), file=sys.stderr)
    print(" ".join(items))
