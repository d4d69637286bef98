"""Bank-slot model of the b80 FD kernel's ds_read_b128 lookups (S limbs 1-8, C limbs
1-12 and 16, radix 6400) for several lane->n layouts of a wave, at three points of
the range: per 16-lane group the most distinct entries on one slot (entry mod 16).
Companion of scripts/ubench/run_lds_stride.sh (the same layouts timed on the
hardware, profiles/r05/lds_stride_b80.log)."""
import sys, random
sys.path.insert(0, '/root/repo')
import nice_amd as N
B = 6400
r = N.get_base_range_u128(80)
GROUPS = [list(range(0,4))+list(range(12,16))+list(range(20,28)), list(range(4,12))+list(range(16,20))+list(range(28,32))]
GROUPS += [[x+32 for x in g] for g in GROUPS]
S_LOOK = list(range(1, 9)); C_LOOK = list(range(1, 13)) + [16]
def limbs(x, n):
    out = []
    for _ in range(n):
        out.append(x % B); x //= B
    return out
def cost(vals):
    t = 0
    for g in GROUPS:
        slots = {}
        for l in g:
            slots.setdefault(vals[l] % 16, set()).add(vals[l])
        t += max(len(s) for s in slots.values())
    return t
def wave(lanes):
    S = [limbs(n*n, 16) for n in lanes]; C = [limbs(n**3, 24) for n in lanes]
    tot = 0; per = {}
    for q in S_LOOK:
        c = cost([s[q] for s in S]); per[f'S{q}'] = c; tot += c
    for q in C_LOOK:
        c = cost([x[q] for x in C]); per[f'C{q}'] = c; tot += c
    return tot, per
rnd = random.Random(3)
for frac in (0.0, 0.3, 0.7):
    n0 = r.range_start + int((r.range_end - r.range_start) * frac)
    for name, f in (("stride240", lambda b, l: b + l * 240), ("stride241", lambda b, l: b + l * 241),
                    ("interleave", lambda b, l: b + l), ("stride3", lambda b, l: b + 3 * l)):
        tot = 0; pers = {}
        K = 24
        for k in range(K):
            b = n0 + rnd.randrange(10**9)
            t, per = wave([f(b, l) for l in range(64)])
            tot += t
            for kk, v in per.items(): pers[kk] = pers.get(kk, 0) + v
        print(f"f={frac} {name}: {tot/K/21:.2f} cycles per ds_read_b128 ({tot/K:.0f} per step) " + " ".join(f"{k}:{v/K:.1f}" for k, v in pers.items()), flush=True)
