#!/usr/bin/env python3
"""Generate golden vectors with the reference's own Python mirror,
scripts/inspect_number.py (compute_niceness, :180-221).

Run in the build container only: it imports the reference from /root/reference
(the reference never travels to the GPU box; only the JSON output does).

    python tests/golden/gen_python_vectors.py          # ~1 min on 8 cores

Ranges use the Rust base-range semantics (common/src/base_range.rs:14-32,
ceiling roots) built from inspect_number's exact root helpers, NOT
inspect_number.get_base_range, which floors the end for b % 5 in {2, 3, 4}
(SURVEY.md section 8c "Known oracle divergence").
"""
import importlib.util
import json
import math
import multiprocessing as mp
import os

REF_SCRIPT = "/root/reference/scripts/inspect_number.py"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "python_vectors.json")

_spec = importlib.util.spec_from_file_location("inspect_number", REF_SCRIPT)
IN = importlib.util.module_from_spec(_spec)
_spec.loader.exec_module(IN)

M128 = (1 << 128) - 1


def rust_base_range(b):
    """base_range.rs:14-32 with malachite ceiling_root semantics."""
    k = b // 5
    r = b % 5
    if r == 0:
        if k == 0:
            return None
        s, e = IN._ceil_cbrt(b ** (3 * k - 1)), b ** k
    elif r == 1:
        return None
    elif r == 2:
        s, e = b ** k, IN._ceil_cbrt(b ** (3 * k + 1))
    elif r == 3:
        s, e = IN._ceil_cbrt(b ** (3 * k + 1)), IN._ceil_sqrt(b ** (2 * k + 1))
    else:
        s, e = IN._ceil_sqrt(b ** (2 * k + 1)), IN._ceil_cbrt(b ** (3 * k + 2))
    return (s, e) if s < e else None


def nu(args):
    n, b = args
    return IN.compute_niceness(n, b)["num_uniques"]


def detailed(pool, start, end, base):
    """Histogram (bins 1..=base) + near-miss list, like process_range_detailed."""
    cutoff = math.floor(0.9 * base)  # inspect_number is_saved threshold (:219)
    us = pool.map(nu, [(n, base) for n in range(start, end)], chunksize=4096)
    hist = [0] * (base + 1)
    misses = []
    for n, u in zip(range(start, end), us):
        hist[u] += 1
        if u > cutoff:
            misses.append([n, u])
    return {"base": base, "start": str(start), "end": str(end),
            "distribution": [[i, hist[i]] for i in range(1, base + 1)],
            "near_misses": [[str(n), u] for n, u in misses]}


def lcg_samples(base, count, seed):
    """client_process_gpu.rs:1394-1400: x = x*6364136223846793005 + i (mod 2^128),
    n = range_start + x % span."""
    r = rust_base_range(base)
    s, e = r
    x = seed
    out = []
    for i in range(count):
        x = (x * 6364136223846793005 + i) & M128
        out.append(s + x % (e - s))
    return out


def main():
    with mp.Pool(8) as pool:
        cases = []
        s40, _ = rust_base_range(40)
        s80, _ = rust_base_range(80)
        s50, _ = rust_base_range(50)
        # SURVEY.md 8c golden vectors, plus extra bases.
        cases.append(dict(detailed(pool, s40, s40 + 1_000_000, 40), name="b40_default_1e6",
                          note="benchmark.rs:58 Default field"))
        cases.append(dict(detailed(pool, s80, s80 + 1_000_000, 80), name="b80_hibase_1e6",
                          note="BASELINE.json hi-base (1e6)"))
        cases.append(dict(detailed(pool, 2_000_000_000_000, 2_000_000_100_000, 40),
                          name="b40_2e12_1e5", note="client_process_gpu.rs:1486 GPU test"))
        cases.append(dict(detailed(pool, 1_000_000, 1_010_000, 10), name="b10_1e6_1e4",
                          note="client_process_gpu.rs:1485 GPU test (out-of-range n)"))
        cases.append(dict(detailed(pool, s50, s50 + 200_000, 50), name="b50_start_2e5",
                          note="massive/msd-effective base"))
        for b in (12, 25, 45, 57, 62, 68, 70, 94, 97):
            r = rust_base_range(b)
            if r is None:
                continue
            s, e = r
            cases.append(dict(detailed(pool, s, min(e, s + 20_000), b), name=f"b{b}_start_2e4",
                              note="extra base"))
        # Sampled n across each base's range (seed client_process_gpu.rs:1394).
        samples = []
        for b in (10, 12, 25, 40, 45, 50, 57, 62, 68, 70, 80, 94, 97):
            if rust_base_range(b) is None:
                continue
            ns = lcg_samples(b, 200, 0x9E3779B97F4A7C15F39CC0605CEDC834)
            us = pool.map(nu, [(n, b) for n in ns])
            samples.append({"base": b, "n": [str(n) for n in ns], "num_uniques": us})
        # Arbitrary n (out of range too) for a spread of bases: exact big-int semantics.
        wild = []
        x = 0xDEADBEEFCAFEF00D0D15EA5EFEEDFACE
        for i in range(400):
            x = (x * 6364136223846793005 + 1442695040888963407) & M128
            bits = 1 + (x >> 100) % 128
            n = (x & ((1 << bits) - 1)) | 1
            b = 2 + (x >> 64) % 127
            wild.append([str(n), b, nu((n, b))])
        ranges = {str(b): (None if rust_base_range(b) is None else
                           [str(v) for v in rust_base_range(b)])
                  for b in range(2, 98)}
    out = {"generator": "tests/golden/gen_python_vectors.py (reference scripts/inspect_number.py)",
           "detailed": cases, "samples": samples, "wild": wild, "base_ranges": ranges}
    with open(OUT, "w") as f:
        json.dump(out, f)
    print("wrote", OUT, os.path.getsize(OUT), "bytes")


if __name__ == "__main__":
    main()
