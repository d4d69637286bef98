"""A/B of two builds of the library in one GPU session: the package under
ab_old/ (a copy of nice_amd with its .so, made on the CPU host) against the
tree's own, alternating child processes; median detailed kernel ms per 1e9
field for each base given (default 40 50 80)."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = r'''
import sys, statistics
sys.path.insert(0, %r)
import nice_amd as N
for base in %r:
    ctx = N.GpuContext(0); s = N.get_base_range_u128(base).range_start
    h, l = ctx.detailed_raw(s, s + 10**9, base)
    ks = []
    for _ in range(5):
        h2, l2 = ctx.detailed_raw(s, s + 10**9, base); ks.append(ctx.kernel_stats().kernel_ms)
        assert h2 == h and l2 == l
    print(base, statistics.median(ks), sum(i * c for i, c in enumerate(h)), flush=True)
'''
bases = [int(x) for x in sys.argv[1:]] or [40, 50, 80]
for rnd in range(3):
    for name, path in (("old", os.path.join(ROOT, "ab_old")), ("new", ROOT)):
        out = subprocess.run([sys.executable, "-c", CHILD % (path, bases)], capture_output=True, text=True,
                             timeout=300)
        if out.returncode:
            print(out.stderr[-3000:])
            sys.exit(1)
        for ln in out.stdout.split("\n"):
            if ln:
                b, ms, chk = ln.split()
                print(f"round {rnd} {name} b{b}: {float(ms):.4f} ms  checksum {chk}", flush=True)
