"""CPU tests of the product library's boundary and host logic (no GPU needed).

- libnice_hip.so loads and exports every function include/nice_hip.h declares;
- host-side number theory (base ranges, cutoff, residue/LSD/stride tables, the
  MSD prefix filter that feeds the niceonly kernel) matches the oracle and the
  reference's golden vectors bit for bit;
- without a GPU, context creation fails loudly (no CPU fallback).
"""
import ctypes
import os
import random
import re

import pytest

import nice_amd as N
from nice_amd import _lib
from oracle import oracle as O

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_library_exports_header_symbols():
    with open(os.path.join(ROOT, "include", "nice_hip.h")) as f:
        hdr = f.read()
    declared = set(re.findall(r"^\s*(?:int|void|const char|uint32_t|uint64_t|double)\s*\*?\s*(nice_\w+)\(",
                              hdr, re.M))
    assert declared, "no declarations parsed"
    assert declared == set(_lib.EXPORTS)
    L = _lib.lib()
    for name in declared:
        assert hasattr(L, name), name


def test_constants():
    assert N.api._const("nice_gpu_batch_size") == 50_000_000      # client_process_gpu.rs:59
    assert N.api._const("nice_processing_chunk_size") == 1_000_000  # :54
    assert all(N.gpu_supports_base(b) for b in range(2, 129))
    assert not N.gpu_supports_base(129)


def test_base_ranges_match_oracle(golden):
    for b in range(2, 129):
        try:
            want = O.base_range(b)
        except OverflowError:
            with pytest.raises(OverflowError):
                N.get_base_range_u128(b)
            continue
        got = N.get_base_range_u128(b)
        assert (None if got is None else (got.range_start, got.range_end)) == want, b
    for c in golden["reference"]["base_range"]["cases"]:
        if c["range"] and c["range"][1] < (1 << 128):
            r = N.get_base_range_u128(c["base"])
            assert (r.range_start, r.range_end) == tuple(c["range"])


def test_cutoff_matches_oracle():
    for b in range(2, 129):
        assert N.get_near_miss_cutoff(b) == O.near_miss_cutoff(b)


@pytest.mark.parametrize("base,k", [(10, 1), (10, 2), (12, 2), (25, 2), (40, 2), (45, 2),
                                    (50, 2), (62, 2), (80, 2), (97, 2)])
def test_stride_table_matches_oracle(base, k):
    t = N.StrideTable.new(base, k)
    M, res = O.stride_residues(base, k)
    assert t.modulus == M and t.valid_residues == res


def test_msd_skippable_matches_oracle(golden):
    rng = random.Random(1234)
    for b in (10, 12, 20, 25, 40, 45, 50, 57, 62, 70, 80, 94, 97):
        s, e = O.base_range(b)
        for _ in range(60):
            a = s + rng.randrange(e - s)
            size = 1 + rng.randrange(max(1, min(e - a, 10 ** rng.randrange(1, 12))))
            assert N.has_duplicate_msd_prefix(N.FieldSize(a, a + size), b) == \
                O.has_duplicate_msd_prefix(a, a + size, b), (b, a, size)
    for c in golden["reference"]["msd"]["early_exit"]:
        assert N.has_duplicate_msd_prefix(N.FieldSize(*c["range"]), c["base"]) == c["skip"]


def test_valid_ranges_match_oracle():
    rng = random.Random(99)
    for b in (10, 40, 45, 50, 62, 80):
        s, e = O.base_range(b)
        for _ in range(6):
            a = s + rng.randrange(max(1, e - s - 10 ** 7))
            size = min(e - a, rng.choice([10 ** 4, 10 ** 5, 10 ** 6, 10 ** 7]))
            got = [(r.range_start, r.range_end) for r in N.get_valid_ranges(N.FieldSize(a, a + size), b)]
            assert got == O.valid_ranges(a, a + size, b), (b, a, size)
    s, _ = O.base_range(40)
    got = N.get_valid_ranges(N.FieldSize(s, s + 10 ** 8), 40, floor_size=4000)
    assert [(r.range_start, r.range_end) for r in got] == O.valid_ranges(s, s + 10 ** 8, 40, 4000)


def test_benchmark_fields():
    f = N.get_benchmark_field(N.BenchmarkMode.EXTRA_LARGE)
    assert (f.base, f.range_start, f.range_size) == (40, 1_916_284_264_916, 10 ** 9)
    f = N.get_benchmark_field(N.BenchmarkMode.BASE_TEN)
    assert (f.base, f.range_start, f.range_end) == (10, 47, 100)
    f = N.get_benchmark_field(N.BenchmarkMode.HI_BASE)
    assert f.base == 80 and f.range_size == 10 ** 9  # benchmark.rs:63 (doc says 1e6)
    f = N.get_benchmark_field(N.BenchmarkMode.MASSIVE)
    assert f.base == 50 and f.range_size == 10 ** 13


def test_field_size_semantics():
    with pytest.raises(ValueError):
        N.FieldSize(5, 5)
    f = N.FieldSize(100, 105)
    assert (f.first(), f.last(), f.size()) == (100, 104, 5)
    assert [(c.start(), c.end()) for c in f.chunks(2)] == [(100, 102), (102, 104), (104, 105)]


def test_no_gpu_fails_loudly():
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    with pytest.raises(N.NiceError):
        N.GpuContext(0)


# --- host-evaluated fast paths of the device kernels (no GPU needed) --------

def _fd2_cuts_py(base):
    """n where a segment ending at e needs more radix-b^2 limbs for D1 = 2e+1,
    E1 = 3e^2+3e+1 or E2 = 6e+6 (fd2_detailed.hip), by exact integer search."""
    B = base * base

    def limbs(x):
        k = 0
        while x >= B ** k:
            k += 1
        return k

    def combo(e):
        return (limbs(2 * e + 1), limbs(3 * e * e + 3 * e + 1), limbs(6 * e + 6))

    s, e = O.base_range(base)
    cuts, a = [], s
    while combo(a + 1) != combo(e):
        lo, hi, cur = a + 1, e, combo(a + 1)
        while lo < hi:
            mid = (lo + hi) // 2
            if combo(mid) == cur:
                lo = mid + 1
            else:
                hi = mid
        cuts.append(lo - 1)
        a = lo - 1
    return cuts


@pytest.mark.parametrize("base", [40, 50, 80])
def test_fd_segment_cuts_match_python(base):
    L = _lib.lib()
    buf = (ctypes.c_uint64 * 16)()
    n = ctypes.c_size_t()
    assert L.nice_fd_segment_cuts(base, buf, 8, ctypes.byref(n)) == 0
    got = [buf[2 * i] | (buf[2 * i + 1] << 64) for i in range(n.value)]
    assert got == _fd2_cuts_py(base) and len(got) == 2
    assert L.nice_fd_segment_cuts(10, buf, 8, ctypes.byref(n)) == 0 and n.value == 0


def _split(x):
    return x & ((1 << 64) - 1), x >> 64


@pytest.mark.parametrize("base", [40, 50, 52, 53, 54, 80])
def test_is_nice_fast_path_matches_oracle(base):
    """radix_fast.hpp's is_nice_fast (the niceonly kernel's in-range check)
    against the oracle's get_is_nice on random in-range n, plus near-nice n
    (the ones that reach the cube scan)."""
    L = _lib.lib()
    rng = random.Random(base)
    s, e = O.base_range(base)
    ns = [s, e - 1] + [rng.randrange(s, e) for _ in range(3000)]
    deep = [n for n in (rng.randrange(s, e) for _ in range(40000)) if O.scan_depth(n, base) > base // 3]
    for n in ns + deep[:500]:
        assert L.nice_check_is_nice_inrange(base, *_split(n)) == int(O.is_nice(n, base)), n
    assert L.nice_check_is_nice_inrange(base, *_split(s - 1)) == _lib.NICE_ERR_INVALID


@pytest.mark.parametrize("base", [40, 50, 52, 53, 54, 80])
def test_unique_fast_path_matches_oracle(base):
    """The digit bits behind is_nice_fast's popcount test: radix_fast.hpp's
    limb path counts the unique digits of n^2 and n^3 exactly as the oracle's
    get_num_unique_digits, at both range ends and on random in-range n."""
    L = _lib.lib()
    rng = random.Random(7 * base)
    s, e = O.base_range(base)
    for n in [s, s + 1, e - 2, e - 1] + [rng.randrange(s, e) for _ in range(2000)]:
        assert L.nice_check_unique_inrange(base, *_split(n)) == O.num_unique_digits(n, base), n
    assert L.nice_check_unique_inrange(base, *_split(e)) == _lib.NICE_ERR_INVALID


@pytest.mark.parametrize("base", [40, 50, 52, 53, 54, 80])
def test_msd_fast_path_matches_oracle(base):
    """radix_fast.hpp's msd_skippable_fast (the device MSD filter's in-range
    check) against the oracle's has_duplicate_msd_prefix, on random ranges of
    every scale, including Filter C ranges (first / b^2 == last / b^2)."""
    L = _lib.lib()
    rng = random.Random(1000 + base)
    s, e = O.base_range(base)
    B = base * base
    cases = []
    for _ in range(1500):
        size = 10 ** rng.uniform(0, 9)
        a = rng.randrange(s, e - int(size) - 1)
        cases.append((a, a + max(1, int(size))))
    for _ in range(1500):  # inside one b^2 block: Filter C applies
        blk = rng.randrange(s // B + 1, e // B - 1) * B
        a = blk + rng.randrange(B - 2)
        cases.append((a, rng.randrange(a + 1, blk + B + 1)))
    hits = 0
    for a, b in cases:
        want = int(O.has_duplicate_msd_prefix(a, b, base))
        hits += want
        assert L.nice_check_msd_skippable_inrange(base, *_split(a), *_split(b)) == want, (a, b)
    assert 0 < hits < len(cases)


def _validate(base, size, hist, lst):
    arr = (_lib.nice_number * max(len(lst), 1))()
    for i, (n, u) in enumerate(lst):
        arr[i].number_lo, arr[i].number_hi, arr[i].num_uniques = n & ((1 << 64) - 1), n >> 64, u
    h = (ctypes.c_uint64 * (base + 1))(*hist)
    return _lib.lib().nice_validate_detailed(base, size & ((1 << 64) - 1), size >> 64, h, arr,
                                             len(lst))


def test_self_check_rejects_corrupted_results():
    """nice_validate_detailed = the server's submit checks (api/src/main.rs:
    309-359), applied by nice_process_range_detailed to its own output: a
    correct oracle result passes, every kind of corruption fails."""
    s, e = 10 ** 6, 10 ** 6 + 10 ** 4
    r = O.process_range_detailed(s, e, 10)
    hist = [0] + [c for _, c in r.distribution]
    lst = list(r.nice_numbers)
    assert len(lst) == 5395
    assert _validate(10, e - s, hist, lst) == _lib.NICE_OK
    bad = hist[:]
    bad[5] += 1  # mass no longer equals the field size
    assert _validate(10, e - s, bad, lst) == _lib.NICE_ERR_INVALID
    assert b"field size" in _lib.lib().nice_last_error()
    bad = hist[:]
    bad[10] -= 1
    bad[9] += 1  # same mass, near-miss bin disagrees with the list
    assert _validate(10, e - s, bad, lst) == _lib.NICE_ERR_INVALID
    assert _validate(10, e - s, hist, lst[:-1]) == _lib.NICE_ERR_INVALID  # dropped entry
    assert _validate(10, e - s, hist, lst + [lst[0]]) == _lib.NICE_ERR_INVALID  # duplicate
    assert _validate(10, e - s, hist, lst[:-1] + [(lst[-1][0], 9)]) == _lib.NICE_ERR_INVALID
    s40 = O.base_range(40)[0]
    r = O.process_range_detailed(s40, s40 + 10 ** 4, 40)
    assert _validate(40, 10 ** 4, [0] + [c for _, c in r.distribution], []) == _lib.NICE_OK


def test_product_library_has_no_probe_kernels():
    """The wrong-by-design bottleneck probes, the first-generation FD kernel and
    the environment tuning knobs exist only in the probe build (-DNICE_PROBES,
    `make -C nice_amd probe`); the shipped library contains none of them."""
    import subprocess
    syms = subprocess.run(["nm", "-C", _lib.LIB_PATH], capture_output=True, text=True,
                          check=True).stdout
    cfgs = [[int(x) for x in m.split(", ")]
            for m in re.findall(r"fd2_kernel<nice::fd2::Cfg<(-?\d+(?:, -?\d+)*)>", syms)]
    assert cfgs, "no fd2 kernels found"
    # Cfg<BASE, ND, NE, NE2, PROBE, WG, VD, LG, PERS, SIB>
    assert all(len(c) == 10 for c in cfgs), cfgs[:3]
    assert all(c[4] == 0 for c in cfgs), "probe instantiation in the product library"
    # neither the split b64 + u16 table layout (VD & 512) nor a forced lookup
    # grouping (the per-base default is -1) is a product variant; PERS is the
    # per-base default (-1) or the rounds fallback of a persistent kernel (0).
    # The sibling-lane kernels name their walk explicitly: three lanes on
    # b40..45 with LG 1 (per-sibling lookup groups) or 100 (the software-
    # pipelined walk), two lanes on b47..55 (short low-digit table) with LG 1
    for c in cfgs:
        assert c[6] & 512 == 0 and c[8] in (-1, 0), c
        assert c[7] == -1 if c[9] <= 1 else ((40 <= c[0] <= 45 and c[9] == 3 and c[7] in (1, 100))
                                             or (47 <= c[0] <= 55 and c[9] == 2 and c[7] == 1)), c
    assert any(c[9] == 3 for c in cfgs), "no three-lane sibling kernel"
    assert any(c[9] == 2 for c in cfgs), "no two-lane sibling kernel"
    assert "detailed_fd_kernel" not in syms
    with open(_lib.LIB_PATH, "rb") as f:
        blob = f.read()
    for knob in (b"NICE_FD2_PROBE", b"NICE_MSD_PROBE", b"NICE_FD_VARIANT", b"NICE_FD2_TCHUNK",
                 b"NICE_FD2_MINCHUNK", b"NICE_FD2_WG512", b"NICE_MSD_TRACE", b"NICE_FD2_LG",
                 b"NICE_FD2_COPIES", b"NICE_FD2_VD", b"NICE_FD2_PERS", b"NICE_FD2_SIB", b"NICE_FD2_SIBROUNDS",
                 b"NICE_FD2_NOMODEL"):
        assert knob not in blob, knob


FD_BASES = [40, 42, 43, 44, 45, 47, 48, 49, 50, 52, 53, 54, 55, 57, 58, 59, 60, 62, 63, 64, 65,
            67, 68, 80]


def test_fd_bases_and_limb_count_cuts():
    """Every base 40..68 with a valid range (and 80) has an FD kernel; the
    host's limb-count cuts (bignum walk, fd2_detailed.hip) equal a Python
    restatement: the n where the radix-b^2 limb counts of 2e+1, 3e^2+3e+1 and
    6e+6 at a segment end e change."""
    L = _lib.lib()
    assert [b for b in range(2, 129) if L.nice_fd_kernel_base(b)] == FD_BASES
    for base in FD_BASES:
        B = base * base

        def limbs(x):
            k = 0
            while x >= B ** k:
                k += 1
            return k

        def combo(e):
            return (limbs(2 * e + 1), limbs(3 * e * e + 3 * e + 1), limbs(6 * e + 6))
        s, e = O.base_range(base)
        want, a = [], s
        while combo(a + 1) != combo(e):
            lo, hi, cur = a + 1, e, combo(a + 1)
            while lo < hi:
                mid = (lo + hi) // 2
                lo, hi = (mid + 1, hi) if combo(mid) == cur else (lo, mid)
            want.append(lo - 1)
            a = lo - 1
        buf = (ctypes.c_uint64 * 16)()
        n = ctypes.c_size_t()
        assert L.nice_fd_segment_cuts(base, buf, 8, n) == 0
        assert [buf[2 * i] | (buf[2 * i + 1] << 64) for i in range(n.value)] == want, base


def _af_step_ref(floor, msd, total):
    """AdaptiveFloor::update's step, restated from client_process_gpu.rs:130-157."""
    gpu_tail = max(total - msd, 0.0)
    if gpu_tail < 0.002:
        ratio = 1.5
    elif msd < 0.002:
        ratio = 1.0 / 1.5
    else:
        ratio = msd / gpu_tail
    factor = min(max(ratio, 1.0 / 1.5), 1.5)
    return min(max(floor * factor, 250.0), 256_000.0)


def test_adaptive_floor_step_matches_reference_rule():
    cases = [(32_000, 0.5, 1.0), (32_000, 0.9, 1.0), (32_000, 0.1, 1.0), (300, 0.001, 0.5),
             (250, 0.0, 0.0), (200_000, 2.0, 2.001), (256_000, 3.0, 4.0), (1000, 0.004, 0.010),
             (1000, 0.0019, 0.010), (1000, 0.5, 0.5019), (12_345.6, 0.25, 0.75)]
    rng = random.Random(7)
    for _ in range(200):
        m = rng.uniform(0, 2)
        cases.append((rng.uniform(100, 300_000), m, m + rng.choice([0.0, 0.001, rng.uniform(0, 3)])))
    for f, m, t in cases:
        assert N.adaptive_floor_step(f, m, t) == pytest.approx(_af_step_ref(f, m, t), rel=1e-12), (f, m, t)


def test_adaptive_floor_seed_and_pin():
    """The process-wide floor (client_process_gpu.rs:160-184): seeded at
    512 000 / logical cores clamped to [250, 256 000] with 3 warmup fields,
    or pinned by NICE_GPU_MSD_FLOOR (no adaptation).  Fresh processes: the
    state is per process, as the reference's OnceLock."""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    code = ("import sys, os; sys.path.insert(0, %r); import nice_amd as N; f, w = N.adaptive_floor(); "
            "print(f, w, len(os.sched_getaffinity(0)))" % root)

    def run(env_val):
        env = dict(os.environ)
        env.pop("NICE_GPU_MSD_FLOOR", None)
        if env_val is not None:
            env["NICE_GPU_MSD_FLOOR"] = env_val
        out = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True,
                             timeout=120, check=True)
        f, w, cpus = out.stdout.split()
        return float(f), int(w), int(cpus)

    f, w, cpus = run(None)
    assert w == 3
    assert 250 <= f <= 256_000 and f >= min(256_000.0, 512_000.0 / cpus)  # cgroup quota can only lower cores
    assert run("64000")[:2] == (64000.0, 0xFFFFFFFF)
    assert run("bogus")[1] == 3


# --- a plain C host of the boundary (examples/nice_field.c) -------------------
def build_c_example():
    """gcc -std=c99 -pedantic -Werror against include/nice_hip.h alone, linked
    to libnice_hip.so: the header is self-contained C and the symbols resolve."""
    import subprocess
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "examples")], check=True)
    return os.path.join(ROOT, "examples", "nice_field")


def run_c_example(*args):
    import subprocess
    r = subprocess.run([build_c_example(), *map(str, args)], capture_output=True, text=True, timeout=300)
    dist, nice = [], []
    for line in r.stdout.splitlines():
        w = line.split()
        if w[0] == "dist":
            dist.append((int(w[1]), int(w[2])))
        elif w[0] == "nice":
            nice.append((int(w[1]), int(w[2])))
    return r.returncode, dist, nice, r.stderr


def test_c_host_example_cpu_mode(golden):
    """The reference's golden vectors through a C host calling the CPU API
    (the client without --gpu): b10 whole range, b40 / b80 first 1e4."""
    for c in golden["reference"]["detailed"]:
        size = [c["size"]] if c["size"] else []
        rc, dist, nice, err = run_c_example("detailed", c["base"], "range", *size)
        assert rc == 0, err
        assert dist == [tuple(x) for x in c["distribution"]], c["source"]
        assert nice == [tuple(x) for x in c["nice_numbers"]], c["source"]
    rc, _, nice, err = run_c_example("niceonly", 10, "range")
    assert rc == 0 and nice == [(69, 10)], err
    rc, _, nice, _ = run_c_example("detailed", 10, 47, 100)
    assert (69, 10) in nice
    # --gpu never falls back to the CPU: without a device it is an error
    n = ctypes.c_int(-1)
    if _lib.lib().nice_device_count(ctypes.byref(n)) != 0 or n.value == 0:
        rc, dist, nice, err = run_c_example("--gpu", "detailed", 10, "range")
        assert rc == 4 and not dist and "device" in err


def test_host_threads_follow_the_affinity_mask():
    """nice_host_threads (the host MSD pool's size at threads = 0) is
    std::thread::available_parallelism(): under `taskset -c 0-1` it is 2
    (client_process_gpu.rs:598), whatever the host's core count."""
    import shutil
    import subprocess
    import sys
    if not shutil.which("taskset"):
        pytest.skip("taskset not available")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    code = "import nice_amd; print(nice_amd.api.host_threads())"
    out = subprocess.run(["taskset", "-c", "0-1", sys.executable, "-c", code], cwd=root,
                         capture_output=True, text=True, check=True).stdout
    assert int(out.strip()) == 2
    out = subprocess.run(["taskset", "-c", "0", sys.executable, "-c", code], cwd=root,
                         capture_output=True, text=True, check=True).stdout
    assert int(out.strip()) == 1


def test_cgroup_quota_rounds_down_like_rust(tmp_path):
    """The cgroup cap of nice_host_threads follows Rust's std
    (available_parallelism -> cgroups::quota_v2): quota / period rounded
    DOWN, at least 1, the tightest of the process's cgroup and its
    ancestors; "max" does not limit."""
    L = _lib.lib()

    def put(rel, text):
        d = tmp_path / rel
        d.mkdir(parents=True, exist_ok=True)
        (d / "cpu.max").write_text(text + "\n")

    root = str(tmp_path).encode()
    put("", "max 100000")
    assert L.nice_debug_cgroup_cpus(root, b"") == 0
    put("a", "150000 100000")          # 1.5 CPUs -> 1 (a ceiling would say 2)
    assert L.nice_debug_cgroup_cpus(root, b"/a") == 1
    put("a", "50000 100000")           # 0.5 CPU -> at least 1
    assert L.nice_debug_cgroup_cpus(root, b"/a") == 1
    put("b", "1600000 100000")
    put("b/c", "max 100000")
    assert L.nice_debug_cgroup_cpus(root, b"/b/c") == 16   # the parent's quota
    put("b/c", "390000 100000")
    assert L.nice_debug_cgroup_cpus(root, b"/b/c/") == 3   # the child's, tighter
    assert L.nice_debug_cgroup_cpus(root, b"/nonexistent") == 0


def test_bad_submit_arguments_fail_at_once():
    """A submit with a bad argument answers NICE_ERR_INVALID immediately (no
    context needed to see it); NICE_ERR_BUSY is its own status."""
    L = _lib.lib()
    t = ctypes.c_int()
    assert L.nice_detailed_submit(None, 5, 0, 10, 0, 40, ctypes.byref(t)) == _lib.NICE_ERR_INVALID
    assert L.nice_niceonly_submit(None, 5, 0, 10, 0, 40, None, ctypes.byref(t)) == _lib.NICE_ERR_INVALID
    assert _lib.NICE_ERR_BUSY not in (_lib.NICE_OK, _lib.NICE_ERR_INVALID, _lib.NICE_ERR_HIP,
                                      _lib.NICE_ERR_CAPACITY, _lib.NICE_ERR_NO_DEVICE,
                                      _lib.NICE_ERR_MSD_OVERFLOW)
