#!/usr/bin/env python3
"""Extract the reference's own golden vectors (its inline Rust unit tests) into
tests/golden/reference_vectors.json.

Run in the build container only (it reads /root/reference, which does not exist
on the GPU box).  The output is data -- inputs and expected outputs that the
reference's tests assert -- with the citing file:line for each group.

    python tests/golden/extract_reference_vectors.py
"""
import json
import os
import re

REF = "/root/reference/common/src"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "reference_vectors.json")


def read(name):
    with open(os.path.join(REF, name)) as f:
        return f.read()


def fn_body(src, name):
    """Text of `fn name(...) { ... }` (brace matched) and its 1-based line."""
    m = re.search(r"fn %s\s*\(" % re.escape(name), src)
    assert m, name
    i = src.index("{", m.end())
    depth, j = 0, i
    while True:
        if src[j] == "{":
            depth += 1
        elif src[j] == "}":
            depth -= 1
            if depth == 0:
                break
        j += 1
    return src[m.start(): j + 1], src[: m.start()].count("\n") + 1


def detailed_case(src, name):
    body, line = fn_body(src, name)
    base = int(re.search(r"let base = (\d+);", body).group(1))
    size = re.search(r"let size = (\d+);", body)
    dist = [(int(a), int(b)) for a, b in re.findall(
        r"num_uniques:\s*(\d+),\s*count:\s*(\d+)", body)]
    nice = [(int(a), int(b)) for a, b in re.findall(
        r"number:\s*(\d+),\s*num_uniques:\s*(\d+)", body)]
    return {
        "source": f"common/src/client_process.rs:{line}",
        "base": base,
        "range": "base_range" if size is None else "base_range_start_plus_size",
        "size": None if size is None else int(size.group(1)),
        "distribution": dist,
        "nice_numbers": nice,
    }


def main():
    cp = read("client_process.rs")
    out = {"detailed": [detailed_case(cp, n) for n in
                        ("process_detailed_b10", "process_detailed_b40", "process_detailed_b80")]}

    nice = []
    for n in ("process_niceonly_b10", "process_niceonly_b40", "process_niceonly_b80"):
        c = detailed_case(cp, n)
        nice.append({"source": c["source"], "base": c["base"], "range": c["range"],
                     "size": c["size"], "k": 1, "nice_numbers": c["nice_numbers"]})
    out["niceonly"] = nice

    br = read("base_range.rs")
    body, line = fn_body(br, "test_get_base_range_natural")
    ranges = []
    for chunk in body.split("assert_eq!(")[1:]:
        m = re.match(r"\s*get_base_range_natural\((\d+)\)", chunk)
        if not m:
            continue
        base = int(m.group(1))
        if re.match(r"\s*get_base_range_natural\(\d+\),\s*None", chunk):
            ranges.append({"base": base, "range": None})
            continue
        nums = re.findall(r'Natural::from(?:_str)?\(\s*"?([\d_]+)"?', chunk)
        nums = [int(x.replace("_", "")) for x in nums]
        assert len(nums) == 2, (base, chunk)
        ranges.append({"base": base, "range": nums})
    out["base_range"] = {"source": f"common/src/base_range.rs:{line}", "cases": ranges}

    rf = read("residue_filter.rs")
    body, line = fn_body(rf, "test_get_residue_filter")
    res = []
    for m in re.finditer(r"get_residue_filter\(&(\d+)\),\s*(Vec::<u32>::new\(\)|Vec::from\(\[(.*?)\]\))",
                         body, re.S):
        vals = [] if m.group(3) is None else [int(x) for x in m.group(3).split(",") if x.strip()]
        res.append({"base": int(m.group(1)), "residues": vals})
    out["residue_filter"] = {"source": f"residue_filter.rs:{line}", "cases": res}

    # Hand-transcribed assertions (data, with citations).
    out["lsd"] = {
        "valid_lsds": [
            {"source": "common/src/lsd_filter.rs:244-247", "base": 10, "lsds": [2, 3, 4, 7, 8, 9]},
            {"source": "common/src/lsd_filter.rs:452-456", "base": 12, "lsds": [2, 3, 5, 7, 8, 11]},
            {"source": "common/src/lsd_filter.rs:482-486", "base": 16,
             "lsds": [2, 3, 5, 6, 7, 9, 10, 11, 13, 14, 15]},
        ],
        "bitmap_points": [
            {"source": "common/src/lsd_filter.rs:548-562", "base": 10, "k": 2,
             "points": {"0": False, "1": False, "12": True, "69": True}},
            {"source": "common/src/lsd_filter.rs:581-582", "base": 10, "k": 3,
             "points": {"69": True}},
        ],
    }
    out["stride"] = [
        {"source": "common/src/stride_filter.rs:162-176", "base": 10, "k": 1, "modulus": 90},
        {"source": "common/src/stride_filter.rs:178-193", "base": 40, "k": 2, "modulus": 62400},
    ]
    out["msd"] = {
        "early_exit": [
            {"source": "common/src/msd_prefix_filter.rs:857-872", "base": 10,
             "range": [3163, 3165], "skip": True},
            {"source": "common/src/msd_prefix_filter.rs:874-887", "base": 10,
             "range": [3163, 3164], "skip": False},
        ],
        "whole_range_no_skip": [
            {"source": "common/src/msd_prefix_filter.rs:901-907", "base": 10},
            {"source": "common/src/msd_prefix_filter.rs:909-915", "base": 40},
            {"source": "common/src/msd_prefix_filter.rs:917-923", "base": 50},
        ],
        "segments": [
            {"source": "common/src/msd_prefix_filter.rs:925-952", "base": 50, "divisor": 100,
             "expect": [[0, False], [10, False], [30, False], [40, False], [50, False],
                        [60, False], [70, False], [80, False], [90, False], [100, True]]},
            {"source": "common/src/msd_prefix_filter.rs:954-981", "base": 50, "divisor": 10000,
             "expect": [[0, False], [10, False], [30, True], [40, True], [50, False],
                        [60, False], [70, False], [80, True], [90, True], [100, False]]},
        ],
    }
    # Known answers quoted by the reference web page (web/index.html:29-30, 43-44).
    out["known_answers"] = [
        {"source": "web/index.html:43-44", "n": 69, "base": 10, "num_uniques": 10},
        {"source": "web/index.html:29-30", "n": 330169542960890, "base": 45, "num_uniques": 44},
    ]
    with open(OUT, "w") as f:
        json.dump(out, f, indent=1)
    print("wrote", OUT)


if __name__ == "__main__":
    main()
