"""Point nice_amd at the probe build of the library (libnice_hip_probe.so,
`make -C nice_amd probe`): the same sources compiled with -DNICE_PROBES, which
adds the bottleneck probes (NICE_FD2_PROBE, NICE_MSD_PROBE: kernels whose
results are wrong by design) and the launch tuning knobs (NICE_FD2_TCHUNK,
NICE_FD2_MINCHUNK, NICE_FD2_WG512, NICE_SLOTS, NICE_SHARED_STREAMS, ...).  The product library ignores all of
them.  Import this module before the first nice_amd call:

    import probe_lib  # noqa: F401  (scripts/ on sys.path)
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
from nice_amd import _lib  # noqa: E402

_lib.LIB_PATH = os.path.join(ROOT, "nice_amd", "libnice_hip_probe.so")
if not os.path.exists(_lib.LIB_PATH):
    raise SystemExit(f"{_lib.LIB_PATH} missing: build it with `make -C nice_amd probe`")
