"""nice_amd -- MI355X (gfx950) field processing for wasabipesto/nice.

The hot path (detailed + niceonly field processing) runs in libnice_hip.so:
hand-written HIP kernels for CDNA4 behind a C ABI (include/nice_hip.h).  This
package is the host-side mirror of the reference's API for that path.
"""
from ._lib import NiceError, NiceLibraryError, build, lib  # noqa: F401
from .api import (CLIENT_VERSION, GPU_BATCH_SIZE, PROCESSING_CHUNK_SIZE, BothModes,  # noqa: F401
                  GpuContext, adaptive_floor, adaptive_floor_step, StrideTable, default_context, get_base_range_u128, get_near_miss_cutoff,
                  get_valid_ranges, gpu_supports_base, has_duplicate_msd_prefix,
                  process_detailed_gpu, process_niceonly_gpu, process_range_detailed,
                  process_range_detailed_gpu, process_range_niceonly,
                  process_range_niceonly_gpu, process_range_detailed_cpu,
                  process_range_niceonly_cpu)
from .benchmark import BenchmarkMode, get_benchmark_field  # noqa: F401
from .types import (DataToClient, DataToServer, FieldResults, FieldSize,  # noqa: F401
                    NiceNumberSimple, SearchMode, UniquesDistributionSimple)
