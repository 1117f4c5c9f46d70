"""mini_parallel_amd -- MI355X-native batched Smith-Waterman short-read scorer.

Drop-in for the batched DP scoring path of bmwoolf/mini_parallel's
`smith_waterman` crate (package `rustseq_mini`).  The product is the C ABI
library ``libmsw.so`` (include/msw.h): hand-written gfx950 HIP kernels plus a
C++ runtime.  This package is the thin host mirror of the reference API.
"""
from ._lib import MswError, LIB_PATH  # noqa: F401
from .aligner import (AFFINE, GPU_MAX_WORK_GROUPS, GPU_WORK_GROUP_SIZE, LINEAR, LINEAR_COORDS,  # noqa: F401
                      Context, Genome, GpuAlignmentResult, GpuDevice, Pending, Scoring,
                      get_chunk_size_reads, get_context, get_gpu_devices, gpu_align,
                      gpu_align_chunk_self, is_gpu_available, pack_batch, pinned_empty)

__version__ = "0.1.0"
