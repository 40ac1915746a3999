"""proovread_amd — MI355X-native implementation of proovread's hot path.

The compute lives in libprgpu.so (HIP kernels for gfx950 behind the C-ABI in
include/prgpu.h).  This package is the host-side mirror of the reference
interfaces for that path (bam2cns / Sam::Seq for the consensus stage, the
seed-extension stage of bwa-proovread mem).
"""
from . import _abi  # noqa: F401

__all__ = ["_abi", "cns"]
