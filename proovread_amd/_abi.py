"""ctypes declarations of include/prgpu.h (the C-ABI of libprgpu.so).

The product path always goes through libprgpu.so; if the library is missing
or no gfx950 device is visible, the calls fail loudly (RuntimeError) — there
is no CPU fallback.
"""
from __future__ import annotations

import ctypes as C
import os
from pathlib import Path

PKG = Path(__file__).resolve().parent
LIBPATH = Path(os.environ.get("PRGPU_LIB", PKG / "libprgpu.so"))

PR_ALN_HAS_SCORE = 1
PR_ALN_NO_QUAL = 2
PR_ALN_NO_SEQ = 4

ERRORS = {
    0: "PR_OK", -1: "PR_ERR_ARG", -2: "PR_ERR_HIP", -3: "PR_ERR_SAM", -4: "PR_ERR_NOSEQ",
    -5: "PR_ERR_BIN_RANGE", -6: "PR_ERR_DIV0", -7: "PR_ERR_CIGAR", -8: "PR_ERR_BEYOND_REF",
    -9: "PR_ERR_CAPACITY", -10: "PR_ERR_UNSUPPORTED",
}

P64 = C.POINTER(C.c_int64)
P32 = C.POINTER(C.c_int32)
PU8 = C.POINTER(C.c_uint8)
PU32 = C.POINTER(C.c_uint32)
PD = C.POINTER(C.c_double)


class CnsParams(C.Structure):
    _fields_ = [
        ("max_coverage", C.c_double), ("bin_size", C.c_double), ("trim", C.c_int32),
        ("indel_taboo_length", C.c_int32), ("indel_taboo", C.c_double), ("min_aln_length", C.c_int32),
        ("max_ins_length", C.c_int32), ("fallback_phred", C.c_int32), ("phred_offset", C.c_int32),
        ("ref_phred_offset", C.c_int32), ("use_ref_qual", C.c_int32), ("qual_weighted", C.c_int32),
        ("detect_chimera", C.c_int32), ("invert_scores", C.c_int32),
    ]


class CnsBatch(C.Structure):
    _fields_ = [
        ("n_lr", C.c_int32), ("lr_off", P64), ("ref_seq", PU8), ("ref_qual", PU8),
        ("ign_off", P64), ("ign", P32), ("aln_off", P64), ("aln_pos", P32), ("aln_score", PD),
        ("aln_flags", PU8), ("aln_seq_off", P64), ("aln_lseq", P32), ("aln_cig_off", P64),
        ("aln_ncig", P32), ("seq_pool", PU8), ("qual_pool", PU8), ("cig_pool", PU32),
        ("seq_pool_len", C.c_int64), ("cig_pool_len", C.c_int64),
    ]


class CnsBounds(C.Structure):
    _fields_ = [("seq_cap", C.c_int64), ("chim_cap", C.c_int64)]


class CnsOut(C.Structure):
    _fields_ = [
        ("out_off", P64), ("status", P32), ("seq_len", P32), ("trace_len", P32), ("ncigar", P32),
        ("nchim", P32), ("seq", PU8), ("qual", PU8), ("trace", PU8), ("cigar", PU32),
        ("chim_off", P64), ("chim", P32), ("kept", PU8), ("bin_bases", P64),
    ]


_lib = None


def lib():
    """Load libprgpu.so (built in-tree by __graft_entry__.build())."""
    global _lib
    if _lib is not None:
        return _lib
    if not LIBPATH.exists():
        raise RuntimeError(f"libprgpu.so not found at {LIBPATH}: run __graft_entry__.build() "
                           "(the HIP extension is required; there is no CPU fallback)")
    L = C.CDLL(str(LIBPATH))
    L.pr_last_error.restype = C.c_char_p
    L.pr_version.restype = C.c_char_p
    L.pr_ctx_create.argtypes = [C.c_int, C.POINTER(C.c_void_p)]
    L.pr_ctx_destroy.argtypes = [C.c_void_p]
    L.pr_device_count.argtypes = [C.POINTER(C.c_int)]
    L.pr_cns_params_default.argtypes = [C.POINTER(CnsParams)]
    L.pr_cns_bounds_of.argtypes = [C.POINTER(CnsBatch), C.POINTER(CnsBounds)]
    L.pr_cns_run.argtypes = [C.c_void_p, C.POINTER(CnsParams), C.POINTER(CnsBatch), C.POINTER(CnsOut)]
    L.pr_cns_upload.argtypes = [C.c_void_p, C.POINTER(CnsBatch)]
    L.pr_cns_launch.argtypes = [C.c_void_p, C.POINTER(CnsParams)]
    L.pr_cns_download.argtypes = [C.c_void_p, C.POINTER(CnsOut)]
    L.pr_cns_last_timing.argtypes = [C.c_void_p, PD, PD]
    L.pr_cns_phase_ticks.argtypes = [C.c_void_p, C.POINTER(C.c_uint64), C.c_int]
    L.pr_cns_resident_stats.argtypes = [C.c_void_p, P64, P64]
    _lib = L
    return L


def check(rc, what):
    if rc != 0:
        msg = lib().pr_last_error().decode(errors="replace")
        raise RuntimeError(f"{what} failed: {ERRORS.get(rc, rc)}: {msg}")


class Context:
    """One HIP device context (one process per GPU)."""

    def __init__(self, device: int = -1):
        L = lib()
        h = C.c_void_p()
        check(L.pr_ctx_create(device, C.byref(h)), "pr_ctx_create")
        self.h = h

    def close(self):
        if self.h:
            lib().pr_ctx_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class DevBuffer:
    """Device memory of a context (pr_dev_alloc): e.g. the int64[2] statistic pr_iter_stats /
    pr_iter_mask fill and an RCCL all-reduce sums across GPUs.  Zeroed at allocation."""

    def __init__(self, ctx: "Context", nbytes: int):
        L = lib()
        L.pr_dev_alloc.argtypes = [C.c_void_p, C.c_int64, C.POINTER(C.c_void_p)]
        L.pr_dev_free.argtypes = [C.c_void_p, C.c_void_p]
        L.pr_dev_download.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int64]
        L.pr_dev_upload.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int64]
        self.ctx, self.nbytes = ctx, nbytes
        p = C.c_void_p()
        check(L.pr_dev_alloc(ctx.h, nbytes, C.byref(p)), "pr_dev_alloc")
        self.ptr = p.value

    def download(self, dtype=None):
        import numpy as np
        a = np.zeros(self.nbytes, np.uint8)
        check(lib().pr_dev_download(self.ctx.h, a.ctypes.data, self.ptr, self.nbytes), "pr_dev_download")
        return a.view(dtype) if dtype is not None else a

    def upload(self, arr):
        import numpy as np
        a = np.ascontiguousarray(arr)
        if a.nbytes > self.nbytes:
            raise ValueError("upload larger than the device buffer")
        check(lib().pr_dev_upload(self.ctx.h, self.ptr, a.ctypes.data, a.nbytes), "pr_dev_upload")

    def close(self):
        if self.ptr and self.ctx.h:   # (never through a destroyed context's handle)
            lib().pr_dev_free(self.ctx.h, self.ptr)
            self.ptr = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class MemGroup(C.Structure):
    _fields_ = [("name", C.c_char * 16), ("cur", C.c_int64), ("peak", C.c_int64), ("at_total_peak", C.c_int64)]


def mem_stats() -> dict:
    """Device memory of the library's buffers (pr_mem_stats): bytes now, the peak since the
    last mem_reset_peak(), and per buffer group {cur, peak, at_total_peak} in bytes."""
    L = lib()
    L.pr_mem_stats.argtypes = [P64, P64, C.POINTER(MemGroup), C.c_int, P32]
    g = (MemGroup * 16)()
    cur, peak, n = C.c_int64(), C.c_int64(), C.c_int32()
    check(L.pr_mem_stats(C.byref(cur), C.byref(peak), g, 16, C.byref(n)), "pr_mem_stats")
    return {"cur": cur.value, "peak": peak.value,
            "groups": {g[k].name.decode(): {"cur": g[k].cur, "peak": g[k].peak, "at_total_peak": g[k].at_total_peak}
                       for k in range(min(n.value, 16))}}


def mem_reset_peak() -> None:
    L = lib()
    L.pr_mem_reset_peak.restype = None
    L.pr_mem_reset_peak()


_default_ctx = None


def default_context() -> Context:
    global _default_ctx
    if _default_ctx is None:
        dev = int(os.environ.get("LOCAL_RANK", "-1"))
        _default_ctx = Context(dev)
    return _default_ctx


def ptr(a, ctype):
    """numpy array -> ctypes pointer (None for None)."""
    if a is None:
        return None
    return a.ctypes.data_as(C.POINTER(ctype))
