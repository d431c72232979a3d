"""ctypes binding of librmd.so — the C ABI declared in include/rmd.h.

This is the reference-side binding a maintainer of qzed/raft-meets-dicl would add:
plain pointers, sizes and the current HIP stream.  There is no CPU fallback: if the library is
missing, or a tensor is not on the GPU, the call raises.
"""

import ctypes
import hashlib
import os

import torch  # noqa: F401  (load torch's libamdhip64 first so librmd.so binds to the same HIP runtime)

RMD_OK = 0
RMD_F32, RMD_F16, RMD_BF16, RMD_BF16X3, RMD_S24 = 0, 1, 2, 3, 4
RMD_LAYOUT_ROWS, RMD_LAYOUT_TILES = 0, 1
MAX_LEVELS = 4

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("RMD_LIBRARY", os.path.join(_HERE, "librmd.so"))


class PyramidDesc(ctypes.Structure):
    """Mirror of rmd_pyramid_desc (include/rmd.h)."""

    _fields_ = [
        ("batch", ctypes.c_int), ("height", ctypes.c_int), ("width", ctypes.c_int),
        ("levels", ctypes.c_int), ("storage", ctypes.c_int),
        ("level_h", ctypes.c_int * MAX_LEVELS), ("level_w", ctypes.c_int * MAX_LEVELS),
        ("tile_h", ctypes.c_int * MAX_LEVELS), ("tile_w", ctypes.c_int * MAX_LEVELS),
        ("tiles_y", ctypes.c_int * MAX_LEVELS), ("tiles_x", ctypes.c_int * MAX_LEVELS),
        ("level_offset", ctypes.c_longlong * MAX_LEVELS),
        ("total_elements", ctypes.c_longlong),
        ("layout", ctypes.c_int), ("query_slots", ctypes.c_int),
    ]


class RmdError(RuntimeError):
    pass


_lib = None

_P = ctypes.c_void_p
_I = ctypes.c_int
_U = ctypes.c_uint
_SIGS = {
    "rmd_pyramid_describe": (_I, [_I, _I, _I, _I, _I, ctypes.POINTER(PyramidDesc)]),
    "rmd_pyramid_describe_layout": (_I, [_I, _I, _I, _I, _I, _I, ctypes.POINTER(PyramidDesc)]),
    "rmd_pyramid_describe_for": (_I, [_I, _I, _I, _I, _I, _I, _I, ctypes.POINTER(PyramidDesc)]),
    "rmd_corr_pyramid_workspace_bytes": (ctypes.c_size_t, [ctypes.POINTER(PyramidDesc), _I, _I]),
    "rmd_corr_pyramid": (_I, [_P, _P, _I, ctypes.c_float, ctypes.POINTER(PyramidDesc), _I, _P, _P, _P]),
    "rmd_corr_lookup": (_I, [_P, ctypes.POINTER(PyramidDesc), _P, _I, _U, _P, _P]),
    "rmd_corr_gemm_kernel": (ctypes.c_char_p, [ctypes.POINTER(PyramidDesc), _I, _I]),
    "rmd_corr_prepare": (_I, [_P, _P, _I, ctypes.c_float, ctypes.POINTER(PyramidDesc), _I, _P, _P]),
    "rmd_corr_pyramid_prepared": (_I, [_I, ctypes.c_float, ctypes.POINTER(PyramidDesc), _I, _P, _P, _P]),
    "rmd_corr_otf_workspace_bytes": (ctypes.c_size_t, [_I] * 6),
    "rmd_corr_otf_prepare": (_I, [_P, _P] + [_I] * 5 + [ctypes.c_float, _I, _P, _P]),
    "rmd_corr_otf_lookup": (_I, [_P] + [_I] * 6 + [_P, _I, _U, _P, _P]),
    "rmd_corr_otf_record_bytes": (ctypes.c_size_t, [_I] * 5),
    "rmd_corr_otf_record": (_I, [_P, _P] + [_I] * 5 + [_U, _P, _P]),
    "rmd_corr_otf_backward_workspace_bytes": (ctypes.c_size_t, [_I] * 6),
    "rmd_corr_otf_backward": (_I, [_P, _P, _P] + [_I] * 5 + [ctypes.c_float, _I, _I, _I, ctypes.POINTER(_P), _P, _P,
                                                               _P, _P]),
    "rmd_corr_grad_targets": (ctypes.c_longlong, [_I, _I, _I]),
    "rmd_corr_lookup_backward": (_I, [_P, ctypes.POINTER(PyramidDesc), _P, _I, _U, _P, _P]),
    "rmd_corr_grad_build": (_I, [ctypes.POINTER(_P), ctypes.POINTER(_P), ctypes.POINTER(_U), _I,
                                 ctypes.POINTER(PyramidDesc), _I, _I, _P, _P]),
    "rmd_corr_grad_build_ex": (_I, [ctypes.POINTER(_P), ctypes.POINTER(_P), ctypes.POINTER(_U), _I,
                                    ctypes.POINTER(PyramidDesc), _I, _I, _I, _P, _P]),
    "rmd_corr_grad_gemm_bf16g": (_I, [_P, ctypes.c_longlong, _P, ctypes.c_longlong, _I, _I, _I, _I, _I, _P, _P, _P]),
    "rmd_corr_pool_targets": (_I, [_P, _I, _I, _I, _I, _I, ctypes.c_float, _P, _P]),
    "rmd_corr_unpool_targets": (_I, [_P, _I, _I, _I, _I, _I, ctypes.c_float, _P, _P]),
    "rmd_corr_grad_gemm_workspace_bytes": (ctypes.c_size_t, [_I, _I, _I, _I]),
    "rmd_corr_grad_gemm": (_I, [_P, ctypes.c_longlong, _P, ctypes.c_longlong, _I, _I, _I, _I, _I, _I, _P, _P, _P]),
    "rmd_dicl_stack": (_I, [_P, _P, _P] + [_I] * 11 + [_P, _P]),
    "rmd_dicl_stack_backward": (_I, [_P, _P] + [_I] * 11 + [_P, _P, _P]),
    "rmd_dicl_stack_int_workspace_bytes": (ctypes.c_size_t, [_I, _I, _I]),
    "rmd_dicl_stack_int": (_I, [_P, _P] + [_I] * 6 + [_P, _P, _P]),
    "rmd_dicl_stack_int_backward": (_I, [_P, _P] + [_I] * 6 + [_P, _P, _P, _P]),
    "rmd_warp_backwards": (_I, [_P, _P, _I, _I, _I, _I, ctypes.c_float, _P, _P, _P]),
    "rmd_warp_backwards_backward": (_I, [_P, _P, _I, _I, _I, _I, ctypes.c_float, _P, _P]),
    "rmd_dicl_stack_int_warped_workspace_bytes": (ctypes.c_size_t, [_I, _I, _I, _I]),
    "rmd_dicl_stack_int_warped": (_I, [_P, _P, _P] + [_I] * 6 + [_P, _P, _P]),
    "rmd_dicl_stack_int_warped_backward": (_I, [_P, _P, _P] + [_I] * 6 + [_P, _P, _P, _P]),
    "rmd_dap": (_I, [_P, _P, _I, _I, _I, _I, _P, _P]),
    "rmd_dap_weight_grad_workspace_bytes": (ctypes.c_size_t, [_I, _I, _I]),
    "rmd_dap_weight_grad": (_I, [_P, _P, _I, _I, _I, _P, _P, _P]),
    "rmd_input_images": (_I, [_P, _I, _I, _I, _I, ctypes.c_float, ctypes.c_float, ctypes.c_float, ctypes.c_float,
                              _I, _I, _I, _I, _I, _P, _P]),
    "rmd_input_flow": (_I, [_P, _P, _I, _I, _I, _I, _I, _I, _I, ctypes.c_float, _P, _P, _P]),
    "rmd_up8": (_I, [_P, _P, _I, _I, _I, ctypes.c_float, _P, _P]),
    "rmd_up8_workspace_bytes": (ctypes.c_size_t, [_I, _I, _I]),
    "rmd_up8_backward": (_I, [_P, _P, _P, _I, _I, _I, ctypes.c_float, _P, _P, _P, _P]),
    "rmd_softargmax": (_I, [_P, _I, _I, _I, _I, _I, ctypes.c_float, _P, _P]),
    "rmd_softargmax_backward": (_I, [_P, _P, _I, _I, _I, _I, _I, ctypes.c_float, _P, _P]),
    "rmd_last_error": (ctypes.c_char_p, []),
    "rmd_version": (ctypes.c_char_p, []),
    "rmd_abi_version": (_I, []),
    "rmd_source_hash": (ctypes.c_char_p, []),
}

# include/rmd.h RMD_ABI_VERSION this binding's signatures (_SIGS) were written for
ABI_VERSION = 2


def lib():
    """Load librmd.so once; raise loudly if it is missing (no fallback path exists)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RmdError(f"rmd: HIP library not found at {LIB_PATH}; build it with "
                           f"`python -c 'import __graft_entry__ as g; g.build()'` (no CPU fallback)")
        l = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in _SIGS.items():
            fn = getattr(l, name)
            fn.restype = res
            fn.argtypes = args
        if l.rmd_abi_version() != ABI_VERSION:
            raise RmdError(f"rmd: {LIB_PATH} implements ABI {l.rmd_abi_version()}, this binding needs "
                           f"ABI {ABI_VERSION} (include/rmd.h RMD_ABI_VERSION); rebuild the library")
        _lib = l
    return _lib


_CSRC = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "csrc")
_HEADER = os.path.join(os.path.dirname(os.path.dirname(_CSRC)), "include", "rmd.h")
_SRC_TAG = b"rmd-src-hash:"


def source_hash():
    """The csrc/Makefile fingerprint recomputed from the tree (None without the sources): sha256 of
    csrc/{*.cpp,*.h,*.hip} in name order, then include/rmd.h, first 16 hex digits."""
    if not os.path.isdir(_CSRC) or not os.path.exists(_HEADER):
        return None
    names = sorted(n for n in os.listdir(_CSRC) if n.endswith((".cpp", ".h", ".hip")))
    h = hashlib.sha256()
    for p in [os.path.join(_CSRC, n) for n in names] + [_HEADER]:
        with open(p, "rb") as f:
            h.update(f.read())
    return h.hexdigest()[:16]


def library_source_hash(path=LIB_PATH):
    """The fingerprint baked into a built library, read from the file without loading it."""
    if not os.path.exists(path):
        return None
    with open(path, "rb") as f:
        data = f.read()
    i = data.find(_SRC_TAG)
    if i < 0:
        return None
    return data[i + len(_SRC_TAG):i + len(_SRC_TAG) + 16].decode("ascii", errors="replace")


def build_info():
    """{"source_hash": library's, "tree_hash": the sources', "sources_match": bool or None}."""
    lh, th = library_source_hash(), source_hash()
    return {"source_hash": lh, "tree_hash": th, "sources_match": (lh == th) if (lh and th) else None}


def symbols():
    return sorted(_SIGS)


def check(rc, what):
    if rc != RMD_OK:
        msg = lib().rmd_last_error().decode(errors="replace")
        raise RmdError(f"{what} failed (code {rc}): {msg}")


def describe(batch, height, width, levels, storage, layout=RMD_LAYOUT_ROWS):
    d = PyramidDesc()
    check(lib().rmd_pyramid_describe_layout(batch, height, width, levels, storage, layout, ctypes.byref(d)),
          "rmd_pyramid_describe")
    return d


def describe_for(batch, height, width, levels, storage, channels, compute):
    """The pyramid rmd_corr_pyramid writes for (channels, compute): tiles layout on the w8 GEMM."""
    d = PyramidDesc()
    check(lib().rmd_pyramid_describe_for(batch, height, width, levels, storage, channels, compute, ctypes.byref(d)),
          "rmd_pyramid_describe_for")
    return d


def stream_ptr(device):
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)
