"""ctypes binding of libfceyolo.so (the C-ABI declared in include/fce_yolo.h).

The library is loaded from ``fce-yolo_amd/lib/libfceyolo.so`` (built in-tree by
``build.py``).  Every wrapper raises ``FceError`` with ``fce_last_error()`` on a non-zero
status; there is no fallback path: if the library is missing, ``lib()`` raises.
"""

from __future__ import annotations

import ctypes as C
import os
from pathlib import Path

LIB_PATH = Path(__file__).resolve().parent / "lib" / "libfceyolo.so"

F16, F32, U8 = 0, 1, 2
NHWC, NCHW = 0, 1
ACT_NONE, ACT_SILU = 0, 1
EPI_STORE, EPI_WSTORE, EPI_ACCUM = 0, 1, 2
PLAN_NO_AUTOTUNE = 1


class FceError(RuntimeError):
    pass


class Tensor(C.Structure):
    _fields_ = [
        ("data", C.c_void_p),
        ("dtype", C.c_int),
        ("layout", C.c_int),
        ("n", C.c_int),
        ("c", C.c_int),
        ("h", C.c_int),
        ("w", C.c_int),
        ("cstride", C.c_int),
        ("coff", C.c_int),
    ]


class ConvDesc(C.Structure):
    _fields_ = [
        ("cin", C.c_int),
        ("cout", C.c_int),
        ("k", C.c_int),
        ("stride", C.c_int),
        ("groups", C.c_int),
        ("act", C.c_int),
        ("up", C.c_int),
        ("epilogue", C.c_int),
        ("fusion_w", C.c_void_p),
        ("fusion_n", C.c_int),
        ("fusion_i", C.c_int),
    ]


class DetectEpi(C.Structure):
    _fields_ = [
        ("pred", C.c_void_p),
        ("anchors", C.c_int),
        ("anchor_offset", C.c_int),
        ("nc", C.c_int),
        ("reg_max", C.c_int),
        ("part", C.c_int),
        ("stride", C.c_float),
        ("best", C.c_void_p),
    ]


class CoordDesc(C.Structure):
    _fields_ = [
        ("inp", C.c_int),
        ("oup", C.c_int),
        ("mid", C.c_int),
        ("heads", C.c_int),
        ("scale", C.c_float),
        ("w", C.c_void_p * 8),
        ("b", C.c_void_p * 8),
        ("id_w", C.c_void_p),
        ("id_b", C.c_void_p),
    ]


class C3k2Desc(C.Structure):
    _fields_ = [
        ("cin", C.c_int),
        ("c", C.c_int),
        ("c_mid", C.c_int),
        ("cout", C.c_int),
        ("w", C.c_void_p * 4),
        ("b", C.c_void_p * 4),
    ]


class DclsDesc(C.Structure):
    """fce_dcls_desc: the Detect cls branch of one level (w / b: dw1, pw1, dw2, pw2, cls)."""
    _fields_ = [
        ("c0", C.c_int),
        ("c3", C.c_int),
        ("nc", C.c_int),
        ("w", C.c_void_p * 5),
        ("b", C.c_void_p * 5),
    ]


class Stem2Desc(C.Structure):
    """fce_stem2_desc: the backbone's first two convs (w / b: stem, second conv)."""
    _fields_ = [
        ("c0", C.c_int),
        ("c1", C.c_int),
        ("w", C.c_void_p * 2),
        ("b", C.c_void_p * 2),
    ]


class BneckDesc(C.Structure):
    """fce_bneck_desc: a chain of n Bottlenecks (w / b: cv1, cv2 of each, in chain order)."""
    _fields_ = [
        ("c", C.c_int),
        ("c_mid", C.c_int),
        ("n", C.c_int),
        ("shortcut", C.c_int),
        ("w", C.c_void_p * 4),
        ("b", C.c_void_p * 4),
    ]


class Pw2Desc(C.Structure):
    """fce_pw2_desc: two chained 1x1 convs (w / b / act: op 1, op 2; epi1 / fw / fn / fi: op 1's BiFPN epilogue)."""
    _fields_ = [
        ("cin1", C.c_int),
        ("cout1", C.c_int),
        ("cin2", C.c_int),
        ("cout2", C.c_int),
        ("act", C.c_int * 2),
        ("w", C.c_void_p * 2),
        ("b", C.c_void_p * 2),
        ("epi1", C.c_int),
        ("fw", C.c_void_p),
        ("fn", C.c_int),
        ("fi", C.c_int),
    ]


class NmsOpts(C.Structure):
    """fce_nms_opts: the non-default arguments of non_max_suppression (utils/nms.py:13-29)."""
    _fields_ = [
        ("conf_thres", C.c_float),
        ("iou_thres", C.c_float),
        ("max_det", C.c_int),
        ("max_nms", C.c_int),
        ("max_wh", C.c_float),
        ("agnostic", C.c_int),
        ("multi_label", C.c_int),
        ("classes", C.c_void_p),
        ("nclasses", C.c_int),
    ]


_P = C.c_void_p
_I = C.c_int
_SZ = C.c_size_t
_PT = C.POINTER(Tensor)
_PCD = C.POINTER(ConvDesc)
_PCO = C.POINTER(CoordDesc)
_PC3 = C.POINTER(C3k2Desc)
_PDC = C.POINTER(DclsDesc)
_PST = C.POINTER(Stem2Desc)
_PBN = C.POINTER(BneckDesc)
_PPW = C.POINTER(Pw2Desc)

_SIGS = {
    "fce_last_error": (C.c_char_p, []),
    "fce_abi_version": (_I, []),
    "fce_device_count": (_I, []),
    "fce_conv_weight_bytes": (_SZ, [_PCD]),
    "fce_conv_pack_weights": (_I, [_PCD, _P, _P]),
    "fce_conv2d": (_I, [_PCD, _PT, _P, _P, _PT, _PT, _P]),
    "fce_conv_variants": (_I, [_PCD, _I, _P, _I]),
    "fce_letterbox": (_I, [_P, _I, _P, _I, _I, _I, _P]),
    "fce_scale_boxes": (_I, [_P, _P, _I, _I, _P, _P]),
    "fce_conv2d_variant": (_I, [_PCD, _PT, _P, _P, _PT, _PT, _I, _P]),
    "fce_conv2d_variant_dup": (_I, [_PCD, _PT, _P, _P, _PT, _PT, _I, _PT, _I, _P]),
    "fce_conv2d_detect": (_I, [_PCD, _PT, _P, _P, C.POINTER(DetectEpi), _P]),
    "fce_maxpool_chain": (_I, [_PT, _PT, _PT, _PT, _I, _P]),
    "fce_weighted_add": (_I, [_PT, _I, _P, _I, _I, _I, _PT, _P]),
    "fce_coord_workspace_bytes": (_SZ, [_PCO, _I, _I, _I]),
    "fce_c3k2_supported": (_I, [_PC3]),
    "fce_c3k2": (_I, [_PC3, _PT, _PT, _P]),
    "fce_net_add_c3k2": (_I, [_P, _PC3, _I, _I, _I, _I]),
    "fce_net_add_c3k2_alt": (_I, [_P, _PC3, _I, _I, _I, _I, _I, _I]),
    "fce_net_c3k2_form": (_I, [_P, _I]),
    "fce_net_set_c3k2_form": (_I, [_P, _I, _I]),
    "fce_net_op_skipped": (_I, [_P, _I]),
    "fce_detect_cls_supported": (_I, [_PDC]),
    "fce_detect_cls": (_I, [_PDC, _PT, C.POINTER(DetectEpi), _P]),
    "fce_net_add_detect_cls_alt": (_I, [_P, _PDC, _I, _I, _I, _I]),
    "fce_net_alt_form": (_I, [_P, _I]),
    "fce_stem_fused_supported": (_I, [_PST]),
    "fce_stem_fused": (_I, [_PST, _PT, _PT, _P]),
    "fce_net_add_stem_alt": (_I, [_P, _PST, _I, _I]),
    "fce_net_set_alt_form": (_I, [_P, _I, _I]),
    "fce_bneck_supported": (_I, [_PBN]),
    "fce_bneck_fused": (_I, [_PBN, _PT, _PT, _P]),
    "fce_net_add_bneck_alt": (_I, [_P, _PBN, _I, _I, _I, _I, _I, _I]),
    "fce_pw2_supported": (_I, [_PPW]),
    "fce_pw2": (_I, [_PPW, _PT, _PT, _PT, _I, _PT, _PT, _PT, _PT, _I, _P]),
    "fce_net_add_pw2_alt": (_I, [_P, _PPW, _I]),
    "fce_bicoordcrossatt": (_I, [_PCO, _PT, _PT, _P, _SZ, _P]),
    "fce_coordatt": (_I, [_PCO, _PT, _PT, _P, _SZ, _P]),
    "fce_coordcrossatt": (_I, [_PCO, _PT, _PT, _P, _SZ, _P]),
    "fce_psa_attention": (_I, [_PT, _I, _I, _I, _P, _P, _PT, _P]),
    "fce_detect_decode": (_I, [_PT, _PT, _I, _P, _I, _P, _P]),
    "fce_nms_workspace_bytes": (_SZ, [_I, _I, _I]),
    "fce_nms": (_I, [_P, _I, _I, _I, C.c_float, C.c_float, _I, _I, C.c_float, _P, _SZ, _P, _P, _P, _P]),
    "fce_nms_best": (_I, [_P, _P, _I, _I, _I, C.c_float, C.c_float, _I, _I, C.c_float, _P, _SZ, _P, _P, _P, _P]),
    "fce_nms_workspace_bytes_ex": (_SZ, [_I, _I, _I, C.POINTER(NmsOpts)]),
    "fce_nms_ex": (_I, [_P, _P, _I, _I, _I, C.POINTER(NmsOpts), _P, _SZ, _P, _P, _P, _P]),
    "fce_copy": (_I, [_PT, _PT, _P]),
    "fce_net_create": (_P, []),
    "fce_net_destroy": (None, [_P]),
    "fce_net_add_buffer": (_I, [_P, _I, _I, _I]),
    "fce_net_add_conv": (_I, [_P, _PCD, _I, _I, _I, _I, _I, _I, _P, _P]),
    "fce_net_add_conv_dup": (_I, [_P, _PCD, _I, _I, _I, _I, _I, _I, _P, _P, _I, _I, _I]),
    "fce_net_add_maxpool_chain": (_I, [_P, _I, _I, _I, _I]),
    "fce_net_add_weighted_add": (_I, [_P, _I, _I, _I, _I, _P, _I, _I, _I, _I, _I]),
    "fce_net_add_coord": (_I, [_P, _I, _PCO, _I, _I, _I, _I]),
    "fce_net_add_psa_attention": (_I, [_P, _I, _I, _I, _I, _P, _P, _I, _I]),
    "fce_net_add_detect": (_I, [_P, _I, _P, _P, _I]),
    "fce_net_add_conv_detect": (_I, [_P, _PCD, _I, _I, _I, _I, C.c_float, _I, _I, _P, _P]),
    "fce_net_plan": (_I, [_P, _I, _I, _I]),
    "fce_net_plan_ex": (_I, [_P, _I, _I, _I, _I]),
    "fce_net_arena_bytes": (_SZ, [_P]),
    "fce_net_num_anchors": (_I, [_P]),
    "fce_net_forward": (_I, [_P, _PT, _P, _I, _P]),
    "fce_net_forward_best": (_I, [_P, _PT, _P, _P, _I, _P]),
    "fce_net_fork_hint": (_I, [_P]),
    "fce_net_set_fork": (_I, [_P, _I]),
    "fce_net_wait_fork": (_I, [_P, _P]),
    "fce_net_profile": (_I, [_P, _PT, _P, _P, _P, _I, _P]),
    "fce_net_num_ops": (_I, [_P]),
    "fce_net_op_variant": (_I, [_P, _I]),
    "fce_net_op_variants": (_I, [_P, _I, _P, _I]),
    "fce_net_set_op_variant": (_I, [_P, _I, _I]),
    "fce_net_tune_record": (_I, [_P, _I, _P, _P, _P]),
    "fce_net_op_info": (_I, [_P, _I, C.c_char_p, _I, C.POINTER(C.c_double), C.POINTER(C.c_double)]),
    "fce_net_buffer": (_I, [_P, _I, _PT]),
}

EXPORTED = tuple(_SIGS)
_lib = None


def lib():
    """Load libfceyolo.so once.  Raises FceError if it has not been built."""
    global _lib
    if _lib is None:
        path = Path(os.environ.get("FCE_YOLO_LIB", LIB_PATH))
        if not path.exists():
            raise FceError(f"libfceyolo.so not found at {path}: run `python fce-yolo_amd/build.py` (no fallback path)")
        L = C.CDLL(str(path))
        for name, (res, args) in _SIGS.items():
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _lib = L
    return _lib


def check(status: int, what: str = ""):
    if status != 0:
        msg = lib().fce_last_error().decode(errors="replace")
        raise FceError(f"{what}: status {status}: {msg}")


def call(name: str, *args):
    st = getattr(lib(), name)(*args)
    check(st, name)
    return st


def tensor(data_ptr: int, dtype: int, layout: int, n: int, c: int, h: int, w: int, cstride: int | None = None,
           coff: int = 0) -> Tensor:
    return Tensor(data_ptr, dtype, layout, n, c, h, w, c if cstride is None else cstride, coff)


def ref(x):
    return C.byref(x) if x is not None else None
