"""ctypes binding of libmhada_hip.so (include/mhada_hip.h).

The library is built in-tree by ``csrc/Makefile`` (``__graft_entry__.build()``).  There is no
fallback: if the library is missing every op raises, so a GPU run can never silently take
a CPU or aten path.
"""
from __future__ import annotations

import ctypes
import os
import threading

LIB_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "libmhada_hip.so")

F32, BF16 = 0, 1
ACT_SOFTMAX, ACT_COSINE = 0, 1
A_ROWS, A_PATCH8, A_CONV3X3, A_CONV3X3_UP2, A_CONV3X3_ZERO, A_SPLIT3 = 0, 1, 2, 3, 4, 5
BF16X3 = 2  # mhada_layernorm y_dtype: three bf16 planes (the A_SPLIT3 operand)
PAD_REFLECT, PAD_ZERO = 0, 1

_c_ll = ctypes.c_longlong
_vp = ctypes.c_void_p


class GemmArgs(ctypes.Structure):
    """mirror of ``mhada_gemm_args``"""
    _fields_ = [
        ("M", ctypes.c_int), ("N", ctypes.c_int), ("K", ctypes.c_int),
        ("nb1", ctypes.c_int), ("nb2", ctypes.c_int),
        ("compute", ctypes.c_int), ("a_mode", ctypes.c_int),
        ("a", _vp), ("a_dtype", ctypes.c_int), ("lda", _c_ll), ("sa1", _c_ll), ("sa2", _c_ll),
        ("a_mu", _vp), ("smu1", _c_ll), ("smu2", _c_ll),
        ("img_c", ctypes.c_int), ("img_h", ctypes.c_int), ("img_w", ctypes.c_int),
        ("w", _vp), ("ldw", _c_ll), ("sw1", _c_ll), ("sw2", _c_ll),
        ("bias", _vp), ("sb1", _c_ll), ("sb2", _c_ll),
        ("r", _vp), ("r_dtype", ctypes.c_int), ("ldr", _c_ll), ("sr1", _c_ll), ("sr2", _c_ll),
        ("c", _vp), ("c_dtype", ctypes.c_int), ("ldc", _c_ll), ("sc1", _c_ll), ("sc2", _c_ll),
        ("relu", ctypes.c_int), ("pad", ctypes.c_int),
        ("c2", _vp), ("ldc2", _c_ll), ("sc21", _c_ll), ("sc22", _c_ll),
        ("vt", _vp), ("ldt", _c_ll), ("svt1", _c_ll), ("svt2", _c_ll),
        ("c2_planes", ctypes.c_int),
    ]


class GemmTnArgs(ctypes.Structure):
    """mirror of ``mhada_gemm_tn_args``"""
    _fields_ = [
        ("M", ctypes.c_int), ("N", ctypes.c_int), ("K", ctypes.c_int),
        ("a", _vp), ("lda", _c_ll), ("b", _vp), ("ldb", _c_ll), ("b_mode", ctypes.c_int),
        ("img_c", ctypes.c_int), ("img_h", ctypes.c_int), ("img_w", ctypes.c_int), ("pad", ctypes.c_int),
        ("c", _vp), ("ldc", _c_ll), ("colsum", _vp),
        ("nb", ctypes.c_int), ("sza", _c_ll), ("szb", _c_ll),
    ]


# name -> (restype, argtypes); every symbol declared in include/mhada_hip.h
_I, _F = ctypes.c_int, ctypes.c_float
SIGNATURES = {
    "mhada_abi_version": (_I, []),
    "mhada_last_error": (ctypes.c_char_p, []),
    "mhada_set_tuning": (_I, [ctypes.c_char_p, _I]),
    "mhada_get_tuning": (_I, [ctypes.c_char_p, ctypes.POINTER(_I)]),
    "mhada_clock_probe": (_I, [_vp, _I, _I, _vp]),
    "mhada_gemm": (_I, [ctypes.POINTER(GemmArgs), _vp]),
    "mhada_layernorm": (_I, [_vp, _vp, _I, _vp, _vp, _I, _I, _F, _vp]),
    "mhada_vit_batch_attn": (_I, [_vp, _vp, _I, _I, _I, _I, _I, _vp]),
    "mhada_pos_embed": (_I, [_vp, _vp, _I, _I, _I, _I, _I, _vp]),
    "mhada_instnorm_stats": (_I, [_vp, _vp, _vp, _vp, _I, _I, _I, _I, _F, _vp]),
    "mhada_fold_block": (_I, [_vp] * 12 + [_F, _I, _I, _I, _vp]),
    "mhada_transpose_v": (_I, [_vp, _vp, _I, _I, _I, _I, _vp]),
    "mhada_cosine_prep": (_I, [_vp, _vp, _I, _I, _I, _I, _I, _vp]),
    "mhada_cosine_moments": (_I, [_vp, _vp, _I, _I, _I, _I, _vp, _vp, _I, _vp]),
    "mhada_cosine_attn": (_I, [_vp, _vp, _vp, _vp, _vp, _vp, _vp, _I, _I, _I, _I, _vp]),
    "mhada_attn": (_I, [_vp] * 8 + [_I, _I, _I, _I, _I, _I, _vp]),
    "mhada_split3_kv": (_I, [_vp, _vp, _vp, _I, _I, _I, _vp]),
    "mhada_kv_proj_split3": (_I, [_vp] * 5 + [_I, _I, _I, _vp]),
    "mhada_split3_rows": (_I, [_vp, _vp, _c_ll, _vp]),
    "mhada_split3_weight": (_I, [_vp, _vp, _I, _I, _I, _vp]),
    "mhada_attn_split3": (_I, [_vp] * 7 + [_I, _I, _I, _I, _vp]),
    "mhada_attn_train_fwd": (_I, [_vp] * 7 + [_I, _I, _I, _vp]),
    "mhada_attn_train_fwd_vt": (_I, [_vp] * 8 + [_I, _I, _I, _vp]),
    "mhada_attn_train_fwd_split3": (_I, [_vp] * 8 + [_I, _I, _I, _vp]),
    "mhada_transpose64": (_I, [_vp, _vp, _I, _I, _I, _vp]),
    "mhada_gemm_n64_split3": (_I, [_vp, _vp, _vp, _I, _I, _I, _I, _c_ll, _I, _c_ll, _c_ll, _I, _c_ll, _vp]),
    "mhada_transpose64_split3": (_I, [_vp, _vp, _I, _I, _I, _vp]),
    "mhada_attn_train_bwd": (_I, [_vp] * 9 + [_I, _I, _I, _vp]),
    "mhada_attn_train_dkv": (_I, [_vp] * 9 + [_I, _I, _I, _vp]),
    "mhada_conv3x3_out3": (_I, [_vp, _I, _vp, _vp, _vp, _I, _I, _I, _I, _I, _vp]),
    "mhada_upsample2x": (_I, [_vp, _vp, _I, _I, _I, _I, _I, _vp]),
    "mhada_warp": (_I, [_vp, _vp, _vp, _I, _I, _I, _I, _I, _vp]),
    "mhada_warp_bwd": (_I, [_vp, _vp, _vp, _I, _I, _I, _I, _I, _vp]),
    "mhada_flow_warp_mask": (_I, [_vp, _vp, _vp, _I, _I, _F, _I, _vp]),
    "mhada_warp_l1": (_I, [_vp, _vp, _vp, _vp, _vp, _vp, _I, _I, _I, _I, _vp]),
    "mhada_frame_ingest": (_I, [_vp, _I, _I, _I, _c_ll, _I, _vp, _I, _I, _vp]),
    "mhada_gemm_tn_splits": (_I, [_I, _I, _I]),
    "mhada_loss_attn": (_I, [_vp] * 7 + [_I, _I, _I, _I, _I, _I, _vp]),
    "mhada_rows_normalize": (_I, [_vp] * 4 + [_I, _I, _I, _I, _vp]),
    "mhada_gemm_tn": (_I, [ctypes.POINTER(GemmTnArgs), _vp, _c_ll, _vp]),
    "mhada_colsum": (_I, [_vp, _vp, _c_ll, _I, _vp, _c_ll, _vp]),
    "mhada_layernorm_fwd": (_I, [_vp, _vp, _vp, _vp, _vp, _I, _I, _F, _vp]),
    "mhada_layernorm_fwd_split3": (_I, [_vp, _vp, _vp, _vp, _vp, _vp, _I, _I, _F, _vp]),
    "mhada_layernorm_bwd": (_I, [_vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _c_ll, _I, _I, _vp]),
    "mhada_pos_embed_bwd": (_I, [_vp, _vp, _I, _I, _I, _I, _I, _vp]),
    "mhada_instnorm_bwd": (_I, [_vp, _vp, _vp, _vp, _vp, _I, _I, _I, _I, _vp]),
    "mhada_attn_train_bwd_prep": (_I, [_vp, _vp, _vp, _vp, _vp, _vp, _c_ll, _vp]),
    "mhada_vit_batch_attn_bwd": (_I, [_vp, _vp, _vp, _I, _I, _I, _I, _vp]),
    "mhada_vit_batch_attn_bwd_split3": (_I, [_vp, _vp, _vp, _vp, _c_ll, _I, _I, _I, _I, _vp]),
    "mhada_relu_bwd": (_I, [_vp, _vp, _vp, _c_ll, _vp]),
    "mhada_feat_stats_work": (_c_ll, [_I, _c_ll, _I]),
    "mhada_feat_stats": (_I, [_vp, _vp, _vp, _vp, _vp, _vp, _c_ll, _I, _c_ll, _I, _vp]),
    "mhada_feat_loss_bwd": (_I, [_vp, _vp, _vp, _vp, _vp, _vp, _F, _vp, _I, _c_ll, _I, _I, _vp]),
    "mhada_reflect_fold": (_I, [_vp, _vp, _I, _I, _I, _I, _vp, _vp]),
    "mhada_maxpool2": (_I, [_vp, _vp, _I, _I, _I, _I, _vp]),
    "mhada_maxpool2_bwd": (_I, [_vp, _vp, _vp, _I, _I, _I, _I, _I, _vp]),
    "mhada_upsample2x_bwd": (_I, [_vp, _vp, _vp, _I, _I, _I, _I, _vp]),
    "mhada_vgg_input": (_I, [_vp, _vp, _I, _I, _I, _I, _vp]),
    "mhada_vgg_input_bwd": (_I, [_vp, _vp, _I, _I, _I, _I, _vp]),
    "mhada_wino_weights": (_I, [_vp, _vp, _I, _I, _vp]),
    "mhada_conv3x3_wgrad_wino_splits": (_I, [_I, _I, _I, _I, _I]),
    "mhada_conv3x3_wgrad_wino": (_I, [_vp, _vp, _vp, _vp, _vp, _c_ll, _I, _I, _I, _I, _I, _c_ll, _I, _vp]),
    "mhada_conv3x3_wino": (_I, [_vp] * 4 + [_I] * 5 + [_c_ll, _I, _I, _I, _vp, _vp]),
    "mhada_vgg_stem_dgrad": (_I, [_vp] * 4 + [_I] * 3 + [_vp]),
    "mhada_out3_dgrad": (_I, [_vp] * 5 + [_I] * 3 + [_vp]),
    "mhada_out3_wgrad_work": (_c_ll, [_I, _I, _I]),
    "mhada_out3_wgrad": (_I, [_vp] * 6 + [_c_ll, _I, _I, _I, _vp]),
}

_lib = None
_lock = threading.Lock()


def load(path: str | None = None) -> ctypes.CDLL:
    """Load (once) and type the library; raises RuntimeError if it is not built."""
    global _lib
    if _lib is not None and path is None:
        return _lib
    with _lock:
        if _lib is not None and path is None:
            return _lib
        p = path or LIB_PATH
        if not os.path.exists(p):
            raise RuntimeError(
                f"MHAda HIP library not found at {p}; build it with "
                "`python -c 'import __graft_entry__ as g; g.build()'` (make -C mhada-style-transfer_amd/csrc)")
        lib = ctypes.CDLL(p)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        if path is None:
            _lib = lib
        return lib


ABI_VERSION = 16


def get_tuning(name: str) -> int:
    v = ctypes.c_int()
    check(load().mhada_get_tuning(name.encode(), ctypes.byref(v)), "mhada_get_tuning")
    return v.value


def set_tuning(name: str, value: int) -> None:
    """Select a kernel variant (include/mhada_hip.h: A/B measurements and rare-path tests)."""
    check(load().mhada_set_tuning(name.encode(), int(value)), "mhada_set_tuning")


class tuning:
    """Context manager: ``with tuning(attn_fixed_shift=0): ...`` restores the previous values."""

    def __init__(self, **knobs: int):
        self.knobs = knobs
        self.saved = {}

    def __enter__(self):
        for k, v in self.knobs.items():
            self.saved[k] = get_tuning(k)
            set_tuning(k, v)
        return self

    def __exit__(self, *exc):
        for k, v in self.saved.items():
            set_tuning(k, v)
        return False


def check(rc: int, what: str) -> None:
    if rc != 0:
        msg = load().mhada_last_error()
        msg = msg.decode() if msg else "unknown error"
        if rc == 1:
            raise ValueError(f"{what}: {msg}")
        raise RuntimeError(f"{what}: {msg}")
