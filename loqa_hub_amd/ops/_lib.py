"""ctypes bindings for the in-tree native libraries (``loqa_hub_amd/_native``).

The libraries are loaded lazily, always *after* ``import torch`` so they bind
to the HIP runtime torch already mapped (same soname ``libamdhip64.so.7``).
On a GPU box a missing library is a hard error: GPU ops never silently fall
back to PyTorch.
"""
from __future__ import annotations

import ctypes
import os
import threading

import torch  # noqa: F401  (must be imported before the HIP libraries)

_HERE = os.path.dirname(os.path.abspath(__file__))
_NATIVE = os.path.join(os.path.dirname(_HERE), "_native")
_lock = threading.Lock()
_kernels = None
_runtime = None

c_void_p = ctypes.c_void_p
c_int = ctypes.c_int
c_ll = ctypes.c_longlong
c_float = ctypes.c_float

class FusedParams(ctypes.Structure):
    """Mirror of ``FusedParams`` in csrc/kernels/gemm_skinny.hip."""
    _fields_ = [
        ("x", c_void_p), ("ldx", c_ll), ("Wp", c_void_p), ("part", c_void_p),
        ("counters", c_void_p),
        ("Mpad", c_int), ("N", c_int), ("K", c_int), ("S", c_int), ("mode", c_int),
        ("norm", c_int),
        ("rowsq_in", c_void_p), ("rowsum_in", c_void_p), ("rowstat_tiles", c_int),
        ("eps", c_float),
        ("colsum", c_void_p), ("bias", c_void_p),
        ("out", c_void_p), ("ldo", c_ll), ("act", c_int),
        ("residual", c_void_p), ("rowsq_out", c_void_p), ("rowsum_out", c_void_p),
        ("positions", c_void_p), ("cs", c_void_p), ("q_out", c_void_p), ("kc", c_void_p),
        ("vc", c_void_p), ("slots", c_void_p),
        ("H", c_int), ("Hkv", c_int), ("D", c_int), ("blk", c_int),
        ("rt", c_int), ("wr", c_int), ("xl", c_int),
        ("pro", c_int), ("pro_ctr", c_void_p), ("pro_wgs", c_int),
        ("car", c_void_p), ("car_which", c_int), ("car_nblk", c_int),
        ("att_q", c_void_p), ("att_q_stride", c_ll), ("att_kc", c_void_p), ("att_vc", c_void_p),
        ("att_cu_q", c_void_p), ("att_ctx", c_void_p), ("att_bt", c_void_p),
        ("att_max_blocks", c_int), ("att_blk", c_int),
        ("att_B", c_int), ("att_Hq", c_int), ("att_Hkv", c_int), ("att_split_keys", c_int),
        ("att_num_splits", c_int), ("att_total_q", c_int),
        ("att_scale", c_float), ("att_part_o", c_void_p), ("att_part_ml", c_void_p),
        ("att_counters", c_void_p),
    ]


class GemmTileParams(ctypes.Structure):
    """Mirror of ``GemmTileParams`` in csrc/kernels/gemm_tile.hip."""
    _fields_ = [
        ("x", c_void_p), ("ldx", c_ll), ("w", c_void_p),
        ("M", c_int), ("N", c_int), ("K", c_int), ("S", c_int),
        ("epi", c_int), ("act", c_int), ("bias", c_void_p),
        ("pos", c_void_p), ("pos_rows", c_int),
        ("y", c_void_p), ("ldy", c_ll), ("part", c_void_p),
        ("conv_cin", c_int), ("conv_tin", c_int), ("conv_tout", c_int), ("conv_stride", c_int),
        ("zeros", c_void_p), ("layout", c_int),
    ]


class GemmSkParams(ctypes.Structure):
    """Mirror of ``GemmSkParams`` in csrc/kernels/gemm_sk.hip."""
    _fields_ = [
        ("x", c_void_p), ("ldx", c_ll), ("w", c_void_p),
        ("M", c_int), ("N", c_int), ("K", c_int), ("S", c_int),
        ("epi", c_int), ("act", c_int), ("bias", c_void_p),
        ("y", c_void_p), ("ldy", c_ll),
        ("ws", c_void_p), ("counters", c_void_p), ("layout", c_int),
    ]


class GemmWsParams(ctypes.Structure):
    """Mirror of ``GemmWsParams`` in csrc/kernels/gemm_ws.hip."""
    _fields_ = [
        ("x", c_void_p), ("ldx", c_ll), ("w", c_void_p),
        ("M", c_int), ("N", c_int), ("K", c_int),
        ("epi", c_int), ("act", c_int), ("bias", c_void_p),
        ("y", c_void_p), ("ldy", c_ll), ("bm", c_int),
        ("S", c_int), ("ws", c_void_p), ("counters", c_void_p),
    ]


_KERNEL_SIGS = {
    "loqa_rmsnorm": [c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_float, c_void_p,
                     c_void_p],
    "loqa_layernorm": [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_float,
                       c_void_p, c_void_p],
    "loqa_silu_mul": [c_void_p, c_void_p, c_ll, c_int, c_void_p],
    "loqa_gelu_bias": [c_void_p, c_void_p, c_void_p, c_ll, c_int, c_int, c_void_p],
    "loqa_rope_kv_append": [c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                            c_int, c_int, c_int, c_int, c_int, c_void_p],
    "loqa_pcm16_f32_sumsq": [c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_ll, c_void_p],
    "loqa_pcm16_f32_pad": [c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_ll, c_void_p],
    "loqa_masked_argmax": [c_void_p, c_int, c_ll, c_int, c_int, c_void_p, c_void_p, c_int,
                           c_void_p, c_void_p, c_void_p],  # (..., out_idx, workspace, stream)
    "loqa_attention": [c_void_p, c_ll, c_void_p, c_void_p, c_ll, c_void_p, c_ll, c_void_p,
                       c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_int, c_int,
                       c_int, c_float, c_int, c_int, c_int, c_int, c_void_p, c_void_p, c_int,
                       c_void_p],
    "loqa_log_mel": [c_void_p, c_int, c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_int,
                     c_void_p, c_void_p, c_void_p, c_int, c_void_p],
    "loqa_im2col_k3": [c_void_p, c_ll, c_ll, c_ll, c_int, c_int, c_int, c_int, c_void_p,
                       c_void_p],
    "loqa_skinny_gemm": [c_void_p, c_ll, c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_int,
                         c_void_p],
    "loqa_shuffle_weight": [c_void_p, c_void_p, c_int, c_int, c_void_p],
    "loqa_skinny_fused": [c_void_p, c_void_p],
    "loqa_gemm_tile": [c_void_p, c_void_p],
    "loqa_gemm_sk": [c_void_p, c_void_p],
    "loqa_gemm_sk_dims": [c_int, c_void_p, c_void_p],
    "loqa_gemm_ws": [c_void_p, c_int, c_void_p],
    "loqa_attn_decode": [c_void_p, c_ll, c_void_p, c_void_p, c_ll, c_void_p, c_void_p, c_ll,
                         c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_int, c_int,
                         c_int, c_float, c_int, c_int, c_int, c_void_p, c_void_p, c_int, c_void_p,
                         c_int, c_int, c_void_p],
    "loqa_slab_rmsnorm": [c_void_p, c_int, c_int, c_void_p, c_int, c_void_p, c_int, c_void_p,
                          c_void_p, c_int, c_float, c_void_p],
    "loqa_slab_rope_append": [c_void_p, c_int, c_int, c_int, c_void_p, c_void_p, c_void_p, c_void_p,
                              c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_void_p, c_void_p],
    "loqa_slab_layernorm": [c_void_p, c_int, c_int, c_void_p, c_int, c_void_p, c_void_p, c_int,
                            c_void_p, c_void_p, c_void_p, c_int, c_float, c_void_p],
    "loqa_slab_bias_act": [c_void_p, c_int, c_int, c_int, c_int, c_void_p, c_int, c_void_p,
                           c_void_p],
    "loqa_embed_pos": [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_void_p],
    "loqa_embed_stats": [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                         c_int, c_int, c_void_p],
    "loqa_conv1d": [c_void_p, c_ll, c_int, c_void_p, c_void_p, c_void_p, c_ll, c_int, c_void_p,
                    c_ll, c_int, c_void_p, c_ll, c_int, c_void_p, c_int, c_int, c_int, c_int, c_int,
                    c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_float, c_int,
                    c_float, c_int, c_int, c_void_p],
    "loqa_relpos_attention": [c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_int,
                              c_int, c_int, c_int, c_int, c_int, c_float, c_void_p],
    "loqa_expand_sample": [c_void_p, c_int, c_void_p, c_int, c_int, c_void_p, c_void_p, c_int,
                           c_int, c_float, ctypes.c_uint, c_void_p, c_void_p],
    "loqa_slab_silu_mul": [c_void_p, c_int, c_int, c_int, c_int, c_void_p, c_void_p],
    "loqa_slab_reduce": [c_void_p, c_int, c_int, c_int, c_int, c_void_p, c_void_p],
    "loqa_step_fetch": [c_void_p, c_void_p, c_int, c_int, c_void_p, c_void_p, c_int, c_int, c_void_p,
                        c_int, c_int, c_void_p, c_void_p],
    "loqa_gemm_prefill2": [c_void_p, c_int, c_int, c_void_p, c_int, c_int, c_void_p, c_void_p, c_int,
                           c_int, c_void_p],
    "loqa_init_uniform4": [c_void_p, c_ll, c_int, c_ll, c_ll, c_ll, ctypes.c_uint, c_float, c_void_p],
    "loqa_step_publish": [c_void_p, c_int, c_void_p, c_int, c_int, c_void_p, c_void_p, c_void_p,
                          c_void_p],
}

# (argtypes, restype) of the custom all-reduce entry points (in the kernels library)
_CAR_SIGS = {
    "loqa_car_create": ([c_int, c_int, c_ll, c_ll], c_void_p),
    "loqa_car_inbuf": ([c_void_p, c_int], c_void_p),
    "loqa_set_launch_prio": ([c_int], None),
    "loqa_car_resid": ([c_void_p, c_int, c_void_p, c_void_p, c_int, c_int, c_int, c_void_p], c_int),
    "loqa_car_argmax": ([c_void_p, c_void_p, c_ll, c_void_p, c_int, c_int, c_int, c_void_p, c_void_p],
                        c_int),
    "loqa_car_handle": ([c_void_p, c_void_p], c_int),
    "loqa_car_handle_size": ([], c_int),
    "loqa_car_open": ([c_void_p, c_void_p], c_int),
    "loqa_car_allreduce": ([c_void_p, c_void_p, c_void_p, c_ll, c_int, c_void_p], c_int),
    "loqa_car_error": ([c_void_p], c_int),
    "loqa_car_clear_error": ([c_void_p], c_int),
    "loqa_car_fill_inbuf": ([c_void_p, c_int, c_void_p, c_ll, c_void_p], c_int),
    "loqa_tp_emul_resid": ([c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_void_p], c_int),
    "loqa_car_destroy": ([c_void_p], None),
}

_RUNTIME_SIGS = {
    "loqa_stager_create": ([c_int, c_ll, c_int], c_void_p),
    "loqa_stager_destroy": ([c_void_p], None),
    "loqa_stager_acquire": ([c_void_p], c_int),
    "loqa_stager_append": ([c_void_p, c_int, c_void_p, c_ll], c_ll),
    "loqa_stager_len": ([c_void_p, c_int], c_ll),
    "loqa_stager_host_ptr": ([c_void_p, c_int], c_void_p),
    "loqa_stager_upload": ([c_void_p, c_int, c_void_p, c_ll, c_void_p], c_int),
    "loqa_stager_release": ([c_void_p, c_int], None),
    "loqa_stager_set_stream": ([c_void_p, c_void_p, c_int], c_int),
    "loqa_stager_flush": ([c_void_p, c_int, c_ll], c_ll),
    "loqa_stager_flushed": ([c_void_p, c_int], c_ll),
    "loqa_memcpy_h2d_async": ([c_void_p, c_void_p, c_ll, c_void_p], c_int),
    "loqa_pool_create": ([c_int, c_int], c_void_p),
    "loqa_pool_destroy": ([c_void_p], None),
    "loqa_pool_debug_hash_mask": ([c_void_p, ctypes.c_ulonglong], None),
    "loqa_pool_free_blocks": ([c_void_p], c_int),
    "loqa_pool_add_seq": ([c_void_p, c_ll, c_void_p, c_int], c_ll),
    "loqa_pool_append": ([c_void_p, c_ll, c_int, c_void_p], c_int),
    "loqa_pool_cache_prefix": ([c_void_p, c_ll, c_void_p, c_int], c_int),
    "loqa_pool_block_table": ([c_void_p, c_ll, c_void_p, c_int], c_int),
    "loqa_pool_step_meta": ([c_void_p, c_int, c_void_p, c_void_p, c_int, c_int, c_int, c_void_p,
                             c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int], c_int),
    "loqa_pool_seq_len": ([c_void_p, c_ll], c_ll),
    "loqa_pool_free_seq": ([c_void_p, c_ll], c_int),
    "loqa_pool_truncate": ([c_void_p, c_ll, c_ll], c_int),
    "loqa_tpctl_open": ([ctypes.c_char_p, c_int, c_int, c_int, c_ll], c_void_p),
    "loqa_tpctl_unlink": ([c_void_p], None),
    "loqa_tpctl_publish": ([c_void_p, c_void_p, c_ll, c_int, c_ll], c_int),
    "loqa_tpctl_recv": ([c_void_p, c_void_p, c_ll, ctypes.POINTER(c_int), c_ll], c_ll),
    "loqa_tpctl_close": ([c_void_p], None),
    "loqa_tpctl_beat": ([c_void_p], None),
    "loqa_tpctl_beat_age": ([c_void_p, c_int], c_ll),
}


class NativeLibraryMissing(RuntimeError):
    pass


def _load(name: str) -> ctypes.CDLL:
    path = os.path.join(_NATIVE, name)
    if not os.path.exists(path):
        raise NativeLibraryMissing(
            f"{path} is missing: run `python -m loqa_hub_amd._native.build` (gfx950)")
    return ctypes.CDLL(path, mode=ctypes.RTLD_GLOBAL)


def kernels() -> ctypes.CDLL:
    global _kernels
    if _kernels is None:
        with _lock:
            if _kernels is None:
                lib = _load("libloqa_kernels.so")
                for fn, sig in _KERNEL_SIGS.items():
                    f = getattr(lib, fn)
                    f.argtypes = sig
                    f.restype = c_int
                for fn, (args, res) in _CAR_SIGS.items():
                    f = getattr(lib, fn)
                    f.argtypes = args
                    f.restype = res
                _kernels = lib
    return _kernels


def runtime() -> ctypes.CDLL:
    global _runtime
    if _runtime is None:
        with _lock:
            if _runtime is None:
                lib = _load("libloqa_runtime.so")
                for fn, (args, res) in _RUNTIME_SIGS.items():
                    f = getattr(lib, fn)
                    f.argtypes = args
                    f.restype = res
                _runtime = lib
    return _runtime


def available() -> bool:
    try:
        kernels()
        return True
    except (NativeLibraryMissing, OSError):
        return False


def check(rc: int, what: str) -> None:
    if rc != 0:
        raise RuntimeError(f"{what} failed with hipError {rc}")


def stream_ptr(t: torch.Tensor) -> int:
    return torch.cuda.current_stream(t.device).cuda_stream


def ptr(t: torch.Tensor | None) -> int | None:
    return None if t is None else t.data_ptr()
