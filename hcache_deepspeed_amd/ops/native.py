"""ctypes bindings of the in-tree native libraries.

Every GPU op of the framework goes through here. On a machine with a GPU the kernel library is
REQUIRED: ``kernels()`` raises if it is missing instead of silently falling back to eager
PyTorch, so a test that passes on the GPU has run the HIP code. CPU tensors use the pure-torch
reference implementations inside each op module (that is what the CPU test-suite exercises).
"""
import ctypes
import os
import threading

import torch

from . import build as _build

_lock = threading.Lock()
_klib = None
_hlib = None

# argument spec letters: p=void*, i=int32, u=uint32, l=int64, f=float, s=hipStream_t
_KERNEL_SIGS = {
    "hds_norm_fwd": "iii" + "p" * 8 + "ii" + "f" + "s",
    "hds_norm_bwd_nparts": "i",
    "hds_norm_bwd_set_max_parts": "i",
    "hds_norm_bwd": "iii" + "p" * 9 + "i" + "pp" + "iii" + "s",
    "hds_rope": "ii" + "pppp" + "l" + "iii" + "l" + "ii" + "f" + "s",
    "hds_glu_fwd": "iipplis",
    "hds_glu_bwd": "iippplis",
    "hds_glu_fwd_t": "i" + "ppp" + "ii" + "s",
    "hds_glu_bwd_t": "i" + "pppp" + "ii" + "s",
    "hds_bias_act_fwd": "iippplis",
    "hds_bias_act_bwd": "iipppplis",
    "hds_adam_flat": "ii" + "ppppp" + "l" + "f" * 7 + "i" + "f" + "pp" + "s",
    "hds_multi_chunk_size": "",
    "hds_adam_multi": "ii" + "pp" + "i" + "f" * 7 + "i" + "f" + "pp" + "s",
    "hds_lion_flat": "ii" + "pppp" + "l" + "f" * 5 + "pp" + "s",
    "hds_adagrad_flat": "ii" + "pppp" + "l" + "f" * 4 + "pp" + "s",
    "hds_lamb_multi": "ii" + "pp" + "i" + "p" + "f" * 10 + "pp" + "s",
    "hds_sumsq": "iplpps",
    "hds_clip_coef": "pffpps",
    "hds_xent": "i" + "pppp" + "l" + "i" + "l" + "i" + "f" + "i" + "f" + "s",
    "hds_attn_fwd": "p" * 8 + "i" * 7 + "f" + "ii" + "s",
    "hds_attn_bwd": "p" * 13 + "i" * 7 + "f" + "ii" + "s",
    "hds_attn_head_dim_supported": "i",
    "hds_attn_config": "iii",
    "hds_attn_fwd_variant": "i",
    "hds_attn_bwd_dq_variant": "i",
    "hds_attn_w64_stamps": "pi",  # A/B library only (build_kernels_diag)
    "hds_attn_diag_build": "",
    "hds_attn_bwd_prio": "i",
    "hds_attn_bwd_pipe": "i",
    "hds_bsattn_fwd": "p" * 8 + "i" * 7 + "f" + "i" + "s",
    "hds_bsattn_bwd": "p" * 15 + "i" * 7 + "f" + "i" + "s",
    "hds_kv_rope_scatter": "i" + "p" + "l" + "pppp" + "i" + "pp" + "i" * 8 + "s",
    "hds_paged_attn": "p" + "l" + "ppp" + "i" + "pp" + "i" * 5 + "f" + "i" + "s",
    "hds_paged_rows_per_atom": "",
    "hds_moe_dispatch": "i" + "pppp" + "iiii" + "s",
    "hds_moe_dispatch_bwd": "i" + "pppp" + "iiii" + "s",
    "hds_moe_combine": "i" + "ppppp" + "iiii" + "s",
    "hds_moe_combine_bwd": "i" + "ppppppp" + "iiii" + "s",
    "hds_quant_int": "i" + "pppp" + "l" + "iii" + "s",
    "hds_dequant_int": "i" + "pppp" + "l" + "iii" + "s",
    "hds_quant_fp8": "i" + "ppp" + "l" + "ii" + "s",
    "hds_dequant_fp8": "i" + "ppp" + "l" + "ii" + "s",
    "hds_int_gemv": "pppp" + "iiiii" + "s",
    "hds_dequant_reduce": "i" + "ppp" + "i" + "l" + "iii" + "s",
    "hds_quant_minifloat": "i" + "ppp" + "l" + "iiiii" + "s",
    "hds_dequant_minifloat": "i" + "ppp" + "l" + "iii" + "s",
    "hds_fp6_gemv": "pppp" + "iiiiii" + "s",
    "hds_transpose_bf16": "pp" + "ii" + "l" + "s",
    "hds_transpose_bf16_var": "pp" + "ii" + "l" + "i" + "s",
    "hds_gemv_bf16_supported": "iii",
    "hds_gemv_bf16": "pppp" + "iii" + "ll" + "s",
    "hds_gemv_fused_bf16": "ppp" + "f" + "pppp" + "iiii" + "ll" + "s",
    "hds_skinny_gemm_bf16": "pppp" + "iii" + "ll" + "s",
    "hds_skinny_set_unroll": "i",
    "hds_wmix_splits": "iii",
    "hds_wmix_supported": "iiii",
    "hds_wmix_gemm": "pppppp" + "iiiiii" + "s",
    "hds_token_gather": "i" + "ppp" + "iiii" + "s",
    "hds_token_scatter": "i" + "ppp" + "iiii" + "s",
    "hds_token_sort": "p" + "ii" + "s",
    "hds_gemm_nt_supported": "iiiiii",
    "hds_gemm_nt": "ppp" + "iiiiii" + "f" + "ii" + "s",
    "hds_gemm_mxfp8_supported": "iiiiii",
    "hds_gemm_mxfp8": "ppppp" + "iiiiii" + "f" + "i" + "s",
    "hds_mx_quant": "ppp" + "l" + "i" + "l" + "s",
    "hds_kv_append": "p" + "ll" + "p" + "ll" + "p" + "lll" + "p" + "lll" + "p" + "iii" + "s",
    "hds_decode_attn_supported": "ii",
    "hds_decode_attn_splits": "iii",
    "hds_decode_attn": "p" + "ll" + "p" + "lll" + "p" + "lll" + "p" + "l" + "p" + "ppp" + "iiiiii" + "f" + "s",
    "hds_decode_attn_len": "p" + "ll" + "p" + "lll" + "p" + "lll" + "p" + "l" + "p" + "ppp" + "iiiiii" + "f" + "pi" + "s",
    "hds_evoformer_bwd": "p" * 10 + "pp" + "i" + "pp" + "iiiii" + "f" + "s",
    "hds_embed_bwd": "i" + "pppp" + "l" + "i" + "ll" + "s",
    "hds_slice_mask": "i" + "ppp" + "iiiii" + "s",
    "hds_grouped_gemm_max_tiles": "ii",
    "hds_grouped_gemm": "ppppp" + "iiiiii" + "s",
    "hds_evoformer_fwd": "ppppp" + "i" + "pp" + "iiiii" + "f" + "s",
    "hds_nhwc_bias_add": "i" + "ppppp" + "l" + "ii" + "s",
    "hds_paged_decode_supported": "ii",
    "hds_paged_decode_splits": "iii",
    "hds_paged_decode": "p" + "l" + "pppp" + "pp" + "iiiiiii" + "f" + "i" + "p" + "s",
    "hds_copy_d2h": "pp" + "l" + "i" + "s",
    "hds_latent_slot_store": "p" + "l" + "pp" + "l" + "i" + "l" + "s",
    "hds_slot_advance": "p" + "i" + "s",
    "hds_symm_header_bytes": "",
    "hds_symm_alloc": "lpp",
    "hds_symm_open": "pp",
    "hds_symm_close": "p",
    "hds_symm_free": "p",
    "hds_symm_error": "p",
    "hds_symm_status_alloc": "p",
    "hds_symm_status_free": "p",
    "hds_symm_clear_error": "p",
    "hds_symm_allreduce": "p" + "ii" + "l" + "u" + "pp" + "l" + "i" + "pp" + "s",
    "hds_symm_allgather": "p" + "ii" + "l" + "u" + "pp" + "l" + "pp" + "s",
    "hds_symm_reduce_scatter": "p" + "ii" + "l" + "u" + "pp" + "l" + "i" + "pp" + "s",
}

_CT = {"p": ctypes.c_void_p, "i": ctypes.c_int, "u": ctypes.c_uint32, "l": ctypes.c_int64, "f": ctypes.c_float, "s": ctypes.c_void_p}


def _bind(lib, sigs):
    for name, spec in sigs.items():
        fn = getattr(lib, name, None)
        if fn is None:
            continue
        fn.argtypes = [_CT[c] for c in spec]
        fn.restype = ctypes.c_int


def _gpu_present():
    try:
        return torch.cuda.is_available()
    except Exception:  # pragma: no cover
        return False


def kernel_lib_path():
    return _build.KERNEL_LIB


def load_kernels(build_if_missing=True):
    """Load (building first if needed) the HIP kernel library. Returns None when unavailable."""
    global _klib
    if _klib is not None:
        return _klib
    with _lock:
        if _klib is not None:
            return _klib
        path = os.environ.get("HDS_KERNEL_LIB") or _build.KERNEL_LIB  # override: an A/B build (ops/build.py)
        if build_if_missing and os.environ.get("HDS_NO_BUILD", "0") != "1" and not os.environ.get("HDS_KERNEL_LIB"):
            try:
                path = _build.build_kernels()
            except Exception:
                if not os.path.exists(path):
                    raise
        if not os.path.exists(path):
            return None
        lib = ctypes.CDLL(path, mode=ctypes.RTLD_GLOBAL)
        _bind(lib, _KERNEL_SIGS)
        # FlashAttention backward with LDS reads pipelined two MFMAs ahead (csrc/kernels/flash_attn.hip PIPE; 2 = + uniform-
        # base LDS-DMA staging of full tiles: 3.80 vs 3.85 ms, profiles/r3/fa_bwd_pipe2_r3q.txt)
        lib.hds_attn_bwd_pipe(int(os.environ.get("HDS_ATTN_BWD_PIPE", "2")))
        # FlashAttention forward variant (csrc/kernels/flash_attn.hip hds_attn_fwd_variant): 11 = one wave per SIMD,
        # 64 rows per wave, hand-scheduled MFMA blocks (flash_attn_w64.hip; 1.074-1.077 ms vs 1.109-1.116 for the
        # 8-wave software-pipelined variant 5 at the bench shape, profiles/r5/fa_fwd_variants_idle_tiles_r5w.log)
        check(lib.hds_attn_fwd_variant(fwd_variant_default()), "hds_attn_fwd_variant")
        # FlashAttention backward dQ kernel (hds_attn_bwd_dq_variant; 1 = one wave per SIMD, 64 rows per wave)
        lib.hds_attn_bwd_dq_variant(int(os.environ.get("HDS_ATTN_DQ_VAR", "0")))
        # skinny GEMM weight loads in flight per lane (16: B = 4 decode 925 vs 881 tok/s with 8, profiles/r6/skinny_u)
        lib.hds_skinny_set_unroll(int(os.environ.get("HDS_SKINNY_U", "16")))
        _klib = lib
        return _klib


# FlashAttention forward variants of the shipped library (flash_attn.hip hds_attn_fwd_variant): 20 the default, 5 the
# 8-wave fallback, 2 the generic 8-wave kernel. The experiment / diagnostic variants exist only in the A/B library
# (ops/build.py build_kernels_diag, loaded through HDS_KERNEL_LIB), where HDS_ATTN_FWD_VAR may name them.
SHIPPED_FWD_VARIANTS = (2, 5, 20)


def fwd_variant_default():
    """The FlashAttention forward variant the library is loaded with (``HDS_ATTN_FWD_VAR`` overrides; a variant the
    shipped library does not carry raises instead of silently running something else)."""
    var = int(os.environ.get("HDS_ATTN_FWD_VAR", "20"))
    diag = os.path.basename(os.environ.get("HDS_KERNEL_LIB", "")) == os.path.basename(_build.DIAG_LIB)
    if var not in SHIPPED_FWD_VARIANTS and not diag:
        raise ValueError(f"HDS_ATTN_FWD_VAR={var}: the shipped FlashAttention library has forward variants "
                         f"{SHIPPED_FWD_VARIANTS}; experiment / diagnostic variants need the A/B library "
                         f"(ops/build.py build_kernels_diag, HDS_KERNEL_LIB={_build.DIAG_LIB})")
    return var


def kernels():
    lib = load_kernels()
    if lib is None:
        raise RuntimeError("hcache_deepspeed_amd: native kernel library libhds_kernels.so is missing; "
                           "run `python -m hcache_deepspeed_amd.ops.build` (refusing to fall back to eager ops on GPU)")
    return lib


def host_lib():
    """Host-side C++ runtime (pinned rings, CPU optimizers, async file I/O)."""
    global _hlib
    if _hlib is not None:
        return _hlib
    with _lock:
        if _hlib is not None:
            return _hlib
        path = _build.HOST_LIB
        if os.environ.get("HDS_NO_BUILD", "0") != "1":
            try:
                path = _build.build_host() or path
            except Exception:
                if not os.path.exists(path):
                    raise
        if not os.path.exists(path):
            raise RuntimeError("hcache_deepspeed_amd: host library libhds_host.so is missing")
        from . import host_sigs
        lib = ctypes.CDLL(path, mode=ctypes.RTLD_GLOBAL)
        host_sigs.bind(lib)
        _hlib = lib
        return _hlib


_DT = {torch.float32: 0, torch.bfloat16: 1, torch.float16: 2}


def dt(t_or_dtype):
    d = t_or_dtype if isinstance(t_or_dtype, torch.dtype) else t_or_dtype.dtype
    if d not in _DT:
        raise TypeError(f"unsupported dtype {d}")
    return _DT[d]


def ptr(t):
    return None if t is None else t.data_ptr()


def stream(device=None):
    return torch.cuda.current_stream(device).cuda_stream


_DEBUG_SYNC = os.environ.get("HDS_DEBUG_SYNC", "0") == "1"


def check(err, what):
    """Raise on a launch error. With ``HDS_DEBUG_SYNC=1`` (race/fault debug mode, pair with
    ``AMD_SERIALIZE_KERNEL=3``) every native launch is followed by a device synchronize, so an asynchronous fault
    (illegal address, assert) is attributed to the kernel that caused it instead of a later unrelated call."""
    if err != 0:
        raise RuntimeError(f"hcache_deepspeed_amd: {what} failed with hipError {err}")
    if _DEBUG_SYNC and torch.cuda.is_available():
        try:
            torch.cuda.synchronize()
        except Exception as e:  # pragma: no cover - GPU fault path
            raise RuntimeError(f"hcache_deepspeed_amd: device fault after {what}: {e}") from e


def use_native(*tensors):
    """True when the tensors live on the GPU (native path mandatory there)."""
    for t in tensors:
        if t is not None and t.is_cuda:
            return True
    return False
