"""ctypes binding of libtvq_hip.so (include/tvq.h).

The library is loaded after `import torch` so that its NEEDED libamdhip64.so.7
resolves to the HIP runtime torch already mapped (same soname): the kernels
share torch's device context and streams.  There is no fallback: if the
library is missing or no GPU is present, the first call raises.
"""
import ctypes
import os
import threading

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get(
    "TVQ_HIP_LIB", os.path.join(os.path.dirname(os.path.dirname(_HERE)), "lib", "libtvq_hip.so"))

P = ctypes.c_void_p
I64 = ctypes.c_int64
I32 = ctypes.c_int
F32 = ctypes.c_float

# name -> argtypes (stream last).  Kept in sync with include/tvq.h (a CPU test
# checks every declared symbol is exported and listed here).
SIGNATURES = {}
_lib = None
_lock = threading.Lock()


def sig(name, *argtypes, restype=I32):
    SIGNATURES[name] = (list(argtypes), restype)


CSRC = os.path.join(os.path.dirname(os.path.dirname(_HERE)), "csrc")


def source_hash():
    """The stamp csrc/Makefile compiles into the library (tvq_source_hash): sha1 of every
    csrc *.hip / *.h sorted by name, then include/tvq.h, first 16 hex digits."""
    import hashlib
    h = hashlib.sha1()
    names = sorted(n for n in os.listdir(CSRC) if n.endswith((".hip", ".h")))
    for n in names + [os.path.join("..", "..", "include", "tvq.h")]:
        with open(os.path.join(CSRC, n), "rb") as f:
            h.update(f.read())
    return h.hexdigest()[:16]


def built_hash(path=None):
    """tvq_source_hash() of the built library at `path` (None if missing or unstamped), read
    from the file's bytes (the literal "tvq_source_hash=<16 hex>" the Makefile compiles in):
    the library is not loaded, so a later ctypes.CDLL of a rebuilt file in this process is
    not handed a stale mapping, and the GPU is not initialised."""
    import re
    path = path or LIB_PATH
    if not os.path.exists(path):
        return None
    with open(path, "rb") as f:
        m = re.search(rb"tvq_source_hash=([0-9a-f]{16})", f.read())
    return m.group(1).decode() if m else None


sig("tvq_source_hash", restype=ctypes.c_char_p)
sig("tvq_build_extra", restype=ctypes.c_char_p)
sig("tvq_conv_bnstats_blocks", I64, I64, I64, I64, I64, I64, I64, I64, I64, restype=I64)
sig("tvq_conv2d_fwd_bnstats", P, I64, I64, I64, I64, P, P, I64, I64, I64, I64, I64, I64, P, P, P)
sig("tvq_bn_train_apply_part", P, I64, I64, I64, P, I64, P, P, P, P, P, F32, F32, P, P, P, P, P, P)
sig("tvq_ups_pack", P, I64, I64, P, P)
sig("tvq_ups_wscatter", P, I64, I64, P, I64, P)
sig("tvq_ups_combine", P, I64, I64, I64, I64, P, I64, P, P, P, P, F32, P, P, P)
sig("tvq_ups_sums", P, P, I64, I64, I64, I64, P, P, P)
sig("tvq_hfe_assemble", P, P, P, P, I64, I64, I64, P, P)
sig("tvq_hfe_assemble_bwd", P, I64, I64, I64, P, P, P, P)
sig("tvq_tied_logits_ce_workspace", I64, I64, restype=I64)
sig("tvq_tied_logits_ce", P, I64, I64, P, I64, P, I64, I64, P, P, P, P, P, P, P, P)
sig("tvq_scalar_ratio", P, P, P, P)
sig("tvq_counter_pool", I64, P, I64)
sig("tvq_counter_capture", I64)
sig("tvq_plan_trace", I64)
sig("tvq_plan_read", ctypes.c_char_p, I64, restype=I64)
sig("tvq_fill", P, I64, ctypes.c_float, P)
sig("tvq_fill2", P, ctypes.c_float, P, ctypes.c_float, P)
sig("tvq_fill_i64", P, I64, I64, P)
sig("tvq_add_i64", P, I64, P)
sig("tvq_sum4", P, P, P, P, P, P, I64, P)
# --- VQ codebook -----------------------------------------------------------
sig("tvq_vq_sqnorm", P, I64, I64, P, P)
sig("tvq_vq_assign_nblocks", I64, restype=I64)
sig("tvq_vq_assign", P, I64, I64, I64, I64, I64, I64, P, P, I64, I32, P, P, P, P, P)
sig("tvq_vq_stats_workspace", I64, I64, restype=I64)
sig("tvq_vq_stats", P, I64, I64, I64, I64, I64, I64, P, I64, P, P, P, P, P)
sig("tvq_vq_ema", P, P, I64, I64, F32, P, P, P)
sig("tvq_vq_finalize", P, P, I64, I64, F32, P, P, I64, P, P, I64, P, P)
sig("tvq_vq_backward", P, P, P, P, I64, I64, P, P)

U64 = ctypes.c_uint64
sig("tvq_vq_assign_svq", P, I64, I64, I64, I64, I64, I64, P, P, I64, I32, F32, P, P, U64, P, P, P,
    P, P)
sig("tvq_vq_assign_rows", P, I64, I64, I64, I64, I64, I64, P, P, I64, I32, F32, P, P, U64, P, P, P,
    P, P, P)
# --- STFT / iSTFT ------------------------------------------------------------
sig("tvq_stft_encode", P, I64, I64, I64, P, P, P, P, P, P)
sig("tvq_istft_decode", P, I64, I64, I64, I64, I64, P, P)
sig("tvq_istft_decode_bwd", P, I64, I64, I64, I64, I64, P, P)
# --- convolutions --------------------------------------------------------------
sig("tvq_conv_out_width", I64, I64, I64, I64)
sig("tvq_conv_config", I64)
sig("tvq_conv_workspace", I64, I64, I64, I64, I64, I64, I64, I64, I64, I64, restype=I64)
sig("tvq_conv2d_fwd", P, I64, I64, I64, I64, P, P, I64, I64, I64, I64, I64, P, P, F32, P, U64, P, P)
sig("tvq_convT2d_fwd", P, I64, I64, I64, I64, P, P, I64, I64, I64, I64, P, P, P, P)
sig("tvq_conv2d_fwd_bn_eval", P, I64, I64, I64, I64, P, P, I64, I64, I64, I64, I64, I64, P, P, P, P,
    F32, P, P, P, P)
sig("tvq_convT2d_fwd_bn_eval", P, I64, I64, I64, I64, P, P, I64, I64, I64, I64, P, P, P, P, F32, P,
    P, P, P)
sig("tvq_conv2d_dgrad", P, I64, I64, I64, I64, P, I64, I64, I64, I64, I64, P, I64, P, P)
sig("tvq_convT2d_dgrad", P, I64, I64, I64, I64, P, I64, I64, I64, I64, P, I64, P, P)
sig("tvq_conv2d_wgrad", P, I64, I64, I64, I64, P, I64, I64, I64, I64, I64, I64, P, P, I64, P, P)
sig("tvq_convT2d_wgrad", P, I64, I64, I64, I64, P, I64, I64, I64, I64, I64, P, I64, P, P)
sig("tvq_channel_sum_workspace", I64, I64, I64, restype=I64)
sig("tvq_channel_sum", P, I64, I64, I64, P, I64, P, P)
# --- BatchNorm / Snake / dropout -----------------------------------------------
sig("tvq_bn_workspace", I64, I64, I64, restype=I64)
sig("tvq_bn_train_fwd", P, I64, I64, I64, P, P, P, P, P, F32, F32, P, P, P, P, P, P, P)
sig("tvq_bn_eval_fwd", P, I64, I64, I64, P, P, P, P, F32, P, P, P, P)
sig("tvq_bn_bwd", P, P, I64, I64, I64, P, P, P, P, P, P, P, P, P, I64, P, P)
sig("tvq_snake_fwd", P, I64, I64, I64, P, P, P)
sig("tvq_snake_workspace", I64, I64, I64, restype=I64)
sig("tvq_snake_bwd", P, P, I64, I64, I64, P, P, P, P, I64, P, P)
sig("tvq_dropout_bwd", P, I64, F32, P, U64, P, P)
sig("tvq_resblock_workspace", I64, I64, I64, I64, restype=I64)
sig("tvq_resblock_saved_floats", I64, I64, I64, I64, restype=I64)
sig("tvq_resblock_train_fwd", P, I64, I64, I64, I64, P, P, P, P, P, P, P, P, F32, F32, P, P, P,
    F32, P, U64, P, P, P, P, P)
sig("tvq_resblock_eval_fwd", P, I64, I64, I64, I64, P, P, P, P, P, P, P, F32, P, P, P, P, P)
sig("tvq_resblock_bwd", P, P, P, I64, I64, I64, I64, P, P, P, P, P, P, F32, P, U64, P, P, P, P,
    P, P, P, P, P, I64, P, P)
sig("tvq_resblock_pair_supported", I64, I64, I64, I64, restype=ctypes.c_int)
sig("tvq_resblock_pair_train_fwd", P, I64, I64, I64, I64, P, P, P, P, P, P, F32, F32, F32, P, U64,
    U64, P, P, P, P, P, P, P, P, P)
sig("tvq_resblock_pair_bwd", P, P, I64, I64, I64, I64, P, P, P, P, P, F32, P, U64, U64, P, P, P, P,
    I64, P, P, P)
sig("tvq_resblock_proj_workspace", I64, I64, I64, I64, I64, restype=I64)
sig("tvq_resblock_proj_saved_floats", I64, I64, I64, I64, I64, restype=I64)
sig("tvq_resblock_proj_train_fwd", P, I64, I64, I64, I64, I64, P, P, P, P, P, P, P, P, F32, F32, P,
    P, P, P, P, F32, P, U64, P, P, P, P, P)
sig("tvq_resblock_proj_eval_fwd", P, I64, I64, I64, I64, I64, P, P, P, P, P, P, P, F32, P, P, P, P,
    P, P, P)
sig("tvq_resblock_proj_bwd", P, P, P, I64, I64, I64, I64, I64, P, P, P, P, P, P, P, F32, P, U64, P,
    P, P, P, P, P, P, P, P, P, P, I64, P, P)
sig("tvq_reduce_rows_workspace", I64, I64, restype=I64)
sig("tvq_reduce_rows", P, I64, I64, I64, P, I64, P, P)
# --- dense GEMM --------------------------------------------------------------
sig("tvq_gemm_workspace", I64, I64, I64, restype=I64)
sig("tvq_gemm", P, I64, I64, P, I64, I64, P, I64, I64, I64, I64, F32, P, P, I64, I64, I64, P, I64, P, P, P)
sig("tvq_wgrad_group_workspace", I64, P, P, P, restype=I64)
sig("tvq_wgrad_group", I64, P, P, P, P, P, P, P, P, P, I64, P, P)
sig("tvq_wgrad_group_bias", I64, P, P, P, P, P, P, P, P, P, P, I64, P, P)
# --- losses / optimizer --------------------------------------------------------
sig("tvq_loss_workspace", I64, restype=I64)
sig("tvq_loss_fwd", P, P, I64, I64, P, P, P)
sig("tvq_loss_bwd", P, P, I64, I64, P, P, P)
sig("tvq_adamw_chunk", restype=I64)
sig("tvq_adamw_gates", P, I64, P, P)
sig("tvq_adamw_begin", P, F32, P, P, I64, P)
sig("tvq_adamw", P, P, P, P, P, I64, P, P, P, F32, F32, F32, F32, P)
sig("tvq_adamw_zero", P, P, P, P, P, I64, P, P, P, F32, F32, F32, F32, I64, P)
sig("tvq_adamw2", P, P, P, P, P, P, P, P, P, P, P, P, P, P, P, I64, P)
sig("tvq_layer_drop", P, ctypes.c_uint64, F32, I64, P, P, I64, P)

# --- MaskGIT transformer ---------------------------------------------------------
sig("tvq_rmsnorm_fwd", P, I64, I64, P, F32, P, P, P)
sig("tvq_norm_bwd_workspace", I64, I64, restype=I64)
sig("tvq_rmsnorm_bwd", P, P, I64, I64, P, F32, P, P, P, P, I64, P, P)
sig("tvq_scale_by", P, I64, P, P, P)
sig("tvq_upsample_nearest_t", P, I64, I64, I64, I64, P, P)
sig("tvq_upsample_nearest_t_bwd", P, I64, I64, I64, I64, P, P)
sig("tvq_batch_colsum", P, I64, I64, I64, I64, I64, P, I64, I64, P)
sig("tvq_class_index", P, I64, F32, I64, P, U64, P, P, P)
sig("tvq_embed_assemble", P, P, I64, I64, I64, I64, P, I64, I64, I64, I64, P, I64, I64, P, P)
sig("tvq_embed_assemble_bwd", P, I64, I64, I64, I64, P, P, I64, I64, I64, P, I64, I64, I64, P, I64, P)
sig("tvq_layernorm_fwd", P, I64, I64, P, P, F32, P, P, P, P)
sig("tvq_layernorm_bwd", P, P, I64, I64, P, P, P, P, P, P, I64, P, P)
sig("tvq_attention_fwd", P, I64, P, I64, P, I64, P, I64, P, I64, I64, I64, I64, F32, F32, P, U64, P)
sig("tvq_attention_bwd", P, I64, P, I64, P, I64, P, I64, P, I64, P, I64, I64, I64, I64, F32, F32, P,
    U64, P, P, P, I64, P)
sig("tvq_embedding_fwd", P, I64, I64, P, P, I64, I64, F32, P, U64, P)
sig("tvq_embedding_bwd_workspace", I64, I64, restype=I64)
sig("tvq_embedding_bwd", P, I64, I64, P, I64, I64, P, I64, I64, F32, P, U64, P, P)
sig("tvq_masked_ce_workspace", I64, restype=I64)
sig("tvq_drop_first_token", P, I64, I64, I64, P, I64, P)
sig("tvq_masked_ce_fwd", P, I64, I64, I64, P, P, P, P, P, P)
sig("tvq_masked_ce_bwd", P, I64, I64, I64, P, P, P, P, P, P, I64, P)
sig("tvq_mask_tokens", P, I64, I64, I64, P, U64, P, P, P, P, P)
sig("tvq_upsample_nearest", P, I64, I64, I64, P, P)
sig("tvq_upsample_nearest_bwd", P, I64, I64, I64, P, P)
sig("tvq_gelu_fwd", P, I64, P, P)
sig("tvq_gelu_bwd", P, P, I64, P, P)
# --- MaskGIT sampling ------------------------------------------------------------
sig("tvq_prior_lf_eval_workspace", I64, I64, I64, I64, restype=I64)
sig("tvq_prior_lf_eval", P, I64, I64, I64, P, I64, I64, P, I64, I64, F32, P, P, P)
sig("tvq_ffn_fwd", P, P, I64, I64, P, P, P, P, P, F32, P, U64, P, P, P, P)
sig("tvq_ffn_bwd", P, P, I64, I64, P, P, P, F32, P, U64, P, P, P, P)
sig("tvq_attn_branch_workspace", I64, I64, restype=I64)
sig("tvq_attn_branch_fwd", P, I64, I64, I64, I64, P, F32, P, P, P, F32, P, U64, P, P, P, P, P, P, P)
sig("tvq_attn_branch_bwd", P, P, I64, I64, I64, I64, P, F32, P, P, P, P, F32, P, U64, P, P, P, P, P,
    P, P, I64, P, P)
sig("tvq_prior_lf_eval_sample", P, I64, I64, I64, P, I64, I64, P, I64, I64, F32, I64, P, P, U64,
    P, P, P, P, I64, P)
sig("tvq_maskgit_sample", P, I64, I64, I64, I64, I64, P, I64, P, P, U64, P, P, P)
sig("tvq_tied_logits_sample_workspace", I64, I64, I64, restype=I64)
sig("tvq_tied_logits_sample", P, I64, I64, P, I64, P, I64, I64, P, I64, P, P, U64, P, P, P, P, P)
sig("tvq_maskgit_remask", P, I64, I64, I64, F32, P, P, U64, P, I64, P, P, P)
sig("tvq_conv_packcache_begin", I64, P, I64, P)
sig("tvq_conv_packcache_end")
sig("tvq_conv_packcache_release", I64)
sig("tvq_conv_packcache_pause", I64)
sig("tvq_conv_packcache_entries", restype=I64)
sig("tvq_conv_wgrad_defer_begin")
sig("tvq_conv_wgrad_defer_flush", P)
sig("tvq_wgrad_defer_begin_stream", P)
sig("tvq_conv_wgrad_defer_pause", I64)
# --- ROCKET features --------------------------------------------------------
sig("tvq_rocket_apply", P, I64, I64, I64, P, P, P, P, P, P, I64, P, P)
# --- FidelityEnhancer (Unet1D eval forward) -----------------------------------
sig("tvq_fe_conv1d_out_len", I64, I64, I64, I64, I64, restype=I64)
sig("tvq_fe_ws_weight", P, I64, I64, F32, P, P)
sig("tvq_fe_conv1d", P, I64, I64, I64, P, P, I64, I64, I64, I64, I64, I64, P, P, I64, P)
sig("tvq_fe_group_norm_snake", P, I64, I64, I64, I64, P, P, P, F32, P, P, P)
sig("tvq_fe_channel_layernorm", P, I64, I64, I64, P, F32, P, P, P)
sig("tvq_fe_linear_attention", P, I64, I64, I64, I64, P, P)
sig("tvq_fe_linear_attention_fused", P, I64, I64, I64, P, I64, I64, P, P)
sig("tvq_fe_attention", P, I64, I64, I64, I64, P, P)
sig("tvq_fe_cat_interp", P, I64, I64, P, I64, I64, I64, I64, P, P)
sig("tvq_fe_ws_weight_bwd", P, I64, I64, F32, P, P, I64, P)
sig("tvq_fe_gn_snake_train_fwd", P, I64, I64, I64, I64, P, P, P, F32, F32, P, U64, P, P, P, P, P)
sig("tvq_fe_gn_snake_bwd", P, P, I64, I64, I64, I64, P, P, P, P, P, F32, P, U64, P, P, P, P, P)
sig("tvq_fe_channel_layernorm_bwd", P, P, I64, I64, I64, P, F32, P, P, P)
sig("tvq_fe_linear_attention_bwd", P, P, I64, I64, I64, I64, P, P)
sig("tvq_fe_attention_bwd", P, P, I64, I64, I64, I64, P, P)
sig("tvq_fe_cat_interp_bwd", P, I64, I64, I64, I64, I64, I64, P, P, P)
# --- trajectory data format (MinMax scaling + layout) -------------------------
F64 = ctypes.c_double
sig("tvq_minmax_fit_workspace", I64, restype=I64)
sig("tvq_minmax_fit", P, I64, I64, F64, F64, P, P, P, P, P, P)
sig("tvq_fid_moments", P, I64, I64, P, P, P)
sig("tvq_minmax_transform", P, I64, I64, I64, P, P, P, P)
sig("tvq_minmax_inverse", P, I64, I64, I64, P, P, P, P)
sig("tvq_codebook_gather_nchw", P, I64, I64, I64, P, P, P)


class NativeError(RuntimeError):
    pass


def lib():
    """Load libtvq_hip.so once; raise loudly if it is missing."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(LIB_PATH):
            raise NativeError(
                f"libtvq_hip.so not found at {LIB_PATH}; build it with "
                "`python -c 'import __graft_entry__ as g; g.build()'` (no CPU fallback exists)")
        h = ctypes.CDLL(LIB_PATH)
        h.tvq_last_error.restype = ctypes.c_char_p
        h.tvq_last_error.argtypes = []
        h.tvq_abi_version.restype = I32
        for name, (args, res) in SIGNATURES.items():
            fn = getattr(h, name)
            fn.argtypes = args
            fn.restype = res
        _lib = h
    return _lib


def stream_ptr():
    return torch.cuda.current_stream().cuda_stream


def ptr(t):
    """Device pointer of a tensor (None -> NULL).  Rejects CPU tensors loudly."""
    if t is None:
        return None
    if not t.is_cuda:
        raise NativeError("tvq HIP kernels need device tensors (got a CPU tensor); "
                          "the product path has no CPU fallback")
    return t.data_ptr()


POOL_SLOTS = 1 << 20
_pools = {}  # device index -> zeroed int32 counter pool registered with the library
_pool_dev = [-1]


def _ensure_pool(h):
    """Register this device's counter pool (tvq_counter_pool) on first use.  The first
    launch on a device is eager (warmup steps precede graph capture)."""
    dev = torch.cuda.current_device()
    if dev == _pool_dev[0]:
        return
    if dev not in _pools:
        pool = torch.zeros(POOL_SLOTS, dtype=torch.int32, device=dev)
        if not torch.cuda.is_current_stream_capturing():
            torch.cuda.synchronize(dev)  # zeroed before any stream's kernel takes a slot
        rc = h.tvq_counter_pool(dev, pool.data_ptr(), POOL_SLOTS)
        if rc != 0:
            raise NativeError(f"tvq_counter_pool failed: {h.tvq_last_error().decode()}")
        _pools[dev] = pool
    _pool_dev[0] = dev


def call(name, *args):
    """Call an int-returning entry point; raise with tvq_last_error() on failure."""
    h = lib()
    _ensure_pool(h)
    rc = getattr(h, name)(*args)
    if rc != 0:
        raise NativeError(f"{name} failed ({rc}): {h.tvq_last_error().decode()}")
    return rc


def value(name, *args):
    return getattr(lib(), name)(*args)


class plan_trace:
    """Record the kernel variants the library's host-side plans launch (tvq_plan_trace);
    `.lines` holds them after the block (tests confirm which kernel a shape took)."""

    def __enter__(self):
        lib().tvq_plan_trace(1)
        self.lines = []
        return self

    def __exit__(self, *exc):
        h = lib()
        n = h.tvq_plan_read(None, 0)
        buf = ctypes.create_string_buffer(int(n) + 1)
        h.tvq_plan_read(buf, n + 1)
        h.tvq_plan_trace(0)
        self.lines = [s for s in buf.value.decode().split("\n") if s]
        return False

    def has(self, prefix):
        return [s for s in self.lines if s.startswith(prefix)]


def grad_sink(p):
    """p.grad when FusedAdamW keeps it as a view of its flat gradient buffer: backward
    kernels then accumulate straight into it and the autograd Function returns None
    for p (no AccumulateGrad kernel).  None otherwise (standard autograd return)."""
    if p is None or not getattr(p, "_tvq_flat", False) or not p.requires_grad:
        return None
    g = p.grad
    if g is None or not g.is_contiguous():
        return None
    return g
