"""ctypes binding of libavsr_hip.so (the C-ABI declared in include/avsr_hip.h).

The product path has no fallback: if the library is missing or fails to load, every op
raises. `torch` is imported first so that the HIP runtime torch ships (same SONAME
libamdhip64.so.7) is the one the library binds to — one runtime per process.
"""
import ctypes
import os

import torch  # noqa: F401  (must precede the library load: shared HIP runtime)

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("AVSR_LIB_PATH_AB") or os.path.join(_HERE, "libavsr_hip.so")   # override: A/B tools only

AVSR_F32, AVSR_BF16 = 0, 1
ACT_NONE, ACT_GELU, ACT_RELU = 0, 1, 2

_c_p = ctypes.c_void_p
_i64 = ctypes.c_int64
_f = ctypes.c_float
_i = ctypes.c_int


class GemmParams(ctypes.Structure):
    _fields_ = [
        ("M", _i), ("N", _i), ("K", _i), ("batch", _i),
        ("dtype", _i), ("a_kmajor", _i), ("b_kmajor", _i), ("c_f32", _i),
        ("A", _c_p), ("lda", _i64), ("strideA", _i64),
        ("B", _c_p), ("ldb", _i64), ("strideB", _i64),
        ("C", _c_p), ("ldc", _i64), ("strideC", _i64),
        ("alpha", _f), ("beta", _f),
        ("bias", _c_p),
        ("act", _i), ("epi_bwd", _i),
        ("preact", _c_p),
        ("res", _c_p), ("ldr", _i64), ("strideR", _i64),
        ("gate", _c_p),
        ("drop_p", _f),
        ("seed", ctypes.c_uint64),
        ("splitk", _i),
        ("ws", _c_p),
        ("db", _c_p),
        ("db_ws", _c_p),
        ("stamp", _c_p),
        ("skinny_ws", _c_p), ("ln_c1", _c_p), ("ln_eps", ctypes.c_float),
        ("kv_k", _c_p), ("kv_v", _c_p), ("kv_pos", _c_p), ("kv_rows", _i),
        ("slab_cnt", _c_p),
    ]


class ConvParams(ctypes.Structure):
    _fields_ = [
        ("dtype", _i),
        ("nimg", _i), ("hin", _i), ("win", _i), ("cin", _i),
        ("hout", _i), ("wout", _i), ("cout", _i),
        ("kh", _i), ("kw", _i), ("sh", _i), ("sw", _i), ("ph", _i), ("pw", _i),
        ("groups", _i),
        ("ldx", _i64), ("ldy", _i64),
        ("x", _c_p), ("w", _c_p), ("y", _c_p),
        ("dx", _c_p), ("dy", _c_p), ("dw", _c_p),
        ("stats", _c_p),
        ("alpha", _f), ("beta", _f),
        ("splitk", _i),
        ("bias", _c_p), ("act", _i), ("preact", _c_p), ("res", _c_p),
        ("ws", _c_p),
        ("bnr_h", _c_p), ("bnr_res", _c_p), ("bnr_scale", _c_p), ("bnr_shift", _c_p), ("bnr_prelu", _c_p),
        ("bnr_mean", _c_p), ("bnr_invstd", _c_p), ("bnr_scale2", _c_p), ("bnr_shift2", _c_p),
        ("bnr_mean2", _c_p), ("bnr_invstd2", _c_p), ("bnr_ws", _c_p),
    ]


class LayerNormParams(ctypes.Structure):
    _fields_ = [
        ("dtype", _i), ("rows", _i), ("N", _i), ("eps", _f),
        ("x", _c_p), ("ldx", _i64), ("y", _c_p), ("ldy", _i64),
        ("gamma", _c_p), ("beta", _c_p), ("mean", _c_p), ("rstd", _c_p),
        ("dy", _c_p), ("lddy", _i64), ("dx", _c_p), ("lddx", _i64),
        ("dres", _c_p), ("lddres", _i64), ("dgamma", _c_p), ("dbeta", _c_p), ("ws", _c_p),
        ("g", _c_p), ("ldg", _i64), ("drop_p", _f), ("seed", ctypes.c_uint64), ("db", _c_p),
    ]


class BnFinalizeParams(ctypes.Structure):
    _fields_ = [
        ("tiles", _i), ("C", _i), ("partials", _c_p), ("gamma", _c_p), ("beta", _c_p),
        ("running_mean", _c_p), ("running_var", _c_p), ("momentum", _f), ("eps", _f),
        ("training", _i), ("mean", _c_p), ("invstd", _c_p), ("scale", _c_p), ("shift", _c_p),
    ]


class BnActParams(ctypes.Structure):
    _fields_ = [
        ("dtype", _i), ("M", _i), ("C", _i),
        ("h", _c_p), ("scale", _c_p), ("shift", _c_p), ("res", _c_p), ("scale2", _c_p), ("shift2", _c_p),
        ("prelu", _c_p), ("y", _c_p), ("dy", _c_p), ("dz", _c_p),
        ("mean", _c_p), ("invstd", _c_p), ("mean2", _c_p), ("invstd2", _c_p),
        ("sums", _c_p), ("dprelu", _c_p), ("dgamma", _c_p), ("dbeta", _c_p), ("dgamma2", _c_p), ("dbeta2", _c_p),
        ("dh", _c_p), ("dh2", _c_p), ("beta_acc", _f), ("ws", _c_p),
    ]


class StemPoolParams(ctypes.Structure):
    _fields_ = [
        ("dtype", _i), ("nimg", _i), ("H", _i), ("W", _i), ("C", _i), ("Ho", _i), ("Wo", _i),
        ("h", _c_p), ("scale", _c_p), ("shift", _c_p), ("prelu", _c_p), ("y", _c_p), ("argmax", _c_p),
        ("dy", _c_p), ("dz", _c_p), ("mean", _c_p), ("invstd", _c_p),
        ("sums", _c_p), ("dprelu", _c_p), ("dgamma", _c_p), ("dbeta", _c_p), ("ws", _c_p),
        ("hmax", _c_p), ("dh", _c_p), ("m_total", _i64),
    ]


class AttnParams(ctypes.Structure):
    _fields_ = [
        ("dtype", _i), ("B", _i), ("H", _i), ("Lq", _i), ("Lk", _i), ("scale", _f),
        ("q", _c_p), ("ldq", _i64), ("k", _c_p), ("ldk", _i64), ("v", _c_p), ("ldv", _i64),
        ("o", _c_p), ("ldo", _i64), ("lse", _c_p), ("klen", _c_p), ("causal", _i),
        ("drop_p", _f), ("seed", ctypes.c_uint64),
        ("dout", _c_p), ("lddo", _i64), ("delta", _c_p), ("dq", _c_p), ("lddq", _i64),
        ("dk", _c_p), ("lddk", _i64), ("dv", _c_p), ("lddv", _i64), ("dq_out", _c_p), ("lddq_out", _i64),
        ("db", _c_p), ("db_ws", _c_p), ("drop_mask", _c_p),
    ]


class XentParams(ctypes.Structure):
    _fields_ = [
        ("dtype", _i), ("rows", _i), ("V", _i), ("x", _c_p), ("ldx", _i64), ("target", _c_p),
        ("smoothing", _f), ("lse", _c_p), ("row_loss", _c_p), ("row_correct", _c_p),
        ("dloss", _c_p), ("coef", _f), ("dx", _c_p), ("lddx", _i64),
    ]


class CtcParams(ctypes.Structure):
    _fields_ = [
        ("dtype", _i), ("B", _i), ("T", _i), ("V", _i), ("Lmax", _i), ("x", _c_p), ("ldx", _i64),
        ("lse", _c_p), ("labels", _c_p), ("label_len", _c_p), ("in_len", _c_p),
        ("alpha", _c_p), ("gamma", _c_p), ("nll", _c_p), ("dloss", _c_p), ("coef", _f),
        ("dx", _c_p), ("lddx", _i64),
    ]


class EwParams(ctypes.Structure):
    _fields_ = [
        ("dtype", _i), ("rows", _i), ("N", _i), ("dy", _c_p), ("lddy", _i64), ("out", _c_p), ("ldout", _i64),
        ("gate", _c_p), ("ldgate", _i64), ("act", _i), ("drop_p", _f), ("seed", ctypes.c_uint64),
        ("alpha", _f), ("db", _c_p), ("ws", _c_p),
    ]


class EmbedParams(ctypes.Structure):
    _fields_ = [
        ("dtype", _i), ("rows", _i), ("L", _i), ("D", _i), ("tok", _c_p), ("table", _c_p), ("pe", _c_p),
        ("scale", _f), ("y", _c_p), ("drop_p", _f), ("seed", ctypes.c_uint64), ("dy", _c_p), ("dtable", _c_p),
        ("pe_row", _c_p),
    ]


class AdamWParams(ctypes.Structure):
    _fields_ = [
        ("n", _i64), ("param", _c_p), ("grad", _c_p), ("exp_avg", _c_p), ("exp_avg_sq", _c_p),
        ("shadow", _c_p), ("shadow_dtype", _i), ("lr", _f), ("beta1", _f), ("beta2", _f), ("eps", _f),
        ("weight_decay", _f), ("bias_corr1", _f), ("bias_corr2", _f), ("sumsq", _c_p), ("max_norm", _f),
        ("grad_scale", _f), ("max_blocks", _i), ("grad_clear", _c_p),
    ]


def fill(struct_cls, **kw):
    """Build a params struct; torch tensors become raw device pointers, None -> NULL."""
    p = struct_cls()
    keep = []
    for k, v in kw.items():
        if v is None:
            continue
        if isinstance(v, torch.Tensor):
            keep.append(v)          # the struct owns a reference: no use-after-free of temporaries
            v = v.data_ptr()
        setattr(p, k, v)
    p._keep = keep
    return p


# (symbol name, params struct or None for custom signature)
class DecAttnParams(ctypes.Structure):
    _fields_ = [
        ("dtype", _i), ("n", _i), ("H", _i), ("klen_max", _i), ("scale", _f),
        ("q", _c_p), ("ldq", _i64), ("k", _c_p), ("ldk", _i64), ("k_bstride", _i64),
        ("v", _c_p), ("ldv", _i64), ("v_bstride", _i64), ("klen", _c_p), ("o", _c_p), ("ldo", _i64),
        ("kidx", _c_p), ("kmap", _c_p), ("ldmap", _i64), ("group", _i), ("ksplit", _i), ("ws", _c_p),
        ("cnt", _c_p),
    ]


class TopkParams(ctypes.Structure):
    _fields_ = [("rows", _i), ("V", _i), ("K", _i), ("x", _c_p), ("ldx", _i64), ("ids", _c_p)]


class CtcPrefixParams(ctypes.Structure):
    _fields_ = [
        ("n", _i), ("T", _i), ("V", _i), ("P", _i), ("blank", _i), ("eos", _i), ("out_len", _i),
        ("logp", _c_p), ("r_prev", _c_p), ("last", _c_p), ("ids", _c_p), ("r_new", _c_p), ("psi", _c_p),
        ("uidx", _c_p), ("logp_ustride", _i64), ("tlen", _c_p), ("out_len_dev", _c_p),
    ]


class BeamSelectParams(ctypes.Structure):
    _fields_ = [
        ("n", _i), ("V", _i), ("P", _i), ("beam", _i), ("blank", _i), ("eos", _i), ("w_dec", _f), ("w_ctc", _f),
        ("dec", _c_p), ("ld", _i64), ("ids", _c_p), ("psi", _c_p), ("s_prev", _c_p), ("score", _c_p),
        ("out_prev", _c_p), ("out_tok", _c_p), ("out_col", _c_p), ("out_score", _c_p), ("out_dec", _c_p),
        ("out_ctc", _c_p), ("out_s", _c_p), ("nseg", _i), ("seg", _c_p),
    ]


class BeamPostParams(ctypes.Structure):
    _fields_ = [
        ("U", _i), ("beam", _i), ("P", _i), ("R", _i), ("Lmax", _i), ("steps_cap", _i), ("eos", _i),
        ("end_detect", _i), ("d_end", ctypes.c_double), ("pos", _c_p), ("maxlen", _c_p),
        ("sel_prev", _c_p), ("sel_tok", _c_p), ("sel_col", _c_p), ("sel_score", _c_p), ("sel_dec", _c_p),
        ("sel_ctc", _c_p), ("sel_s", _c_p),
        ("tok", _c_p), ("score", _c_p), ("sdec", _c_p), ("sctc", _c_p), ("s_prev", _c_p), ("src", _c_p),
        ("bp_prev", _c_p), ("bp_tok", _c_p), ("end_flag", _c_p), ("end_score", _c_p), ("end_dec", _c_p),
        ("end_ctc", _c_p), ("best_len", _c_p), ("best_end", _c_p), ("done", _c_p),
    ]


class FbankParams(ctypes.Structure):
    _fields_ = [
        ("B", _i), ("T", _i), ("wav", _c_p), ("ldw", _i64), ("n_samples", _c_p),
        ("bins", _i * 28), ("preemph", _f), ("ln_eps", _f), ("out", _c_p),
    ]


class TimeMaskParams(ctypes.Structure):
    _fields_ = [("B", _i), ("L", _i), ("nspan", _i), ("row_bytes", _i64), ("clip_stride_bytes", _i64),
                ("x", _c_p), ("spans", _c_p)]


class AddNoiseParams(ctypes.Structure):
    _fields_ = [("B", _i), ("L", _i), ("x", _c_p), ("ldx", _i64), ("noise", _c_p), ("ldn", _i64),
                ("lengths", _c_p), ("snr_db", _c_p), ("y", _c_p), ("ldy", _i64), ("ws", _c_p)]


class VideoNormParams(ctypes.Structure):
    _fields_ = [
        ("B", _i), ("T", _i), ("H", _i), ("W", _i), ("crop", _i), ("oy", _i), ("ox", _i),
        ("frames", _c_p), ("mean", _f), ("std", _f), ("out", _c_p),
    ]


SYMBOLS = {
    "avsr_version": ([], ctypes.c_char_p),
    "avsr_set_option": ([_i, _i64], _i),
    "avsr_get_option": ([_i], _i64),
    "avsr_gemm": ([ctypes.POINTER(GemmParams), _c_p], _i),
    "avsr_gemm_wgrad_group": ([ctypes.POINTER(GemmParams), _i, _c_p], _i),
    "avsr_gemm_skinny_splits": ([_i, _i, _i], _i),
    "avsr_conv_fwd": ([ctypes.POINTER(ConvParams), _c_p], _i),
    "avsr_conv_bwd_data": ([ctypes.POINTER(ConvParams), _c_p], _i),
    "avsr_conv_bwd_weight": ([ctypes.POINTER(ConvParams), _c_p], _i),
    "avsr_conv_stat_tiles": ([ctypes.POINTER(ConvParams)], _i),
    "avsr_conv_bnr_tiles": ([ctypes.POINTER(ConvParams)], _i),
    "avsr_conv_wgrad_ws": ([ctypes.POINTER(ConvParams)], _i64),
    "avsr_layernorm_fwd": ([ctypes.POINTER(LayerNormParams), _c_p], _i),
    "avsr_layernorm_bwd": ([ctypes.POINTER(LayerNormParams), _c_p], _i),
    "avsr_bn_finalize": ([ctypes.POINTER(BnFinalizeParams), _c_p], _i),
    "avsr_bn_act_fwd": ([ctypes.POINTER(BnActParams), _c_p], _i),
    "avsr_bn_act_bwd_reduce": ([ctypes.POINTER(BnActParams), _c_p], _i),
    "avsr_bn_bwd_apply": ([ctypes.POINTER(BnActParams), _c_p], _i),
    "avsr_stem_pool_fwd": ([ctypes.POINTER(StemPoolParams), _c_p], _i),
    "avsr_stem_pool_bwd_apply": ([ctypes.POINTER(StemPoolParams), _c_p], _i),
    "avsr_bn_bwd_finalize": ([ctypes.POINTER(BnActParams), _i, _c_p], _i),
    "avsr_avgpool_fwd": ([_i, _i, _i, _i, _c_p, _c_p, _c_p], _i),
    "avsr_avgpool_bwd": ([_i, _i, _i, _i, _c_p, _c_p, _c_p], _i),
    "avsr_attn_fwd": ([ctypes.POINTER(AttnParams), _c_p], _i),
    "avsr_debug_attn_stamps": ([_c_p], _i),
    "avsr_attn_bwd_prep": ([ctypes.POINTER(AttnParams), _c_p], _i),
    "avsr_attn_bwd": ([ctypes.POINTER(AttnParams), _c_p], _i),
    "avsr_attn_dropmask": ([ctypes.POINTER(AttnParams), _c_p], _i),
    "avsr_row_lse": ([ctypes.POINTER(XentParams), _c_p], _i),
    "avsr_lsm_fwd": ([ctypes.POINTER(XentParams), _c_p], _i),
    "avsr_lsm_bwd": ([ctypes.POINTER(XentParams), _c_p], _i),
    "avsr_ctc_fwd": ([ctypes.POINTER(CtcParams), _c_p], _i),
    "avsr_ctc_bwd": ([ctypes.POINTER(CtcParams), _c_p], _i),
    "avsr_loss_finalize": ([_i, _c_p, _i, _c_p, _c_p, _f, _i, _c_p, _c_p], _i),
    "avsr_ew_bwd": ([ctypes.POINTER(EwParams), _c_p], _i),
    "avsr_colsum_defer": ([_i], _i),
    "avsr_colsum_flush": ([_c_p], _i),
    "avsr_colsum_inline": ([_i], _i),
    "avsr_dropout_fwd": ([ctypes.POINTER(EwParams), _c_p], _i),
    "avsr_mask_rows": ([_i, _i, _i, _i, _c_p, _i64, _c_p, _c_p], _i),
    "avsr_embed_fwd": ([ctypes.POINTER(EmbedParams), _c_p], _i),
    "avsr_embed_bwd": ([ctypes.POINTER(EmbedParams), _c_p], _i),
    "avsr_cast": ([_i, _i, _i, _i, _c_p, _i64, _c_p, _i64, _f, _f, _c_p], _i),
    "avsr_cast_flat": ([_i, _i, _i64, _c_p, _c_p, _c_p], _i),
    "avsr_stem_pack": ([_i, _i, _i, _c_p, _c_p, _c_p], _i),
    "avsr_stem_wpack": ([_i, _c_p, _c_p, _c_p], _i),
    "avsr_stem_conv_tiles": ([_i, _i], _i),
    "avsr_stem_wpack2": ([_c_p, _c_p, _c_p], _i),
    "avsr_stem_conv_fwd": ([_i, _i, _c_p, _c_p, _c_p, _c_p, _c_p], _i),
    "avsr_stem_wgrad_unpack": ([_c_p, _c_p, _c_p], _i),
    "avsr_audio_pack": ([_i, _i, _i, _i, _c_p, _c_p, _c_p], _i),
    "avsr_weightnorm_fwd": ([_i, _i, _i, _i, _c_p, _c_p, _c_p, _c_p, _c_p], _i),
    "avsr_weightnorm_bwd": ([_i, _i, _i, _c_p, _c_p, _c_p, _c_p, _c_p, _c_p, _c_p, _c_p], _i),
    "avsr_sumsq": ([_c_p, _i64, _c_p, _c_p, _c_p], _i),
    "avsr_adamw": ([ctypes.POINTER(AdamWParams), _c_p], _i),
    "avsr_log_softmax_rows": ([_i, _i, _i, _c_p, _i64, _c_p, _i64, _c_p], _i),
    "avsr_dec_attn": ([ctypes.POINTER(DecAttnParams), _c_p], _i),
    "avsr_row_topk": ([ctypes.POINTER(TopkParams), _c_p], _i),
    "avsr_log_softmax_topk": ([_i, _i, _i, _c_p, _i64, _c_p, _i64, _i, _c_p, _c_p], _i),
    "avsr_ctc_prefix": ([ctypes.POINTER(CtcPrefixParams), _c_p], _i),
    "avsr_beam_select": ([ctypes.POINTER(BeamSelectParams), _c_p], _i),
    "avsr_beam_step_prep": ([_i, _i, _c_p, _c_p, _c_p, _c_p], _i),
    "avsr_beam_kv_put": ([_i, _i, _i, _c_p, _i64, _c_p, _c_p, _c_p, _c_p], _i),
    "avsr_beam_post": ([ctypes.POINTER(BeamPostParams), _c_p], _i),
    "avsr_gather_rows": ([_i, _i, _i64, _c_p, _i64, _i64, _c_p, _i64, _i64, _c_p, _c_p], _i),
    "avsr_fbank_stack": ([ctypes.POINTER(FbankParams), _c_p], _i),
    "avsr_video_normalize": ([ctypes.POINTER(VideoNormParams), _c_p], _i),
    "avsr_time_mask": ([ctypes.POINTER(TimeMaskParams), _c_p], _i),
    "avsr_add_noise": ([ctypes.POINTER(AddNoiseParams), _c_p], _i),
    "avsr_rgb_to_gray": ([_c_p, _c_p, _i64, _c_p], _i),
}

_lib = None


class AvsrLibError(RuntimeError):
    pass


def load():
    """Load the library (raises AvsrLibError if it is missing: no fallback path)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise AvsrLibError(f"{LIB_PATH} not built: run `python -c 'import __graft_entry__ as g; g.build()'`")
    lib = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)
    for name, (argtypes, restype) in SYMBOLS.items():
        if os.environ.get("AVSR_LIB_PATH_AB") and not hasattr(lib, name):
            continue                # an older A/B build: entry points it predates stay unbound
        fn = getattr(lib, name)
        fn.argtypes = argtypes
        fn.restype = restype
    _lib = lib
    return lib


def check(rc, op):
    if rc != 0:
        raise AvsrLibError(f"{op} failed with code {rc}")


# kernel-selection options (avsr_hip.h AVSR_OPT_*, AVSR_TILE_*): A/B tools and variant tests
OPTIONS = {"gemm_tile": 0, "attn_sq_fwd": 1, "attn_sq_bwd": 2, "wgrad_dual": 3, "conv_192": 4, "conv_s2phase": 5,
           "conv_patch": 6, "conv_wpatch": 7, "stem_pool_2x2": 8,
           "stem_wpatch": 9}
TILES = ["128", "256", "256x128", "128x256", "128s3", "128s4", "128w8s3", "128w8s4", "pp", "96", "128x64", "192",
         "192x256", "192s3", "192w8", "192w8s3", "64", "192w8s4", "64s4"]


def set_option(name, value):
    """avsr_set_option by name; gemm_tile takes a tile name (TILES) or None / "auto"; returns
    the previous value"""
    if name == "gemm_tile" and not isinstance(value, int):
        value = 0 if value in (None, "auto") else TILES.index(value) + 1
    lib = load()
    prev = get_option(name)
    check(lib.avsr_set_option(OPTIONS[name], int(value)), f"avsr_set_option({name}, {value})")
    return prev


def get_option(name):
    return int(load().avsr_get_option(OPTIONS[name]))


_raw_stream = getattr(torch._C, "_cuda_getCurrentRawStream", None)
_get_device = getattr(torch._C, "_cuda_getDevice", None) or torch.cuda.current_device


def stream_ptr(device=None):
    """the current HIP stream of `device` (default: the current device) as a void pointer;
    the raw-stream query skips building a torch Stream object on every launch"""
    if _raw_stream is not None:
        idx = _get_device() if device is None else torch.device(device).index
        if idx is None:
            idx = _get_device()
        return ctypes.c_void_p(_raw_stream(idx))
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)
