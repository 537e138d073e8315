"""ctypes binding of libsat_hip.so (the C ABI declared in include/sat_hip.h).

The product path has no fallback: if the library is missing, or a tensor is not
on a HIP device, every op raises.  ``torch`` is imported first so that the HIP
runtime torch ships (same SONAME as the one hipcc links) is the one the library
binds to.
"""
import ctypes
import os

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("SAT_HIP_LIB_TUNING") or os.path.join(_HERE, "libsat_hip.so")   # override: A/B builds only

SAT_F32, SAT_BF16 = 0, 1
IMG_NCHW, IMG_NHWC, IMG_S2D16 = 0, 1, 2
ACT_NONE, ACT_RELU, ACT_TANH, ACT_SIGMOID = 0, 1, 2, 3

c_int, c_int64, c_float, c_void_p, c_size_t, c_uint64 = (ctypes.c_int, ctypes.c_int64, ctypes.c_float,
                                                        ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint64)


class SatConvGeom(ctypes.Structure):
    _fields_ = [(n, c_int) for n in ("N", "H", "W", "C", "KH", "KW", "stride", "pad", "OH", "OW")]


ABI_VERSION = 9   # include/sat_hip.h SAT_ABI_VERSION: the library must match these structs


class SatPolicy(ctypes.Structure):
    """Per-call kernel selection (include/sat_hip.h SatPolicy); all zeros = the library's defaults."""
    _fields_ = [(n, c_int) for n in ("conv_pipe", "conv_stream", "conv3x3_ws", "conv_slices", "skinny", "gemm_stages",
                                     "gemm_tile", "gemm_linear_order", "gemm_epilogue", "split_gemm", "split_k",
                                     "attn_bwd", "attn_bwd_chunks", "attn_pipe")] + \
               [("decoder_splits", c_int * 4), ("greedy_step", c_int), ("embed_grad", c_int), ("stamps", c_void_p),
                ("stamp_capacity", c_int)]

    def __init__(self, **kw):
        splits = kw.pop("decoder_splits", None)
        super().__init__(**kw)
        if splits is not None:
            self.decoder_splits[:] = list(splits)


class SatGemmArgs(ctypes.Structure):
    _fields_ = [("M", c_int), ("N", c_int), ("K", c_int), ("dtype", c_int),
                ("A", c_void_p), ("lda", c_int64), ("transA", c_int),
                ("B", c_void_p), ("ldb", c_int64), ("transB", c_int),
                ("C", c_void_p), ("ldc", c_int64), ("c_dtype", c_int),
                ("alpha", c_float), ("beta", c_float),
                ("bias", c_void_p),
                ("add1", c_void_p), ("ld_add1", c_int64), ("add1_dtype", c_int),
                ("act", c_int),
                ("aux", c_void_p), ("ld_aux", c_int64), ("aux_dtype", c_int),
                ("policy", ctypes.POINTER(SatPolicy)),
                ("workspace", c_void_p), ("workspace_bytes", c_int64)]


class SatDecoderDims(ctypes.Structure):
    _fields_ = [("B", c_int), ("L", c_int), ("D", c_int), ("E", c_int), ("V", c_int), ("T", c_int),
                ("tf", c_int), ("ado", c_int), ("attention", c_int), ("bert", c_int), ("training", c_int),
                ("dtype", c_int), ("start_token", c_int), ("has_dropout_mask", c_int), ("seed", c_uint64),
                ("seed_ptr", c_void_p), ("split_target", c_int), ("policy", ctypes.POINTER(SatPolicy))]


LAYOUT_FIELDS = ("embedding", "init_w", "init_b", "hcat_w", "hcat_b", "attW_w", "attW_b", "v_w", "v_b", "wih",
                 "bih", "fh_w", "fh_b", "fz_w", "fz_b", "fout_w", "fout_b", "do_w", "do_b", "total", "wih_ctx_t",
                 "hcat_t")


class SatDecoderLayout(ctypes.Structure):
    _fields_ = [(n, c_int64) for n in LAYOUT_FIELDS]


# (name, restype, argtypes) of every exported entry point, in header order.
_SIGNATURES = [
    ("sat_abi_version", c_int, []),
    ("sat_error_string", ctypes.c_char_p, [c_int]),
    ("sat_gemm", c_int, [ctypes.POINTER(SatGemmArgs), c_void_p]),
    ("sat_gemm_workspace_bytes", c_size_t, []),
    ("sat_cast", c_int, [c_void_p, c_int, c_void_p, c_int, c_int64, c_void_p]),
    ("sat_mean_rows_abi", c_int, [c_void_p, c_int, c_int, c_int, c_int, c_void_p, c_void_p, c_void_p]),
    ("sat_nchw_to_nhwc", c_int, [c_int, c_int, c_int, c_int, c_int, c_int, c_void_p, c_void_p, c_void_p]),
    ("sat_nchw_to_s2d", c_int, [c_int, c_int, c_int, c_int, c_int, c_void_p, c_void_p, c_void_p]),
    ("sat_conv2d_nhwc", c_int, [ctypes.POINTER(SatConvGeom), c_int, c_int, c_void_p, c_void_p, c_void_p, c_void_p,
                                c_int, c_void_p, ctypes.POINTER(SatPolicy), c_void_p]),
    ("sat_mfma_frag_layout", c_int, [c_int, c_int, c_void_p, c_void_p, c_void_p]),
    ("sat_bottleneck_fused_supported", c_int, [c_int, c_int, c_int, c_int, c_int]),
    ("sat_bottleneck_fused", c_int, [c_int, c_int, c_int, c_int, c_int, c_int, c_void_p, c_void_p, c_void_p,
                                     c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, ctypes.POINTER(SatPolicy),
                                     c_void_p]),
    ("sat_conv3x3_frag_supported", c_int, [c_int, c_int, c_int, c_int]),
    ("sat_conv3x3_frag", c_int, [c_int, c_int, c_int, c_int, c_int, c_void_p, c_void_p, c_void_p, c_void_p,
                                 ctypes.POINTER(SatPolicy), c_void_p]),
    ("sat_conv1x1_frag_supported", c_int, [c_int, c_int, c_int, c_int, c_int]),
    ("sat_conv1x1_frag", c_int, [c_int, c_int, c_int, c_int, c_int, c_int, c_void_p, c_void_p, c_void_p, c_void_p,
                                 ctypes.POINTER(SatPolicy), c_void_p]),
    ("sat_maxpool2d_nhwc", c_int, [c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_void_p, c_void_p,
                                   c_int, c_int, c_void_p]),
    ("sat_attention_forward", c_int, [c_int, c_int, c_int, c_int, c_int, c_void_p, c_void_p, c_void_p, c_void_p,
                                      c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                      c_void_p, c_void_p]),
    ("sat_decoder_workspace_bytes", c_size_t, [ctypes.POINTER(SatDecoderDims)]),
    ("sat_decoder_instance", c_int, [ctypes.POINTER(SatDecoderDims), ctypes.POINTER(SatDecoderLayout),
                                     ctypes.POINTER(c_int), c_int]),
    ("sat_decoder_refresh_transposed", c_int, [ctypes.POINTER(SatDecoderDims), ctypes.POINTER(SatDecoderLayout),
                                               c_void_p, c_void_p]),
    ("sat_decoder_forward", c_int, [ctypes.POINTER(SatDecoderDims), ctypes.POINTER(SatDecoderLayout), c_void_p,
                                    c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_size_t, c_void_p,
                                    c_void_p, c_void_p, c_void_p]),
    ("sat_decoder_backward", c_int, [ctypes.POINTER(SatDecoderDims), ctypes.POINTER(SatDecoderLayout), c_void_p,
                                     c_void_p, c_void_p, c_void_p, c_size_t, c_void_p, c_void_p, c_void_p,
                                     c_void_p, c_void_p, c_int, c_int, c_void_p]),
    ("sat_decoder_step_bench", c_int, [ctypes.POINTER(SatDecoderDims), ctypes.POINTER(SatDecoderLayout), c_void_p,
                                       c_void_p, c_void_p, c_void_p, c_size_t, c_void_p, c_void_p, c_int, c_void_p,
                                       c_void_p]),
    ("sat_decoder_beam_workspace_bytes", c_size_t, [ctypes.POINTER(SatDecoderDims), c_int]),
    ("sat_decoder_beam_search", c_int, [ctypes.POINTER(SatDecoderDims), ctypes.POINTER(SatDecoderLayout), c_void_p,
                                        c_void_p, c_void_p, c_int, c_int, c_void_p, c_size_t, c_void_p, c_void_p,
                                        c_void_p, c_void_p, c_void_p, c_void_p]),
    ("sat_caption_loss_workspace_bytes", c_size_t, [c_int, c_int, c_int]),
    ("sat_caption_loss_forward", c_int, [c_int, c_int, c_int, c_int, c_int, c_void_p, c_void_p, c_void_p, c_float,
                                         c_int, c_int, c_int, c_int, c_void_p, c_void_p, c_void_p]),
    ("sat_caption_loss_forward_loss_out", c_int, [c_int, c_int, c_int, c_int, c_int, c_void_p, c_void_p, c_void_p,
                                                  c_float, c_int, c_int, c_int, c_int, c_void_p, c_void_p, c_void_p,
                                                  c_void_p]),
    ("sat_caption_loss_backward", c_int, [c_int, c_int, c_int, c_int, c_int, c_void_p, c_void_p, c_float,
                                          c_void_p, c_void_p, c_void_p, c_void_p, c_void_p]),
    ("sat_caption_loss_backward_relu", c_int, [c_int, c_int, c_int, c_int, c_int, c_void_p, c_void_p, c_float,
                                          c_void_p, c_void_p, c_void_p, c_void_p, c_void_p]),
    ("sat_caption_loss_backward_ld", c_int, [c_int, c_int, c_int, c_int, c_int, c_void_p, c_void_p, c_float,
                                             c_void_p, c_void_p, c_void_p, c_int64, c_void_p, c_int, c_void_p]),
    ("sat_images_workspace_bytes", c_size_t, [c_int, c_int, c_int]),
    ("sat_images_max_downscale", c_int, []),
    ("sat_images_to_input", c_int, [c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_int,
                                    ctypes.POINTER(c_float), ctypes.POINTER(c_float), c_int, c_int, c_int, c_void_p,
                                    c_void_p, c_size_t, c_void_p]),
    ("sat_adam_step", c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int64, c_float, c_float,
                              c_float, c_float, c_float, c_void_p]),
]
EXPORTED = [s[0] for s in _SIGNATURES]

_lib = None


def lib():
    """Load (once) and return the HIP library; raise if it is missing."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"sat_amd: HIP library not found at {LIB_PATH}; build it with "
                               "`python -c 'import __graft_entry__ as g; g.build()'` (make -C "
                               "show-attend-and-tell_amd/csrc)")
        handle = ctypes.CDLL(LIB_PATH)
        for name, res, args in _SIGNATURES:
            fn = getattr(handle, name)
            fn.restype = res
            fn.argtypes = args
        version = handle.sat_abi_version()
        if version != ABI_VERSION:
            raise RuntimeError(f"sat_amd: {LIB_PATH} has C-ABI version {version}, this package binds version "
                               f"{ABI_VERSION}; rebuild it (make -C show-attend-and-tell_amd/csrc)")
        _lib = handle
    return _lib


def check(code, what):
    if code != 0:
        msg = lib().sat_error_string(code)
        raise RuntimeError(f"sat_amd: {what} failed with code {code}: {msg.decode() if msg else '?'}")


def dtype_code(dt):
    if dt == torch.float32:
        return SAT_F32
    if dt == torch.bfloat16:
        return SAT_BF16
    raise TypeError(f"sat_amd: unsupported dtype {dt} (float32 or bfloat16)")


def require_device(*tensors):
    for t in tensors:
        if t is not None and t.device.type != "cuda":
            raise RuntimeError("sat_amd: tensors must live on a HIP device (the product path has no CPU fallback)")


def ptr(t):
    return None if t is None else ctypes.c_void_p(t.data_ptr())


def policy_ptr(policy):
    """ctypes pointer to a SatPolicy (None -> NULL = the library's defaults)."""
    return None if policy is None else ctypes.pointer(policy)


def stream_of(t):
    return ctypes.c_void_p(torch.cuda.current_stream(t.device).cuda_stream)
