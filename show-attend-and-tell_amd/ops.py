"""Tensor-level wrappers over the C ABI (shape checks, output allocation, stream).

Every function here launches HIP kernels on the tensors' current stream and
never falls back to a PyTorch compute op.
"""
import ctypes

import torch

from . import _lib as L


def linear(x, weight, bias=None, act=L.ACT_NONE, out_dtype=None, weight_lp=None):
    """y = act(x @ weight.T + bias) on MFMA (nn.Linear forward).  x [M,K] (f32|bf16),
    weight [N,K] f32 (or weight_lp bf16 when x is bf16)."""
    L.require_device(x, weight)
    M, K = x.shape
    N = weight.shape[0]
    dt = L.dtype_code(x.dtype)
    if dt == L.SAT_F32:
        w = weight
    elif weight_lp is not None:
        w = weight_lp
    else:
        w = cast_(weight.contiguous(), torch.empty(weight.shape, device=weight.device, dtype=torch.bfloat16))
    out_dtype = out_dtype or torch.float32
    y = torch.empty(M, N, device=x.device, dtype=out_dtype)
    gemm(x, w, y, bias=bias, act=act)
    return y


_GEMM_WS = {}


def gemm_workspace(device, stream):
    """The split-K workspace sat_gemm may use (include/sat_hip.h SatGemmArgs.workspace), one per device and stream:
    calls ordered on one stream share it.

    The split kernel's arrival tickets and partial tiles live in the workspace, so two launches that may run at the
    same time must not share one.  Under stream capture the current stream is torch's shared capture stream, and
    graphs captured on it could be replayed concurrently on different streams: during a capture every call gets a
    workspace of its own (allocated in the graph's private pool, alive as long as the graph's pool).  Graphs that use
    ``gemm`` on the cached workspace (eager calls) are therefore never tied to each other."""
    if torch.cuda.is_current_stream_capturing():
        return torch.empty(int(L.lib().sat_gemm_workspace_bytes()), dtype=torch.uint8, device=device)
    key = (torch.device(device).index, stream.value or 0)
    ws = _GEMM_WS.get(key)
    if ws is None:
        ws = torch.empty(int(L.lib().sat_gemm_workspace_bytes()), dtype=torch.uint8, device=device)
        _GEMM_WS[key] = ws
    return ws


def _may_split(A, C, bias, aux, act, K):
    """Whether sat_gemm could take the split-K path for this call (csrc/gemmsplit.hip split_eligible): bf16 operands,
    an fp32 C, no bias / aux / activation epilogue and a long K.  Other calls never touch a workspace."""
    return (A.dtype == torch.bfloat16 and C.dtype == torch.float32 and bias is None and aux is None
            and act == L.ACT_NONE and K >= 512)


def gemm(A, B, C, *, transA=False, transB=False, alpha=1.0, beta=0.0, bias=None, add1=None, act=L.ACT_NONE,
         aux=None, policy=None, workspace=True):
    """C = act(alpha * A' B'^T + bias + add1 + beta*C) with A' = A or A^T, B'(n,k) = B[n,k] or B[k,n].
    ``policy``: an optional ``sat_amd.Policy`` (per-call kernel selection; None = library defaults).
    ``workspace``: True = this stream's cached split-K workspace (``gemm_workspace``), a uint8 device tensor, or
    None (products with fp32 output and a k-major operand then run unsplit)."""
    L.require_device(A, B, C)
    dt = L.dtype_code(A.dtype)
    if B.dtype != A.dtype:
        raise TypeError("sat_amd.gemm: A and B must share a dtype")
    M = A.shape[1] if transA else A.shape[0]
    K = A.shape[0] if transA else A.shape[1]
    N = B.shape[1] if transB else B.shape[0]
    Kb = B.shape[0] if transB else B.shape[1]
    if Kb != K or C.shape[0] != M or C.shape[1] != N:
        raise ValueError(f"sat_amd.gemm: shape mismatch A{tuple(A.shape)} B{tuple(B.shape)} C{tuple(C.shape)}")
    for t in (A, B, C, add1, aux):
        if t is not None and t.stride(-1) != 1:
            raise ValueError("sat_amd.gemm: operands must be row-major with unit inner stride")
    a = L.SatGemmArgs()
    a.M, a.N, a.K, a.dtype = M, N, K, dt
    a.A, a.lda, a.transA = A.data_ptr(), A.stride(0), int(transA)
    a.B, a.ldb, a.transB = B.data_ptr(), B.stride(0), int(transB)
    a.C, a.ldc, a.c_dtype = C.data_ptr(), C.stride(0), L.dtype_code(C.dtype)
    a.alpha, a.beta = alpha, beta
    a.bias = bias.data_ptr() if bias is not None else None
    if add1 is not None:
        a.add1, a.ld_add1, a.add1_dtype = add1.data_ptr(), add1.stride(0), L.dtype_code(add1.dtype)
    a.act = act
    if aux is not None:
        a.aux, a.ld_aux, a.aux_dtype = aux.data_ptr(), aux.stride(0), L.dtype_code(aux.dtype)
    a.policy = L.policy_ptr(policy)
    stream = L.stream_of(C)
    if workspace is True:
        workspace = (gemm_workspace(C.device, stream)
                     if policy is not None or _may_split(A, C, bias, aux, act, K) else None)
    if workspace is not None:
        a.workspace, a.workspace_bytes = workspace.data_ptr(), workspace.numel() * workspace.element_size()
    L.check(L.lib().sat_gemm(ctypes.byref(a), stream), "sat_gemm")
    return C


def cast_(src, dst):
    """dst.copy_(src) between float32/bfloat16 storage, on the HIP path."""
    L.require_device(src, dst)
    assert src.numel() == dst.numel() and src.is_contiguous() and dst.is_contiguous()
    L.check(L.lib().sat_cast(L.ptr(src), L.dtype_code(src.dtype), L.ptr(dst), L.dtype_code(dst.dtype),
                             src.numel(), L.stream_of(dst)), "sat_cast")
    return dst


def nchw_to_nhwc(x, c_pad, dtype):
    """[N,C,H,W] f32 -> [N,H,W,c_pad] (dtype), zero-padded channels."""
    L.require_device(x)
    x = x.contiguous() if not x.is_contiguous() else x
    if x.dtype != torch.float32:
        raise TypeError("images must be float32 (post-Normalize domain, train.py:27-32)")
    N, C, H, W = x.shape
    y = torch.empty(N, H, W, c_pad, device=x.device, dtype=dtype)
    L.check(L.lib().sat_nchw_to_nhwc(N, C, H, W, c_pad, L.dtype_code(dtype), L.ptr(x), L.ptr(y), L.stream_of(y)),
            "sat_nchw_to_nhwc")
    return y


def nchw_to_s2d(x, dtype):
    """[N,C,H,W] f32 (C <= 4, H, W even) -> space-to-depth [N,H/2,W/2,16] (dtype)."""
    L.require_device(x)
    x = x.contiguous() if not x.is_contiguous() else x
    if x.dtype != torch.float32:
        raise TypeError("images must be float32 (post-Normalize domain, train.py:27-32)")
    N, C, H, W = x.shape
    y = torch.empty(N, H // 2, W // 2, 16, device=x.device, dtype=dtype)
    L.check(L.lib().sat_nchw_to_s2d(N, C, H, W, L.dtype_code(dtype), L.ptr(x), L.ptr(y), L.stream_of(y)),
            "sat_nchw_to_s2d")
    return y


# Normalize(mean, std) of the reference's transform (train.py:27-32), as float32
IMAGE_MEAN = (0.485, 0.456, 0.406)
IMAGE_STD = (0.229, 0.224, 0.225)


def images_to_input(packed, layout=L.IMG_NCHW, dtype=torch.float32, c_pad=8, size=(224, 224),
                    mean=IMAGE_MEAN, std=IMAGE_STD):
    """Decoded uint8 images (a device-resident ``data.PackedImages``) -> the reference's
    Resize(size) + ToTensor + Normalize(mean, std), bit-identical to PIL + torch, written straight
    into ``layout``: IMG_NCHW [B,3,H,W] f32, IMG_NHWC [B,H,W,c_pad] (dtype) or IMG_S2D16
    [B,H/2,W/2,16] (dtype)."""
    L.require_device(packed.pixels, packed.offsets, packed.sizes)
    lib = L.lib()
    B = packed.count
    OH, OW = size
    mx = lib.sat_images_max_downscale()
    if packed.max_h > mx * OH or packed.max_w > mx * OW:
        raise ValueError(f"images_to_input: {packed.max_h}x{packed.max_w} exceeds the {mx}x downscale limit "
                         f"to {OH}x{OW}")
    dev = packed.pixels.device
    if layout == L.IMG_NCHW:
        if dtype != torch.float32:
            raise TypeError("images_to_input: the NCHW layout is the reference's float32 tensor")
        out = torch.empty(B, 3, OH, OW, device=dev, dtype=torch.float32)
    elif layout == L.IMG_NHWC:
        out = torch.empty(B, OH, OW, c_pad, device=dev, dtype=dtype)
    elif layout == L.IMG_S2D16:
        out = torch.empty(B, OH // 2, OW // 2, 16, device=dev, dtype=dtype)
    else:
        raise ValueError(f"images_to_input: unknown layout {layout}")
    ws_bytes = lib.sat_images_workspace_bytes(B, OH, OW)
    ws = torch.empty(ws_bytes, device=dev, dtype=torch.uint8)
    m = (ctypes.c_float * 3)(*mean)
    sd = (ctypes.c_float * 3)(*std)
    L.check(lib.sat_images_to_input(L.ptr(packed.pixels), L.ptr(packed.offsets), L.ptr(packed.sizes), B,
                                    packed.max_h, packed.max_w, OH, OW, m, sd, layout, c_pad, L.dtype_code(dtype),
                                    L.ptr(out), L.ptr(ws), ws_bytes, L.stream_of(out)), "sat_images_to_input")
    return out


def conv2d_nhwc(x, w, bias, stride, pad, relu, residual=None, out=None, out_hw=None, policy=None):
    """x [N,H,W,C] ; w [Cout,KH,KW,C] (same dtype) ; bias f32 [Cout].  ``pad`` pads top/left;
    ``out_hw`` (default: symmetric padding) fixes the output size; ``policy``: optional per-call kernel
    selection (``sat_amd.Policy``)."""
    L.require_device(x, w)
    N, H, W, C = x.shape
    Cout, KH, KW, Cw = w.shape
    assert Cw == C, (w.shape, x.shape)
    if out_hw is None:
        OH = (H + 2 * pad - KH) // stride + 1
        OW = (W + 2 * pad - KW) // stride + 1
    else:
        OH, OW = out_hw
    y = out if out is not None else torch.empty(N, OH, OW, Cout, device=x.device, dtype=x.dtype)
    g = L.SatConvGeom(N, H, W, C, KH, KW, stride, pad, OH, OW)
    if residual is not None:
        assert residual.shape == y.shape and residual.dtype == y.dtype
    L.check(L.lib().sat_conv2d_nhwc(ctypes.byref(g), Cout, L.dtype_code(x.dtype), L.ptr(x), L.ptr(w), L.ptr(bias),
                                    L.ptr(residual), int(relu), L.ptr(y), L.policy_ptr(policy), L.stream_of(y)),
            "sat_conv2d_nhwc")
    return y


def mfma_frag_layout(w2d):
    """[N, K] bf16 -> the register-direct MFMA fragment layout sat_bottleneck_fused streams."""
    L.require_device(w2d)
    N, K = w2d.shape
    src = w2d.contiguous()
    dst = torch.empty_like(src)
    L.check(L.lib().sat_mfma_frag_layout(N, K, L.ptr(src), L.ptr(dst), L.stream_of(dst)), "sat_mfma_frag_layout")
    return dst


def bottleneck_fused_supported(H, W, Cin, Cmid, dtype):
    return bool(L.lib().sat_bottleneck_fused_supported(H, W, Cin, Cmid, L.dtype_code(dtype)))


def bottleneck_fused(x, f1, f2, f3, out=None, policy=None):
    """One identity-residual stride-1 bottleneck in one launch.  x NHWC [N,H,W,Cin]; f1/f2/f3 =
    (fragment-layout weight, fp32 bias) of the folded c1 / c2 / c3 (Encoder plan)."""
    L.require_device(x)
    N, H, W, C = x.shape
    Cmid = f1[1].shape[0]
    y = out if out is not None else torch.empty_like(x)
    L.check(L.lib().sat_bottleneck_fused(N, H, W, C, Cmid, L.dtype_code(x.dtype), L.ptr(x), L.ptr(f1[0]),
                                         L.ptr(f1[1]), L.ptr(f2[0]), L.ptr(f2[1]), L.ptr(f3[0]), L.ptr(f3[1]),
                                         L.ptr(y), L.policy_ptr(policy), L.stream_of(y)), "sat_bottleneck_fused")
    return y


def conv3x3_frag_supported(H, W, C, dtype):
    return bool(L.lib().sat_conv3x3_frag_supported(H, W, C, L.dtype_code(dtype)))


def conv3x3_frag(x, f, out=None, policy=None):
    """relu(conv3x3(x, pad 1) + b) with f = (fragment-layout weight, fp32 bias) of a folded [C][3][3][C]
    conv (a layer3 bottleneck's c2).  x NHWC [N,H,W,C]; bit-identical to conv2d_nhwc."""
    L.require_device(x)
    if not x.is_contiguous():
        raise ValueError("conv3x3_frag: x must be a contiguous NHWC tensor")
    N, H, W, C = x.shape
    y = out if out is not None else torch.empty_like(x)
    L.check(L.lib().sat_conv3x3_frag(N, H, W, C, L.dtype_code(x.dtype), L.ptr(x), L.ptr(f[0]), L.ptr(f[1]),
                                     L.ptr(y), L.policy_ptr(policy), L.stream_of(y)), "sat_conv3x3_frag")
    return y


def conv1x1_frag_supported(H, W, Cin, Cout, dtype):
    return bool(L.lib().sat_conv1x1_frag_supported(H, W, Cin, Cout, L.dtype_code(dtype)))


def conv1x1_frag(x, f, out=None, policy=None):
    """relu(x . W^T + b) with f = (fragment-layout weight, fp32 bias) of a folded [Cout][Cin] 1x1 conv (a
    layer3 bottleneck's c1).  x NHWC [N,H,W,Cin]; bit-identical to conv2d_nhwc."""
    L.require_device(x)
    if not x.is_contiguous():
        raise ValueError("conv1x1_frag: x must be a contiguous NHWC tensor")
    N, H, W, C = x.shape
    Cout = f[1].shape[0]
    y = out if out is not None else torch.empty(N, H, W, Cout, dtype=x.dtype, device=x.device)
    L.check(L.lib().sat_conv1x1_frag(N, H, W, C, Cout, L.dtype_code(x.dtype), L.ptr(x), L.ptr(f[0]), L.ptr(f[1]),
                                     L.ptr(y), L.policy_ptr(policy), L.stream_of(y)), "sat_conv1x1_frag")
    return y


def maxpool2d_nhwc(x, k, stride, pad=0):
    L.require_device(x)
    N, H, W, C = x.shape
    OH = (H + 2 * pad - k) // stride + 1
    OW = (W + 2 * pad - k) // stride + 1
    y = torch.empty(N, OH, OW, C, device=x.device, dtype=x.dtype)
    L.check(L.lib().sat_maxpool2d_nhwc(N, H, W, C, k, stride, pad, L.dtype_code(x.dtype), L.ptr(x), L.ptr(y), OH, OW,
                                       L.stream_of(y)), "sat_maxpool2d_nhwc")
    return y


def adam_step_(param, grad, exp_avg, exp_avg_sq, param_lp, beta1, beta2, eps, step_size, bc2_sqrt):
    L.check(L.lib().sat_adam_step(L.ptr(param), L.ptr(grad), L.ptr(exp_avg), L.ptr(exp_avg_sq), L.ptr(param_lp),
                                  param.numel(), beta1, beta2, eps, step_size, bc2_sqrt, L.stream_of(param)),
            "sat_adam_step")
