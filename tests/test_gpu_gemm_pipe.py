"""gemm_pipe_kernel (csrc/gemmpipe.hip): the 256x128 pipelined bf16 GEMM with fp32 output and k-major operands
that runs the decoder's weight / input gradients (decoder.py:117-125,149-158 backward).

Every operand layout (A and B each row-major or k-major), the split-K atomic epilogue (fewer tiles than CUs),
the plain epilogue with bias + ReLU, beta = 1 accumulation, and edges: M not a multiple of 256, N not a multiple
of 128, K not a multiple of 64 (the buffer-resource zero fill), each against an fp64 product of the same bf16
operands (fp32 accumulation: 2e-5 relative) and against the 128x128 tile kernel (SatPolicy.gemm_pipe = 1).
The same cases through hipBLASLt (csrc/gemmlib.hip, SatPolicy.gemm_lib = 2), which runs the decoder's weight
gradients by default.
"""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(scope="module")
def sat():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    import sat_amd
    return sat_amd


def rel(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


CASES = [
    # M, N, K, transA, transB, beta, bias_relu
    (10000, 512, 3328, True, True, 0.0, False),    # dW f_out: 160 tiles -> split-K
    (2048, 2048, 3328, True, True, 0.0, False),    # dW W_ih[:, E:]
    (4608, 512, 3328, True, True, 1.0, False),     # dW [U; f_beta; W_hh], accumulate
    (512, 2048, 6272, True, True, 0.0, False),     # dW attention.W (K = B L)
    (3328, 512, 10000, False, True, 0.0, False),   # dX f_out (B k-major)
    (3328, 2048, 512, False, True, 0.0, False),    # dX f_z
    (1000, 200, 1000, True, True, 0.0, False),     # edges everywhere: M, N, K tails
    (300, 136, 520, False, True, 0.0, True),       # plain epilogue with bias + ReLU, tails
    (1024, 1024, 2048, True, False, 0.0, False),   # A k-major, B row-major
    (520, 264, 776, False, False, 1.0, False),     # row-major both (mode 2 only), accumulate
]


@pytest.mark.parametrize("M,N,K,transA,transB,beta,bias_relu", CASES)
def test_gemm_pipe_matches_fp64_and_tile_kernel(sat, M, N, K, transA, transB, beta, bias_relu):
    from sat_amd import ops
    g = torch.Generator().manual_seed(M + 3 * N + 7 * K)
    A = torch.randn(M, K, generator=g).bfloat16()
    Bm = torch.randn(N, K, generator=g).bfloat16()
    C0 = torch.randn(M, N, generator=g)
    bias = torch.randn(N, generator=g) if bias_relu else None
    ref = A.double() @ Bm.double().T + beta * C0.double()
    if bias_relu:
        ref = (ref + bias.double()).clamp_min(0.0)
    Ad = (A.T.contiguous() if transA else A).to(DEV)
    Bd = (Bm.T.contiguous() if transB else Bm).to(DEV)
    kw = dict(transA=transA, transB=transB, beta=beta)
    if bias_relu:
        kw.update(bias=bias.to(DEV), act=sat._lib.ACT_RELU)
    out = {}
    for mode in (2, 1):   # every eligible problem on the pipelined kernel / never (hipBLASLt off in both)
        C = C0.clone().to(DEV)
        ops.gemm(Ad, Bd, C, policy=sat.Policy(gemm_pipe=mode, gemm_lib=1), **kw)
        torch.cuda.synchronize()
        out[mode] = C.cpu()
    assert torch.isfinite(out[2]).all()
    assert rel(out[2], ref) < 2e-5, rel(out[2], ref)
    assert rel(out[2], out[1]) < 2e-5


def test_gemm_pipe_leaves_rows_past_m_alone(sat):
    """C is a view into a larger buffer: rows / columns outside [M, N] keep their values (the zero fill of the
    edges must not be stored)."""
    from sat_amd import ops
    g = torch.Generator().manual_seed(11)
    M, N, K = 300, 136, 3328
    A = torch.randn(K, M, generator=g).bfloat16().to(DEV)
    Bm = torch.randn(K, N, generator=g).bfloat16().to(DEV)
    big = torch.full((M + 5, N + 8), 7.0, device=DEV)
    C = big[:M, :N]
    ops.gemm(A, Bm, C, transA=True, transB=True, policy=sat.Policy(gemm_pipe=2, gemm_lib=1))
    torch.cuda.synchronize()
    ref = A.double().T @ Bm.double()
    assert rel(C, ref) < 2e-5
    assert (big[M:] == 7.0).all() and (big[:, N:] == 7.0).all()


@pytest.mark.parametrize("M,N,K,transA,transB,beta,bias_relu", [c for c in CASES if not c[6]])
def test_gemm_lib_matches_fp64(sat, M, N, K, transA, transB, beta, bias_relu):
    """hipBLASLt (SatPolicy.gemm_lib = 2) on the same products: fp32 accumulation of the same bf16 operands."""
    from sat_amd import ops
    g = torch.Generator().manual_seed(M + 5 * N + 3 * K)
    A = torch.randn(M, K, generator=g).bfloat16()
    Bm = torch.randn(N, K, generator=g).bfloat16()
    C0 = torch.randn(M, N, generator=g)
    ref = A.double() @ Bm.double().T + beta * C0.double()
    Ad = (A.T.contiguous() if transA else A).to(DEV)
    Bd = (Bm.T.contiguous() if transB else Bm).to(DEV)
    big = torch.full((M + 3, N + 8), 7.0, device=DEV)
    C = big[:M, :N]
    C.copy_(C0.to(DEV))
    ops.gemm(Ad, Bd, C, transA=transA, transB=transB, beta=beta, policy=sat.Policy(gemm_lib=2))
    torch.cuda.synchronize()
    assert rel(C, ref) < 2e-5, rel(C, ref)
    assert (big[M:] == 7.0).all() and (big[:, N:] == 7.0).all()
