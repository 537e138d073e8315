"""split_gemm_kernel (csrc/gemmsplit.hip): the pipelined bf16 GEMM with fp32 output, a k-major operand and a
deterministic split-K that runs the decoder's batched weight / input gradients (decoder.py:115,117-125,149-158 and
attention.py:15-16 backward, train.py:163).

Every operand layout with a k-major operand (A k-major, B k-major or both) and the NN products the tile kernel would
split with fp32 atomics, both tile heights (SatPolicy.split_gemm
= 2: 128 rows, 3: 256 rows), forced split counts (SatPolicy.split_k) and the planner's choice, beta = 1
accumulation, an fp32 addend, and edges (M not a multiple of the tile height, N not a multiple of 128, K not a
multiple of 64: the buffer-resource zero fill), each against an fp64 product of the same bf16 operands (fp32
accumulation: 2e-5 relative) and against the 128x128 tile kernel (SatPolicy.split_gemm = 1).  The split-K sum runs
in split order whichever workgroup arrives last, so repeated launches are bit-identical.
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
    # M, N, K, transA, transB, beta
    (10000, 512, 3328, True, True, 0.0),    # dW f_out
    (2048, 2048, 3328, True, True, 0.0),    # dW W_ih[:, E:]
    (4608, 512, 3328, True, True, 1.0),     # dW [U; f_beta; W_hh], accumulate
    (512, 2048, 6272, True, True, 0.0),     # dW attention.W (K = B L)
    (512, 2048, 3328, True, True, 0.0),     # dW f_z
    (3328, 512, 10000, False, True, 0.0),   # dX f_out (B k-major)
    (3328, 512, 2048, False, True, 0.0),    # dX embedding
    (1000, 200, 1000, True, True, 0.0),     # edges everywhere: M, N, K tails
    (1024, 1024, 2048, True, False, 0.0),   # A k-major, B row-major
    (300, 136, 520, False, True, 1.0),      # B k-major, tails, accumulate
    (300, 136, 1104, False, False, 0.0),    # NN with few tiles and K >= 1024 (the tile kernel's atomic split-K case)
    (3, 512, 2624, False, False, 0.0),      # the per-step dh GEMM of a 3-row batch (K = 5E + D, 41 k-tiles)
]
# (split_gemm, split_k): the planner, both tile heights unsplit and split
FORMS = [(0, 0), (2, 1), (2, 2), (2, 4), (3, 1), (3, 2), (3, 3)]


def _operands(M, N, K, transA, transB, seed):
    g = torch.Generator().manual_seed(seed)
    A = torch.randn(M, K, generator=g).bfloat16()
    Bm = torch.randn(N, K, generator=g).bfloat16()
    C0 = torch.randn(M, N, generator=g)
    Ad = (A.T.contiguous() if transA else A).to(DEV)
    Bd = (Bm.T.contiguous() if transB else Bm).to(DEV)
    return A, Bm, C0, Ad, Bd


@pytest.mark.parametrize("M,N,K,transA,transB,beta", CASES)
def test_split_gemm_matches_fp64_and_tile_kernel(sat, M, N, K, transA, transB, beta):
    from sat_amd import ops
    A, Bm, C0, Ad, Bd = _operands(M, N, K, transA, transB, M + 3 * N + 7 * K)
    ref = A.double() @ Bm.double().T + beta * C0.double()
    tile = C0.clone().to(DEV)
    ops.gemm(Ad, Bd, tile, transA=transA, transB=transB, beta=beta, policy=sat.Policy(split_gemm=1))
    for form, splits in FORMS:
        big = torch.full((M + 3, N + 8), 7.0, device=DEV)   # C as a view: rows / columns past it stay untouched
        C = big[:M, :N]
        C.copy_(C0.to(DEV))
        ops.gemm(Ad, Bd, C, transA=transA, transB=transB, beta=beta,
                 policy=sat.Policy(split_gemm=form, split_k=splits))
        torch.cuda.synchronize()
        assert torch.isfinite(C).all(), (form, splits)
        assert rel(C, ref) < 2e-5, (form, splits, rel(C, ref))
        assert rel(C, tile) < 2e-5, (form, splits)
        assert (big[M:] == 7.0).all() and (big[:, N:] == 7.0).all(), (form, splits)


@pytest.mark.parametrize("form,splits", [(2, 4), (3, 2), (0, 0)])
def test_split_gemm_bit_identical_across_launches(sat, form, splits):
    """The last-arriving split adds the partial tiles in split order: the same bits whichever split finished last."""
    from sat_amd import ops
    M, N, K = 512, 2048, 3328
    _, _, _, Ad, Bd = _operands(M, N, K, True, True, 5)
    pol = sat.Policy(split_gemm=form, split_k=splits)
    outs = []
    for _ in range(4):
        C = torch.empty(M, N, device=DEV)
        ops.gemm(Ad, Bd, C, transA=True, transB=True, policy=pol)
        outs.append(C)
    torch.cuda.synchronize()
    for o in outs[1:]:
        assert torch.equal(o, outs[0])


def test_split_gemm_addend_and_poisoned_workspace(sat):
    """C = A B^T + add1 (the embedding gradient's ado term), with the workspace's tickets and partial tiles
    poisoned before the call: the launch zeroes its own tickets (SatGemmArgs.workspace contract)."""
    from sat_amd import ops
    M, N, K = 3328, 512, 2048
    A, Bm, _, Ad, Bd = _operands(M, N, K, False, True, 9)
    add1 = torch.randn(M, N, generator=torch.Generator().manual_seed(2))
    ref = A.double() @ Bm.double().T + add1.double()
    ws = torch.full((int(sat._lib.lib().sat_gemm_workspace_bytes()),), 0xA5, dtype=torch.uint8, device=DEV)
    for splits in (2, 3):
        C = torch.empty(M, N, device=DEV)
        ops.gemm(Ad, Bd, C, transB=True, add1=add1.to(DEV), workspace=ws,
                 policy=sat.Policy(split_gemm=2, split_k=splits))
        torch.cuda.synchronize()
        assert rel(C, ref) < 2e-5, (splits, rel(C, ref))


def test_split_gemm_without_workspace_runs_unsplit(sat):
    """No workspace: the split kernel declines a product it would split (it falls through to the tile kernel), and
    the few-tile NN long-K shape the tile kernel splits with atomics does not run unsplit on a handful of
    workgroups either: both stay correct."""
    from sat_amd import ops
    M, N, K = 512, 512, 3328
    A, Bm, _, Ad, Bd = _operands(M, N, K, True, True, 4)
    C = torch.empty(M, N, device=DEV)
    ops.gemm(Ad, Bd, C, transA=True, transB=True, workspace=None, policy=sat.Policy(split_k=4))
    torch.cuda.synchronize()
    assert rel(C, A.double() @ Bm.double().T) < 2e-5
    A, Bm, _, Ad, Bd = _operands(300, 136, 1104, False, False, 6)
    C = torch.empty(300, 136, device=DEV)
    ops.gemm(Ad, Bd, C, workspace=None)
    torch.cuda.synchronize()
    assert rel(C, A.double() @ Bm.double().T) < 2e-5


def test_gemm_workspace_private_per_capture(sat):
    """Two graphs captured on torch's shared capture stream get split-K workspaces of their own (their tickets
    would race if the graphs were replayed concurrently on two streams), and replaying both concurrently gives the
    eager results."""
    from sat_amd import ops
    M, N, K = 512, 2048, 3328
    _, _, _, Ad, Bd = _operands(M, N, K, True, True, 11)
    eager = torch.empty(M, N, device=DEV)
    ops.gemm(Ad, Bd, eager, transA=True, transB=True)
    seen = []
    orig = ops.gemm_workspace

    def spy(device, stream):
        ws = orig(device, stream)
        seen.append(ws.data_ptr())
        return ws
    outs, graphs = [], []
    ops.gemm_workspace = spy
    try:
        for _ in range(2):
            C = torch.empty(M, N, device=DEV)
            g = torch.cuda.CUDAGraph()
            torch.cuda.synchronize()
            with torch.cuda.graph(g):
                ops.gemm(Ad, Bd, C, transA=True, transB=True)
            outs.append(C)
            graphs.append(g)
    finally:
        ops.gemm_workspace = orig
    assert len(seen) == 2 and seen[0] != seen[1]
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    torch.cuda.synchronize()
    for _ in range(3):
        for C in outs:
            C.fill_(float("nan"))
        torch.cuda.synchronize()
        with torch.cuda.stream(s1):
            graphs[0].replay()
        with torch.cuda.stream(s2):
            graphs[1].replay()
        torch.cuda.synchronize()
        for C in outs:
            assert torch.equal(C, eager)


def test_gemm_output_past_2gib_uses_plain_stores(sat):
    """An fp32 output whose byte extent passes 2 GiB: the buffer-resource epilogues (32-bit offsets, sat_out_rsrc's
    cap) must not take it -- the rows past 2 GiB are checked against the fp64 product."""
    from sat_amd import ops
    M, N, K = 66000, 8192, 64   # 2.16 GB of fp32 C
    g = torch.Generator().manual_seed(3)
    A = torch.randn(M, K, generator=g).bfloat16()
    Bm = torch.randn(N, K, generator=g).bfloat16()
    C = torch.full((M, N), float("nan"), device=DEV)
    ops.gemm(A.to(DEV), Bm.to(DEV), C)
    torch.cuda.synchronize()
    rows = torch.tensor([0, 1, 65535, 65536, M - 2, M - 1])
    ref = A[rows].double() @ Bm.double().T
    got = C[rows.to(DEV)].cpu()
    assert torch.isfinite(got).all()
    assert rel(got, ref) < 2e-5
    del C
    torch.cuda.empty_cache()
