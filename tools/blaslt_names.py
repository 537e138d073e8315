"""Calibration only: run hipBLASLt on the ResNet152 layer-3 GEMM shapes (bf16) so a rocprofv3 kernel
trace shows which macro-tile kernels the vendor library picks."""
import torch
for M, N, K in [(25088, 256, 2304), (25088, 1024, 256), (25088, 256, 1024), (100352, 128, 1152)]:
    A = torch.randn(M, K, device="cuda").bfloat16()
    B = torch.randn(N, K, device="cuda").bfloat16()
    for _ in range(5):
        torch.mm(A, B.t())
torch.cuda.synchronize()
