// LDS-DMA throughput probe (diagnostics, not product code): how fast can one CU pull 32-KiB
// k-tiles from L2 into LDS with global_load_lds_dwordx4, as a function of waves per workgroup,
// ring depth (tiles in flight), workgroups per CU and whether every tile ends in a workgroup
// barrier -- the load side of fast_gemm_kernel's main loop without MFMA or fragment reads.
//
//   hipcc --offload-arch=gfx950 -O3 -o tools/dma_probe tools/dma_probe.hip && tools/dma_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include <cstdlib>

typedef __attribute__((address_space(3))) void lds_void;
typedef __attribute__((address_space(1))) const void gbl_void;

constexpr int TILE = 32768;   // bytes per k-tile (128 x 128 bf16 A + B of BK 64)

template <int N>
__device__ __forceinline__ void wait_vm() {
  if constexpr (N == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  else if constexpr (N == 2) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
  else if constexpr (N == 4) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  else if constexpr (N == 8) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
  else if constexpr (N == 12) asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
  else if constexpr (N == 32) asm volatile("s_waitcnt vmcnt(32)" ::: "memory");
  else if constexpr (N == 16) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
  else if constexpr (N == 24) asm volatile("s_waitcnt vmcnt(24)" ::: "memory");
  else static_assert(N < 0, "vmcnt");
}

// NW waves (of which LW issue the DMA), NS-deep ring (NS-1 tiles in flight), BAR: s_barrier
// after each tile's wait
template <int NW, int NS, bool BAR, int LW = NW>
__global__ __launch_bounds__(NW * 64) void probe(const char* __restrict__ src, long span, int iters, int* sink) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int PER_WAVE = TILE / 1024 / LW;   // 1-KiB instructions per loader wave per tile
  const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const long base = (long)blockIdx.x * 7919 * TILE;
  auto issue = [&](int k) {
    if (w >= LW) return;
    char* dst = smem + (k % NS) * TILE;
    const long off = (base + (long)k * TILE) % span;
#pragma unroll
    for (int j = 0; j < PER_WAVE; ++j) {
      const int ins = w * PER_WAVE + j;
      __builtin_amdgcn_global_load_lds((gbl_void*)(src + off + ins * 1024 + lane * 16), (lds_void*)(dst + ins * 1024),
                                       16, 0, 0);
    }
  };
  for (int p = 0; p < NS - 1; ++p) issue(p);
  for (int k = 0; k < iters; ++k) {
    if (k + NS - 1 < iters) {
      wait_vm<(NS - 2) * PER_WAVE>();   // tile k landed (NS-2 younger tiles may be in flight)
    } else {
      wait_vm<0>();
    }
    if constexpr (BAR) __builtin_amdgcn_s_barrier();
    if (k + NS - 1 < iters) issue(k + NS - 1);
  }
  wait_vm<0>();
  if (threadIdx.x == 0 && smem[5] == 123) sink[0] = 1;
}

// Register staging for comparison: each wave loads its share of tile k+1 into VGPRs
// (global_load_dwordx4), then after the barrier writes it to LDS (ds_write_b128).
template <int NW>
__global__ __launch_bounds__(NW * 64) void probe_reg(const char* __restrict__ src, long span, int iters, int* sink) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int PER_WAVE = TILE / 1024 / NW;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const long base = (long)blockIdx.x * 7919 * TILE;
  uint4 r[PER_WAVE];
  auto load = [&](int k) {
    const long off = (base + (long)k * TILE) % span;
#pragma unroll
    for (int j = 0; j < PER_WAVE; ++j) r[j] = *(const uint4*)(src + off + (w * PER_WAVE + j) * 1024 + lane * 16);
  };
  load(0);
  for (int k = 0; k < iters; ++k) {
    char* dst = smem + (k & 1) * TILE;
#pragma unroll
    for (int j = 0; j < PER_WAVE; ++j) *(uint4*)(dst + (w * PER_WAVE + j) * 1024 + lane * 16) = r[j];
    if (k + 1 < iters) load(k + 1);
    __syncthreads();
  }
  if (threadIdx.x == 0 && smem[5] == 123) sink[0] = 1;
}

template <int NW>
void run_reg(const char* name, const char* src, long span, int cus, int wg_per_cu, int* sink) {
  const int iters = 64, grid = cus * wg_per_cu, reps = 10;
  const size_t lds = 2 * (size_t)TILE;
  hipFuncSetAttribute((const void*)probe_reg<NW>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  hipEvent_t a, b;
  hipEventCreate(&a); hipEventCreate(&b);
  for (int q = 0; q < 3; ++q) hipLaunchKernelGGL(probe_reg<NW>, dim3(grid), dim3(NW * 64), lds, 0, src, span, iters, sink);
  hipEventRecord(a);
  for (int q = 0; q < reps; ++q) hipLaunchKernelGGL(probe_reg<NW>, dim3(grid), dim3(NW * 64), lds, 0, src, span, iters, sink);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms = 0.f;
  hipEventElapsedTime(&ms, a, b);
  const double bytes = (double)grid * iters * TILE * reps;
  printf("%-34s wg/cu %d  %7.1f GB/s per CU  %6.2f TB/s chip  %.3f us per tile per wg\n", name, wg_per_cu,
         bytes / (ms * 1e-3) / cus / 1e9, bytes / (ms * 1e-3) / 1e12, ms * 1e3 / reps / iters);
  hipEventDestroy(a); hipEventDestroy(b);
}

template <int NW, int NS, bool BAR, int LW = NW>
void run(const char* name, const char* src, long span, int cus, int wg_per_cu, int* sink) {
  const int iters = 64;
  const int grid = cus * wg_per_cu;
  const size_t lds = (size_t)NS * TILE;
  hipFuncSetAttribute((const void*)probe<NW, NS, BAR, LW>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  hipEvent_t a, b;
  hipEventCreate(&a); hipEventCreate(&b);
  for (int r = 0; r < 3; ++r) hipLaunchKernelGGL((probe<NW, NS, BAR, LW>), dim3(grid), dim3(NW * 64), lds, 0, src, span, iters, sink);
  hipEventRecord(a);
  const int reps = 10;
  for (int r = 0; r < reps; ++r) hipLaunchKernelGGL((probe<NW, NS, BAR, LW>), dim3(grid), dim3(NW * 64), lds, 0, src, span, iters, sink);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms = 0.f;
  hipEventElapsedTime(&ms, a, b);
  const double bytes = (double)grid * iters * TILE * reps;
  printf("%-34s wg/cu %d  %7.1f GB/s per CU  %6.2f TB/s chip  %.3f us per tile per wg\n", name, wg_per_cu,
         bytes / (ms * 1e-3) / cus / 1e9, bytes / (ms * 1e-3) / 1e12, ms * 1e3 / reps / iters);
  hipEventDestroy(a); hipEventDestroy(b);
}

int main() {
  int cus = 0;
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  const long span = (getenv("SPAN_KB") ? atol(getenv("SPAN_KB")) : 8192) * 1024L;   // working set
  char* src = nullptr;
  int* sink = nullptr;
  hipMalloc(&src, span + TILE);
  hipMalloc(&sink, 4);
  hipMemset(src, 1, span + TILE);
  for (int wpc : {1, 2}) {
    run_reg<8>("REG 8 waves, 1 tile ahead", src, span, cus, wpc, sink);
    run_reg<4>("REG 4 waves, 1 tile ahead", src, span, cus, wpc, sink);
    run<8, 2, true, 4>("8 waves (4 load), 1 tile, barrier", src, span, cus, wpc, sink);
    run<8, 2, true, 2>("8 waves (2 load), 1 tile, barrier", src, span, cus, wpc, sink);
    run<4, 2, true, 2>("4 waves (2 load), 1 tile, barrier", src, span, cus, wpc, sink);
    run<2, 2, true>("2 waves, 1 tile in flight, barrier", src, span, cus, wpc, sink);
    run<8, 2, true>("8 waves, 1 tile in flight, barrier", src, span, cus, wpc, sink);
    run<8, 2, false>("8 waves, 1 tile in flight, no bar", src, span, cus, wpc, sink);
    run<8, 3, true>("8 waves, 2 tiles in flight, barrier", src, span, cus, wpc, sink);
    run<4, 2, true>("4 waves, 1 tile in flight, barrier", src, span, cus, wpc, sink);
    run<4, 3, true>("4 waves, 2 tiles in flight, barrier", src, span, cus, wpc, sink);
    if (wpc == 1) {
      run<8, 4, true>("8 waves, 3 tiles in flight, barrier", src, span, cus, wpc, sink);
      run<4, 4, true>("4 waves, 3 tiles in flight, barrier", src, span, cus, wpc, sink);
      run<16, 3, true>("16 waves, 2 tiles in flight, barrier", src, span, cus, wpc, sink);
    }
  }
  hipFree(src);
  hipFree(sink);
  return 0;
}
