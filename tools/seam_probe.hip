// Diagnostics (not product code): the cost of a grid-wide seam inside one persistent kernel against a kernel
// boundary between dependent launches in a hipGraph, on the decoder's per-step scale (256 workgroups, a few KB
// of work each).  DESIGN.md 7 cites the guide for "a persistent decoder loop costs more than it saves"; this
// measures it on the box.
//
//   hipcc -O3 --offload-arch=gfx950 tools/seam_probe.hip -o tools/seam_probe && tools/seam_probe
//
// Persistent form: every workgroup runs R rounds; a round = 0, 4 or 16 KB read + written (write-back or write-through
// 16-B stores), then a grid
// barrier: every storing wave's vmcnt(0), workgroup barrier, one lane's agent release fence + agent atomic add on
// the round counter, polling with agent-scope relaxed loads until all workgroups arrived, an agent acquire fence,
// workgroup barrier (cdna_hip_programming.md sec. 6 Guideline 16).  Every poll loop is capped (a missing arrival
// would exit with an error flag instead of hanging the GPU).  Launch form: R launches of the one-round kernel
// captured in a hipGraph and replayed.
#include <hip/hip_runtime.h>
#include <stdio.h>

#define CHECK(x)                                                            \
  do {                                                                      \
    hipError_t e = (x);                                                     \
    if (e != hipSuccess) {                                                  \
      printf("HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); \
      return 1;                                                             \
    }                                                                       \
  } while (0)

constexpr int NWG = 256, NT = 256, MAXW = 16384 / 16;   // up to 16 KB per workgroup per round

// `words` 16-B words read and written per workgroup; wt: the stores write through (sc1 buffer stores)
__device__ __forceinline__ void round_work(const uint4* in, uint4* out, int r, int words, int wt) {
  const __amdgpu_buffer_rsrc_t ro = __builtin_amdgcn_make_buffer_rsrc((void*)out, (short)0, 0x7fffffff, 0x00020000);
  typedef unsigned __attribute__((ext_vector_type(4))) u4;
  for (int i = threadIdx.x; i < words; i += NT) {
    uint4 v = in[(long)blockIdx.x * MAXW + i];
    v.x += r;
    const int off = (int)(((long)blockIdx.x * MAXW + i) * 16);
    if (wt) __builtin_amdgcn_raw_buffer_store_b128(u4{v.x, v.y, v.z, v.w}, ro, off, 0, 16);
    else __builtin_amdgcn_raw_buffer_store_b128(u4{v.x, v.y, v.z, v.w}, ro, off, 0, 0);
  }
}

__global__ __launch_bounds__(NT) void persistent_kernel(const uint4* in, uint4* out, unsigned* counter, int rounds,
                                                        unsigned* err, int words, int wt) {
  for (int r = 0; r < rounds; ++r) {
    round_work(in, out, r, words, wt);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      __hip_atomic_fetch_add(counter, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const unsigned target = (unsigned)(r + 1) * gridDim.x;
      long spins = 0;
      while (__hip_atomic_load(counter, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
        __builtin_amdgcn_s_sleep(1);
        if (++spins > 20000000L) {   // never reached when every workgroup is resident: exit instead of hanging
          __hip_atomic_fetch_add(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          break;
        }
      }
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    }
    __syncthreads();
  }
}

__global__ __launch_bounds__(NT) void round_kernel(const uint4* in, uint4* out, int r, int words, int wt) {
  round_work(in, out, r, words, wt);
}

int main() {
  const int R = 200;
  uint4 *in, *out;
  unsigned *counter, *err;
  CHECK(hipMalloc(&in, (size_t)NWG * MAXW * sizeof(uint4)));
  CHECK(hipMalloc(&out, (size_t)NWG * MAXW * sizeof(uint4)));
  CHECK(hipMalloc(&counter, sizeof(unsigned)));
  CHECK(hipMalloc(&err, sizeof(unsigned)));
  CHECK(hipMemset(in, 0, (size_t)NWG * MAXW * sizeof(uint4)));
  CHECK(hipMemset(err, 0, sizeof(unsigned)));
  hipStream_t s;
  CHECK(hipStreamCreate(&s));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  float ms = 0.f;

  unsigned herr = 0;
  for (int words : {0, 256, MAXW}) {
    for (int wt = 0; wt < 2; ++wt) {
      if (words == 0 && wt) continue;
      float per_round = 0.f, per_launch = 0.f;
      // persistent: one launch of R rounds
      for (int rep = 0; rep < 3; ++rep) {
        CHECK(hipMemsetAsync(counter, 0, sizeof(unsigned), s));
        CHECK(hipEventRecord(e0, s));
        hipLaunchKernelGGL(persistent_kernel, dim3(NWG), dim3(NT), 0, s, in, out, counter, R, err, words, wt);
        CHECK(hipEventRecord(e1, s));
        CHECK(hipEventSynchronize(e1));
        CHECK(hipEventElapsedTime(&ms, e0, e1));
        per_round = ms * 1e3f / R;
      }
      // launches: R dependent one-round launches in a graph
      hipGraph_t g;
      hipGraphExec_t ge;
      CHECK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
      for (int r = 0; r < R; ++r) hipLaunchKernelGGL(round_kernel, dim3(NWG), dim3(NT), 0, s, in, out, r, words, wt);
      CHECK(hipStreamEndCapture(s, &g));
      CHECK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
      for (int rep = 0; rep < 3; ++rep) {
        CHECK(hipEventRecord(e0, s));
        CHECK(hipGraphLaunch(ge, s));
        CHECK(hipEventRecord(e1, s));
        CHECK(hipEventSynchronize(e1));
        CHECK(hipEventElapsedTime(&ms, e0, e1));
        per_launch = ms * 1e3f / R;
      }
      CHECK(hipGraphExecDestroy(ge));
      CHECK(hipGraphDestroy(g));
      printf("%5d B per workgroup (%s stores): persistent %.2f us per round, graph %.2f us per launch\n", words * 16,
             wt ? "write-through" : "write-back", per_round, per_launch);
    }
  }
  CHECK(hipMemcpy(&herr, err, sizeof(unsigned), hipMemcpyDeviceToHost));
  printf("barrier timeouts: %u\n", herr);
  return herr ? 2 : 0;
}
