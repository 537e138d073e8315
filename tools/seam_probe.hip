// Diagnostics (not product code): the cost of a grid-wide seam inside one persistent kernel against a kernel
// boundary between dependent launches in a hipGraph, on the decoder's per-step scale (256 workgroups, a few KB
// of work each).  DESIGN.md 7 cites the guide for "a persistent decoder loop costs more than it saves"; this
// measures it on the box.
//
//   hipcc -O3 --offload-arch=gfx950 tools/seam_probe.hip -o tools/seam_probe && tools/seam_probe
//
// Persistent form: every workgroup runs R rounds; a round = 16 KB read + 16 KB write (vector memory), then a grid
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

constexpr int NWG = 256, NT = 256, WORDS = 16384 / 16;   // 16 KB per workgroup per round

__device__ __forceinline__ void round_work(const uint4* in, uint4* out, int r) {
  for (int i = threadIdx.x; i < WORDS; i += NT) {
    uint4 v = in[(long)blockIdx.x * WORDS + i];
    v.x += r;
    out[(long)blockIdx.x * WORDS + i] = v;
  }
}

__global__ __launch_bounds__(NT) void persistent_kernel(const uint4* in, uint4* out, unsigned* counter, int rounds,
                                                        unsigned* err) {
  for (int r = 0; r < rounds; ++r) {
    round_work(in, out, r);
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

__global__ __launch_bounds__(NT) void round_kernel(const uint4* in, uint4* out, int r) { round_work(in, out, r); }

int main() {
  const int R = 200;
  uint4 *in, *out;
  unsigned *counter, *err;
  CHECK(hipMalloc(&in, (size_t)NWG * WORDS * sizeof(uint4)));
  CHECK(hipMalloc(&out, (size_t)NWG * WORDS * sizeof(uint4)));
  CHECK(hipMalloc(&counter, sizeof(unsigned)));
  CHECK(hipMalloc(&err, sizeof(unsigned)));
  CHECK(hipMemset(in, 0, (size_t)NWG * WORDS * sizeof(uint4)));
  CHECK(hipMemset(err, 0, sizeof(unsigned)));
  hipStream_t s;
  CHECK(hipStreamCreate(&s));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  float ms = 0.f;

  // persistent: one launch of R rounds (plus a 1-round launch to subtract the launch itself)
  for (int rep = 0; rep < 3; ++rep) {
    for (int rounds : {1, R}) {
      CHECK(hipMemsetAsync(counter, 0, sizeof(unsigned), s));
      CHECK(hipEventRecord(e0, s));
      hipLaunchKernelGGL(persistent_kernel, dim3(NWG), dim3(NT), 0, s, in, out, counter, rounds, err);
      CHECK(hipEventRecord(e1, s));
      CHECK(hipEventSynchronize(e1));
      CHECK(hipEventElapsedTime(&ms, e0, e1));
      if (rep == 2) printf("persistent %3d rounds: %8.2f us  (%.2f us per round)\n", rounds, ms * 1e3, ms * 1e3 / rounds);
    }
  }
  unsigned herr = 0;
  CHECK(hipMemcpy(&herr, err, sizeof(unsigned), hipMemcpyDeviceToHost));

  // launches: R dependent one-round launches in a graph
  hipGraph_t g;
  hipGraphExec_t ge;
  CHECK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
  for (int r = 0; r < R; ++r) hipLaunchKernelGGL(round_kernel, dim3(NWG), dim3(NT), 0, s, in, out, r);
  CHECK(hipStreamEndCapture(s, &g));
  CHECK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
  for (int rep = 0; rep < 3; ++rep) {
    CHECK(hipEventRecord(e0, s));
    CHECK(hipGraphLaunch(ge, s));
    CHECK(hipEventRecord(e1, s));
    CHECK(hipEventSynchronize(e1));
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    if (rep == 2) printf("graph of %d launches: %8.2f us  (%.2f us per launch)\n", R, ms * 1e3, ms * 1e3 / R);
  }
  printf("barrier timeouts: %u\n", herr);
  CHECK(hipGraphExecDestroy(ge));
  CHECK(hipGraphDestroy(g));
  return herr ? 2 : 0;
}
