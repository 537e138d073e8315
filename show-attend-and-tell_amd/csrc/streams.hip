// CU-partitioned streams: the latency-bound decoder chain and the chip-filling conv trunk of the
// next batch run side by side on disjoint CU sets, so a decoder kernel never queues behind a
// long-running encoder workgroup.
#include "sat_common.h"
#include "sat_internal.h"

extern "C" int sat_device_cu_count(int* ncu) {
  SAT_REQUIRE(ncu);
  int dev = 0;
  SAT_CHECK(hipGetDevice(&dev));
  SAT_CHECK(hipDeviceGetAttribute(ncu, hipDeviceAttributeMultiprocessorCount, dev));
  return 0;
}

extern "C" int sat_stream_create_cu_mask(const uint32_t* mask, int words, void** stream_out) {
  SAT_REQUIRE(mask && words > 0 && words <= 32 && stream_out);
  hipStream_t s = nullptr;
  SAT_CHECK(hipExtStreamCreateWithCUMask(&s, (uint32_t)words, mask));
  *stream_out = (void*)s;
  return 0;
}

extern "C" int sat_stream_destroy(void* stream) {
  SAT_REQUIRE(stream);
  SAT_CHECK(hipStreamDestroy((hipStream_t)stream));
  return 0;
}

namespace {
// diagnostics: which hardware CU each workgroup landed on (HW_ID + XCC_ID register reads), so the
// runtime's CU-mask bit order can be mapped to XCDs / shader engines (tools/cu_probe.py)
__global__ __launch_bounds__(64) void cu_probe_kernel(uint32_t* out, int spin) {
  const uint32_t hw = __builtin_amdgcn_s_getreg((31 << 11) | 4);     // HW_REG_HW_ID, 32 bits
  const uint32_t xcc = __builtin_amdgcn_s_getreg((31 << 11) | 20);   // HW_REG_XCC_ID, 32 bits
  long t0 = __builtin_readcyclecounter();
  while (__builtin_readcyclecounter() - t0 < spin) __builtin_amdgcn_s_sleep(1);
  if (threadIdx.x == 0) {
    out[2 * blockIdx.x] = hw;
    out[2 * blockIdx.x + 1] = xcc;
  }
}
}  // namespace

extern "C" int sat_probe_cu_ids(int nblocks, int spin_cycles, uint32_t* out, void* stream) {
  SAT_REQUIRE(out && nblocks > 0 && spin_cycles >= 0);
  hipLaunchKernelGGL(cu_probe_kernel, dim3(nblocks), dim3(64), 0, (hipStream_t)stream, out, spin_cycles);
  SAT_CHECK(hipGetLastError());
  return 0;
}
