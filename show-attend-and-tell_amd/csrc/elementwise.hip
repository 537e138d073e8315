// Memory-bound helper kernels: layout conversion, max-pool, casts, reductions
// over rows/columns, embedding gather / scatter-add, greedy argmax and the Adam
// step.  All are HBM-bound streaming kernels: 16-B accesses where the layout
// allows, grid-stride loops capped at ~8 blocks per CU.
#include "sat_common.h"
#include "sat_internal.h"

namespace {

constexpr int kMaxGrid = 2048;
inline int grid_for(long n, int per_block = 256) {
  long g = (n + per_block - 1) / per_block;
  return (int)(g < 1 ? 1 : (g > kMaxGrid ? kMaxGrid : g));
}

// ---- NCHW fp32 -> NHWC (T), channels zero-padded to Cp ----------------------
// one pixel per thread: C coalesced channel-plane loads, one 16-B store when Cp*sizeof(T) == 16
template <typename T>
__global__ void nchw_to_nhwc_kernel(const float* __restrict__ x, T* __restrict__ y, int N, int C, int H, int W,
                                    int Cp) {
  long total = (long)N * H * W;
  for (long p = blockIdx.x * (long)blockDim.x + threadIdx.x; p < total; p += (long)gridDim.x * blockDim.x) {
    long n = p / ((long)H * W), hw = p - n * H * W;
    const float* src = x + n * C * H * W + hw;
    T* dst = y + p * Cp;
    if (Cp * sizeof(T) == 16) {
      uint4 u;
      T* h = (T*)&u;
#pragma unroll
      for (int c = 0; c < 16 / (int)sizeof(T); ++c) h[c] = (T)(c < C ? src[(long)c * H * W] : 0.f);
      *(uint4*)dst = u;
    } else {
      for (int c = 0; c < Cp; ++c) dst[c] = (T)(c < C ? src[(long)c * H * W] : 0.f);
    }
  }
}

// ---- NCHW fp32 -> space-to-depth NHWC (T): [N, H/2, W/2, 16], channel (sy*2+sx)*C + c ----------
// The ResNet stem (7x7 / stride 2, Cin = 3) becomes a 4x4 / stride 1 conv over 16 channels
// (12 real): K = 256 instead of 7*7*8 = 392, and half the input bytes of the 8-channel layout.
// One output pixel (32 B) per thread.
template <typename T>
__global__ void nchw_to_s2d16_kernel(const float* __restrict__ x, T* __restrict__ y, int N, int C, int H, int W) {
  const int H2 = H / 2, W2 = W / 2;
  const long total = (long)N * H2 * W2;
  for (long p = blockIdx.x * (long)blockDim.x + threadIdx.x; p < total; p += (long)gridDim.x * blockDim.x) {
    const long n = p / ((long)H2 * W2), r = p - n * H2 * W2;
    const int by = (int)(r / W2), bx = (int)(r - (long)by * W2);
    const float* src = x + n * C * H * W;
    float v[16];
#pragma unroll
    for (int q = 0; q < 16; ++q) v[q] = 0.f;
#pragma unroll
    for (int sy = 0; sy < 2; ++sy)
#pragma unroll
      for (int sx = 0; sx < 2; ++sx)
        for (int c = 0; c < C; ++c)
          v[(sy * 2 + sx) * C + c] = src[((long)c * H + 2 * by + sy) * W + 2 * bx + sx];
    T* dst = y + p * 16;
#pragma unroll
    for (int q = 0; q < 16; ++q) dst[q] = (T)v[q];
  }
}

// RGB (C = 3) bf16 form of the above: one output pixel per thread, the two input columns of each
// (channel, row) as one 8-byte load, the 16 output channels as two 16-byte stores.
__global__ __launch_bounds__(256) void nchw3_to_s2d16_bf16_kernel(const float* __restrict__ x, bf16* __restrict__ y,
                                                                  int N, int H, int W) {
  const int H2 = H / 2, W2 = W / 2;
  const long p = blockIdx.x * (long)blockDim.x + threadIdx.x;
  if (p >= (long)N * H2 * W2) return;
  const long n = p / ((long)H2 * W2), r = p - n * H2 * W2;
  const int by = (int)(r / W2), bx = (int)(r - (long)by * W2);
  const float* src = x + n * 3 * H * W;
  float2 v[2][3];
#pragma unroll
  for (int sy = 0; sy < 2; ++sy)
#pragma unroll
    for (int c = 0; c < 3; ++c) v[sy][c] = *(const float2*)(src + ((long)c * H + 2 * by + sy) * W + 2 * bx);
  uint4 u[2];
  bf16* o = (bf16*)u;
#pragma unroll
  for (int q = 0; q < 16; ++q) o[q] = (bf16)0.f;
#pragma unroll
  for (int sy = 0; sy < 2; ++sy)
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      o[(sy * 2 + 0) * 3 + c] = (bf16)v[sy][c].x;
      o[(sy * 2 + 1) * 3 + c] = (bf16)v[sy][c].y;
    }
  uint4* dst = (uint4*)(y + p * 16);   // plain stores: write-through measured slower for the stem (profiles/r4_s19)
  dst[0] = u[0];
  dst[1] = u[1];
}

// ---- max-pool NHWC (floor mode), 8 channels per thread (16-B bf16 / 2x16-B f32 accesses) ----
template <typename T>
__global__ void maxpool_kernel(const T* __restrict__ x, T* __restrict__ y, int N, int H, int W, int C, int k,
                               int stride, int pad, int OH, int OW) {
  const int C8 = C / 8;
  long total = (long)N * OH * OW * C8;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int c8 = (int)(i % C8);
    long p = i / C8;
    const int ow = (int)(p % OW); p /= OW;
    const int oh = (int)(p % OH); const int n = (int)(p / OH);
    float m[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) m[e] = -INFINITY;
    for (int kh = 0; kh < k; ++kh) {
      const int ih = oh * stride - pad + kh;
      if (ih < 0 || ih >= H) continue;
      for (int kw = 0; kw < k; ++kw) {
        const int iw = ow * stride - pad + kw;
        if (iw < 0 || iw >= W) continue;
        const T* src = x + (((long)n * H + ih) * W + iw) * C + c8 * 8;
        T v[8];
        if constexpr (sizeof(T) == 2) {
          *(uint4*)v = *(const uint4*)src;
        } else {
          *(uint4*)v = *(const uint4*)src;
          *(uint4*)(v + 4) = *(const uint4*)(src + 4);
        }
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float f = (float)v[e];
          m[e] = (f > m[e] || f != f) ? f : m[e];   // NaN propagates like torch max_pool2d
        }
      }
    }
    T o[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = (T)m[e];
    T* dst = y + i * 8;
    if constexpr (sizeof(T) == 2) {
      *(uint4*)dst = *(uint4*)o;
    } else {
      *(uint4*)dst = *(uint4*)o;
      *(uint4*)(dst + 4) = *(uint4*)(o + 4);
    }
  }
}

// bf16 k x k pool (the ResNet152 3x3/s2/p1 stem pool): one output pixel x 8 channels per thread,
// every window tap requested before the first compare (clamped address + validity select), one
// pass over the grid: the grid-stride form above issues its taps behind per-tap branches.
template <int KS>
__global__ __launch_bounds__(256) void maxpool_bf16_kernel(const bf16* __restrict__ x, bf16* __restrict__ y, int N,
                                                           int H, int W, int C, int stride, int pad, int OH,
                                                           int OW) {
  const int C8 = C / 8;
  const long i = blockIdx.x * (long)blockDim.x + threadIdx.x;
  if (i >= (long)N * OH * OW * C8) return;
  const int c8 = (int)(i % C8);
  long p = i / C8;
  const int ow = (int)(p % OW); p /= OW;
  const int oh = (int)(p % OH); const int n = (int)(p / OH);
  uint4 v[KS * KS];
  bool ok[KS * KS];
#pragma unroll
  for (int kh = 0; kh < KS; ++kh)
#pragma unroll
    for (int kw = 0; kw < KS; ++kw) {
      const int ih = oh * stride - pad + kh, iw = ow * stride - pad + kw;
      const bool in = ih >= 0 && ih < H && iw >= 0 && iw < W;
      const int ihc = in ? ih : 0, iwc = in ? iw : 0;
      ok[kh * KS + kw] = in;
      v[kh * KS + kw] = *(const uint4*)(x + (((long)n * H + ihc) * W + iwc) * C + c8 * 8);
    }
  float m[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) m[e] = -INFINITY;
#pragma unroll
  for (int t = 0; t < KS * KS; ++t) {
    if (!ok[t]) continue;
    const bf16* h = (const bf16*)&v[t];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float f = (float)h[e];
      m[e] = (f > m[e] || f != f) ? f : m[e];   // NaN propagates like torch max_pool2d
    }
  }
  uint4 u;
  bf16* o = (bf16*)&u;
#pragma unroll
  for (int e = 0; e < 8; ++e) o[e] = (bf16)m[e];
  *(uint4*)(y + i * 8) = u;   // plain: write-through measured slower for the stem pool (profiles/r4_s19)
}

template <typename TI, typename TO>
__global__ void cast_kernel(const TI* __restrict__ x, TO* __restrict__ y, long n) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
    y[i] = (TO)(float)x[i];
}

// ---- mean over L: a [B,L,D] -> out [B,D] (fp32 accumulate) -------------------
template <typename T>
__global__ void mean_rows_kernel(const T* __restrict__ a, int L, int D, float* __restrict__ out_f32,
                                 T* __restrict__ out_t) {
  int b = blockIdx.y;
  int d = blockIdx.x * blockDim.x + threadIdx.x;
  if (d >= D) return;
  const T* p = a + (long)b * L * D + d;
  float s = 0.f;
  for (int l = 0; l < L; ++l) s += (float)p[(long)l * D];
  s /= (float)L;
  if (out_f32) out_f32[(long)b * D + d] = s;
  if (out_t) out_t[(long)b * D + d] = (T)s;
}

// 16-byte vectors (VEC columns per thread), 8 rows requested per batch; the same ascending-l
// summation per element as mean_rows_kernel
template <typename T>
__global__ __launch_bounds__(256) void mean_rows_vec_kernel(const T* __restrict__ a, int L, int D,
                                                            float* __restrict__ out_f32, T* __restrict__ out_t) {
  constexpr int VEC = 16 / sizeof(T);
  const int b = blockIdx.y;
  const int d = (blockIdx.x * 256 + threadIdx.x) * VEC;
  if (d >= D) return;
  const T* p = a + (long)b * L * D + d;
  float acc[VEC];
#pragma unroll
  for (int j = 0; j < VEC; ++j) acc[j] = 0.f;
  int l = 0;
  for (; l + 8 <= L; l += 8) {
    uint4 u[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) u[k] = *(const uint4*)(p + (long)(l + k) * D);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const T* h = (const T*)&u[k];
#pragma unroll
      for (int j = 0; j < VEC; ++j) acc[j] += (float)h[j];
    }
  }
  for (; l < L; ++l) {
    const uint4 u = *(const uint4*)(p + (long)l * D);
    const T* h = (const T*)&u;
#pragma unroll
    for (int j = 0; j < VEC; ++j) acc[j] += (float)h[j];
  }
#pragma unroll
  for (int j = 0; j < VEC; ++j) {
    const float m = acc[j] / (float)L;
    if (out_f32) out_f32[(long)b * D + d + j] = m;
    if (out_t) out_t[(long)b * D + d + j] = (T)m;
  }
}

// ---- column sums: out[n] (+)= sum_r X[r*ld + n] ----------------------------
// pass 1: grid (ceil(N/256), RS) partial sums over row chunks; pass 2 folds them.  The bodies take the block
// coordinates as arguments so the multi-segment kernels below (several column sums in one launch pair) run
// exactly the same arithmetic as the single ones.
template <typename T>
__device__ __forceinline__ void colsum_partial_body(const T* __restrict__ X, long ld, int R, int N, int rows_per,
                                                    float* __restrict__ part, int bx, int by) {
  int n = bx * 256 + (int)threadIdx.x;
  if (n >= N) return;
  int r0 = by * rows_per, r1 = min(R, r0 + rows_per);
  float s = 0.f;
  for (int r = r0; r < r1; ++r) s += (float)X[(long)r * ld + n];
  part[(long)by * N + n] = s;
}
template <typename T>
__global__ void colsum_partial_kernel(const T* __restrict__ X, long ld, int R, int N, int rows_per,
                                      float* __restrict__ part) {
  colsum_partial_body<T>(X, ld, R, N, rows_per, part, blockIdx.x, blockIdx.y);
}
// 16-byte rows chunks per thread (VEC columns), 4 rows in flight per iteration
template <typename T>
__device__ __forceinline__ void colsum_partial_vec_body(const T* __restrict__ X, long ld, int R, int N, int rows_per,
                                                        float* __restrict__ part, int bx, int by) {
  constexpr int VEC = 16 / sizeof(T);
  const int n = (bx * 256 + (int)threadIdx.x) * VEC;
  if (n >= N) return;
  const int r0 = by * rows_per, r1 = min(R, r0 + rows_per);
  float acc[VEC];
#pragma unroll
  for (int j = 0; j < VEC; ++j) acc[j] = 0.f;
  int r = r0;
  for (; r + 4 <= r1; r += 4) {
    uint4 u[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) u[q] = *(const uint4*)(X + (long)(r + q) * ld + n);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const T* h = (const T*)&u[q];
#pragma unroll
      for (int j = 0; j < VEC; ++j) acc[j] += (float)h[j];
    }
  }
  for (; r < r1; ++r) {
    uint4 u = *(const uint4*)(X + (long)r * ld + n);
    const T* h = (const T*)&u;
#pragma unroll
    for (int j = 0; j < VEC; ++j) acc[j] += (float)h[j];
  }
#pragma unroll
  for (int j = 0; j < VEC; ++j) part[(long)by * N + n + j] = acc[j];
}
template <typename T>
__global__ void colsum_partial_vec_kernel(const T* __restrict__ X, long ld, int R, int N, int rows_per,
                                          float* __restrict__ part) {
  colsum_partial_vec_body<T>(X, ld, R, N, rows_per, part, blockIdx.x, blockIdx.y);
}

// N output columns; the partials have NP >= N columns per row chunk (NP > N: the vector partials ran over the padded
// width)
__device__ __forceinline__ void colsum_final_body(const float* __restrict__ part, int RS, int N, int NP,
                                                  float* __restrict__ out, int accumulate, float* __restrict__ out2,
                                                  int bx) {
  int n = bx * 256 + (int)threadIdx.x;
  if (n >= N) return;
  // four independent partial sums (a single chain serialises RS L2 round trips), fixed order
  float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
  int i = 0;
  for (; i + 4 <= RS; i += 4) {
    s0 += part[(long)i * NP + n];
    s1 += part[(long)(i + 1) * NP + n];
    s2 += part[(long)(i + 2) * NP + n];
    s3 += part[(long)(i + 3) * NP + n];
  }
  for (; i < RS; ++i) s0 += part[(long)i * NP + n];
  const float s = (s0 + s1) + (s2 + s3);
  out[n] = accumulate ? out[n] + s : s;
  if (out2) out2[n] = accumulate ? out2[n] + s : s;
}
__global__ void colsum_final_kernel(const float* __restrict__ part, int RS, int N, int NP, float* __restrict__ out,
                                    int accumulate, float* __restrict__ out2) {
  colsum_final_body(part, RS, N, NP, out, accumulate, out2, blockIdx.x);
}

// geometry of one column sum (shared by sat_colsum and sat_colsum_multi): RS row chunks of rows_per rows; np columns
// of partials (N, or N rounded up to the vector width when the caller's rows are readable that far: the decoder's
// zero-padded d logits, whose odd BERT vocabulary otherwise took the scalar kernel)
struct ColsumPlan {
  bool vok;
  int colblocks, RS, rows_per, np;
};
inline ColsumPlan colsum_plan(const void* X, int dtype, long ld, int R, int N, int readable = 0) {
  ColsumPlan p;
  const int vec = dtype == SAT_BF16 ? 8 : 4;
  const int nr = (N + vec - 1) / vec * vec;
  p.vok = (N % vec == 0 || (readable && nr <= ld)) && ld % vec == 0 && ((uintptr_t)X & 15) == 0;
  p.np = p.vok ? nr : N;
  p.colblocks = sat_cdiv(N, 256 * (p.vok ? vec : 1));
  int RS = 1;
  while (p.colblocks * RS < 512 && RS < 64 && (R + RS * 2 - 1) / (RS * 2) >= 16) RS *= 2;
  int rows_per = sat_cdiv(R, RS);
  RS = sat_cdiv(R, rows_per > 0 ? rows_per : 1);
  if (R <= 0) { RS = 1; rows_per = 0; }
  p.RS = RS;
  p.rows_per = rows_per;
  return p;
}

constexpr int kColsumMaxSegs = 8;
struct ColsumMultiArgs {
  int n;
  struct Seg {
    const void* X; long ld; int R, N, np, dtype, vok, colblocks, RS, rows_per, accumulate;
    int blk0, fblk0;            // first partial / final block of this segment
    float* part; float* out; float* out2;
  } seg[kColsumMaxSegs];
};
__device__ __forceinline__ int colsum_seg_of(const ColsumMultiArgs& a, int b, bool final_pass) {
  int i = 0;
  for (int k = 1; k < a.n; ++k)
    if ((final_pass ? a.seg[k].fblk0 : a.seg[k].blk0) <= b) i = k;
  return i;
}
__global__ void colsum_multi_partial_kernel(ColsumMultiArgs a) {
  const int b = blockIdx.x;
  const auto& sg = a.seg[colsum_seg_of(a, b, false)];
  const int lb = b - sg.blk0, bx = lb % sg.colblocks, by = lb / sg.colblocks;
  if (sg.vok) {
    if (sg.dtype == SAT_BF16) colsum_partial_vec_body<bf16>((const bf16*)sg.X, sg.ld, sg.R, sg.np, sg.rows_per, sg.part, bx, by);
    else colsum_partial_vec_body<float>((const float*)sg.X, sg.ld, sg.R, sg.np, sg.rows_per, sg.part, bx, by);
  } else {
    if (sg.dtype == SAT_BF16) colsum_partial_body<bf16>((const bf16*)sg.X, sg.ld, sg.R, sg.N, sg.rows_per, sg.part, bx, by);
    else colsum_partial_body<float>((const float*)sg.X, sg.ld, sg.R, sg.N, sg.rows_per, sg.part, bx, by);
  }
}
__global__ void colsum_multi_final_kernel(ColsumMultiArgs a) {
  const int b = blockIdx.x;
  const auto& sg = a.seg[colsum_seg_of(a, b, true)];
  colsum_final_body(sg.part, sg.RS, sg.N, sg.np, sg.out, sg.accumulate, sg.out2, b - sg.fblk0);
}

// zero several fp32 row blocks (rows x cols at a row stride ld; contiguous ranges as one row) in one launch
constexpr int kZeroMaxSegs = 12;
struct ZeroMultiArgs {
  int n;
  float* p[kZeroMaxSegs];
  long rows[kZeroMaxSegs], cols[kZeroMaxSegs], ld[kZeroMaxSegs];
};
#ifndef SAT_ZERO_CPOL   // diagnostics builds: the accumulator zeroing's store policy (sat_common.h)
#define SAT_ZERO_CPOL SAT_OUT_CPOL
#endif
__global__ void zero_multi_kernel(ZeroMultiArgs a) {
  const long stride = (long)gridDim.x * blockDim.x;
  for (int k = 0; k < a.n; ++k) {
    float* p = a.p[k];
    const long R = a.rows[k], C = a.cols[k], ld = a.ld[k];
    // 16-B write-through stores while the segment's byte extent fits the buffer resource (< 2 GiB)
    if (((uintptr_t)p & 15) == 0 && C % 4 == 0 && ld % 4 == 0 && 4 * ((R - 1) * ld + C) < (1L << 31)) {
      const long c4 = C >> 2, n4 = R * c4;
      // write-through zeros (sat_common.h): megabytes of gradient accumulators that would otherwise sit dirty in
      // the L2s while the encoder's kernel boundaries run beside this graph
      const __amdgpu_buffer_rsrc_t rp = sat_out_rsrc(p, 4 * ((R - 1) * ld + C));
      for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n4; i += stride) {
        const long r = i / c4;
        sat_st16<SAT_ZERO_CPOL>(rp, (unsigned)((r * ld + 4 * (i - r * c4)) * 4), make_uint4(0u, 0u, 0u, 0u));
      }
    } else {
      for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < R * C; i += stride) {
        const long r = i / C;
        p[r * ld + (i - r * C)] = 0.f;
      }
    }
  }
}

// ---- embedding gather: out[r, :] = W[tok[r], :] ------------------------------
template <typename T>
__global__ void embed_gather_kernel(const float* __restrict__ W, const int32_t* __restrict__ tok, int R,
                                    long tok_stride_b, int T1, int E, T* __restrict__ out, long out_ld) {
  // row r = b*T1 + t ; tokens laid out [B][T1] with row stride tok_stride_b
  int r = blockIdx.x;
  if (r >= R) return;
  int b = r / T1, t = r - b * T1;
  int id = tok[(long)b * tok_stride_b + t];
  const float* src = W + (long)id * E;
  T* dst = out + (long)r * out_ld;
  for (int e = threadIdx.x; e < E; e += blockDim.x) dst[e] = (T)src[e];
}

// teacher forcing: the fed tokens straight from the int64 captions (tok[b, t] = captions[b, t], t < T-1) and
// their embedding rows in one launch
template <typename OT>
__global__ void embed_gather_captions_kernel(const float* __restrict__ W, const int64_t* __restrict__ caps, int R,
                                             int T, int T1, int E, OT* __restrict__ out, long out_ld,
                                             int32_t* __restrict__ tok) {
  const int r = blockIdx.x;
  if (r >= R) return;
  const int b = r / T1, t = r - b * T1;
  const int id = (int)caps[(long)b * T + t];
  if (threadIdx.x == 0) tok[r] = id;
  const float* src = W + (long)id * E;
  OT* dst = out + (long)r * out_ld;
  if ((E & 3) == 0 && ((uintptr_t)src & 15) == 0) {
    for (int e = 4 * threadIdx.x; e < E; e += 4 * blockDim.x) {
      const float4 v = *(const float4*)(src + e);
      dst[e] = (OT)v.x; dst[e + 1] = (OT)v.y; dst[e + 2] = (OT)v.z; dst[e + 3] = (OT)v.w;
    }
  } else {
    for (int e = threadIdx.x; e < E; e += blockDim.x) dst[e] = (OT)src[e];
  }
}

// ---- embedding backward: G[tok[r], :] += dX[r, :] (fp32 atomics) -------------
__global__ void embed_scatter_kernel(const float* __restrict__ dX, const int32_t* __restrict__ tok, int R, int E,
                                     float* __restrict__ G) {
  int r = blockIdx.x;
  if (r >= R) return;
  int id = tok[r];
  const float* src = dX + (long)r * E;
  float* dst = G + (long)id * E;
  for (int e = threadIdx.x; e < E; e += blockDim.x) atomicAdd(dst + e, src[e]);
}

// ---- deterministic embedding backward: per-token sums in row order (sat_embed_scatter_add_sorted) ----
// 1. rank sort: every row's place in (token, row) order -- #rows with a smaller token + #earlier rows with the same
//    token -- counted against all R tokens held in LDS (R^2 compares spread over R threads, no barriers between
//    passes); it also records each sorted position's token segment [start, end);
// 2. the sorted positions are cut into pieces of kEmbPiece: a piece loads its rows' gradients at once and sums each run
//    of one token in row order; a run that is a whole segment is added to G[tok] directly, a run cut by a piece
//    boundary goes to the piece's head (slot 0) or tail (slot 1) partial;
// 3. the piece where a cut segment starts adds that segment's partials in a fixed tree order (four interleaved piece
//    chains, then the chains in order) and adds the sum to G[tok].
// Every G row is written by one thread per column, once: the same bits on every run.
constexpr int kEmbSortMax = 16384, kEmbPiece = 32;
// 16 rows per workgroup x 16 parts of the token range per row (thread = part * 16 + row: the lanes of one part read
// the same LDS words), the parts' counts summed in LDS
constexpr int kRankRows = 16, kRankParts = 16;
__global__ __launch_bounds__(256) void embed_rank_kernel(const int32_t* __restrict__ tok, int R,
                                                         int32_t* __restrict__ perm, int32_t* __restrict__ stok,
                                                         int32_t* __restrict__ seg) {
  __shared__ __attribute__((aligned(16))) int32_t st[kEmbSortMax];
  __shared__ int cnt[3][kRankParts][kRankRows];
  const int R4 = (R + 3) & ~3;
  for (int i = threadIdx.x; i < R4; i += blockDim.x) st[i] = i < R ? tok[i] : 0x7fffffff;   // past R: no token
  __syncthreads();
  const int rl = threadIdx.x & (kRankRows - 1), part = threadIdx.x / kRankRows;
  const int r = blockIdx.x * kRankRows + rl;
  const int k = r < R ? st[r] : 0;
  // this part's range of the (4-token) words
  const int words = R4 / 4, per = (words + kRankParts - 1) / kRankParts;
  const int w0 = part * per, w1 = min(words, w0 + per);
  int less = 0, before = 0, eq = 0;
#pragma unroll 4
  for (int wi = w0; wi < w1; ++wi) {
    const int i = 4 * wi;
    const int4 x = *(const int4*)(st + i);
    less += (x.x < k) + (x.y < k) + (x.z < k) + (x.w < k);
    eq += (x.x == k) + (x.y == k) + (x.z == k) + (x.w == k);
    before += ((x.x == k) & (i < r)) + ((x.y == k) & (i + 1 < r)) + ((x.z == k) & (i + 2 < r)) + ((x.w == k) & (i + 3 < r));
  }
  cnt[0][part][rl] = less; cnt[1][part][rl] = eq; cnt[2][part][rl] = before;
  __syncthreads();
  if (part != 0 || r >= R) return;
  for (int q = 1; q < kRankParts; ++q) { less += cnt[0][q][rl]; eq += cnt[1][q][rl]; before += cnt[2][q][rl]; }
  const int pos = less + before;
  perm[pos] = r;
  stok[pos] = k;
  seg[2 * pos] = less;          // the token's segment of sorted positions: [less, less + eq)
  seg[2 * pos + 1] = less + eq;
}

// grid (pieces, ceil(E / 256)), 64 threads: thread owns 4 columns
__global__ __launch_bounds__(64) void embed_segsum_kernel(const float* __restrict__ dX, int E,
                                                          const int32_t* __restrict__ perm,
                                                          const int32_t* __restrict__ stok,
                                                          const int32_t* __restrict__ seg, int R, float* G,
                                                          float* __restrict__ part, int accumulate) {
  const int p = blockIdx.x, e = blockIdx.y * 256 + 4 * threadIdx.x;
  const int s0 = p * kEmbPiece, n = min(R - s0, kEmbPiece);
  __shared__ int sr[kEmbPiece], stk[kEmbPiece], sa[kEmbPiece], sb[kEmbPiece];
  if ((int)threadIdx.x < n) {
    sr[threadIdx.x] = perm[s0 + threadIdx.x];
    stk[threadIdx.x] = stok[s0 + threadIdx.x];
    sa[threadIdx.x] = seg[2 * (s0 + threadIdx.x)];
    sb[threadIdx.x] = seg[2 * (s0 + threadIdx.x) + 1];
  }
  __syncthreads();
  if (e >= E) return;
  float4 x[kEmbPiece];   // every row of the piece requested before the first add
#pragma unroll
  for (int i = 0; i < kEmbPiece; ++i)
    x[i] = i < n ? *(const float4*)(dX + (long)sr[i] * E + e) : make_float4(0.f, 0.f, 0.f, 0.f);
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  int rs = 0;
#pragma unroll
  for (int i = 0; i < kEmbPiece; ++i) {
    if (i < n) {
      acc = f4add(acc, x[i]);
      if (i + 1 == n || stk[i + 1] != stk[i]) {   // the run [rs, i] of token stk[i] ends in this piece
        if (sa[i] == s0 + rs && sb[i] == s0 + i + 1) {
          // beta = 0: G was zeroed on this stream (the decoder's zeroing launch), 0 + acc is acc: store only
          float4* g = (float4*)(G + (long)stk[i] * E + e);
          *g = accumulate ? f4add(*g, acc) : acc;
        } else {
          *(float4*)(part + ((long)p * 2 + (rs == 0 ? 0 : 1)) * E + e) = acc;
        }
        acc = make_float4(0.f, 0.f, 0.f, 0.f);
        rs = i + 1;
      }
    }
  }
}

// grid (pieces, ceil(E / 256)), 256 threads = 4 chains x 64 threads
__global__ __launch_bounds__(256) void embed_segfix_kernel(const int32_t* __restrict__ stok,
                                                           const int32_t* __restrict__ seg, int R, int E,
                                                           const float* __restrict__ part, float* G,
                                                           int accumulate) {
  const int p = blockIdx.x, chain = threadIdx.x >> 6, e = blockIdx.y * 256 + 4 * (threadIdx.x & 63);
  const int s0 = p * kEmbPiece, s1 = min(R, s0 + kEmbPiece);
  const int sa = seg[2 * (s1 - 1)], sb = seg[2 * (s1 - 1) + 1];   // the segment of the piece's last position
  if (sb <= s1 || sa < s0) return;   // the segment ends in this piece, or started in an earlier one
  __shared__ float4 cs[3][64];
  const int p1 = (sb - 1) / kEmbPiece;   // the piece where the segment ends
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  if (e < E) {
    // chain c: the head partials of pieces p + 1 + c, p + 5 + c, .. <= p1, eight loads in flight at a time
    for (int q0 = p + 1 + chain; q0 <= p1; q0 += 32) {
      float4 y[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int q = q0 + 4 * u;
        y[u] = q <= p1 ? *(const float4*)(part + (long)q * 2 * E + e) : make_float4(0.f, 0.f, 0.f, 0.f);
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) acc = f4add(acc, y[u]);
    }
  }
  if (chain > 0) cs[chain - 1][threadIdx.x & 63] = acc;
  __syncthreads();
  if (chain != 0 || e >= E) return;
  const float4 own = *(const float4*)(part + ((long)p * 2 + (sa == s0 ? 0 : 1)) * E + e);
  const float4 sum = f4add(own, f4add(f4add(acc, cs[0][threadIdx.x]), f4add(cs[1][threadIdx.x], cs[2][threadIdx.x])));
  float4* g = (float4*)(G + (long)stok[s1 - 1] * E + e);
  *g = accumulate ? f4add(*g, sum) : sum;
}

// ---- greedy argmax over V (first index wins ties, decoder.py:132) ----------
__device__ __forceinline__ bool am_better(float x, int xi, float y, int yi) { return sat_argmax_better(x, xi, y, yi); }
__device__ __forceinline__ void am_wave_reduce(float& v, int& i) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float ov = __shfl_xor(v, o, 64);
    const int oi = __shfl_xor(i, o, 64);
    if (am_better(ov, oi, v, i)) { v = ov; i = oi; }
  }
}
// One 256-thread workgroup per row.  Vector path (16-B aligned rows): every thread requests all
// its 16-B vectors of a 256 x AM_NV x VEC-element pass before the first compare (the old
// element-per-iteration loop waited out one load latency per element: 17.6 us per 128 x 10000 row
// block), then a shuffle reduction per wave and one LDS exchange across the four waves.
constexpr int AM_NV = 8;
template <typename T, bool VECP>
__global__ __launch_bounds__(256) void argmax_kernel(const T* __restrict__ X, long ld, int V, int32_t* __restrict__ out,
                                                     long out_stride, const float* __restrict__ emb, int E,
                                                     T* __restrict__ emb_out, long emb_ld) {
  constexpr int VEC = 16 / sizeof(T);
  const int b = blockIdx.x, tid = threadIdx.x;
  const T* row = X + (long)b * ld;
  float best = -INFINITY;
  int bi = 0x7fffffff;
  if constexpr (VECP) {
    const int nvec = V / VEC;
    for (int base = 0; base < nvec; base += 256 * AM_NV) {
      uint4 u[AM_NV];
#pragma unroll
      for (int j = 0; j < AM_NV; ++j) {
        const int vi = base + j * 256 + tid;
        u[j] = vi < nvec ? *(const uint4*)(row + (long)vi * VEC) : make_uint4(0, 0, 0, 0);
      }
#pragma unroll
      for (int j = 0; j < AM_NV; ++j) {
        const int vi = base + j * 256 + tid;
        if (vi < nvec) {
          const T* h = (const T*)&u[j];
#pragma unroll
          for (int e = 0; e < VEC; ++e) {
            const float x = (float)h[e];
            if (am_better(x, vi * VEC + e, best, bi)) { best = x; bi = vi * VEC + e; }
          }
        }
      }
    }
    for (int v = nvec * VEC + tid; v < V; v += 256) {
      const float x = (float)row[v];
      if (am_better(x, v, best, bi)) { best = x; bi = v; }
    }
  } else {
    for (int v = tid; v < V; v += 256) {
      const float x = (float)row[v];
      if (am_better(x, v, best, bi)) { best = x; bi = v; }
    }
  }
  am_wave_reduce(best, bi);
  __shared__ float sv[4];
  __shared__ int si[4];
  if ((tid & 63) == 0) { sv[tid >> 6] = best; si[tid >> 6] = bi; }
  __syncthreads();
  best = sv[0]; bi = si[0];
#pragma unroll
  for (int w = 1; w < 4; ++w)
    if (am_better(sv[w], si[w], best, bi)) { best = sv[w]; bi = si[w]; }
  int id = bi;
  if (id < 0 || id >= V) id = 0;
  if (tid == 0 && out) out[(long)b * out_stride] = id;
  if (emb_out) {
    const float* src = emb + (long)id * E;
    for (int e = tid; e < E; e += 256) emb_out[(long)b * emb_ld + e] = (T)src[e];
  }
}

// ---- Adam (torch.optim.Adam single-tensor algorithm) ------------------------
// torch's single-tensor Adam arithmetic for one element (exp_avg.lerp_(grad, 1-beta1): the weight < 0.5
// branch of at::lerp; exp_avg_sq.mul_(beta2).addcmul_(grad, grad, 1-beta2); addcdiv_ with the bias corrections)
__device__ __forceinline__ void adam_elem(float& pi, float gi, float& mi, float& vi, float w1, float b2, float eps,
                                          float step_size, float bc2_sqrt) {
  mi = mi + w1 * (gi - mi);
  vi = vi * b2 + (1.f - b2) * gi * gi;
  const float denom = sqrtf(vi) / bc2_sqrt + eps;
  pi = pi + (-step_size) * (mi / denom);
}
// 16-byte vectors of 4 elements where the range is 16-B aligned (the decoder's flat parameter groups are
// 64-element aligned), the scalar form for the tail / unaligned ranges: the same per-element arithmetic
__global__ void adam_kernel(float* __restrict__ p, const float* __restrict__ g, float* __restrict__ m,
                            float* __restrict__ v, bf16* __restrict__ p_lp, long n, float b1, float b2, float eps,
                            float step_size, float bc2_sqrt) {
  const float w1 = 1.f - b1;
  const long stride = (long)gridDim.x * blockDim.x;
  const bool vec = ((((uintptr_t)p | (uintptr_t)g | (uintptr_t)m | (uintptr_t)v) & 15) == 0) &&
                   (((uintptr_t)p_lp & 7) == 0);
  const long n4 = vec ? n >> 2 : 0;
  // plain write-back stores (write-through measured neutral here, profiles/r4_s14 / r4_s19)
  const __amdgpu_buffer_rsrc_t rp = sat_out_rsrc(p, 4 * n), rm = sat_out_rsrc(m, 4 * n), rv = sat_out_rsrc(v, 4 * n);
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n4; i += stride) {
    float4 pp = ((float4*)p)[i], mm = ((float4*)m)[i], vv = ((float4*)v)[i];
    const float4 gg = ((const float4*)g)[i];
    adam_elem(pp.x, gg.x, mm.x, vv.x, w1, b2, eps, step_size, bc2_sqrt);
    adam_elem(pp.y, gg.y, mm.y, vv.y, w1, b2, eps, step_size, bc2_sqrt);
    adam_elem(pp.z, gg.z, mm.z, vv.z, w1, b2, eps, step_size, bc2_sqrt);
    adam_elem(pp.w, gg.w, mm.w, vv.w, w1, b2, eps, step_size, bc2_sqrt);
    sat_st16<0>(rp, (unsigned)(i * 16), *(const uint4*)&pp);
    sat_st16<0>(rm, (unsigned)(i * 16), *(const uint4*)&mm);
    sat_st16<0>(rv, (unsigned)(i * 16), *(const uint4*)&vv);
    if (p_lp) {
      uint2 o;
      bf16* ob = (bf16*)&o;
      ob[0] = (bf16)pp.x; ob[1] = (bf16)pp.y; ob[2] = (bf16)pp.z; ob[3] = (bf16)pp.w;
      ((uint2*)p_lp)[i] = o;
    }
  }
  for (long i = (n4 << 2) + blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += stride) {
    float pi = p[i], mi = m[i], vi = v[i];
    adam_elem(pi, g[i], mi, vi, w1, b2, eps, step_size, bc2_sqrt);
    m[i] = mi; v[i] = vi; p[i] = pi;
    if (p_lp) p_lp[i] = (bf16)pi;
  }
}

}  // namespace

// ============================ internal launchers ============================
int sat_mean_rows(const void* a, int B, int L, int D, int dtype, float* out_f32, void* out_t, hipStream_t s) {
  const int vec = dtype == SAT_BF16 ? 8 : 4;
  if (D % vec == 0 && ((uintptr_t)a & 15) == 0) {
    dim3 g(sat_cdiv(D / vec, 256), B);
    if (dtype == SAT_BF16)
      hipLaunchKernelGGL(mean_rows_vec_kernel<bf16>, g, dim3(256), 0, s, (const bf16*)a, L, D, out_f32, (bf16*)out_t);
    else
      hipLaunchKernelGGL(mean_rows_vec_kernel<float>, g, dim3(256), 0, s, (const float*)a, L, D, out_f32, (float*)out_t);
    return (int)hipGetLastError();
  }
  dim3 grid(sat_cdiv(D, 256), B);
  if (dtype == SAT_BF16)
    hipLaunchKernelGGL(mean_rows_kernel<bf16>, grid, dim3(256), 0, s, (const bf16*)a, L, D, out_f32, (bf16*)out_t);
  else
    hipLaunchKernelGGL(mean_rows_kernel<float>, grid, dim3(256), 0, s, (const float*)a, L, D, out_f32, (float*)out_t);
  return (int)hipGetLastError();
}

int sat_colsum(const void* X, int dtype, long ld, int R, int N, float* out, int accumulate, float* out2,
               float* scratch, hipStream_t s, int cols_readable) {
  if (N <= 0) return 0;
  const ColsumPlan p = colsum_plan(X, dtype, ld, R, N, cols_readable);
  dim3 g1(p.colblocks, p.RS);
  if (p.vok) {
    if (dtype == SAT_BF16)
      hipLaunchKernelGGL(colsum_partial_vec_kernel<bf16>, g1, dim3(256), 0, s, (const bf16*)X, ld, R, p.np, p.rows_per, scratch);
    else
      hipLaunchKernelGGL(colsum_partial_vec_kernel<float>, g1, dim3(256), 0, s, (const float*)X, ld, R, p.np, p.rows_per, scratch);
  } else if (dtype == SAT_BF16)
    hipLaunchKernelGGL(colsum_partial_kernel<bf16>, g1, dim3(256), 0, s, (const bf16*)X, ld, R, N, p.rows_per, scratch);
  else
    hipLaunchKernelGGL(colsum_partial_kernel<float>, g1, dim3(256), 0, s, (const float*)X, ld, R, N, p.rows_per, scratch);
  hipLaunchKernelGGL(colsum_final_kernel, dim3(sat_cdiv(N, 256)), dim3(256), 0, s, scratch, p.RS, N, p.np, out, accumulate,
                     out2);
  return (int)hipGetLastError();
}

int sat_colsum_multi(const SatColsumSeg* segs, int n, float* scratch, hipStream_t s) {
  if (n <= 0) return 0;
  if (n > kColsumMaxSegs) return (int)hipErrorInvalidValue;
  ColsumMultiArgs a{};
  int blk = 0, fblk = 0, k = 0;
  long off = 0;
  for (int i = 0; i < n; ++i) {
    const SatColsumSeg& g = segs[i];
    if (g.N <= 0) continue;
    const ColsumPlan p = colsum_plan(g.X, g.dtype, g.ld, g.R, g.N, g.cols_readable);
    auto& sg = a.seg[k++];
    sg.X = g.X; sg.ld = g.ld; sg.R = g.R; sg.N = g.N; sg.np = p.np; sg.dtype = g.dtype; sg.vok = p.vok;
    sg.colblocks = p.colblocks; sg.RS = p.RS; sg.rows_per = p.rows_per; sg.accumulate = g.accumulate;
    sg.blk0 = blk; sg.fblk0 = fblk;
    sg.part = scratch + off; sg.out = g.out; sg.out2 = g.out2;
    blk += p.colblocks * p.RS;
    fblk += sat_cdiv(g.N, 256);
    off += (long)p.RS * p.np;
  }
  a.n = k;
  if (k == 0) return 0;
  hipLaunchKernelGGL(colsum_multi_partial_kernel, dim3(blk), dim3(256), 0, s, a);
  hipLaunchKernelGGL(colsum_multi_final_kernel, dim3(fblk), dim3(256), 0, s, a);
  return (int)hipGetLastError();
}

int sat_zero_segs(const SatZeroSeg* seg, int n, hipStream_t s) {
  if (n <= 0) return 0;
  if (n > kZeroMaxSegs) return (int)hipErrorInvalidValue;
  ZeroMultiArgs a{};
  long tot = 0;
  for (int i = 0; i < n; ++i) {
    a.p[i] = seg[i].p;
    a.rows[i] = seg[i].rows; a.cols[i] = seg[i].cols; a.ld[i] = seg[i].ld;
    tot += seg[i].rows * seg[i].cols;
  }
  a.n = n;
  long g = (tot / 4 + 255) / 256;
  g = g < 1 ? 1 : (g > 2048 ? 2048 : g);
  hipLaunchKernelGGL(zero_multi_kernel, dim3((int)g), dim3(256), 0, s, a);
  return (int)hipGetLastError();
}
int sat_zero_multi(float* const* ptrs, const long* counts, int n, hipStream_t s) {
  if (n > kZeroMaxSegs) return (int)hipErrorInvalidValue;
  SatZeroSeg seg[kZeroMaxSegs];
  for (int i = 0; i < n; ++i) seg[i] = SatZeroSeg{ptrs[i], 1, counts[i], counts[i]};
  return sat_zero_segs(seg, n, s);
}
// up to 64 row chunks of the (possibly padded: + up to 7 columns per segment, <= 8 segments) partial width
size_t sat_colsum_scratch_floats(int R, int N) { (void)R; return (size_t)64 * ((N > 0 ? N : 1) + 64); }

int sat_embed_gather(const float* W, const int32_t* tok, int B, int T1, long tok_stride_b, int E, int dtype,
                     void* out, long out_ld, hipStream_t s) {
  int R = B * T1;
  if (R <= 0) return 0;
  if (dtype == SAT_BF16)
    hipLaunchKernelGGL(embed_gather_kernel<bf16>, dim3(R), dim3(256), 0, s, W, tok, R, tok_stride_b, T1, E,
                       (bf16*)out, out_ld);
  else
    hipLaunchKernelGGL(embed_gather_kernel<float>, dim3(R), dim3(256), 0, s, W, tok, R, tok_stride_b, T1, E,
                       (float*)out, out_ld);
  return (int)hipGetLastError();
}

int sat_embed_gather_captions(const float* W, const int64_t* caps, int B, int T, int E, int dtype, void* out,
                              long out_ld, int32_t* tok, hipStream_t s) {
  const int T1 = T - 1, R = B * T1;
  if (R <= 0) return 0;
  if (dtype == SAT_BF16)
    hipLaunchKernelGGL(embed_gather_captions_kernel<bf16>, dim3(R), dim3(128), 0, s, W, caps, R, T, T1, E, (bf16*)out,
                       out_ld, tok);
  else
    hipLaunchKernelGGL(embed_gather_captions_kernel<float>, dim3(R), dim3(128), 0, s, W, caps, R, T, T1, E,
                       (float*)out, out_ld, tok);
  return (int)hipGetLastError();
}

int sat_embed_scatter_add(const float* dX, const int32_t* tok, int R, int E, float* G, hipStream_t s) {
  if (R <= 0) return 0;
  hipLaunchKernelGGL(embed_scatter_kernel, dim3(R), dim3(256), 0, s, dX, tok, R, E, G);
  return (int)hipGetLastError();
}

int sat_embed_sorted_max_rows() { return kEmbSortMax; }
// workspace: perm [R], stok [R], seg [2R] (int32), then the piece partials [pieces][2][E] fp32
static long embed_part_off(int R) { return (4L * R * 4 + 255) / 256 * 256; }
size_t sat_embed_sorted_ws_bytes(int R, int E) {
  return (size_t)(embed_part_off(R) + (long)sat_cdiv(R, kEmbPiece) * 2 * E * 4);
}
int sat_embed_scatter_add_sorted(const float* dX, const int32_t* tok, int R, int E, float* G, int accumulate, void* ws,
                                 hipStream_t s) {
  if (R <= 0) return 0;
  if (R > kEmbSortMax || E % 4 || ((uintptr_t)dX & 15) || ((uintptr_t)G & 15) || !ws) return (int)hipErrorInvalidValue;
  int32_t* perm = (int32_t*)ws;
  int32_t* stok = perm + R;
  int32_t* seg = stok + R;
  float* part = (float*)((char*)ws + embed_part_off(R));
  const int pieces = sat_cdiv(R, kEmbPiece);
  hipLaunchKernelGGL(embed_rank_kernel, dim3(sat_cdiv(R, kRankRows)), dim3(kRankRows * kRankParts), 0, s, tok, R,
                     perm, stok, seg);
  const dim3 g(pieces, sat_cdiv(E, 256));
  hipLaunchKernelGGL(embed_segsum_kernel, g, dim3(64), 0, s, dX, E, perm, stok, seg, R, G, part, accumulate);
  hipLaunchKernelGGL(embed_segfix_kernel, g, dim3(256), 0, s, stok, seg, R, E, part, G, accumulate);
  return (int)hipGetLastError();
}

int sat_argmax_rows(const void* X, int dtype, long ld, int B, int V, int32_t* out, long out_stride,
                    const float* emb, int E, void* emb_out, long emb_ld, hipStream_t s) {
  const int esz = dtype == SAT_BF16 ? 2 : 4;
  const bool vec = ((uintptr_t)X & 15) == 0 && (ld * esz) % 16 == 0;
  if (dtype == SAT_BF16) {
    if (vec) hipLaunchKernelGGL((argmax_kernel<bf16, true>), dim3(B), dim3(256), 0, s, (const bf16*)X, ld, V, out, out_stride, emb, E, (bf16*)emb_out, emb_ld);
    else hipLaunchKernelGGL((argmax_kernel<bf16, false>), dim3(B), dim3(256), 0, s, (const bf16*)X, ld, V, out, out_stride, emb, E, (bf16*)emb_out, emb_ld);
  } else {
    if (vec) hipLaunchKernelGGL((argmax_kernel<float, true>), dim3(B), dim3(256), 0, s, (const float*)X, ld, V, out, out_stride, emb, E, (float*)emb_out, emb_ld);
    else hipLaunchKernelGGL((argmax_kernel<float, false>), dim3(B), dim3(256), 0, s, (const float*)X, ld, V, out, out_stride, emb, E, (float*)emb_out, emb_ld);
  }
  return (int)hipGetLastError();
}

int sat_cast_launch(const void* x, int xd, void* y, int yd, long n, hipStream_t s) {
  if (n <= 0) return 0;
  int g = grid_for(n);
  if (xd == SAT_F32 && yd == SAT_BF16) hipLaunchKernelGGL((cast_kernel<float, bf16>), dim3(g), dim3(256), 0, s, (const float*)x, (bf16*)y, n);
  else if (xd == SAT_BF16 && yd == SAT_F32) hipLaunchKernelGGL((cast_kernel<bf16, float>), dim3(g), dim3(256), 0, s, (const bf16*)x, (float*)y, n);
  else if (xd == SAT_F32) hipLaunchKernelGGL((cast_kernel<float, float>), dim3(g), dim3(256), 0, s, (const float*)x, (float*)y, n);
  else hipLaunchKernelGGL((cast_kernel<bf16, bf16>), dim3(g), dim3(256), 0, s, (const bf16*)x, (bf16*)y, n);
  return (int)hipGetLastError();
}

// ================================ C ABI =====================================
extern "C" int sat_abi_version(void) { return SAT_ABI_VERSION; }

extern "C" const char* sat_error_string(int code) {
  if (code == 0) return "success";
  if (code == SAT_ERR_INVALID) return "invalid argument or unsupported shape";
  return hipGetErrorString((hipError_t)code);
}

extern "C" int sat_cast(const void* x, int x_dtype, void* y, int y_dtype, int64_t n, void* stream) {
  SAT_REQUIRE(x && y && n >= 0);
  return sat_cast_launch(x, x_dtype, y, y_dtype, n, (hipStream_t)stream);
}

extern "C" int sat_mean_rows_abi(const void* a, int B, int L, int D, int dtype, float* out_f32, void* out_t,
                                 void* stream) {
  SAT_REQUIRE(a && B > 0 && L > 0 && D > 0);
  return sat_mean_rows(a, B, L, D, dtype, out_f32, out_t, (hipStream_t)stream);
}

extern "C" int sat_nchw_to_nhwc(int N, int C, int H, int W, int Cp, int dtype, const float* x, void* y,
                                void* stream) {
  SAT_REQUIRE(x && y && Cp >= C && C > 0);
  long pix = (long)N * H * W;
  int g = grid_for(pix);
  if (dtype == SAT_BF16)
    hipLaunchKernelGGL(nchw_to_nhwc_kernel<bf16>, dim3(g), dim3(256), 0, (hipStream_t)stream, x, (bf16*)y, N, C, H, W, Cp);
  else
    hipLaunchKernelGGL(nchw_to_nhwc_kernel<float>, dim3(g), dim3(256), 0, (hipStream_t)stream, x, (float*)y, N, C, H, W, Cp);
  return (int)hipGetLastError();
}

extern "C" int sat_nchw_to_s2d(int N, int C, int H, int W, int dtype, const float* x, void* y, void* stream) {
  SAT_REQUIRE(x && y && C > 0 && 4 * C <= 16 && H % 2 == 0 && W % 2 == 0);
  const int g = grid_for((long)N * (H / 2) * (W / 2));
  if (dtype == SAT_BF16 && C == 3 && ((uintptr_t)x & 7) == 0 && ((uintptr_t)y & 15) == 0) {
    const long total = (long)N * (H / 2) * (W / 2);
    hipLaunchKernelGGL(nchw3_to_s2d16_bf16_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0,
                       (hipStream_t)stream, x, (bf16*)y, N, H, W);
  } else if (dtype == SAT_BF16)
    hipLaunchKernelGGL(nchw_to_s2d16_kernel<bf16>, dim3(g), dim3(256), 0, (hipStream_t)stream, x, (bf16*)y, N, C, H, W);
  else
    hipLaunchKernelGGL(nchw_to_s2d16_kernel<float>, dim3(g), dim3(256), 0, (hipStream_t)stream, x, (float*)y, N, C, H, W);
  return (int)hipGetLastError();
}

extern "C" int sat_maxpool2d_nhwc(int N, int H, int W, int C, int k, int stride, int pad, int dtype, const void* x,
                                  void* y, int OH, int OW, void* stream) {
  SAT_REQUIRE(x && y && k > 0 && stride > 0);
  SAT_REQUIRE(OH == (H + 2 * pad - k) / stride + 1 && OW == (W + 2 * pad - k) / stride + 1);
  SAT_REQUIRE(C % 8 == 0 && ((uintptr_t)x & 15) == 0 && ((uintptr_t)y & 15) == 0);
  long total = (long)N * OH * OW * (C / 8);
  int g = grid_for(total);
  if (dtype == SAT_BF16 && k == 3) {
    hipLaunchKernelGGL(maxpool_bf16_kernel<3>, dim3((unsigned)((total + 255) / 256)), dim3(256), 0,
                       (hipStream_t)stream, (const bf16*)x, (bf16*)y, N, H, W, C, stride, pad, OH, OW);
  } else if (dtype == SAT_BF16)
    hipLaunchKernelGGL(maxpool_kernel<bf16>, dim3(g), dim3(256), 0, (hipStream_t)stream, (const bf16*)x, (bf16*)y, N, H,
                       W, C, k, stride, pad, OH, OW);
  else
    hipLaunchKernelGGL(maxpool_kernel<float>, dim3(g), dim3(256), 0, (hipStream_t)stream, (const float*)x, (float*)y, N,
                       H, W, C, k, stride, pad, OH, OW);
  return (int)hipGetLastError();
}

extern "C" int sat_adam_step(float* param, const float* grad, float* exp_avg, float* exp_avg_sq, void* param_lp,
                             int64_t n, float beta1, float beta2, float eps, float step_size,
                             float bias_correction2_sqrt, void* stream) {
  SAT_REQUIRE(param && grad && exp_avg && exp_avg_sq && n >= 0);
  // chunks of at most 2^28 elements: the kernel's buffer resources (sat_out_rsrc) take 32-bit byte offsets
  constexpr int64_t kChunk = 1L << 28;
  for (int64_t i = 0; i < n; i += kChunk) {
    const int64_t m = n - i < kChunk ? n - i : kChunk;
    hipLaunchKernelGGL(adam_kernel, dim3(grid_for((m + 3) / 4)), dim3(256), 0, (hipStream_t)stream, param + i, grad + i,
                       exp_avg + i, exp_avg_sq + i, param_lp ? (bf16*)param_lp + i : nullptr, (long)m, beta1, beta2,
                       eps, step_size, bias_correction2_sqrt);
    SAT_LAUNCH_CHECK();
  }
  return 0;
}
