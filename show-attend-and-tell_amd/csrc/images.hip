// Streaming image input: decoded uint8 RGB images of any size -> the
// reference's transform (train.py:27-32: Resize((224, 224)) -> ToTensor -> Normalize) -> the
// encoder's first-layer layout, on the GPU.
//
// Resize is torchvision 0.16's PIL path, i.e. Pillow's two-pass 8-bit resampler (Pillow 10.1.0
// pinned by the reference's requirements.txt; unchanged through 12.x), restated from its published
// algorithm (libImaging/Resample.c: precompute_coeffs, normalize_coeffs_8bpc,
// ImagingResampleHorizontal_8bpc / Vertical_8bpc, BILINEAR support 1.0):
//   * per axis and output index: scale = in / out, filterscale = max(scale, 1), support =
//     filterscale, center = (i + 0.5) * scale, taps [xmin, xmin + n) with xmin = (int)(center -
//     support + 0.5) clamped to 0 and xmin + n = min((int)(center + support + 0.5), in); weights
//     w_x = tri((x + xmin - center + 0.5) / filterscale) normalised to sum 1 in double, then fixed
//     point int32 = (int)(w * 2^22 +- 0.5);
//   * horizontal pass first into an 8-bit intermediate, then the vertical pass; each output byte is
//     clip8((2^21 + sum_x in_x * k_x) >> 22), exactly as Pillow rounds.
// The coefficient tables are computed on the device in double with contraction off (the same IEEE
// operations as Pillow's C), so the resized bytes are bit-identical to PIL's.  ToTensor / Normalize
// are ((float)u / 255 - mean) / std in fp32 with IEEE division, bit-identical to torch's
// img.float().div(255).sub_(mean).div_(std).
//
// Layout: pixels of image b start at offsets[b] (HWC, 3 bytes per pixel); sizes[b] = (H, W).
// Work split: one workgroup per (image, 8 output rows).  The workgroup resamples the input rows
// those output rows need horizontally into LDS (at most RCAP rows x OW x 3 bytes; taller spans are
// processed in sub-chunks), then resamples vertically and writes the requested layout:
//   SAT_IMG_NCHW  [B, 3, OH, OW] fp32 (the reference's tensor),
//   SAT_IMG_NHWC  [B, OH, OW, c_pad] (dtype), channels >= 3 zero (VGG19 first conv),
//   SAT_IMG_S2D16 [B, OH/2, OW/2, 16] (dtype), channel (sy*2 + sx)*3 + c, 12..15 zero (ResNet152
//   space-to-depth stem; the same layout as sat_nchw_to_s2d).
// The whole job is one pass over the uint8 input (re-reads only where 8-row tiles' spans overlap)
// plus one write of the output: HBM-bound byte work, no MFMA.
#include "sat_common.h"
#include "sat_internal.h"

#include <cmath>

namespace {

constexpr int KMAX = 32;        // taps per output index: support <= 15.5, i.e. downscale <= 15x
constexpr int PREC = 22;        // Pillow PRECISION_BITS (32 - 8 - 2)
constexpr int TY = 16;          // output rows per workgroup
constexpr int RCAP = 48;        // horizontally resampled rows held in LDS (RCAP * OW * 4 B: 42 KiB at OW = 224)
constexpr int MAX_OW = 512;

struct Axis {                   // one axis' table for one image: bounds then weights
  int* lo;                      // [out] first input index
  int* n;                       // [out] number of taps
  int* k;                       // [out][KMAX] fixed-point weights
};

__device__ __forceinline__ Axis axis_at(int* ws, int b, int axis, int OH, int OW) {
  // per image: H axis (OH entries) then W axis (OW entries); each entry 2 + KMAX ints
  const long per_img = (long)(OH + OW) * (2 + KMAX);
  int* base = ws + 1 + b * per_img + (axis == 0 ? 0 : (long)OH * (2 + KMAX));
  const int out = axis == 0 ? OH : OW;
  return Axis{base, base + out, base + 2 * out};
}

// Pillow precompute_coeffs + normalize_coeffs_8bpc for BILINEAR, box (0, 0, in, out)
#pragma clang fp contract(off)
__device__ __forceinline__ double tri_tap(int x, int xmin, double center, double ss) {
  double t = (x + xmin - center + 0.5) * ss;
  if (t < 0.0) t = -t;
  return t < 1.0 ? 1.0 - t : 0.0;
}
__global__ void coeff_kernel(const int32_t* __restrict__ sizes, int OH, int OW, int* ws) {
  const int b = blockIdx.x;
  const int inH = sizes[2 * b], inW = sizes[2 * b + 1];
  for (int idx = threadIdx.x; idx < OH + OW; idx += blockDim.x) {
    const int axis = idx < OH ? 0 : 1;
    const int i = axis == 0 ? idx : idx - OH;
    const int in = axis == 0 ? inH : inW, out = axis == 0 ? OH : OW;
    const Axis ax = axis_at(ws, b, axis, OH, OW);
    const double scale = (double)(float)in / out;   // (in1 - in0) in float, as Pillow's box
    const double filterscale = scale < 1.0 ? 1.0 : scale;
    const double support = 1.0 * filterscale;
    const double center = 0.0 + (i + 0.5) * scale;
    const double ss = 1.0 / filterscale;
    int xmin = (int)(center - support + 0.5);
    if (xmin < 0) xmin = 0;
    int xmax = (int)(center + support + 0.5);
    if (xmax > in) xmax = in;
    xmax -= xmin;
    if (xmax > KMAX || xmax < 0 || in <= 0) {   // host validates sizes; never index past the table
      ws[0] = 1;
      xmax = xmax < 0 ? 0 : (xmax > KMAX ? KMAX : xmax);
    }
    // pass 1: the normaliser ww (Pillow sums the taps in order); pass 2 recomputes each tap
    // (identical doubles) and quantises w / ww -- no per-thread array
    double ww = 0.0;
    for (int x = 0; x < xmax; ++x) ww += tri_tap(x, xmin, center, ss);
    for (int x = 0; x < KMAX; ++x) {
      int q = 0;
      if (x < xmax) {
        double w = tri_tap(x, xmin, center, ss);
        if (ww != 0.0) w /= ww;
        q = w < 0 ? (int)(-0.5 + w * (1 << PREC)) : (int)(0.5 + w * (1 << PREC));
      }
      ax.k[(long)i * KMAX + x] = q;
    }
    ax.lo[i] = xmin;
    ax.n[i] = xmax;
  }
}
#pragma clang fp contract(on)

__device__ __forceinline__ int clip8(int v) {
  if (v >= (1 << PREC << 8)) return 255;
  if (v <= 0) return 0;
  return v >> PREC;
}

// LDS: tmp [RCAP rows][OW] packed RGB0 u32 (horizontal result, 8-bit per channel), then the
// image's horizontal table (lo + KH weights per output column) and the tile's vertical table.
template <int LAYOUT, typename T>
__global__ __launch_bounds__(256) void resample_kernel(const uint8_t* __restrict__ pix,
                                                       const int64_t* __restrict__ offsets,
                                                       const int32_t* __restrict__ sizes, int OH, int OW,
                                                       int c_pad, int KH, int KV, float m0, float m1, float m2,
                                                       float s0, float s1, float s2, const int* __restrict__ ws_c,
                                                       T* __restrict__ out) {
  extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
  uint32_t* tmp = lds;                                   // RCAP * OW
  int* hlo = (int*)(lds + RCAP * OW);                    // OW
  int* hn = hlo + OW;                                    // OW
  int* hk = hn + OW;                                     // OW * KH
  int* vlo = hk + OW * KH;                               // TY
  int* vn = vlo + TY;                                    // TY
  int* vk = vn + TY;                                     // TY * KV
  int* ws = const_cast<int*>(ws_c);
  const int b = blockIdx.y;
  const int y0 = blockIdx.x * TY;
  const int yend = y0 + TY < OH ? y0 + TY : OH;
  const int inW = sizes[2 * b + 1];
  const uint8_t* src = pix + offsets[b];
  const Axis vy = axis_at(ws, b, 0, OH, OW);
  const Axis hx = axis_at(ws, b, 1, OH, OW);
  const int tid = threadIdx.x;
  for (int i = tid; i < OW * KH; i += blockDim.x) {
    const int xx = i / KH, x = i - xx * KH;
    hk[i] = hx.k[(long)xx * KMAX + x];
  }
  for (int i = tid; i < OW; i += blockDim.x) {
    hlo[i] = hx.lo[i];
    hn[i] = hx.n[i];
  }
  for (int i = tid; i < (yend - y0) * KV; i += blockDim.x) {
    const int yl = i / KV, y = i - yl * KV;
    vk[i] = vy.k[(long)(y0 + yl) * KMAX + y];
  }
  for (int i = tid; i < yend - y0; i += blockDim.x) {
    vlo[i] = vy.lo[y0 + i];
    vn[i] = vy.n[y0 + i];
  }
  __syncthreads();
  if (hn[0] > KH || vn[0] > KV) {   // tables wider than the launch assumed: flag, leave (uniform)
    if (tid == 0) ws[0] = 3;
    return;
  }
  const float mean[3] = {m0, m1, m2}, stdv[3] = {s0, s1, s2};
  // vertical resample of (output row yy, column xx), all 3 channels, from LDS rows based at r0
  auto vres = [&](int yy, int xx, int r0, float (&v)[3]) {
    const int yl = yy - y0;
    const int lo = vlo[yl] - r0, n = vn[yl];
    const int* k = vk + yl * KV;
    int a0 = 1 << (PREC - 1), a1 = a0, a2 = a0;
#pragma unroll 4
    for (int y = 0; y < n; ++y) {
      const uint32_t p = tmp[(lo + y) * OW + xx];
      const int w = k[y];
      a0 += (int)(p & 255u) * w;
      a1 += (int)((p >> 8) & 255u) * w;
      a2 += (int)((p >> 16) & 255u) * w;
    }
    v[0] = ((float)clip8(a0) / 255.0f - mean[0]) / stdv[0];
    v[1] = ((float)clip8(a1) / 255.0f - mean[1]) / stdv[1];
    v[2] = ((float)clip8(a2) / 255.0f - mean[2]) / stdv[2];
  };

  int ys = y0;
  while (ys < yend) {
    // rows [ys, ye) whose input span fits in RCAP LDS rows (uniform across the workgroup); an
    // S2D16 chunk always holds whole row pairs
    const int step = LAYOUT == SAT_IMG_S2D16 ? 2 : 1;
    const int r0 = vlo[ys - y0];
    int ye = ys + step;
    while (ye + step <= yend && vlo[ye + step - 1 - y0] + vn[ye + step - 1 - y0] - r0 <= RCAP) ye += step;
    const int nrows = vlo[ye - 1 - y0] + vn[ye - 1 - y0] - r0;   // one row pair spans <= 15.5 + KMAX rows
    if (nrows > RCAP) {          // unreachable for validated sizes; uniform exit, flag the error
      if (tid == 0) ws[0] = 2;
      return;
    }
    // horizontal pass: input rows [r0, r0 + nrows) -> tmp (8-bit per channel, clip8-rounded like
    // Pillow's intermediate image); one output pixel (3 channels) per thread
    for (int idx = tid; idx < nrows * OW; idx += blockDim.x) {
      const int r = idx / OW, xx = idx - r * OW;
      const int n = hn[xx];
      const int* k = hk + xx * KH;
      const uint8_t* row = src + ((long)(r0 + r) * inW + hlo[xx]) * 3;
      int a0 = 1 << (PREC - 1), a1 = a0, a2 = a0;
      if (KH <= 8) {   // the common <= 3x downscale: all taps' loads issued before the multiplies
        uint8_t px[8][3];
#pragma unroll
        for (int x = 0; x < 8; ++x)
#pragma unroll
          for (int c = 0; c < 3; ++c) px[x][c] = x < n ? row[3 * x + c] : (uint8_t)0;
#pragma unroll
        for (int x = 0; x < 8; ++x) {
          const int w = x < n ? k[x] : 0;
          a0 += (int)px[x][0] * w;
          a1 += (int)px[x][1] * w;
          a2 += (int)px[x][2] * w;
        }
      } else {
        for (int x = 0; x < n; ++x) {
          const int w = k[x];
          a0 += (int)row[3 * x] * w;
          a1 += (int)row[3 * x + 1] * w;
          a2 += (int)row[3 * x + 2] * w;
        }
      }
      tmp[idx] = (uint32_t)clip8(a0) | ((uint32_t)clip8(a1) << 8) | ((uint32_t)clip8(a2) << 16);
    }
    __syncthreads();
    if constexpr (LAYOUT == SAT_IMG_NCHW) {   // one pixel per thread, 3 coalesced plane stores
      const int per = (ye - ys) * OW;
      for (int idx = tid; idx < per; idx += blockDim.x) {
        const int yl = idx / OW, xx = idx - yl * OW, yy = ys + yl;
        float v[3];
        vres(yy, xx, r0, v);
#pragma unroll
        for (int c = 0; c < 3; ++c) out[(((long)b * 3 + c) * OH + yy) * OW + xx] = (T)v[c];
      }
    } else if constexpr (LAYOUT == SAT_IMG_NHWC) {   // one output pixel (c_pad channels) per thread
      const int per = (ye - ys) * OW;
      for (int idx = tid; idx < per; idx += blockDim.x) {
        const int yl = idx / OW, xx = idx - yl * OW, yy = ys + yl;
        float v[3];
        vres(yy, xx, r0, v);
        T* dst = out + (((long)b * OH + yy) * OW + xx) * c_pad;
        if (c_pad * (int)sizeof(T) == 16) {
          uint4 u = make_uint4(0, 0, 0, 0);
          T* h = (T*)&u;
#pragma unroll
          for (int c = 0; c < 3; ++c) h[c] = (T)v[c];
          *(uint4*)dst = u;
        } else {
          for (int c = 0; c < c_pad; ++c) dst[c] = (T)(c < 3 ? v[c] : 0.f);
        }
      }
    } else {   // S2D16: one 2x2 block (16 channels) per thread
      const int W2 = OW / 2, per = (ye - ys) / 2 * W2;
      for (int idx = tid; idx < per; idx += blockDim.x) {
        const int pl = idx / W2, bx = idx - pl * W2, by = (ys >> 1) + pl;
        T q[16];
#pragma unroll
        for (int j = 12; j < 16; ++j) q[j] = (T)0.f;
#pragma unroll
        for (int sy = 0; sy < 2; ++sy)
#pragma unroll
          for (int sx = 0; sx < 2; ++sx) {
            float v[3];
            vres(2 * by + sy, 2 * bx + sx, r0, v);
#pragma unroll
            for (int c = 0; c < 3; ++c) q[(sy * 2 + sx) * 3 + c] = (T)v[c];
          }
        T* dst = out + (((long)b * (OH / 2) + by) * W2 + bx) * 16;
        if constexpr (sizeof(T) == 2) {
          *(uint4*)dst = *(const uint4*)&q[0];
          *(uint4*)(dst + 8) = *(const uint4*)&q[8];
        } else {
#pragma unroll
          for (int j = 0; j < 16; ++j) dst[j] = q[j];
        }
      }
    }
    __syncthreads();
    ys = ye;
  }
}

inline int ksize_for(int in, int out) {   // Pillow: (int)ceil(support) * 2 + 1, support = max(in / out, 1)
  const double sc = (double)in / out;
  return (int)std::ceil(sc < 1.0 ? 1.0 : sc) * 2 + 1;
}

template <int LAYOUT, typename T>
void launch_resample(const uint8_t* pix, const int64_t* offsets, const int32_t* sizes, int B, int max_h,
                     int max_w, int OH, int OW, int c_pad, const float* mean, const float* stdv, const int* ws,
                     void* out, hipStream_t s) {
  const int KH = ksize_for(max_w, OW), KV = ksize_for(max_h, OH);
  const size_t lds = (size_t)RCAP * OW * 4 + (size_t)OW * (2 + KH) * 4 + (size_t)TY * (2 + KV) * 4;
  const dim3 grid(sat_cdiv(OH, TY), B);
  hipLaunchKernelGGL((resample_kernel<LAYOUT, T>), grid, dim3(256), lds, s, pix, offsets, sizes, OH, OW, c_pad, KH,
                     KV, mean[0], mean[1], mean[2], stdv[0], stdv[1], stdv[2], ws, (T*)out);
}

}  // namespace

extern "C" size_t sat_images_workspace_bytes(int B, int OH, int OW) {
  if (B <= 0 || OH <= 0 || OW <= 0) return 0;
  return (1 + (size_t)B * (OH + OW) * (2 + KMAX)) * sizeof(int);
}

extern "C" int sat_images_max_downscale(void) { return (KMAX - 1) / 2; }

namespace {
// A resample / coefficient kernel that hit an unreachable-for-validated-sizes limit sets ws[0] and
// leaves its tile unwritten: turn the whole batch into NaN so the failure shows in the encoder output
// and the loss instead of passing uninitialised memory on (reads one int when all is well).
template <typename T>
__global__ void poison_on_error_kernel(const int* __restrict__ ws, T* __restrict__ out, long n) {
  if (ws[0] == 0) return;
  const T nan = (T)__builtin_nanf("");
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) out[i] = nan;
}
}  // namespace

extern "C" int sat_images_to_input(const uint8_t* pixels, const int64_t* offsets, const int32_t* sizes, int B,
                                   int max_h, int max_w, int OH, int OW, const float* mean, const float* stdv,
                                   int layout, int c_pad, int dtype, void* out, void* workspace,
                                   size_t workspace_bytes, void* stream) {
  SAT_REQUIRE(pixels && offsets && sizes && mean && stdv && out && workspace && B > 0);
  SAT_REQUIRE(OH > 0 && OW > 0 && OW <= MAX_OW && max_h > 0 && max_w > 0);
  // taps per output index = 2 * ceil(in / out) + 1 at most: keep within KMAX
  SAT_REQUIRE(2 * sat_cdiv(max_h, OH) + 1 <= KMAX && 2 * sat_cdiv(max_w, OW) + 1 <= KMAX);
  SAT_REQUIRE(workspace_bytes >= sat_images_workspace_bytes(B, OH, OW));
  SAT_REQUIRE(dtype == SAT_F32 || dtype == SAT_BF16);
  if (layout == SAT_IMG_NCHW) SAT_REQUIRE(dtype == SAT_F32);
  else if (layout == SAT_IMG_NHWC) SAT_REQUIRE(c_pad >= 3 && c_pad <= 64);
  else if (layout == SAT_IMG_S2D16) SAT_REQUIRE(OH % 2 == 0 && OW % 2 == 0);
  else return SAT_ERR_INVALID;
  hipStream_t s = (hipStream_t)stream;
  int* ws = (int*)workspace;
  SAT_CHECK(hipMemsetAsync(ws, 0, sizeof(int), s));
  hipLaunchKernelGGL(coeff_kernel, dim3(B), dim3(256), 0, s, sizes, OH, OW, ws);
  SAT_CHECK(hipGetLastError());
  if (layout == SAT_IMG_NCHW)
    launch_resample<SAT_IMG_NCHW, float>(pixels, offsets, sizes, B, max_h, max_w, OH, OW, 0, mean, stdv, ws, out, s);
  else if (layout == SAT_IMG_NHWC && dtype == SAT_BF16)
    launch_resample<SAT_IMG_NHWC, bf16>(pixels, offsets, sizes, B, max_h, max_w, OH, OW, c_pad, mean, stdv, ws, out, s);
  else if (layout == SAT_IMG_NHWC)
    launch_resample<SAT_IMG_NHWC, float>(pixels, offsets, sizes, B, max_h, max_w, OH, OW, c_pad, mean, stdv, ws, out, s);
  else if (dtype == SAT_BF16)
    launch_resample<SAT_IMG_S2D16, bf16>(pixels, offsets, sizes, B, max_h, max_w, OH, OW, 16, mean, stdv, ws, out, s);
  else
    launch_resample<SAT_IMG_S2D16, float>(pixels, offsets, sizes, B, max_h, max_w, OH, OW, 16, mean, stdv, ws, out, s);
  SAT_CHECK(hipGetLastError());
  const long n = layout == SAT_IMG_NCHW ? (long)B * 3 * OH * OW
                 : layout == SAT_IMG_NHWC ? (long)B * OH * OW * c_pad : (long)B * (OH / 2) * (OW / 2) * 16;
  if (dtype == SAT_BF16)
    hipLaunchKernelGGL(poison_on_error_kernel<bf16>, dim3(256), dim3(256), 0, s, ws, (bf16*)out, n);
  else
    hipLaunchKernelGGL(poison_on_error_kernel<float>, dim3(256), dim3(256), 0, s, ws, (float*)out, n);
  return (int)hipGetLastError();
}
