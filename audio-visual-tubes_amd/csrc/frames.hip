// Frame transform of the reference's dataset on the device (datasets/dataloader.py:47-62; SURVEY
// §8f rank 4): Resize(short side, PIL BICUBIC) -> crop (Random/Center) -> optional horizontal flip
// -> ToTensor -> Normalize(mean, std), from decoded RGB uint8 frames to the float32 [n][3][S][S]
// tensor the reference's DataLoader yields.
//
// The resize is Pillow's separable fixed-point resampler (Image.resize(size, BICUBIC), Pillow
// 12.2.0 in this image): per output index, weights of the a = -0.5 bicubic kernel stretched by the
// downscale factor, normalised in double, rounded to int32 with 22 fraction bits; a horizontal pass
// into an 8-bit intermediate, then a vertical pass, each accumulated in int32 from 1 << 21, shifted
// and clipped to [0, 255].  The coefficients are computed on the device in double precision with
// contraction off (Pillow's x86-64 build does a separate multiply and add), so the output is
// bit-identical to Pillow.  Only the crop window's columns (horizontal pass) and rows (vertical
// pass) are computed: every output pixel of the resampler is independent of the others.
//
// Two launches per batch: (1) horizontal pass, one thread per crop column, rows restricted to those
// the crop's vertical taps read, written as planar uint8 [n][3][Hmax][S]; (2) vertical pass + crop +
// flip + /255 + normalise, one thread per output pixel column, coalesced fp32 stores.  HBM-bound:
// the source bytes once (L2 catches the tap overlap), 3 B per intermediate pixel, 12 B per output.
#include "avt_common.h"

namespace avt {

constexpr int FR_PREC = 22;  // Pillow: PRECISION_BITS = 32 - 8 - 2
constexpr int FR_KMAX = 32;  // taps per output index: downscale factor <= 7.5
constexpr int FR_T = 256;    // threads per block = max crop size

struct FrameDesc {  // the int64[8] row of the descriptor table, as passed in
  long long off, H, W, rh, rw, ci, cj, flip;
};

__device__ __forceinline__ double bicubic_w(double x) {
#pragma clang fp contract(off)
  const double a = -0.5;
  if (x < 0.0) x = -x;
  if (x < 1.0) return ((a + 2.0) * x - (a + 3.0)) * x * x + 1;
  if (x < 2.0) return (((x - 5) * x + 8) * x - 4) * a;
  return 0.0;
}

// Pillow precompute_coeffs (box = whole image) + normalize_coeffs_8bpc for output index xx.
// Returns the tap count; k[0..count) are the fixed-point weights, *first the first source index.
__device__ int frame_coeffs(int in_size, int out_size, int xx, int* k, int* first) {
#pragma clang fp contract(off)
  const double scale = (double)in_size / (double)out_size;
  const double filterscale = scale < 1.0 ? 1.0 : scale;
  const double support = 2.0 * filterscale;
  const double center = ((double)xx + 0.5) * scale;
  const double ss = 1.0 / filterscale;
  int xmin = (int)(center - support + 0.5);
  if (xmin < 0) xmin = 0;
  int xmax = (int)(center + support + 0.5);
  if (xmax > in_size) xmax = in_size;
  xmax -= xmin;
  if (xmax > FR_KMAX) xmax = FR_KMAX;  // only past the host-checked factor 7.5: wrong, never out of bounds
  double w[FR_KMAX];
  double ww = 0.0;
  for (int x = 0; x < xmax; ++x) {
    w[x] = bicubic_w(((double)(x + xmin) - center + 0.5) * ss);
    ww += w[x];
  }
  for (int x = 0; x < xmax; ++x) {
    const double v = ww != 0.0 ? w[x] / ww : w[x];
    const double f = v * (double)(1 << FR_PREC);
    k[x] = v < 0 ? (int)(-0.5 + f) : (int)(0.5 + f);
  }
  *first = xmin;
  return xmax;
}

__device__ __forceinline__ int clip8(int ss) {
  const int v = ss >> FR_PREC;
  return v < 0 ? 0 : (v > 255 ? 255 : v);
}

// (1) horizontal pass: tmp[img][c][y][x] for crop columns x (resized column cj + x) and the rows y
// the vertical taps of crop rows ci .. ci+S-1 read.
__global__ __launch_bounds__(FR_T) void frames_hpass_kernel(const unsigned char* __restrict__ src,
                                                            const long long* __restrict__ desc, int S, int Hmax,
                                                            int rows_per_block, unsigned char* __restrict__ tmp) {
  __shared__ int kk[FR_KMAX][FR_T];
  __shared__ int yr[2];
  const int img = blockIdx.y, x = threadIdx.x;
  const FrameDesc d = reinterpret_cast<const FrameDesc*>(desc)[img];
  const int H = (int)d.H, W = (int)d.W;
  if (threadIdx.x < 2) {  // source rows read by the vertical taps of the first / last crop row
    int kt[FR_KMAX], f;
    const int yy = (int)d.ci + (threadIdx.x ? S - 1 : 0);
    const int n = frame_coeffs(H, (int)d.rh, yy, kt, &f);
    yr[threadIdx.x] = threadIdx.x ? f + n : f;
  }
  int xmin = 0, cnt = 0;
  if (x < S) {
    int kt[FR_KMAX];
    cnt = frame_coeffs(W, (int)d.rw, (int)d.cj + x, kt, &xmin);
    for (int t = 0; t < cnt; ++t) kk[t][x] = kt[t];
  }
  __syncthreads();
  const int y0 = max(yr[0], blockIdx.x * rows_per_block), y1 = min(yr[1], (blockIdx.x + 1) * rows_per_block);
  if (x >= S) return;
  const unsigned char* im = src + d.off;
  const size_t plane = (size_t)Hmax * S;
  unsigned char* o = tmp + (size_t)img * 3 * plane;
  for (int y = y0; y < y1; ++y) {
    const unsigned char* row = im + ((size_t)y * W + xmin) * 3;
    int s0 = 1 << (FR_PREC - 1), s1 = s0, s2 = s0;
    for (int t = 0; t < cnt; ++t) {
      const int w = kk[t][x];
      s0 += (int)row[3 * t + 0] * w;
      s1 += (int)row[3 * t + 1] * w;
      s2 += (int)row[3 * t + 2] * w;
    }
    const size_t at = (size_t)y * S + x;
    o[at] = (unsigned char)clip8(s0);
    o[plane + at] = (unsigned char)clip8(s1);
    o[2 * plane + at] = (unsigned char)clip8(s2);
  }
}

// (2) vertical pass of crop row i + horizontal flip + ToTensor + Normalize -> out[img][c][i][j].
__global__ __launch_bounds__(FR_T) void frames_vpass_kernel(const unsigned char* __restrict__ tmp,
                                                            const long long* __restrict__ desc, int S, int Hmax,
                                                            float m0, float m1, float m2, float s0, float s1,
                                                            float s2, float* __restrict__ out) {
  __shared__ int kk[FR_KMAX];
  __shared__ int hdr[2];
  const int i = blockIdx.x, img = blockIdx.y, j = threadIdx.x;
  const FrameDesc d = reinterpret_cast<const FrameDesc*>(desc)[img];
  if (threadIdx.x == 0) {
    int kt[FR_KMAX], f;
    const int n = frame_coeffs((int)d.H, (int)d.rh, (int)d.ci + i, kt, &f);
    for (int t = 0; t < n; ++t) kk[t] = kt[t];
    hdr[0] = f;
    hdr[1] = n;
  }
  __syncthreads();
  if (j >= S) return;
  const int ymin = hdr[0], cnt = hdr[1];
  const int x = d.flip ? S - 1 - j : j;
  const size_t plane = (size_t)Hmax * S;
  const unsigned char* t0 = tmp + (size_t)img * 3 * plane + (size_t)ymin * S + x;
  int a0 = 1 << (FR_PREC - 1), a1 = a0, a2 = a0;
  for (int t = 0; t < cnt; ++t) {
    const int w = kk[t];
    a0 += (int)t0[(size_t)t * S] * w;
    a1 += (int)t0[plane + (size_t)t * S] * w;
    a2 += (int)t0[2 * plane + (size_t)t * S] * w;
  }
  // ToTensor (x / 255) then Normalize ((x - mean) / std), float32 as torchvision does it
  float* o = out + ((size_t)img * 3 * S + i) * S + j;
  const size_t cs = (size_t)S * S;
  o[0] = ((float)clip8(a0) / 255.f - m0) / s0;
  o[cs] = ((float)clip8(a1) / 255.f - m1) / s1;
  o[2 * cs] = ((float)clip8(a2) / 255.f - m2) / s2;
}

}  // namespace avt

using namespace avt;

// src: decoded RGB frames, uint8 HWC, packed at byte offsets desc[i].off; desc: DEVICE int64
// [n][8] = {off, H, W, resized_h, resized_w, crop_top, crop_left, flip}; tmp: device scratch of
// n * 3 * Hmax * S bytes (Hmax >= every H); mean / std: HOST float[3]; out: float32 [n][3][S][S].
// The host-side checks (sizes, downscale factor <= 7.5 so that <= 32 taps, crop inside the resized
// image, Hmax >= H) are the caller's (avt_amd.frames); given them the kernels read only inside each
// frame and write only inside tmp / out.
extern "C" int avt_frames_transform(const void* src, const long long* desc, int n, int S, int Hmax, void* tmp,
                                    const float* mean, const float* std, float* out, void* stream) {
  AVT_REQUIRE(src && desc && tmp && mean && std && out, "frames_transform: null pointer");
  AVT_REQUIRE(n >= 1 && S >= 1 && S <= FR_T && Hmax >= 1, "frames_transform: need n >= 1, 1 <= S <= 256");
  const int rows_per_block = 32;
  hipLaunchKernelGGL(frames_hpass_kernel, dim3((Hmax + rows_per_block - 1) / rows_per_block, n), dim3(FR_T), 0,
                     (hipStream_t)stream, (const unsigned char*)src, desc, S, Hmax, rows_per_block,
                     (unsigned char*)tmp);
  int rc = check_launch("frames_hpass");
  if (rc != AVT_OK) return rc;
  hipLaunchKernelGGL(frames_vpass_kernel, dim3(S, n), dim3(FR_T), 0, (hipStream_t)stream, (const unsigned char*)tmp,
                     desc, S, Hmax, mean[0], mean[1], mean[2], std[0], std[1], std[2], out);
  return check_launch("frames_vpass");
}
