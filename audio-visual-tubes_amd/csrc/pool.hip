// Pooling on the trunks, NHWC bf16.
//  * MaxPool2d(3, 2, 1) after the stem (models/base_models.py:143, 203): fwd saves the window
//    argmax (uint8, 0..8, first max wins like torch); bwd is a gather over the <=4 windows that
//    cover each input pixel (no atomics).
//  * AdaptiveMaxPool2d(1) + F.normalize(dim=1) on the audio layer4 map (model.py:96,120-122):
//    fwd writes the unit vector (fp32), its argmax and the pre-normalisation norm; bwd routes the
//    normalize-backward gradient to the argmax (dense bf16 write, zeros elsewhere).
#include "avt_common.h"

namespace avt {

__global__ __launch_bounds__(256) void maxpool3s2_fwd_kernel(const bf16_t* __restrict__ x, bf16_t* __restrict__ y,
                                                             unsigned char* __restrict__ idx, int N, int H, int W,
                                                             int C, int P, int Q) {
  const int cv = C / 8;
  const long long total = (long long)N * P * Q * cv;
  for (long long t = blockIdx.x * (long long)blockDim.x + threadIdx.x; t < total; t += (long long)gridDim.x * blockDim.x) {
    const int c8 = (int)(t % cv);
    long long pix = t / cv;
    const int q = (int)(pix % Q);
    pix /= Q;
    const int p = (int)(pix % P);
    const int n = (int)(pix / P);
    float best[8];
    int bi[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      best[e] = -INFINITY;
      bi[e] = 0;
    }
    for (int r = 0; r < 3; ++r) {
      const int h = p * 2 - 1 + r;
      if (h < 0 || h >= H) continue;
      for (int s = 0; s < 3; ++s) {
        const int w = q * 2 - 1 + s;
        if (w < 0 || w >= W) continue;
        const u32x4 v = *reinterpret_cast<const u32x4*>(x + (((size_t)n * H + h) * W + w) * C + c8 * 8);
        const unsigned* u = reinterpret_cast<const unsigned*>(&v);
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float f = bf2f((e & 1) ? (u[e >> 1] >> 16) : (u[e >> 1] & 0xffff));
          if (f > best[e] || f != f) {
            best[e] = f;
            bi[e] = r * 3 + s;
          }
        }
      }
    }
    u32x4 o;
    unsigned* ou = reinterpret_cast<unsigned*>(&o);
#pragma unroll
    for (int e = 0; e < 4; ++e) ou[e] = pack2(best[2 * e], best[2 * e + 1]);
    const size_t off = (((size_t)n * P + p) * Q + q) * C + c8 * 8;
    *reinterpret_cast<u32x4*>(y + off) = o;
    unsigned long long ib = 0;
#pragma unroll
    for (int e = 0; e < 8; ++e) ib |= (unsigned long long)bi[e] << (8 * e);
    *reinterpret_cast<unsigned long long*>(idx + off) = ib;
  }
}

__global__ __launch_bounds__(256) void maxpool3s2_bwd_kernel(const bf16_t* __restrict__ gy,
                                                             const unsigned char* __restrict__ idx,
                                                             bf16_t* __restrict__ gx, int N, int H, int W, int C, int P,
                                                             int Q) {
  const int cv = C / 8;
  const long long total = (long long)N * H * W * cv;
  for (long long t = blockIdx.x * (long long)blockDim.x + threadIdx.x; t < total; t += (long long)gridDim.x * blockDim.x) {
    const int c8 = (int)(t % cv);
    long long pix = t / cv;
    const int w = (int)(pix % W);
    pix /= W;
    const int h = (int)(pix % H);
    const int n = (int)(pix / H);
    float acc[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) acc[e] = 0.f;
    // windows p with 2p-1 <= h <= 2p+1
    const int p_lo = h / 2, p_hi = min(P - 1, (h + 1) / 2);
    const int q_lo = w / 2, q_hi = min(Q - 1, (w + 1) / 2);
    for (int p = p_lo; p <= p_hi; ++p) {
      const int kh = h - (2 * p - 1);
      if (kh < 0 || kh > 2) continue;
      for (int q = q_lo; q <= q_hi; ++q) {
        const int kw = w - (2 * q - 1);
        if (kw < 0 || kw > 2) continue;
        const int pos = kh * 3 + kw;
        const size_t off = (((size_t)n * P + p) * Q + q) * C + c8 * 8;
        const unsigned long long ib = *reinterpret_cast<const unsigned long long*>(idx + off);
        const u32x4 v = *reinterpret_cast<const u32x4*>(gy + off);
        const unsigned* u = reinterpret_cast<const unsigned*>(&v);
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          if ((int)((ib >> (8 * e)) & 0xff) == pos)
            acc[e] += bf2f((e & 1) ? (u[e >> 1] >> 16) : (u[e >> 1] & 0xffff));
        }
      }
    }
    u32x4 o;
    unsigned* ou = reinterpret_cast<unsigned*>(&o);
#pragma unroll
    for (int e = 0; e < 4; ++e) ou[e] = pack2(acc[2 * e], acc[2 * e + 1]);
    *reinterpret_cast<u32x4*>(gx + (((size_t)n * H + h) * W + w) * C + c8 * 8) = o;
  }
}

// One block of 1024 threads per sample: thread = (8-channel block cg, row group rg); each thread
// scans rows rg, rg + RG, ... with 16-B loads (four in flight), then the RG partial (max, first
// argmax) per channel are merged through LDS (ties -> the smaller row, i.e. the first maximum like
// torch).  Only B blocks: the per-thread row loop is the latency, so it is kept short.
constexpr int kAPoolT = 1024;
__device__ __forceinline__ void apool_take(const u32x4& v, int i, float* best, int* bi) {
  const unsigned* u = reinterpret_cast<const unsigned*>(&v);
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const float f = bf2f((e & 1) ? (u[e >> 1] >> 16) : (u[e >> 1] & 0xffff));
    if (f > best[e] || (f != f && best[e] == best[e])) {
      best[e] = f;
      bi[e] = i;
    }
  }
}
__global__ __launch_bounds__(kAPoolT) void audio_pool_norm_fwd_kernel(const bf16_t* __restrict__ a,
                                                                      float* __restrict__ an, int* __restrict__ amax,
                                                                      float* __restrict__ anorm, int HW, int C) {
  __shared__ float sv[kAPoolT * 8];
  __shared__ int si[kAPoolT * 8];
  __shared__ float red[16];
  const int b = blockIdx.x, cvn = C / 8, RG = kAPoolT / cvn;
  const int cg = threadIdx.x % cvn, rg = threadIdx.x / cvn;
  float best[8];
  int bi[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    best[e] = -INFINITY;
    bi[e] = 0;
  }
  const bf16_t* src = a + (size_t)b * HW * C + cg * 8;
  int i = rg;
  for (; i + 3 * RG < HW; i += 4 * RG) {  // rows taken in increasing order: the first max is kept
    u32x4 v[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) v[k] = *reinterpret_cast<const u32x4*>(src + (size_t)(i + k * RG) * C);
#pragma unroll
    for (int k = 0; k < 4; ++k) apool_take(v[k], i + k * RG, best, bi);
  }
  for (; i < HW; i += RG) apool_take(*reinterpret_cast<const u32x4*>(src + (size_t)i * C), i, best, bi);
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    sv[rg * C + cg * 8 + e] = best[e];
    si[rg * C + cg * 8 + e] = bi[e];
  }
  __syncthreads();
  float m = 0.f;
  if (threadIdx.x < C) {
    const int c = threadIdx.x;
    float bv = -INFINITY;
    int bx = 0;
    bool first = true;
    for (int g = 0; g < RG; ++g) {
      const float v = sv[g * C + c];
      const int ix = si[g * C + c];
      if (g >= HW) break;  // row group saw no rows
      const bool vnan = v != v, bnan = bv != bv;
      bool take;
      if (first) take = true;
      else if (vnan || bnan) take = vnan && (!bnan || ix < bx);
      else take = v > bv || (v == bv && ix < bx);
      if (take) {
        bv = v;
        bx = ix;
        first = false;
      }
    }
    m = bv;
    amax[(size_t)b * C + c] = bx;
  }
  const float ss = block_sum(threadIdx.x < C ? m * m : 0.f, red);
  const float nrm = sqrtf(ss);
  const float d = fmaxf(nrm, 1e-12f);
  if (threadIdx.x < C) an[(size_t)b * C + threadIdx.x] = m / d;
  if (threadIdx.x == 0) anorm[b] = nrm;
}

// g_pool = (g - an*<an,g>)/max(norm,eps) (identity-free when norm <= eps: g/eps);
// ga[b, i, c] = (i == amax[b,c]) ? g_pool[b,c] : 0
__global__ void audio_pool_norm_bwd_kernel(const float* __restrict__ gan, const float* __restrict__ an,
                                           const int* __restrict__ amax, const float* __restrict__ anorm,
                                           bf16_t* __restrict__ ga, int HW, int C) {
  __shared__ float red[16];
  __shared__ float gp[1024];
  __shared__ int am[1024];
  const int b = blockIdx.x, c = threadIdx.x;
  const float g = c < C ? gan[(size_t)b * C + c] : 0.f;
  const float y = c < C ? an[(size_t)b * C + c] : 0.f;
  const float dot = block_sum(g * y, red);
  const float nrm = anorm[b];
  float gpc;
  if (nrm > 1e-12f)
    gpc = (g - y * dot) / nrm;
  else
    gpc = g / 1e-12f;
  if (c < C) {
    gp[c] = gpc;
    am[c] = amax[(size_t)b * C + c];
  }
  __syncthreads();
  // dense write of rows [r0, r1) of the [HW][C] map of sample b (8 channels per thread-iteration);
  // blockIdx.y slices the rows so that B x slices blocks share the store stream
  const int cv = C / 8;
  const int rps = (HW + gridDim.y - 1) / gridDim.y;
  const int r0 = blockIdx.y * rps, r1 = min(HW, r0 + rps);
  bf16_t* dst = ga + (size_t)b * HW * C;
  for (int t = r0 * cv + threadIdx.x; t < r1 * cv; t += blockDim.x) {
    const int i = t / cv, c0 = (t - i * cv) * 8;
    float f[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) f[e] = (am[c0 + e] == i) ? gp[c0 + e] : 0.f;
    u32x4 o;
    o.x = pack2(f[0], f[1]);
    o.y = pack2(f[2], f[3]);
    o.z = pack2(f[4], f[5]);
    o.w = pack2(f[6], f[7]);
    *reinterpret_cast<u32x4*>(dst + (size_t)i * C + c0) = o;
  }
}

static int grid_for(long long n) {
  long long b = (n + 255) / 256;
  if (b > 8192) b = 8192;
  if (b < 1) b = 1;
  return (int)b;
}

}  // namespace avt

using namespace avt;

extern "C" int avt_maxpool3s2_fwd(const void* x, void* y, void* idx, int N, int H, int W, int C, void* stream) {
  AVT_REQUIRE(x && y && idx, "maxpool_fwd: null pointer");
  AVT_REQUIRE(C % 8 == 0, "maxpool_fwd: C=%d must be a multiple of 8", C);
  const int P = (H + 2 - 3) / 2 + 1, Q = (W + 2 - 3) / 2 + 1;
  hipLaunchKernelGGL(maxpool3s2_fwd_kernel, dim3(grid_for((long long)N * P * Q * (C / 8))), dim3(256), 0,
                     (hipStream_t)stream, (const bf16_t*)x, (bf16_t*)y, (unsigned char*)idx, N, H, W, C, P, Q);
  return check_launch("maxpool_fwd");
}

extern "C" int avt_maxpool3s2_bwd(const void* gy, const void* idx, void* gx, int N, int H, int W, int C, void* stream) {
  AVT_REQUIRE(gy && idx && gx, "maxpool_bwd: null pointer");
  AVT_REQUIRE(C % 8 == 0, "maxpool_bwd: C=%d must be a multiple of 8", C);
  const int P = (H + 2 - 3) / 2 + 1, Q = (W + 2 - 3) / 2 + 1;
  hipLaunchKernelGGL(maxpool3s2_bwd_kernel, dim3(grid_for((long long)N * H * W * (C / 8))), dim3(256), 0,
                     (hipStream_t)stream, (const bf16_t*)gy, (const unsigned char*)idx, (bf16_t*)gx, N, H, W, C, P, Q);
  return check_launch("maxpool_bwd");
}

extern "C" int avt_audio_pool_norm_fwd(const void* a, float* an, int* amax, float* anorm, int B, int HW, int C,
                                       void* stream) {
  AVT_REQUIRE(a && an && amax && anorm, "audio_pool_norm_fwd: null pointer");
  AVT_REQUIRE(C >= 64 && C <= 512 && (C & (C - 1)) == 0, "audio_pool_norm_fwd: C=%d unsupported", C);
  AVT_REQUIRE(HW > 0, "audio_pool_norm_fwd: empty map");
  hipLaunchKernelGGL(audio_pool_norm_fwd_kernel, dim3(B), dim3(kAPoolT), 0, (hipStream_t)stream, (const bf16_t*)a, an,
                     amax, anorm, HW, C);
  return check_launch("audio_pool_norm_fwd");
}

extern "C" int avt_audio_pool_norm_bwd(const float* gan, const float* an, const int* amax, const float* anorm, void* ga,
                                       int B, int HW, int C, void* stream) {
  AVT_REQUIRE(gan && an && amax && anorm && ga, "audio_pool_norm_bwd: null pointer");
  AVT_REQUIRE(C % 64 == 0 && C <= 1024, "audio_pool_norm_bwd: C=%d unsupported", C);
  AVT_REQUIRE(B > 0 && HW > 0, "audio_pool_norm_bwd: empty map");
  hipLaunchKernelGGL(audio_pool_norm_bwd_kernel, dim3(B, min(HW, 8)), dim3(C), 0, (hipStream_t)stream, gan, an, amax, anorm,
                     (bf16_t*)ga, HW, C);
  return check_launch("audio_pool_norm_bwd");
}
