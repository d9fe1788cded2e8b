// Optimizer, weight packing, input layout and error plumbing for libavt.
//  * Adam with coupled L2 weight decay over one flat fp32 buffer (torch.optim.Adam semantics as
//    constructed at train_hardway_1frame.py:116 and stepped at :134).
//  * Weight packing: fp32 master weights (OHWI memory order, i.e. channels_last OIHW params) ->
//    bf16 fwd operand [K][Kg] (stem channels padded) and bf16 dgrad operand [C][R*S*K].
//  * Input layout: fp32 NCHW (the reference's frames.float()/spec.float(), train_hardway_1frame.py:129)
//    -> bf16 NHWC with channels padded to Cp.
#include "avt_common.h"
#include <stdarg.h>

namespace avt {

static thread_local char g_err[512] = "";

void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

int check_launch(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    set_error("%s: %s", what, hipGetErrorString(e));
    return AVT_EHIP;
  }
  return AVT_OK;
}

// coef (optional): device {step_size, bc2_sqrt, beta1, beta2, eps, weight_decay} written by
// adam_prep_kernel (graph-replayable form: the hyper-parameters are read on the device every launch)
__global__ __launch_bounds__(256) void adam_kernel(float* __restrict__ p, const float* __restrict__ g,
                                                   float* __restrict__ m, float* __restrict__ v, long long n,
                                                   float gscale, float b1, float b2, float eps, float wd,
                                                   float step_size, float bc2_sqrt, const float* __restrict__ coef) {
  if (coef) {
    step_size = coef[0];
    bc2_sqrt = coef[1];
    b1 = coef[2];
    b2 = coef[3];
    eps = coef[4];
    wd = coef[5];
  }
  const long long nv = n / 4;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < nv; i += (long long)gridDim.x * blockDim.x) {
    f32x4 pp = reinterpret_cast<f32x4*>(p)[i];
    f32x4 gg = reinterpret_cast<const f32x4*>(g)[i];
    f32x4 mm = reinterpret_cast<f32x4*>(m)[i];
    f32x4 vv = reinterpret_cast<f32x4*>(v)[i];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float gr = gg[e] * gscale + wd * pp[e];
      mm[e] = b1 * mm[e] + (1.f - b1) * gr;
      vv[e] = b2 * vv[e] + (1.f - b2) * gr * gr;
      const float denom = sqrtf(vv[e]) / bc2_sqrt + eps;
      pp[e] = pp[e] - step_size * mm[e] / denom;
    }
    reinterpret_cast<f32x4*>(p)[i] = pp;
    reinterpret_cast<f32x4*>(m)[i] = mm;
    reinterpret_cast<f32x4*>(v)[i] = vv;
  }
  // tail
  if (blockIdx.x == 0 && threadIdx.x < (n & 3)) {
    const long long i = nv * 4 + threadIdx.x;
    const float gr = g[i] * gscale + wd * p[i];
    m[i] = b1 * m[i] + (1.f - b1) * gr;
    v[i] = b2 * v[i] + (1.f - b2) * gr * gr;
    p[i] = p[i] - step_size * m[i] / (sqrtf(v[i]) / bc2_sqrt + eps);
  }
}

// w: [K][R][S][C] fp32 -> fwd [K][Kg] bf16 with (r,s,c<Cp) packing, zero for c>=C and k>=R*S*Cp
__global__ void pack_fwd_kernel(const float* __restrict__ w, bf16_t* __restrict__ out, int K, int RS, int C, int Cp,
                                int Kg) {
  const long long total = (long long)K * Kg;
  for (long long t = blockIdx.x * (long long)blockDim.x + threadIdx.x; t < total; t += (long long)gridDim.x * blockDim.x) {
    const int k = (int)(t / Kg), col = (int)(t % Kg);
    const int rs = col / Cp, c = col % Cp;
    float val = 0.f;
    if (rs < RS && c < C) val = w[((size_t)k * RS + rs) * C + c];
    out[t] = f2bf(val);
  }
}

// w: [K][R][S][C] fp32 -> dgrad [C][R][S][K] bf16
__global__ void pack_dgrad_kernel(const float* __restrict__ w, bf16_t* __restrict__ out, int K, int RS, int C) {
  const long long total = (long long)K * RS * C;
  for (long long t = blockIdx.x * (long long)blockDim.x + threadIdx.x; t < total; t += (long long)gridDim.x * blockDim.x) {
    const int k = (int)(t % K);
    const long long r2 = t / K;
    const int rs = (int)(r2 % RS), c = (int)(r2 / RS);
    out[t] = f2bf(w[((size_t)k * RS + rs) * C + c]);
  }
}

// Batched packing of many conv weights (one fwd + one dgrad launch): blockIdx.y = conv index.
struct PackDesc {
  const float* w;   // [K][R][S][C] fp32
  bf16_t* fwd;      // [K][Kg] or null
  bf16_t* dgrad;    // [C][R*S*K] or null
  int K, RS, C, Cp, Kg, pad_;
};

// fwd image [K][Kg] (rows zero-padded from R*S*Cp to Kg, channels from C to Cp).  The common case
// (Cp == C, Kg == R*S*C) is a contiguous fp32 -> bf16 copy, 8 elements (2 x 16 B in, 16 B out) per
// thread; the stems take the scalar path.
__global__ __launch_bounds__(256) void pack_fwd_batched_kernel(const PackDesc* __restrict__ descs) {
  const PackDesc d = descs[blockIdx.y];
  if (!d.fwd) return;
  const int row = d.RS * d.C;
  const int total = d.K * d.Kg;
  const int tid = blockIdx.x * 256 + threadIdx.x, nthr = gridDim.x * 256;
  if (d.Cp == d.C && d.Kg == row && (total & 7) == 0 && (((uintptr_t)d.w | (uintptr_t)d.fwd) & 15) == 0) {
    for (int v = tid; v < total / 8; v += nthr) {
      const float4 a = reinterpret_cast<const float4*>(d.w)[2 * v];
      const float4 b = reinterpret_cast<const float4*>(d.w)[2 * v + 1];
      u32x4 o;
      o.x = pack2(a.x, a.y);
      o.y = pack2(a.z, a.w);
      o.z = pack2(b.x, b.y);
      o.w = pack2(b.z, b.w);
      reinterpret_cast<u32x4*>(d.fwd)[v] = o;
    }
  } else {
    for (int t = tid; t < total; t += nthr) {
      const int k = t / d.Kg, col = t - k * d.Kg;
      const int rs = col / d.Cp, c = col - rs * d.Cp;
      float val = 0.f;
      if (rs < d.RS && c < d.C) val = d.w[((size_t)k * d.RS + rs) * d.C + c];
      d.fwd[t] = f2bf(val);
    }
  }
}

// dgrad image [C][R*S][K] = transpose of w[K][R*S][C] per tap: 64x64 (k, c) tiles through LDS so
// that both the fp32 reads (along c) and the bf16 writes (along k) are contiguous.  K, C multiples of 64 and 16-byte
// aligned operands (every conv but the stems): 16-byte loads (4 c) and stores (8 k) per thread; else one element.
__global__ __launch_bounds__(256) void pack_dgrad_batched_kernel(const PackDesc* __restrict__ descs) {
  __shared__ __attribute__((aligned(16))) float tile[64][68];
  const PackDesc d = descs[blockIdx.y];
  if (!d.dgrad) return;
  const int kt = (d.K + 63) / 64, ct = (d.C + 63) / 64;
  const int ntiles = d.RS * kt * ct;
  const bool vec = (d.K % 64 == 0) && (d.C % 64 == 0) && ((((uintptr_t)d.w) | ((uintptr_t)d.dgrad)) & 15) == 0;
  for (int tile_id = blockIdx.x; tile_id < ntiles; tile_id += gridDim.x) {
    const int rs = tile_id / (kt * ct);
    const int rem = tile_id - rs * kt * ct;
    const int k0 = (rem / ct) * 64, c0 = (rem % ct) * 64;
    __syncthreads();
    if (vec) {
      const int c4 = (threadIdx.x & 15) * 4;
#pragma unroll
      for (int i = 0; i < 4; ++i) {  // rows k0 + (tid / 16) + 16 i, columns c0 + c4 .. +3
        const int k = (int)(threadIdx.x >> 4) + 16 * i;
        const float4 v = *reinterpret_cast<const float4*>(d.w + ((size_t)(k0 + k) * d.RS + rs) * d.C + c0 + c4);
        *reinterpret_cast<float4*>(&tile[k][c4]) = v;
      }
      __syncthreads();
#pragma unroll
      for (int j = 0; j < 2; ++j) {  // output row c0 + q / 8, columns k0 + (q % 8) * 8 .. +7
        const int q = (int)threadIdx.x + 256 * j;
        const int c = q >> 3, kk = (q & 7) * 8;
        u32x4 o;
        o.x = pack2(tile[kk + 0][c], tile[kk + 1][c]);
        o.y = pack2(tile[kk + 2][c], tile[kk + 3][c]);
        o.z = pack2(tile[kk + 4][c], tile[kk + 5][c]);
        o.w = pack2(tile[kk + 6][c], tile[kk + 7][c]);
        *reinterpret_cast<u32x4*>(d.dgrad + ((size_t)(c0 + c) * d.RS + rs) * d.K + k0 + kk) = o;
      }
    } else {
      const int lx = threadIdx.x & 63, ly = threadIdx.x >> 6;  // 64 x 4
      for (int i = ly; i < 64; i += 4) {  // row k0+i, column c0+lx
        const int k = k0 + i, c = c0 + lx;
        tile[i][lx] = (k < d.K && c < d.C) ? d.w[((size_t)k * d.RS + rs) * d.C + c] : 0.f;
      }
      __syncthreads();
      for (int i = ly; i < 64; i += 4) {  // output row c0+i, column k0+lx
        const int c = c0 + i, k = k0 + lx;
        if (c < d.C && k < d.K) d.dgrad[((size_t)c * d.RS + rs) * d.K + k] = f2bf(tile[lx][i]);
      }
    }
  }
}

// x [N][C][T][H][W] fp32 -> y [(N T)][H][W][Cp] bf16 (channels >= C zero): 'b c t h w -> (b t) h w c'
// (train_hardway.py:130-131 einops fold); T = 1 is plain NCHW -> NHWC.
__global__ void nchw_to_nhwc_kernel(const float* __restrict__ x, bf16_t* __restrict__ y, int N, int C, int T, int H,
                                    int W, int Cp) {
  const long long hw_n = (long long)H * W;
  const long long total = (long long)N * T * hw_n;
  for (long long t = blockIdx.x * (long long)blockDim.x + threadIdx.x; t < total; t += (long long)gridDim.x * blockDim.x) {
    const long long r = t / hw_n;  // output image (n, tt)
    const long long hw = t % hw_n;
    const int n = (int)(r / T), tt = (int)(r % T);
    const float* src = x + ((size_t)n * C * T + tt) * hw_n + hw;  // + c*T*hw_n
    if (Cp == 4) {
      float v[4];
#pragma unroll
      for (int c = 0; c < 4; ++c) v[c] = c < C ? src[(size_t)c * T * hw_n] : 0.f;
      u32x2 o;
      o[0] = pack2(v[0], v[1]);
      o[1] = pack2(v[2], v[3]);
      *reinterpret_cast<u32x2*>(y + t * 4) = o;
    } else {
      for (int c = 0; c < Cp; ++c) y[t * Cp + c] = f2bf(c < C ? src[(size_t)c * T * hw_n] : 0.f);
    }
  }
}

// As nchw_to_nhwc_kernel, four consecutive pixels per thread: one float4 load per channel and one
// 8-/32-byte store, 32-bit index math (the generic form's 64-bit divisions and scalar accesses ran
// at ~3 TB/s).  Needs H*W % 4 == 0, x 16-byte aligned, Cp in {1, 4}, N*T*H*W*Cp < 2^31.
template <int CP>
__global__ void nchw_to_nhwc4_kernel(const float* __restrict__ x, bf16_t* __restrict__ y, int C, int T, int hw_n,
                                     int total4) {
  for (int q = blockIdx.x * blockDim.x + threadIdx.x; q < total4; q += gridDim.x * blockDim.x) {
    const int t = q * 4;  // first of the 4 pixels (same image: hw_n % 4 == 0)
    const int r = t / hw_n, hw = t - r * hw_n;
    const int n = r / T, tt = r - n * T;
    const float* src = x + ((size_t)n * C * T + tt) * hw_n + hw;
    if (CP == 4) {
      f32x4 v[4];
#pragma unroll
      for (int c = 0; c < 4; ++c)
        v[c] = c < C ? *reinterpret_cast<const f32x4*>(src + (size_t)c * T * hw_n) : f32x4{0.f, 0.f, 0.f, 0.f};
      u32x4 o0, o1;  // pixels (0, 1) and (2, 3), 4 channels each
      o0[0] = pack2(v[0][0], v[1][0]);
      o0[1] = pack2(v[2][0], v[3][0]);
      o0[2] = pack2(v[0][1], v[1][1]);
      o0[3] = pack2(v[2][1], v[3][1]);
      o1[0] = pack2(v[0][2], v[1][2]);
      o1[1] = pack2(v[2][2], v[3][2]);
      o1[2] = pack2(v[0][3], v[1][3]);
      o1[3] = pack2(v[2][3], v[3][3]);
      *reinterpret_cast<u32x4*>(y + (size_t)t * 4) = o0;
      *reinterpret_cast<u32x4*>(y + (size_t)t * 4 + 8) = o1;
    } else {
      const f32x4 v = *reinterpret_cast<const f32x4*>(src);
      u32x2 o;
      o[0] = pack2(v[0], v[1]);
      o[1] = pack2(v[2], v[3]);
      *reinterpret_cast<u32x2*>(y + t) = o;
    }
  }
}

static bool nhwc4_ok(const float* x, const void* y, long long N, int C, int T, int H, int W, int Cp) {
  const long long hw = (long long)H * W;
  return (Cp == 4 || (Cp == 1 && C == 1)) && hw % 4 == 0 && ((uintptr_t)x & 15) == 0 && ((uintptr_t)y & 15) == 0 &&
         N * T * hw * Cp < (1ll << 31) && C <= Cp;
}

// NHWC bf16 -> NCHW fp32 (hooks / returning trunk maps in the reference layout)
__global__ void nhwc_to_nchw_kernel(const bf16_t* __restrict__ x, float* __restrict__ y, int N, int C, int HW) {
  const long long total = (long long)N * C * HW;
  for (long long t = blockIdx.x * (long long)blockDim.x + threadIdx.x; t < total; t += (long long)gridDim.x * blockDim.x) {
    const int hw = (int)(t % HW);
    const long long r = t / HW;
    const int c = (int)(r % C), n = (int)(r / C);
    y[t] = bf2f(x[((size_t)n * HW + hw) * C + c]);
  }
}

// t = ++*step; coef = {lr / (1 - b1^t), sqrt(1 - b2^t), b1, b2, eps, wd} in double, as the host
// path computes them; hyper = device {lr, beta1, beta2, eps, weight_decay}
__global__ void adam_prep_kernel(int* __restrict__ step, const float* __restrict__ hyper, float* __restrict__ coef) {
  const int t = *step + 1;
  *step = t;
  const float lr = hyper[0], b1 = hyper[1], b2 = hyper[2];
  const double bc1 = 1.0 - pow((double)b1, t);
  const double bc2 = 1.0 - pow((double)b2, t);
  coef[0] = (float)(lr / bc1);
  coef[1] = (float)sqrt(bc2);
  coef[2] = b1;
  coef[3] = b2;
  coef[4] = hyper[3];
  coef[5] = hyper[4];
}

static int grid_for(long long n) {
  long long b = (n + 255) / 256;
  if (b > 8192) b = 8192;
  if (b < 1) b = 1;
  return (int)b;
}

// ---- measured peaks (bench.py's roofline denominators, re-measured on the box in the same run) ----
// Back-to-back bf16 MFMA on register operands holding pseudo-random bf16 values in [-1, 1) (the chip's
// clock under MFMA load depends on the operand bits: zeros clock ~19 % higher, MI355X_MICROARCH.md DVFS
// item 1), NACC independent accumulators per wave, one 256-thread block per CU = one wave per SIMD.
__device__ __forceinline__ unsigned peak_hash(unsigned x) {
  x ^= x >> 16;
  x *= 0x7feb352dU;
  x ^= x >> 15;
  x *= 0x846ca68bU;
  x ^= x >> 16;
  return x;
}

template <int SHAPE>  // 0: v_mfma_f32_32x32x16_bf16 (4 accumulators), 1: v_mfma_f32_16x16x32_bf16 (8)
__global__ __launch_bounds__(1024) void peak_mfma_kernel(float* __restrict__ sink, int iters, unsigned seed) {
  const unsigned g = blockIdx.x * 256u + threadIdx.x;
  bf16x8 a, b;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    // bf16 with a random mantissa and sign, exponent of [0.5, 1)
    const unsigned ha = peak_hash(seed ^ (g * 16u + j)), hb = peak_hash(~seed ^ (g * 16u + 8u + j));
    a[j] = __builtin_bit_cast(__bf16, (unsigned short)(0x3f00u | (ha & 0x807fu)));
    b[j] = __builtin_bit_cast(__bf16, (unsigned short)(0x3f00u | (hb & 0x807fu)));
  }
  float s = 0.f;
  if constexpr (SHAPE == 0) {
    f32x16 acc[4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int v = 0; v < 16; ++v) acc[i][v] = 0.f;
#pragma nounroll
    for (int it = 0; it < iters; ++it)
#pragma unroll
      for (int i = 0; i < 4; ++i) acc[i] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, acc[i], 0, 0, 0);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int v = 0; v < 16; ++v) s += acc[i][v];
  } else {
    f32x4 acc[8];
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int v = 0; v < 4; ++v) acc[i][v] = 0.f;
    // (bounds of 1024 threads keep the accumulators in VGPRs: at 256 the allocator put them in AGPRs and
    // rotated them through ~50 accvgpr moves per iteration, which halved the measured 16x16x32 rate)
#pragma nounroll
    for (int it = 0; it < iters; ++it)
#pragma unroll
      for (int i = 0; i < 8; ++i) acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, acc[i], 0, 0, 0);
#pragma unroll
    for (int i = 0; i < 8; ++i) s += (acc[i][0] + acc[i][1]) + (acc[i][2] + acc[i][3]);
  }
  sink[g] = s;  // keeps the loop live; one vector store per lane
}

// grid-stride 16-byte copy (the HBM read + write rate a streaming kernel reaches on this box)
__global__ __launch_bounds__(256) void copy16_kernel(const u32x4* __restrict__ src, u32x4* __restrict__ dst, long long n) {
  for (long long i = blockIdx.x * 256ll + threadIdx.x; i < n; i += (long long)gridDim.x * 256) dst[i] = src[i];
}


// ---- input gradient of the 7x7 / s2 / p3 stem conv ----
// One thread per input pixel (n, h, w): the output positions (p, q) that read it are p = (h + 3 - r) / 2 for the
// rows r of matching parity (<= 4 of the 7), likewise q; gx[c] = sum over those (r, s) and the 64 output channels
// of gy[n][p][q][k] * w[k][r][s][c], in a fixed order.  The weights (64 x 49 x Cin fp32) sit in LDS tap-major
// ([r][s][k][4]).  VALU work: an optional path (only when the trunk input requires grad), not the train step's.
constexpr int kStemDgThreads = 256;
__global__ __launch_bounds__(kStemDgThreads) void stem_dgrad_kernel(const bf16_t* __restrict__ gy,
                                                                   const float* __restrict__ w, float* __restrict__ gx,
                                                                   int N, int H, int W, int P, int Q, int Cin) {
  __shared__ float ws[49 * 64 * 4];
  for (int i = threadIdx.x; i < 49 * 64 * 4; i += kStemDgThreads) {
    const int c = i & 3, k = (i >> 2) & 63, t = i >> 8;  // t = r * 7 + s
    ws[i] = c < Cin ? w[((size_t)k * 49 + t) * Cin + c] : 0.f;
  }
  __syncthreads();
  const long long pix = blockIdx.x * (long long)kStemDgThreads + threadIdx.x;
  if (pix >= (long long)N * H * W) return;
  const int n = (int)(pix / ((long long)H * W));
  const int rem = (int)(pix - (long long)n * H * W);
  const int h = rem / W, x = rem - h * W;
  float acc[4] = {0.f, 0.f, 0.f, 0.f};
  for (int r = (h + 3) & 1; r < 7; r += 2) {
    const int p = (h + 3 - r) >> 1;
    if (p < 0 || p >= P) continue;
    for (int s = (x + 3) & 1; s < 7; s += 2) {
      const int q = (x + 3 - s) >> 1;
      if (q < 0 || q >= Q) continue;
      const u32x4* row = reinterpret_cast<const u32x4*>(gy + (((size_t)n * P + p) * Q + q) * 64);
      const float* wt = ws + (r * 7 + s) * 256;
#pragma unroll 2
      for (int k8 = 0; k8 < 8; ++k8) {
        const u32x4 v = row[k8];
        const unsigned* u = reinterpret_cast<const unsigned*>(&v);
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float g = bf2f((bf16_t)(e & 1 ? u[e >> 1] >> 16 : u[e >> 1] & 0xffff));
          const float4 wk = *reinterpret_cast<const float4*>(wt + (k8 * 8 + e) * 4);
          acc[0] += g * wk.x;
          acc[1] += g * wk.y;
          acc[2] += g * wk.z;
          acc[3] += g * wk.w;
        }
      }
    }
  }
  for (int c = 0; c < Cin; ++c) gx[(((size_t)n * Cin + c) * H + h) * W + x] = acc[c];
}
}  // namespace avt

using namespace avt;

extern "C" const char* avt_last_error(void) { return g_err; }

extern "C" int avt_abi_version(void) { return 1; }

extern "C" int avt_build_flags(void) {
#ifdef AVT_DIAG
  return AVT_BUILD_DIAG;
#else
  return 0;
#endif
}

extern "C" long long avt_peak_mfma_flops(int shape, int blocks, int iters) {
  if ((shape != 0 && shape != 1) || blocks < 1 || iters < 1) return -1;
  // 32x32x16: 4 accumulators x 32*32*16*2 FLOP; 16x16x32: 8 x 16*16*32*2 -- per wave and iteration
  const long long per_wave_iter = shape == 0 ? 4ll * 32768 : 8ll * 16384;
  return per_wave_iter * iters * blocks * 4;
}

extern "C" int avt_peak_mfma(float* sink, int shape, int blocks, int iters, unsigned seed, void* stream) {
  AVT_REQUIRE(sink && (shape == 0 || shape == 1) && blocks >= 1 && iters >= 1, "peak_mfma: bad arguments");
  if (shape == 0)
    hipLaunchKernelGGL(peak_mfma_kernel<0>, dim3(blocks), dim3(256), 0, (hipStream_t)stream, sink, iters, seed);
  else
    hipLaunchKernelGGL(peak_mfma_kernel<1>, dim3(blocks), dim3(256), 0, (hipStream_t)stream, sink, iters, seed);
  return check_launch("peak_mfma");
}

extern "C" int avt_copy16(void* dst, const void* src, size_t bytes, int blocks, void* stream) {
  AVT_REQUIRE(dst && src && bytes % 16 == 0 && blocks >= 1, "copy16: bad arguments");
  AVT_REQUIRE(((uintptr_t)dst | (uintptr_t)src) % 16 == 0, "copy16: buffers must be 16-byte aligned");
  hipLaunchKernelGGL(copy16_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, (const u32x4*)src, (u32x4*)dst,
                     (long long)(bytes / 16));
  return check_launch("copy16");
}

// torch.optim.Adam (amsgrad=False, maximize=False) with coupled L2 weight decay on one flat segment;
// grad is multiplied by grad_scale first (1/world for a summed all-reduce).
extern "C" int avt_adam_step(float* param, const float* grad, float* exp_avg, float* exp_avg_sq, long long n,
                             float grad_scale, float lr, float beta1, float beta2, float eps, float weight_decay,
                             int step, void* stream) {
  AVT_REQUIRE(param && grad && exp_avg && exp_avg_sq, "adam_step: null pointer");
  AVT_REQUIRE(step >= 1, "adam_step: step must be >= 1");
  AVT_REQUIRE(((uintptr_t)param | (uintptr_t)grad | (uintptr_t)exp_avg | (uintptr_t)exp_avg_sq) % 16 == 0,
              "adam_step: buffers must be 16-byte aligned");
  if (n == 0) return AVT_OK;
  const double bc1 = 1.0 - pow((double)beta1, step);
  const double bc2 = 1.0 - pow((double)beta2, step);
  const float step_size = (float)(lr / bc1);
  const float bc2_sqrt = (float)sqrt(bc2);
  hipLaunchKernelGGL(adam_kernel, dim3(grid_for(n / 4 + 1)), dim3(256), 0, (hipStream_t)stream, param, grad, exp_avg,
                     exp_avg_sq, n, grad_scale, beta1, beta2, eps, weight_decay, step_size, bc2_sqrt, nullptr);
  return check_launch("adam_step");
}

// Same update with the step counter AND the hyper-parameters on the device: hyper = {lr, beta1,
// beta2, eps, weight_decay} (5 floats, read at every launch), step an int incremented here, the bias
// corrections computed there.  Every launch argument is step-invariant, so the call can be captured
// once into a HIP graph and replayed, and a learning-rate schedule (MultiStepLR,
// train_hardway_1frame.py:118) or a restored checkpoint takes effect by writing `hyper`.
// coef: AVT_ADAM_COEF_FLOATS floats of scratch.
extern "C" int avt_adam_step_dev(float* param, const float* grad, float* exp_avg, float* exp_avg_sq, long long n,
                                 float grad_scale, const float* hyper, int* step, float* coef, void* stream) {
  AVT_REQUIRE(param && grad && exp_avg && exp_avg_sq && hyper && step && coef, "adam_step_dev: null pointer");
  AVT_REQUIRE(((uintptr_t)param | (uintptr_t)grad | (uintptr_t)exp_avg | (uintptr_t)exp_avg_sq) % 16 == 0,
              "adam_step_dev: buffers must be 16-byte aligned");
  if (n == 0) return AVT_OK;
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(adam_prep_kernel, dim3(1), dim3(1), 0, st, step, hyper, coef);
  hipLaunchKernelGGL(adam_kernel, dim3(grid_for(n / 4 + 1)), dim3(256), 0, st, param, grad, exp_avg, exp_avg_sq, n,
                     grad_scale, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, (const float*)coef);
  return check_launch("adam_step_dev");
}

extern "C" int avt_pack_conv_weight(const float* w, int K, int R, int S, int C, int Cp, int Kg, void* out_fwd,
                                    void* out_dgrad, void* stream) {
  AVT_REQUIRE(w, "pack_conv_weight: null pointer");
  AVT_REQUIRE(Cp >= C && Kg >= R * S * Cp, "pack_conv_weight: bad padding");
  hipStream_t st = (hipStream_t)stream;
  if (out_fwd)
    hipLaunchKernelGGL(pack_fwd_kernel, dim3(grid_for((long long)K * Kg)), dim3(256), 0, st, w, (bf16_t*)out_fwd, K,
                       R * S, C, Cp, Kg);
  if (out_dgrad)
    hipLaunchKernelGGL(pack_dgrad_kernel, dim3(grid_for((long long)K * R * S * C)), dim3(256), 0, st, w,
                       (bf16_t*)out_dgrad, K, R * S, C);
  return check_launch("pack_conv_weight");
}

// descs: device array of n records {const float* w; void* fwd; void* dgrad; int K, RS, C, Cp, Kg, pad}
// (48 bytes each, layout of PackDesc); two launches pack every conv weight of the model.
extern "C" size_t avt_pack_desc_bytes(void) { return sizeof(PackDesc); }

extern "C" int avt_conv_stem_dgrad(const void* gy, const float* w, float* gx, int N, int H, int W, int Cin,
                                   void* stream) {
  AVT_REQUIRE(gy && w && gx, "conv_stem_dgrad: null pointer");
  AVT_REQUIRE(N > 0 && H > 0 && W > 0 && Cin >= 1 && Cin <= 4, "conv_stem_dgrad: N=%d H=%d W=%d Cin=%d", N, H, W, Cin);
  const int P = (H + 6 - 7) / 2 + 1, Q = (W + 6 - 7) / 2 + 1;
  const long long pix = (long long)N * H * W;
  AVT_REQUIRE(pix < (1LL << 31) * (long long)kStemDgThreads, "conv_stem_dgrad: input too large");
  hipLaunchKernelGGL(stem_dgrad_kernel, dim3((unsigned)((pix + kStemDgThreads - 1) / kStemDgThreads)),
                     dim3(kStemDgThreads), 0, (hipStream_t)stream, (const bf16_t*)gy, w, gx, N, H, W, P, Q, Cin);
  return check_launch("conv_stem_dgrad");
}

extern "C" int avt_pack_conv_weights_batched(const void* descs, int n, long long max_elems, void* stream) {
  AVT_REQUIRE(descs && n > 0, "pack_conv_weights_batched: bad arguments");
  AVT_REQUIRE(max_elems >= 0 && max_elems < (1ll << 31), "pack_conv_weights_batched: max_elems out of range");
  long long bx = (max_elems / 8 + 255) / 256;  // fwd: 8 elements per thread
  if (bx > 1024) bx = 1024;
  if (bx < 1) bx = 1;
  long long tx = max_elems / 4096 + 1;  // dgrad: 64x64 tiles
  if (tx > 512) tx = 512;
  hipLaunchKernelGGL(pack_fwd_batched_kernel, dim3((unsigned)bx, n), dim3(256), 0, (hipStream_t)stream,
                     (const PackDesc*)descs);
  hipLaunchKernelGGL(pack_dgrad_batched_kernel, dim3((unsigned)tx, n), dim3(256), 0, (hipStream_t)stream,
                     (const PackDesc*)descs);
  return check_launch("pack_conv_weights_batched");
}

// One of the two launches of avt_pack_conv_weights_batched: which = 1 the fwd images, 2 the dgrad images
// (the step issues each trunk's fwd pack at the head of its own branch and the dgrad packs, needed
// only by the backward, behind the shorter trunk's forward)
extern "C" int avt_pack_conv_weights_part(const void* descs, int n, long long max_elems, int which, void* stream) {
  AVT_REQUIRE(descs && n > 0 && (which == 1 || which == 2), "pack_conv_weights_part: bad arguments");
  AVT_REQUIRE(max_elems >= 0 && max_elems < (1ll << 31), "pack_conv_weights_part: max_elems out of range");
  if (which == 1) {
    long long bx = (max_elems / 8 + 255) / 256;
    bx = bx > 1024 ? 1024 : (bx < 1 ? 1 : bx);
    hipLaunchKernelGGL(pack_fwd_batched_kernel, dim3((unsigned)bx, n), dim3(256), 0, (hipStream_t)stream,
                       (const PackDesc*)descs);
  } else {
    long long tx = max_elems / 4096 + 1;
    tx = tx > 512 ? 512 : tx;
    hipLaunchKernelGGL(pack_dgrad_batched_kernel, dim3((unsigned)tx, n), dim3(256), 0, (hipStream_t)stream,
                       (const PackDesc*)descs);
  }
  return check_launch("pack_conv_weights_part");
}

// avt_adam_step_dev in two parts: prep advances the device step counter and writes coef once per step;
// apply updates one 16-byte-aligned region from coef -- the train step updates each trunk's region at
// the end of that trunk's backward branch (the shorter trunk's update overlaps the longer's backward)
extern "C" int avt_adam_prep_dev(const float* hyper, int* step, float* coef, void* stream) {
  AVT_REQUIRE(hyper && step && coef, "adam_prep_dev: null pointer");
  hipLaunchKernelGGL(adam_prep_kernel, dim3(1), dim3(1), 0, (hipStream_t)stream, step, hyper, coef);
  return check_launch("adam_prep_dev");
}

extern "C" int avt_adam_apply_dev(float* param, const float* grad, float* exp_avg, float* exp_avg_sq, long long n,
                                  float grad_scale, const float* coef, void* stream) {
  AVT_REQUIRE(param && grad && exp_avg && exp_avg_sq && coef, "adam_apply_dev: null pointer");
  AVT_REQUIRE(((uintptr_t)param | (uintptr_t)grad | (uintptr_t)exp_avg | (uintptr_t)exp_avg_sq) % 16 == 0,
              "adam_apply_dev: buffers must be 16-byte aligned");
  if (n == 0) return AVT_OK;
  hipLaunchKernelGGL(adam_kernel, dim3(grid_for(n / 4 + 1)), dim3(256), 0, (hipStream_t)stream, param, grad, exp_avg,
                     exp_avg_sq, n, grad_scale, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, coef);
  return check_launch("adam_apply_dev");
}

extern "C" int avt_nchw_to_nhwc_bf16(const float* x, void* y, int N, int C, int H, int W, int Cp, void* stream) {
  AVT_REQUIRE(x && y && Cp >= C, "nchw_to_nhwc_bf16: bad arguments");
  if (nhwc4_ok(x, y, N, C, 1, H, W, Cp)) {
    const int total4 = (int)((long long)N * H * W / 4);
    if (Cp == 4)
      hipLaunchKernelGGL(nchw_to_nhwc4_kernel<4>, dim3(grid_for(total4)), dim3(256), 0, (hipStream_t)stream, x,
                         (bf16_t*)y, C, 1, H * W, total4);
    else
      hipLaunchKernelGGL(nchw_to_nhwc4_kernel<1>, dim3(grid_for(total4)), dim3(256), 0, (hipStream_t)stream, x,
                         (bf16_t*)y, C, 1, H * W, total4);
    return check_launch("nchw_to_nhwc_bf16");
  }
  hipLaunchKernelGGL(nchw_to_nhwc_kernel, dim3(grid_for((long long)N * H * W)), dim3(256), 0, (hipStream_t)stream, x,
                     (bf16_t*)y, N, C, 1, H, W, Cp);
  return check_launch("nchw_to_nhwc_bf16");
}

extern "C" int avt_ncthw_to_nhwc_bf16(const float* x, void* y, int N, int C, int T, int H, int W, int Cp,
                                      void* stream) {
  AVT_REQUIRE(x && y && Cp >= C && T >= 1, "ncthw_to_nhwc_bf16: bad arguments");
  AVT_REQUIRE(Cp != 4 || ((uintptr_t)y & 7) == 0, "ncthw_to_nhwc_bf16: y must be 8-byte aligned");
  hipLaunchKernelGGL(nchw_to_nhwc_kernel, dim3(grid_for((long long)N * T * H * W)), dim3(256), 0, (hipStream_t)stream,
                     x, (bf16_t*)y, N, C, T, H, W, Cp);
  return check_launch("ncthw_to_nhwc_bf16");
}

extern "C" int avt_nhwc_bf16_to_nchw(const void* x, float* y, int N, int C, int HW, void* stream) {
  AVT_REQUIRE(x && y, "nhwc_bf16_to_nchw: null pointer");
  hipLaunchKernelGGL(nhwc_to_nchw_kernel, dim3(grid_for((long long)N * C * HW)), dim3(256), 0, (hipStream_t)stream,
                     (const bf16_t*)x, y, N, C, HW);
  return check_launch("nhwc_bf16_to_nchw");
}
