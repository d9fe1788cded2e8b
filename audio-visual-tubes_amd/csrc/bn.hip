// Train-mode BatchNorm2d (+ReLU, +residual) for the ResNet-18 trunks, NHWC bf16 activations,
// fp32 math, fp64 statistic accumulation.  Semantics of torch BatchNorm2d as used at
// models/base_models.py:39,46-49,120-121,141 (eps 1e-5, momentum 0.1): normalise with the biased
// batch variance, update running_var with the unbiased one.
//
//   fwd : the conv epilogue adds per-128-row-tile (sum_t, M2_t, sum_t^2/n_t) into an fp64
//         accumulator [AVT_BN_SLOTS][C][3]; bn_finalize merges the slots exactly
//         (M2 = sum M2_t + sum sum_t^2/n_t - S^2/N, Chan's formula), writes scale/shift/mean/invstd,
//         updates running stats and re-zeroes the accumulator; bn_apply (+residual, +ReLU).
//   bwd : bn_bwd_reduce adds per-block (sum g', sum g'*xhat) (g' = g*[y>0]) into an fp64
//         accumulator [AVT_BN_SLOTS][C][2] -> bn_bwd_finalize (dgamma, dbeta, k1, k2; re-zeroes) ->
//         bn_bwd_apply: g_c = gamma*invstd*(g' - k1 - xhat*k2).
//         avt_bn_relu_bwd recomputes the ReLU mask from (xc, scale, shift) instead of reading y
//         (BasicBlock.bn1, base_models.py:47-48); the stem's bn1+relu+maxpool is fused both ways
//         (avt_stem_*, below) so its full-resolution activation is never stored.
#include "avt_common.h"

namespace avt {

__device__ __forceinline__ void unpack8(const u32x4& v, float* f) {
  const unsigned* u = reinterpret_cast<const unsigned*>(&v);
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    f[2 * e] = bf2f(u[e] & 0xffff);
    f[2 * e + 1] = bf2f(u[e] >> 16);
  }
}
__device__ __forceinline__ u32x4 pack8(const float* f) {
  u32x4 v;
  v.x = pack2(f[0], f[1]);
  v.y = pack2(f[2], f[3]);
  v.z = pack2(f[4], f[5]);
  v.w = pack2(f[6], f[7]);
  return v;
}

// one thread per channel
__global__ __launch_bounds__(256) void bn_finalize_kernel(double* __restrict__ acc, long long rows, int C,
                                                          const float* __restrict__ gamma,
                                                          const float* __restrict__ beta, float* running_mean,
                                                          float* running_var, float momentum, float eps, float* scale,
                                                          float* shift, float* save_mean, float* save_invstd) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  double S = 0.0, Q = 0.0, R = 0.0;
#pragma unroll
  for (int s = 0; s < AVT_BN_SLOTS; ++s) {
    double* a = acc + ((size_t)s * C + c) * 3;
    S += a[0];
    Q += a[1];
    R += a[2];
    a[0] = 0.0;
    a[1] = 0.0;
    a[2] = 0.0;
  }
  const double n = (double)rows;
  const double mean = S / n;
  double m2 = Q + (R - S * mean);
  if (m2 < 0.0) m2 = 0.0;
  const float var = (float)(m2 / n);
  const float inv = rsqrtf(var + eps);
  const float sc = gamma[c] * inv;
  scale[c] = sc;
  shift[c] = beta[c] - (float)mean * sc;
  if (save_mean) save_mean[c] = (float)mean;
  if (save_invstd) save_invstd[c] = inv;
  if (running_mean) {
    const float unb = n > 1.0 ? (float)(m2 / (n - 1.0)) : var;
    running_mean[c] = (1.f - momentum) * running_mean[c] + momentum * (float)mean;
    running_var[c] = (1.f - momentum) * running_var[c] + momentum * unb;
  }
}

// out = [relu]( x*scale + shift + [residual*rscale + rshift | residual] )
// The channel block of vector i is i % (C/8); POW2 (C/8 a power of two) takes it as a bit mask.
// The per-channel constants are re-read every iteration (L1 hits): hoisting them costs enough
// VGPRs to drop occupancy, which this HBM-bound loop needs more.
template <bool POW2>
__device__ __forceinline__ int chan_block(long long i, int cv) {
  return POW2 ? (int)((unsigned)i & (unsigned)(cv - 1)) : (int)(i % cv);
}

template <bool POW2>
__global__ __launch_bounds__(256) void bn_apply_kernel(const bf16_t* __restrict__ x, const float* __restrict__ scale,
                                                       const float* __restrict__ shift,
                                                       const bf16_t* __restrict__ res, const float* __restrict__ rscale,
                                                       const float* __restrict__ rshift, bf16_t* __restrict__ out,
                                                       long long nvec, int C, int relu) {
  const int cv = C / 8;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < nvec; i += (long long)gridDim.x * blockDim.x) {
    const int c0 = chan_block<POW2>(i, cv) * 8;
    float f[8];
    unpack8(reinterpret_cast<const u32x4*>(x)[i], f);
#pragma unroll
    for (int e = 0; e < 8; ++e) f[e] = __builtin_fmaf(f[e], scale[c0 + e], shift[c0 + e]);
    if (res) {
      float r[8];
      unpack8(reinterpret_cast<const u32x4*>(res)[i], r);
      if (rscale) {
#pragma unroll
        for (int e = 0; e < 8; ++e) f[e] += r[e] * rscale[c0 + e] + rshift[c0 + e];
      } else {
#pragma unroll
        for (int e = 0; e < 8; ++e) f[e] += r[e];
      }
    }
    if (relu) {
#pragma unroll
      for (int e = 0; e < 8; ++e) f[e] = fmaxf(f[e], 0.f);
    }
    reinterpret_cast<u32x4*>(out)[i] = pack8(f);
  }
}

// ReLU mask of the backward pass.  Either read from the saved output y (y > 0) or recomputed
// from the pre-activation: relu(fma(xc, mscale, mshift)) > 0 -- the exact expression bn_apply
// evaluated in the forward, so the mask is identical without re-reading y.
__device__ __forceinline__ void relu_mask8(float* gg, const float* xx, const bf16_t* __restrict__ y, size_t off,
                                           const float* __restrict__ mscale, const float* __restrict__ mshift,
                                           int c0) {
  if (y) {
    float yy[8];
    unpack8(reinterpret_cast<const u32x4*>(y)[off], yy);
#pragma unroll
    for (int e = 0; e < 8; ++e) gg[e] = yy[e] > 0.f ? gg[e] : 0.f;
  } else if (mscale) {
#pragma unroll
    for (int e = 0; e < 8; ++e) gg[e] = __builtin_fmaf(xx[e], mscale[c0 + e], mshift[c0 + e]) > 0.f ? gg[e] : 0.f;
  }
}

// Per-block sums of g' and g'*xhat added into acc[block % SLOTS][C][2].  Block: 256 threads; a
// thread owns channel chunk (tid % (C/8)) and walks rows tid/(C/8) + k*(256/(C/8)).
__global__ __launch_bounds__(256) void bn_bwd_reduce_kernel(const bf16_t* __restrict__ g, const bf16_t* __restrict__ y,
                                                            const float* __restrict__ mscale,
                                                            const float* __restrict__ mshift,
                                                            const bf16_t* __restrict__ xc, const float* __restrict__ mean,
                                                            const float* __restrict__ invstd, double* __restrict__ acc,
                                                            long long rows, int C, int rows_per_block) {
  __shared__ float red[2048 * 2];  // [256/(C/8)][C][2] = 4096 floats for any C
  const int cv = C / 8;
  const int chunk = threadIdx.x % cv, r0 = threadIdx.x / cv, rstep = 256 / cv;
  const int c0 = chunk * 8;
  float mu[8], is[8], s1[8], s2[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    mu[e] = mean[c0 + e];
    is[e] = invstd[c0 + e];
    s1[e] = 0.f;
    s2[e] = 0.f;
  }
  const long long rbeg = (long long)blockIdx.x * rows_per_block;
  const long long rend = min(rows, rbeg + rows_per_block);
  for (long long r = rbeg + r0; r < rend; r += rstep) {
    const size_t off = (size_t)r * cv + chunk;
    float gg[8], xx[8];
    unpack8(reinterpret_cast<const u32x4*>(g)[off], gg);
    unpack8(reinterpret_cast<const u32x4*>(xc)[off], xx);
    relu_mask8(gg, xx, y, off, mscale, mshift, c0);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      s1[e] += gg[e];
      s2[e] += gg[e] * (xx[e] - mu[e]) * is[e];
    }
  }
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    red[(r0 * C + c0 + e) * 2] = s1[e];
    red[(r0 * C + c0 + e) * 2 + 1] = s2[e];
  }
  __syncthreads();
  double* slot = acc + (size_t)(blockIdx.x % AVT_BN_SLOTS) * C * 2;
  for (int c = threadIdx.x; c < C; c += blockDim.x) {
    float a = 0.f, b = 0.f;
    for (int k = 0; k < rstep; ++k) {
      a += red[(k * C + c) * 2];
      b += red[(k * C + c) * 2 + 1];
    }
    atomicAdd(slot + 2 * c, (double)a);
    atomicAdd(slot + 2 * c + 1, (double)b);
  }
}

// dgamma/dbeta (accumulated into the gradient if non-null) and k1,k2; re-zeroes acc.
__global__ __launch_bounds__(256) void bn_bwd_finalize_kernel(double* __restrict__ acc, int C, double inv_rows,
                                                              float* dgamma, float* dbeta, float* k1, float* k2) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  double a = 0.0, b = 0.0;
#pragma unroll
  for (int s = 0; s < AVT_BN_SLOTS; ++s) {
    double* p = acc + ((size_t)s * C + c) * 2;
    a += p[0];
    b += p[1];
    p[0] = 0.0;
    p[1] = 0.0;
  }
  if (dbeta) dbeta[c] += (float)a;
  if (dgamma) dgamma[c] += (float)b;
  k1[c] = (float)(a * inv_rows);
  k2[c] = (float)(b * inv_rows);
}

// g_c = gamma*invstd*(g' - k1 - xhat*k2); optionally also writes g' (masked grad) to gmask_out.
template <bool POW2>
__global__ __launch_bounds__(256) void bn_bwd_apply_kernel(const bf16_t* __restrict__ g, const bf16_t* __restrict__ y,
                                                           const float* __restrict__ mscale,
                                                           const float* __restrict__ mshift,
                                                           const bf16_t* __restrict__ xc, const float* __restrict__ mean,
                                                           const float* __restrict__ invstd,
                                                           const float* __restrict__ gamma, const float* __restrict__ k1,
                                                           const float* __restrict__ k2, bf16_t* __restrict__ gc,
                                                           bf16_t* __restrict__ gmask_out, long long nvec, int C) {
  const int cv = C / 8;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < nvec; i += (long long)gridDim.x * blockDim.x) {
    const int c0 = chan_block<POW2>(i, cv) * 8;
    float gg[8], xx[8], o[8];
    unpack8(reinterpret_cast<const u32x4*>(g)[i], gg);
    unpack8(reinterpret_cast<const u32x4*>(xc)[i], xx);
    relu_mask8(gg, xx, y, (size_t)i, mscale, mshift, c0);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int c = c0 + e;
      const float xh = (xx[e] - mean[c]) * invstd[c];
      o[e] = gamma[c] * invstd[c] * (gg[e] - k1[c] - xh * k2[c]);
    }
    reinterpret_cast<u32x4*>(gc)[i] = pack8(o);
    if (gmask_out) reinterpret_cast<u32x4*>(gmask_out)[i] = pack8(gg);
  }
}

static int ew_grid(long long nvec) {
  long long b = (nvec + 255) / 256;
  if (b > 4096) b = 4096;
  if (b < 1) b = 1;
  return (int)b;
}

// ---------------------------------------------------------------------------------------------
// Stem: bn1 -> relu -> MaxPool2d(3,2,1) (models/base_models.py:200-203) without materialising the
// full-resolution activation h0 = relu(bn(c0)), the largest tensor of either trunk.
//   fwd : one thread per (pooled pixel, 8 channels) evaluates h0 on its 3x3 window exactly as
//         bn_apply would (fma, relu, bf16 round), keeps the first max, and writes the pooled value,
//         the window argmax and carg = c0 at the argmax (the only pre-activations the backward's
//         reduction needs).
//   bwd : g'(h,w) = [h0(h,w) > 0] * sum of gy over the windows whose argmax is (h,w).  Its two
//         BN reductions (sum g', sum g'*xhat) are taken over the pooled grid from (gy, carg) --
//         a position picked by several windows contributes once per window, which sums to the
//         same total -- and the apply pass gathers g' per input pixel like maxpool3s2_bwd.
// One block per output row (n, p) [fwd] / input row (n, h) [bwd]; the block's threads stride over
// that row's (column, 8-channel block) items; cv = C/8 = 1 << cvs.
__global__ __launch_bounds__(256) void stem_bn_relu_maxpool_fwd_kernel(
    const bf16_t* __restrict__ c, const float* __restrict__ scale, const float* __restrict__ shift,
    bf16_t* __restrict__ y, unsigned char* __restrict__ idx, bf16_t* __restrict__ carg, int H, int W, int C, int cvs,
    int P, int Q) {
  const int row = blockIdx.x;  // n * P + p
  const int n = row / P, p = row - n * P;
  const int cv = 1 << cvs;
  const int r_lo = p == 0 ? 1 : 0, r_hi = min(2, H - 1 - (2 * p - 1));
  const bf16_t* cimg = c + (size_t)n * H * W * C;
  for (int t = threadIdx.x; t < Q * cv; t += 256) {
    const int q = t >> cvs, c8 = t & (cv - 1);
    float sc[8], sh[8], best[8], bc[8];
    int bi[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      sc[e] = scale[c8 * 8 + e];
      sh[e] = shift[c8 * 8 + e];
      best[e] = -INFINITY;
      bc[e] = 0.f;
      bi[e] = 0;
    }
    for (int r = r_lo; r <= r_hi; ++r) {
      const int h = p * 2 - 1 + r;
      for (int s = 0; s < 3; ++s) {
        const int w = q * 2 - 1 + s;
        if (w < 0 || w >= W) continue;
        float xv[8];
        unpack8(*reinterpret_cast<const u32x4*>(cimg + ((size_t)h * W + w) * C + c8 * 8), xv);
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float f = bf2f(f2bf(fmaxf(__builtin_fmaf(xv[e], sc[e], sh[e]), 0.f)));
          if (f > best[e] || f != f) {
            best[e] = f;
            bc[e] = xv[e];
            bi[e] = r * 3 + s;
          }
        }
      }
    }
    const size_t off = ((size_t)row * Q + q) * C + c8 * 8;
    *reinterpret_cast<u32x4*>(y + off) = pack8(best);
    *reinterpret_cast<u32x4*>(carg + off) = pack8(bc);
    unsigned long long ib = 0;
#pragma unroll
    for (int e = 0; e < 8; ++e) ib |= (unsigned long long)bi[e] << (8 * e);
    *reinterpret_cast<unsigned long long*>(idx + off) = ib;
  }
}

__global__ __launch_bounds__(256) void stem_maxpool_bn_bwd_apply_kernel(
    const bf16_t* __restrict__ gy, const unsigned char* __restrict__ idx, const bf16_t* __restrict__ c,
    const float* __restrict__ scale, const float* __restrict__ shift, const float* __restrict__ mean,
    const float* __restrict__ invstd, const float* __restrict__ gamma, const float* __restrict__ k1,
    const float* __restrict__ k2, bf16_t* __restrict__ gc, int H, int W, int C, int cvs, int P, int Q) {
  const int row = blockIdx.x;  // n * H + h
  const int n = row / H, h = row - n * H;
  const int cv = 1 << cvs;
  // pooled rows p with 2p-1 <= h <= 2p+1, and the window row kh = h - (2p-1) in each
  const int p_lo = h >> 1, p_hi = min(P - 1, (h + 1) >> 1);
  for (int t = threadIdx.x; t < W * cv; t += 256) {
    const int w = t >> cvs, c8 = t & (cv - 1);
    float gg[8], xx[8], o[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) gg[e] = 0.f;
    const int q_lo = w >> 1, q_hi = min(Q - 1, (w + 1) >> 1);
    for (int p = p_lo; p <= p_hi; ++p) {
      const int kh = h - (2 * p - 1);
      for (int q = q_lo; q <= q_hi; ++q) {
        const int pos = kh * 3 + (w - (2 * q - 1));
        const size_t off = (((size_t)n * P + p) * Q + q) * C + c8 * 8;
        const unsigned long long ib = *reinterpret_cast<const unsigned long long*>(idx + off);
        float gv[8];
        unpack8(*reinterpret_cast<const u32x4*>(gy + off), gv);
#pragma unroll
        for (int e = 0; e < 8; ++e)
          if ((int)((ib >> (8 * e)) & 0xff) == pos) gg[e] += gv[e];
      }
    }
    const size_t xo = ((size_t)row * W + w) * C + c8 * 8;
    unpack8(*reinterpret_cast<const u32x4*>(c + xo), xx);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int ch = c8 * 8 + e;
      gg[e] = __builtin_fmaf(xx[e], scale[ch], shift[ch]) > 0.f ? gg[e] : 0.f;
      const float xh = (xx[e] - mean[ch]) * invstd[ch];
      o[e] = gamma[ch] * invstd[ch] * (gg[e] - k1[ch] - xh * k2[ch]);
    }
    *reinterpret_cast<u32x4*>(gc + xo) = pack8(o);
  }
}

static void bn_bwd_reduce_launch(const bf16_t* g, const bf16_t* y, const float* mscale, const float* mshift,
                                 const bf16_t* xc, const float* mean, const float* invstd, double* acc, long long rows,
                                 int C, hipStream_t st) {
  // ~2 blocks per CU of rows
  long long rpb = (rows + 511) / 512;
  const int rstep = 256 / (C / 8);
  rpb = ((rpb + rstep - 1) / rstep) * rstep;
  if (rpb < rstep) rpb = rstep;
  const int nblk = (int)((rows + rpb - 1) / rpb);
  hipLaunchKernelGGL(bn_bwd_reduce_kernel, dim3(nblk), dim3(256), 0, st, g, y, mscale, mshift, xc, mean, invstd, acc,
                     rows, C, (int)rpb);
}

}  // namespace avt

using namespace avt;

extern "C" size_t avt_bn_acc_doubles(int C) { return (size_t)AVT_BN_SLOTS * C * 3; }

extern "C" int avt_bn_finalize(double* acc, long long rows, int C, const float* gamma, const float* beta,
                               float* running_mean, float* running_var, float momentum, float eps, float* scale,
                               float* shift, float* save_mean, float* save_invstd, void* stream) {
  AVT_REQUIRE(acc && gamma && beta && scale && shift, "bn_finalize: null pointer");
  AVT_REQUIRE(rows > 0 && C > 0, "bn_finalize: empty input");
  hipLaunchKernelGGL(bn_finalize_kernel, dim3((C + 255) / 256), dim3(256), 0, (hipStream_t)stream, acc, rows, C, gamma,
                     beta, running_mean, running_var, momentum, eps, scale, shift, save_mean, save_invstd);
  return check_launch("bn_finalize");
}

extern "C" int avt_bn_apply(const void* x, const float* scale, const float* shift, const void* residual,
                            const float* rscale, const float* rshift, void* out, long long rows, int C, int relu,
                            void* stream) {
  AVT_REQUIRE(x && scale && shift && out, "bn_apply: null pointer");
  AVT_REQUIRE(C % 8 == 0, "bn_apply: C=%d must be a multiple of 8", C);
  AVT_REQUIRE((rscale == nullptr) == (rshift == nullptr), "bn_apply: rscale/rshift must be both set or both null");
  const long long nvec = rows * C / 8;
  if (nvec == 0) return AVT_OK;
  const int grid = ew_grid(nvec);
  if (256 % (C / 8) == 0)
    hipLaunchKernelGGL(bn_apply_kernel<true>, dim3(grid), dim3(256), 0, (hipStream_t)stream, (const bf16_t*)x, scale,
                       shift, (const bf16_t*)residual, rscale, rshift, (bf16_t*)out, nvec, C, relu);
  else
    hipLaunchKernelGGL(bn_apply_kernel<false>, dim3(grid), dim3(256), 0, (hipStream_t)stream, (const bf16_t*)x, scale,
                       shift, (const bf16_t*)residual, rscale, rshift, (bf16_t*)out, nvec, C, relu);
  return check_launch("bn_apply");
}

// workspace: AVT_BN_SLOTS*C*2 doubles (must be zero on entry; left zero on exit) + 2*C floats
extern "C" size_t avt_bn_bwd_workspace(long long rows, int C) {
  (void)rows;
  return (size_t)AVT_BN_SLOTS * C * 2 * sizeof(double) + 2 * (size_t)C * sizeof(float);
}

extern "C" int avt_bn_bwd(const void* g, const void* y, const void* xc, const float* mean, const float* invstd,
                          const float* gamma, float* dgamma, float* dbeta, void* gc, void* gmask_out,
                          void* workspace, long long rows, int C, void* stream) {
  AVT_REQUIRE(g && xc && mean && invstd && gamma && gc && workspace, "bn_bwd: null pointer");
  AVT_REQUIRE(C % 8 == 0 && C <= 2048 && 256 % (C / 8) == 0, "bn_bwd: C=%d unsupported", C);
  AVT_REQUIRE(rows > 0, "bn_bwd: empty input");
  AVT_REQUIRE(((uintptr_t)workspace & 7) == 0, "bn_bwd: workspace must be 8-byte aligned");
  double* acc = (double*)workspace;
  float* k1 = (float*)(acc + (size_t)AVT_BN_SLOTS * C * 2);
  float* k2 = k1 + C;
  hipStream_t st = (hipStream_t)stream;
  bn_bwd_reduce_launch((const bf16_t*)g, (const bf16_t*)y, nullptr, nullptr, (const bf16_t*)xc, mean, invstd, acc,
                       rows, C, st);
  hipLaunchKernelGGL(bn_bwd_finalize_kernel, dim3((C + 255) / 256), dim3(256), 0, st, acc, C, 1.0 / (double)rows,
                     dgamma, dbeta, k1, k2);
  const long long nvec = rows * C / 8;
  hipLaunchKernelGGL(bn_bwd_apply_kernel<true>, dim3(ew_grid(nvec)), dim3(256), 0, st, (const bf16_t*)g, (const bf16_t*)y,
                     nullptr, nullptr, (const bf16_t*)xc, mean, invstd, gamma, k1, k2, (bf16_t*)gc,
                     (bf16_t*)gmask_out, nvec, C);
  return check_launch("bn_bwd");
}

// BN + ReLU backward with the mask recomputed from the pre-activation xc and the forward's
// (scale, shift): y is never read.  Same workspace contract as avt_bn_bwd.
extern "C" int avt_bn_relu_bwd(const void* g, const void* xc, const float* scale, const float* shift,
                               const float* mean, const float* invstd, const float* gamma, float* dgamma, float* dbeta,
                               void* gc, void* workspace, long long rows, int C, void* stream) {
  AVT_REQUIRE(g && xc && scale && shift && mean && invstd && gamma && gc && workspace, "bn_relu_bwd: null pointer");
  AVT_REQUIRE(C % 8 == 0 && C <= 2048 && 256 % (C / 8) == 0, "bn_relu_bwd: C=%d unsupported", C);
  AVT_REQUIRE(rows > 0, "bn_relu_bwd: empty input");
  AVT_REQUIRE(((uintptr_t)workspace & 7) == 0, "bn_relu_bwd: workspace must be 8-byte aligned");
  double* acc = (double*)workspace;
  float* k1 = (float*)(acc + (size_t)AVT_BN_SLOTS * C * 2);
  float* k2 = k1 + C;
  hipStream_t st = (hipStream_t)stream;
  bn_bwd_reduce_launch((const bf16_t*)g, nullptr, scale, shift, (const bf16_t*)xc, mean, invstd, acc, rows, C, st);
  hipLaunchKernelGGL(bn_bwd_finalize_kernel, dim3((C + 255) / 256), dim3(256), 0, st, acc, C, 1.0 / (double)rows,
                     dgamma, dbeta, k1, k2);
  const long long nvec = rows * C / 8;
  hipLaunchKernelGGL(bn_bwd_apply_kernel<true>, dim3(ew_grid(nvec)), dim3(256), 0, st, (const bf16_t*)g, nullptr, scale,
                     shift, (const bf16_t*)xc, mean, invstd, gamma, k1, k2, (bf16_t*)gc, nullptr, nvec, C);
  return check_launch("bn_relu_bwd");
}

static int ilog2(int v) {
  int l = 0;
  while ((1 << l) < v) ++l;
  return l;
}

extern "C" int avt_stem_bn_relu_maxpool_fwd(const void* c, const float* scale, const float* shift, void* y, void* idx,
                                            void* carg, int N, int H, int W, int C, void* stream) {
  AVT_REQUIRE(c && scale && shift && y && idx && carg, "stem_bn_relu_maxpool_fwd: null pointer");
  AVT_REQUIRE(C % 8 == 0 && 256 % (C / 8) == 0, "stem_bn_relu_maxpool_fwd: C=%d unsupported", C);
  AVT_REQUIRE(N > 0 && H > 0 && W > 0, "stem_bn_relu_maxpool_fwd: empty input");
  const int P = (H + 2 - 3) / 2 + 1, Q = (W + 2 - 3) / 2 + 1;
  hipLaunchKernelGGL(stem_bn_relu_maxpool_fwd_kernel, dim3(N * P), dim3(256), 0, (hipStream_t)stream,
                     (const bf16_t*)c, scale, shift, (bf16_t*)y, (unsigned char*)idx, (bf16_t*)carg, H, W, C,
                     ilog2(C / 8), P, Q);
  return check_launch("stem_bn_relu_maxpool_fwd");
}

extern "C" int avt_stem_maxpool_bn_relu_bwd(const void* gy, const void* idx, const void* carg, const void* c,
                                            const float* scale, const float* shift, const float* mean,
                                            const float* invstd, const float* gamma, float* dgamma, float* dbeta,
                                            void* gc, void* workspace, int N, int H, int W, int C, void* stream) {
  AVT_REQUIRE(gy && idx && carg && c && scale && shift && mean && invstd && gamma && gc && workspace,
              "stem_maxpool_bn_relu_bwd: null pointer");
  AVT_REQUIRE(C % 8 == 0 && C <= 2048 && 256 % (C / 8) == 0, "stem_maxpool_bn_relu_bwd: C=%d unsupported", C);
  AVT_REQUIRE(N > 0 && H > 0 && W > 0, "stem_maxpool_bn_relu_bwd: empty input");
  AVT_REQUIRE(((uintptr_t)workspace & 7) == 0, "stem_maxpool_bn_relu_bwd: workspace must be 8-byte aligned");
  const int P = (H + 2 - 3) / 2 + 1, Q = (W + 2 - 3) / 2 + 1;
  double* acc = (double*)workspace;
  float* k1 = (float*)(acc + (size_t)AVT_BN_SLOTS * C * 2);
  float* k2 = k1 + C;
  hipStream_t st = (hipStream_t)stream;
  bn_bwd_reduce_launch((const bf16_t*)gy, nullptr, scale, shift, (const bf16_t*)carg, mean, invstd, acc,
                       (long long)N * P * Q, C, st);
  hipLaunchKernelGGL(bn_bwd_finalize_kernel, dim3((C + 255) / 256), dim3(256), 0, st, acc, C,
                     1.0 / ((double)N * H * W), dgamma, dbeta, k1, k2);
  hipLaunchKernelGGL(stem_maxpool_bn_bwd_apply_kernel, dim3(N * H), dim3(256), 0, st, (const bf16_t*)gy,
                     (const unsigned char*)idx, (const bf16_t*)c, scale, shift, mean, invstd, gamma, k1, k2,
                     (bf16_t*)gc, H, W, C, ilog2(C / 8), P, Q);
  return check_launch("stem_maxpool_bn_relu_bwd");
}
