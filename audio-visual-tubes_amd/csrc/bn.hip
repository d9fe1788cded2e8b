// Train-mode BatchNorm2d (+ReLU, +residual) for the ResNet-18 trunks, NHWC bf16 activations,
// fp32 math, fp64 statistic accumulation.  Semantics of torch BatchNorm2d as used at
// models/base_models.py:39,46-49,120-121,141 (eps 1e-5, momentum 0.1): normalise with the biased
// batch variance, update running_var with the unbiased one.
//
//   fwd : the conv epilogue stores per-row-tile (sum_t, M2_t, sum_t^2/n_t) into its own slot of an fp64
//         accumulator (avt_common.h: one slot per tile or persistent block, plain stores); bn_finalize
//         merges the slots in slot order (M2 = sum M2_t + sum sum_t^2/n_t - S^2/N, Chan's formula), writes
//         scale/shift/mean/invstd and updates the running stats; bn_apply (+residual, +ReLU).
//   bwd : bn_bwd_reduce stores per-block (sum g', sum g'*xhat) (g' = g*[y>0]) into slot blockIdx of an fp64
//         accumulator -> bn_bwd_finalize (dgamma, dbeta, k1, k2) -> bn_bwd_apply:
//         g_c = gamma*invstd*(g' - k1 - xhat*k2).
//   Deterministic: no atomics; the same inputs give the same bits on every run.
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

// The slot sums of kFinCB consecutive channels [c0, c0 + kFinCB), W statistics each, in a fixed order.  A
// slot's run of E = kFinCB * W doubles is contiguous; a wave-load covers SPI = 64 / E slots (lane = (slot
// offset so, element e)), so wave w, lane (so, e) adds slots (i kFinWaves + w) SPI + so for i = 0, 1, ... in
// turn, 8 loads in flight per batch (one round trip for up to 8 * kFinWaves * SPI slots: 1024 fwd / bwd);
// the lanes' partials meet in LDS in (wave, slot offset) order.  tot[e] on return (after a barrier).
// Launch: kFinThreads threads per kFinCB channels -- many small blocks, since a finalize is latency-bound.
constexpr int kFinWaves = 16, kFinThreads = kFinWaves * 64, kFinCB = 4;
template <int W>
__device__ __forceinline__ void slot_sums(const double* __restrict__ acc, const double* __restrict__ slots, int C,
                                          int c0, long long rows, double* red, double* tot) {
  constexpr int E = kFinCB * W, SPI = 64 / E, STEP = kFinWaves * SPI;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int so = lane / E, e = lane - so * E;
  // the header's slot count, bounded by the workspace's capacity: a producer that skipped its header (or a
  // workspace handed over uninitialised) gives NaN statistics, never reads beyond the slots
  const double hn = acc[0] + acc[1];
  const bool bad = !(hn >= 0.0 && hn <= (double)bn_slot_cap(rows));
  const int n = bad ? 0 : (int)hn;
  double s = 0.0;
  if (so < SPI && c0 + e / W < C) {
    const double* base = slots + (size_t)c0 * W + e;
    const unsigned stride = (unsigned)(C * W);
    for (int k0 = w * SPI + so; k0 < n; k0 += 8 * STEP) {
      double v[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int k = k0 + i * STEP;
        v[i] = k < n ? base[(size_t)k * stride] : 0.0;
      }
#pragma unroll
      for (int i = 0; i < 8; ++i) s += v[i];
    }
  }
  red[threadIdx.x] = s;
  __syncthreads();
  if (threadIdx.x < E) {
    double t = 0.0;
    for (int ww = 0; ww < kFinWaves; ++ww)
#pragma unroll
      for (int o = 0; o < SPI; ++o) t += red[ww * 64 + o * E + threadIdx.x];
    tot[threadIdx.x] = bad ? __builtin_nan("") : t;
  }
  __syncthreads();
}

__global__ __launch_bounds__(kFinThreads) void bn_finalize_kernel(double* __restrict__ acc, long long rows, int C,
                                                                  const float* __restrict__ gamma,
                                                                  const float* __restrict__ beta, float* running_mean,
                                                                  float* running_var, float momentum, float eps,
                                                                  float* scale, float* shift, float* save_mean,
                                                                  float* save_invstd, long long rep) {
  __shared__ double red[kFinThreads], tot[kFinCB * 3];
  const int c0 = blockIdx.x * kFinCB;
  slot_sums<3>(acc, bn_fwd_slots(acc), C, c0, rows, red, tot);
  const int c = c0 + (int)threadIdx.x;
  if (threadIdx.x >= kFinCB || c >= C) return;
  const double S = tot[threadIdx.x * 3], Q = tot[threadIdx.x * 3 + 1], R = tot[threadIdx.x * 3 + 2];
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
    // unbiased variance of the logical batch, in which each accumulated row occurs `rep` times
    const double nl = n * (double)rep;
    const float unb = nl > 1.0 ? (float)(m2 * (double)rep / (nl - 1.0)) : var;
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

// Bit e of the result: bf16 element e of v is > 0 (positive and non-zero as int16) -- the ReLU
// backward's `result > 0` evaluated on the stored output.
__device__ __forceinline__ unsigned pos_bits8(const u32x4& v) {
  const unsigned* u = reinterpret_cast<const unsigned*>(&v);
  unsigned b = 0;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    b |= ((short)(u[e] & 0xffff) > 0 ? 1u : 0u) << (2 * e);
    b |= ((short)(u[e] >> 16) > 0 ? 1u : 0u) << (2 * e + 1);
  }
  return b;
}

// mk (optional, with relu): the ReLU mask of out as bits, one byte per 8 channels ([rows][C/8] u8):
// the backward reads 1/16 of the bytes of out for it.
template <bool POW2>
__global__ __launch_bounds__(256) void bn_apply_kernel(const bf16_t* __restrict__ x, const float* __restrict__ scale,
                                                       const float* __restrict__ shift,
                                                       const bf16_t* __restrict__ res, const float* __restrict__ rscale,
                                                       const float* __restrict__ rshift, bf16_t* __restrict__ out,
                                                       unsigned char* __restrict__ mk, long long nvec, int C, int relu) {
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
    const u32x4 o = pack8(f);
    reinterpret_cast<u32x4*>(out)[i] = o;
    if (mk) mk[i] = (unsigned char)pos_bits8(o);
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
  // four rows per iteration: 8-12 independent 16-B loads in flight per thread (HBM-bound: the
  // bytes in flight per CU set the achieved bandwidth); the remaining rows one at a time
  long long r = rbeg + r0;
  constexpr int U = 4;
  for (; r + (U - 1) * rstep < rend; r += U * rstep) {
    u32x4 gq[U], xq[U], yq[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const size_t o = (size_t)(r + u * rstep) * cv + chunk;
      gq[u] = reinterpret_cast<const u32x4*>(g)[o];
      xq[u] = reinterpret_cast<const u32x4*>(xc)[o];
      if (y) yq[u] = reinterpret_cast<const u32x4*>(y)[o];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      float gg[8], xx[8];
      unpack8(gq[u], gg);
      unpack8(xq[u], xx);
      if (y) {
        float yy[8];
        unpack8(yq[u], yy);
#pragma unroll
        for (int e = 0; e < 8; ++e) gg[e] = yy[e] > 0.f ? gg[e] : 0.f;
      } else if (mscale) {
#pragma unroll
        for (int e = 0; e < 8; ++e) gg[e] = __builtin_fmaf(xx[e], mscale[c0 + e], mshift[c0 + e]) > 0.f ? gg[e] : 0.f;
      }
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        s1[e] += gg[e];
        s2[e] += gg[e] * (xx[e] - mu[e]) * is[e];
      }
    }
  }
  for (; r < rend; r += rstep) {
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
  bn_write_header(acc, gridDim.x, 0);
  double* slot = bn_bwd_slots(acc, C) + (size_t)blockIdx.x * C * 2;  // this block's own slot
  for (int c = threadIdx.x; c < C; c += blockDim.x) {
    float a = 0.f, b = 0.f;
    for (int k = 0; k < rstep; ++k) {
      a += red[(k * C + c) * 2];
      b += red[(k * C + c) * 2 + 1];
    }
    slot[2 * c] = (double)a;
    slot[2 * c + 1] = (double)b;
  }
}

// dgamma/dbeta (accumulated into the gradient if non-null) and k1,k2 of channels [c0, c0 + kFinCB) from the
// slots of workspace acc (slot_sums; every thread of the block calls it)
__device__ __forceinline__ void bn_bwd_finalize_cb(double* __restrict__ acc, int C, int c0, double inv_rows,
                                                   float* dgamma, float* dbeta, float* k1, float* k2) {
  __shared__ double red[kFinThreads], tot[kFinCB * 2];
  slot_sums<2>(acc, bn_bwd_slots(acc, C), C, c0, __double2ll_rn(1.0 / inv_rows), red, tot);
  const int c = c0 + (int)threadIdx.x;
  if (threadIdx.x >= kFinCB || c >= C) return;
  const double a = tot[threadIdx.x * 2], b = tot[threadIdx.x * 2 + 1];
  if (dbeta) dbeta[c] += (float)a;
  if (dgamma) dgamma[c] += (float)b;
  k1[c] = (float)(a * inv_rows);
  k2[c] = (float)(b * inv_rows);
}

// launch: kFinThreads threads per kFinCB channels
__global__ __launch_bounds__(kFinThreads) void bn_bwd_finalize_kernel(double* __restrict__ acc, int C, double inv_rows,
                                                                      float* dgamma, float* dbeta, float* k1, float* k2) {
  bn_bwd_finalize_cb(acc, C, blockIdx.x * kFinCB, inv_rows, dgamma, dbeta, k1, k2);
}

// both BNs of a first block in one launch: blocks [0, G) the first BN's channel groups, [G, 2G) the second's
__global__ __launch_bounds__(kFinThreads) void bn_bwd_finalize2_kernel(double* __restrict__ acc, double* __restrict__ acc2,
                                                                       int C, double inv_rows, float* dgamma,
                                                                       float* dbeta, float* k1, float* k2,
                                                                       float* dgamma2, float* dbeta2, float* k1b,
                                                                       float* k2b) {
  const int G = (C + kFinCB - 1) / kFinCB;
  if ((int)blockIdx.x < G)
    bn_bwd_finalize_cb(acc, C, blockIdx.x * kFinCB, inv_rows, dgamma, dbeta, k1, k2);
  else
    bn_bwd_finalize_cb(acc2, C, (blockIdx.x - G) * kFinCB, inv_rows, dgamma2, dbeta2, k1b, k2b);
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

// ---------------------------------------------------------------------------------------------
// Block-output BN backward from the ReLU mask bits (avt_bn_apply_mask): g' = g * bit, and -- for a
// first block -- bn2 and downsample.1 in one pass over (g, mask, xc, xc2): they share g' (the ReLU
// sits after their sum, base_models.py:64-67), so g and the mask are read once for both.
struct MaskBwdArgs {
  const bf16_t* g;
  const unsigned char* mk;  // [rows][C/8] mask bits
  const bf16_t* xc;
  const float* mean;
  const float* invstd;
  double* acc;              // [SLOTS][C][2]: (sum g', sum g' * xhat)
  const bf16_t* xc2;        // TWO: the second BN's pre-activation / statistics / accumulator
  const float* mean2;
  const float* invstd2;
  double* acc2;
  long long rows;
  int C, rows_per_block;
};

__device__ __forceinline__ void mask8(float* gg, unsigned bits) {
#pragma unroll
  for (int e = 0; e < 8; ++e) gg[e] = (bits >> e) & 1u ? gg[e] : 0.f;
}

template <bool TWO>
__global__ __launch_bounds__(256) void bn_bwd_mask_reduce_kernel(MaskBwdArgs a) {
  constexpr int NS = TWO ? 3 : 2;
  __shared__ float red[2048 * NS];  // [256/(C/8)][C][NS]
  const int C = a.C, cv = C / 8;
  const int chunk = threadIdx.x % cv, r0 = threadIdx.x / cv, rstep = 256 / cv;
  const int c0 = chunk * 8;
  float mu[8], is[8], mu2[8], is2[8], s1[8], s2[8], s3[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    mu[e] = a.mean[c0 + e];
    is[e] = a.invstd[c0 + e];
    if (TWO) {
      mu2[e] = a.mean2[c0 + e];
      is2[e] = a.invstd2[c0 + e];
    }
    s1[e] = s2[e] = s3[e] = 0.f;
  }
  const long long rbeg = (long long)blockIdx.x * a.rows_per_block;
  const long long rend = min(a.rows, rbeg + a.rows_per_block);
  auto body = [&](const u32x4& gq, unsigned bits, const u32x4& xq, const u32x4& x2q) {
    float gg[8], xx[8];
    unpack8(gq, gg);
    unpack8(xq, xx);
    mask8(gg, bits);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      s1[e] += gg[e];
      s2[e] += gg[e] * (xx[e] - mu[e]) * is[e];
    }
    if (TWO) {
      float x2[8];
      unpack8(x2q, x2);
#pragma unroll
      for (int e = 0; e < 8; ++e) s3[e] += gg[e] * (x2[e] - mu2[e]) * is2[e];
    }
  };
  long long r = rbeg + r0;
  constexpr int U = 4;  // rows in flight per thread (HBM-bound: bytes in flight per CU)
  for (; r + (U - 1) * rstep < rend; r += U * rstep) {
    u32x4 gq[U], xq[U], x2q[U];
    unsigned bq[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const size_t o = (size_t)(r + u * rstep) * cv + chunk;
      gq[u] = reinterpret_cast<const u32x4*>(a.g)[o];
      xq[u] = reinterpret_cast<const u32x4*>(a.xc)[o];
      if (TWO) x2q[u] = reinterpret_cast<const u32x4*>(a.xc2)[o];
      bq[u] = a.mk[o];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) body(gq[u], bq[u], xq[u], TWO ? x2q[u] : xq[u]);
  }
  for (; r < a.rows && r < rend; r += rstep) {
    const size_t o = (size_t)r * cv + chunk;
    const u32x4 gq = reinterpret_cast<const u32x4*>(a.g)[o];
    const u32x4 xq = reinterpret_cast<const u32x4*>(a.xc)[o];
    body(gq, a.mk[o], xq, TWO ? reinterpret_cast<const u32x4*>(a.xc2)[o] : xq);
  }
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    red[(r0 * C + c0 + e) * NS] = s1[e];
    red[(r0 * C + c0 + e) * NS + 1] = s2[e];
    if (TWO) red[(r0 * C + c0 + e) * NS + 2] = s3[e];
  }
  __syncthreads();
  bn_write_header(a.acc, gridDim.x, 0);
  if (TWO) bn_write_header(a.acc2, gridDim.x, 0);
  const size_t slot = (size_t)blockIdx.x * C * 2;  // this block's own slot
  double* s1p = bn_bwd_slots(a.acc, C) + slot;
  double* s2p = TWO ? bn_bwd_slots(a.acc2, C) + slot : nullptr;
  for (int c = threadIdx.x; c < C; c += blockDim.x) {
    float x = 0.f, y = 0.f, z = 0.f;
    for (int k = 0; k < rstep; ++k) {
      x += red[(k * C + c) * NS];
      y += red[(k * C + c) * NS + 1];
      if (TWO) z += red[(k * C + c) * NS + 2];
    }
    s1p[2 * c] = (double)x;
    s1p[2 * c + 1] = (double)y;
    if (TWO) {
      s2p[2 * c] = (double)x;
      s2p[2 * c + 1] = (double)z;
    }
  }
}

// gc = gamma*invstd*(g' - k1 - xhat*k2) (and gc2 for the second BN) from the finalized k1/k2
struct MaskApplyArgs {
  const bf16_t* g;
  const unsigned char* mk;
  const bf16_t* xc;
  const float *mean, *invstd, *gamma, *k1, *k2;
  bf16_t* gc;
  const bf16_t* xc2;
  const float *mean2, *invstd2, *gamma2, *k1b, *k2b;
  bf16_t* gc2;
  long long nvec;
  int C;
};

template <bool TWO>
__global__ __launch_bounds__(256) void bn_bwd_mask_apply_kernel(MaskApplyArgs a) {
  const int cv = a.C / 8;  // a power of two dividing 256 (checked by the host)
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < a.nvec;
       i += (long long)gridDim.x * blockDim.x) {
    const int c0 = (int)((unsigned)i & (unsigned)(cv - 1)) * 8;
    float gg[8], xx[8], o[8];
    unpack8(reinterpret_cast<const u32x4*>(a.g)[i], gg);
    unpack8(reinterpret_cast<const u32x4*>(a.xc)[i], xx);
    const unsigned bits = a.mk[i];
    u32x4 x2q;
    if (TWO) x2q = reinterpret_cast<const u32x4*>(a.xc2)[i];
    mask8(gg, bits);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int c = c0 + e;
      const float xh = (xx[e] - a.mean[c]) * a.invstd[c];
      o[e] = a.gamma[c] * a.invstd[c] * (gg[e] - a.k1[c] - xh * a.k2[c]);
    }
    reinterpret_cast<u32x4*>(a.gc)[i] = pack8(o);
    if (TWO) {
      unpack8(x2q, xx);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int c = c0 + e;
        const float xh = (xx[e] - a.mean2[c]) * a.invstd2[c];
        o[e] = a.gamma2[c] * a.invstd2[c] * (gg[e] - a.k1b[c] - xh * a.k2b[c]);
      }
      reinterpret_cast<u32x4*>(a.gc2)[i] = pack8(o);
    }
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
  const bf16_t* cimg = c + (size_t)n * H * W * C;
  // window rows 2p-1+r, r = 0..2 (validity is block-uniform); loads use clamped coordinates and
  // out-of-image taps are masked, so all nine 16-B loads of a thread issue together
  bool rok[3];
  int hh[3];
#pragma unroll
  for (int r = 0; r < 3; ++r) {
    const int h = p * 2 - 1 + r;
    rok[r] = h >= 0 && h < H;
    hh[r] = min(max(h, 0), H - 1);
  }
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
    u32x4 v[9];
    bool ok[9];
#pragma unroll
    for (int r = 0; r < 3; ++r)
#pragma unroll
      for (int s2 = 0; s2 < 3; ++s2) {
        const int w = q * 2 - 1 + s2;
        ok[r * 3 + s2] = rok[r] && w >= 0 && w < W;
        const int wc = min(max(w, 0), W - 1);
        v[r * 3 + s2] = *reinterpret_cast<const u32x4*>(cimg + ((size_t)hh[r] * W + wc) * C + c8 * 8);
      }
#pragma unroll
    for (int k = 0; k < 9; ++k) {
      if (!ok[k]) continue;
      float xv[8];
      unpack8(v[k], xv);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float f = bf2f(f2bf(fmaxf(__builtin_fmaf(xv[e], sc[e], sh[e]), 0.f)));
        if (f > best[e] || f != f) {
          best[e] = f;
          bc[e] = xv[e];
          bi[e] = k;
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

// LDS capacity for the two pooled rows a bwd block reads: 2 x Q x C x (2 B grad + 1 B argmax)
constexpr int kStemLdsBytes = 48 * 1024;

// One block per PAIR of input rows (2p, 2p+1) of image n: the windows covering them are pooled rows p
// (row 2p: window row kh = 1; row 2p+1: kh = 2) and p+1 (row 2p+1: kh = 0), so the block stages those two
// pooled rows of gy and argmax into LDS once for both input rows (a row per block staged ~1.5 pooled rows
// per input row) and has twice the items in flight.  For input pixel (h, w) the candidate windows are
// (p_h, q) with q = w/2 (kw = 1 if w even, 2 if odd) and, for odd w, q+1 (kw = 0); g' = [h0 > 0] * the
// sum of gy over the candidates whose argmax is (h, w); gc = gamma*invstd*(g' - k1 - xhat*k2).
constexpr int kStemBwdThreads = 512;
__global__ __launch_bounds__(kStemBwdThreads) void stem_maxpool_bn_bwd_apply_kernel(
    const bf16_t* __restrict__ gy, const unsigned char* __restrict__ idx, const bf16_t* __restrict__ c,
    const float* __restrict__ scale, const float* __restrict__ shift, const float* __restrict__ mean,
    const float* __restrict__ invstd, const float* __restrict__ gamma, const float* __restrict__ k1,
    const float* __restrict__ k2, bf16_t* __restrict__ gc, int H, int W, int C, int cvs, int P, int Q) {
  extern __shared__ __attribute__((aligned(16))) char lds[];  // 6*Q*C bytes (dynamic)
  const int hp = (H + 1) >> 1;
  const int n = blockIdx.x / hp, p = blockIdx.x - n * hp;
  const int cv = 1 << cvs;
  const bool two_rows = 2 * p + 1 < H;
  const bool p_next = p + 1 < P;
  const int rowg = Q * C * 2, rowi = Q * C;  // bytes of one pooled row of gy / argmax
  bf16_t* lg = reinterpret_cast<bf16_t*>(lds);
  unsigned char* li = reinterpret_cast<unsigned char*>(lds + 2 * rowg);
  const int items_row = W * cv, items = (two_rows ? 2 : 1) * items_row;
  // the pre-activations of this thread's items first: independent of the staged rows, their HBM latency
  // overlaps the staging and its barrier
  constexpr int kItems = 6;
  u32x4 cx[kItems];
  const size_t img_row0 = (size_t)n * H + 2 * p;  // input row 2p of image n
  // item t -> (input row 2p + r, pixel w, the thread's channel chunk): per row the even pixels first, then the
  // odd ones, so that a wave's items share their candidate-window pattern (even h / w: one window row / column,
  // odd: two) and the absent candidates are skipped by wave-uniform branches
  const int cw = threadIdx.x & (cv - 1), we_items = ((W + 1) >> 1) * cv;
  auto item_pix = [&](int t, int& r, int& w) {
    r = t >= items_row ? 1 : 0;
    const int tw = t - r * items_row;
    w = tw < we_items ? 2 * (tw >> cvs) : 2 * ((tw - we_items) >> cvs) + 1;
  };
#pragma unroll
  for (int j = 0; j < kItems; ++j) {
    const int t = threadIdx.x + kStemBwdThreads * j;
    if (t < items) {
      int r, w;
      item_pix(t, r, w);
      cx[j] = *reinterpret_cast<const u32x4*>(c + ((img_row0 + r) * W + w) * C + cw * 8);
    }
  }
  // the thread's 8 channels are the same for all its items (kStemBwdThreads is a multiple of C / 8): their
  // per-channel constants are loaded once, not per item (7 x 8 scalar loads per item were the kernel's
  // vector-memory instruction stream)
  const int c8 = cw;
  float k_sc[8], k_sh[8], k_mu[8], k_is[8], k_k1[8], k_k2[8], k_gi[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const int ch = c8 * 8 + e;
    k_sc[e] = scale[ch];
    k_sh[e] = shift[ch];
    k_mu[e] = mean[ch];
    k_is[e] = invstd[ch];
    k_k1[e] = k1[ch];
    k_k2[e] = k2[ch];
    k_gi[e] = gamma[ch] * k_is[e];
  }
  // stage the (<= 2) pooled rows of gy and argmax: every load issued before any LDS store
  const int ng = rowg / 16, ni = rowi / 16, nrows = p_next ? 2 : 1, nst = nrows * (ng + ni);
  constexpr int kStage = 4;
  u32x4 sv[kStage];
  const u32x4* sg = reinterpret_cast<const u32x4*>(gy + ((size_t)n * P + p) * Q * C);
  const u32x4* si = reinterpret_cast<const u32x4*>(idx + ((size_t)n * P + p) * Q * C);
  // rounds of kStage loads per thread (one round up to W = 168 at C = 64; wider rows take more, up to the LDS bound)
  for (int t0 = 0; t0 < nst; t0 += kStage * kStemBwdThreads) {
#pragma unroll
    for (int j = 0; j < kStage; ++j) {
      const int t = t0 + threadIdx.x + kStemBwdThreads * j;
      if (t < nst) sv[j] = t < nrows * ng ? sg[t] : si[t - nrows * ng];  // consecutive pooled rows are contiguous
    }
#pragma unroll
    for (int j = 0; j < kStage; ++j) {
      const int t = t0 + threadIdx.x + kStemBwdThreads * j;
      if (t < nst) {
        char* dst = t < nrows * ng ? lds + (size_t)t * 16 : lds + 2 * rowg + (size_t)(t - nrows * ng) * 16;
        *reinterpret_cast<u32x4*>(dst) = sv[j];
      }
    }
  }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < kItems; ++j) {
    const int t = threadIdx.x + kStemBwdThreads * j;
    if (t >= items) break;
    int r, w;
    item_pix(t, r, w);
    // window row of (2p + r) in pooled row p: kh0 = 1 + r; in pooled row p + 1 (odd rows only): kh0 - 2;
    // column: q0 = w / 2 at kw0 (1 for even w, 2 for odd) and, odd w only, q0 + 1 at kw0 - 2
    const int kh0 = 1 + r, q0 = w >> 1, kw0 = (w & 1) + 1;
    const bool p_two = r == 1 && p_next, q_two = (w & 1) && q0 + 1 < Q;
    float gg[8], xx[8], o[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) gg[e] = 0.f;
    // g' += gy of a candidate window whose argmax is (h, w), in the order (p, q0), (p, q0+1), (p+1, q0), (p+1, q0+1)
    auto cand = [&](int lrow, int q, int pos) {
      const int el = lrow * Q * C + q * C + c8 * 8;
      const unsigned long long iv = *reinterpret_cast<const unsigned long long*>(li + el);
      float f[8];
      unpack8(*reinterpret_cast<const u32x4*>(lg + el), f);
#pragma unroll
      for (int e = 0; e < 8; ++e) gg[e] += ((int)((iv >> (8 * e)) & 0xff) == pos) ? f[e] : 0.f;
    };
    cand(0, q0, kh0 * 3 + kw0);
    if (q_two) cand(0, q0 + 1, kh0 * 3 + kw0 - 2);
    if (p_two) {
      cand(1, q0, (kh0 - 2) * 3 + kw0);
      if (q_two) cand(1, q0 + 1, (kh0 - 2) * 3 + kw0 - 2);
    }
    const size_t xo = ((img_row0 + r) * W + w) * C + c8 * 8;
    unpack8(cx[j], xx);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      gg[e] = __builtin_fmaf(xx[e], k_sc[e], k_sh[e]) > 0.f ? gg[e] : 0.f;
      const float xh = (xx[e] - k_mu[e]) * k_is[e];
      o[e] = k_gi[e] * (gg[e] - k_k1[e] - xh * k_k2[e]);
    }
    *reinterpret_cast<u32x4*>(gc + xo) = pack8(o);
  }
}

static void bn_bwd_reduce_launch(const bf16_t* g, const bf16_t* y, const float* mscale, const float* mshift,
                                 const bf16_t* xc, const float* mean, const float* invstd, double* acc, long long rows,
                                 int C, hipStream_t st) {
  // ~2 blocks per CU of rows (more blocks measured slower: their fp64 atomics contend)
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

extern "C" size_t avt_bn_acc_doubles(long long rows, int C) {
  return rows < 0 || C <= 0 ? 0 : (size_t)kBnHdr + (size_t)bn_slot_cap(rows) * C * 3;
}

extern "C" int avt_bn_finalize(double* acc, long long rows, int C, const float* gamma, const float* beta,
                               float* running_mean, float* running_var, float momentum, float eps, float* scale,
                               float* shift, float* save_mean, float* save_invstd, void* stream) {
  AVT_REQUIRE(acc && gamma && beta && scale && shift, "bn_finalize: null pointer");
  AVT_REQUIRE(rows > 0 && C > 0, "bn_finalize: empty input");
  hipStream_t st = (hipStream_t)stream;
  if (diag_skip(1, st)) return AVT_OK;
  for (int rep = diag_skip(32, st) ? 2 : 1; rep > 0; --rep)  // (AVT_DIAG bit 32: each launched twice, timing only)
    hipLaunchKernelGGL(bn_finalize_kernel, dim3((C + kFinCB - 1) / kFinCB), dim3(kFinThreads), 0, st, acc, rows, C,
                       gamma, beta, running_mean, running_var, momentum, eps, scale, shift, save_mean, save_invstd, 1LL);
  return check_launch("bn_finalize");
}

// As avt_bn_finalize for a logical batch in which every accumulated row occurs `rep` times (the
// tube step's t-fold repeated spectrogram, train_3D.py:128-130, run once per distinct clip):
// mean and biased variance are those of the distinct rows; the running variance gets the
// unbiased factor of the rows*rep logical rows, exactly as BatchNorm2d over the repeated batch.
extern "C" int avt_bn_finalize_rep(double* acc, long long rows, long long rep, int C, const float* gamma,
                                   const float* beta, float* running_mean, float* running_var, float momentum,
                                   float eps, float* scale, float* shift, float* save_mean, float* save_invstd,
                                   void* stream) {
  AVT_REQUIRE(acc && gamma && beta && scale && shift, "bn_finalize_rep: null pointer");
  AVT_REQUIRE(rows > 0 && C > 0 && rep >= 1, "bn_finalize_rep: empty input");
  if (!diag_skip(1, (hipStream_t)stream)) hipLaunchKernelGGL(bn_finalize_kernel, dim3((C + kFinCB - 1) / kFinCB), dim3(kFinThreads), 0, (hipStream_t)stream, acc, rows, C, gamma,
                     beta, running_mean, running_var, momentum, eps, scale, shift, save_mean, save_invstd, rep);
  return check_launch("bn_finalize_rep");
}

extern "C" int avt_bn_apply(const void* x, const float* scale, const float* shift, const void* residual,
                            const float* rscale, const float* rshift, void* out, long long rows, int C, int relu,
                            void* stream) {
  AVT_REQUIRE(x && scale && shift && out, "bn_apply: null pointer");
  AVT_REQUIRE(C % 8 == 0, "bn_apply: C=%d must be a multiple of 8", C);
  AVT_REQUIRE((rscale == nullptr) == (rshift == nullptr), "bn_apply: rscale/rshift must be both set or both null");
  const long long nvec = rows * C / 8;
  if (nvec == 0 || diag_skip(16, (hipStream_t)stream)) return AVT_OK;
  const int grid = ew_grid(nvec);
  if (256 % (C / 8) == 0)
    hipLaunchKernelGGL(bn_apply_kernel<true>, dim3(grid), dim3(256), 0, (hipStream_t)stream, (const bf16_t*)x, scale,
                       shift, (const bf16_t*)residual, rscale, rshift, (bf16_t*)out, nullptr, nvec, C, relu);
  else
    hipLaunchKernelGGL(bn_apply_kernel<false>, dim3(grid), dim3(256), 0, (hipStream_t)stream, (const bf16_t*)x, scale,
                       shift, (const bf16_t*)residual, rscale, rshift, (bf16_t*)out, nullptr, nvec, C, relu);
  return check_launch("bn_apply");
}

extern "C" int avt_bn_apply_mask(const void* x, const float* scale, const float* shift, const void* residual,
                                 const float* rscale, const float* rshift, void* out, void* mask, long long rows,
                                 int C, void* stream) {
  AVT_REQUIRE(x && scale && shift && out && mask, "bn_apply_mask: null pointer");
  AVT_REQUIRE(C % 8 == 0 && 256 % (C / 8) == 0, "bn_apply_mask: C=%d unsupported", C);
  AVT_REQUIRE((rscale == nullptr) == (rshift == nullptr), "bn_apply_mask: rscale/rshift must be both set or both null");
  const long long nvec = rows * C / 8;
  if (nvec == 0 || diag_skip(16, (hipStream_t)stream)) return AVT_OK;
  hipLaunchKernelGGL(bn_apply_kernel<true>, dim3(ew_grid(nvec)), dim3(256), 0, (hipStream_t)stream, (const bf16_t*)x,
                     scale, shift, (const bf16_t*)residual, rscale, rshift, (bf16_t*)out, (unsigned char*)mask, nvec, C,
                     1);
  return check_launch("bn_apply_mask");
}

extern "C" int avt_bn_bwd_mask(const void* g, const void* mask, const avt_bn_bwd_target* t1,
                               const avt_bn_bwd_target* t2, long long rows, int C, void* stream) {
  AVT_REQUIRE(g && mask && t1, "bn_bwd_mask: null pointer");
  AVT_REQUIRE(C % 8 == 0 && C <= 2048 && 256 % (C / 8) == 0, "bn_bwd_mask: C=%d unsupported", C);
  AVT_REQUIRE(rows > 0, "bn_bwd_mask: empty input");
  const avt_bn_bwd_target* ts[2] = {t1, t2};
  for (int k = 0; k < (t2 ? 2 : 1); ++k) {
    const avt_bn_bwd_target* t = ts[k];
    AVT_REQUIRE(t->xc && t->mean && t->invstd && t->gamma && t->gc && t->workspace, "bn_bwd_mask: null target pointer");
    AVT_REQUIRE(((uintptr_t)t->workspace & 7) == 0, "bn_bwd_mask: workspace must be 8-byte aligned");
  }
  hipStream_t st = (hipStream_t)stream;
  double* acc = (double*)t1->workspace;
  float* k1 = (float*)(acc + kBnHdr);
  double* acc2 = t2 ? (double*)t2->workspace : nullptr;
  float* k1b = t2 ? (float*)(acc2 + kBnHdr) : nullptr;
  MaskBwdArgs a{};
  a.g = (const bf16_t*)g;
  a.mk = (const unsigned char*)mask;
  a.xc = (const bf16_t*)t1->xc;
  a.mean = t1->mean;
  a.invstd = t1->invstd;
  a.acc = acc;
  if (t2) {
    a.xc2 = (const bf16_t*)t2->xc;
    a.mean2 = t2->mean;
    a.invstd2 = t2->invstd;
    a.acc2 = acc2;
  }
  a.rows = rows;
  a.C = C;
  long long rpb = (rows + 511) / 512;  // ~2 blocks per CU of rows, as bn_bwd_reduce_launch
  const int rstep = 256 / (C / 8);
  rpb = ((rpb + rstep - 1) / rstep) * rstep;
  if (rpb < rstep) rpb = rstep;
  a.rows_per_block = (int)rpb;
  const int nblk = (int)((rows + rpb - 1) / rpb);
  const double inv_rows = 1.0 / (double)rows;
  MaskApplyArgs p{};
  p.g = a.g;
  p.mk = a.mk;
  p.xc = a.xc;
  p.mean = t1->mean;
  p.invstd = t1->invstd;
  p.gamma = t1->gamma;
  p.k1 = k1;
  p.k2 = k1 + C;
  p.gc = (bf16_t*)t1->gc;
  p.nvec = rows * C / 8;
  p.C = C;
  if (t2) {
    if (!diag_skip(8, st)) hipLaunchKernelGGL(bn_bwd_mask_reduce_kernel<true>, dim3(nblk), dim3(256), 0, st, a);
    if (diag_skip(64, st)) hipLaunchKernelGGL(bn_bwd_finalize2_kernel, dim3(2 * ((C + kFinCB - 1) / kFinCB)), dim3(kFinThreads), 0, st, acc, acc2, C, inv_rows,
                       t1->dgamma, t1->dbeta, k1, k1 + C, t2->dgamma, t2->dbeta, k1b, k1b + C);
    if (!diag_skip(2, st)) hipLaunchKernelGGL(bn_bwd_finalize2_kernel, dim3(2 * ((C + kFinCB - 1) / kFinCB)), dim3(kFinThreads), 0, st, acc, acc2, C, inv_rows,
                       t1->dgamma, t1->dbeta, k1, k1 + C, t2->dgamma, t2->dbeta, k1b, k1b + C);
    p.xc2 = (const bf16_t*)t2->xc;
    p.mean2 = t2->mean;
    p.invstd2 = t2->invstd;
    p.gamma2 = t2->gamma;
    p.k1b = k1b;
    p.k2b = k1b + C;
    p.gc2 = (bf16_t*)t2->gc;
    hipLaunchKernelGGL(bn_bwd_mask_apply_kernel<true>, dim3(ew_grid(p.nvec)), dim3(256), 0, st, p);
  } else {
    if (!diag_skip(8, st)) hipLaunchKernelGGL(bn_bwd_mask_reduce_kernel<false>, dim3(nblk), dim3(256), 0, st, a);
    if (diag_skip(64, st)) hipLaunchKernelGGL(bn_bwd_finalize_kernel, dim3((C + kFinCB - 1) / kFinCB), dim3(kFinThreads), 0, st, acc, C, inv_rows, t1->dgamma,
                       t1->dbeta, k1, k1 + C);
    if (!diag_skip(2, st)) hipLaunchKernelGGL(bn_bwd_finalize_kernel, dim3((C + kFinCB - 1) / kFinCB), dim3(kFinThreads), 0, st, acc, C, inv_rows, t1->dgamma,
                       t1->dbeta, k1, k1 + C);
    hipLaunchKernelGGL(bn_bwd_mask_apply_kernel<false>, dim3(ew_grid(p.nvec)), dim3(256), 0, st, p);
  }
  return check_launch("bn_bwd_mask");
}

// workspace: header + k1/k2 (2C floats) + the slots of up to `rows` rows (avt_common.h); any contents on entry
extern "C" size_t avt_bn_bwd_workspace(long long rows, int C) {
  if (rows < 0 || C <= 0) return 0;
  return ((size_t)kBnHdr + (size_t)C + (size_t)bn_slot_cap(rows) * C * 2) * sizeof(double);
}

extern "C" int avt_bn_bwd(const void* g, const void* y, const void* xc, const float* mean, const float* invstd,
                          const float* gamma, float* dgamma, float* dbeta, void* gc, void* gmask_out,
                          void* workspace, long long rows, int C, void* stream) {
  AVT_REQUIRE(g && xc && mean && invstd && gamma && gc && workspace, "bn_bwd: null pointer");
  AVT_REQUIRE(C % 8 == 0 && C <= 2048 && 256 % (C / 8) == 0, "bn_bwd: C=%d unsupported", C);
  AVT_REQUIRE(rows > 0, "bn_bwd: empty input");
  AVT_REQUIRE(((uintptr_t)workspace & 7) == 0, "bn_bwd: workspace must be 8-byte aligned");
  double* acc = (double*)workspace;
  float* k1 = (float*)(acc + kBnHdr);
  float* k2 = k1 + C;
  hipStream_t st = (hipStream_t)stream;
  if (!diag_skip(8, st))
    bn_bwd_reduce_launch((const bf16_t*)g, (const bf16_t*)y, nullptr, nullptr, (const bf16_t*)xc, mean, invstd, acc,
                         rows, C, st);
  if (diag_skip(64, st)) hipLaunchKernelGGL(bn_bwd_finalize_kernel, dim3((C + kFinCB - 1) / kFinCB), dim3(kFinThreads), 0, st, acc, C, 1.0 / (double)rows,
                     dgamma, dbeta, k1, k2);
  if (!diag_skip(2, st)) hipLaunchKernelGGL(bn_bwd_finalize_kernel, dim3((C + kFinCB - 1) / kFinCB), dim3(kFinThreads), 0, st, acc, C, 1.0 / (double)rows,
                     dgamma, dbeta, k1, k2);
  const long long nvec = rows * C / 8;
  hipLaunchKernelGGL(bn_bwd_apply_kernel<true>, dim3(ew_grid(nvec)), dim3(256), 0, st, (const bf16_t*)g, (const bf16_t*)y,
                     nullptr, nullptr, (const bf16_t*)xc, mean, invstd, gamma, k1, k2, (bf16_t*)gc,
                     (bf16_t*)gmask_out, nvec, C);
  return check_launch("bn_bwd");
}

// BN backward whose reductions were already accumulated into the workspace by a dgrad epilogue
// (avt_conv2d_dgrad_bn) over the pre-masked g': finalize (dgamma, dbeta, k1, k2 from the
// accumulator) + apply gc = gamma*invstd*(g' - k1 - xhat*k2).  Same workspace contract as avt_bn_bwd.
extern "C" int avt_bn_bwd_premasked(const void* gm, const void* xc, const float* mean, const float* invstd,
                                    const float* gamma, float* dgamma, float* dbeta, void* gc, void* workspace,
                                    long long rows, int C, void* stream) {
  AVT_REQUIRE(gm && xc && mean && invstd && gamma && gc && workspace, "bn_bwd_premasked: null pointer");
  AVT_REQUIRE(C % 8 == 0 && C <= 2048 && 256 % (C / 8) == 0, "bn_bwd_premasked: C=%d unsupported", C);
  AVT_REQUIRE(rows > 0, "bn_bwd_premasked: empty input");
  AVT_REQUIRE(((uintptr_t)workspace & 7) == 0, "bn_bwd_premasked: workspace must be 8-byte aligned");
  double* acc = (double*)workspace;
  float* k1 = (float*)(acc + kBnHdr);
  float* k2 = k1 + C;
  hipStream_t st = (hipStream_t)stream;
  if (diag_skip(64, st)) hipLaunchKernelGGL(bn_bwd_finalize_kernel, dim3((C + kFinCB - 1) / kFinCB), dim3(kFinThreads), 0, st, acc, C, 1.0 / (double)rows,
                     dgamma, dbeta, k1, k2);
  if (!diag_skip(2, st)) hipLaunchKernelGGL(bn_bwd_finalize_kernel, dim3((C + kFinCB - 1) / kFinCB), dim3(kFinThreads), 0, st, acc, C, 1.0 / (double)rows,
                     dgamma, dbeta, k1, k2);
  const long long nvec = rows * C / 8;
  hipLaunchKernelGGL(bn_bwd_apply_kernel<true>, dim3(ew_grid(nvec)), dim3(256), 0, st, (const bf16_t*)gm, nullptr,
                     nullptr, nullptr, (const bf16_t*)xc, mean, invstd, gamma, k1, k2, (bf16_t*)gc, nullptr, nvec, C);
  return check_launch("bn_bwd_premasked");
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
  float* k1 = (float*)(acc + kBnHdr);
  float* k2 = k1 + C;
  hipStream_t st = (hipStream_t)stream;
  if (!diag_skip(8, st))
    bn_bwd_reduce_launch((const bf16_t*)g, nullptr, scale, shift, (const bf16_t*)xc, mean, invstd, acc, rows, C, st);
  if (diag_skip(64, st)) hipLaunchKernelGGL(bn_bwd_finalize_kernel, dim3((C + kFinCB - 1) / kFinCB), dim3(kFinThreads), 0, st, acc, C, 1.0 / (double)rows,
                     dgamma, dbeta, k1, k2);
  if (!diag_skip(2, st)) hipLaunchKernelGGL(bn_bwd_finalize_kernel, dim3((C + kFinCB - 1) / kFinCB), dim3(kFinThreads), 0, st, acc, C, 1.0 / (double)rows,
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
  AVT_REQUIRE((long long)((W + 1) / 2 + 1) * C * 6 <= kStemLdsBytes && (long long)2 * W * (C / 8) <= 6 * kStemBwdThreads,
              "stem_maxpool_bn_relu_bwd: W=%d C=%d too wide", W, C);
  AVT_REQUIRE(N > 0 && H > 0 && W > 0, "stem_maxpool_bn_relu_bwd: empty input");
  AVT_REQUIRE(((uintptr_t)workspace & 7) == 0, "stem_maxpool_bn_relu_bwd: workspace must be 8-byte aligned");
  const int P = (H + 2 - 3) / 2 + 1, Q = (W + 2 - 3) / 2 + 1;
  double* acc = (double*)workspace;
  float* k1 = (float*)(acc + kBnHdr);
  float* k2 = k1 + C;
  hipStream_t st = (hipStream_t)stream;
  bn_bwd_reduce_launch((const bf16_t*)gy, nullptr, scale, shift, (const bf16_t*)carg, mean, invstd, acc,
                       (long long)N * P * Q, C, st);
  if (diag_skip(64, st)) hipLaunchKernelGGL(bn_bwd_finalize_kernel, dim3((C + kFinCB - 1) / kFinCB), dim3(kFinThreads), 0, st, acc, C,
                     1.0 / ((double)N * H * W), dgamma, dbeta, k1, k2);
  if (!diag_skip(2, st)) hipLaunchKernelGGL(bn_bwd_finalize_kernel, dim3((C + kFinCB - 1) / kFinCB), dim3(kFinThreads), 0, st, acc, C,
                     1.0 / ((double)N * H * W), dgamma, dbeta, k1, k2);
  hipLaunchKernelGGL(stem_maxpool_bn_bwd_apply_kernel, dim3(N * ((H + 1) / 2)), dim3(kStemBwdThreads), (size_t)6 * Q * C,
                     st, (const bf16_t*)gy,
                     (const unsigned char*)idx, (const bf16_t*)c, scale, shift, mean, invstd, gamma, k1, k2,
                     (bf16_t*)gc, H, W, C, ilog2(C / 8), P, Q);
  return check_launch("stem_maxpool_bn_relu_bwd");
}
