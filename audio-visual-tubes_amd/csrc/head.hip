// Hard-way head (fp32): per-location cosine-similarity map, sigmoid trimap, hard-negative
// logits, cross-entropy, and their backward.  Restates model.py:114-154 (AVENet.forward after
// the trunks) and model.py:46-60 (HardWayAttention) with the CE of train_hardway_1frame.py:130-131.
//
// Data: v   [B][P][C] bf16 (vision layer4, NHWC; P = h*w),  an [B][C] fp32 (unit audio vector)
//       inv [B][P] = 1/max(||v[b,p,:]||, 1e-12),  A0 [B][P][B] fp32 (row (i,p), column j)
// All similarity/trimap math stays fp32 (bf16 sigmoids underflow: SURVEY §0.7).
#include "avt_common.h"

namespace avt {

// 8 consecutive elements of a bf16 or fp32 row as fp32
__device__ __forceinline__ void load8f(const bf16_t* p, float* o) {
  const u32x4 q = *reinterpret_cast<const u32x4*>(p);
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    o[2 * e] = bf2f((bf16_t)(q[e] & 0xffff));
    o[2 * e + 1] = bf2f((bf16_t)(q[e] >> 16));
  }
}
__device__ __forceinline__ void load8f(const float* p, float* o) {
  const f32x4 a = *reinterpret_cast<const f32x4*>(p), b = *reinterpret_cast<const f32x4*>(p + 4);
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    o[e] = a[e];
    o[4 + e] = b[e];
  }
}
__device__ __forceinline__ void store8f(bf16_t* p, const float* x) {
  u32x4 o;
#pragma unroll
  for (int e = 0; e < 4; ++e) o[e] = pack2(x[2 * e], x[2 * e + 1]);
  *reinterpret_cast<u32x4*>(p) = o;
}
__device__ __forceinline__ void store8f(float* p, const float* x) {
  *reinterpret_cast<f32x4*>(p) = f32x4{x[0], x[1], x[2], x[3]};
  *reinterpret_cast<f32x4*>(p + 4) = f32x4{x[4], x[5], x[6], x[7]};
}

// ---- per-(b,p) norms of the vision map: one wave per row of C channels ----
// NORM = false (HardWayAttention, model.py:46-60, which takes the features as given): inv = 1.
template <typename T, bool NORM>
__global__ __launch_bounds__(256) void vis_norm_kernel(const T* __restrict__ v, float* __restrict__ inv,
                                                       float* __restrict__ vsum, int rows, int C) {
  const int w = (blockIdx.x * blockDim.x + threadIdx.x) >> 6, lane = threadIdx.x & 63;
  if (w >= rows) return;
  const T* src = v + (size_t)w * C;
  float ss = 0.f, s = 0.f;
  for (int c = lane * 8; c < C; c += 512) {
    float x[8];
    load8f(src + c, x);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      ss += x[e] * x[e];
      s += x[e];
    }
  }
  ss = wave_sum(ss);
  s = wave_sum(s);
  if (lane == 0) {
    inv[w] = NORM ? 1.f / fmaxf(sqrtf(ss), 1e-12f) : 1.f;
    vsum[w] = s;
  }
}

// ---- small fp32 GEMM with strided operands ----
//   C[m][n] (+)= rowscale[m] * sum_k A(m,k) * kscale[k] * B(k,n)
//   A(m,k) = a[m*sam + k*sak] (TA = bf16_t or float), B(k,n) = b[k*sbk + n*sbn] (TB)
//   split-K over gridDim.z: split z stores its partial product into c + z * M * ldc (a workspace), which
//   sgemm_sum_splits_kernel then sums in split order into the output (deterministic); accum = 1 adds to C.
// 64x64 block tile, 32-deep k-tiles staged through LDS as fp32; four waves each own a 32x32 quarter
// on the fp32 matrix cores (v_mfma_f32_32x32x2_f32: full fp32 products and fp32 accumulation, as
// the reference's fp32 einsum -- only the summation order differs), 16 MFMAs per k-tile.  Each
// thread fetches 8 consecutive elements along an operand's unit-stride dimension (16-B loads where
// aligned and in bounds), and the next k-tile's loads are issued before the current tile's MFMAs.
template <typename T>
__device__ __forceinline__ float ldf(const T* p, size_t i);
template <>
__device__ __forceinline__ float ldf<float>(const float* p, size_t i) { return p[i]; }
template <>
__device__ __forceinline__ float ldf<bf16_t>(const bf16_t* p, size_t i) { return bf2f(p[i]); }

// 8 elements p[i], p[i + st], ..., p[i + 7 st] (only the first `n` valid; the rest 0)
template <typename T>
__device__ __forceinline__ void ld8(const T* p, size_t i, long long st, int n, float* o) {
  const T* q = p + i;
  if (n >= 8 && st == 1 && ((uintptr_t)q & 15) == 0) {
    if constexpr (sizeof(T) == 2) {
      const u32x4 v = *reinterpret_cast<const u32x4*>(q);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        o[2 * e] = bf2f((bf16_t)(v[e] & 0xffff));
        o[2 * e + 1] = bf2f((bf16_t)(v[e] >> 16));
      }
    } else {
      const f32x4 v0 = *reinterpret_cast<const f32x4*>(q);
      const f32x4 v1 = *reinterpret_cast<const f32x4*>(q + 4);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        o[e] = v0[e];
        o[4 + e] = v1[e];
      }
    }
    return;
  }
#pragma unroll
  for (int e = 0; e < 8; ++e) o[e] = e < n ? ldf<T>(p, i + (size_t)e * st) : 0.f;
}

constexpr int kSgKT = 32;  // k-tile depth

template <typename TA, typename TB>
__global__ __launch_bounds__(256) void sgemm_kernel(int M, int N, int K, const TA* __restrict__ a, long long sam,
                                                    long long sak, const TB* __restrict__ b, long long sbk,
                                                    long long sbn, const float* __restrict__ rowscale,
                                                    const float* __restrict__ kscale, float* __restrict__ c,
                                                    long long ldc, int k_per_split, int accum) {
  __shared__ __attribute__((aligned(16))) float As[kSgKT][64 + 4];
  __shared__ __attribute__((aligned(16))) float Bs[kSgKT][64 + 4];
  const int tid = threadIdx.x;
  const int m0 = blockIdx.y * 64, n0 = blockIdx.x * 64;
  const int kbeg = blockIdx.z * k_per_split, kend = min(K, kbeg + k_per_split);
  const int lane = tid & 63, wid = tid >> 6;
  const int wm = wid >> 1, wn = wid & 1;       // this wave's 32x32 quarter
  const int frow = lane & 31, fk = lane >> 5;  // MFMA operand lane: row/col, k within the pair
  // per-thread fetch: 8 consecutive elements along the unit-stride dimension (k when sak/sbk == 1,
  // else m / n), i.e. (row tid/4, k 8*(tid%4)..) or (k tid/8, rows 8*(tid%8)..)
  const bool a_kf = (sak == 1), b_kf = (sbk == 1);
  const int a_r = a_kf ? tid >> 2 : (tid & 7) * 8, a_k = a_kf ? (tid & 3) * 8 : tid >> 3;
  const int b_r = b_kf ? tid >> 2 : (tid & 7) * 8, b_k = b_kf ? (tid & 3) * 8 : tid >> 3;
  float ra[8], rb[8];
  auto fetch = [&](int k0) {
    const int gk = k0 + a_k, gm = m0 + a_r;
    if (a_kf) {
      const int n = (gm < M) ? min(8, kend - gk) : 0;
      ld8<TA>(a, (size_t)gm * sam + gk, 1, n, ra);
      if (kscale)
#pragma unroll
        for (int e = 0; e < 8; ++e) ra[e] *= (e < n) ? kscale[gk + e] : 0.f;
    } else {
      const int n = (gk < kend) ? min(8, M - gm) : 0;
      ld8<TA>(a, (size_t)gk * sak + (size_t)gm * sam, sam, n, ra);
      if (kscale && n > 0) {
        const float ks = kscale[gk];
#pragma unroll
        for (int e = 0; e < 8; ++e) ra[e] *= ks;
      }
    }
    const int gk2 = k0 + b_k, gn = n0 + b_r;
    if (b_kf) {
      const int n = (gn < N) ? min(8, kend - gk2) : 0;
      ld8<TB>(b, (size_t)gn * sbn + gk2, 1, n, rb);
    } else {
      const int n = (gk2 < kend) ? min(8, N - gn) : 0;
      ld8<TB>(b, (size_t)gk2 * sbk + (size_t)gn * sbn, sbn, n, rb);
    }
  };
  auto stash = [&]() {
    if (a_kf) {
#pragma unroll
      for (int e = 0; e < 8; ++e) As[a_k + e][a_r] = ra[e];
    } else {
      *reinterpret_cast<f32x4*>(&As[a_k][a_r]) = f32x4{ra[0], ra[1], ra[2], ra[3]};
      *reinterpret_cast<f32x4*>(&As[a_k][a_r + 4]) = f32x4{ra[4], ra[5], ra[6], ra[7]};
    }
    if (b_kf) {
#pragma unroll
      for (int e = 0; e < 8; ++e) Bs[b_k + e][b_r] = rb[e];
    } else {
      *reinterpret_cast<f32x4*>(&Bs[b_k][b_r]) = f32x4{rb[0], rb[1], rb[2], rb[3]};
      *reinterpret_cast<f32x4*>(&Bs[b_k][b_r + 4]) = f32x4{rb[4], rb[5], rb[6], rb[7]};
    }
  };
  f32x16 acc;
#pragma unroll
  for (int v = 0; v < 16; ++v) acc[v] = 0.f;
  if (kbeg < kend) fetch(kbeg);
  for (int k0 = kbeg; k0 < kend; k0 += kSgKT) {
    stash();
    __syncthreads();
    if (k0 + kSgKT < kend) fetch(k0 + kSgKT);  // in flight during this tile's MFMAs
#pragma unroll
    for (int kp = 0; kp < kSgKT; kp += 2) {
      const float av = As[kp + fk][wm * 32 + frow];
      const float bv = Bs[kp + fk][wn * 32 + frow];
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(av, bv, acc, 0, 0, 0);
    }
    __syncthreads();
  }
  // C layout of a 32x32 MFMA tile: element v of lane l is row (v&3) + 8(v>>2) + 4(l>>5), column l&31
  const int gn = n0 + wn * 32 + frow;
#pragma unroll
  for (int v = 0; v < 16; ++v) {
    const int gm = m0 + wm * 32 + (v & 3) + 8 * (v >> 2) + 4 * fk;
    if (gm >= M || gn >= N) continue;
    const float r = acc[v] * (rowscale ? rowscale[gm] : 1.f);
    if (gridDim.z > 1)
      c[(size_t)blockIdx.z * M * ldc + (size_t)gm * ldc + gn] = r;
    else if (accum)
      c[(size_t)gm * ldc + gn] += r;
    else
      c[(size_t)gm * ldc + gn] = r;
  }
}

__device__ __forceinline__ float sigm(float z) { return 1.f / (1.f + __expf(-z)); }

// ---- logits: one block per row i ----
// save layout (floats per row): [0..B) s_ij, [B..2B) W_ij, 2B: s1, 2B+1: W1, 2B+2: s2, 2B+3: W2
__global__ __launch_bounds__(1024) void hardway_logits_kernel(const float* __restrict__ A0, const float* __restrict__ vsum,
                                                             const float* __restrict__ inv, int B, int P, int C,
                                                             float eps1, float eps2, float tau, int trimap, int use_neg,
                                                             float* __restrict__ logits, float* __restrict__ Aout,
                                                             float* __restrict__ Pos, float* __restrict__ Neg,
                                                             float* __restrict__ wA, float* __restrict__ save) {
  __shared__ float red[16];
  __shared__ float part_w[1024], part_x[1024];
  const int i = blockIdx.x, tid = threadIdx.x, nthr = blockDim.x;
  const int L = B + 1 + (use_neg ? 1 : 0);
  const float* row = A0 + (size_t)i * P * B;
  float* sv = save + (size_t)i * (2 * B + 4);
  const float inv_t = 1.f / tau;
  // sim[i, j] over the P positions: the block takes jb = min(B, nthr) columns per pass and splits
  // each column's P positions over nsub = nthr / jb threads (coalesced over j), then combines the
  // partial sums through LDS -- B columns x P serial steps would leave most of the chip idle
  const int jb = min(B, nthr), nsub = nthr / jb;
  const int jl = tid % jb, part = tid / jb;
  for (int j0 = 0; j0 < B; j0 += jb) {
    const int j = j0 + jl;
    float sw = 0.f, swx = 0.f;
    if (j < B && part < nsub)
      for (int p = part; p < P; p += nsub) {
        const float x = row[(size_t)p * B + j];
        const float w = sigm((x - eps1) * inv_t);
        sw += w;
        swx += w * x;
      }
    part_w[tid] = sw;
    part_x[tid] = swx;
    __syncthreads();
    if (part == 0 && j < B) {
      float tw = 0.f, tx = 0.f;
      for (int k = 0; k < nsub; ++k) {
        tw += part_w[k * jb + jl];
        tx += part_x[k * jb + jl];
      }
      const float s = tx / tw;
      sv[j] = s;
      sv[B + j] = tw;
      logits[(size_t)i * L + 1 + j] = s * (j == i ? -99.f : 1.f) / 0.07f;
    }
    __syncthreads();
  }
  // positive / negative on A = A0[i, :, i]
  float s1w = 0.f, s1x = 0.f, s2w = 0.f, s2x = 0.f, pp = 0.f;
  for (int p = tid; p < P; p += blockDim.x) {
    const float x = row[(size_t)p * B + i];
    const float w = sigm((x - eps1) * inv_t);
    const float wn = trimap ? sigm(-(x - eps2) * inv_t) : sigm(-(x - eps1) * inv_t);
    s1w += w;
    s1x += w * x;
    s2w += wn;
    s2x += wn * x;
    pp += w * w;
    Aout[(size_t)i * P + p] = x;
    Pos[(size_t)i * P + p] = w;
    Neg[(size_t)i * P + p] = wn;
  }
  s1w = block_sum(s1w, red);
  s1x = block_sum(s1x, red);
  s2w = block_sum(s2w, red);
  s2x = block_sum(s2x, red);
  pp = block_sum(pp, red);
  const float s1 = s1x / s1w, s2 = s2x / s2w;
  if (tid == 0) {
    sv[2 * B] = s1;
    sv[2 * B + 1] = s1w;
    sv[2 * B + 2] = s2;
    sv[2 * B + 3] = s2w;
    logits[(size_t)i * L] = s1 / 0.07f;
    if (use_neg) logits[(size_t)i * L + B + 1] = s2 / 0.07f;
  }
  // weighted_A = mean_c(vhat) * Pos / max(||Pos||, 1e-12)   (model.py:148-152)
  const float pn = 1.f / fmaxf(sqrtf(pp), 1e-12f);
  for (int p = tid; p < P; p += blockDim.x) {
    const size_t r = (size_t)i * P + p;
    wA[r] = vsum[r] * inv[r] / (float)C * Pos[r] * pn;
  }
}

// ---- CE(target 0), mean over the B rows, times `scale`: loss and dlogits ----
// one block of 1024 threads; wave w handles rows w, w+16, ... with lane-parallel max/sum
__global__ __launch_bounds__(1024) void hardway_ce_kernel(const float* __restrict__ logits, int B, int L, float scale,
                                                          float* __restrict__ loss, float* __restrict__ dlogits) {
  // one wave per row, the 16 waves' rows in groups of 4 whose loads are all issued up front (a row of
  // L <= 256 logits is 4 values per lane); wider rows take the strided loop
  __shared__ float red[16];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  constexpr int RG = 4;
  float part = 0.f;
  for (int i0 = w * RG; i0 < B; i0 += 16 * RG) {
    if (L <= 256) {
      float x[RG][4];
#pragma unroll
      for (int r = 0; r < RG; ++r)
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const int j = lane + 64 * k;
          x[r][k] = (i0 + r < B && j < L) ? logits[(size_t)(i0 + r) * L + j] : -INFINITY;
        }
#pragma unroll
      for (int r = 0; r < RG; ++r) {
        const int i = i0 + r;
        if (i >= B) break;
        const float mx = wave_max(fmaxf(fmaxf(x[r][0], x[r][1]), fmaxf(x[r][2], x[r][3])));
        float se = 0.f;
#pragma unroll
        for (int k = 0; k < 4; ++k) se += lane + 64 * k < L ? expf(x[r][k] - mx) : 0.f;
        se = wave_sum(se);
        const float lse = mx + logf(se);
        if (lane == 0) part += lse - x[r][0];
        if (dlogits) {
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            const int j = lane + 64 * k;
            if (j < L) dlogits[(size_t)i * L + j] = (expf(x[r][k] - lse) - (j == 0 ? 1.f : 0.f)) * scale / (float)B;
          }
        }
      }
      continue;
    }
    for (int i = i0; i < min(B, i0 + RG); ++i) {
      const float* r = logits + (size_t)i * L;
      float mx = -INFINITY;
      for (int j = lane; j < L; j += 64) mx = fmaxf(mx, r[j]);
      mx = wave_max(mx);
      float se = 0.f;
      for (int j = lane; j < L; j += 64) se += expf(r[j] - mx);
      se = wave_sum(se);
      const float lse = mx + logf(se);
      if (lane == 0) part += lse - r[0];
      if (dlogits) {
        for (int j = lane; j < L; j += 64) {
          const float sm = expf(r[j] - lse);
          dlogits[(size_t)i * L + j] = (sm - (j == 0 ? 1.f : 0.f)) * scale / (float)B;
        }
      }
    }
  }
  const float tot = block_sum(part, red);
  if (threadIdx.x == 0 && loss) *loss = tot / (float)B;
}

// ---- backward of the logits w.r.t. A0: blocks (i, slice of the P*B elements of row i); dA0 [B][P][B] ----
__global__ __launch_bounds__(256) void hardway_logits_bwd_kernel(const float* __restrict__ A0,
                                                                 const float* __restrict__ save,
                                                                 const float* __restrict__ dlogits, int B, int P,
                                                                 float eps1, float eps2, float tau, int trimap,
                                                                 int use_neg, float* __restrict__ dA0) {
  const int i = blockIdx.x;
  const int L = B + 1 + (use_neg ? 1 : 0);
  const float* row = A0 + (size_t)i * P * B;
  float* drow = dA0 + (size_t)i * P * B;
  const float* sv = save + (size_t)i * (2 * B + 4);
  const float inv_t = 1.f / tau;
  const float* dl = dlogits + (size_t)i * L;
  const float s1 = sv[2 * B], W1 = sv[2 * B + 1], s2 = sv[2 * B + 2], W2 = sv[2 * B + 3];
  const float ds1 = dl[0] / 0.07f;
  const float ds2 = use_neg ? dl[B + 1] / 0.07f : 0.f;
  const size_t n = (size_t)P * B;
  for (size_t t = (size_t)blockIdx.y * blockDim.x + threadIdx.x; t < n; t += (size_t)gridDim.y * blockDim.x) {
    const int j = (int)(t % B);
    const float x = row[t];
    const float w = sigm((x - eps1) * inv_t);
    const float wd = w * (1.f - w) * inv_t;
    const float dsim = dl[1 + j] * (j == i ? -99.f : 1.f) / 0.07f;
    float g = dsim * (w + wd * (x - sv[j])) / sv[B + j];
    if (j == i) {
      g += ds1 * (w + wd * (x - s1)) / W1;
      if (use_neg) {
        const float wn = trimap ? sigm(-(x - eps2) * inv_t) : sigm(-(x - eps1) * inv_t);
        const float wnd = -wn * (1.f - wn) * inv_t;
        g += ds2 * (wn + wnd * (x - s2)) / W2;
      }
    }
    drow[t] = g;
  }
}

// ---- normalize backward for the vision map: gv = inv*(dvh - vh*<vh,dvh>), vh = v*inv ----
// dm (optional) [rows]: gradient w.r.t. mean_c(vh) (weighted_A path) — adds dm/C to every channel of dvh.
// NORM = false (no normalisation in the forward): gv = dvh (+ dm/C).
template <typename T, bool NORM>
__global__ __launch_bounds__(256) void vis_norm_bwd_kernel(const T* __restrict__ v, const float* __restrict__ inv,
                                                           const float* __restrict__ dvh, const float* __restrict__ dm,
                                                           T* __restrict__ gv, int rows, int C) {
  const int w = (blockIdx.x * blockDim.x + threadIdx.x) >> 6, lane = threadIdx.x & 63;
  if (w >= rows) return;
  const T* src = v + (size_t)w * C;
  const float* d = dvh + (size_t)w * C;
  const float iv = inv[w];
  const float dmc = dm ? dm[w] / (float)C : 0.f;
  float dot = 0.f;
  if (NORM) {
    for (int c = lane * 8; c < C; c += 512) {
      float x[8];
      load8f(src + c, x);
#pragma unroll
      for (int e = 0; e < 8; ++e) dot += x[e] * (d[c + e] + dmc);
    }
    dot = wave_sum(dot) * iv;  // <vh, dvh>
  }
  for (int c = lane * 8; c < C; c += 512) {
    float x[8], o[8];
    if (NORM) load8f(src + c, x);
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = NORM ? iv * (d[c + e] + dmc - x[e] * iv * dot) : d[c + e] + dmc;
    store8f(gv + (size_t)w * C + c, o);
  }
}

// ---- weighted_A backward (model.py:148-152): one block per row i ----
// wA[i,p] = m[i,p] * Pos[i,p] / max(||Pos_i||, 1e-12),  m = mean_c(vh) = vsum*inv/C,
// Pos = sigmoid((A - eps1)/tau), A[i,p] = A0[i,p,i].  Given g = dwA:
//   dm[i,p]      = g * Pos * pn                                 (-> every channel of dvh, /C)
//   dPos         = (u - Pos * pn^2 * <Pos,u>) * pn,  u = g*m    (F.normalize backward, ||Pos|| > eps)
//                = u * pn                                       (||Pos|| <= eps: clamp_min passes no grad)
//   dA0[i,p,i]  += dPos * Pos*(1-Pos)/tau                       (A is the diagonal of A0)
// Runs after hardway_logits_bwd_kernel (read-modify-write of the diagonal it wrote).
__global__ __launch_bounds__(256) void hardway_wa_bwd_kernel(const float* __restrict__ A0, const float* __restrict__ dwA,
                                                             const float* __restrict__ vsum,
                                                             const float* __restrict__ inv, int B, int P, int C,
                                                             float eps1, float tau, float* __restrict__ dA0,
                                                             float* __restrict__ dm) {
  __shared__ float red[16];
  const int i = blockIdx.x, tid = threadIdx.x;
  const float inv_t = 1.f / tau, invC = 1.f / (float)C;
  const float* row = A0 + (size_t)i * P * B;
  const size_t r0 = (size_t)i * P;
  float pp = 0.f, dot = 0.f;
  for (int p = tid; p < P; p += blockDim.x) {
    const float w = sigm((row[(size_t)p * B + i] - eps1) * inv_t);
    const float m = vsum[r0 + p] * inv[r0 + p] * invC;
    pp += w * w;
    dot += w * dwA[r0 + p] * m;
  }
  pp = block_sum(pp, red);
  dot = block_sum(dot, red);
  const float nrm = sqrtf(pp);
  const float pn = 1.f / fmaxf(nrm, 1e-12f);
  const float proj = nrm > 1e-12f ? dot * pn * pn : 0.f;
  for (int p = tid; p < P; p += blockDim.x) {
    const size_t d = (size_t)p * B + i;
    const float w = sigm((row[d] - eps1) * inv_t);
    const float g = dwA[r0 + p];
    const float m = vsum[r0 + p] * inv[r0 + p] * invC;
    const float dpos = (g * m - w * proj) * pn;
    dA0[(size_t)i * P * B + d] += dpos * w * (1.f - w) * inv_t;
    dm[r0 + p] = g * w * pn;
  }
}

// ---- gradients arriving through the returned A, Pos, Neg (model.py:124-135, returned at 154) ----
// A[i,p] = A0[i,p,i]; Pos = sigmoid((A-eps1)/tau); Neg = 1 - sigmoid((A-eps2)/tau) (tri_map) or 1 - Pos:
//   dA0[i,p,i] += gA + gPos * Pos(1-Pos)/tau - gNeg * Neg(1-Neg)/tau      (any of gA/gPos/gNeg may be NULL)
// Runs after hardway_logits_bwd_kernel (read-modify-write of the diagonal it wrote).
__global__ __launch_bounds__(256) void hardway_aux_bwd_kernel(const float* __restrict__ A0, const float* __restrict__ gA,
                                                              const float* __restrict__ gPos,
                                                              const float* __restrict__ gNeg, int B, int P, float eps1,
                                                              float eps2, float tau, int trimap,
                                                              float* __restrict__ dA0) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= B * P) return;
  const int i = t / P, p = t - i * P;
  const size_t d = ((size_t)i * P + p) * B + i;
  const float x = A0[d], inv_t = 1.f / tau;
  float g = gA ? gA[t] : 0.f;
  if (gPos) {
    const float w = sigm((x - eps1) * inv_t);
    g += gPos[t] * w * (1.f - w) * inv_t;
  }
  if (gNeg) {
    const float wn = trimap ? sigm(-(x - eps2) * inv_t) : sigm(-(x - eps1) * inv_t);
    g -= gNeg[t] * wn * (1.f - wn) * inv_t;
  }
  dA0[d] += g;
}

// ---- the 16-frame two-view losses of train_hardway.py:134-142, one block of 1024 threads ----
//   hardway = lw*CE1, aug = lw*CE2 (CE1/CE2: the hardway_ce outputs), l2 = (100-lw)*MSE(wA1, wA2),
//   consistency = Prop(wA1) + Prop(wA2),  Prop(x) = mean |x[:,s+1] - x[:,s]| over (clip, s, p)
//   (losses.py:16-23 with x = weighted.reshape(b, t, h, w)),
//   combined = (hardway + aug)/2 + l2 + consistency.
// out[5] = {combined, hardway, aug, l2, consistency}; d1/d2 = d(combined)/d(wA1), d(wA2) (the
// logits gradients come from hardway_ce with scale lw/2).  wA rows are '(b t)', clip-major.
__device__ __forceinline__ float sgnf(float x) { return x > 0.f ? 1.f : (x < 0.f ? -1.f : 0.f); }

__global__ __launch_bounds__(1024) void twoview_loss_kernel(const float* __restrict__ ce1, const float* __restrict__ ce2,
                                                            const float* __restrict__ w1, const float* __restrict__ w2,
                                                            int b, int t, int P, float lw, float* __restrict__ out,
                                                            float* __restrict__ d1, float* __restrict__ d2) {
  __shared__ float red[16];
  const long long n = (long long)b * t * P;
  const float kmse = (100.f - lw) / (float)n;
  const float kprop = 1.f / ((float)b * (float)(t - 1) * (float)P);
  float se = 0.f, a1 = 0.f, a2 = 0.f;
  for (long long e = threadIdx.x; e < n; e += blockDim.x) {
    const int s = (int)((e / P) % t);
    const float x1 = w1[e], x2 = w2[e];
    const float df = x1 - x2;
    se += df * df;
    float g1 = 2.f * df * kmse, g2 = -2.f * df * kmse;
    if (s + 1 < t) {  // diff (s+1) - s
      const float u1 = w1[e + P] - x1, u2 = w2[e + P] - x2;
      a1 += fabsf(u1);
      a2 += fabsf(u2);
      g1 -= sgnf(u1) * kprop;
      g2 -= sgnf(u2) * kprop;
    }
    if (s > 0) {  // diff s - (s-1)
      g1 += sgnf(x1 - w1[e - P]) * kprop;
      g2 += sgnf(x2 - w2[e - P]) * kprop;
    }
    d1[e] = g1;
    d2[e] = g2;
  }
  se = block_sum(se, red);
  a1 = block_sum(a1, red);
  a2 = block_sum(a2, red);
  if (threadIdx.x == 0) {
    const float hard = lw * ce1[0], aug = lw * ce2[0];
    const float l2 = se * kmse, cons = a1 * kprop + a2 * kprop;
    out[0] = (hard + aug) * 0.5f + l2 + cons;
    out[1] = hard;
    out[2] = aug;
    out[3] = l2;
    out[4] = cons;
  }
}

// ---- PropagationLoss (losses.py:16-23) on x [b][t][P]: loss and d(loss)/dx, one block ----
// ---- losses.py on a multi-block grid: every element's gradient in one grid-stride pass, each block's
// partial |.| sum into ws[block], then ONE block sums ws[0..nblk) in a fixed order (deterministic) ----
constexpr int kLossMaxBlocks = 1024;

__device__ __forceinline__ void block_partial(float a, float* red, float* ws) {
  a = block_sum(a, red);
  if (threadIdx.x == 0) ws[blockIdx.x] = a;
}

// loss = scale * sum_{i < n} ws[i], summed by one block in a fixed order
__global__ __launch_bounds__(256) void loss_finish_kernel(const float* __restrict__ ws, int n, float scale,
                                                          float* __restrict__ loss) {
  __shared__ float red[16];
  float a = 0.f;
  for (int i = threadIdx.x; i < n; i += blockDim.x) a += ws[i];
  a = block_sum(a, red);
  if (threadIdx.x == 0) *loss = a * scale;
}

// PropagationLoss (losses.py:16-23) on x [b][t][P]: mean over (b, s < t-1, p) of |x[b,s+1,p] - x[b,s,p]|
__global__ __launch_bounds__(256) void propagation_loss_kernel(const float* __restrict__ x, int t, int P, long long n,
                                                               float k, float* __restrict__ dx, float* __restrict__ ws) {
  __shared__ float red[16];
  float a = 0.f;
  for (long long e = blockIdx.x * (long long)blockDim.x + threadIdx.x; e < n; e += (long long)gridDim.x * blockDim.x) {
    const int s = (int)((e / P) % t);
    float g = 0.f;
    if (s + 1 < t) {
      const float u = x[e + P] - x[e];
      a += fabsf(u);
      g -= sgnf(u) * k;
    }
    if (s > 0) g += sgnf(x[e] - x[e - P]) * k;
    if (dx) dx[e] = g;
  }
  block_partial(a, red, ws);
}

// ---- NPRatio (losses.py:7-14) on x [b][t][P]: loss = mean_b mean_s |S[b,s+1] - S[b,s]|, S = sum_p x ----
// pass 1: S[r] (one wave per row) into ws; pass 2: dx[b,s,p] = dloss/dS[b,s] for every p, and the
// per-block partial sums of |S[r+1] - S[r]| over the rows the block's first elements start
__global__ __launch_bounds__(256) void npratio_rows_kernel(const float* __restrict__ x, int rows, int P,
                                                           float* __restrict__ S) {
  const int lane = threadIdx.x & 63;
  const int nw = (gridDim.x * blockDim.x) >> 6;
  for (int r = (blockIdx.x * blockDim.x + threadIdx.x) >> 6; r < rows; r += nw) {
    float a = 0.f;
    for (int p = lane; p < P; p += 64) a += x[(size_t)r * P + p];
    a = wave_sum(a);
    if (lane == 0) S[r] = a;
  }
}

__global__ __launch_bounds__(256) void npratio_loss_kernel(const float* __restrict__ S, int rows, int t, int P,
                                                           float k, float* __restrict__ dx, float* __restrict__ ws) {
  __shared__ float red[16];
  float acc = 0.f;
  for (int r = blockIdx.x * blockDim.x + threadIdx.x; r < rows; r += gridDim.x * blockDim.x)
    if (r % t + 1 < t) acc += fabsf(S[r + 1] - S[r]);
  block_partial(acc, red, ws);
  if (dx) {
    const long long n = (long long)rows * P;
    for (long long e = blockIdx.x * (long long)blockDim.x + threadIdx.x; e < n; e += (long long)gridDim.x * blockDim.x) {
      const int r = (int)(e / P), s = r % t;
      float g = 0.f;
      if (s + 1 < t) g -= sgnf(S[r + 1] - S[r]) * k;
      if (s > 0) g += sgnf(S[r] - S[r - 1]) * k;
      dx[e] = g;
    }
  }
}

// ---- FlipLoss (losses.py:25-36): nn.L1Loss()(y, hflip(x)) over rows of W (the last dim) ----
// loss = mean |y[r,w] - x[r,W-1-w]|; dy = sgn(.)/n, dx[r,W-1-w] = -sgn(.)/n (sgn(0) = 0, as torch)
__global__ __launch_bounds__(256) void flip_l1_loss_kernel(const float* __restrict__ x, const float* __restrict__ y,
                                                           long long n, int W, float inv_n, float* __restrict__ dx,
                                                           float* __restrict__ dy, float* __restrict__ ws) {
  __shared__ float red[16];
  float acc = 0.f;
  for (long long e = blockIdx.x * (long long)blockDim.x + threadIdx.x; e < n; e += (long long)gridDim.x * blockDim.x) {
    const long long r = e / W;
    const int wc = (int)(e - r * W);
    const long long ef = r * W + (W - 1 - wc);
    const float d = y[e] - x[ef];
    acc += fabsf(d);
    if (dy) dy[e] = sgnf(d) * inv_n;
    if (dx) dx[ef] = -sgnf(d) * inv_n;
  }
  block_partial(acc, red, ws);
}

static int loss_blocks(long long n) {
  long long b = (n + 1023) / 1024;  // ~4 elements per thread
  return (int)(b < 1 ? 1 : (b > kLossMaxBlocks ? kLossMaxBlocks : b));
}

__global__ __launch_bounds__(256) void zero_f32_kernel(float* __restrict__ p, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) p[i] = 0.f;
}

// out[r * ldc + c] (+)= sum over s = 0 .. splits-1 of part[s * n + r * N + c] (dense M x N partials), in that order
__global__ __launch_bounds__(256) void sgemm_sum_splits_kernel(const float* __restrict__ part, int splits, long long n,
                                                               int N, long long ldc, float* __restrict__ out, int accum) {
  for (long long i = blockIdx.x * 256ll + threadIdx.x; i < n; i += (long long)gridDim.x * 256) {
    float v = 0.f;
    for (int s = 0; s < splits; ++s) v += part[s * n + i];
    const long long r = i / N, o = r * ldc + (i - r * N);
    out[o] = accum ? out[o] + v : v;
  }
}

// split-K partials of the head GEMMs: at most kSgSplits splits of an M x N output
constexpr int kSgSplits = 64;

// C = ... with up to `splits` k-splits; ws: kSgSplits * M * N floats for the split partials (NULL: one split)
template <typename TA, typename TB>
static void sgemm(int M, int N, int K, const TA* a, long long sam, long long sak, const TB* b, long long sbk,
                  long long sbn, const float* rowscale, const float* kscale, float* c, long long ldc, int splits,
                  hipStream_t st, int accum = 0, float* ws = nullptr) {
  if (ws == nullptr) splits = 1;
  if (splits > kSgSplits) splits = kSgSplits;
  int kps = (K + splits - 1) / splits;
  kps = ((kps + kSgKT - 1) / kSgKT) * kSgKT;
  splits = (K + kps - 1) / kps;
  dim3 grid((N + 63) / 64, (M + 63) / 64, splits);
  if (splits > 1) {
    hipLaunchKernelGGL((sgemm_kernel<TA, TB>), grid, dim3(256), 0, st, M, N, K, a, sam, sak, b, sbk, sbn, rowscale,
                       kscale, ws, (long long)N, kps, 0);
    const long long n = (long long)M * N;  // the partials are dense M x N; the sum honours ldc
    hipLaunchKernelGGL(sgemm_sum_splits_kernel, dim3((unsigned)min(2048LL, (n + 255) / 256)), dim3(256), 0, st, ws,
                       splits, n, N, ldc, c, accum);
  } else {
    hipLaunchKernelGGL((sgemm_kernel<TA, TB>), grid, dim3(256), 0, st, M, N, K, a, sam, sak, b, sbk, sbn, rowscale,
                       kscale, c, ldc, kps, accum);
  }
}

}  // namespace avt

using namespace avt;

extern "C" size_t avt_hardway_save_floats(int B) { return (size_t)B * (2 * B + 4); }

extern "C" size_t avt_hardway_bwd_ws_floats(int B, int C) { return B > 0 && C > 0 ? (size_t)kSgSplits * B * C : 0; }

// Forward of the hard-way head from the trunk outputs.
//   v [B][P][C] bf16, an [B][C] fp32 (unit audio vectors)
//   outputs: logits [B][B+2|B+1], A/Pos/Neg/wA [B][P]
//   saved for backward: inv [B][P], vsum [B][P], A0 [B][P][B], save [B][2B+4]
extern "C" int avt_hardway_fwd(const void* v, const float* an, int B, int P, int C, float eps1, float eps2, float tau,
                               int trimap, int use_neg, float* inv, float* vsum, float* A0, float* save, float* logits,
                               float* Aout, float* Pos, float* Neg, float* wA, void* stream) {
  AVT_REQUIRE(v && an && inv && vsum && A0 && save && logits && Aout && Pos && Neg && wA, "hardway_fwd: null pointer");
  AVT_REQUIRE(C % 8 == 0 && B >= 1 && P >= 1, "hardway_fwd: bad shape B=%d P=%d C=%d", B, P, C);
  hipStream_t st = (hipStream_t)stream;
  const int rows = B * P;
  hipLaunchKernelGGL((vis_norm_kernel<bf16_t, true>), dim3((rows + 3) / 4), dim3(256), 0, st, (const bf16_t*)v, inv,
                     vsum, rows, C);
  // A0[(i,p)][j] = inv[(i,p)] * sum_c v[(i,p)][c] * an[j][c]
  sgemm<bf16_t, float>(rows, B, C, (const bf16_t*)v, C, 1, an, 1, C, inv, nullptr, A0, B, 1, st);
  hipLaunchKernelGGL(hardway_logits_kernel, dim3(B), dim3(1024), 0, st, A0, vsum, inv, B, P, C, eps1, eps2, tau,
                     trimap, use_neg, logits, Aout, Pos, Neg, wA, save);
  return check_launch("hardway_fwd");
}

extern "C" int avt_hardway_ce(const float* logits, int B, int L, float scale, float* loss, float* dlogits,
                              void* stream) {
  AVT_REQUIRE(logits, "hardway_ce: null pointer");
  hipLaunchKernelGGL(hardway_ce_kernel, dim3(1), dim3(1024), 0, (hipStream_t)stream, logits, B, L, scale, loss, dlogits);
  return check_launch("hardway_ce");
}

// Backward from dlogits (and optionally d weighted_A) to the trunk outputs.
//   workspace: dA0 [B][P][B] fp32 + dvh [B][P][C] fp32 (+ dm [B][P] with dwA)
//   dwA [B][P] (NULL: the logits are the only loss input, the 1-frame step); needs vsum from the
//   forward and the vision gradient (gv).
//   outputs: gv [B][P][C] bf16 (grad of the vision layer4 map; dvh = gv = NULL skips it), gan [B][C] fp32
//   (grad of the unit audio vectors; gan_accumulate = 1 adds to gan instead of overwriting it)
//   gA/gPos/gNeg [B][P] (each may be NULL): upstream gradients of the returned A, Pos, Neg maps
//   (avt_hardway_bwd_ex; avt_hardway_bwd = all three NULL)
extern "C" int avt_hardway_bwd_ex(const void* v, const float* an, const float* inv, const float* A0,
                                  const float* save, const float* dlogits, int B, int P, int C, float eps1, float eps2,
                                  float tau, int trimap, int use_neg, const float* dwA, const float* vsum, float* dm,
                                  const float* gA, const float* gPos, const float* gNeg, float* dA0, float* dvh,
                                  void* gv, float* gan, int gan_accumulate, float* ws, void* stream) {
  AVT_REQUIRE(v && an && inv && A0 && save && dlogits && dA0 && gan, "hardway_bwd: null pointer");
  AVT_REQUIRE((dvh == nullptr) == (gv == nullptr), "hardway_bwd: dvh and gv must be both set or both null");
  AVT_REQUIRE(dwA == nullptr || (vsum && dm && gv), "hardway_bwd: dwA needs vsum, dm and the vision gradient");
  hipStream_t st = (hipStream_t)stream;
  const int rows = B * P;
  // ~8 elements per thread: B = 128 -> 128 x 12 blocks instead of 128 long-running ones
  const int nslice = (int)min(64LL, max(1LL, ((long long)P * B + 2047) / 2048));
  hipLaunchKernelGGL(hardway_logits_bwd_kernel, dim3(B, nslice), dim3(256), 0, st, A0, save, dlogits, B, P, eps1, eps2,
                     tau, trimap, use_neg, dA0);
  if (dwA != nullptr)
    hipLaunchKernelGGL(hardway_wa_bwd_kernel, dim3(B), dim3(256), 0, st, A0, dwA, vsum, inv, B, P, C, eps1, tau, dA0, dm);
  if (gA != nullptr || gPos != nullptr || gNeg != nullptr)
    hipLaunchKernelGGL(hardway_aux_bwd_kernel, dim3((rows + 255) / 256), dim3(256), 0, st, A0, gA, gPos, gNeg, B, P,
                       eps1, eps2, tau, trimap, dA0);
  // dvh[(i,p)][c] = sum_j dA0[(i,p)][j] * an[j][c]   (skipped when the vision map is detached:
  // the tube head, whose video features come from a detached forward hook, model.py:12-15)
  if (gv != nullptr) sgemm<float, float>(rows, C, B, dA0, B, 1, an, C, 1, nullptr, nullptr, dvh, C, 1, st);
  // gan[j][c] (+)= sum_{(i,p)} dA0[(i,p)][j] * inv[(i,p)] * v[(i,p)][c]: split-K over the B*P rows through the
  // ws partials, summed in split order (deterministic)
  int splits = rows / 256;
  if (splits < 1) splits = 1;
  sgemm<float, bf16_t>(B, C, rows, dA0, 1, B, (const bf16_t*)v, C, 1, nullptr, inv, gan, C, splits, st,
                       gan_accumulate, ws);
  if (gv != nullptr)
    hipLaunchKernelGGL((vis_norm_bwd_kernel<bf16_t, true>), dim3((rows + 3) / 4), dim3(256), 0, st, (const bf16_t*)v,
                       inv, dvh, dwA != nullptr ? dm : nullptr, (bf16_t*)gv, rows, C);
  return check_launch("hardway_bwd");
}

extern "C" int avt_hardway_bwd(const void* v, const float* an, const float* inv, const float* A0, const float* save,
                               const float* dlogits, int B, int P, int C, float eps1, float eps2, float tau, int trimap,
                               int use_neg, const float* dwA, const float* vsum, float* dm, float* dA0, float* dvh,
                               void* gv, float* gan, int gan_accumulate, void* stream) {
  return avt_hardway_bwd_ex(v, an, inv, A0, save, dlogits, B, P, C, eps1, eps2, tau, trimap, use_neg, dwA, vsum, dm,
                            nullptr, nullptr, nullptr, dA0, dvh, gv, gan, gan_accumulate, nullptr, stream);
}

// Standalone HardWayAttention (model.py:38-60): the head on fp32 features taken as given (no
// normalisation inside; FullModel normalises before the call), trimap and Neg on, fp32 throughout.
//   v [B][P][C] fp32 ('(b t) (h w) c' of video_features), an [B][C] fp32 (audio_features)
//   outputs: logits [B][B+2], A [B][P] (+ Pos/Neg/wA [B][P], scratch of the shared logits kernel)
//   saved for backward: inv [B][P] (= 1), vsum [B][P], A0 [B][P][B], save [B][2B+4]
extern "C" int avt_hardway_attention_fwd(const float* v, const float* an, int B, int P, int C, float eps1, float eps2,
                                         float tau, float* inv, float* vsum, float* A0, float* save, float* logits,
                                         float* Aout, float* Pos, float* Neg, float* wA, void* stream) {
  AVT_REQUIRE(v && an && inv && vsum && A0 && save && logits && Aout && Pos && Neg && wA,
              "hardway_attention_fwd: null pointer");
  AVT_REQUIRE(C % 8 == 0 && B >= 1 && P >= 1, "hardway_attention_fwd: bad shape B=%d P=%d C=%d", B, P, C);
  hipStream_t st = (hipStream_t)stream;
  const int rows = B * P;
  hipLaunchKernelGGL((vis_norm_kernel<float, false>), dim3((rows + 3) / 4), dim3(256), 0, st, v, inv, vsum, rows, C);
  sgemm<float, float>(rows, B, C, v, C, 1, an, 1, C, nullptr, nullptr, A0, B, 1, st);
  hipLaunchKernelGGL(hardway_logits_kernel, dim3(B), dim3(1024), 0, st, A0, vsum, inv, B, P, C, eps1, eps2, tau, 1, 1,
                     logits, Aout, Pos, Neg, wA, save);
  return check_launch("hardway_attention_fwd");
}

// Backward of avt_hardway_attention_fwd from d logits (and optionally d A): gv [B][P][C] fp32 (d video
// features; dvh [B][P][C] fp32 and dA0 [B][P][B] are workspace), gan [B][C] fp32 (d audio features).
extern "C" int avt_hardway_attention_bwd(const float* v, const float* an, const float* inv, const float* A0,
                                         const float* save, const float* dlogits, const float* gA, int B, int P,
                                         int C, float eps1, float eps2, float tau, float* dA0, float* dvh, float* gv,
                                         float* gan, float* ws, void* stream) {
  AVT_REQUIRE(v && an && inv && A0 && save && dlogits && dA0 && dvh && gv && gan,
              "hardway_attention_bwd: null pointer");
  AVT_REQUIRE(C % 8 == 0 && B >= 1 && P >= 1, "hardway_attention_bwd: bad shape B=%d P=%d C=%d", B, P, C);
  hipStream_t st = (hipStream_t)stream;
  const int rows = B * P;
  const int nslice = (int)min(64LL, max(1LL, ((long long)P * B + 2047) / 2048));
  hipLaunchKernelGGL(hardway_logits_bwd_kernel, dim3(B, nslice), dim3(256), 0, st, A0, save, dlogits, B, P, eps1, eps2,
                     tau, 1, 1, dA0);
  if (gA != nullptr)
    hipLaunchKernelGGL(hardway_aux_bwd_kernel, dim3((rows + 255) / 256), dim3(256), 0, st, A0, gA, nullptr, nullptr,
                       B, P, eps1, eps2, tau, 1, dA0);
  sgemm<float, float>(rows, C, B, dA0, B, 1, an, C, 1, nullptr, nullptr, dvh, C, 1, st);
  int splits = rows / 256;
  if (splits < 1) splits = 1;
  sgemm<float, float>(B, C, rows, dA0, 1, B, v, C, 1, nullptr, nullptr, gan, C, splits, st, 0, ws);
  hipLaunchKernelGGL((vis_norm_bwd_kernel<float, false>), dim3((rows + 3) / 4), dim3(256), 0, st, v, inv, dvh,
                     nullptr, gv, rows, C);
  return check_launch("hardway_attention_bwd");
}

// The 16-frame two-view loss combination (train_hardway.py:134-142) from the two CE values.
extern "C" int avt_twoview_loss(const float* ce1, const float* ce2, const float* wA1, const float* wA2, int b, int t,
                                int P, float loss_weight, float* out, float* dwA1, float* dwA2, void* stream) {
  AVT_REQUIRE(ce1 && ce2 && wA1 && wA2 && out && dwA1 && dwA2, "twoview_loss: null pointer");
  AVT_REQUIRE(b >= 1 && t >= 2 && P >= 1, "twoview_loss: need b >= 1, t >= 2 frames, P >= 1 (b=%d t=%d P=%d)", b, t, P);
  hipLaunchKernelGGL(twoview_loss_kernel, dim3(1), dim3(1024), 0, (hipStream_t)stream, ce1, ce2, wA1, wA2, b, t, P,
                     loss_weight, out, dwA1, dwA2);
  return check_launch("twoview_loss");
}

// scratch floats the three losses below need: per-block partial sums (+ NPRatio's row sums S)
extern "C" size_t avt_loss_workspace_floats(long long n, long long rows) {
  return (size_t)kLossMaxBlocks + (size_t)(rows > 0 ? rows : 0);
}

// PropagationLoss (losses.py:16-23) of x [b][t][P]; dx (optional) = d(loss)/dx.  ws: avt_loss_workspace_floats.
extern "C" int avt_propagation_loss(const float* x, int b, int t, int P, float* loss, float* dx, float* ws,
                                    void* stream) {
  AVT_REQUIRE(x && loss && ws, "propagation_loss: null pointer");
  AVT_REQUIRE(b >= 1 && t >= 2 && P >= 1, "propagation_loss: need b >= 1, t >= 2, P >= 1 (b=%d t=%d P=%d)", b, t, P);
  hipStream_t st = (hipStream_t)stream;
  const long long n = (long long)b * t * P;
  const float k = 1.f / ((float)b * (float)(t - 1) * (float)P);
  const int nb = loss_blocks(n);
  hipLaunchKernelGGL(propagation_loss_kernel, dim3(nb), dim3(256), 0, st, x, t, P, n, k, dx, ws);
  hipLaunchKernelGGL(loss_finish_kernel, dim3(1), dim3(256), 0, st, ws, nb, k, loss);
  return check_launch("propagation_loss");
}

// NPRatio (losses.py:7-14) of x [b][t][P]; dx (optional) = d(loss)/dx.  ws: avt_loss_workspace_floats(n, b*t).
extern "C" int avt_npratio_loss(const float* x, int b, int t, int P, float* loss, float* dx, float* ws,
                                void* stream) {
  AVT_REQUIRE(x && loss && ws, "npratio_loss: null pointer");
  AVT_REQUIRE(b >= 1 && t >= 2 && P >= 1, "npratio_loss: need b >= 1, t >= 2, P >= 1 (b=%d t=%d P=%d)", b, t, P);
  hipStream_t st = (hipStream_t)stream;
  const int rows = b * t;
  const float k = 1.f / ((float)b * (float)(t - 1));
  float* S = ws + kLossMaxBlocks;
  const int rb = (int)((rows + 3) / 4 < 4096 ? (rows + 3) / 4 : 4096);  // 4 waves per block, one row each
  hipLaunchKernelGGL(npratio_rows_kernel, dim3(rb), dim3(256), 0, st, x, rows, P, S);
  const int nb = loss_blocks((long long)rows * P);
  hipLaunchKernelGGL(npratio_loss_kernel, dim3(nb), dim3(256), 0, st, S, rows, t, P, k, dx, ws);
  hipLaunchKernelGGL(loss_finish_kernel, dim3(1), dim3(256), 0, st, ws, nb, k, loss);
  return check_launch("npratio_loss");
}

// FlipLoss (losses.py:25-36): nn.L1Loss()(y, hflip(x)) over `rows` rows of W; dx / dy (optional) gradients.
extern "C" int avt_flip_l1_loss(const float* x, const float* y, long long rows, int W, float* loss, float* dx,
                                float* dy, float* ws, void* stream) {
  AVT_REQUIRE(x && y && loss && ws, "flip_l1_loss: null pointer");
  AVT_REQUIRE(rows >= 1 && W >= 1, "flip_l1_loss: empty input");
  hipStream_t st = (hipStream_t)stream;
  const long long n = rows * W;
  const float inv_n = 1.f / (float)n;
  const int nb = loss_blocks(n);
  hipLaunchKernelGGL(flip_l1_loss_kernel, dim3(nb), dim3(256), 0, st, x, y, n, W, inv_n, dx, dy, ws);
  hipLaunchKernelGGL(loss_finish_kernel, dim3(1), dim3(256), 0, st, ws, nb, inv_n, loss);
  return check_launch("flip_l1_loss");
}

