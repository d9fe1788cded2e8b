// Implicit-GEMM convolution for the ResNet-18 trunks (fwd, dgrad, wgrad) on gfx950 MFMA.
//
// Replaces the implicit cuDNN/MKLDNN Conv2d of models/base_models.py:23-30 (conv3x3/conv1x1),
// :135-138 (7x7/s2 stems) as called from BasicBlock.forward (:53-69) and _forward_impl (:195-210).
//
// Layout: activations NHWC bf16; weights packed bf16.  fp32 accumulate in MFMA AGPRs.
//   fwd   : C[m = (n,p,q)][k_out]      = sum_{(r,s,c)}  X[n, p*st-pad+r, q*st-pad+s, c] * W[k_out][(r,s,c)]
//   dgrad : C[m = (n,h,w)][c]          = sum_{(r,s,k)}  DY[n, (h+pad-r)/st, (w+pad-s)/st, k] * WT[c][(r,s,k)]
//   wgrad : DW[k_out][(r,s,c)]        += sum_{(n,p,q)}  DY[(n,p,q)][k_out] * X[n, p*st-pad+r, q*st-pad+s, c]
// fwd/dgrad ("NT"): both operands K-contiguous in LDS, fragments by ds_read_b128 (XOR-swizzled rows).
// wgrad ("TN"): both operands pixel-major in LDS, fragments by ds_read_b64_tr_b16 (hardware transpose).
// MFMA: v_mfma_f32_32x32x16_bf16, 4 waves (2x2) per 256-thread block, register-staged double buffer.
#include "avt_common.h"

namespace avt {

#include "conv_params.h"

template <int MODE, int CVEC, int BM, int BN>
__global__ __launch_bounds__(256) void gemm_nt_kernel(GemmNTParams p) {
  constexpr int TM = BM / 64, TN = BN / 64;  // 32x32 tiles per wave (waves 2x2)
  constexpr int AR = BM / 64, BR = BN / 64;  // staged rows per thread
  constexpr int STAGE_BYTES = 2 * (BM + BN) * 64;
  constexpr int CT_LD = BN + 8;  // epilogue tile row (bf16 elements)
  constexpr int EPI_BYTES = BM * CT_LD * 2;
  constexpr int SMEM = (STAGE_BYTES > EPI_BYTES ? STAGE_BYTES : EPI_BYTES);
  __shared__ __attribute__((aligned(16))) char smem[SMEM + 4 * BN * 4];
  float* red = reinterpret_cast<float*>(smem + SMEM);  // [2][2][BN] stats scratch

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid >> 1, wn = wid & 1;
  const int nnt = p.Ng / BN;
  const int mt = blockIdx.x / nnt, nt = blockIdx.x % nnt;
  const int m0 = mt * BM, n0 = nt * BN;

  // ---- per-thread load assignment: chunk (tid&3) of rows (tid>>2) + 64*i ----
  const int lchunk = tid & 3, lrow = tid >> 2;
  int a_pix[AR], a_y[AR], a_x[AR];
  bool a_ok[AR];
#pragma unroll
  for (int i = 0; i < AR; ++i) {
    const int m = m0 + lrow + 64 * i;
    a_ok[i] = m < p.M;
    const int mm = a_ok[i] ? m : 0;
    const int hw = p.OH * p.OW;
    const int n = mm / hw, rem = mm - n * hw;
    const int oh = rem / p.OW, ow = rem - oh * p.OW;
    a_pix[i] = n * p.IH * p.IW;
    if (MODE == MODE_FWD) {
      a_y[i] = oh * p.stride - p.pad;
      a_x[i] = ow * p.stride - p.pad;
    } else {
      a_y[i] = oh + p.pad;
      a_x[i] = ow + p.pad;
    }
  }
  const bf16_t* bptr[BR];
#pragma unroll
  for (int i = 0; i < BR; ++i) bptr[i] = p.wmat + (size_t)(n0 + lrow + 64 * i) * p.Kg + lchunk * 8;

  u32x4 ra[AR], rb[BR];
  const int nkt = p.Kg / 32;

  auto load_tile = [&](int kt) {
    const int k0 = kt * 32;
#pragma unroll
    for (int i = 0; i < BR; ++i) rb[i] = *reinterpret_cast<const u32x4*>(bptr[i] + k0);
    if (CVEC == 8) {
      const int rs = k0 / p.IC, c0 = k0 - rs * p.IC;
      const int r = rs / p.S, s = rs - r * p.S;
#pragma unroll
      for (int i = 0; i < AR; ++i) {
        int y, x;
        bool ok = a_ok[i];
        if (MODE == MODE_FWD) {
          y = a_y[i] + r;
          x = a_x[i] + s;
        } else {
          int yn = a_y[i] - r, xn = a_x[i] - s;
          if (p.stride == 2) {
            ok = ok && ((yn & 1) == 0) && ((xn & 1) == 0);
            yn >>= 1;
            xn >>= 1;
          }
          y = yn;
          x = xn;
        }
        ok = ok && y >= 0 && y < p.IH && x >= 0 && x < p.IW;
        u32x4 v = {0u, 0u, 0u, 0u};
        if (ok) v = *reinterpret_cast<const u32x4*>(p.act + (size_t)(a_pix[i] + y * p.IW + x) * p.IC + c0 + lchunk * 8);
        ra[i] = v;
      }
    } else {
      // stems: C == CVEC (1 or 4), k = (r*S + s)*C + c; positions beyond R*S are zero padding
      const int kc = k0 + lchunk * 8;
#pragma unroll
      for (int i = 0; i < AR; ++i) {
        unsigned short e[8];
#pragma unroll
        for (int g = 0; g < 8 / CVEC; ++g) {
          const int pos = (kc + g * CVEC) / CVEC;
          const int r = pos / p.S, s = pos - r * p.S;
          const int y = a_y[i] + r, x = a_x[i] + s;
          const bool ok = a_ok[i] && pos < p.R * p.S && y >= 0 && y < p.IH && x >= 0 && x < p.IW;
          const bf16_t* src = p.act + (size_t)(a_pix[i] + y * p.IW + x) * CVEC;
          if (CVEC == 4) {
            u32x2 v = {0u, 0u};
            if (ok) v = *reinterpret_cast<const u32x2*>(src);
            e[g * 4 + 0] = v.x & 0xffff;
            e[g * 4 + 1] = v.x >> 16;
            e[g * 4 + 2] = v.y & 0xffff;
            e[g * 4 + 3] = v.y >> 16;
          } else {
            e[g] = ok ? src[0] : (unsigned short)0;
          }
        }
        u32x4 v;
        v.x = e[0] | ((unsigned)e[1] << 16);
        v.y = e[2] | ((unsigned)e[3] << 16);
        v.z = e[4] | ((unsigned)e[5] << 16);
        v.w = e[6] | ((unsigned)e[7] << 16);
        ra[i] = v;
      }
    }
  };
  auto store_tile = [&](int buf) {
    char* As = smem + buf * (BM + BN) * 64;
    char* Bs = As + BM * 64;
#pragma unroll
    for (int i = 0; i < AR; ++i) *reinterpret_cast<u32x4*>(As + swz64(lrow + 64 * i, lchunk)) = ra[i];
#pragma unroll
    for (int i = 0; i < BR; ++i) *reinterpret_cast<u32x4*>(Bs + swz64(lrow + 64 * i, lchunk)) = rb[i];
  };

  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int v = 0; v < 16; ++v) acc[i][j][v] = 0.f;

  load_tile(0);
  store_tile(0);
  __syncthreads();
  const int frow = lane & 31, fhalf = lane >> 5;
  for (int kt = 0; kt < nkt; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nkt) load_tile(kt + 1);
    const char* As = smem + cur * (BM + BN) * 64;
    const char* Bs = As + BM * 64;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      bf16x8 af[TM], bfr[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int row = wm * (BM / 2) + i * 32 + frow;
        af[i] = *reinterpret_cast<const bf16x8*>(As + swz64(row, ks * 2 + fhalf));
      }
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int row = wn * (BN / 2) + j * 32 + frow;
        bfr[j] = *reinterpret_cast<const bf16x8*>(Bs + swz64(row, ks * 2 + fhalf));
      }
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
    if (kt + 1 < nkt) store_tile(cur ^ 1);
    __syncthreads();
  }

  // ---- epilogue: BN partial statistics over valid rows (fp32, before rounding) ----
  const int rows_valid = min(BM, p.M - m0);
  if (MODE == MODE_FWD && p.stats != nullptr) {
    float colsum[TN];
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      float s = 0.f;
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int v = 0; v < 16; ++v) {
          const int r = wm * (BM / 2) + i * 32 + (v & 3) + 8 * (v >> 2) + 4 * fhalf;
          if (r < rows_valid) s += acc[i][j][v];
        }
      s += __shfl_xor(s, 32, 64);
      colsum[j] = s;
      if (lane < 32) red[wm * BN + wn * (BN / 2) + j * 32 + lane] = s;
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int c = wn * (BN / 2) + j * 32 + frow;
      const float mean = (red[c] + red[BN + c]) / (float)rows_valid;
      float q = 0.f;
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int v = 0; v < 16; ++v) {
          const int r = wm * (BM / 2) + i * 32 + (v & 3) + 8 * (v >> 2) + 4 * fhalf;
          const float d = acc[i][j][v] - mean;
          if (r < rows_valid) q += d * d;
        }
      q += __shfl_xor(q, 32, 64);
      if (lane < 32) red[2 * BN + wm * BN + c] = q;
      (void)colsum;
    }
    __syncthreads();
    bn_write_header(p.stats, (p.M + BM - 1) / BM, 0, mt == 0 && n0 == 0);
    double* acc_slot = bn_fwd_slots(p.stats) + (size_t)mt * p.Ng * 3;  // this row tile's own slot
    for (int c = tid; c < BN; c += 256) {
      const double s = (double)red[c] + (double)red[BN + c];
      const double m2 = (double)red[2 * BN + c] + (double)red[3 * BN + c];
      double* a = acc_slot + (size_t)(n0 + c) * 3;
      a[0] = s;
      a[1] = m2;
      a[2] = s * s / (double)rows_valid;
    }
  }

  // ---- epilogue: bf16 tile through LDS, 16-byte coalesced stores ----
  bf16_t* Ct = reinterpret_cast<bf16_t*>(smem);
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int v = 0; v < 16; ++v) {
        const int r = wm * (BM / 2) + i * 32 + (v & 3) + 8 * (v >> 2) + 4 * fhalf;
        const int c = wn * (BN / 2) + j * 32 + frow;
        Ct[r * CT_LD + c] = f2bf(acc[i][j][v]);
      }
  __syncthreads();
  constexpr int CPR = BN / 8;  // 16-byte chunks per row
  for (int idx = tid; idx < BM * CPR; idx += 256) {
    const int r = idx / CPR, cc = idx - r * CPR;
    if (r >= rows_valid) continue;
    u32x4 v = *reinterpret_cast<const u32x4*>(Ct + r * CT_LD + cc * 8);
    const size_t off = (size_t)(m0 + r) * p.Ng + n0 + cc * 8;
    if (p.add != nullptr) {
      u32x4 a = *reinterpret_cast<const u32x4*>(p.add + off);
      unsigned* vv = reinterpret_cast<unsigned*>(&v);
      unsigned* aa = reinterpret_cast<unsigned*>(&a);
      if (p.amask != nullptr) {
        const unsigned bits = p.amask[off >> 3];
#pragma unroll
        for (int e = 0; e < 4; ++e)
          aa[e] &= ((bits >> (2 * e)) & 1u ? 0x0000ffffu : 0u) | ((bits >> (2 * e + 1)) & 1u ? 0xffff0000u : 0u);
      }
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float lo = bf2f(vv[e] & 0xffff) + bf2f(aa[e] & 0xffff);
        const float hi = bf2f(vv[e] >> 16) + bf2f(aa[e] >> 16);
        vv[e] = pack2(lo, hi);
      }
    }
    *reinterpret_cast<u32x4*>(p.out + off) = v;
  }
}

// ------------------------------------------------------------------------------------------------
// TN kernel (wgrad): DW[k_out][col] += sum_pix DY[pix][k_out] * X(pix, col)
// ------------------------------------------------------------------------------------------------

template <int CVEC, int BM, int BN>
__global__ __launch_bounds__(256) void gemm_tn_kernel(GemmTNParams p) {
  constexpr int TM = BM / 64, TN = BN / 64;
  constexpr int ALD = BM + 32, BLD = BN + 32;  // row strides (elements): +64 B keeps tr reads conflict-free
  constexpr int ACPR = BM / 8, BCPR = BN / 8;  // 16-B chunks per pixel row
  constexpr int AROWS = 32 * ACPR / 256, BROWS = 32 * BCPR / 256;  // rows staged per thread
  constexpr int ASTEP = 256 / ACPR, BSTEP = 256 / BCPR;
  constexpr int BUF = 32 * (ALD + BLD);  // elements per buffer
  __shared__ __attribute__((aligned(16))) bf16_t smem[2 * BUF];

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid >> 1, wn = wid & 1;
  const int nnt = p.Ng / BN;
  const int mt = blockIdx.x / nnt, nt = blockIdx.x % nnt;
  const int m0 = mt * BM, n0 = nt * BN;
  const int nkt_total = (p.Kred + 31) / 32;
  const int kt_begin = blockIdx.y * p.kt_per_split;
  const int kt_end = min(nkt_total, kt_begin + p.kt_per_split);
  if (kt_begin >= kt_end) return;

  const int a_chunk = tid % ACPR, a_row = tid / ACPR;
  const int b_chunk = tid % BCPR, b_row = tid / BCPR;
  // this thread's patch columns: col = n0 + 8*b_chunk + e
  const int colbase = n0 + 8 * b_chunk;
  int b_r = 0, b_s = 0, b_c = 0;
  if (CVEC == 8) {
    const int rs = colbase / p.Cp;
    b_c = colbase - rs * p.Cp;
    b_r = rs / p.S;
    b_s = rs - b_r * p.S;
  }
  const bool b_colok = colbase < p.R * p.S * p.Cp;
  const int PQ = p.P * p.Q;

  u32x4 ra[AROWS], rb[BROWS];
  auto load_tile = [&](int kt) {
    const int pix0 = kt * 32;
#pragma unroll
    for (int i = 0; i < AROWS; ++i) {
      const int pix = pix0 + a_row + ASTEP * i;
      u32x4 v = {0u, 0u, 0u, 0u};
      if (pix < p.Kred) v = *reinterpret_cast<const u32x4*>(p.dy + (size_t)pix * p.Mg + m0 + a_chunk * 8);
      ra[i] = v;
    }
#pragma unroll
    for (int i = 0; i < BROWS; ++i) {
      const int pix = pix0 + b_row + BSTEP * i;
      const bool pok = pix < p.Kred;
      const int pp = pok ? pix : 0;
      const int n = pp / PQ, rem = pp - n * PQ;
      const int oh = rem / p.Q, ow = rem - oh * p.Q;
      const int y0 = oh * p.stride - p.pad, x0 = ow * p.stride - p.pad;
      const bf16_t* img = p.x + (size_t)n * p.H * p.W * p.Cp;
      if (CVEC == 8) {
        const int y = y0 + b_r, x = x0 + b_s;
        u32x4 v = {0u, 0u, 0u, 0u};
        if (pok && b_colok && y >= 0 && y < p.H && x >= 0 && x < p.W)
          v = *reinterpret_cast<const u32x4*>(img + (size_t)(y * p.W + x) * p.Cp + b_c);
        rb[i] = v;
      } else {
        unsigned short e[8];
#pragma unroll
        for (int g = 0; g < 8 / CVEC; ++g) {
          const int pos = (colbase + g * CVEC) / CVEC;
          const int r = pos / p.S, s = pos - r * p.S;
          const int y = y0 + r, x = x0 + s;
          const bool ok = pok && pos < p.R * p.S && y >= 0 && y < p.H && x >= 0 && x < p.W;
          const bf16_t* src = img + (size_t)(y * p.W + x) * CVEC;
          if (CVEC == 4) {
            u32x2 v = {0u, 0u};
            if (ok) v = *reinterpret_cast<const u32x2*>(src);
            e[g * 4 + 0] = v.x & 0xffff;
            e[g * 4 + 1] = v.x >> 16;
            e[g * 4 + 2] = v.y & 0xffff;
            e[g * 4 + 3] = v.y >> 16;
          } else {
            e[g] = ok ? src[0] : (unsigned short)0;
          }
        }
        u32x4 v;
        v.x = e[0] | ((unsigned)e[1] << 16);
        v.y = e[2] | ((unsigned)e[3] << 16);
        v.z = e[4] | ((unsigned)e[5] << 16);
        v.w = e[6] | ((unsigned)e[7] << 16);
        rb[i] = v;
      }
    }
  };
  auto store_tile = [&](int buf) {
    bf16_t* As = smem + buf * BUF;
    bf16_t* Bs = As + 32 * ALD;
#pragma unroll
    for (int i = 0; i < AROWS; ++i) *reinterpret_cast<u32x4*>(As + (a_row + ASTEP * i) * ALD + a_chunk * 8) = ra[i];
#pragma unroll
    for (int i = 0; i < BROWS; ++i) *reinterpret_cast<u32x4*>(Bs + (b_row + BSTEP * i) * BLD + b_chunk * 8) = rb[i];
  };

  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int v = 0; v < 16; ++v) acc[i][j][v] = 0.f;

  // tr-read lane geometry: group g = lane>>4 (16 lanes), t = lane&15 = 4q + pp
  const int g = lane >> 4, t = lane & 15, q = t >> 2, pq = t & 3;
  const int tr_row = (g >> 1) * 8 + q;        // + 16*ks + 4*rr
  const int tr_col = (g & 1) * 16 + 4 * pq;   // + tile column base

  load_tile(kt_begin);
  store_tile(0);
  __syncthreads();
  for (int kt = kt_begin; kt < kt_end; ++kt) {
    const int cur = (kt - kt_begin) & 1;
    if (kt + 1 < kt_end) load_tile(kt + 1);
    typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
    const bf16_t* As = smem + cur * BUF;
    const bf16_t* Bs = As + 32 * ALD;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      bf16x8 af[TM], bfr[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int col = wm * (BM / 2) + i * 32 + tr_col;
        const bf16_t* a0 = As + (ks * 16 + tr_row) * ALD + col;
        s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(a0));
        s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(a0 + 4 * ALD));
        short tmp[8] = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        af[i] = __builtin_bit_cast(bf16x8, tmp);
      }
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int col = wn * (BN / 2) + j * 32 + tr_col;
        const bf16_t* b0 = Bs + (ks * 16 + tr_row) * BLD + col;
        s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(b0));
        s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(b0 + 4 * BLD));
        short tmp[8] = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        bfr[j] = __builtin_bit_cast(bf16x8, tmp);
      }
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
    if (kt + 1 < kt_end) store_tile(cur ^ 1);
    __syncthreads();
  }

  // ---- epilogue: fp32 atomics into DW[k_out][(r,s,c_real)] ----
  const int ldw = p.R * p.S * p.Creal;
  const int frow = lane & 31, fhalf = lane >> 5;
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int col = n0 + wn * (BN / 2) + j * 32 + frow;
    const int rs = col / p.Cp, c = col - rs * p.Cp;
    const bool cok = rs < p.R * p.S && c < p.Creal;
    const int dcol = rs * p.Creal + c;
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int v = 0; v < 16; ++v) {
        const int row = m0 + wm * (BM / 2) + i * 32 + (v & 3) + 8 * (v >> 2) + 4 * fhalf;
        if (cok && row < p.Mg) atomicAdd(p.dw + (size_t)row * ldw + dcol, acc[i][j][v]);
      }
  }
}

#include "conv_epi.h"
#include "conv_nt_pipe.h"
#include "conv_tn_pipe.h"
#include "conv_halo.h"
#include "conv_c64.h"
#include "conv_wgrad_halo.h"
#include "conv_stem.h"
#include "conv_stem_wgrad.h"

static int g_stem_kernel = -1;  // 7x7/s2 stem forwards on conv_stem_fwd_kernel: -1 = env AVT_STEM (default 1;
                                // 0 = the generic gather kernel, ~1.7x slower: tools/stem_bench.py)
static int stem_enabled() {
  if (g_stem_kernel < 0) {
    const char* e = getenv("AVT_STEM");
    g_stem_kernel = e ? atoi(e) : 1;
  }
  return g_stem_kernel;
}

static int g_stem_wgrad = -1;  // 7x7/s2 stem wgrads on conv_stem_wgrad_kernel: -1 = env AVT_STEM_WGRAD (default 1)
static int stem_wgrad_enabled() {
  if (g_stem_wgrad < 0) {
    const char* e = getenv("AVT_STEM_WGRAD");
    g_stem_wgrad = e ? atoi(e) : 1;
  }
  return g_stem_wgrad;
}

static int g_nt64_config = -1;  // tile config of the pipelined NT kernel for 64-wide GEMM N (A/B knob; -1 auto)
static int g_nt128_config = -1; // ... and for GEMM N % 128 == 0 (-1: by GEMM M, see launch_nt)
static int g_wgrad_blocks = 0;     // wgrad split-K: 0 = wave model (wgrad_plan), >0 = fixed block target
static int g_wgrad_min_kt = 4;
// largest split count that goes through a slab (deterministic: split partials summed in split order); beyond it
// fp32 atomics (non-deterministic summation order; an A/B knob only: AVT_WGRAD_SLAB_MAX / avt_set_wgrad_slab_max)
static int g_wgrad_slab_max = 1 << 30;
static int g_wgrad_wave_cost = 16; // per-block fixed cost (prologue fill + epilogue) in k-tiles
static int g_wgrad_big = -1;       // allow the 8-wave 256-wide wgrad tiles (-1: env AVT_WGRAD_BIG, default 1)
static int g_wgrad_nst = -1, g_wgrad_nst_big = -1;  // TN ring depth (4-wave / 8-wave tiles); -1: env
static int g_wgrad_slots_pct = -1;  // wgrad planner's slot share: 0 auto (by batch), 1-100 fixed, -1 env AVT_WGRAD_SLOTS_PCT
static int g_small_tile_pct = -2;  // 64-row fwd/dgrad tiles for small GEMMs (use_small_tile): % of the CUs; -2: env
static int g_wgrad_halo = -1;      // 3x3/s1 wgrad on the halo kernel (conv_wgrad_halo.h): 0 off, 1 nine taps per
                                   // block, 2 one filter row per block, 3 (default) the one-row form for K = 64
                                   // (layer 1: 480-550 -> 670-715 TFLOP/s), tap-gather elsewhere; -1 = env AVT_WGRAD_HALO
static int num_cus() {
  static int n = 0;
  if (n == 0) {
    int d = 0;
    hipDeviceProp_t pr;
    n = (hipGetDevice(&d) == hipSuccess && hipGetDeviceProperties(&pr, d) == hipSuccess && pr.multiProcessorCount > 0)
            ? pr.multiProcessorCount
            : 256;
  }
  return n;
}
static int g_halo = -1;  // 3x3/s1 fwd/dgrad on the halo-reuse kernel: -1 = env AVT_HALO (default 1)
static int halo_enabled() {
  if (g_halo < 0) {
    const char* e = getenv("AVT_HALO");
    g_halo = e ? atoi(e) : 1;
  }
  return g_halo;
}
// weight-ring stages of the layer3/4 halo tiles (A/B knobs): AVT_HALO_NST for the 128 x 128 tile (default 2:
// two blocks per CU; 3 = one block: B=128 layer3/4 -12..-20 %), AVT_HALO_SMALL_NST for the 64 x 128
// small-batch tile (default 3, still two blocks per CU: B=32 layer3 +3..16 %, vision layer4 +3..20 %;
// 4 and 5 leave one block per CU and lose; tools/conv_bench.py --stages)
static int g_halo_nst = -1, g_halo_small_nst = -1;  // -1: from the environment; avt_set_halo_stages
static int halo_nst() {
  if (g_halo_nst < 0) g_halo_nst = getenv("AVT_HALO_NST") ? atoi(getenv("AVT_HALO_NST")) : 2;
  return g_halo_nst;
}
static int halo_small_nst() {
  if (g_halo_small_nst < 0) g_halo_small_nst = getenv("AVT_HALO_SMALL_NST") ? atoi(getenv("AVT_HALO_SMALL_NST")) : 3;
  return g_halo_small_nst;
}
// the 8-wave 256 x 128 halo tile (one block per CU) in place of the 128 x 128 one where measured faster
// (tools/conv_bench.py --halo 1,2; B=128): layer4 (K = 4608: V +5..7 %, A +6..7 %; B=32 A +9 %) and GEMMs
// whose 256-row tiles fit one wave of blocks (vision layer3: +7..11 %); the audio layer3 GEMM
// (324 tiles, 1.3 waves) loses 13 %.  AVT_HALO8=0 keeps the 128 x 128 tile everywhere.
static int g_halo8 = -1;
static bool halo8_pick(const GemmNTParams& p) {
  if (g_halo8 < 0) g_halo8 = getenv("AVT_HALO8") ? atoi(getenv("AVT_HALO8")) : 1;
  if (!g_halo8) return false;
  if (p.IC >= 512) return true;
  // (A/B, env AVT_HALO8_PCT, default 100: the grid of 256-row tiles may reach that % of the CUs -- in the step the
  // other trunk's kernels fill a partial second round)
  static const int pct = getenv("AVT_HALO8_PCT") ? atoi(getenv("AVT_HALO8_PCT")) : 100;
  return (long)((p.M + 255) / 256) * (p.Ng / 128) * 100 <= (long)num_cus() * pct;
}
// weight-ring stages of the 8-wave 256 x 128 halo tile (A/B knob AVT_HALO8_NST: 3 default, or 4 -- the tile runs
// one block per CU either way, so a fourth stage is one more weight tile in flight for free LDS)
static int g_halo8_nst = -1;  // -1: env AVT_HALO8_NST (default 3)
static int halo8_nst() {
  if (g_halo8_nst < 0) g_halo8_nst = getenv("AVT_HALO8_NST") ? atoi(getenv("AVT_HALO8_NST")) : 3;
  return g_halo8_nst;
}
// wave layout of the 256 x 128 halo tile (A/B knob AVT_HALO8_FORM): 0 = 8 waves of 64 x 64 (TM = TN = 2: every
// fragment read feeds two MFMAs, 1 KB of LDS reads per MFMA), 1 = 4 waves of 128 x 64 (TM = 4, TN = 2: 0.75 KB per
// MFMA, one wave per SIMD with the whole register file)
static int g_halo8_form = -1;  // -1: env AVT_HALO8_FORM (default 0)
static int halo8_form() {
  if (g_halo8_form < 0) g_halo8_form = getenv("AVT_HALO8_FORM") ? atoi(getenv("AVT_HALO8_FORM")) : 0;
  return g_halo8_form;
}
static int g_c64 = -1;  // layer-1 (C = K = 64, 3x3/s1) fwd/dgrad on conv_c64_kernel: -1 = env AVT_C64 (default 1)
static int c64_enabled() {
  if (g_c64 < 0) {
    const char* e = getenv("AVT_C64");
    g_c64 = e ? atoi(e) : 1;
  }
  return g_c64;
}

static int g_s2_one = -1;  // stride-2 dgrad parity classes in one launch: -1 = env AVT_S2_ONE (default 1)
static int s2_one() {
  if (g_s2_one < 0) {
    const char* e = getenv("AVT_S2_ONE");
    g_s2_one = e ? atoi(e) : 1;
  }
  return g_s2_one;
}

static int g_conv_variant = -1;  // -1: read AVT_CONV_VARIANT once (0 = register-staged, 1 = LDS-DMA)
static int conv_variant() {
  if (g_conv_variant < 0) {
    const char* e = getenv("AVT_CONV_VARIANT");
    g_conv_variant = e ? atoi(e) : 1;
  }
  return g_conv_variant;
}

}  // namespace avt

using namespace avt;

extern "C" int avt_set_conv_variant(int v) {
  avt::g_conv_variant = v;
  return AVT_OK;
}

extern "C" int avt_set_c64(int on) {
  g_c64 = on ? 1 : 0;
  return AVT_OK;
}

extern "C" int avt_set_s2_dgrad_one(int on) {
  g_s2_one = on ? 1 : 0;
  return AVT_OK;
}

extern "C" int avt_set_halo(int on) {
  avt::g_halo = on < 0 ? 0 : (on > 2 ? 2 : on);
  return AVT_OK;
}

extern "C" int avt_set_halo8(int on) {
  avt::g_halo8 = on < 0 ? -1 : (on ? 1 : 0);
  return AVT_OK;
}

extern "C" int avt_set_halo_stages(int nst128, int nst64) {
  AVT_REQUIRE(nst128 >= 2 && nst128 <= 5 && nst64 >= 2 && nst64 <= 5, "set_halo_stages: nst128, nst64 in 2..5");
  avt::g_halo_nst = nst128;
  avt::g_halo_small_nst = nst64;
  return AVT_OK;
}

extern "C" int avt_set_nt64_config(int cfg) {
  AVT_REQUIRE(cfg >= -1 && cfg <= 8, "set_nt64_config: cfg in -1..8");
  g_nt64_config = cfg;
  return AVT_OK;
}

extern "C" int avt_set_nt128_config(int cfg) {
  AVT_REQUIRE(cfg >= -1 && cfg <= 6, "set_nt128_config: cfg=%d out of range", cfg);
  avt::g_nt128_config = cfg;
  return AVT_OK;
}

extern "C" int avt_set_wgrad_policy(int target_blocks, int min_ktiles) {
  AVT_REQUIRE(target_blocks >= 0 && min_ktiles >= 1, "set_wgrad_policy: bad arguments");
  avt::g_wgrad_blocks = target_blocks;
  avt::g_wgrad_min_kt = min_ktiles;
  return AVT_OK;
}

extern "C" int avt_set_wgrad_slab_max(int max_splits, int wave_cost) {
  AVT_REQUIRE(max_splits >= 0 && wave_cost >= 0, "set_wgrad_slab_max: bad arguments");
  avt::g_wgrad_slab_max = max_splits;
  avt::g_wgrad_wave_cost = wave_cost;
  return AVT_OK;
}

extern "C" int avt_set_stem_wgrad(int on) {
  avt::g_stem_wgrad = on ? 1 : 0;
  return AVT_OK;
}

extern "C" int avt_set_stem_kernel(int on) {
  avt::g_stem_kernel = on ? 1 : 0;
  return AVT_OK;
}

extern "C" int avt_set_small_tiles(int waves) {
  AVT_REQUIRE(waves >= -2 && waves <= 64, "avt_set_small_tiles: %d (blocks per CU; 0 never, -1 always, -2 env)", waves);
  avt::g_small_tile_pct = waves > 0 ? 100 * waves : waves;
  return AVT_OK;
}

extern "C" int avt_set_wgrad_tiles(int big) {
  avt::g_wgrad_big = big ? 1 : 0;
  return AVT_OK;
}

// TN wgrad ring depth: nst for the 4-wave tiles (4, 6 or 8), nst_big for the 8-wave 256 x 256 tile (3-5)
extern "C" int avt_set_wgrad_nst(int nst, int nst_big) {
  AVT_REQUIRE(nst >= 4 && nst <= 8 && nst_big >= 3 && nst_big <= 5, "set_wgrad_nst: nst in 4..8, nst_big in 3..5");
  avt::g_wgrad_nst = nst;
  avt::g_wgrad_nst_big = nst_big;
  return AVT_OK;
}

// share of the chip's block slots the tap-gather wgrad's split planner assumes: 0 auto (65 % at batch <= 32, 75 % at
// <= 64, else 100 %), 1-100 fixed, -1 back to env AVT_WGRAD_SLOTS_PCT.  Size workspaces after changing it.
extern "C" int avt_set_wgrad_slots_pct(int pct) {
  AVT_REQUIRE(pct >= -1 && pct <= 100, "avt_set_wgrad_slots_pct: %d (0 auto, 1-100 fixed, -1 env)", pct);
  avt::g_wgrad_slots_pct = pct;
  return AVT_OK;
}

// ------------------------------------------------------------------------------------------------
// C-ABI
// ------------------------------------------------------------------------------------------------
static inline int conv_out(int in, int k, int st, int pad) { return (in + 2 * pad - k) / st + 1; }

template <int MODE, int WM, int WN, int TM, int TN, int NST, int BK>
static void launch_pipe_one(const GemmNTParams& p, const NTPipeArgsV& ta0, hipStream_t st) {
  constexpr int BM = WM * TM * 32, BN = WN * TN * 32;
  const int grid = ((p.M + BM - 1) / BM) * (p.Ng / BN);
  if (grid <= 0) return;
  NTPipeArgsV ta = ta0;  // the output grid's row divisors (per parity class for a multi-class dgrad)
  ta.div_hw = make_magic((unsigned)(p.OH * p.OW));
  ta.div_ow = make_magic((unsigned)p.OW);
  for (int k = 0; k < 4; ++k) {
    const int ph = (ta.cls_meta[k] >> 8) & 1, pw = (ta.cls_meta[k] >> 9) & 1;
    const int oh = (ta.OHf - ph + 1) >> 1, ow = (ta.OWf - pw + 1) >> 1;
    ta.cdiv_hw[k] = make_magic((unsigned)(oh > 0 && ow > 0 ? oh * ow : 1));
    ta.cdiv_ow[k] = make_magic((unsigned)(ow > 0 ? ow : 1));
  }
  if (p.IT > 1 || p.OT > 1 || p.KT > 1 || ta.ntaps > 32) {  // Conv3d / the folded 49-tap video stem
    if constexpr (MODE == MODE_FWD)
      hipLaunchKernelGGL((conv_nt_pipe_kernel<MODE, WM, WN, TM, TN, NST, BK, true>), dim3(grid), dim3(WM * WN * 64), 0,
                         st, p, ta);
  } else if (MODE == MODE_DGRAD && p.bx != nullptr) {
    hipLaunchKernelGGL((conv_nt_pipe_kernel<MODE, WM, WN, TM, TN, NST, BK, false, true>), dim3(grid),
                       dim3(WM * WN * 64), 0, st, p, narrow_args(ta));
  } else {
    hipLaunchKernelGGL((conv_nt_pipe_kernel<MODE, WM, WN, TM, TN, NST, BK>), dim3(grid), dim3(WM * WN * 64), 0, st, p,
                       narrow_args(ta));
  }
}

// Builds the tap list(s) and launches: fwd / stride-1 dgrad in one launch; a stride-2 dgrad as
// four parity-class launches, each walking only its class's taps.
template <int MODE, int WM, int WN, int TM, int TN, int NST = 4, int BK = 32>
static void launch_glds(const GemmNTParams& p, hipStream_t st) {
  if (BK == 64 && p.IC % 64 != 0) {  // a 64-deep k-tile needs whole 64-channel taps
    launch_glds<MODE, 2, 2, 2, (WN * TN * 32) / 64, 3, 32>(p, st);  // 4-wave k32 tile of the same width
    return;
  }
  NTPipeArgsV ta{};
  const int batch = p.M / (p.OT * p.OH * p.OW);
  ta.act_bytes = (unsigned)((size_t)batch * p.IT * p.IH * p.IW * p.IC * 2);
  ta.w_bytes = (unsigned)((size_t)p.Ng * p.Kg * 2);
  if (MODE == MODE_FWD || p.stride == 1) {
    ta.ntaps = p.KT * p.R * p.S;
    for (int kt = 0; kt < p.KT; ++kt)
      for (int r = 0; r < p.R; ++r)
        for (int s = 0; s < p.S; ++s) {
          const int t = (kt * p.R + r) * p.S + s;
          ta.tap_w[t] = t;
          ta.tap_dt[t] = MODE == MODE_FWD ? kt - p.pad_t : p.pad_t - kt;
          ta.tap_dy[t] = MODE == MODE_FWD ? r - p.pad : p.pad - r;
          ta.tap_dx[t] = MODE == MODE_FWD ? s - p.pad : p.pad - s;
        }
    launch_pipe_one<MODE, WM, WN, TM, TN, NST, BK>(p, ta, st);
    return;
  }
  ta.cls = 1;
  ta.OHf = p.OH;
  ta.OWf = p.OW;
  // one launch for all classes (no BN-backward epilogue): blocks of the classes with the most taps
  // are dispatched first, and the classes' tails overlap instead of running as four short grids
  if (s2_one() && p.bx == nullptr && p.R * p.S <= 9) {
    struct Cls { int ph, pw, n, tiles; } cl[4];
    int ncl = 0;
    constexpr int BM = WM * TM * 32, BN = WN * TN * 32;
    for (int ph = 0; ph < 2; ++ph)
      for (int pw = 0; pw < 2; ++pw) {
        int n = 0;
        for (int r = 0; r < p.R; ++r)
          for (int s = 0; s < p.S; ++s) n += !(((ph + p.pad - r) & 1) || ((pw + p.pad - s) & 1));
        const int m = batch * ((p.OH - ph + 1) / 2) * ((p.OW - pw + 1) / 2);
        if (m == 0 || (n == 0 && p.add != nullptr && p.add == p.out)) continue;  // see below
        cl[ncl++] = Cls{ph, pw, n, ((m + BM - 1) / BM) * (p.Ng / BN)};
      }
    for (int i = 1; i < ncl; ++i)  // most taps first (stable)
      for (int j = i; j > 0 && cl[j].n > cl[j - 1].n; --j) std::swap(cl[j], cl[j - 1]);
    NTPipeArgsV tc = ta;
    tc.ncls = ncl;
    tc.batch = batch;
    tc.ntaps = 0;
    int start = 0;
    for (int k = 0; k < ncl; ++k) {
      const int first = tc.ntaps;
      for (int r = 0; r < p.R; ++r)
        for (int s = 0; s < p.S; ++s) {
          if (((cl[k].ph + p.pad - r) & 1) || ((cl[k].pw + p.pad - s) & 1)) continue;
          tc.tap_w[tc.ntaps] = r * p.S + s;
          tc.tap_dy[tc.ntaps] = (cl[k].ph + p.pad - r) / 2;
          tc.tap_dx[tc.ntaps] = (cl[k].pw + p.pad - s) / 2;
          ++tc.ntaps;
        }
      tc.cls_start[k] = start;
      tc.cls_meta[k] = cl[k].n | first << 4 | cl[k].ph << 8 | cl[k].pw << 9;
      start += cl[k].tiles;
    }
    if (ncl == 0 || start == 0) return;
    tc.ph = cl[0].ph;  // ncls == 1: the plain class mode (then tc.ntaps == cl[0].n)
    tc.pw = cl[0].pw;
    GemmNTParams pc = p;
    pc.OH = (p.OH - cl[0].ph + 1) / 2;
    pc.OW = (p.OW - cl[0].pw + 1) / 2;
    pc.M = batch * pc.OH * pc.OW;
    if (ncl > 1) pc.M = start / (p.Ng / BN) * BM;  // launch_pipe_one's grid = start; each block takes its class's M
    launch_pipe_one<MODE, WM, WN, TM, TN, NST, BK>(pc, tc, st);
    return;
  }
  // the class launches that carry the BN-backward epilogue store their partial sums into consecutive
  // slot ranges of one accumulator (conv_epi.h): pass 0 counts the call's slots, pass 1 launches
  constexpr int BMc = WM * TM * 32, BNc = WN * TN * 32;
  int ep_total = 0, ep_base = 0;
  for (int pass = 0; pass < 2; ++pass)
    for (int ph = 0; ph < 2; ++ph)
      for (int pw = 0; pw < 2; ++pw) {
        NTPipeArgsV tc = ta;
        tc.ph = ph;
        tc.pw = pw;
        tc.ntaps = 0;
        for (int r = 0; r < p.R; ++r)
          for (int s = 0; s < p.S; ++s) {
            if (((ph + p.pad - r) & 1) || ((pw + p.pad - s) & 1)) continue;
            tc.tap_w[tc.ntaps] = r * p.S + s;
            tc.tap_dy[tc.ntaps] = (ph + p.pad - r) / 2;
            tc.tap_dx[tc.ntaps] = (pw + p.pad - s) / 2;
            ++tc.ntaps;
          }
        GemmNTParams pc = p;
        if (p.bskip00 && ph == 0 && pw == 0) pc.bx = pc.bx2 = nullptr;
        pc.OH = (p.OH - ph + 1) / 2;
        pc.OW = (p.OW - pw + 1) / 2;
        pc.M = batch * pc.OH * pc.OW;
        // a class no tap reaches (e.g. 3 of the 4 classes of a 1x1/s2 downsample) runs with an empty
        // K loop: its rows are written as 0 (+ add) -- or, accumulating in place (add == out), are
        // already final and are skipped
        if (tc.ntaps == 0 && p.add != nullptr && p.add == p.out) continue;
        const int rtiles = (pc.M + BMc - 1) / BMc;  // the class's row tiles = its statistic slots
        if (rtiles * (p.Ng / BNc) <= 0) continue;
        if (pass == 0) {
          if (pc.bx != nullptr) ep_total += rtiles;
          continue;
        }
        pc.bslot_base = ep_base;
        pc.bslot_total = ep_total;
        if (pc.bx != nullptr) ep_base += rtiles;
        launch_pipe_one<MODE, WM, WN, TM, TN, NST, BK>(pc, tc, st);
      }
}

constexpr int kHaloPR = 416;  // patch rows the halo kernels' LDS holds: 256 + 2W + 2 <= 416 -> W <= 79

// 3x3 / stride 1 / pad 1 Conv2d, 64-channel multiples, image width <= 79: the halo-reuse kernel
static bool halo_eligible(const GemmNTParams& p) {
  const int h = halo_enabled();
  if (!h || p.R != 3 || p.S != 3 || p.stride != 1 || p.pad != 1 || p.IC % 64 != 0 || p.IT > 1 || p.OT > 1 || p.KT > 1 ||
      p.IH != p.OH || p.IW != p.OW)
    return false;
  if (h == 2) return 256 + 2 * p.OW + 2 <= kHaloPR && (p.Ng % 128 == 0 || p.Ng == 64);  // 8-wave forms (A/B)
  // W <= 19 (layer3/4): 4-wave 128x128; W <= 79 (layer2): 8-wave 256x128 (measured with the unrolled tap
  // loop: audio layer2 +6-10 % at B=128 and +28 % at B=32 over the tap gather, vision layer2 +0-6 %)
  static const int l2 = getenv("AVT_HALO_L2") ? atoi(getenv("AVT_HALO_L2")) : 1;  // A/B: 0 = layer2 on the tap gather
  return p.Ng % 128 == 0 && (128 + 2 * p.OW + 2 <= 168 || (l2 && 256 + 2 * p.OW + 2 <= kHaloPR));
}

// Small GEMMs (a few clips per GPU: BASELINE configs[2] runs 32 per GPU): a tile grid that leaves
// most of the 256 CUs idle loses more than a smaller tile's lower reuse costs.  Rows per tile drop
// from 128 to 64 when the 128-row grid would not give g_small_tile_pct % of the CUs a block.
// Measured per shape (tools/conv_bench.py --small): a 128-row grid of fewer blocks than CUs runs faster alone on
// 64-row tiles (e.g. B=32 layer3 263 -> 354 TFLOP/s), one of 1-2 blocks per CU does not (B=32 audio layer4 769 ->
// 541).  In the step the other trunk's kernels take the CUs a 128-row grid leaves: at 100 % (rounds 2-5) the
// 64-row tiles lost 1.6 % at B=32 and 0.5 % at B=64 against none, and gained 2.2 % on the tube step's 8-clip audio
// trunk (profiles/r6_ab_small_tiles*.txt); the default is AVT_SMALL_TILES_PCT (50).  avt_set_small_tiles(w) / env
// AVT_SMALL_TILES = w blocks per CU (100 w %), 0 never, -1 always.
static bool use_small_tile(const GemmNTParams& p, int BN) {
  if (g_small_tile_pct == -2) {
    const char* e = getenv("AVT_SMALL_TILES");
    const char* ep = getenv("AVT_SMALL_TILES_PCT");
    const int w = e ? atoi(e) : 1;
    g_small_tile_pct = e ? (w > 0 ? 100 * w : w) : ep ? atoi(ep) : 50;
  }
  if (g_small_tile_pct == 0) return false;
  if (g_small_tile_pct < 0) return true;
  const long long blocks128 = (long long)((p.M + 127) / 128) * (p.Ng / BN);
  return blocks128 * 100 < (long long)g_small_tile_pct * num_cus();
}

template <int MODE, int WM, int WN, int TM, int TN, int NSTB, int PRMAX, bool EPI, int OPT = 0>
static void launch_halo_one(const GemmNTParams& p, const HaloArgs& ha, int grid, hipStream_t st) {
  hipLaunchKernelGGL((conv_halo_kernel<MODE, WM, WN, TM, TN, NSTB, PRMAX, EPI, false, 0, OPT>), dim3(grid),
                     dim3(WM * WN * 64), 0, st, p, ha);
}

// OPT 4: the Conv3d 3x3x3 / stride 1 / pad 1 form (conv_halo.h; forward only)
template <int MODE, int WM, int WN, int TM, int TN, int NSTB = 3, int PRMAX = kHaloPR, int OPT = 0>
static void launch_halo(const GemmNTParams& p, hipStream_t st, int ksplit = 1, float* part = nullptr,
                        int* cnt = nullptr) {
  constexpr int BM = WM * TM * 32, BN = WN * TN * 32;
  HaloArgs ha{};
  ha.ksplit = ksplit;
  ha.cps = p.IC / 64 / ksplit;
#ifdef AVT_DIAG  // wrong-results timing diagnostics: the -DAVT_DIAG build only
  static const int hdbg = getenv("AVT_HALO_DBG") ? atoi(getenv("AVT_HALO_DBG")) : 0;
  ha.dbg = hdbg;
#endif
  ha.part = part;
  ha.cnt = cnt;
  const int batch = p.M / (p.OH * p.OW);
  ha.act_bytes = (unsigned)((size_t)batch * p.IH * p.IW * p.IC * 2);
  ha.w_bytes = (unsigned)((size_t)p.Ng * p.Kg * 2);
  ha.W = p.OW;
  ha.H = p.OH;
  for (int r = 0; r < 3; ++r)
    for (int s = 0; s < 3; ++s) {
      const int t = r * 3 + s;
      const int dy = MODE == MODE_FWD ? r - 1 : 1 - r, dx = MODE == MODE_FWD ? s - 1 : 1 - s;
      ha.tap_dy[t] = dy;
      ha.tap_dx[t] = dx;
      ha.tap_disp[t] = dy * p.OW + dx;
      ha.tap_w[t] = t;
    }
  if constexpr ((OPT & 4) != 0) {
    ha.T = p.IT;
    ha.div_hw = make_magic((unsigned)(p.OH * p.OW));
    ha.div_t = make_magic((unsigned)p.IT);
  }
  const int grid = ((p.M + BM - 1) / BM) * (p.Ng / BN) * ksplit;
  if (grid > 0 && ksplit > 1) {
    hipLaunchKernelGGL((conv_halo_kernel<MODE, WM, WN, TM, TN, NSTB, PRMAX, false, true>), dim3(grid),
                       dim3(WM * WN * 64), 0, st, p, ha);
    return;
  }
  if (grid <= 0) return;
  if constexpr ((OPT & 4) != 0)
    launch_halo_one<MODE, WM, WN, TM, TN, NSTB, PRMAX, false, OPT>(p, ha, grid, st);
  else if (MODE == MODE_DGRAD && p.bx != nullptr)
    launch_halo_one<MODE, WM, WN, TM, TN, NSTB, PRMAX, true, OPT>(p, ha, grid, st);
  else
    launch_halo_one<MODE, WM, WN, TM, TN, NSTB, PRMAX, false, OPT>(p, ha, grid, st);
}

// A/B knob: the 8-wave 256 x 128 halo tile with two taps per barrier and waves 4-7 at s_setprio 1 (conv_halo.h OPT 3)
// for the long-K convs (>= 8 (virtual) chunks: the 2-D layer4, C = 512; the Conv3d layer3/4).  +3..11 % per shape at
// B=128 in tools/halo_bench on random operands (profiles/r6_halo_bench_prio_tps2.txt), but +-0.1 % on the B=128 step
// (profiles/r6_ab_tps2_b128.txt) and +-2 % on the Conv3d shapes (r6_conv3d_halo.txt): off by default.
// avt_set_halo_tps2 / env AVT_HALO_TPS2 (0 default, 1 on; -1 back to the environment)
static int g_halo_tps2 = -1;
static int halo_tps2(const GemmNTParams& p, int vt = 1) {
  if (g_halo_tps2 < 0) g_halo_tps2 = getenv("AVT_HALO_TPS2") ? atoi(getenv("AVT_HALO_TPS2")) : 0;
  const int nv = p.IC / 64 * vt;
  return g_halo_tps2 && p.IC % 64 == 0 && nv % 2 == 0 && nv >= 8;
}

// Conv3d 3x3x3 / stride 1 / pad 1 with T' = T on the halo kernel's three-patch form: the R3D-18 layer2-4 convs (N %
// 128 == 0, W <= 79; 256 x 128 tile) and layer1 (N = 64, W <= 115; 256 x 64 tile).  Per shape at b=8 x 16 frames
// (profiles/r6_conv3d_halo.txt) 1094-1209 TFLOP/s against 886-928 for the tap gather on layer2-4, 789 against 549-635 on
// layer1.  avt_set_halo3d / env AVT_HALO3D: 2 (default) both, 1 layer2-4 only, 0 the tap-gather kernel
static int g_halo3d = -1;
static int halo3d_enabled() {
  if (g_halo3d < 0) g_halo3d = getenv("AVT_HALO3D") ? atoi(getenv("AVT_HALO3D")) : 2;
  return g_halo3d;
}
static bool halo3d_launch(const GemmNTParams& p, hipStream_t st) {
  if (!halo3d_enabled() || p.KT != 3 || p.R != 3 || p.S != 3 || p.stride != 1 || p.pad != 1 || p.pad_t != 1 ||
      p.IT != p.OT || p.IH != p.OH || p.IW != p.OW || p.IC % 64 != 0 || conv_variant() != 1)
    return false;
  if (p.Ng == 64) {  // R3D-18 layer1 (K = 64, W = 112): 256 x 64 on 8 waves of 32 x 64, a 488-row patch (W <= 115)
    if (halo3d_enabled() < 2 || 256 + 2 * p.OW + 2 > 488) return false;
    launch_halo<MODE_FWD, 8, 1, 1, 2, 3, 488, 4>(p, st);
    return true;
  }
  if (p.Ng % 128 != 0 || 256 + 2 * p.OW + 2 > kHaloPR) return false;
  if (256 + 2 * p.OW + 2 <= 336 && halo_tps2(p, 3))
    launch_halo<MODE_FWD, 4, 2, 2, 2, 2, 336, 7>(p, st);  // 256 x 128, 8 waves, W <= 39, two taps per barrier
  else if (256 + 2 * p.OW + 2 <= 336)
    launch_halo<MODE_FWD, 4, 2, 2, 2, 3, 336, 4>(p, st);  // 256 x 128, 8 waves, W <= 39
  else
    launch_halo<MODE_FWD, 4, 2, 2, 2, 2, kHaloPR, 4>(p, st);  // W <= 79: 2 weight stages to fit the 416-row patches
  return true;
}

// the 4-wave 128 x 128 halo tile by weight-ring depth (avt_set_halo_stages / AVT_HALO_NST): 2 stages (80 KB
// LDS, 2 blocks per CU; one 16 KiB weight stage in flight behind each step's 16 MFMAs per wave) or 3-5
// (96-128 KB, 1 block per CU; NSTB-1 stages in flight)
template <int MODE>
static void launch_halo128(const GemmNTParams& p, hipStream_t st, int ks = 1, float* part = nullptr,
                           int* cnt = nullptr) {
  switch (halo_nst()) {
    case 3: launch_halo<MODE, 2, 2, 2, 2, 3, 168>(p, st, ks, part, cnt); break;
    case 4: launch_halo<MODE, 2, 2, 2, 2, 4, 168>(p, st, ks, part, cnt); break;
    case 5: launch_halo<MODE, 2, 2, 2, 2, 5, 168>(p, st, ks, part, cnt); break;
    default: launch_halo<MODE, 2, 2, 2, 2, 2, 168>(p, st, ks, part, cnt); break;
  }
}

// ---- split-K for the 128 x 128 halo tile (layer3/4 at a few clips per GPU) ----
// A 128-row grid of fewer blocks than the chip holds leaves CUs idle, and the 64-row tile that fills
// it moves twice the weight bytes per FLOP through L2 -> LDS.  Split-K keeps the 128 x 128 tile and
// gives each of `ksplit` blocks per tile a range of the 64-channel chunks; the last block to finish a
// tile sums the fp32 partials (conv_halo.h).  Plan: ksplit = the smallest divisor of the chunk count
// whose grid reaches g_splitk_blocks (AVT_SPLITK_BLOCKS, default 2 blocks per CU); AVT_HALO_SPLITK /
// avt_set_halo_splitk(s > 0) forces the largest divisor <= s, 1 turns it off.
static int g_halo_splitk = -1, g_splitk_blocks = -1;
struct SplitWs {
  float* part;
  int* cnt;
  long long part_floats;  // sizes the caller allocated (avt_conv2d_splitk_plan at the time of the call)
  int counters;
};
static bool halo_splitk_shape(const GemmNTParams& p) {
  return halo_eligible(p) && conv_variant() == 1 && p.Ng % 128 == 0 && 128 + 2 * p.OW + 2 <= 168 &&
         p.bx == nullptr;
}
static int halo_splitk(const GemmNTParams& p) {
  if (g_halo_splitk < 0) g_halo_splitk = getenv("AVT_HALO_SPLITK") ? atoi(getenv("AVT_HALO_SPLITK")) : 0;
  if (g_splitk_blocks < 0)
    g_splitk_blocks = getenv("AVT_SPLITK_BLOCKS") ? atoi(getenv("AVT_SPLITK_BLOCKS")) : 2 * num_cus();
  if (!halo_splitk_shape(p)) return 1;
  const int nchunk = p.IC / 64;
  const long long tiles = (long long)((p.M + 127) / 128) * (p.Ng / 128);
  if (g_halo_splitk > 0) {
    int s = 1;
    for (int d = 1; d <= nchunk && d <= g_halo_splitk; ++d)
      if (nchunk % d == 0) s = d;
    return s;
  }
  if (tiles >= g_splitk_blocks) return 1;
  int s = 1;
  for (int d = 2; d <= nchunk; ++d)
    if (nchunk % d == 0) {
      s = d;
      if (tiles * d >= g_splitk_blocks) break;
    }
  return s;
}

// C = K = 64 3x3/s1/p1 Conv2d (the layer-1 convs), image width <= 95, not a BN-epilogue dgrad and not
// in-place: the persistent resident-weight kernel (conv_c64.h); off with the halo kernels (halo 0: the
// tap-gather kernel everywhere, as the bitwise-order tests need) or avt_set_c64(0)
static bool c64_eligible(const GemmNTParams& p) {
  return c64_enabled() && halo_enabled() && conv_variant() == 1 && p.IC == 64 && p.Ng == 64 && p.Kg == 576 &&
         p.R == 3 && p.S == 3 && p.stride == 1 && p.pad == 1 && p.IT == 1 && p.OT == 1 && p.KT == 1 && p.IH == p.OH &&
         p.IW == p.OW && 256 + 2 * p.OW + 2 <= c64::PRMAX && p.bx == nullptr && (p.add == nullptr || p.add != p.out);
}

template <int MODE>
static void launch_c64(const GemmNTParams& p, hipStream_t st) {
  C64Args ca{};
  const int batch = p.M / (p.OH * p.OW);
  ca.act_bytes = (unsigned)((size_t)batch * p.IH * p.IW * 64 * 2);
  ca.w_bytes = (unsigned)((size_t)64 * 576 * 2);
  ca.W = p.OW;
  ca.H = p.OH;
  ca.tiles = (p.M + c64::BM - 1) / c64::BM;
#ifdef AVT_DIAG  // wrong-results timing diagnostics: the -DAVT_DIAG build only
  static const int dbg = getenv("AVT_C64_DBG") ? atoi(getenv("AVT_C64_DBG")) : 0;
  ca.dbg = dbg;
#else
  ca.dbg = 0;
#endif
  for (int r = 0; r < 3; ++r)
    for (int s = 0; s < 3; ++s) {
      const int t = r * 3 + s;
      const int dy = MODE == MODE_FWD ? r - 1 : 1 - r, dx = MODE == MODE_FWD ? s - 1 : 1 - s;
      ca.tap_dy[t] = dy;
      ca.tap_dx[t] = dx;
    }
  // as few blocks as the same number of tile rounds needs (1568 vision tiles at B=128: 7 rounds on 224
  // blocks, not 6.1 on 256): the CUs left over take the other trunk's concurrent kernels
  // (A/B, env AVT_C64_SHARE, default 100: the share of the CUs the persistent grid may take -- the rest run the
  // other trunk's kernels)
  static const int c64_share = getenv("AVT_C64_SHARE") ? atoi(getenv("AVT_C64_SHARE")) : 100;
  const int cus = max(1, num_cus() * min(max(c64_share, 1), 100) / 100);
  const int rounds = (ca.tiles + cus - 1) / cus;
  const int grid = rounds > 0 ? (ca.tiles + rounds - 1) / rounds : 0;
  if (grid <= 0) return;
  // 8-wave blocks (two waves per SIMD; default): layer-1 fwd/dgrad 519/630 -> 638/762 TFLOP/s (vision), step
  // 12.61 k -> 12.86 k clips/s in the same-box A/B; AVT_C64_WAVES=4: the 4-wave form
  static const int w8 = !(getenv("AVT_C64_WAVES") && atoi(getenv("AVT_C64_WAVES")) == 4);
  if constexpr (MODE == MODE_DGRAD) {
    if (p.add != nullptr && p.amask != nullptr) {
      if (w8)
        hipLaunchKernelGGL((conv_c64_kernel<MODE, 2, 8>), dim3(grid), dim3(512), 0, st, p, ca);
      else
        hipLaunchKernelGGL((conv_c64_kernel<MODE, 2>), dim3(grid), dim3(256), 0, st, p, ca);
      return;
    }
    if (p.add != nullptr) {
      if (w8)
        hipLaunchKernelGGL((conv_c64_kernel<MODE, 1, 8>), dim3(grid), dim3(512), 0, st, p, ca);
      else
        hipLaunchKernelGGL((conv_c64_kernel<MODE, 1>), dim3(grid), dim3(256), 0, st, p, ca);
      return;
    }
  }
  if (w8)
    hipLaunchKernelGGL((conv_c64_kernel<MODE, 0, 8>), dim3(grid), dim3(512), 0, st, p, ca);
  else
    hipLaunchKernelGGL((conv_c64_kernel<MODE, 0>), dim3(grid), dim3(256), 0, st, p, ca);
}

template <int MODE, int CVEC, int BM, int BN>
static void launch_nt(const GemmNTParams& p, hipStream_t st, const SplitWs* ws = nullptr) {
  if (CVEC == 8 && c64_eligible(p)) {
    launch_c64<MODE>(p, st);
    return;
  }
  if (CVEC == 8 && ws != nullptr && p.IT == 1 && p.OT == 1 && p.KT == 1) {
    const int ks = halo_splitk(p);
    const long long tiles = (long long)((p.M + 127) / 128) * (p.Ng / 128);
    // the plan is re-made at every call from the current knobs: a workspace sized for another plan
    // (the knobs changed after it was allocated) runs the shape without split-K rather than overrun it
    if (ks > 1 && tiles * ks * 128 * 128 <= ws->part_floats && tiles <= ws->counters) {
      launch_halo128<MODE>(p, st, ks, ws->part, ws->cnt);
      return;
    }
  }
  if (CVEC == 8 && conv_variant() == 1 && p.IT == 1 && p.OT == 1 && p.KT == 1 && g_nt128_config < 0 && (g_nt64_config < 0 || g_nt64_config == 1) &&
      p.bx == nullptr && use_small_tile(p, p.Ng % 128 == 0 ? 128 : 64)) {
    if (p.Ng % 128 == 0) {
      if (halo_eligible(p) && 64 + 2 * p.OW + 2 <= 104) {  // 64 x 128 halo tile
        switch (halo_small_nst()) {
          case 3: launch_halo<MODE, 2, 2, 1, 2, 3, 104>(p, st); break;
          case 4: launch_halo<MODE, 2, 2, 1, 2, 4, 104>(p, st); break;
          case 5: launch_halo<MODE, 2, 2, 1, 2, 5, 104>(p, st); break;
          default: launch_halo<MODE, 2, 2, 1, 2, 2, 104>(p, st); break;
        }
      }
      else
        launch_glds<MODE, 2, 2, 1, 2, 3>(p, st);  // 64 x 128, k32, 3 stages
    } else {
      launch_glds<MODE, 2, 2, 1, 1, 3>(p, st);  // 64 x 64, k32, 3 stages
    }
    return;
  }
  if (CVEC == 8 && conv_variant() == 1 && halo_eligible(p)) {
    // measured (tools/conv_bench.py): the 4-wave 128 x 128 form at 2 blocks per CU beats the tap
    // gather on layer3/4 (W <= 19: +2..16 %); the 8-wave 256-row forms a patch of the wider layer1/2
    // images needs (1 block per CU) lose to it (-1..-20 %), so those keep the tap-gather kernel
    if (p.Ng % 128 == 0 && (g_halo == 2 || 128 + 2 * p.OW + 2 > 168 || halo8_pick(p))) {
      if (256 + 2 * p.OW + 2 <= 336) {
        if (halo8_form() == 1)
          launch_halo<MODE, 2, 2, 4, 2, 3, 336>(p, st);  // same tile on 4 waves of 128 x 64 (0.75 KB LDS per MFMA)
        else if (halo8_nst() == 4)
          launch_halo<MODE, 4, 2, 2, 2, 4, 336>(p, st);  // 4-stage weight ring: 150 KB of LDS, still 1 block/CU
        else if (halo_tps2(p))
          launch_halo<MODE, 4, 2, 2, 2, 2, 336, 3>(p, st);  // ... two taps per barrier (layer4)
        else
          launch_halo<MODE, 4, 2, 2, 2, 3, 336>(p, st);  // 256 x 128, 8 waves, W <= 39 (layer2)
      }
      else
        launch_halo<MODE, 4, 2, 2, 2, 2>(p, st);  // W <= 79: 2 weight stages to fit the 416-row patches
    }
    else if (g_halo == 2)
      launch_halo<MODE, 4, 2, 2, 1>(p, st);  // 256 x 64, 8 waves (A/B only)
    else
      launch_halo128<MODE>(p, st);  // 128 x 128, 4 waves
    return;
  }
  if (CVEC == 8 && conv_variant() == 1) {
    if (p.Ng % 128 == 0) {
      // default: 256-row tiles (8 waves) where the GEMM is tall enough to fill the chip with them
      // (layer2, the stride-2 convs), 128 x 128 k64 tiles for the short layer3/4 GEMMs
      // Conv3d (27 taps: 3x the K of a 3x3) keeps the 128 x 128 k64 tile unless K is short: on the R3D-18
      // trunk (tools/conv3d_bench.py, profiles/r5_conv3d_tiles.txt) it is 10-15 % faster than the 256-row
      // form on layer2/3's 3x3x3 convs; at layer2.0's K = 1728 the two are within 3 %
      const bool vid = p.IT > 1 || p.OT > 1 || p.KT > 1;
      const int cfg = g_nt128_config >= 0 ? g_nt128_config : (p.M >= 65536 && (!vid || p.Kg < 3072) ? 6 : 1);
      switch (cfg) {
        case 1: launch_glds<MODE, 2, 2, 2, 2, 2, 64>(p, st); break;  // 128 x 128, k64, 2 stages
        case 2: launch_glds<MODE, 2, 2, 2, 2, 3, 64>(p, st); break;  // 128 x 128, k64, 3 stages
        case 3: launch_glds<MODE, 2, 2, 4, 2, 3>(p, st); break;      // 256 x 128, k32, 3 stages
        case 4: launch_glds<MODE, 2, 2, 4, 2, 2, 64>(p, st); break;  // 256 x 128, k64, 2 stages
        case 5: launch_glds<MODE, 4, 2, 2, 2, 2, 64>(p, st); break;  // 256 x 128, 8 waves, k64, 2 stages
        case 6: launch_glds<MODE, 4, 2, 2, 2, 3>(p, st); break;      // 256 x 128, 8 waves, k32, 3 stages
        default: launch_glds<MODE, 2, 2, 2, 2>(p, st); break;        // 128 x 128, k32, 4 stages
      }
    } else {  // 64-wide N (layer1 / stem-fed convs)
      // auto (-1): 1, or 2 (4 stages) for a Conv3d -- R3D-18 layer1, profiles/r5_conv3d_tiles.txt: 548-579 us
      // against 557-683 us per conv, ahead in every ordering measured
      switch (g_nt64_config >= 0 ? g_nt64_config : (p.IT > 1 || p.OT > 1 || p.KT > 1 ? 2 : 1)) {
        case 0: launch_glds<MODE, 4, 1, 2, 2, 4>(p, st); break;  // 256 x 64, 4 stages
        case 2: launch_glds<MODE, 2, 2, 2, 1, 4>(p, st); break;  // 128 x 64, 4 stages
        case 3: launch_glds<MODE, 4, 1, 2, 2, 2>(p, st); break;  // 256 x 64, 2 stages
        case 4: launch_glds<MODE, 2, 2, 2, 1, 3, 64>(p, st); break;  // 128 x 64, k64, 3 stages
        case 5: launch_glds<MODE, 4, 1, 2, 2, 2, 64>(p, st); break;  // 256 x 64, k64, 2 stages
        case 6: launch_glds<MODE, 2, 2, 2, 1, 2, 64>(p, st); break;  // 128 x 64, k64, 2 stages
        case 7: launch_glds<MODE, 4, 2, 2, 1, 3, 64>(p, st); break;  // 256 x 64, 8 waves, k64, 3 stages
        case 8: launch_glds<MODE, 4, 2, 2, 1, 2, 64>(p, st); break;  // 256 x 64, 8 waves, k64, 2 stages
        default: launch_glds<MODE, 2, 2, 2, 1, 3>(p, st); break;  // 128 x 64, 3 stages
      }
    }
    return;
  }
  const int grid = ((p.M + BM - 1) / BM) * (p.Ng / BN);
  hipLaunchKernelGGL((gemm_nt_kernel<MODE, CVEC, BM, BN>), dim3(grid), dim3(256), 0, st, p);
}


static int conv2d_fwd_impl(const void* x, const void* wpack, void* y, double* bn_acc, int N, int H, int W, int Cp,
                           int K, int R, int S, int stride, int pad, int Kg, const SplitWs* ws, void* stream);

extern "C" int avt_conv2d_fwd(const void* x, const void* wpack, void* y, double* bn_acc, int N, int H, int W,
                              int Cp, int K, int R, int S, int stride, int pad, int Kg, void* stream) {
  return conv2d_fwd_impl(x, wpack, y, bn_acc, N, H, W, Cp, K, R, S, stride, pad, Kg, nullptr, stream);
}

// split-K workspace of a 3x3/s1 conv (halo kernel): *part_floats fp32 partials, *counters ints (zero
// before the first launch; the kernel leaves them zero).  Both 0: the shape runs without split-K.
extern "C" int avt_conv2d_splitk_plan(int N, int H, int W, int C, int K, int R, int S, int stride, int pad, int dgrad,
                                      long long* part_floats, int* counters) {
  AVT_REQUIRE(part_floats && counters, "conv2d_splitk_plan: null pointer");
  *part_floats = 0;
  *counters = 0;
  GemmNTParams p{};
  p.IT = p.OT = p.KT = 1;
  p.R = R; p.S = S; p.stride = stride; p.pad = pad;
  if (dgrad) {
    p.IH = conv_out(H, R, stride, pad); p.IW = conv_out(W, S, stride, pad); p.IC = K;
    p.OH = H; p.OW = W; p.Ng = C;
  } else {
    p.IH = H; p.IW = W; p.IC = C;
    p.OH = conv_out(H, R, stride, pad); p.OW = conv_out(W, S, stride, pad); p.Ng = K;
  }
  p.M = N * p.OH * p.OW;
  if (p.IC % 64 != 0 || p.Ng % 64 != 0 || p.M <= 0) return AVT_OK;
  const int ks = halo_splitk(p);
  if (ks <= 1) return AVT_OK;
  const int tiles = ((p.M + 127) / 128) * (p.Ng / 128);
  *part_floats = (long long)tiles * ks * 128 * 128;
  *counters = tiles;
  return AVT_OK;
}

extern "C" int avt_set_halo8_nst(int nst) {
  AVT_REQUIRE(nst == -1 || nst == 3 || nst == 4, "set_halo8_nst: -1, 3 or 4");
  avt::g_halo8_nst = nst;  // -1: back to the environment default
  return AVT_OK;
}

extern "C" int avt_set_halo8_form(int form) {
  AVT_REQUIRE(form >= -1 && form <= 1, "set_halo8_form: -1, 0 or 1");
  avt::g_halo8_form = form;  // -1: back to the environment default
  return AVT_OK;
}

extern "C" int avt_set_halo_splitk(int ksplit, int target_blocks) {
  AVT_REQUIRE(ksplit >= 0 && target_blocks >= 0, "set_halo_splitk: bad arguments");
  g_halo_splitk = ksplit;
  g_splitk_blocks = target_blocks > 0 ? target_blocks : 2 * num_cus();
  return AVT_OK;
}

extern "C" int avt_conv2d_fwd_ws(const void* x, const void* wpack, void* y, double* bn_acc, int N, int H, int W,
                                 int Cp, int K, int R, int S, int stride, int pad, int Kg, float* part,
                                 long long part_floats, int* cnt, int counters, void* stream) {
  AVT_REQUIRE(part_floats >= 0 && counters >= 0, "conv2d_fwd_ws: negative workspace size");
  const SplitWs ws{part, cnt, part_floats, counters};
  return conv2d_fwd_impl(x, wpack, y, bn_acc, N, H, W, Cp, K, R, S, stride, pad, Kg, (part && cnt) ? &ws : nullptr,
                         stream);
}

static int conv2d_fwd_impl(const void* x, const void* wpack, void* y, double* bn_acc, int N, int H, int W, int Cp,
                           int K, int R, int S, int stride, int pad, int Kg, const SplitWs* ws, void* stream) {
  AVT_REQUIRE(x && wpack && y, "conv2d_fwd: null pointer");
  AVT_REQUIRE(K % 64 == 0, "conv2d_fwd: K=%d must be a multiple of 64", K);
  AVT_REQUIRE(Kg % 32 == 0 && Kg >= R * S * Cp, "conv2d_fwd: Kg=%d must be a multiple of 32 >= R*S*C", Kg);
  AVT_REQUIRE(Cp % 32 == 0 || Cp == 4 || Cp == 1, "conv2d_fwd: C=%d unsupported (need %%32, or stem 1/4)", Cp);
  AVT_REQUIRE(Cp % 32 != 0 || Kg == R * S * Cp, "conv2d_fwd: Kg must equal R*S*C for C%%32==0");
  AVT_REQUIRE(Cp % 32 != 0 || R * S <= kMaxTaps, "conv2d_fwd: at most %d taps for C%%32==0", kMaxTaps);
  AVT_REQUIRE(stride == 1 || stride == 2, "conv2d_fwd: stride must be 1 or 2");
  GemmNTParams p{};
  p.act = (const bf16_t*)x;
  p.wmat = (const bf16_t*)wpack;
  p.out = (bf16_t*)y;
  p.add = nullptr;
  p.stats = bn_acc;
  p.IH = H; p.IW = W; p.IC = Cp;
  p.OH = conv_out(H, R, stride, pad);
  p.OW = conv_out(W, S, stride, pad);
  p.IT = p.OT = p.KT = 1;
  p.pad_t = 0;
  p.M = N * p.OH * p.OW;
  AVT_REQUIRE((size_t)N * H * W * Cp * 2 < (1ull << 31) && (size_t)p.M * K * 2 < (1ull << 31),
              "conv2d_fwd: activation tensors must stay below 2 GiB (32-bit buffer offsets)");
  p.Ng = K;
  p.Kg = Kg;
  p.R = R; p.S = S; p.stride = stride; p.pad = pad;
  hipStream_t st = (hipStream_t)stream;
  if ((Cp == 4 || Cp == 1) && stem_enabled() && K == 64 && R == 7 && S == 7 && stride == 2 && pad == 3 &&
      (Cp == 4 ? stem_fits<4>(p.OW) : stem_fits<1>(p.OW))) {
    StemArgs sa{};
    sa.x = p.act;
    sa.w = p.wmat;
    sa.y = p.out;
    sa.stats = bn_acc;
    sa.x_bytes = (unsigned)((size_t)N * H * W * Cp * 2);
    sa.y_bytes = (unsigned)((size_t)p.M * K * 2);
    sa.N = N;
    sa.IH = H; sa.IW = W; sa.OH = p.OH; sa.OW = p.OW; sa.Kg = Kg;
    sa.tiles_per_row = (p.OW + 31) / 32;
    sa.total_tiles = N * p.OH * sa.tiles_per_row;
    const int blocks = (sa.total_tiles + kStemNW - 1) / kStemNW;  // kStemNW wave tiles per block round
    const int grid = blocks < num_cus() ? blocks : num_cus();
    const size_t lds = Cp == 4 ? stem_lds_bytes<4>() : stem_lds_bytes<1>();
    if (Cp == 4)
      hipLaunchKernelGGL(conv_stem_fwd_kernel<4>, dim3(grid), dim3(kStemNW * 64), lds, st, sa);
    else
      hipLaunchKernelGGL(conv_stem_fwd_kernel<1>, dim3(grid), dim3(kStemNW * 64), lds, st, sa);
    return check_launch("conv2d_fwd (stem)");
  }
  const bool bn128 = (K % 128 == 0);
  if (Cp == 4) {
    launch_nt<MODE_FWD, 4, 128, 64>(p, st);
  } else if (Cp == 1) {
    launch_nt<MODE_FWD, 1, 128, 64>(p, st);
  } else if (bn128) {
    launch_nt<MODE_FWD, 8, 128, 128>(p, st, ws);
  } else {
    launch_nt<MODE_FWD, 8, 128, 64>(p, st);
  }
  return check_launch("conv2d_fwd");
}

static int conv2d_dgrad_impl(const void* dy, const void* wt, void* dx, const void* add, const void* add_mask, int N,
                             int H, int W, int C, int K, int R, int S, int stride, int pad, const avt_dgrad_bn_epi* epi,
                             void* stream, const SplitWs* ws = nullptr) {
  AVT_REQUIRE(dy && wt && dx, "conv2d_dgrad: null pointer");
  AVT_REQUIRE(epi == nullptr || (epi->xc && epi->stats && epi->acc), "conv2d_dgrad: epilogue needs xc, stats, acc");
  AVT_REQUIRE(epi == nullptr || epi->xc2 == nullptr || (epi->stats2 && epi->acc2),
              "conv2d_dgrad: second BN needs stats2 and acc2");
  AVT_REQUIRE(epi == nullptr || ((uintptr_t)epi->acc & 7) == 0, "conv2d_dgrad: acc must be 8-byte aligned");
  // only the LDS-DMA kernels write the epilogue's slots and header; the register-staged gemm_nt_kernel ignores it
  AVT_REQUIRE(epi == nullptr || conv_variant() == 1,
              "conv2d_dgrad: the BatchNorm-backward epilogue needs the LDS-DMA kernels (avt_set_conv_variant(1))");
  AVT_REQUIRE(C % 64 == 0 && K % 32 == 0, "conv2d_dgrad: C=%d K=%d unsupported", C, K);
  AVT_REQUIRE(stride == 1 || stride == 2, "conv2d_dgrad: stride must be 1 or 2");
  AVT_REQUIRE(R * S <= 32, "conv2d_dgrad: at most 32 taps");
  GemmNTParams p{};
  p.act = (const bf16_t*)dy;
  p.wmat = (const bf16_t*)wt;
  p.out = (bf16_t*)dx;
  p.add = (const bf16_t*)add;
  p.amask = (const unsigned char*)add_mask;
  p.stats = nullptr;
  p.IH = conv_out(H, R, stride, pad);
  p.IW = conv_out(W, S, stride, pad);
  p.IC = K;
  p.OH = H; p.OW = W;
  p.IT = p.OT = p.KT = 1;
  p.pad_t = 0;
  p.M = N * H * W;
  AVT_REQUIRE((size_t)p.M * C * 2 < (1ull << 31) && (size_t)N * p.IH * p.IW * K * 2 < (1ull << 31),
              "conv2d_dgrad: activation tensors must stay below 2 GiB (32-bit buffer offsets)");
  p.Ng = C;
  p.Kg = R * S * K;
  p.R = R; p.S = S; p.stride = stride; p.pad = pad;
  if (epi != nullptr) {
    p.bx = (const bf16_t*)epi->xc;
    p.by = (const bf16_t*)epi->y;
    p.bst = epi->stats;
    p.bacc = epi->acc;
    p.bx2 = (const bf16_t*)epi->xc2;
    p.bst2 = epi->stats2;
    p.bacc2 = epi->acc2;
    p.bskip00 = epi->skip_class00;
    p.bappend = epi->append_slots ? 1 : 0;
  }
  hipStream_t st = (hipStream_t)stream;
  if (C % 128 == 0)
    launch_nt<MODE_DGRAD, 8, 128, 128>(p, st, ws);
  else
    launch_nt<MODE_DGRAD, 8, 128, 64>(p, st);
  return check_launch("conv2d_dgrad");
}

// avt_conv2d_dgrad / avt_conv2d_dgrad_mask (add_mask optional) with a split-K workspace
extern "C" int avt_conv2d_dgrad_ws(const void* dy, const void* wt, void* dx, const void* add, const void* add_mask,
                                   int N, int H, int W, int C, int K, int R, int S, int stride, int pad, float* part,
                                   long long part_floats, int* cnt, int counters, void* stream) {
  AVT_REQUIRE(add_mask == nullptr || (add && add != dx), "conv2d_dgrad_ws: add_mask needs add, not aliasing dx");
  AVT_REQUIRE(part_floats >= 0 && counters >= 0, "conv2d_dgrad_ws: negative workspace size");
  const SplitWs ws{part, cnt, part_floats, counters};
  return conv2d_dgrad_impl(dy, wt, dx, add, add_mask, N, H, W, C, K, R, S, stride, pad, nullptr, stream,
                           (part && cnt) ? &ws : nullptr);
}

extern "C" int avt_conv2d_dgrad_bn(const void* dy, const void* wt, void* dx, const void* add, int N, int H, int W,
                                   int C, int K, int R, int S, int stride, int pad, const avt_dgrad_bn_epi* epi,
                                   void* stream) {
  return conv2d_dgrad_impl(dy, wt, dx, add, nullptr, N, H, W, C, K, R, S, stride, pad, epi, stream);
}

extern "C" int avt_conv2d_dgrad(const void* dy, const void* wt, void* dx, const void* add, int N, int H, int W, int C,
                                int K, int R, int S, int stride, int pad, void* stream) {
  return conv2d_dgrad_impl(dy, wt, dx, add, nullptr, N, H, W, C, K, R, S, stride, pad, nullptr, stream);
}

extern "C" int avt_conv2d_dgrad_mask(const void* dy, const void* wt, void* dx, const void* add, const void* add_mask,
                                     int N, int H, int W, int C, int K, int R, int S, int stride, int pad,
                                     void* stream) {
  AVT_REQUIRE(add && add_mask, "conv2d_dgrad_mask: add and add_mask are required");
  AVT_REQUIRE(add != dx, "conv2d_dgrad_mask: add must not alias dx");
  return conv2d_dgrad_impl(dy, wt, dx, add, add_mask, N, H, W, C, K, R, S, stride, pad, nullptr, stream);
}

// Conv3d forward (the R3D-18 video trunk, models/resnet3D.py:14-28 conv3x3x3 / conv1x1x1, called
// from BasicBlock.forward 45-61): x NDHWC bf16 [N][T][H][W][Cp], wpack bf16 [K][(kt,r,s,c)],
// y NDHWC bf16 [N][T'][H'][W'][K] with T' = T + 2*pad_t - KT + 1 (temporal stride 1, as every
// Conv3d of the R3D-18 built by model.py:20 after the stem) and spatial stride `stride`.
// BN statistics are accumulated in the epilogue exactly as conv2d_fwd.
extern "C" int avt_conv3d_fwd(const void* x, const void* wpack, void* y, double* bn_acc, int N, int T, int H, int W,
                              int Cp, int K, int KT, int R, int S, int stride, int pad_t, int pad, void* stream) {
  AVT_REQUIRE(x && wpack && y, "conv3d_fwd: null pointer");
  AVT_REQUIRE(K % 64 == 0, "conv3d_fwd: K=%d must be a multiple of 64", K);
  AVT_REQUIRE(Cp % 32 == 0, "conv3d_fwd: C=%d must be a multiple of 32", Cp);
  AVT_REQUIRE(KT * R * S <= kMaxTaps && KT >= 1 && R >= 1 && S >= 1, "conv3d_fwd: at most %d taps", kMaxTaps);
  AVT_REQUIRE(stride == 1 || stride == 2, "conv3d_fwd: spatial stride must be 1 or 2");
  GemmNTParams p{};
  p.act = (const bf16_t*)x;
  p.wmat = (const bf16_t*)wpack;
  p.out = (bf16_t*)y;
  p.add = nullptr;
  p.stats = bn_acc;
  p.IT = T; p.IH = H; p.IW = W; p.IC = Cp;
  p.OT = T + 2 * pad_t - KT + 1;
  p.OH = conv_out(H, R, stride, pad);
  p.OW = conv_out(W, S, stride, pad);
  AVT_REQUIRE(p.OT >= 1 && p.OH >= 1 && p.OW >= 1, "conv3d_fwd: empty output");
  p.M = N * p.OT * p.OH * p.OW;
  p.Ng = K;
  p.Kg = KT * R * S * Cp;
  p.KT = KT; p.R = R; p.S = S; p.stride = stride; p.pad = pad; p.pad_t = pad_t;
  AVT_REQUIRE((size_t)N * T * H * W * Cp * 2 < (1ull << 31) && (size_t)p.M * K * 2 < (1ull << 31),
              "conv3d_fwd: activation tensors must stay below 2 GiB (32-bit buffer offsets)");
  AVT_REQUIRE(conv_variant() == 1, "conv3d_fwd: needs the LDS-DMA conv kernels (AVT_CONV_VARIANT=1)");
  hipStream_t st = (hipStream_t)stream;
  if (halo3d_launch(p, st)) return check_launch("conv3d_fwd");
  if (K % 128 == 0)
    launch_nt<MODE_FWD, 8, 128, 128>(p, st);
  else
    launch_nt<MODE_FWD, 8, 128, 64>(p, st);
  return check_launch("conv3d_fwd");
}

// wgrad launch plan: tile shape, split-K and (pipelined kernel) the fp32 partial slab it needs.
struct WgradPlan {
  GemmTNParams p;
  int BM, BN, tiles, splits;
  int nst;              // LDS ring stages of the pipelined kernel
  int kg;               // wave groups per block splitting its k range (conv_tn_pipe_kernel KG)
  bool pipe;            // LDS-DMA pipelined kernel (C % 8 == 0) vs register-staged (stems)
  size_t slab_bytes;    // splits * Mg * Ng * 4 when split-K partials go through a slab
};

static WgradPlan wgrad_plan(int N, int H, int W, int Cp, int Creal, int K, int R, int S, int stride, int pad) {
  static bool env_read = false;  // A/B knobs: AVT_WGRAD_SLAB_MAX, AVT_WGRAD_WAVE_COST (as avt_set_wgrad_slab_max)
  if (!env_read) {
    env_read = true;
    if (const char* e = getenv("AVT_WGRAD_SLAB_MAX")) g_wgrad_slab_max = atoi(e);
    if (const char* e = getenv("AVT_WGRAD_WAVE_COST")) g_wgrad_wave_cost = atoi(e);
  }
  WgradPlan pl{};
  GemmTNParams& p = pl.p;
  p.Mg = K;
  p.H = H; p.W = W; p.Cp = Cp; p.Creal = Creal;
  p.P = conv_out(H, R, stride, pad);
  p.Q = conv_out(W, S, stride, pad);
  p.R = R; p.S = S; p.stride = stride; p.pad = pad;
  p.Kred = N * p.P * p.Q;
  const int ncols = R * S * Cp;
  pl.pipe = (Cp % 8 == 0) && conv_variant() == 1;
  pl.BN = (ncols % 128 == 0 || ncols > 128) ? 128 : 64;
  pl.BM = (K % 128 == 0 && Cp % 8 == 0) || (K % 128 == 0 && Cp == 4) ? 128 : 64;
  // 8-wave 256-wide tiles halve the LDS fill bytes per flop where the GEMM is wide enough
  // (layer4: K_out 512, R*S*C >= 2304); split-K supplies the parallelism
  if (g_wgrad_big < 0) g_wgrad_big = getenv("AVT_WGRAD_BIG") ? atoi(getenv("AVT_WGRAD_BIG")) : 1;
  if (pl.pipe && g_wgrad_big) {
    if (K % 256 == 0 && K >= 512 && pl.BN == 128) pl.BM = 256;  // measured: a loss on layer3 (K_out 256)
    if (ncols >= 2048 && pl.BM == 256) pl.BN = 256;
  }
  p.Ng = ((ncols + pl.BN - 1) / pl.BN) * pl.BN;
  pl.tiles = (p.Mg / pl.BM) * (p.Ng / pl.BN);
  const int nkt = (p.Kred + 31) / 32;
  // Split-K count.  The grid runs in "waves" of resident blocks (CUs x blocks per CU, set by the
  // ring's LDS: 4 stages x 32 pixels x (BM+BN) bf16 for the 4-wave tiles, 3 stages for the 8-wave
  // ones, whose 256x256 form is also held to one block per CU by its registers).  For w = 1..4
  // waves take the largest split count that fits, s_w = floor(w*slots/tiles), and keep the one
  // with the least w * (ceil(nkt/s_w) + wave_cost) -- k-tiles per block plus its fixed
  // prologue/epilogue cost.
  // 1x1 convs (the downsample shortcuts): a k-tile is only 32 pixels x (BM + BN) operand rows while
  // the epilogue still writes a BM x BN fp32 tile, so blocks need deeper K ranges than the wave
  // model picks (measured, tools/conv_bench.py: min 24 k-tiles takes the six downsample wgrads from
  // 0.239 to 0.143 ms at B = 128; the 3x3 shapes keep their optimum at 4)
  static const int min_kt_1x1 = getenv("AVT_WGRAD_MIN_KT_1X1") ? atoi(getenv("AVT_WGRAD_MIN_KT_1X1")) : 24;
  const int min_kt = (R * S == 1) ? max(g_wgrad_min_kt, min_kt_1x1) : g_wgrad_min_kt;
  int splits;
  const bool big = pl.BM == 256 || pl.BN == 256;
  // ring depth: 4 stages (4-wave tiles: two blocks per CU at 128 x 128) / 3 (8-wave); a deeper ring
  // (AVT_WGRAD_NST / AVT_WGRAD_NST_BIG, or avt_set_wgrad_nst) keeps more k-tiles in flight for a
  // block alone on its CU -- the small-batch regime, where a block's k range is short and its DMA
  // latency is exposed (one stage = 32 pixels x (BM + BN) bf16)
  if (g_wgrad_nst < 0) g_wgrad_nst = getenv("AVT_WGRAD_NST") ? atoi(getenv("AVT_WGRAD_NST")) : 4;
  if (g_wgrad_nst_big < 0) g_wgrad_nst_big = getenv("AVT_WGRAD_NST_BIG") ? atoi(getenv("AVT_WGRAD_NST_BIG")) : 3;
  // (the 256 x 128 8-wave tile always runs the 3-stage ring, launch_tn: nst_big is the 256 x 256 tile's)
  pl.nst = (pl.BM == 256 && pl.BN == 256) ? g_wgrad_nst_big : big ? 3 : g_wgrad_nst;
  if (g_wgrad_blocks > 0) {
    splits = g_wgrad_blocks / pl.tiles;
  } else {
    int occ = max(1, 163840 / (pl.nst * 64 * (pl.BM + pl.BN)));
    if (pl.BM == 256 && pl.BN == 256) occ = 1;
    // The share of the chip's block slots the model assumes the wgrad has: with both trunks' backward on two streams a
    // wgrad shares the chip with the other trunk's kernels, and fewer splits mean fewer partials through the slab and
    // a shorter reduce.  Auto (default): 65 % for a batch of <= 32, 75 % for <= 64, else 100 % -- measured same-box
    // (profiles/r6_ab_wgrad_slots*.txt): 65 % is +3.3 % at B=32, 75 % +0.7 % at B=64, and 50 % -1.8 % at B=128.
    // AVT_WGRAD_SLOTS_PCT / avt_set_wgrad_slots_pct fix it (1-100; 0 = auto).
    if (g_wgrad_slots_pct < 0) g_wgrad_slots_pct = getenv("AVT_WGRAD_SLOTS_PCT") ? atoi(getenv("AVT_WGRAD_SLOTS_PCT")) : 0;
    const int slots_pct = g_wgrad_slots_pct > 0 ? min(g_wgrad_slots_pct, 100) : N <= 32 ? 65 : N <= 64 ? 75 : 100;
    const long long slots = max(1LL, (long long)num_cus() * occ * slots_pct / 100);
    long long best = -1;
    splits = 1;
    for (int w = 1; w <= 4; ++w) {
      const int s_w = (int)(w * slots / pl.tiles);
      if (s_w < 1) continue;
      const int kps_w = max(min_kt, (nkt + s_w - 1) / s_w);
      const long long waves = (((long long)pl.tiles * ((nkt + kps_w - 1) / kps_w)) + slots - 1) / slots;
      const long long cost = waves * (kps_w + g_wgrad_wave_cost);
      if (best < 0 || cost < best) {
        best = cost;
        splits = s_w;
      }
    }
  }
  if (splits < 1) splits = 1;
  int kps = (nkt + splits - 1) / splits;
  if (kps < min_kt) kps = min_kt;
  pl.splits = (nkt + kps - 1) / kps;
  // two wave groups per block (AVT_WGRAD_KG, default 2): the pairs of blocks the plan puts on one CU
  // become one 8-wave block over both k ranges with ONE partial tile -- half the split-K slab bytes
  // (or atomics) at the same waves per CU; 4-wave tiles on the 4-stage ring (2 x 64 KB of LDS at 128 x 128)
  static const int kg_env = getenv("AVT_WGRAD_KG") ? atoi(getenv("AVT_WGRAD_KG")) : 2;
  pl.kg = 1;
  const int pair_occ = 163840 / (pl.nst * 64 * (pl.BM + pl.BN));  // 4-wave blocks per CU (2 at 128 x 128)
  // (3x3 only: the 1x1 shortcuts' deep k ranges lost 25-30 % at B = 128 as pairs)
  if (kg_env >= 2 && pl.pipe && !big && pl.nst == 4 && pair_occ == 2 && pl.splits >= 2 && R * S > 1) {
    pl.kg = 2;
    kps *= 2;
    pl.splits = (nkt + kps - 1) / kps;
  }
  p.kt_per_split = kps;
  // slab + reduce pass for moderate split counts (measured faster on layer3/4); very deep splits
  // (layer1/2: 100-200 splits of a small output) keep the fp32 atomics, which overlap the compute
  // (the slab holds whole tiles in register order: splits x Mg x Ng, conv_tn_pipe.h)
  pl.slab_bytes = (pl.pipe && pl.splits > 1 && pl.splits <= g_wgrad_slab_max)
                      ? (size_t)pl.splits * p.Mg * p.Ng * sizeof(float)
                      : 0;
  return pl;
}

// Deferred split-K reduces, batched (avt_wgrad_reduce_batch): a trunk's wgrads leave their slabs (avt_conv2d_wgrad_defer)
// and one launch sums all of them at the end of the trunk's backward segment -- blockIdx.y = the slab, a grid-stride
// loop over its float4 positions; per position the splits in order, 8 loads in flight: the order of
// wgrad_slab_reduce_native_kernel with G = 1, so the bits are the same as the per-wgrad reduce launches'.
// (The reduces are off the backward's dgrad chain; at 32 clips per GPU their ~34 separate launches cost up to 7 % of
// the step: profiles/r6_slab_skip.txt.)
constexpr int kSlabBatch = 24;
struct SlabReduceBatch {
  int n;
  avt_slab_reduce_desc e[kSlabBatch];
};

__global__ __launch_bounds__(256) void wgrad_slab_reduce_batch_kernel(SlabReduceBatch b) {
  const avt_slab_reduce_desc& E = b.e[blockIdx.y];
  const int NW = E.wm * E.wn;
  const long long per_tile = (long long)NW * E.tm * E.tn * 4 * 64;
  const long long total = (long long)E.tiles * per_tile;
  const f32x4* s4 = reinterpret_cast<const f32x4*>(E.slab);
  const int BM = E.wm * E.tm * 32, BN = E.wn * E.tn * 32;
  for (long long f = (long long)blockIdx.x * 256 + threadIdx.x; f < total; f += (long long)gridDim.x * 256) {
    f32x4 a = {0.f, 0.f, 0.f, 0.f};
    for (int s0 = 0; s0 < E.splits; s0 += 8) {
      f32x4 v[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) v[i] = s0 + i < E.splits ? s4[f + (s0 + i) * total] : f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int i = 0; i < 8; ++i) a += v[i];
    }
    const int lane = (int)(f & 63);
    long long r = f >> 6;
    const int q = (int)(r & 3);
    r >>= 2;
    const int jj = (int)(r % E.tn);
    r /= E.tn;
    const int i = (int)(r % E.tm);
    r /= E.tm;
    const int wid = (int)(r % NW);
    const int tile = (int)(r / NW);
    const int mt = tile / E.nnt, nt = tile - mt * E.nnt;
    const int wm = wid / E.wn, wn = wid % E.wn;
    const int col = nt * BN + wn * (BN / E.wn) + jj * 32 + (lane & 31);
    const int r0 = mt * BM + wm * (BM / E.wm) + i * 32 + 8 * q + 4 * (lane >> 5);
    if (col < E.ldw) {
#pragma unroll
      for (int e = 0; e < 4; ++e)
        if (r0 + e < E.Mg) E.dw[(size_t)(r0 + e) * E.ldw + col] += a[e];
    }
  }
}

template <int WM, int WN, int TM, int TN, int NST, int KG>
static void launch_tn_one(dim3 grid, const GemmTNPipeParams& pp, hipStream_t st) {
  if (pp.cnt != nullptr)
    hipLaunchKernelGGL((conv_tn_pipe_kernel<WM, WN, TM, TN, NST, KG, true>), grid, dim3(WM * WN * 64 * KG), 0, st, pp);
  else
    hipLaunchKernelGGL((conv_tn_pipe_kernel<WM, WN, TM, TN, NST, KG>), grid, dim3(WM * WN * 64 * KG), 0, st, pp);
}

// the wgrad plan's launch shape runs the fused in-kernel slab reduce (launch_tn_one; the deeper-ring A/B variants
// keep the separate reduce)
static bool tn_fusable(const WgradPlan& pl) {
  if (!pl.pipe || pl.splits < 2) return false;
  if (pl.BM == 256 && pl.BN == 256) return pl.nst < 4;
  if (pl.BM == 256) return true;
  return pl.kg == 2 || pl.nst < 6;
}

template <int CVEC, int BM, int BN>
static void launch_tn(const WgradPlan& pl, float* slab, hipStream_t st, int* tickets = nullptr) {
  GemmTNParams p = pl.p;
  if (pl.pipe) {
    GemmTNPipeParams pp;
    pp.p = p;
    pp.div_pq = make_magic((unsigned)(p.P * p.Q));
    pp.div_q = make_magic((unsigned)p.Q);
    pp.dy_bytes = (unsigned)((size_t)p.Kred * p.Mg * 2);
    pp.x_bytes = (unsigned)((size_t)(p.Kred / (p.P * p.Q)) * p.H * p.W * p.Cp * 2);
    pp.slab = slab;
    pp.cnt = (slab != nullptr && tickets != nullptr && tn_fusable(pl)) ? tickets : nullptr;
    pp.slab_bytes = (unsigned)pl.slab_bytes;
    pp.splits = pl.splits;
    const dim3 grid(pl.tiles * pl.splits);
    if constexpr (BM == 256 && BN == 256) {
      if (pl.nst >= 5)
        hipLaunchKernelGGL((conv_tn_pipe_kernel<4, 2, 2, 4, 5>), grid, dim3(512), 0, st, pp);
      else if (pl.nst == 4)
        hipLaunchKernelGGL((conv_tn_pipe_kernel<4, 2, 2, 4, 4>), grid, dim3(512), 0, st, pp);
      else
        launch_tn_one<4, 2, 2, 4, 3, 1>(grid, pp, st);
    } else if constexpr (BM == 256) {
      launch_tn_one<4, 2, 2, 2, 3, 1>(grid, pp, st);
    } else {
      if (pl.kg == 2)
        launch_tn_one<2, 2, BM / 64, BN / 64, 4, 2>(grid, pp, st);
      else if (pl.nst >= 8)
        hipLaunchKernelGGL((conv_tn_pipe_kernel<2, 2, BM / 64, BN / 64, 8>), grid, dim3(256), 0, st, pp);
      else if (pl.nst >= 6)
        hipLaunchKernelGGL((conv_tn_pipe_kernel<2, 2, BM / 64, BN / 64, 6>), grid, dim3(256), 0, st, pp);
      else
        launch_tn_one<2, 2, BM / 64, BN / 64, 4, 1>(grid, pp, st);
    }
    return;
  }
  if constexpr (BM <= 128)
    hipLaunchKernelGGL((gemm_tn_kernel<CVEC, BM, BN>), dim3(pl.tiles, pl.splits), dim3(256), 0, st, p);
}

// ---- halo wgrad plan (conv_wgrad_halo.h) ----
static int g_wgrad_halo_rw = -1;  // rows per wave of the K = 64 halo wgrad: 32 (default) or 64; -1: env AVT_WGRAD_HALO_RW
static int wgrad_halo_rw() {
  if (g_wgrad_halo_rw < 0) g_wgrad_halo_rw = getenv("AVT_WGRAD_HALO_RW") ? atoi(getenv("AVT_WGRAD_HALO_RW")) : 32;
  return g_wgrad_halo_rw;
}
static int g_row3_min_kt = -1;  // ROW3 split floor (k-tiles per split); -1: env AVT_ROW3_MIN_KT
static int row3_min_kt() {
  if (g_row3_min_kt < 0) g_row3_min_kt = getenv("AVT_ROW3_MIN_KT") ? atoi(getenv("AVT_ROW3_MIN_KT")) : 8;
  if (g_row3_min_kt < 1) g_row3_min_kt = 1;
  return g_row3_min_kt;
}
static int g_row3_kg = -1;  // ROW3 k groups per block (1 or 2); -1: env AVT_ROW3_KG
static int row3_kg() {
  if (g_row3_kg < 0) g_row3_kg = getenv("AVT_ROW3_KG") ? atoi(getenv("AVT_ROW3_KG")) : 2;
  return (g_row3_kg == 2 || g_row3_kg == 4) ? g_row3_kg : 1;
}
static int g_row3_pf = -1;  // ROW3 (KG 2): next tile's first fragments read behind the MFMAs (default: +3-4 %);
                            // -1: env AVT_ROW3_PF
static int row3_pf() {
  if (g_row3_pf < 0) g_row3_pf = getenv("AVT_ROW3_PF") ? atoi(getenv("AVT_ROW3_PF")) : 1;
  return g_row3_pf;
}
static int wgrad_halo_enabled() {
  if (g_wgrad_halo < 0) {
    const char* e = getenv("AVT_WGRAD_HALO");
    g_wgrad_halo = e ? atoi(e) : 3;
  }
  return g_wgrad_halo;
}

struct WgradHaloPlan {
  bool ok;
  bool row3; // one filter row (3 taps) per block: WM x 2 waves of 64 x 96, strip of PR - 2 PW patch rows
  int kg;    // ROW3: k groups per block (KG groups of WM x 2 waves on interleaved k-tiles, one partial per block;
             // WM 2: at most 2)
  int WM;    // 2: BM 128 (4 waves), 1: BM 64 (2 waves)
  int RW;    // output channels per wave: 64, or 32 (9-tap form, K = 64: 4 waves of 32 x 288, two per SIMD)
  WgradHaloArgs a;
  size_t slab_bytes;
  int groups, per_group;  // reduce: split groups (pass 1), then one ordered pass over the group heads
};

static constexpr int kRow3PrMax = 40;  // strip rows staged by the ROW3 form
// default form 3 takes ROW3 from this many output pixels up (B = 128: 401 k vision / 624 k audio); below
// it the fixed cost of the split partials (slab + ordered reduce) loses to the tap-gather kernel (B = 32:
// 100 k / 156 k pixels, -1.5 % per step in a same-box A/B)
static constexpr long long kRow3MinPixels = 200000;

static WgradHaloPlan wgrad_halo_plan(int N, int H, int W, int Cp, int Creal, int K, int R, int S, int stride, int pad) {
  WgradHaloPlan pl{};
  pl.ok = false;
  int mode = wgrad_halo_enabled();
  if (mode == 3) mode = (K == 64 && (long long)N * H * W >= kRow3MinPixels) ? 2 : 0;
  if (!mode || R != 3 || S != 3 || stride != 1 || pad != 1 || Cp != Creal || Cp % 64 != 0 ||
      K % 64 != 0 || conv_variant() != 1)
    return pl;
  WgradHaloArgs& a = pl.a;
  a.N = N; a.H = H; a.W = W; a.C = Cp; a.K = K;
  pl.row3 = mode == 2;
  pl.kg = 1;
  pl.WM = (K % 128 == 0) ? 2 : 1;
  pl.RW = 64;
  if (!pl.row3 && K == 64 && wgrad_halo_rw() == 32) {  // 4 waves of 32 x 288 (144 accumulator registers: two waves per SIMD)
    pl.WM = 2;
    pl.RW = 32;
  }
  if (pl.row3 && getenv("AVT_ROW3_WM") && atoi(getenv("AVT_ROW3_WM")) == 1) pl.WM = 1;  // A/B: 64-row blocks at K >= 128
  const int BM = pl.WM * pl.RW;  // after every WM override: the plan and the launch use the same block rows
  const int ncols = pl.row3 ? 192 : 576;  // GEMM columns per block
  const int PRMAX = pl.row3 ? kRow3PrMax : (pl.WM == 2 && pl.RW == 64) ? 160 : 72;
  if (pl.row3) pl.kg = pl.WM == 1 ? row3_kg() : (row3_kg() >= 2 ? 2 : 1);
  const int per_cu = pl.row3 ? (pl.WM == 1 ? 4 : 2) / pl.kg : (pl.WM == 2 && pl.RW == 64) ? 1 : 2;  // resident blocks per CU
  auto staged = [&](int pr, int pw) { return pl.row3 ? pr - 2 * pw : pr; };
  const double t_mfma = 2.0 * 32 * BM * ncols / (4 * 1024.0);
  auto cost = [&](long long tiles, int pr) {  // pr: staged patch rows
    const double fill = (32.0 * BM * 2 + pr * 128.0) / (29.0 / per_cu);
    return (double)tiles * (t_mfma > fill ? t_mfma : fill);
  };
  double best = -1;
  // raster: 32 consecutive pixels span at most ceil(31/W)+1 rows
  {
    const int span = (W >= 32 ? 2 : (31 + W - 1) / W + 1);
    const int pr = (span + 2) * (W + 2);
    if (!pl.row3 && staged(pr, W + 2) <= PRMAX) {  // (ROW3: windows only -- fixed fragment rows)
      const long long tiles = (long long)(H * W + 31) / 32;
      best = cost(tiles, staged(pr, W + 2));
      a.raster = 1; a.R = 1; a.CW = 32; a.lcw = 5; a.wcols = 1; a.tiles_img = (int)tiles; a.PW = W + 2; a.PR = pr;
    }
  }
  const int shapes[4][2] = {{1, 32}, {2, 16}, {4, 8}, {8, 4}};
  for (auto& sh : shapes) {
    const int r = sh[0], cw = sh[1];
    const int pr = (r + 2) * (cw + 2);
    if (staged(pr, cw + 2) > PRMAX) continue;
    const int bands = (H + r - 1) / r, wcols = (W + cw - 1) / cw;
    const double c = cost((long long)bands * wcols, staged(pr, cw + 2));
    if (best < 0 || c < best * 0.999) {
      best = c;
      a.raster = 0; a.R = r; a.CW = cw; a.lcw = 31 - __builtin_clz(cw); a.wcols = wcols; a.tiles_img = bands * wcols;
      a.PW = cw + 2; a.PR = pr;
    }
  }
  if (best < 0) return pl;
  a.nkt = N * a.tiles_img;
  const int per_split = (K / BM) * (Cp / 64) * (pl.row3 ? 3 : 1);
  // (A/B, env AVT_WGRAD_HALO_SHARE, default 100: the share of the chip's block slots the split count assumes)
  static const int halo_share = getenv("AVT_WGRAD_HALO_SHARE") ? atoi(getenv("AVT_WGRAD_HALO_SHARE")) : 100;
  const long long slots = max(1LL, (long long)num_cus() * per_cu * min(max(halo_share, 1), 100) / 100);
  int splits = (int)(slots / per_split);
  if (pl.row3) {  // at least row3_min_kt() k-tiles per split: the slab (splits x 147 KB at K 64) is the cost at small N
    const int cap = a.nkt / row3_min_kt();
    if (splits > cap) splits = cap;
  }
  if (splits < 1) splits = 1;
  if (splits > a.nkt) splits = a.nkt;
  const int kps = (a.nkt + splits - 1) / splits;
  a.kt_per_split = kps;
  a.splits = (a.nkt + kps - 1) / kps;  // every split non-empty
  a.div_w = make_magic((unsigned)W);
  a.div_tiles = make_magic((unsigned)a.tiles_img);
  a.div_wcols = make_magic((unsigned)a.wcols);
  a.dy_bytes = (unsigned)((size_t)N * H * W * K * 2);
  a.x_bytes = (unsigned)((size_t)N * H * W * Cp * 2);
  pl.slab_bytes = a.splits > 1 ? (size_t)a.splits * K * 9 * Cp * sizeof(float) : 0;
  pl.per_group = 16;
  pl.groups = (a.splits + pl.per_group - 1) / pl.per_group;
  pl.ok = true;
  return pl;
}

static void launch_wgrad_halo(WgradHaloPlan& pl, const bf16_t* x, const bf16_t* dy, float* dw, float* slab,
                              hipStream_t st) {
  WgradHaloArgs& a = pl.a;
  a.x = x;
  a.dy = dy;
  a.dw = dw;
  a.slab = slab;
  const int BM = pl.WM * pl.RW;
  const int grid = (a.K / BM) * (a.C / 64) * (pl.row3 ? 3 : 1) * a.splits;
  if (pl.row3 && pl.WM == 2 && pl.kg == 2)
    hipLaunchKernelGGL((conv_wgrad_halo_kernel<2, 4, kRow3PrMax, 64, true, 2>), dim3(grid), dim3(512), 0, st, a);
  else if (pl.row3 && pl.WM == 2)
    hipLaunchKernelGGL((conv_wgrad_halo_kernel<2, 4, kRow3PrMax, 64, true>), dim3(grid), dim3(256), 0, st, a);
  else if (pl.row3 && pl.kg == 4)
    hipLaunchKernelGGL((conv_wgrad_halo_kernel<1, 4, kRow3PrMax, 64, true, 4>), dim3(grid), dim3(512), 0, st, a);
  else if (pl.row3 && pl.kg == 2 && row3_pf())
    hipLaunchKernelGGL((conv_wgrad_halo_kernel<1, 4, kRow3PrMax, 64, true, 2, true>), dim3(grid), dim3(256), 0, st, a);
  else if (pl.row3 && pl.kg == 2)
    hipLaunchKernelGGL((conv_wgrad_halo_kernel<1, 4, kRow3PrMax, 64, true, 2>), dim3(grid), dim3(256), 0, st, a);
  else if (pl.row3)
    hipLaunchKernelGGL((conv_wgrad_halo_kernel<1, 4, kRow3PrMax, 64, true>), dim3(grid), dim3(128), 0, st, a);
  else if (pl.RW == 32)
    hipLaunchKernelGGL((conv_wgrad_halo_kernel<2, 6, 72, 32>), dim3(grid), dim3(256), 0, st, a);
  else if (pl.WM == 2)
    hipLaunchKernelGGL((conv_wgrad_halo_kernel<2, 5, 160>), dim3(grid), dim3(256), 0, st, a);
  else
    hipLaunchKernelGGL((conv_wgrad_halo_kernel<1, 6, 72>), dim3(grid), dim3(128), 0, st, a);
  if (slab) {  // ordered: groups of per_group splits, then the group heads
    const long long n = (long long)a.K * 9 * a.C;
    const unsigned gx = (unsigned)((n / 4 + 255) / 256), gx64 = (unsigned)((n / 4 + 63) / 64);
    if (pl.groups > 1)
      hipLaunchKernelGGL(wgrad_halo_reduce_kernel, dim3(gx, (unsigned)pl.groups), dim3(256), 0, st, slab, a.splits, 1,
                         pl.per_group, n, dw);
    // the final pass is latency-bound (one thread per 4 outputs, a serial chain of entries): 64-thread blocks
    hipLaunchKernelGGL(wgrad_halo_reduce_kernel, dim3(gx64, 1), dim3(64), 0, st, slab, pl.groups > 1 ? pl.groups : a.splits,
                       pl.groups > 1 ? pl.per_group : 1, pl.groups > 1 ? pl.groups : a.splits, n, dw);
  }
}

extern "C" int avt_set_halo_tps2(int on) {
  AVT_REQUIRE(on >= -1 && on <= 1, "avt_set_halo_tps2: %d (0 one tap per barrier, 1 two, -1 env AVT_HALO_TPS2)", on);
  g_halo_tps2 = on;
  return AVT_OK;
}

extern "C" int avt_set_halo3d(int on) {
  AVT_REQUIRE(on >= -1 && on <= 2, "avt_set_halo3d: %d (0 tap gather, 1 halo for K %% 128 == 0, 2 also K = 64, -1 env "
              "AVT_HALO3D)", on);
  g_halo3d = on;
  return AVT_OK;
}

extern "C" int avt_set_wgrad_row3(int kg, int min_kt, int pf) {
  AVT_REQUIRE(kg == -1 || kg == 1 || kg == 2 || kg == 4, "avt_set_wgrad_row3: kg=%d (1, 2 or 4)", kg);
  AVT_REQUIRE(min_kt == -1 || min_kt >= 1, "avt_set_wgrad_row3: min_kt=%d", min_kt);
  AVT_REQUIRE(pf >= -1 && pf <= 1, "avt_set_wgrad_row3: pf=%d", pf);
  // -1 resets a value to its environment default (re-read on next use), as the sibling setters do
  g_row3_kg = kg;
  g_row3_min_kt = min_kt;
  g_row3_pf = pf;
  return AVT_OK;
}

extern "C" int avt_set_wgrad_halo(int on) {
  AVT_REQUIRE(on >= -1 && on <= 3, "avt_set_wgrad_halo: %d (0 off, 1 nine taps, 2 one filter row per block, 3 = 2 for K 64, -1 env)", on);
  avt::g_wgrad_halo = on;
  return AVT_OK;
}

namespace avt {
// stem wgrad on conv_stem_wgrad_kernel: grid (one block per CU at most) and its slab bytes; grid 0 = n/a
struct StemWgradPlan {
  int grid = 0;
  size_t slab_bytes = 0;
  StemWgradArgs a{};
};
static StemWgradPlan stem_wgrad_plan(int N, int H, int W, int Cp, int Creal, int K, int R, int S, int stride, int pad) {
  StemWgradPlan pl;
  if (!((Cp == 4 || Cp == 1) && stem_wgrad_enabled() && K == 64 && R == 7 && S == 7 && stride == 2 && pad == 3 &&
        Creal >= 1 && Creal <= Cp && N >= 1))
    return pl;
  const int OH = (H + 2 * pad - R) / stride + 1, OW = (W + 2 * pad - S) / stride + 1;
  if (OH < 1 || OW < 1) return pl;
  if ((size_t)N * H * W * Cp * 2 >= (1ull << 31) || (size_t)N * OH * OW * 64 * 2 >= (1ull << 31)) return pl;  // 32-bit offsets
  pl.a.N = N; pl.a.IH = H; pl.a.IW = W; pl.a.OH = OH; pl.a.OW = OW; pl.a.Creal = Creal;
  pl.a.tiles_per_row = (OW + 31) / 32;
  pl.a.total_tiles = N * OH * pl.a.tiles_per_row;
  const int nw = Cp == 4 ? StemWgradCfg<4>::NW : StemWgradCfg<1>::NW;
  const int blocks = (pl.a.total_tiles + nw - 1) / nw;
  pl.grid = blocks < num_cus() ? blocks : num_cus();
  pl.slab_bytes = (size_t)pl.grid * 64 * 49 * Creal * sizeof(float);
  return pl;
}
}  // namespace avt

// A/B knob: the fused slab reduce (conv_tn_pipe.h FUSED) for the tap-gather wgrads, avt_set_wgrad_fused / env
// AVT_WGRAD_FUSED (0 default = the separate reduce launch; 1 = fused up to g_wgrad_fused_max_bytes of other splits'
// partials per tile).  Bitwise equal where the separate reduce runs one wave per position, but SLOWER: the wgrad
// family 355 -> 214 TF/s, the step -7 % at B=32 and -1.7 % at B=128 (profiles/r6_ab_wgrad_fused.txt) -- the
// write-through partials and the last block's serial read of the other splits cost more than the reduce launch
static int g_wgrad_fused = -1;
static long long g_wgrad_fused_max_bytes = -1;
static bool wgrad_fused_plan(const WgradPlan& pl) {
  if (g_wgrad_fused < 0) g_wgrad_fused = getenv("AVT_WGRAD_FUSED") ? atoi(getenv("AVT_WGRAD_FUSED")) : 0;
  if (g_wgrad_fused_max_bytes < 0)
    g_wgrad_fused_max_bytes = getenv("AVT_WGRAD_FUSED_MAX_KB") ? 1024LL * atoll(getenv("AVT_WGRAD_FUSED_MAX_KB"))
                                                               : 2048LL * 1024;
  return g_wgrad_fused && pl.slab_bytes > 0 && tn_fusable(pl) &&
         (long long)(pl.splits - 1) * pl.BM * pl.BN * 4 <= g_wgrad_fused_max_bytes;
}

extern "C" int avt_set_wgrad_fused(int on, int max_kb) {
  AVT_REQUIRE(on >= -1 && on <= 1, "avt_set_wgrad_fused: %d (0 separate reduce, 1 fused, -1 env AVT_WGRAD_FUSED)", on);
  AVT_REQUIRE(max_kb >= -1, "avt_set_wgrad_fused: max_kb=%d", max_kb);
  g_wgrad_fused = on;
  g_wgrad_fused_max_bytes = max_kb < 0 ? -1 : 1024LL * max_kb;
  return AVT_OK;
}

// tickets the fused wgrad slab reduce needs for this conv (avt_conv2d_wgrad_tk), 0: the shape does not use it
extern "C" int avt_conv2d_wgrad_tickets(int N, int H, int W, int Cp, int Creal, int K, int R, int S, int stride,
                                        int pad) {
  using namespace avt;
  if (stem_wgrad_plan(N, H, W, Cp, Creal, K, R, S, stride, pad).grid > 0) return 0;
  if (wgrad_halo_plan(N, H, W, Cp, Creal, K, R, S, stride, pad).ok) return 0;
  const WgradPlan pl = wgrad_plan(N, H, W, Cp, Creal, K, R, S, stride, pad);
  return wgrad_fused_plan(pl) ? pl.tiles : 0;
}

extern "C" size_t avt_conv2d_wgrad_workspace(int N, int H, int W, int Cp, int Creal, int K, int R, int S, int stride,
                                             int pad) {
  const StemWgradPlan sp = stem_wgrad_plan(N, H, W, Cp, Creal, K, R, S, stride, pad);
  if (sp.grid > 0) return sp.slab_bytes;
  const WgradHaloPlan hp = wgrad_halo_plan(N, H, W, Cp, Creal, K, R, S, stride, pad);
  if (hp.ok) return hp.slab_bytes;
  return wgrad_plan(N, H, W, Cp, Creal, K, R, S, stride, pad).slab_bytes;
}

// dw += wgrad.  With a workspace of avt_conv2d_wgrad_workspace() bytes the split-K partials go
// through an fp32 slab + one reduction pass (deterministic, 2x cheaper than atomics); without it
// (or for the stems) they are added with fp32 atomics.  dw must hold zero or a gradient to add to.
extern "C" int avt_conv2d_wgrad_tk(const void* x, const void* dy, float* dw, int N, int H, int W, int Cp, int Creal,
                                   int K, int R, int S, int stride, int pad, void* workspace, size_t ws_bytes,
                                   int* tickets, int n_tickets, void* stream);

extern "C" int avt_conv2d_wgrad(const void* x, const void* dy, float* dw, int N, int H, int W, int Cp, int Creal,
                                int K, int R, int S, int stride, int pad, void* workspace, size_t ws_bytes,
                                void* stream) {
  return avt_conv2d_wgrad_tk(x, dy, dw, N, H, W, Cp, Creal, K, R, S, stride, pad, workspace, ws_bytes, nullptr, 0,
                             stream);
}

// tickets: >= avt_conv2d_wgrad_tickets() ints, zero on entry (the kernel leaves them zero), or null: the split-K slab
// is summed by the last block of each tile instead of a separate reduce launch (same bits)
static int conv2d_wgrad_impl(const void* x, const void* dy, float* dw, int N, int H, int W, int Cp, int Creal, int K,
                             int R, int S, int stride, int pad, void* workspace, size_t ws_bytes, int* tickets,
                             int n_tickets, avt_slab_reduce_desc* defer, void* stream);

extern "C" int avt_conv2d_wgrad_tk(const void* x, const void* dy, float* dw, int N, int H, int W, int Cp, int Creal,
                                   int K, int R, int S, int stride, int pad, void* workspace, size_t ws_bytes,
                                   int* tickets, int n_tickets, void* stream) {
  return conv2d_wgrad_impl(x, dy, dw, N, H, W, Cp, Creal, K, R, S, stride, pad, workspace, ws_bytes, tickets,
                           n_tickets, nullptr, stream);
}

extern "C" int avt_conv2d_wgrad_defer(const void* x, const void* dy, float* dw, int N, int H, int W, int Cp, int Creal,
                                      int K, int R, int S, int stride, int pad, void* workspace, size_t ws_bytes,
                                      avt_slab_reduce_desc* desc, void* stream) {
  AVT_REQUIRE(desc, "conv2d_wgrad_defer: null descriptor");
  desc->splits = 0;
  return conv2d_wgrad_impl(x, dy, dw, N, H, W, Cp, Creal, K, R, S, stride, pad, workspace, ws_bytes, nullptr, 0, desc,
                           stream);
}

extern "C" int avt_wgrad_reduce_batch(const avt_slab_reduce_desc* descs, int n, void* stream) {
  AVT_REQUIRE(n >= 0 && (n == 0 || descs), "wgrad_reduce_batch: bad arguments");
  hipStream_t st = (hipStream_t)stream;
  for (int k0 = 0; k0 < n; k0 += kSlabBatch) {
    SlabReduceBatch b{};
    b.n = n - k0 < kSlabBatch ? n - k0 : kSlabBatch;
    long long maxpos = 0;
    for (int k = 0; k < b.n; ++k) {
      const avt_slab_reduce_desc& d = descs[k0 + k];
      AVT_REQUIRE(d.slab && d.dw && d.splits >= 1 && d.tiles >= 1 && d.nnt >= 1 && d.wm >= 1 && d.wn >= 1 &&
                      d.tm >= 1 && d.tn >= 1,
                  "wgrad_reduce_batch: descriptor %d is not from avt_conv2d_wgrad_defer", k0 + k);
      b.e[k] = d;
      const long long pos = (long long)d.tiles * d.wm * d.wn * d.tm * d.tn * 4 * 64;
      maxpos = pos > maxpos ? pos : maxpos;
    }
    long long gx = (maxpos + 255) / 256;
    if (gx > 1024) gx = 1024;
    if (b.n > 0)
      hipLaunchKernelGGL(wgrad_slab_reduce_batch_kernel, dim3((unsigned)gx, (unsigned)b.n), dim3(256), 0, st, b);
  }
  return check_launch("wgrad_reduce_batch");
}

static int conv2d_wgrad_impl(const void* x, const void* dy, float* dw, int N, int H, int W, int Cp, int Creal, int K,
                             int R, int S, int stride, int pad, void* workspace, size_t ws_bytes, int* tickets,
                             int n_tickets, avt_slab_reduce_desc* defer, void* stream) {
  AVT_REQUIRE(x && dy && dw, "conv2d_wgrad: null pointer");
  AVT_REQUIRE(K % 64 == 0, "conv2d_wgrad: K=%d must be a multiple of 64", K);
  AVT_REQUIRE(Cp % 8 == 0 || Cp == 4 || Cp == 1, "conv2d_wgrad: C=%d unsupported", Cp);
  AVT_REQUIRE(Creal <= Cp, "conv2d_wgrad: Creal > Cp");
  AVT_REQUIRE(Cp % 8 != 0 || Creal == Cp, "conv2d_wgrad: channel padding only for the stems");
  StemWgradPlan sp = stem_wgrad_plan(N, H, W, Cp, Creal, K, R, S, stride, pad);
  if (sp.grid > 0 && workspace != nullptr && ws_bytes >= sp.slab_bytes) {
    sp.a.x = (const bf16_t*)x;
    sp.a.dy = (const bf16_t*)dy;
    sp.a.slab = (float*)workspace;
    sp.a.x_bytes = (unsigned)((size_t)N * H * W * Cp * 2);
    sp.a.dy_bytes = (unsigned)((size_t)N * sp.a.OH * sp.a.OW * 64 * 2);
    hipStream_t st = (hipStream_t)stream;
    if (Cp == 4)
      hipLaunchKernelGGL(conv_stem_wgrad_kernel<4>, dim3(sp.grid), dim3(StemWgradCfg<4>::NW * 64),
                         stem_wgrad_lds_bytes<4>(), st, sp.a);
    else
      hipLaunchKernelGGL(conv_stem_wgrad_kernel<1>, dim3(sp.grid), dim3(StemWgradCfg<1>::NW * 64),
                         stem_wgrad_lds_bytes<1>(), st, sp.a);
    const int n = 64 * 49 * Creal;
    hipLaunchKernelGGL(stem_wgrad_reduce_kernel, dim3((n + 63) / 64), dim3(1024), 0, st, (const float*)workspace,
                       sp.grid, n, dw);
    return check_launch("conv2d_wgrad(stem)");
  }
  WgradHaloPlan hp = wgrad_halo_plan(N, H, W, Cp, Creal, K, R, S, stride, pad);
  if (hp.ok) {
    // without the workspace the split partials are added with fp32 atomics
    float* hslab = (hp.slab_bytes > 0 && workspace != nullptr && ws_bytes >= hp.slab_bytes) ? (float*)workspace : nullptr;
    launch_wgrad_halo(hp, (const bf16_t*)x, (const bf16_t*)dy, dw, hslab, (hipStream_t)stream);
    return check_launch("conv2d_wgrad(halo)");
  }
  WgradPlan pl = wgrad_plan(N, H, W, Cp, Creal, K, R, S, stride, pad);
  pl.p.dy = (const bf16_t*)dy;
  pl.p.x = (const bf16_t*)x;
  pl.p.dw = dw;
  float* slab = (pl.slab_bytes > 0 && workspace != nullptr && ws_bytes >= pl.slab_bytes) ? (float*)workspace : nullptr;
  hipStream_t st = (hipStream_t)stream;
  const int BM = pl.BM, BN = pl.BN;
  int* tk = (slab != nullptr && tickets != nullptr && n_tickets >= pl.tiles && Cp % 8 == 0 && wgrad_fused_plan(pl))
                ? tickets
                : nullptr;
  if (Cp == 4) {
    if (BM == 128) launch_tn<4, 128, 128>(pl, slab, st); else launch_tn<4, 64, 128>(pl, slab, st);
  } else if (Cp == 1) {
    if (BN == 128) launch_tn<1, 64, 128>(pl, slab, st); else launch_tn<1, 64, 64>(pl, slab, st);
  } else if (BM == 256) {
    if (BN == 256) launch_tn<8, 256, 256>(pl, slab, st, tk);
    else launch_tn<8, 256, 128>(pl, slab, st, tk);  // the plan pairs BM 256 with BN >= 128 only
  } else if (BN == 128) {
    if (BM == 128) launch_tn<8, 128, 128>(pl, slab, st, tk); else launch_tn<8, 64, 128>(pl, slab, st, tk);
  } else {
    if (BM == 128) launch_tn<8, 128, 64>(pl, slab, st, tk); else launch_tn<8, 64, 64>(pl, slab, st, tk);
  }
  if (slab && tk == nullptr && !diag_skip(4, st)) {
    // G waves per 64 slab positions: 1 where the positions alone give ~64 K threads, else up to min(splits, 16)
    const int wm = BM == 256 ? 4 : 2, wn = 2, tm = BM == 64 ? 1 : 2, tn = BN == 256 ? 4 : BN == 128 ? 2 : 1;
    const long long positions = (long long)pl.tiles * wm * wn * tm * tn * 4 * 64;
    int G = 1;
    while (G * 2 <= pl.splits && G * 2 <= 16 && positions * G < 65536) G *= 2;
    if (defer != nullptr && G == 1) {  // left for the batched reduce (the same order: G = 1)
      defer->slab = slab;
      defer->dw = dw;
      defer->splits = pl.splits;
      defer->tiles = pl.tiles;
      defer->nnt = pl.p.Ng / BN;
      defer->Mg = pl.p.Mg;
      defer->ldw = R * S * Creal;
      defer->wm = wm; defer->wn = wn; defer->tm = tm; defer->tn = tn;
      return check_launch("conv2d_wgrad");
    }
    const int nwb = G > 4 ? G : 4, ngrp = nwb / G;
    long long blocks = (positions + 64LL * ngrp - 1) / (64LL * ngrp);
    if (blocks > 4096) blocks = 4096;
    if (blocks < 1) blocks = 1;
    const int nnt = pl.p.Ng / BN, ldw = R * S * Creal;
    const dim3 g((unsigned)blocks), b(nwb * 64);
    if (BM == 256 && BN == 256)
      hipLaunchKernelGGL((wgrad_slab_reduce_native_kernel<4, 2, 2, 4>), g, b, 0, st, slab, pl.splits, pl.tiles, nnt,
                         pl.p.Mg, ldw, G, dw);
    else if (BM == 256)
      hipLaunchKernelGGL((wgrad_slab_reduce_native_kernel<4, 2, 2, 2>), g, b, 0, st, slab, pl.splits, pl.tiles, nnt,
                         pl.p.Mg, ldw, G, dw);
    else if (BM == 128 && BN == 128)
      hipLaunchKernelGGL((wgrad_slab_reduce_native_kernel<2, 2, 2, 2>), g, b, 0, st, slab, pl.splits, pl.tiles, nnt,
                         pl.p.Mg, ldw, G, dw);
    else if (BM == 128)
      hipLaunchKernelGGL((wgrad_slab_reduce_native_kernel<2, 2, 2, 1>), g, b, 0, st, slab, pl.splits, pl.tiles, nnt,
                         pl.p.Mg, ldw, G, dw);
    else if (BN == 128)
      hipLaunchKernelGGL((wgrad_slab_reduce_native_kernel<2, 2, 1, 2>), g, b, 0, st, slab, pl.splits, pl.tiles, nnt,
                         pl.p.Mg, ldw, G, dw);
    else
      hipLaunchKernelGGL((wgrad_slab_reduce_native_kernel<2, 2, 1, 1>), g, b, 0, st, slab, pl.splits, pl.tiles, nnt,
                         pl.p.Mg, ldw, G, dw);
  }
  return check_launch("conv2d_wgrad");
}
