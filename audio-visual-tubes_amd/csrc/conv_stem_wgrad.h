// Weight gradient of the 7x7 / stride 2 / pad 3 stems (models/base_models.py:135-138 under the
// reference's autograd): DW[k][r][s][c] = sum_pix DY[pix][k] * X[n, 2*oh - 3 + r, 2*ow - 3 + s, c],
// 64 output channels, C = 4 (vision, 3 real channels) or C = 1 (audio).  Included by conv_gemm.hip
// inside namespace avt after conv_stem.h (uses xcd_remap, tn_swz, wave_lds_sync, kStemPC).
//
// The generic TN kernel gathers the 1-/4-channel patch columns element by element (155-210 us at
// B = 128 against a ~30-45 us HBM floor).  Here, as in the stem forward, every wave streams its own
// 32-pixel tiles of one output row with no block barrier in the main loop:
//   * the tile's DY rows [32 pix][64 ch] (4 KB, 16-byte loads; rows past the image edge zero) and
//     its input patch (7 input rows x 70 columns, zeros outside the image) go to the wave's own
//     double-buffered LDS region (buffer loads; zeros by an out-of-range offset): the next tile's
//     are in flight in registers while this tile multiplies;
//   * GEMM with pixels as the MFMA k dimension: both operands are pixel-major, so the fragments come
//     out of LDS with ds_read_b64_tr_b16 from per-lane row addresses (4 consecutive GEMM columns of
//     one pixel per lane-address):
//       DY:  row = pixel, columns = output channels (XOR-swizzled 16-B chunks);
//       X:   C = 4: column (r, s, c) of pixel q = patch[r][2q + s][c]: GEMM column 32 r + 4 s + c
//                   (s = 7 a dummy tap), 4 consecutive columns = one 8-byte patch pixel; 7 column
//                   tiles, 64 x 224 accumulators per wave (AGPRs; one wave per SIMD);
//            C = 1: column 8 r + s (r = 7 and s = 7 dummies): patch[r][2q + s .. 2q + s + 3], an
//                   8-byte read aligned only for even q -- odd pixels read a second copy of the
//                   patch stored two elements earlier; 2 column tiles, 64 x 64 per wave;
//   * at the end the waves' tiles are summed in LDS in wave order, and each block writes its partial
//     of the real columns to a slab row (no atomics: deterministic) that
//     stem_wgrad_reduce_kernel adds into dw [64][7][7][Creal] in a fixed order.
#pragma once

struct StemWgradArgs {
  const bf16_t* x;   // [N][IH][IW][C]
  const bf16_t* dy;  // [N][OH][OW][64]
  float* slab;       // [gridDim][64 * 49 * Creal]
  unsigned x_bytes, dy_bytes;
  int N, IH, IW, OH, OW, Creal;
  int tiles_per_row, total_tiles;
};

template <int C>
struct StemWgradCfg {
  static constexpr int NW = C == 4 ? 4 : 8;                  // waves per block (C = 4: one per SIMD)
  static constexpr int NT = C == 4 ? 7 : 2;                  // 32-column GEMM tiles
  static constexpr int NCOL = NT * 32;
  static constexpr int ROWS = C == 4 ? 7 : 8;                // patch rows (C = 1: + a zero row r = 7)
  static constexpr int ROWB = C == 4 ? kStemPC * 8 : 144;    // bytes per patch row (C = 1: 70 x 2, 8-B aligned)
  static constexpr int COPY = C == 4 ? 1 : 2;                // patch copies (C = 1: + the 2-element shift)
  static constexpr int PB = ROWS * ROWB * COPY;              // patch bytes per buffer
  static constexpr int DYB = 32 * 128;                       // DY tile bytes
  static constexpr int STAGE = DYB + PB;
  static constexpr int WAVE_LDS = 2 * STAGE;
  static constexpr int LPL = (ROWS * kStemPC + 63) / 64;     // patch items per lane
  static constexpr int LDS_MAIN = NW * WAVE_LDS;
  static constexpr int LDS_RED = 64 * NCOL * 4;
  static constexpr int LDS = LDS_MAIN > LDS_RED ? LDS_MAIN : LDS_RED;
};

template <int C>
__global__ __launch_bounds__(StemWgradCfg<C>::NW * 64) __attribute__((amdgpu_waves_per_eu(1, C == 4 ? 1 : 2)))
void conv_stem_wgrad_kernel(StemWgradArgs a) {
  using Cfg = StemWgradCfg<C>;
  constexpr int NW = Cfg::NW, NT = Cfg::NT, NCOL = Cfg::NCOL, ROWS = Cfg::ROWS, ROWB = Cfg::ROWB;
  constexpr int PB = Cfg::PB, DYB = Cfg::DYB, STAGE = Cfg::STAGE, LPL = Cfg::LPL;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  char* const wbase = smem + wid * Cfg::WAVE_LDS;  // stage b: DY at wbase + b*STAGE, patch after it

  typedef typename std::conditional<C == 4, u32x2, unsigned short>::type item_t;
  struct Set {
    u32x4 dy[4];
    item_t px[LPL];
  };
  const int per_img = a.OH * a.tiles_per_row;
  const int P = a.OH * a.OW;
  // buffer loads: rows past the image edge and patch pixels outside the image read zeros through an
  // out-of-range offset (no branches)
  const __amdgpu_buffer_rsrc_t rsx = __builtin_amdgcn_make_buffer_rsrc((void*)a.x, (short)0, (int)a.x_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t rsd = __builtin_amdgcn_make_buffer_rsrc((void*)a.dy, (short)0, (int)a.dy_bytes, 0x00020000);
  auto load_tile = [&](int t, Set& S) {
    if (t >= a.total_tiles) return;
    const int img = t / per_img, rem = t - img * per_img;
    const int oh = rem / a.tiles_per_row, ow0 = (rem - oh * a.tiles_per_row) * 32;
    const int dbase = (img * P + oh * a.OW + ow0) * 128;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int u = lane + 64 * i, r = u >> 3, cc = u & 7;
      S.dy[i] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(
                                             rsd, ow0 + r < a.OW ? dbase + r * 128 + cc * 16 : (int)kOOB, 0, 0));
    }
    const int y0 = 2 * oh - 3, x0 = 2 * ow0 - 3, base = img * a.IH;
#pragma unroll
    for (int i = 0; i < LPL; ++i) {
      const int u = lane + 64 * i;
      const int g = u / kStemPC, col = u - g * kStemPC;
      const int yy = y0 + g, xx = x0 + col;
      const bool ok = g < 7 && (unsigned)yy < (unsigned)a.IH && (unsigned)xx < (unsigned)a.IW;
      const int off = ok ? ((base + yy) * a.IW + xx) * (C * 2) : (int)kOOB;
      if constexpr (C == 4)
        S.px[i] = __builtin_bit_cast(u32x2, __builtin_amdgcn_raw_buffer_load_b64(rsx, off, 0, 0));
      else
        S.px[i] = __builtin_amdgcn_raw_buffer_load_b16(rsx, off, 0, 0);
    }
  };
  auto store_tile = [&](int b, const Set& S) {
    char* st = wbase + b * STAGE;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int u = lane + 64 * i, r = u >> 3, cc = u & 7;
      *reinterpret_cast<u32x4*>(st + r * 128 + ((cc ^ tn_swz<128>(r)) << 4)) = S.dy[i];
    }
    char* ps = st + DYB;
#pragma unroll
    for (int i = 0; i < LPL; ++i) {
      const int u = lane + 64 * i;
      if (u < ROWS * kStemPC) {
        const int g = u / kStemPC, col = u - g * kStemPC;
        if constexpr (C == 4) {
          *reinterpret_cast<item_t*>(ps + g * ROWB + col * 8) = S.px[i];
        } else {
          *reinterpret_cast<item_t*>(ps + g * ROWB + col * 2) = S.px[i];
          if (col >= 2) *reinterpret_cast<item_t*>(ps + ROWS * ROWB + g * ROWB + (col - 2) * 2) = S.px[i];
        }
      }
    }
  };

  f32x16 acc[2][NT];
#pragma unroll
  for (int m = 0; m < 2; ++m)
#pragma unroll
    for (int n = 0; n < NT; ++n)
#pragma unroll
      for (int v = 0; v < 16; ++v) acc[m][n][v] = 0.f;

  // tr-read lane geometry (as conv_wgrad_halo_kernel): group g = lane>>4, t16 = 4 q4 + pq; the lane
  // points at GEMM row (pixel) 16 ks + tr_row (+ 4), columns tr_col .. tr_col + 3 of a 32-column tile
  const int g4 = lane >> 4, t16 = lane & 15, q4 = t16 >> 2, pq = t16 & 3;
  const int tr_row = (g4 >> 1) * 8 + q4;
  const int tr_col = (g4 & 1) * 16 + 4 * pq;
  typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

  const int stride = gridDim.x * NW;
  // one tile from buffer b; the next tile's loads are in flight meanwhile (a second set in flight
  // spilled the 64 x 224 accumulator kernel)
  auto tile = [&](int t, int b, Set& nxt) {
    load_tile(t + stride, nxt);
    wave_lds_sync();
    const char* As = wbase + b * STAGE;
    const char* Ps = As + DYB;
    // all fragments of a k-step are read before its MFMAs, the next k-step's while they run
    // (sched_barrier fences; one wave per SIMD has no other wave to hide the LDS latency behind)
    auto tr8 = [&](const char* p0, const char* p1) -> bf16x8 {
      const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(p0));
      const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(p1));
      const short tmp[8] = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      return __builtin_bit_cast(bf16x8, tmp);
    };
    bf16x8 fa[2][2], fb[2][NT];
    auto load_frags = [&](int ks) {
      const int row = 16 * ks + tr_row;  // and row + 4 (same swizzle: tn_swz<128> looks at bit 1)
#pragma unroll
      for (int m = 0; m < 2; ++m) {
        const int c = m * 32 + tr_col;
        const char* a0 = As + row * 128 + (((c >> 3) ^ tn_swz<128>(row)) << 4) + (c & 7) * 2;
        fa[ks][m] = tr8(a0, a0 + 4 * 128);
      }
#pragma unroll
      for (int n = 0; n < NT; ++n) {
        if constexpr (C == 4) {  // column tile n = patch row r; tap s = tr_col / 4
          const int s = tr_col >> 2;
          fb[ks][n] = tr8(Ps + n * ROWB + (2 * row + s) * 8, Ps + n * ROWB + (2 * (row + 4) + s) * 8);
        } else {  // columns 32 n + tr_col: r = 4 n + tr_col / 8, s0 = tr_col % 8 (0 or 4)
          const int r = 4 * n + (tr_col >> 3), s0 = tr_col & 7;
          // pixel q: elements 2q + s0 .. + 3; odd q from the copy shifted by two elements
          const char* base = Ps + (row & 1) * ROWS * ROWB + r * ROWB;
          fb[ks][n] = tr8(base + (2 * row + s0 - 2 * (row & 1)) * 2, base + (2 * (row + 4) + s0 - 2 * (row & 1)) * 2);
        }
      }
    };
    load_frags(0);
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      if (ks == 0) load_frags(1);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int n = 0; n < NT; ++n)
#pragma unroll
        for (int m = 0; m < 2; ++m)
          acc[m][n] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[ks][m], fb[ks][n], acc[m][n], 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);
    }
    if (t + stride < a.total_tiles) {
      wave_lds_sync();
      store_tile(b ^ 1, nxt);
    }
  };

  int t = xcd_remap(blockIdx.x, gridDim.x) * NW + wid;
  Set sn;
  if (t < a.total_tiles) {
    load_tile(t, sn);
    store_tile(0, sn);
  }
  for (int b = 0; t < a.total_tiles; t += stride, b ^= 1) tile(t, b, sn);

  // ---- sum the waves' tiles in LDS in wave order (deterministic), then this block's slab row ----
  float* red = reinterpret_cast<float*>(smem);  // [64][NCOL]
  const int frow = lane & 31, fhalf = lane >> 5;
  for (int w = 0; w < NW; ++w) {
    __syncthreads();
    if (wid == w) {
#pragma unroll
      for (int m = 0; m < 2; ++m)
#pragma unroll
        for (int n = 0; n < NT; ++n)
#pragma unroll
          for (int v = 0; v < 16; ++v) {
            const int k = m * 32 + (v & 3) + 8 * (v >> 2) + 4 * fhalf;
            float* q = red + k * NCOL + n * 32 + frow;
            *q = w == 0 ? acc[m][n][v] : *q + acc[m][n][v];
          }
    }
  }
  __syncthreads();
  const int per_k = 49 * a.Creal;
  float* dst = a.slab + (size_t)blockIdx.x * 64 * per_k;
  for (int e = tid; e < 64 * per_k; e += NW * 64) {
    const int k = e / per_k, rem = e - k * per_k;
    const int rs = rem / a.Creal, c = rem - rs * a.Creal;
    const int r = rs / 7, s = rs - r * 7;
    const int col = C == 4 ? r * 32 + s * 4 + c : r * 8 + s;
    dst[e] = red[k * NCOL + col];
  }
}

// dw[i] += sum_b slab[b][i] in a fixed order: 64 columns x 16 block groups per 1024-thread block
__global__ __launch_bounds__(1024) void stem_wgrad_reduce_kernel(const float* __restrict__ slab, int nslab, int n,
                                                                 float* __restrict__ dw) {
  __shared__ float part[16][64];
  const int col = threadIdx.x & 63, grp = threadIdx.x >> 6;
  const int i = blockIdx.x * 64 + col;
  float s = 0.f;
  if (i < n) {
#pragma unroll 4
    for (int b = grp; b < nslab; b += 16) s += slab[(size_t)b * n + i];
  }
  part[grp][col] = s;
  __syncthreads();
  if (grp == 0 && i < n) {
    float t = 0.f;
#pragma unroll
    for (int q = 0; q < 16; ++q) t += part[q][col];
    dw[i] += t;
  }
}

template <int C>
static size_t stem_wgrad_lds_bytes() {
  return (size_t)StemWgradCfg<C>::LDS;
}
