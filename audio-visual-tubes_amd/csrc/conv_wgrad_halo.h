// Halo-reuse wgrad for the 3x3 / stride-1 / pad-1 convolutions (most of ResNet-18's weight-gradient
// FLOPs).  Included by conv_gemm.hip inside namespace avt after conv_tn_pipe.h (uses wait_vmcnt,
// xcd_remap, buf_lds16, kOOB, MagicDiv, magic_div, tn_swz).
//
//   DW[k][t][c] += sum_pix DY[pix][k] * X[pix + disp_t][c]      (t = 3x3 tap, disp_t = dy*W + dx)
//
// conv_tn_pipe_kernel streams the gathered X operand through LDS once per tap (9x per input row).
// Here a block owns BM output channels x ALL 9 taps x one 64-channel chunk (576 GEMM columns): per
// k-tile of 32 output pixels it stages the DY tile [32 pix][BM] and the input "patch" those pixels'
// 3x3 neighbourhoods cover -- [patch rows][64 ch], zero-padded at the image border -- and every tap
// reads its B fragments from the patch at a row displacement, so the X fill per k-tile drops from
// 9 x 32 rows to the patch (60-160 rows).  A k-tile is either 32 consecutive pixels of one image
// (raster; narrow maps, patch = (rows spanned + 2) x (W + 2)) or an R x CW window (R*CW = 32;
// wide maps, patch = (R + 2) x (CW + 2)).  Pixels past the image read zero DY rows; patch pixels
// outside the image are zero (out-of-range buffer loads), so no tap needs a mask.  Fragments are
// read with ds_read_b64_tr_b16 from per-lane row addresses (the transposition works on whatever
// rows the lanes point at).  Each wave (one per SIMD): 64 output channels x 9 of the 18 32-column
// subtiles -- 18 accumulator tiles, each A fragment used 9x and each B fragment 2x, which keeps the
// LDS reads at ~0.6 KB per MFMA (the 1 x 9 form needed 1.1 KB and was LDS-bound).  Split-K over
// k-tiles; partials go to an fp32 slab (plain stores) reduced by wgrad_halo_reduce_kernel, or fp32
// atomics without a workspace.
//
// STATUS: correct (tests/test_kernels_gpu.py runs every 3x3/s1 wgrad case through it) but SLOWER
// than the tap-gather kernel (230-320 vs 450-820 TFLOP/s at the trunk shapes), so it is off by
// default (avt_set_wgrad_halo / AVT_WGRAD_HALO=1).  Why: a wave tile of 64 x 288 needs 288 fp32
// accumulator registers; with 256 AGPRs the compiler shuffles accumulators through v_accvgpr moves
// (~16 per MFMA in the k loop, SQ_INSTS_VALU/SQ_INSTS_MFMA = 33).  The 32 x 288 tile (144
// registers, 2 waves/SIMD) has no spill but reads each B fragment in 4 waves (1.1 KB of LDS per
// MFMA: LDS-bound).  The 9-tap N dimension does not split into a <= 256-register wave tile with
// fragment reuse on both operands; a 32-channel-chunk / 3-tap-per-wave layout is the next try.
#pragma once

struct WgradHaloArgs {
  const bf16_t* dy;  // [N][H][W][K]
  const bf16_t* x;   // [N][H][W][C]
  float* dw;         // [K][9][C] fp32 (accumulated into)
  float* slab;       // non-null: split partials -> slab[split][K][9C]
  unsigned dy_bytes, x_bytes;
  int N, H, W, C, K;
  int raster;        // 1: k-tile = 32 consecutive pixels of one image; 0: R x CW window
  int R, CW, lcw;    // window shape (lcw = log2 CW)
  int wcols;         // windows per band (2-D)
  int tiles_img;     // k-tiles per image
  int PW, PR;        // patch row width / patch rows (pixels)
  int nkt, kt_per_split, splits;
  MagicDiv div_w, div_tiles;
};

// WM x 2 waves, one per SIMD (2 x 9 accumulator tiles = 288 registers per lane): BM = 64 WM
template <int WM, int NST, int PRMAX>
__global__ __launch_bounds__(WM * 2 * 64) __attribute__((amdgpu_waves_per_eu(1, 1)))
void conv_wgrad_halo_kernel(WgradHaloArgs a) {
  constexpr int NW = WM * 2, BM = WM * 64;
  constexpr int AROWB = BM * 2;                    // bytes per DY row (pixel)
  constexpr int A_RPI = 1024 / AROWB;              // DY rows per 1 KiB DMA instruction
  constexpr int A_BYTES = 32 * AROWB;
  constexpr int AI = A_BYTES / 1024 / NW;          // DY instructions per wave
  static_assert(AI * NW * 1024 == A_BYTES, "DY tile / wave split");
  constexpr int PINSTR = PRMAX / 8;                // patch instructions (8 rows of 128 B each)
  constexpr int PIW = (PINSTR + NW - 1) / NW;      // per wave (dummies past PINSTR)
  constexpr int P_BYTES = PRMAX * 128;
  constexpr int STAGE = A_BYTES + P_BYTES;
  constexpr int LPT = AI + PIW;
  static_assert(PRMAX % 8 == 0, "PRMAX");
  __shared__ __attribute__((aligned(16))) char smem[NST * STAGE + 1024];
  char* junk = smem + NST * STAGE;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid % WM, hn = wid / WM;  // 64-row slice of BM, half of the 18 column subtiles
  const int ct_count = a.C / 64, per_split = (a.K / BM) * ct_count;
  const int lin = xcd_remap(blockIdx.x, gridDim.x);
  const int split = lin / per_split, rest = lin - split * per_split;
  const int mt = rest / ct_count, ct = rest - mt * ct_count;
  const int m0 = mt * BM, c0 = ct * 64;
  const int kt_begin = split * a.kt_per_split;
  const int kt_end = min(a.nkt, kt_begin + a.kt_per_split);
  if (kt_begin >= kt_end) return;  // never with a slab: the plan leaves no empty split
  const int nk = kt_end - kt_begin;
  const int H = a.H, W = a.W, HW = H * W;

  const __amdgpu_buffer_rsrc_t rs_dy = __builtin_amdgcn_make_buffer_rsrc((void*)a.dy, (short)0, (int)a.dy_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t rs_x = __builtin_amdgcn_make_buffer_rsrc((void*)a.x, (short)0, (int)a.x_bytes, 0x00020000);

  // ---- DMA lane geometry ----
  int a_row[AI], a_ky[AI], a_kx[AI];  // pixel k of the DY rows this lane fills
  unsigned a_colB[AI];
#pragma unroll
  for (int i = 0; i < AI; ++i) {
    a_row[i] = (wid * AI + i) * A_RPI + lane / (AROWB / 16);
    const int pc = lane % (AROWB / 16);
    a_colB[i] = (unsigned)((m0 + ((pc ^ tn_swz<AROWB>(a_row[i])) * 8)) * 2);
    a_ky[i] = a_row[i] >> a.lcw;
    a_kx[i] = a_row[i] & (a.CW - 1);
  }
  int p_dy[PIW], p_dx[PIW];
  bool p_in[PIW];
  unsigned p_colB[PIW];
#pragma unroll
  for (int i = 0; i < PIW; ++i) {
    const int q = i * NW + wid;
    const int pr = q * 8 + lane / 8;
    p_in[i] = q < PINSTR && pr < a.PR;
    const int py = pr / a.PW;
    p_dy[i] = py;
    p_dx[i] = pr - py * a.PW;
    p_colB[i] = (unsigned)((c0 + (((lane & 7) ^ tn_swz<128>(pr)) * 8)) * 2);
  }

  // k-tile -> image n and patch origin (y_o, x_o); pixel k -> (y, x) (raster: from p0)
  struct Tile {
    int n, p0, y0, x0, yo, xo;
  };
  auto tile_of = [&](int kt) {
    Tile t;
    const unsigned n = magic_div((unsigned)kt, a.div_tiles);
    const int ti = kt - (int)n * a.tiles_img;
    t.n = (int)n;
    if (a.raster) {
      t.p0 = ti * 32;
      t.y0 = (int)magic_div((unsigned)t.p0, a.div_w);
      t.x0 = 0;
      t.yo = t.y0 - 1;
      t.xo = -1;
    } else {
      const int band = ti / a.wcols;
      t.p0 = 0;
      t.y0 = band * a.R;
      t.x0 = (ti - band * a.wcols) * a.CW;
      t.yo = t.y0 - 1;
      t.xo = t.x0 - 1;
    }
    return t;
  };

  auto issue = [&](int kt, int stage) {
    char* As = smem + stage * STAGE;
    char* Ps = As + A_BYTES;
    const bool live = kt < kt_end;
    const Tile t = tile_of(live ? kt : kt_begin);
#pragma unroll
    for (int i = 0; i < AI; ++i) {
      int y, x;
      bool ok;
      if (a.raster) {
        const int p = t.p0 + a_row[i];
        y = (int)magic_div((unsigned)p, a.div_w);
        x = p - y * W;
        ok = p < HW;
      } else {
        y = t.y0 + a_ky[i];
        x = t.x0 + a_kx[i];
        ok = y < H && x < W;
      }
      ok = ok && live;
      buf_lds16(rs_dy, As + (wid * AI + i) * 1024, ok ? (unsigned)(((t.n * H + y) * W + x) * a.K * 2) + a_colB[i] : kOOB);
    }
#pragma unroll
    for (int i = 0; i < PIW; ++i) {
      const int q = i * NW + wid;
      const int py = t.yo + p_dy[i], px = t.xo + p_dx[i];
      const bool pok = live && p_in[i] && (unsigned)py < (unsigned)H && (unsigned)px < (unsigned)W;
      buf_lds16(rs_x, q < PINSTR ? Ps + q * 1024 : junk,
                pok ? (unsigned)(((t.n * H + py) * W + px) * a.C * 2) + p_colB[i] : kOOB);
    }
  };

  f32x16 acc[2][9];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int s = 0; s < 9; ++s)
#pragma unroll
      for (int v = 0; v < 16; ++v) acc[i][s][v] = 0.f;

  // tr-read lane geometry (as conv_tn_pipe_kernel): group g = lane>>4, t = lane&15 = 4q + pq
  const int g = lane >> 4, t16 = lane & 15, q4 = t16 >> 2, pq = t16 & 3;
  const int tr_row = (g >> 1) * 8 + q4;        // + 16*ks + 4*rr
  const int tr_col = (g & 1) * 16 + 4 * pq;
  const int a_sw = tn_swz<AROWB>(q4);
  typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

#pragma unroll
  for (int s = 0; s < NST - 1; ++s) issue(kt_begin + s, s);

  for (int k = 0; k < nk; ++k) {
    wait_vmcnt<(NST - 2) * LPT>();
    ring_barrier();
    const char* As = smem + (k % NST) * STAGE;
    const char* Ps = As + A_BYTES;
    // patch row (tap centre) of this lane's 4 fragment pixels: k = 16 ks + tr_row + 4 rr
    int pb[4];
    {
      const Tile t = tile_of(kt_begin + k);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int kk = 16 * (j >> 1) + tr_row + 4 * (j & 1);
        int y, x;
        if (a.raster) {
          const int p = min(t.p0 + kk, HW - 1);  // pixels past the image: any in-patch row (DY is 0)
          y = (int)magic_div((unsigned)p, a.div_w);
          x = p - y * W;
        } else {
          y = t.y0 + (kk >> a.lcw);
          x = t.x0 + (kk & (a.CW - 1));
        }
        pb[j] = (y - t.yo) * a.PW + (x - t.xo);
      }
    }
    bf16x8 af[2][2];
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int c = wm * 64 + i * 32 + tr_col;
        const char* a0 = As + (ks * 16 + tr_row) * AROWB + ((c >> 3) ^ a_sw) * 16 + (c & 7) * 2;
        s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(a0));
        s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(a0 + 4 * AROWB));
        short tmp[8] = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        af[ks][i] = __builtin_bit_cast(bf16x8, tmp);
      }
    issue(kt_begin + k + NST - 1, (k + NST - 1) % NST);  // the stage read at step k-1: all waves passed
    // all 9 B fragments of a k-step are read before its 18 MFMAs, and the next k-step's reads are
    // issued while those run (two fragment buffers): one wave per SIMD has no other wave to hide
    // the LDS latency behind
    bf16x8 bfr[2][9];
    auto load_b = [&](int ks, int buf) {
#pragma unroll
      for (int s = 0; s < 9; ++s) {
        const int cs = hn * 9 + s;  // column subtile: tap cs/2, channel half cs%2
        const int tap = cs >> 1, hh = cs & 1;
        const int dyt = tap / 3 - 1, dxt = tap - (tap / 3) * 3 - 1;
        const int disp = dyt * a.PW + dxt;
        const int rlo = pb[2 * ks] + disp, rhi = pb[2 * ks + 1] + disp;
        const int c = hh * 32 + tr_col;
        const char* b0 = Ps + rlo * 128 + (((c >> 3) ^ tn_swz<128>(rlo)) << 4) + (c & 7) * 2;
        const char* b1 = Ps + rhi * 128 + (((c >> 3) ^ tn_swz<128>(rhi)) << 4) + (c & 7) * 2;
        s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(b0));
        s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(b1));
        short tmp[8] = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        bfr[buf][s] = __builtin_bit_cast(bf16x8, tmp);
      }
    };
    load_b(0, 0);
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      if (ks == 0) load_b(1, 1);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int s = 0; s < 9; ++s) {
        acc[0][s] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[ks][0], bfr[ks][s], acc[0][s], 0, 0, 0);
        acc[1][s] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[ks][1], bfr[ks][s], acc[1][s], 0, 0, 0);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  wait_vmcnt<0>();

  // ---- epilogue: DW[m][tap][c] (slab: this split's partial, plain stores; else fp32 atomics) ----
  const int ldw = 9 * a.C;
  float* dst = a.slab ? a.slab + (size_t)split * a.K * ldw : a.dw;
  const int frow = lane & 31, fhalf = lane >> 5;
#pragma unroll
  for (int s = 0; s < 9; ++s) {
    const int cs = hn * 9 + s;
    const int tap = cs >> 1, hh = cs & 1;
    const int col = tap * a.C + c0 + hh * 32 + frow;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int v = 0; v < 16; ++v) {
        const int row = m0 + wm * 64 + i * 32 + (v & 3) + 8 * (v >> 2) + 4 * fhalf;
        if (a.slab)
          dst[(size_t)row * ldw + col] = acc[i][s][v];
        else
          atomicAdd(dst + (size_t)row * ldw + col, acc[i][s][v]);
      }
  }
}

// dw[i] += sum_{s in this block's split group} slab[s][i]; blockIdx.y = split group (fp32 atomics
// across groups, a plain add for a single group): deep split counts stay parallel
__global__ __launch_bounds__(256) void wgrad_halo_reduce_kernel(const float* __restrict__ slab, int splits, int per_group,
                                                                long long n, float* __restrict__ dw) {
  const long long i = (blockIdx.x * 256LL + threadIdx.x) * 4;
  if (i >= n) return;
  const int s0 = blockIdx.y * per_group, s1 = min(splits, s0 + per_group);
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  for (int s = s0; s < s1; ++s) acc += *reinterpret_cast<const f32x4*>(slab + (size_t)s * n + i);
  if (gridDim.y == 1) {
    f32x4 d = *reinterpret_cast<const f32x4*>(dw + i);
    *reinterpret_cast<f32x4*>(dw + i) = d + acc;
  } else {
#pragma unroll
    for (int e = 0; e < 4; ++e) atomicAdd(dw + i + e, acc[e]);
  }
}
