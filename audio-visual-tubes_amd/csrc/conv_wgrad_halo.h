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
// Forms.  Nine taps per block (avt_set_wgrad_halo(1)): each wave RW output channels x 9 of the 18
// 32-column subtiles.  Slower than the tap-gather kernel (230-320 vs 450-820 TFLOP/s at the trunk shapes):
// a wave tile of 64 x 288 needs 288 accumulator registers (the compiler shuffles them through
// v_accvgpr moves, SQ_INSTS_VALU/SQ_INSTS_MFMA = 33), and the 32 x 288 tile reads each B fragment in 4
// waves (1.1 KB of LDS per MFMA).  One filter row per block (ROW3; avt_set_wgrad_halo(2), and the
// default for K = 64, the layer-1 convs): a block owns 64 output channels x the 3 taps of filter row fr x
// 64 channels, stages the DY tile and only the patch rows row fr reads (R x (CW + 2) rows), and each of
// its 2 waves holds 64 x 96 (3 taps x one 32-channel half; 96 accumulator registers, two waves per SIMD,
// 2 A + 3 B fragment reads per 6 MFMAs).  What made it fast is the address arithmetic, not the tile:
// windows only, so every fragment row is fixed per lane; DMA offsets = per-tile scalar base + fixed
// per-lane offset; the k loop unrolled by the ring depth so every LDS address is a per-lane register +
// immediate (VALU per k-tile ~110 -> ~45: layer-1 356 -> 493 (vision) and 411 -> 610 (audio) TFLOP/s
// including the slab reduce; the kernel alone 671 / 715 TFLOP/s against 486 / 523 for the tap-gather
// kernel on the same box).
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
  MagicDiv div_w, div_tiles, div_wcols;
};

// WM x 2 waves.  ROW3 = false: each wave RW output channels x 9 of the 18 column subtiles: RW = 64 (2 x 9
// accumulator tiles = 288 registers per lane, one wave per SIMD) or 32 (9 tiles, 144 registers: two waves per
// SIMD -- two blocks per CU).  ROW3 = true (RW = 64): the block owns one filter row fr (3 taps) and stages only
// the patch rows that row reads (the "strip": PR - 2 PW rows); each wave 64 output channels x 3 taps x one
// 32-channel half = 6 accumulator tiles, 2 A + 3 B fragment reads per 6 MFMAs.  BM = RW * WM
template <int WM, int NST, int PRMAX, int RW = 64, bool ROW3 = false, int KG = 1, bool PF = false>
__global__ __launch_bounds__(WM * 2 * KG * 64) __attribute__((amdgpu_waves_per_eu(RW == 64 && !ROW3 ? 1 : 2, RW == 64 && !ROW3 ? 1 : 2)))
void conv_wgrad_halo_kernel(WgradHaloArgs a) {
  static_assert(!ROW3 || RW == 64, "ROW3 form: 64 rows per wave");
  static_assert(KG == 1 || ROW3, "k groups: ROW3 form only");
  static_assert(!PF || (ROW3 && NST >= 4), "PF: ROW3 form, a 4+ stage ring");
  constexpr int NW = WM * 2, BM = WM * RW, TR = RW / 32;
  constexpr int NS = ROW3 ? 3 : 9;                 // column subtiles per wave
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
  __shared__ __attribute__((aligned(16))) char smem[KG * NST * STAGE + 1024];
  char* junk = smem + KG * NST * STAGE;

  const int tid = threadIdx.x, lane = tid & 63;
  // KG k groups of NW waves: group kg takes the block's k-tiles kg, kg + KG, ... on its own ring; the
  // groups' partial tiles are summed in LDS (fixed order) before the one store per block
  const int wall = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int kg = wall / NW, wid = wall - kg * NW;
  char* ring = smem + kg * NST * STAGE;
  const int wm = wid % WM, hn = wid / WM;  // RW-row slice of BM, half of the 18 column subtiles
  constexpr int NFR = ROW3 ? 3 : 1;  // filter rows split over blocks
  const int ct_count = a.C / 64, per_split = (a.K / BM) * ct_count * NFR;
  const int lin = xcd_remap(blockIdx.x, gridDim.x);
  const int split = lin / per_split;
  int rest = lin - split * per_split;
  const int fr = ROW3 ? rest % 3 : 0;
  rest /= NFR;
  const int mt = rest / ct_count, ct = rest - mt * ct_count;
  const int m0 = mt * BM, c0 = ct * 64;
  const int kt_begin = split * a.kt_per_split;
  const int kt_end = min(a.nkt, kt_begin + a.kt_per_split);
  if (kt_begin >= kt_end) return;  // never with a slab: the plan leaves no empty split
  const int nk = kt_end - kt_begin;
  const int H = a.H, W = a.W, HW = H * W;
  const int PRS = ROW3 ? a.PR - 2 * a.PW : a.PR;  // patch rows staged (ROW3: logical rows fr*PW .. +PRS)

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
    p_in[i] = q < PINSTR && pr < PRS;
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
    if (!ROW3 && a.raster) {
      t.p0 = ti * 32;
      t.y0 = (int)magic_div((unsigned)t.p0, a.div_w);
      t.x0 = 0;
      t.yo = t.y0 - 1;
      t.xo = -1;
    } else {
      const int band = (int)magic_div((unsigned)ti, a.div_wcols);
      t.p0 = 0;
      t.y0 = band * a.R;
      t.x0 = (ti - band * a.wcols) * a.CW;
      t.yo = t.y0 - 1;
      t.xo = t.x0 - 1;
    }
    return t;
  };

  // ROW3 (windows only): a DMA lane's source offset is a per-tile scalar base plus a fixed per-lane offset
  unsigned a_lo[AI];
  int p_lo[PIW];
#pragma unroll
  for (int i = 0; i < AI; ++i) a_lo[i] = (unsigned)((a_ky[i] * W + a_kx[i]) * a.K * 2) + a_colB[i];
#pragma unroll
  for (int i = 0; i < PIW; ++i) p_lo[i] = (p_dy[i] * W + p_dx[i]) * a.C * 2 + (int)p_colB[i];

  // ROW3: LDS byte addresses as integers; p_dy3 folds the lane's "past the patch" flag into its row (out of any image)
  const unsigned ring_lds = (unsigned)(size_t)(lds_void_t*)ring, junk_lds = (unsigned)(size_t)(lds_void_t*)junk;
  int p_dy3[PIW];
#pragma unroll
  for (int i = 0; i < PIW; ++i) p_dy3[i] = p_in[i] ? p_dy[i] : (1 << 20);
  // ROW3: the issue cursor -- image, band and window column of the next tile to issue (tiles go out in order,
  // KG apart): advanced with scalar adds, not two magic divisions per tile (the scalar instruction stream, one
  // per CU, was ~7 per MFMA)
  int cur_n = 0, cur_band = 0, cur_wc = 0;
  const int bands = ROW3 ? a.tiles_img / a.wcols : 1;
  if constexpr (ROW3) {
    const int kt0 = kt_begin + kg;
    cur_n = (int)magic_div((unsigned)kt0, a.div_tiles);
    const int ti = kt0 - cur_n * a.tiles_img;
    cur_band = (int)magic_div((unsigned)ti, a.div_wcols);
    cur_wc = ti - cur_band * a.wcols;
  }
  auto issue = [&](int kt, int stage) {
    char* As = ring + stage * STAGE;
    char* Ps = As + A_BYTES;
    const bool live = kt < kt_end;
    if constexpr (ROW3) {
      const int y0 = cur_band * a.R, x0 = cur_wc * a.CW;
      const unsigned abase = (unsigned)(((cur_n * H + y0) * W + x0) * a.K * 2);
      // a tile past the split's end: every bound fails (no per-load `live` term)
      const int py0 = live ? y0 - 1 + fr : H, hy = live ? H - y0 : 0, wx = W - x0, xo = x0 - 1;
      const int pbase = ((cur_n * H + py0) * W + xo) * a.C * 2;
      const unsigned sa = ring_lds + (unsigned)(stage * STAGE);
      cur_wc += KG;  // the next tile of this group (past the split's end: bases unused, the loads are out of range)
      while (cur_wc >= a.wcols) {
        cur_wc -= a.wcols;
        if (++cur_band == bands) {
          cur_band = 0;
          ++cur_n;
        }
      }
#pragma unroll
      for (int i = 0; i < AI; ++i) {
        const bool ok = a_ky[i] < hy && a_kx[i] < wx;
        buf_lds16_at(rs_dy, sa + (unsigned)((wid * AI + i) * 1024), ok ? abase + a_lo[i] : kOOB);
      }
#pragma unroll
      for (int i = 0; i < PIW; ++i) {
        const int q = i * NW + wid;
        const bool pok = (unsigned)(py0 + p_dy3[i]) < (unsigned)H && (unsigned)(xo + p_dx[i]) < (unsigned)W;
        buf_lds16_at(rs_x, q < PINSTR ? sa + (unsigned)(A_BYTES + q * 1024) : junk_lds, pok ? (unsigned)(pbase + p_lo[i]) : kOOB);
      }
      return;
    }
    const Tile t = tile_of(live ? kt : kt_begin);
#pragma unroll
    for (int i = 0; i < AI; ++i) {
      int y, x;
      bool ok;
      if (!ROW3 && a.raster) {
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
      const int py = t.yo + fr + p_dy[i], px = t.xo + p_dx[i];
      const bool pok = live && p_in[i] && (unsigned)py < (unsigned)H && (unsigned)px < (unsigned)W;
      buf_lds16(rs_x, q < PINSTR ? Ps + q * 1024 : junk,
                pok ? (unsigned)(((t.n * H + py) * W + px) * a.C * 2) + p_colB[i] : kOOB);
    }
  };

  f32x16 acc[TR][NS];
#pragma unroll
  for (int i = 0; i < TR; ++i)
#pragma unroll
    for (int s = 0; s < NS; ++s)
#pragma unroll
      for (int v = 0; v < 16; ++v) acc[i][s][v] = 0.f;

  // tr-read lane geometry (as conv_tn_pipe_kernel): group g = lane>>4, t = lane&15 = 4q + pq
  const int g = lane >> 4, t16 = lane & 15, q4 = t16 >> 2, pq = t16 & 3;
  const int tr_row = (g >> 1) * 8 + q4;        // + 16*ks + 4*rr
  const int tr_col = (g & 1) * 16 + 4 * pq;
  const int a_sw = tn_swz<AROWB>(q4);
  typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

#pragma unroll
  for (int s = 0; s < NST - 1; ++s) issue(kt_begin + s * KG + kg, s);

  // patch row (tap centre) of a fragment pixel k = 16 ks + tr_row + 4 rr (j = 2 ks + rr); the window
  // form's rows are the same for every k-tile (ROW3 plans only windows: computed once)
  auto pixel_rows = [&](int kt, int* pb) {
    const Tile t = tile_of(kt);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int kk = 16 * (j >> 1) + tr_row + 4 * (j & 1);
      int y, x;
      if (!ROW3 && a.raster) {
        const int p = min(t.p0 + kk, HW - 1);  // pixels past the image: any in-patch row (DY is 0)
        y = (int)magic_div((unsigned)p, a.div_w);
        x = p - y * W;
      } else {
        y = t.y0 + (kk >> a.lcw);
        x = t.x0 + (kk & (a.CW - 1));
      }
      pb[j] = (y - t.yo) * a.PW + (x - t.xo);
    }
  };
  int pb[4];
  if (ROW3) pixel_rows(kt_begin, pb);

  // one k-tile: rs = the stage it reads, is = the stage the DMA issued here fills
  auto step = [&](int k, int rs, int is) {
    wait_vmcnt<(NST - 2) * LPT>();
    ring_barrier();
    const char* As = ring + rs * STAGE;
    const char* Ps = As + A_BYTES;
    if (!ROW3) pixel_rows(kt_begin + k, pb);
    bf16x8 af[2][TR];
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int i = 0; i < TR; ++i) {
        const int c = wm * RW + i * 32 + tr_col;
        const char* a0 = As + (ks * 16 + tr_row) * AROWB + ((c >> 3) ^ a_sw) * 16 + (c & 7) * 2;
        s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(a0));
        s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(a0 + 4 * AROWB));
        short tmp[8] = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        af[ks][i] = __builtin_bit_cast(bf16x8, tmp);
      }
    issue(kt_begin + (k + NST - 1) * KG + kg, is);  // the stage read at step k-1: all waves passed
    // all 9 B fragments of a k-step are read before its 18 MFMAs, and the next k-step's reads are
    // issued while those run (two fragment buffers): one wave per SIMD has no other wave to hide
    // the LDS latency behind
    bf16x8 bfr[2][NS];
    // subtile s -> tap and channel half; row displacement from the logical patch row of the tap centre
    // (ROW3: the staged strip starts at logical row fr*PW, so a tap of row fr sits PW rows up)
    auto sub = [&](int s, int& tap, int& hh, int& disp) {
      if (ROW3) {
        tap = fr * 3 + s;
        hh = hn;
        disp = -a.PW + (s - 1);
      } else {
        const int cs = hn * 9 + s;  // column subtile: tap cs/2, channel half cs%2
        tap = cs >> 1;
        hh = cs & 1;
        const int dyt = tap / 3 - 1, dxt = tap - (tap / 3) * 3 - 1;
        disp = dyt * a.PW + dxt;
      }
    };
    auto load_b = [&](int ks, int buf) {
#pragma unroll
      for (int s = 0; s < NS; ++s) {
        int tap, hh, disp;
        sub(s, tap, hh, disp);
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
      for (int s = 0; s < NS; ++s)
#pragma unroll
        for (int i = 0; i < TR; ++i)
          acc[i][s] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[ks][i], bfr[ks][s], acc[i][s], 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);
    }
  };
  if constexpr (PF) {
    // PF: each step's wait + barrier also publish the NEXT tile, whose first k-step fragments are read
    // behind this step's MFMAs -- a step's MFMAs start right after its barrier instead of one LDS round
    // trip later (ROW3 has only 2 k-steps per barrier).  One tile fewer in flight on the DMA side.
    auto load_a = [&](const char* As, int ks, bf16x8* dst) {
#pragma unroll
      for (int i = 0; i < TR; ++i) {
        const int c = wm * RW + i * 32 + tr_col;
        const char* a0 = As + (ks * 16 + tr_row) * AROWB + ((c >> 3) ^ a_sw) * 16 + (c & 7) * 2;
        s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(a0));
        s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(a0 + 4 * AROWB));
        dst[i] = __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
      }
    };
    auto load_b = [&](const char* Ps, int ks, bf16x8* dst) {
#pragma unroll
      for (int s = 0; s < NS; ++s) {  // ROW3: tap fr*3 + s, channel half hn, PW rows up (see step)
        const int disp = -a.PW + (s - 1);
        const int rlo = pb[2 * ks] + disp, rhi = pb[2 * ks + 1] + disp;
        const int c = hn * 32 + tr_col;
        const char* b0 = Ps + rlo * 128 + (((c >> 3) ^ tn_swz<128>(rlo)) << 4) + (c & 7) * 2;
        const char* b1 = Ps + rhi * 128 + (((c >> 3) ^ tn_swz<128>(rhi)) << 4) + (c & 7) * 2;
        s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(b0));
        s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(b1));
        dst[s] = __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
      }
    };
    bf16x8 a0n[TR], b0n[NS];  // k-step 0 fragments of the step about to run
    const int nloop = (nk + KG - 1) / KG;
    wait_vmcnt<(NST - 2) * LPT>();  // tile 0 (every wave's, after the barrier)
    ring_barrier();
    load_a(ring, 0, a0n);
    load_b(ring + A_BYTES, 0, b0n);
    auto step_pf = [&](int k, int rs, int is) {
      wait_vmcnt<(NST - 3) * LPT>();  // tiles k and k+1
      ring_barrier();
      const char* As = ring + rs * STAGE;
      bf16x8 a1[TR], b1[NS];
      load_a(As, 1, a1);
      issue(kt_begin + (k + NST - 1) * KG + kg, is);  // the stage read at step k-1 (and prefetched before)
      load_b(As + A_BYTES, 1, b1);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int s = 0; s < NS; ++s)
#pragma unroll
        for (int i = 0; i < TR; ++i)
          acc[i][s] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0n[i], b0n[s], acc[i][s], 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int s = 0; s < NS; ++s)
#pragma unroll
        for (int i = 0; i < TR; ++i)
          acc[i][s] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1[i], b1[s], acc[i][s], 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);
      if (k + 1 < nloop) {  // the next tile: published by this step's barrier
        const char* An = ring + ((rs + 1) % NST) * STAGE;
        load_a(An, 0, a0n);
        load_b(An + A_BYTES, 0, b0n);
      }
    };
    for (int k0 = 0; k0 < nloop; k0 += NST) {
#pragma unroll
      for (int u = 0; u < NST; ++u)
        if (k0 + u < nloop) step_pf(k0 + u, u, (u + NST - 1) % NST);
    }
  } else if constexpr (ROW3) {
    // stages as compile-time constants: every LDS address is a fixed per-lane offset + immediate.  Every
    // group runs the same number of steps (a group past its last tile reads zeros): the barriers pair up
    const int nloop = (nk + KG - 1) / KG;
    for (int k0 = 0; k0 < nloop; k0 += NST) {
#pragma unroll
      for (int u = 0; u < NST; ++u)
        if (k0 + u < nloop) step(k0 + u, u, (u + NST - 1) % NST);
    }
  } else {
    for (int k = 0; k < nk; ++k) step(k, k % NST, (k + NST - 1) % NST);
  }
  wait_vmcnt<0>();
  if constexpr (KG > 1) {
    // groups 1..KG-1 pass their accumulators through LDS (lane-contiguous: conflict-free); group 0 adds
    // them in group order
    constexpr int GF = NW * TR * NS * 16 * 64;  // floats per group
    static_assert((KG - 1) * GF * 4 <= KG * NST * STAGE, "k-group exchange fits the rings");
    float* xs = reinterpret_cast<float*>(smem);
    ring_barrier();  // every wave's last fragment reads are done
    if (kg > 0) {
      float* xg = xs + (kg - 1) * GF;
#pragma unroll
      for (int i = 0; i < TR; ++i)
#pragma unroll
        for (int s = 0; s < NS; ++s)
#pragma unroll
          for (int v = 0; v < 16; ++v) xg[(((wid * TR + i) * NS + s) * 16 + v) * 64 + lane] = acc[i][s][v];
    }
    __syncthreads();
    if (kg > 0) return;
    for (int g2 = 0; g2 < KG - 1; ++g2) {
      const float* xg = xs + g2 * GF;
#pragma unroll
      for (int i = 0; i < TR; ++i)
#pragma unroll
        for (int s = 0; s < NS; ++s)
#pragma unroll
          for (int v = 0; v < 16; ++v) acc[i][s][v] += xg[(((wid * TR + i) * NS + s) * 16 + v) * 64 + lane];
    }
  }
  // ---- epilogue: DW[m][tap][c] (slab: this split's partial, plain stores; else fp32 atomics) ----
  const int ldw = 9 * a.C;
  float* dst = a.slab ? a.slab + (size_t)split * a.K * ldw : a.dw;
  const int frow = lane & 31, fhalf = lane >> 5;
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    int tap, hh;
    if (ROW3) {
      tap = fr * 3 + s;
      hh = hn;
    } else {
      const int cs = hn * 9 + s;
      tap = cs >> 1;
      hh = cs & 1;
    }
    const int col = tap * a.C + c0 + hh * 32 + frow;
#pragma unroll
    for (int i = 0; i < TR; ++i)
#pragma unroll
      for (int v = 0; v < 16; ++v) {
        const int row = m0 + wm * RW + i * 32 + (v & 3) + 8 * (v >> 2) + 4 * fhalf;
        if (a.slab)
          dst[(size_t)row * ldw + col] = acc[i][s][v];
        else
          atomicAdd(dst + (size_t)row * ldw + col, acc[i][s][v]);
      }
  }
}

// Ordered two-pass reduction of the split partials (deterministic): entry e (e < count) is
// slab[e * step * n ...].  blockIdx.y = group of per_group consecutive entries, summed in order; with
// several groups each group's sum overwrites its first entry (pass 1), with one group it is added to dw
// (pass 2 runs over the group heads: step = per_group of pass 1)
__global__ __launch_bounds__(256) void wgrad_halo_reduce_kernel(float* __restrict__ slab, int count, int step,
                                                                int per_group, long long n, float* __restrict__ dw) {
  const long long i = ((long long)blockIdx.x * blockDim.x + threadIdx.x) * 4;
  if (i >= n) return;
  const int s0 = blockIdx.y * per_group, s1 = min(count, s0 + per_group);
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  int s = s0;
  for (; s + 8 <= s1; s += 8) {  // eight loads in flight, added in entry order
    f32x4 v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = *reinterpret_cast<const f32x4*>(slab + (size_t)(s + u) * step * n + i);
#pragma unroll
    for (int u = 0; u < 8; ++u) acc += v[u];
  }
  for (; s < s1; ++s) acc += *reinterpret_cast<const f32x4*>(slab + (size_t)s * step * n + i);
  if (gridDim.y == 1) {
    f32x4 d = *reinterpret_cast<const f32x4*>(dw + i);
    *reinterpret_cast<f32x4*>(dw + i) = d + acc;
  } else {
    *reinterpret_cast<f32x4*>(slab + (size_t)s0 * step * n + i) = acc;
  }
}
