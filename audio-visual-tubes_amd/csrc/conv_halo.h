// Halo-reuse implicit-GEMM 3x3 / stride-1 / pad-1 convolution (fwd and dgrad), NHWC bf16, MFMA.
// Included by conv_gemm.hip inside namespace avt (after conv_nt_pipe.h: wait_vmcnt, xcd_remap,
// buf_lds16, swz_rb, kOOB, GemmNTParams, MODE_*).
//
// For a 3x3 stride-1 "same" conv the output grid equals the input grid, so output pixel m reads
// input pixel m + (dy*W + dx) for its 9 taps (dy, dx in -1..1; image borders masked).  A tile of BM
// consecutive output pixels [m0, m0+BM) therefore reads only the contiguous input range
// [m0 - W - 1, m0 + BM + W + 1): its "patch".  The tap-gather kernel (conv_nt_pipe_kernel) moves
// every input row through L2 -> LDS once per tap (9x); this kernel moves the patch once per 64-channel
// chunk and reads the 9 tap-shifted windows out of LDS, so the activation fill per chunk drops from
// 9*BM rows to BM + 2W + 2 rows (1.2-1.9x BM at the trunk shapes).  The k loop walks (chunk, tap),
// tap fastest: per step one weight tile [BN x 64] streams through an NSTB-stage ring, and 1/9 of
// the NEXT chunk's patch streams into the other half of a double-buffered patch (pieces issued only
// once the step reading the previous chunk's last tap has passed, so the buffer is free).
// Masked taps (image border, m >= M) read a zero row.  Dgrad (stride 1) is the same loop over dy
// with the flipped taps and the [C][(r,s,k)] weight operand.
#pragma once

struct HaloArgs {
  unsigned act_bytes, w_bytes;
  int W, H;              // image (= output) width / height
  int tap_disp[9];       // input-pixel displacement dy*W + dx of each tap
  int tap_dy[9], tap_dx[9];
  int tap_w[9];          // weight tap index of each listed tap
  // split-K (short grids: a few clips per GPU): ksplit blocks per output tile, each over cps of the
  // 64-channel chunks; each stores its fp32 partial tile to part (register order, write-through) and
  // takes a ticket on cnt[tile]; the last to arrive sums the ksplit partials in split order (so the
  // result does not depend on arrival order), resets the ticket and runs the epilogue
  int ksplit, cps;
  float* part;           // [tiles][ksplit][BM*BN]
  int* cnt;              // [tiles], zero between launches
  int dbg;               // -DAVT_DIAG build only (AVT_HALO_DBG; wrong results): 1 weight DMA out of range (issued,
                         // no traffic), 2 patch DMA likewise, 4 no per-tap barrier, 8 no MFMA, 16 no epilogue stores
  // Conv3d 3x3x3 / stride 1 / pad 1 (OPT bit 4): T frames per clip; frame f = (pixel / (H W)) % T
  int T;
  MagicDiv div_hw, div_t;
};
#ifdef AVT_DIAG
#define HALO_DBG(bit) (ha.dbg & (bit))
#else
#define HALO_DBG(bit) false
#endif

// (store_wt16 / load_wt16, the write-through split-K hand-off: conv_nt_pipe.h)

// LDS chunk swizzle of a 128-B row (8 16-B chunks): the 32x32x16 fragment reads (lanes 0-31 one chunk of 32
// consecutive rows) are conflict-free with chunk ^ ((row >> 1) & 7) -- for ANY first row, which the tap shifts of
// the patch make arbitrary (exhaustive check over the 16 offsets)
__device__ __forceinline__ int halo_swz(int row) { return (row >> 1) & 7; }

// WM x WN waves, each TM x TN 32x32 output blocks (v_mfma_f32_32x32x16_bf16): BM = WM*TM*32 rows, BN = WN*TN*32
// columns.  (A 16x16x32 form and a SIMD-partner stagger of the 8-wave tiles were measured in rounds 3-4 and
// removed in round 5: DESIGN.md section 6.)
// NSTB: weight-ring stages.  PRMAX: patch rows the LDS is sized for (>= BM + 2W + 2).
// EPI: a dgrad with the BatchNorm-backward store epilogue (conv_epi.h; GemmNTParams::bx set).
// LDS of the main loop (two patch buffers + the weight ring): two blocks per CU when two fit in 160 KB
template <int WN, int TN, int NSTB, int PRMAX, int TPS = 1>
constexpr int halo_blocks_per_cu() {
  return 2 * (2 * (PRMAX * 128 + 1024) + NSTB * TPS * WN * TN * 32 * 128 + 4096) <= 160 * 1024 ? 2 : 1;
}

// PREF (1, 2): fragments are read PREF k-steps ahead, across the per-step barrier (see the main loop).  Bench-only
// (tools/halo_bench.hip, profiles/r5_halo_bench_pref.txt): +1..6 % on the layer4 shapes with a 4-stage ring, -3..5 %
// on layer2; libavt launches PREF = 0
// OPT (A/B bits, tools/halo_bench.hip): 1 = waves NW/2 .. NW-1 at s_setprio 1 through the main loop
// (MI355X_MICROARCH.md "static priority for the younger half"); 2 = two taps per step: one counted wait + block
// barrier per two taps instead of per tap, NSTB = 2 ring stages of two weight tiles each (see the main loop);
// 4 = Conv3d 3x3x3 / stride 1 / pad 1 (fwd): every 64-channel chunk is three "virtual chunks", one per temporal
// tap dt = -1, 0, 1, each with its own patch -- the input rows [m0 - W - 1 + dt H W, ...) -- read by its 9 spatial
// taps (weight taps 9 (dt + 1) .. 9 (dt + 1) + 8).  Since the output and input grids coincide (T' = T), an output row
// in frame f reads frame f + dt of its own clip wherever the spatial tap is valid, except across the clip ends: a
// patch row is zeroed at the DMA (kOOB) when dt = +1 and its pixel is a clip's frame 0, or dt = -1 and frame T - 1 --
// rows only an output frame -1 or T would read.  The per-lane spatial tap masks are the 2-D ones.
template <int MODE, int WM, int WN, int TM, int TN, int NSTB, int PRMAX, bool EPI = false, bool SPLIT = false,
          int PREF = 0, int OPT = 0>
__global__ __launch_bounds__(WM * WN * 64, (halo_blocks_per_cu<WN, TN, NSTB, PRMAX, (OPT & 2) ? 2 : 1>())) void conv_halo_kernel(
    GemmNTParams p, HaloArgs ha) {
  // fragment geometry: FM x FN MFMA tiles of FR rows per wave, KS k-steps of KD per 64-channel tap
  constexpr int FR = 32, FM = TM, FN = TN;
  constexpr int KD = 16;
  constexpr int NW = WM * WN, NT = NW * 64;
  constexpr int BM = WM * TM * 32, BN = WN * TN * 32;
  constexpr int BK = 64, RB = 128, RPI = 8;  // 64 channels = one 128-B row; 8 rows per 1 KiB DMA
  constexpr int BR = BN / (NW * RPI);        // weight-tile DMA instructions per wave per step
  static_assert(BR >= 1 && BR * NW * RPI == BN, "weight tile / wave split");
  constexpr int PINSTR = (PRMAX + RPI - 1) / RPI;  // DMA instructions per patch
  static_assert(NSTB >= 2 && NSTB <= 5, "NSTB");
  constexpr int NPIECE = 10 - NSTB;  // patch pieces ride on taps NSTB-1 .. 8
  constexpr int AP = (PINSTR + NPIECE * NW - 1) / (NPIECE * NW);  // patch instructions per wave per piece
  constexpr int ABUF = PRMAX * RB + 1024;  // a patch buffer + 8 zero rows (masked taps read them)
  constexpr int BSTAGE = BN * RB;
  constexpr int TPS = (OPT & 2) ? 2 : 1;  // taps (weight tiles) per ring stage
  constexpr int CT_LD = BN + 8;
  constexpr int EPI_BYTES = BM * CT_LD * 2;
  constexpr int MAIN = 2 * ABUF + NSTB * TPS * BSTAGE;
  constexpr int SMEM = (MAIN > EPI_BYTES ? MAIN : EPI_BYTES);
  static_assert(PRMAX % RPI == 0, "PRMAX");
  static_assert(SMEM + 2 * WM * BN * 4 <= 160 * 1024, "LDS budget of a CU");
  __shared__ __attribute__((aligned(16))) char smem[SMEM + 2 * WM * BN * 4];
  char* zrow = smem + PRMAX * RB;  // buffer 0's zero rows: also the sink of the constant-count dummy DMAs
  float* red = reinterpret_cast<float*>(smem + SMEM);  // [2][WM][BN] epilogue scratch

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid / WN, wn = wid % WN;
  const int nnt = p.Ng / BN;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  // split-K: the split is the slowest index, so an XCD's blocks share one K range of the weights
  const int ntile = SPLIT ? gridDim.x / ha.ksplit : gridDim.x;
  const int split = SPLIT ? bid / ntile : 0, tile = bid - split * ntile;
  const int mt = tile / nnt, nt = tile - mt * nnt;
  const int m0 = mt * BM, n0 = nt * BN;
  const int W = ha.W, H = ha.H, hw = W * H;
  const int pre = W + 1;  // patch row of output pixel m0 is pre
  const int PR = BM + 2 * pre;
  constexpr int VT = (OPT & 4) ? 3 : 1;  // virtual chunks (temporal taps) per 64-channel chunk
  static_assert(VT == 1 || (MODE == MODE_FWD && !SPLIT && !EPI), "Conv3d halo: forward, no split-K");
  const int nchunk = (SPLIT ? ha.cps : p.IC / BK) * VT;  // (virtual) chunks of this block's K range
  const int cbase = SPLIT ? split * ha.cps : 0;
  const int S = nchunk * 9;

  if (tid < 128) reinterpret_cast<u32x4*>(zrow + (tid >> 6) * ABUF)[tid & 63] = u32x4{0u, 0u, 0u, 0u};
  __syncthreads();

  const __amdgpu_buffer_rsrc_t rsa = __builtin_amdgcn_make_buffer_rsrc((void*)p.act, (short)0, (int)ha.act_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t rsb = __builtin_amdgcn_make_buffer_rsrc((void*)p.wmat, (short)0, (int)ha.w_bytes, 0x00020000);

  // ---- DMA lane geometry: lane -> (row within the 8-row instruction, 16-B chunk) ----
  const int lrow = lane >> 3, pchunk = lane & 7;
  // patch instruction q (of PINSTR) covers patch rows 8q..8q+7; row pr = 8q + lrow holds input pixel
  // m0 - pre + pr, its chunk (pchunk ^ swz) stored at lane position pchunk (source-side swizzle)
  // vc: (virtual) chunk index, cbase included
  auto patch_voff = [&](int q, int vc) -> unsigned {
    const int chunk_c = vc / VT;
    const int dt = vc - chunk_c * VT - (VT == 3 ? 1 : 0);
    const int pr = q * RPI + lrow;
    const int pix = m0 - pre + pr + dt * hw;
    if (q >= PINSTR || pr >= PR || pix < 0 || pix >= p.M) return kOOB;
    if constexpr (VT == 3) {
      if (dt != 0) {  // across a clip end (see above)
        const unsigned f = magic_div((unsigned)pix, ha.div_hw);
        const unsigned fr = f - magic_div(f, ha.div_t) * (unsigned)ha.T;
        if (fr == (dt > 0 ? 0u : (unsigned)(ha.T - 1))) return kOOB;
      }
    }
    const int lc = pchunk ^ halo_swz(pr);
    return (unsigned)(((long long)pix * p.IC + chunk_c * BK + lc * 8) * 2);
  };
  // weight-tile offset of (virtual) chunk vc (cbase included), spatial tap tn: the Conv3d weight operand is
  // [K][kt][r][s][C], kt = dt + 1
  auto w_off = [&](int vc, int tn) -> unsigned {
    const int chunk_c = vc / VT, kt = vc - chunk_c * VT;
    return (unsigned)(((kt * 9 + ha.tap_w[tn]) * p.IC + chunk_c * BK) * 2);
  };
  unsigned b_off[BR];
#pragma unroll
  for (int i = 0; i < BR; ++i) {
    const int row = (wid * BR + i) * RPI + lrow;
    const int lc = pchunk ^ halo_swz(row);
    b_off[i] = (unsigned)(((size_t)(n0 + row) * p.Kg + lc * 8) * 2);
  }
  // ---- fragment rows of this lane: rows wm*(BM/WM) + i*FR + (lane % FR); per row a 9-bit tap mask.  The
  //      lane's k chunk within a k-step: fhalf (lanes 32-63 take k 8..15) ----
  const int frow = lane & (FR - 1), fhalf = lane / FR;
  unsigned fmask[FM];
#pragma unroll
  for (int i = 0; i < FM; ++i) {
    const int row = wm * (BM / WM) + i * FR + frow;
    const int m = m0 + row;
    const bool ok = m < p.M;
    const int mm = ok ? m : 0;
    const int n = mm / hw, rem = mm - n * hw;
    const int oh = rem / W, ow = rem - oh * W;
    unsigned mk = 0;
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      const int y = oh + ha.tap_dy[t], x = ow + ha.tap_dx[t];
      mk |= (ok && y >= 0 && y < H && x >= 0 && x < W ? 1u : 0u) << t;
    }
    fmask[i] = mk;
  }
  // ---- per-lane A row address of every (tap, row block), relative to the patch buffer: masked taps read
  //      the buffer's zero rows at the bank position the real row would have; the fragment-chunk swizzle
  //      g = fhalf ^ (pr >> 1) & 7 sits in bits 4-6 (rows are 128 B), so a k-step's chunk is one XOR.
  //      B: per (column block, k-step) offset in a ring stage.  With the tap loop unrolled the k loop is
  //      ds_read + MFMA (tap, stage and buffer are compile-time; a rolled (chunk, tap) loop spent ~11
  //      other instructions per MFMA) ----
  unsigned arow[9][FM];
#pragma unroll
  for (int t = 0; t < 9; ++t)
#pragma unroll
    for (int i = 0; i < FM; ++i) {
      const int pr = wm * (BM / WM) + i * FR + frow + pre + ha.tap_disp[t];
      const bool v = (fmask[i] >> t) & 1u;
      arow[t][i] = (unsigned)((v ? pr * RB : PRMAX * RB + (pr & 7) * RB) | ((fhalf ^ halo_swz(pr)) << 4));
    }
  constexpr int KS = BK / KD;
  int boffs[FN][KS];
#pragma unroll
  for (int j = 0; j < FN; ++j)
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      const int row = wn * (BN / WN) + j * FR + frow;
      boffs[j][ks] = row * RB + (((2 * ks + fhalf) ^ halo_swz(row)) << 4);
    }

  // ---- issue of step (chunk cn, tap tn): weight tile into ring stage (cn*9+tn) % NSTB, and for tn >=
  //      NSTB-1 one piece of chunk cn+1's patch into patch buffer (cn+1) & 1 (which held chunk cn-1, whose
  //      last reader has passed) ----
  auto issue = [&](int cn, int tn, int stage) {
    char* Bs = smem + 2 * ABUF + stage * BSTAGE;
    const bool live = cn < nchunk;
    const unsigned boff = w_off(cbase * VT + cn, tn);
#pragma unroll
    for (int i = 0; i < BR; ++i)
      buf_lds16(rsb, Bs + (wid * BR + i) * 1024, (live && !HALO_DBG(1)) ? b_off[i] + boff : kOOB);
    if (tn >= NSTB - 1) {
      char* Ab = smem + ((cn + 1) & 1) * ABUF;
      const bool alive = live && cn + 1 < nchunk;
#pragma unroll
      for (int a = 0; a < AP; ++a) {
        const int q = ((tn - (NSTB - 1)) * AP + a) * NW + wid;  // pieces 0..6 of the patch
        const bool inrange = q < PINSTR;
        // out-of-range instructions still issue (constant vmcnt): zeros into the zero area
        buf_lds16(rsa, inrange ? Ab + q * 1024 : zrow,
                  (alive && inrange && !HALO_DBG(2)) ? patch_voff(q, cbase * VT + cn + 1) : kOOB);
      }
    }
  };

  // accumulators: AV fp32 per lane per MFMA tile; element v of tile (i, j) is output row acc_row(i, v),
  // column wn*(BN/WN) + j*FR + frow
  constexpr int AV = 16;
  using acc_t = f32x16;
  auto acc_row = [&](int i, int v) -> int { return wm * (BM / WM) + i * FR + (v & 3) + 8 * (v >> 2) + 4 * fhalf; };
  acc_t acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j)
#pragma unroll
      for (int v = 0; v < AV; ++v) acc[i][j][v] = 0.f;

  // prologue: chunk 0's whole patch, then steps 0 .. NSTB-2 (two taps per step: step 0's two weight tiles)
  for (int q = wid; q < PINSTR; q += NW) buf_lds16(rsa, smem + q * 1024, patch_voff(q, cbase * VT));
  if constexpr (TPS == 1) {
#pragma unroll
    for (int j = 0; j < NSTB - 1; ++j) issue(0, j, j);
  }

  if constexpr ((OPT & 1) != 0) {
    if (wid >= NW / 2) __builtin_amdgcn_s_setprio(1);
  }
  bf16x8 af[2][FM], bfr[2][FN];
  auto mma = [&](int buf) {
    if (HALO_DBG(8)) return;
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[buf][i], bfr[buf][j], acc[i][j], 0, 0, 0);
      }
  };
  if constexpr (TPS == 2) {
    // Two taps per step.  A chunk pair (c, c+1; nchunk is even) is 18 taps = 9 steps; step j of a pair multiplies
    // pair taps 2j and 2j+1 (pair tap T is tap T % 9 of chunk c + T / 9, whose patch sits in buffer T / 9).  Ring:
    // 2 stages of two weight tiles; after barrier j a step issues step j+1's two tiles into the stage step j-1 read,
    // and one quarter of a patch: steps 0-3 chunk c+1's (buffer 1: its last reader, the previous pair's step 8, is
    // behind barrier 0), steps 5-8 chunk c+2's (buffer 0: last read at step 4).  A step's own patch piece may stay in
    // flight past the next step's wait, except where the next step reads that patch (steps 4 and 0).  The weight
    // tiles get one step (two taps) of latency cover, as the one-tap 3-stage ring gives them; the barriers halve.
    // Accumulation order: the same as the one-tap loop (bitwise equal results).
    static_assert(NSTB == 2 && !PREF && !SPLIT, "two taps per step: a 2-stage ring, no PREF / split-K");
    constexpr int AP2 = (PINSTR + 4 * NW - 1) / (4 * NW);  // patch instructions per wave per quarter
    auto issue_w = [&](int cn, int tn, char* Bs) {
      const bool live = cn < nchunk;
      const unsigned boff = w_off(cbase * VT + cn, tn);
#pragma unroll
      for (int i = 0; i < BR; ++i)
        buf_lds16(rsb, Bs + (wid * BR + i) * 1024, (live && !HALO_DBG(1)) ? b_off[i] + boff : kOOB);
    };
    auto issue_piece = [&](int cn, int piece) {  // quarter `piece` of chunk cn's patch into buffer cn & 1
      char* Ab = smem + (cn & 1) * ABUF;
      const bool alive = cn < nchunk;
#pragma unroll
      for (int a = 0; a < AP2; ++a) {
        const int q = (piece * AP2 + a) * NW + wid;
        const bool inrange = q < PINSTR;
        buf_lds16(rsa, inrange ? Ab + q * 1024 : zrow,
                  (alive && inrange && !HALO_DBG(2)) ? patch_voff(q, cbase * VT + cn) : kOOB);
      }
    };
    char* const Bring = smem + 2 * ABUF;
    issue_w(0, 0, Bring);
    issue_w(0, 1, Bring + BSTAGE);
    for (int c = 0; c < nchunk; c += 2) {
      const int sp = (c >> 1) & 1;  // ring stage of this pair's step 0 (9 steps per pair)
#pragma unroll
      for (int j = 0; j < 9; ++j) {
        if (j == 0 || j == 4 || j == 5)
          wait_vmcnt<0>();
        else
          wait_vmcnt<AP2>();
        if (!HALO_DBG(4)) ring_barrier();
        const int stage = (sp + j) & 1;
        const char* Bs = Bring + stage * 2 * BSTAGE;
        auto load_frags = [&](int kk, int buf) {  // k-step kk of this step: tap 2j + kk / KS, k-step kk % KS
          const int T = 2 * j + kk / KS, ks = kk % KS;
          const char* Ab = smem + (T / 9) * ABUF;
          const char* Bt = Bs + (kk / KS) * BSTAGE;
#pragma unroll
          for (int i = 0; i < FM; ++i)
            af[buf][i] = *reinterpret_cast<const bf16x8*>(Ab + (arow[T % 9][i] ^ (unsigned)(ks << 5)));
#pragma unroll
          for (int jj = 0; jj < FN; ++jj) bfr[buf][jj] = *reinterpret_cast<const bf16x8*>(Bt + boffs[jj][ks]);
        };
        load_frags(0, 0);
        {
          char* Bn = Bring + (stage ^ 1) * 2 * BSTAGE;
          const int T0 = 2 * (j + 1), T1 = T0 + 1;
          issue_w(c + T0 / 9, T0 % 9, Bn);
          issue_w(c + T1 / 9, T1 % 9, Bn + BSTAGE);
          if (j < 4)
            issue_piece(c + 1, j);
          else if (j >= 5)
            issue_piece(c + 2, j - 5);
        }
#pragma unroll
        for (int kk = 0; kk < 2 * KS; ++kk) {
          if (kk + 1 < 2 * KS) {
            load_frags(kk + 1, (kk + 1) & 1);
            __builtin_amdgcn_sched_barrier(0);
          }
          mma(kk & 1);
          if (kk + 1 < 2 * KS) __builtin_amdgcn_sched_barrier(0);
        }
      }
    }
  } else if constexpr (PREF) {
    // PREF: each step's barrier also publishes the NEXT step's weight tile (and, at a chunk's last tap, the whole
    // next patch), so the next step's first k-step fragments are read during this step's last MFMAs and the
    // MFMAs of a step start right at its barrier -- no LDS round trip between the barrier and the first MFMA.
    // Stages: step s reads stage s % NSTB, step s+1's tile sits landed in the next one, the DMA issued at step s
    // fills step s+NSTB-1's (the stage step s-1 read: every wave retired those reads at barrier s).  The DMA has
    // NSTB-2 steps to land (one at NSTB 3).  Accumulation order: unchanged (bitwise the same results).
    static_assert(NSTB >= 3 && (KS & 1) == 0, "PREF: a 3+ stage ring, even k-steps");
    // the step-0 wait and barrier (weights of steps 0 .. NSTB-2 and chunk 0's patch were issued above)
    // (taps 1 .. NSTB-2 carry no patch piece: only their weight tiles may be outstanding)
    wait_vmcnt<(NSTB - 2) * BR>();
    ring_barrier();
    // PREF + 1 fragment buffers; k-step kk = t * KS + ks of a chunk uses buffer kk % NB (36 k-steps per chunk:
    // NB divides it, so the buffer is a compile-time constant)
    constexpr int NB = PREF + 1;
    static_assert((9 * KS) % NB == 0 && PREF <= KS, "PREF");
    bf16x8 pa[NB][FM], pb[NB][FN];
    auto frags = [&](const char* Ab, const char* Bs, int t, int ks, int buf) {
#pragma unroll
      for (int i = 0; i < FM; ++i)
        pa[buf][i] = *reinterpret_cast<const bf16x8*>(Ab + (arow[t][i] ^ (unsigned)(ks << 5)));
#pragma unroll
      for (int j = 0; j < FN; ++j) pb[buf][j] = *reinterpret_cast<const bf16x8*>(Bs + boffs[j][ks]);
    };
    auto mmab = [&](int buf) {
      if (HALO_DBG(8)) return;
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j) {
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(pa[buf][i], pb[buf][j], acc[i][j], 0, 0, 0);
        }
    };
#pragma unroll
    for (int kk = 0; kk < PREF; ++kk) frags(smem, smem + 2 * ABUF, 0, kk, kk);
    for (int c = 0; c < nchunk; ++c) {
      const char* Ab = smem + (c & 1) * ABUF;          // patch buffer of this chunk
      const char* Abn = smem + ((c + 1) & 1) * ABUF;   // ... and of the next (its first k-steps' prefetch)
#pragma unroll
      for (int t = 0; t < 9; ++t) {
        const int stage = NSTB == 3 ? t % 3 : (c * 9 + t) % NSTB;
        const int nstage = NSTB == 3 ? (t + 1) % 3 : (c * 9 + t + 1) % NSTB;
        // wait: step s+1's weights have landed once only what was issued after them may be outstanding --
        // step s+1's own patch piece (relaxed, as below) and the issues of steps s+2 .. s+NSTB-2
        int pieces = ((t + 1) % 9 >= NSTB - 1) ? 1 : 0;
#pragma unroll
        for (int j = 2; j <= NSTB - 2; ++j) pieces += ((t + j) % 9 >= NSTB - 1) ? 1 : 0;
        constexpr int W0 = (NSTB - 3) * BR;
        if (pieces == 0)
          wait_vmcnt<W0>();
        else if (pieces == 1)
          wait_vmcnt<W0 + AP>();
        else if (pieces == 2)
          wait_vmcnt<W0 + 2 * AP>();
        else
          wait_vmcnt<W0 + 3 * AP>();
        ring_barrier();
        const char* Bs = smem + 2 * ABUF + stage * BSTAGE;
        const char* Bn = smem + 2 * ABUF + nstage * BSTAGE;
        const bool more = t < 8 || c + 1 < nchunk;  // a next step exists (wave-uniform)
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) {
          const int kk = t * KS + ks, tk = kk + PREF;  // k-step read now (PREF ahead), in this chunk's numbering
          if (tk < 9 * KS) {
            if (tk / KS == t)
              frags(Ab, Bs, t, tk % KS, tk % NB);
            else
              frags(Ab, Bn, t + 1, tk % KS, tk % NB);
          } else if (more) {
            frags(Abn, Bn, 0, tk - 9 * KS, tk % NB);
          }
          __builtin_amdgcn_sched_barrier(0);
          mmab(kk % NB);
          __builtin_amdgcn_sched_barrier(0);
          if (ks == 0) {  // the stage step s-1 read (every wave passed barrier s)
            const int tn = t + NSTB - 1 >= 9 ? t + NSTB - 1 - 9 : t + NSTB - 1;
            const int cn = t + NSTB - 1 >= 9 ? c + 1 : c;
            issue(cn, tn, (stage + NSTB - 1) % NSTB);
            __builtin_amdgcn_sched_barrier(0);
          }
        }
      }
    }
  } else
  for (int c = 0; c < nchunk; ++c) {
    const char* Ab = smem + (c & 1) * ABUF;  // patch buffer of this chunk
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      {
        // step s = c*9 + t: its stage is s % NSTB -- (c + t) % 2 for NSTB 2 (9 odd), t % 3 for 3
        const int stage = NSTB == 2 ? (c + t) & 1 : NSTB == 3 ? t % 3 : (c * 9 + t) % NSTB;
        // step s's weight tile has landed once only what was issued after it may be outstanding: step s's own
        // patch piece (issued right after its weights; a piece of the NEXT chunk, read only from that chunk's
        // first step, whose wait -- tap 0 carries no piece -- covers every piece issued before it) and steps
        // s+1 .. s+NSTB-2: BR weight loads each + AP for those with a tap >= NSTB-1 (t is a constant after
        // unrolling).  Leaving the own piece outstanding gives every piece one more step to land (the patch
        // is the operand that misses L2).  -DAVT_HALO_STRICT_WAIT: the step's own piece is waited for too.
        int pieces = 0;
#ifndef AVT_HALO_STRICT_WAIT
        pieces += (t >= NSTB - 1) ? 1 : 0;
#endif
#pragma unroll
        for (int j = 1; j <= NSTB - 2; ++j) pieces += ((t + j) % 9 >= NSTB - 1) ? 1 : 0;
        constexpr int W0 = (NSTB - 2) * BR;
        if (pieces == 0)
          wait_vmcnt<W0>();
        else if (pieces == 1)
          wait_vmcnt<W0 + AP>();
        else if (pieces == 2)
          wait_vmcnt<W0 + 2 * AP>();
        else if (pieces == 3)
          wait_vmcnt<W0 + 3 * AP>();
        else
          wait_vmcnt<W0 + 4 * AP>();
        if (!HALO_DBG(4)) ring_barrier();
        const char* Bs = smem + 2 * ABUF + stage * BSTAGE;
        auto load_frags = [&](int ks, int buf) {
#pragma unroll
          for (int i = 0; i < FM; ++i)
            af[buf][i] = *reinterpret_cast<const bf16x8*>(Ab + (arow[t][i] ^ (unsigned)(ks << 5)));
#pragma unroll
          for (int j = 0; j < FN; ++j) bfr[buf][j] = *reinterpret_cast<const bf16x8*>(Bs + boffs[j][ks]);
        };
        load_frags(0, 0);
        {  // the ring stage read at step s-1; every wave has passed that
          const int tn = t + NSTB - 1 >= 9 ? t + NSTB - 1 - 9 : t + NSTB - 1;
          const int cn = t + NSTB - 1 >= 9 ? c + 1 : c;
          const int stn = NSTB == 2 ? (stage ^ 1) : (stage + NSTB - 1) % NSTB;
          issue(cn, tn, stn);
        }
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) {
          if (ks + 1 < KS) {
            load_frags(ks + 1, (ks + 1) & 1);
            __builtin_amdgcn_sched_barrier(0);
          }
          mma(ks & 1);
          if (ks + 1 < KS) __builtin_amdgcn_sched_barrier(0);
        }
      }
    }
  }
  wait_vmcnt<0>();
  if constexpr ((OPT & 1) != 0) __builtin_amdgcn_s_setprio(0);
  __syncthreads();

  if constexpr (SPLIT) {
    // partial tile in register order: (wave, i, j, quarter) x 64 lanes x 16 B -- 1 KiB per instruction
    const __amdgpu_buffer_rsrc_t rsp = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(ha.part + (size_t)tile * ha.ksplit * BM * BN), (short)0, (int)(ha.ksplit * BM * BN * 4), 0x00020000);
    auto poff = [&](int s, int i, int j, int q) -> unsigned {
      return (unsigned)((((s * NW + wid) * TM + i) * TN + j) * 4 + q) * 1024u + lane * 16u;
    };
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int q = 0; q < 4; ++q)
          store_wt16(rsp, poff(split, i, j, q),
                     f32x4{acc[i][j][4 * q], acc[i][j][4 * q + 1], acc[i][j][4 * q + 2], acc[i][j][4 * q + 3]});
    wait_vmcnt<0>();  // this wave's partial has left for memory
    __syncthreads();  // ... and every other wave's
    int* flag = reinterpret_cast<int*>(red);
    if (tid == 0) flag[0] = __hip_atomic_fetch_add(ha.cnt + tile, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();
    const int ticket = flag[0];
    __syncthreads();  // every wave has read it before the epilogue reuses the scratch
    if (ticket != ha.ksplit - 1) return;  // not the last split of this tile
    if (tid == 0) ha.cnt[tile] = 0;        // ready for the next launch
    // sum the partials in split order (own one from registers): arrival order does not change the bits
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        f32x16 tot;
#pragma unroll
        for (int v = 0; v < 16; ++v) tot[v] = 0.f;
        for (int s = 0; s < ha.ksplit; ++s) {
          if (s == split) {
            tot += acc[i][j];
          } else {
#pragma unroll
            for (int q = 0; q < 4; ++q) {
              const f32x4 v4 = load_wt16(rsp, poff(s, i, j, q));
#pragma unroll
              for (int e = 0; e < 4; ++e) tot[4 * q + e] += v4[e];
            }
          }
        }
        acc[i][j] = tot;
      }
  }

  // ---- epilogue (as conv_nt_pipe_kernel): BN partial statistics, bf16 tile through LDS, (+ add) ----
  const int rows_valid = min(BM, p.M - m0);
  if (MODE == MODE_FWD && p.stats != nullptr) {
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      float sm = 0.f;
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int v = 0; v < AV; ++v)
          if (acc_row(i, v) < rows_valid) sm += acc[i][j][v];
#pragma unroll
      for (int o = FR; o < 64; o <<= 1) sm += __shfl_xor(sm, o, 64);
      if (lane < FR) red[wm * BN + wn * (BN / WN) + j * FR + lane] = sm;
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const int cc = wn * (BN / WN) + j * FR + frow;
      float tot = 0.f;
#pragma unroll
      for (int k = 0; k < WM; ++k) tot += red[k * BN + cc];
      const float mean = tot / (float)rows_valid;
      float q = 0.f;
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int v = 0; v < AV; ++v) {
          const float d = acc[i][j][v] - mean;
          if (acc_row(i, v) < rows_valid) q += d * d;
        }
#pragma unroll
      for (int o = FR; o < 64; o <<= 1) q += __shfl_xor(q, o, 64);
      if (lane < FR) red[WM * BN + wm * BN + cc] = q;
    }
    __syncthreads();
    // this row tile's own slot (avt_common.h): (M + BM - 1) / BM slots, plain stores
    bn_write_header(p.stats, (p.M + BM - 1) / BM, 0, mt == 0 && n0 == 0);
    double* acc_slot = bn_fwd_slots(p.stats) + (size_t)mt * p.Ng * 3;
    for (int cc = tid; cc < BN; cc += NT) {
      double sd = 0.0, m2 = 0.0;
#pragma unroll
      for (int k = 0; k < WM; ++k) {
        sd += (double)red[k * BN + cc];
        m2 += (double)red[WM * BN + k * BN + cc];
      }
      double* a = acc_slot + (size_t)(n0 + cc) * 3;
      a[0] = sd;
      a[1] = m2;
      a[2] = sd * sd / (double)rows_valid;
    }
  }
  bf16_t* Ct = reinterpret_cast<bf16_t*>(smem);
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j)
#pragma unroll
      for (int v = 0; v < AV; ++v) Ct[acc_row(i, v) * CT_LD + wn * (BN / WN) + j * FR + frow] = f2bf(acc[i][j][v]);
  __syncthreads();
  if (!HALO_DBG(16))
    epi_store<NT, BM, BN, EPI>(p, Ct, CT_LD, n0, rows_valid, mt, (p.M + BM - 1) / BM,
                               [&](int r) -> size_t { return (size_t)(m0 + r); },
                        reinterpret_cast<float*>(smem));
}
