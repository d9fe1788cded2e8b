// wgrad ("TN") implicit GEMM, LDS-DMA pipeline (C % 8 == 0).  Included by conv_gemm.hip inside
// namespace avt after conv_nt_pipe.h (uses GemmTNParams, buf_lds16, wait_vmcnt, kOOB).
//
//   DW[k_out][(r,s,c)] += sum_{pix} DY[pix][k_out] * X(pix; r,s,c)
//
// Both operands are pixel-major: a k-tile is 32 consecutive output pixels; the LDS images are
// [32 pix][BM] and [32 pix][BN] bf16 with unpadded rows whose 16-B chunks are XOR-swizzled
// (chunk ^ f(row)) so that the ds_read_b64_tr_b16 fragment reads are bank-conflict-free.  The
// images are filled with `buffer_load_dwordx4 ... lds` (lane-linear; the swizzle goes on the
// source chunk).  Each lane owns one fixed logical chunk (a fixed k_out block for DY, a fixed
// (r,s,c) patch column block for X); per k-tile it decomposes its pixel(s) with magic-number
// divisions.  NST-stage ring, NST-1 tiles in flight, split-K over blockIdx.y, fp32 atomics.
#pragma once

// (MagicDiv, make_magic, magic_div: avt_common.h)

struct GemmTNPipeParams {
  GemmTNParams p;
  MagicDiv div_pq, div_q;
  unsigned dy_bytes, x_bytes;
  float* slab;  // non-null: store the split's partial tile to slab[split][Mg][R*S*C] (plain stores)
  // FUSED: per-tile tickets (zero on entry, left zero) and the slab's bytes; the last block of a tile to take its
  // ticket sums the tile's `splits` partials in split order into DW (no separate reduce launch)
  int* cnt;
  unsigned slab_bytes;
  int splits;
};

template <int ROWB>
__device__ __forceinline__ int tn_swz(int row) {  // chunk XOR for a row of ROWB bytes
  return ROWB >= 256 ? ((row & 3) << 2) : (((row >> 1) & 1) << 2);
}

// 4 or 8 waves as WM x WN, each wave TM x TN tiles of 32x32 (8 waves need BM, BN >= 128).
// KG = 2: two such wave groups per block split the block's k range in halves, each through its own LDS
// ring, and meet in LDS at the end -- one partial tile per block instead of two (the split-K slab
// traffic, which dominates the short-batch wgrads, halves at the same number of waves)
// FUSED: the split-K slab is reduced by the last block of each tile (write-through partial stores, one agent-scope
// ticket per block, the last reads the partials back in split order -- the order wgrad_slab_reduce_native_kernel uses
// with G = 1, so the two paths give the same bits); every block of the grid takes a ticket, an empty k range included
template <int WM, int WN, int TM, int TN, int NST, int KG = 1, bool FUSED = false>
__global__ __launch_bounds__(WM * WN * 64 * KG) void conv_tn_pipe_kernel(GemmTNPipeParams pp) {
  constexpr int NW = WM * WN;  // waves per group
  static_assert(KG == 1 || KG == 2, "one or two k groups");
  static_assert(NW == 4 || NW == 8, "4 or 8 waves");
  constexpr int BM = WM * TM * 32, BN = WN * TN * 32;
  static_assert(BM == 64 || BM == 128 || BM == 256, "BM");
  static_assert(BN == 64 || BN == 128 || BN == 256, "BN");
  constexpr int AROWB = BM * 2, BROWB = BN * 2;          // bytes per pixel row
  constexpr int A_RPI = 1024 / AROWB, B_RPI = 1024 / BROWB;  // rows per 1 KiB instruction
  constexpr int AI = 32 / A_RPI / NW, BI = 32 / B_RPI / NW;  // instructions per wave per tile
  static_assert(AI >= 1 && BI >= 1 && AI * A_RPI * NW == 32 && BI * B_RPI * NW == 32, "tile/wave split");
  constexpr int LPT = AI + BI;
  constexpr int A_BYTES = 32 * AROWB, STAGE = 32 * (AROWB + BROWB);
  __shared__ __attribute__((aligned(16))) char smem_all[KG * NST * STAGE];
  const GemmTNParams& p = pp.p;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wtot = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int kgi = KG > 1 ? wtot / NW : 0;  // this wave's k group
  const int wid = wtot - kgi * NW;
  char* const smem = smem_all + kgi * (NST * STAGE);  // the group's ring
  const int wm = wid / WN, wn = wid % WN;
  const int nnt = p.Ng / BN;
  const int ntiles = (p.Mg / BM) * nnt;
  // 1-D grid of ntiles x splits, remapped so that each XCD runs a contiguous range: the tiles of
  // one pixel range (split) share its DY/X rows through that XCD's L2
  const int lin = xcd_remap(blockIdx.x, gridDim.x);
  const int split = lin / ntiles, tile = lin - split * ntiles;
  const int mt = tile / nnt, nt = tile - mt * nnt;
  const int m0 = mt * BM, n0 = nt * BN;
  const int nkt_total = (p.Kred + 31) / 32;
  const int kb_begin = split * p.kt_per_split;
  int kb_end = min(nkt_total, kb_begin + p.kt_per_split);
  if (kb_begin >= kb_end) {
    if constexpr (!FUSED) return;
    kb_end = kb_begin;  // an empty range still stores a (zero) partial and takes its ticket
  }
  // this group's half of the block's k range; both groups run `nkt` steps (the shorter one on
  // out-of-range dummy tiles, which load zeros), so the block-wide barriers pair up
  const int nkt = (kb_end - kb_begin + KG - 1) / KG;
  const int kt_begin = kb_begin + kgi * nkt;
  const int kt_end = min(kb_end, kt_begin + nkt);

  const __amdgpu_buffer_rsrc_t rsa = __builtin_amdgcn_make_buffer_rsrc((void*)p.dy, (short)0, (int)pp.dy_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t rsb = __builtin_amdgcn_make_buffer_rsrc((void*)p.x, (short)0, (int)pp.x_bytes, 0x00020000);

  // Lanes: row-in-instruction and physical chunk; the logical chunk a lane fetches is its
  // physical chunk XOR the swizzle of the LDS row it fills (per instruction: 512-B rows put only
  // two rows in one 1 KiB instruction, so the row's swizzle depends on the instruction).
  const int a_r = lane / (AROWB / 16), a_pc = lane % (AROWB / 16);
  const int b_r = lane / (BROWB / 16), b_pc = lane % (BROWB / 16);

  // Per-slot pixel state, advanced incrementally by 32 pixels per tile (no divisions in the loop):
  // 32 = step_oh*Q + step_ow; offsets use 24-bit multiplies (full-rate v_mul_u32_u24).
  const int sh = p.stride - 1;
  const unsigned rowB = (unsigned)(p.W * p.Cp * 2), pixB = (unsigned)(p.Cp * 2);
  const unsigned imgB = (unsigned)(p.H * p.W * p.Cp * 2);
  const int step_oh = 32 / p.Q, step_ow = 32 - (32 / p.Q) * p.Q;
  const bool tiny = p.P * p.Q < 32;
  int b_oh[BI], b_ow[BI], y_off[BI], x_off[BI];
  unsigned b_nb[BI], cB[BI];
  bool b_colok[BI];
#pragma unroll
  for (int i = 0; i < BI; ++i) {
    const int row = (wid * BI + i) * B_RPI + b_r;
    const int col = n0 + (b_pc ^ tn_swz<BROWB>(row)) * 8;  // (r, s, c) patch column of this lane
    const int rs = col / p.Cp;
    const int b_c = col - rs * p.Cp;
    const int b_rr = rs / p.S, b_ss = rs - b_rr * p.S;
    b_colok[i] = col < p.R * p.S * p.Cp;
    y_off[i] = b_rr - p.pad;
    x_off[i] = b_colok[i] ? b_ss - p.pad : (1 << 20);  // a column past R*S*C: always out of the image
    cB[i] = (unsigned)(b_c * 2);
    const int pix = kt_begin * 32 + row;
    const unsigned n = magic_div((unsigned)pix, pp.div_pq);
    const unsigned rem = (unsigned)pix - n * (unsigned)(p.P * p.Q);
    const unsigned oh = magic_div(rem, pp.div_q);
    b_oh[i] = (int)oh;
    b_ow[i] = (int)(rem - oh * (unsigned)p.Q);
    b_nb[i] = n * imgB;
  }
  unsigned a_off[AI];
#pragma unroll
  for (int i = 0; i < AI; ++i) {
    const int row = (wid * AI + i) * A_RPI + a_r;
    const unsigned a_coff = (unsigned)((m0 + (a_pc ^ tn_swz<AROWB>(row)) * 8) * 2);
    a_off[i] = (unsigned)(kt_begin * 32 + row) * (unsigned)(p.Mg * 2) + a_coff;
  }
  const unsigned a_step = 32u * (unsigned)(p.Mg * 2);

  // the ring's LDS byte address as an integer, converted once (a generic-to-LDS pointer conversion per DMA costs a
  // null check: 2 scalar instructions)
  const unsigned smem_lds = (unsigned)(size_t)(lds_void_t*)smem;
  auto issue = [&](int kt, int stage) {  // tiles are issued in order; kt past the end is a dummy
    const unsigned As = smem_lds + (unsigned)(stage * STAGE);
    const unsigned Bs = As + A_BYTES;
    const bool live = kt < kt_end;
    // pixels past the batch (the last tile) need no test: their DY rows and image offsets lie past the end of
    // the buffers, whose loads return zeros; a dead tile fails the row bound (H -> 0)
    const unsigned Hl = live ? (unsigned)p.H : 0u;
#pragma unroll
    for (int i = 0; i < AI; ++i) {
      buf_lds16_at(rsa, As + (unsigned)((wid * AI + i) * 1024), live ? a_off[i] : kOOB);
      a_off[i] += a_step;
    }
#pragma unroll
    for (int i = 0; i < BI; ++i) {
      const int y = (b_oh[i] << sh) + y_off[i], x = (b_ow[i] << sh) + x_off[i];
      const bool ok = (unsigned)y < Hl && (unsigned)x < (unsigned)p.W;
      const unsigned off = b_nb[i] + __umul24((unsigned)y, rowB) + __umul24((unsigned)x, pixB) + cB[i];
      buf_lds16_at(rsb, Bs + (unsigned)((wid * BI + i) * 1024), ok ? off : kOOB);
      // advance 32 pixels, branch-free (selects, no exec-mask branches: the scalar stream is one per CU)
      int ow = b_ow[i] + step_ow, oh = b_oh[i] + step_oh;
      const bool wr = ow >= p.Q;
      ow = wr ? ow - p.Q : ow;
      oh = wr ? oh + 1 : oh;
      if (!tiny) {
        const bool nx = oh >= p.P;  // next image
        b_oh[i] = nx ? oh - p.P : oh;
        b_nb[i] = nx ? b_nb[i] + imgB : b_nb[i];
      } else {  // images of fewer than 32 pixels: several per tile (uniform branch)
        while (oh >= p.P) {
          oh -= p.P;
          b_nb[i] += imgB;
        }
        b_oh[i] = oh;
      }
      b_ow[i] = ow;
    }
  };

  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int v = 0; v < 16; ++v) acc[i][j][v] = 0.f;

  // tr-read lane geometry: group g = lane>>4 (16 lanes), t = lane&15 = 4q + pq
  const int g = lane >> 4, t = lane & 15, q = t >> 2, pq = t & 3;
  const int tr_row = (g >> 1) * 8 + q;         // + 16*ks + 4*rr
  const int tr_col = (g & 1) * 16 + 4 * pq;    // element column within a 32-wide fragment block
  const int a_sw = tn_swz<AROWB>(q), b_sw = tn_swz<BROWB>(q);  // row & 3 == q for every read row
  typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

#pragma unroll
  for (int s = 0; s < NST - 1; ++s) issue(kt_begin + s, s);

  bf16x8 af[2][TM], bfr[2][TN];  // fragments of k-step ks live in [ks & 1]
  auto load_frags = [&](const char* As, const char* Bs, int ks, int buf) {
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int c = wm * (BM / WM) + i * 32 + tr_col;
      const int off = ((c >> 3) ^ a_sw) * 16 + (c & 7) * 2;
      const char* a0 = As + (ks * 16 + tr_row) * AROWB + off;
      s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(a0));
      s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(a0 + 4 * AROWB));
      // concatenated as a vector (an element-wise short[8] went through ~5 v_mov/v_bfi per fragment)
      af[buf][i] = __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
    }
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int c = wn * (BN / WN) + j * 32 + tr_col;
      const int off = ((c >> 3) ^ b_sw) * 16 + (c & 7) * 2;
      const char* b0 = Bs + (ks * 16 + tr_row) * BROWB + off;
      s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(b0));
      s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(b0 + 4 * BROWB));
      // concatenated as a vector (an element-wise short[8] went through ~5 v_mov/v_bfi per fragment)
      bfr[buf][j] = __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
    }
  };
  auto mma = [&](int buf) {
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[buf][i], bfr[buf][j], acc[i][j], 0, 0, 0);
  };
  auto step = [&](int k, int rs, int is) {  // rs: the stage read, is: the stage the DMA issued here fills
    wait_vmcnt<(NST - 2) * LPT>();
    ring_barrier();
    const char* As = smem + rs * STAGE;
    const char* Bs = As + A_BYTES;
    load_frags(As, Bs, 0, 0);
    issue(kt_begin + k + NST - 1, is);
    // step 1's fragments are read while step 0 multiplies
    load_frags(As, Bs, 1, 1);
    __builtin_amdgcn_sched_barrier(0);
    mma(0);
    __builtin_amdgcn_sched_barrier(0);
    mma(1);
  };
  {
    // (reading the next tile's first fragments across the barrier, as the row-form wgrad does, was measured
    // 3-6 % slower here: with a 4-stage ring it leaves one tile in flight)
    // unrolled by the ring depth: the stages are compile-time constants, so every fragment address is
    // a fixed per-lane register + immediate (no per-read address adds; +0-2 % over the rolled loop)
    for (int k0 = 0; k0 < nkt; k0 += NST) {
#pragma unroll
      for (int u = 0; u < NST; ++u)
        if (k0 + u < nkt) step(k0 + u, u, (u + NST - 1) % NST);
    }
  }
  wait_vmcnt<0>();
  if constexpr (KG > 1) {  // group 1's accumulators into group 0's, through the (now idle) rings
    __syncthreads();
    f32x4* xch = reinterpret_cast<f32x4*>(smem_all) + wid * (TM * TN * 4 * 64) + lane;
    if (kgi == 1) {
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
          for (int q4 = 0; q4 < 4; ++q4)
            xch[((i * TN + j) * 4 + q4) * 64] =
                f32x4{acc[i][j][4 * q4], acc[i][j][4 * q4 + 1], acc[i][j][4 * q4 + 2], acc[i][j][4 * q4 + 3]};
    }
    __syncthreads();
    if (kgi == 1) {
      if constexpr (!FUSED) return;
    } else {
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int q4 = 0; q4 < 4; ++q4) {
          const f32x4 o = xch[((i * TN + j) * 4 + q4) * 64];
#pragma unroll
          for (int e = 0; e < 4; ++e) acc[i][j][4 * q4 + e] += o[e];
        }
    }
  }

  if constexpr (FUSED) {
    // the partial in register order, write-through (group 0's waves; group 1's accumulators were added above)
    constexpr int PER_WAVE = TM * TN * 4 * 64;  // float4s per wave
    constexpr int PER_TILE = NW * PER_WAVE;
    const __amdgpu_buffer_rsrc_t rss = __builtin_amdgcn_make_buffer_rsrc((void*)pp.slab, (short)0, (int)pp.slab_bytes,
                                                                         0x00020000);
    if (kgi == 0) {
      const unsigned base = (unsigned)(((split * ntiles + tile) * NW + wid) * PER_WAVE + lane) * 16u;
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
          for (int q = 0; q < 4; ++q)
            store_wt16(rss, base + (unsigned)(((i * TN + j) * 4 + q) * 64 * 16),
                       f32x4{acc[i][j][4 * q], acc[i][j][4 * q + 1], acc[i][j][4 * q + 2], acc[i][j][4 * q + 3]});
    }
    wait_vmcnt<0>();  // this wave's partial has left for memory
    __syncthreads();  // ... and every other wave's
    int* flag = reinterpret_cast<int*>(smem_all);
    if (tid == 0) flag[0] = __hip_atomic_fetch_add(pp.cnt + tile, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();
    if (flag[0] != pp.splits - 1) return;  // not the last split of this tile (block-uniform)
    if (tid == 0) pp.cnt[tile] = 0;        // ready for the next launch
    // DW += sum over splits s = 0, 1, ... of the partials, every block thread on its own float4 positions, PU at a
    // time with their split loads in flight together
    constexpr int NTB = NW * 64 * KG, PU = 4;
    const int ldw = p.R * p.S * p.Creal;
    for (int f0 = tid; f0 < PER_TILE; f0 += NTB * PU) {
      f32x4 a[PU];
#pragma unroll
      for (int u = 0; u < PU; ++u) a[u] = f32x4{0.f, 0.f, 0.f, 0.f};
      for (int s0 = 0; s0 < pp.splits; s0 += 4) {
        f32x4 v[4][PU];
#pragma unroll
        for (int k = 0; k < 4; ++k)
#pragma unroll
          for (int u = 0; u < PU; ++u) {
            const int f = f0 + u * NTB;
            v[k][u] = (s0 + k < pp.splits && f < PER_TILE)
                          ? load_wt16(rss, (unsigned)((s0 + k) * ntiles + tile) * (unsigned)(PER_TILE * 16) +
                                               (unsigned)f * 16u)
                          : f32x4{0.f, 0.f, 0.f, 0.f};
          }
#pragma unroll
        for (int k = 0; k < 4; ++k)
#pragma unroll
          for (int u = 0; u < PU; ++u) a[u] += v[k][u];
      }
#pragma unroll
      for (int u = 0; u < PU; ++u) {
        const int f = f0 + u * NTB;
        if (f >= PER_TILE) continue;
        // register-order position -> (wave, i, j, quarter, lane) -> DW rows r0 .. r0+3 of column col
        const int ln = f & 63, qq = (f >> 6) & 3;
        const int r = f >> 8;
        const int jj = r % TN, ii = (r / TN) % TM, wv = r / (TN * TM);
        const int wmv = wv / WN, wnv = wv % WN;
        const int col = n0 + wnv * (BN / WN) + jj * 32 + (ln & 31);
        const int r0 = m0 + wmv * (BM / WM) + ii * 32 + 8 * qq + 4 * (ln >> 5);
        if (col < ldw) {
#pragma unroll
          for (int e = 0; e < 4; ++e)
            if (r0 + e < p.Mg) p.dw[(size_t)(r0 + e) * ldw + col] += a[u][e];
        }
      }
    }
    return;
  }

  // ---- epilogue: the partial tile to the slab in register order -- [split][tile][wave][i][j][quarter]
  //      x 64 lanes x 16 B, one coalesced 1 KiB store per instruction, no per-element address math
  //      (wgrad_slab_reduce_native_kernel maps it back to DW) -- or fp32 atomics into DW[k_out][(r,s,c)] ----
  if (pp.slab) {
    f32x4* dst = reinterpret_cast<f32x4*>(pp.slab) +
                 ((size_t)(split * ntiles + tile) * NW + wid) * (TM * TN * 4 * 64) + lane;
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int q = 0; q < 4; ++q)
          dst[((i * TN + j) * 4 + q) * 64] =
              f32x4{acc[i][j][4 * q], acc[i][j][4 * q + 1], acc[i][j][4 * q + 2], acc[i][j][4 * q + 3]};
    return;
  }
  const int ldw = p.R * p.S * p.Creal;  // Cp == Creal for this kernel
  const int frow = lane & 31, fhalf = lane >> 5;
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int cc = n0 + wn * (BN / WN) + j * 32 + frow;
    const bool cok = cc < ldw;
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int v = 0; v < 16; ++v) {
        const int row = m0 + wm * (BM / WM) + i * 32 + (v & 3) + 8 * (v >> 2) + 4 * fhalf;
        if (cok && row < p.Mg) atomicAdd(p.dw + (size_t)row * ldw + cc, acc[i][j][v]);
      }
  }
}

// DW += sum over splits of the register-order partial tiles of conv_tn_pipe_kernel<WM, WN, TM, TN, *>, in a
// fixed order with a position's splits in flight together: G waves (a power of two, fixed per shape; > 1 only
// where the slab has too few positions to fill the chip: many splits of few tiles) share 64 consecutive float4
// positions, one per lane; wave j of the G adds splits j, j + G, j + 2G, ... in turn (8 loads in flight per
// batch) and the G partials meet in LDS in wave order.  blockDim = 64 * max(4, G).  Each position then makes
// four DW read-modify-writes (rows r0 .. r0+3 of one column; 32 consecutive columns per half-wave).
template <int WM, int WN, int TM, int TN>
__global__ __launch_bounds__(1024) void wgrad_slab_reduce_native_kernel(const float* __restrict__ slab, int splits,
                                                                       int ntiles, int nnt, int Mg, int ldw, int G,
                                                                       float* __restrict__ dw) {
  constexpr int NW = WM * WN, BM = WM * TM * 32, BN = WN * TN * 32;
  constexpr int PER_TILE = NW * TM * TN * 4 * 64;  // float4s per tile (a multiple of 64)
  __shared__ f32x4 red[16][64];
  const long long total = (long long)ntiles * PER_TILE;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, nwb = blockDim.x >> 6;
  const int grp = w / G, j = w - grp * G, ngrp = nwb / G;
  const f32x4* s4 = reinterpret_cast<const f32x4*>(slab);
  for (long long f0 = (long long)blockIdx.x * 64 * ngrp; f0 < total; f0 += (long long)gridDim.x * 64 * ngrp) {
    const long long f = f0 + (long long)grp * 64 + lane;
    f32x4 a = {0.f, 0.f, 0.f, 0.f};
    if (f < total) {
      for (int s0 = j; s0 < splits; s0 += 8 * G) {
        f32x4 v[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          const int sp = s0 + i * G;
          v[i] = sp < splits ? s4[f + sp * total] : f32x4{0.f, 0.f, 0.f, 0.f};
        }
#pragma unroll
        for (int i = 0; i < 8; ++i) a += v[i];
      }
    }
    if (G > 1) {  // block-uniform
      red[w][lane] = a;
      __syncthreads();
      if (j == 0)
        for (int k = 1; k < G; ++k) a += red[w + k][lane];
    }
    if (j == 0 && f < total) {
      long long r = f >> 6;
      const int q = (int)(r & 3);
      r >>= 2;
      const int jj = (int)(r % TN);
      r /= TN;
      const int i = (int)(r % TM);
      r /= TM;
      const int wid = (int)(r % NW);
      const int tile = (int)(r / NW);
      const int mt = tile / nnt, nt = tile - mt * nnt;
      const int wm = wid / WN, wn = wid % WN;
      const int col = nt * BN + wn * (BN / WN) + jj * 32 + (lane & 31);
      const int r0 = mt * BM + wm * (BM / WM) + i * 32 + 8 * q + 4 * (lane >> 5);
      if (col < ldw) {
#pragma unroll
        for (int e = 0; e < 4; ++e)
          if (r0 + e < Mg) dw[(size_t)(r0 + e) * ldw + col] += a[e];
      }
    }
    if (G > 1) __syncthreads();
  }
}
