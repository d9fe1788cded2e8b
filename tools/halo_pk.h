// EXPERIMENT, not in libavt (tools/halo_bench.hip; measured in profiles/r5_halo_bench_pk.txt: no faster than
// conv_halo_kernel -- see DESIGN.md round 5).  Persistent halo conv (3x3 / stride 1 / pad 1 fwd and dgrad, NHWC bf16, v_mfma_f32_32x32x16_bf16): the
// conv_halo_kernel main loop run over a SEQUENCE of work items per block, with the pipeline carried from one
// item into the next.  Included by tools/halo_bench.hip inside namespace avt after conv_halo.h (HaloArgs, halo_swz,
// wait_vmcnt, ring_barrier, buf_lds16, store_wt16 / load_wt16, xcd_remap, kOOB).
//
// Why (tools/halo_bench.hip, one round of 256 tiles vs two): a conv_halo_kernel tile pays ~10 us outside its
// k loop -- the first patch and weight stages load with nothing to overlap, and the epilogue's C tile goes
// through LDS and out to HBM while the MFMAs idle -- once per tile, so a grid of 1.5-2.5 tiles per CU pays it 2-3
// times.  Here a block keeps streaming: the next item's patch rides in the current item's last chunk as an
// ordinary "next chunk", its first weight tiles are already in the ring, and the epilogue stores straight from
// the accumulators (lane pairs exchange one value by DPP, each lane stores two adjacent bf16 outputs), so the
// stores drain while the next item computes.  The LDS holds only the ring, the two patch buffers and the small
// statistics scratch.
//
// Work items (HaloArgs::pk):
//   pk = 1  whole tiles: block b takes tiles b, b + G, b + 2G, ... (G = gridDim.x <= tiles);
//   pk = 2  stream-K: the (tile, 64-channel chunk) units are cut into G equal contiguous ranges, so every block
//           does the same MFMA work whatever the tile count (a 392-tile grid on 256 CUs: 1.53 tiles of work per CU
//           instead of 2 rounds).  A tile cut between blocks b and b+1 has its chunks 0..k-1 at the END of block
//           b's range and k..nc-1 at the START of block b+1's.  Each block walks its range in DESCENDING tile
//           order, so block b does that head FIRST: it stores the fp32 accumulators after chunk k-1 (the partial)
//           and sets a flag; block b+1 reaches the tail LAST, waits for the flag (long set by then), loads the
//           partial into its accumulators and continues with chunk k.  The fp32 accumulation order is the unsplit
//           tile's, so outputs and statistics are bitwise conv_halo_kernel's.  Every range holds >= nc units (the
//           host checks), so a tile is cut at most once and a block only waits on its neighbour's FIRST item.
// Hand-off (MI355X_MICROARCH.md, hand-off table row 1): sc1 stores of the partial, the storing waves' counted
// vmcnt covering them, a workgroup barrier, one lane's agent-scope flag store; the consumer polls with sc1 loads,
// passes a workgroup barrier, loads the partial with sc1 loads and resets the flag (one producer, one consumer
// per flag and launch: every flag is zero again when the launch ends).
#pragma once

// the persistent kernel's arguments: HaloArgs + pixel -> (image, row) magic divisors and the item mode
struct HaloPkArgs : HaloArgs {
  MagicDiv div_hw, div_w;
  int pk;  // 1 whole tiles per block, 2 stream-K ranges (part / cnt: the partials and flags, one per block)
};

template <int MODE, int WM, int WN, int TM, int TN, int NSTB, int PRMAX, int PK, int DBG = 0>
__global__ __launch_bounds__(WM * WN * 64, (halo_blocks_per_cu<WN, TN, NSTB, PRMAX>())) void conv_halo_pk_kernel(
    GemmNTParams p, HaloPkArgs ha) {
  constexpr int FR = 32, FM = TM, FN = TN, KS = 4;
  constexpr int NW = WM * WN, NT = NW * 64;
  constexpr int BM = WM * TM * 32, BN = WN * TN * 32;
  constexpr int BK = 64, RB = 128, RPI = 8;
  constexpr int BR = BN / (NW * RPI);
  static_assert(BR >= 1 && BR * NW * RPI == BN, "weight tile / wave split");
  constexpr int PINSTR = (PRMAX + RPI - 1) / RPI;
  static_assert(NSTB >= 3 && NSTB <= 4, "NSTB: the step's stage is t % NSTB only for NSTB 3 (9 % 3 == 0)");
  constexpr int NPIECE = 10 - NSTB;
  constexpr int AP = (PINSTR + NPIECE * NW - 1) / (NPIECE * NW);
  constexpr int ABUF = PRMAX * RB + 1024;
  constexpr int BSTAGE = BN * RB;
  constexpr int MAIN = 2 * ABUF + NSTB * BSTAGE;
  static_assert(PRMAX % RPI == 0, "PRMAX");
  static_assert(MAIN + 2 * WM * BN * 4 + 64 <= 160 * 1024, "LDS budget of a CU");
  __shared__ __attribute__((aligned(16))) char smem[MAIN + 2 * WM * BN * 4 + 64];
  char* zrow = smem + PRMAX * RB;
  float* red = reinterpret_cast<float*>(smem + MAIN);    // [2][WM][BN] statistics scratch
  int* flagw = reinterpret_cast<int*>(smem + MAIN + 2 * WM * BN * 4);  // the consumer's poll result

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid / WN, wn = wid % WN;
  const int nnt = p.Ng / BN, nmt = (p.M + BM - 1) / BM, tiles = nmt * nnt, nc = p.IC / BK;
  const int G = gridDim.x, b = xcd_remap(blockIdx.x, G);
  const int W = ha.W, H = ha.H, hw = W * H;
  const int pre = W + 1, PR = BM + 2 * pre;
  // tap t = (r, s): input displacement (dy, dx) = (r-1, s-1) (fwd) or (1-r, 1-s) (dgrad, flipped); weight tap t
  auto tdy = [](int t) constexpr { return MODE == MODE_FWD ? t / 3 - 1 : 1 - t / 3; };
  auto tdx = [](int t) constexpr { return MODE == MODE_FWD ? t % 3 - 1 : 1 - t % 3; };

  // ---- this block's work items (T, [ca, cb)), in processing order ----
  int u0 = 0, u1 = 0;  // stream-K unit range (tiles * nc * G < 2^31: the host checks)
  int T_first, T_last, T_step;
  if constexpr (PK == 2) {
    const int U = tiles * nc;
    u0 = U * b / G;
    u1 = U * (b + 1) / G;
    T_first = (u1 - 1) / nc;
    T_last = u0 / nc;
    T_step = -1;
  } else {
    T_first = b;
    T_last = b + ((tiles - 1 - b) / G) * G;
    T_step = G;
  }
  auto item_ca = [&](int T) -> int { return PK == 2 ? (u0 > T * nc ? u0 - T * nc : 0) : 0; };
  auto item_cb = [&](int T) -> int { return PK == 2 ? (u1 < (T + 1) * nc ? u1 - T * nc : nc) : nc; };

  if (tid < 128) reinterpret_cast<u32x4*>(zrow + (tid >> 6) * ABUF)[tid & 63] = u32x4{0u, 0u, 0u, 0u};
  __syncthreads();

  const __amdgpu_buffer_rsrc_t rsa = __builtin_amdgcn_make_buffer_rsrc((void*)p.act, (short)0, (int)ha.act_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t rsb = __builtin_amdgcn_make_buffer_rsrc((void*)p.wmat, (short)0, (int)ha.w_bytes, 0x00020000);
  const int out_bytes = p.M * p.Ng * 2;
  const __amdgpu_buffer_rsrc_t rs_out = __builtin_amdgcn_make_buffer_rsrc((void*)p.out, (short)0, out_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t rs_add = __builtin_amdgcn_make_buffer_rsrc((void*)p.add, (short)0, out_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t rs_am = __builtin_amdgcn_make_buffer_rsrc((void*)p.amask, (short)0, out_bytes / 16, 0x00020000);

  const int lrow = lane >> 3, pchunk = lane & 7;
  // patch DMA offset of instruction q of tile T's patch, 64-channel chunk c (tile-dependent: m0)
  // patch DMA offset of instruction q of the patch at pixel pbase = m0 - pre, channel offset cofs = chunk * 64
  auto patch_voff = [&](int pbase, int q, int cofs) -> unsigned {
    const int pr = q * RPI + lrow;
    const int pix = pbase + pr;
    const bool ok = pr < PR && pix >= 0 && pix < p.M;
    const int lc = pchunk ^ halo_swz(pr);
    return ok ? (unsigned)((pix * p.IC + cofs + lc * 8) * 2) : kOOB;  // 32-bit: activations stay below 2 GiB
  };
  // the patch pieces' lane terms (piece k, instruction a: patch row pr = q * 8 + lrow, q = (k AP + a) NW + wid):
  // pl = the row's byte offset within a pixel-0 patch (its chunk swizzle included), or -1 past the patch rows
  constexpr int NPQ = NPIECE * AP;
  int pl[NPQ], prr[NPQ];
#pragma unroll
  for (int k = 0; k < NPQ; ++k) {
    const int q = k * NW + wid;
    const int pr = q * RPI + lrow;
    prr[k] = pr;
    pl[k] = (q < PINSTR && pr < PR) ? (pr * p.IC + (pchunk ^ halo_swz(pr)) * 8) * 2 : -1;
  }
  unsigned b_row[BR];  // weight DMA offset of this lane's row, without the tile's column base
#pragma unroll
  for (int i = 0; i < BR; ++i) {
    const int row = (wid * BR + i) * RPI + lrow;
    const int lc = pchunk ^ halo_swz(row);
    b_row[i] = (unsigned)(((size_t)row * p.Kg + lc * 8) * 2);
  }
  const int frow = lane & (FR - 1), fhalf = lane / FR;
  int boffs[FN][KS];
#pragma unroll
  for (int j = 0; j < FN; ++j)
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      const int row = wn * (BN / WN) + j * FR + frow;
      boffs[j][ks] = row * RB + (((2 * ks + fhalf) ^ halo_swz(row)) << 4);
    }
  // A row address of every (tap, row block) for the tile at m0 (conv_halo_kernel's arow; recomputed per item)
  unsigned arow[9][FM];
  auto set_rows = [&](int m0) {
    int sl = lane;  // opaque lane id: the per-(tap, row block) terms stay inside the item loop, not in registers
    asm volatile("" : "+v"(sl));
    const int sfr = sl & (FR - 1), sfh = sl / FR;
#pragma unroll
    for (int i = 0; i < FM; ++i) {
      const int row = wm * (BM / WM) + i * FR + sfr;
      const int m = m0 + row;
      const bool ok = m < p.M;
      const int mm = ok ? m : 0;
      const int n = (int)magic_div((unsigned)mm, ha.div_hw), rem = mm - n * hw;
      const int oh = (int)magic_div((unsigned)rem, ha.div_w), ow = rem - oh * W;
#pragma unroll
      for (int t = 0; t < 9; ++t) {
        const int y = oh + tdy(t), x = ow + tdx(t);
        const bool v = ok && y >= 0 && y < H && x >= 0 && x < W;
        const int pr = row + pre + tdy(t) * W + tdx(t);
        arow[t][i] = (unsigned)((v ? pr * RB : PRMAX * RB + (pr & 7) * RB) | ((sfh ^ halo_swz(pr)) << 4));
      }
    }
  };

  // ---- the step sequence: items x chunks x taps.  A chunk's descriptor (tile, channel chunk); the weights of a
  //      step (T, c, tap) go to ring stage (global step) % NSTB; patch pieces of the chunk AFTER the current one ride
  //      on the current chunk's taps 0 .. 8-(NSTB-1), into patch buffer (global chunk + 1) & 1 ----
  // wbase: ((tile column) * BN * Kg + chunk * 64) * 2 bytes, the weights of tap tn at + tn * IC * 2
  auto issue_w = [&](bool live, unsigned wbase, int tn, int stage) {
    char* Bs = smem + 2 * ABUF + stage * BSTAGE;
    const unsigned base = wbase + (unsigned)(tn * p.IC * 2);
#pragma unroll
    for (int i = 0; i < BR; ++i) buf_lds16(rsb, Bs + (wid * BR + i) * 1024, live ? b_row[i] + base : kOOB);
  };
  // pieces of the patch at pbase (= m0 - pre), channel offset cofs: row pr's pixel is pbase + pr
  auto issue_p = [&](bool live, int pbase, int cofs, int piece, int buf) {
    char* Ab = smem + buf * ABUF;
    const unsigned ub = (unsigned)((pbase * p.IC + cofs) * 2);
#pragma unroll
    for (int a = 0; a < AP; ++a) {
      const int k = piece * AP + a, q = k * NW + wid;
      const bool inrange = q < PINSTR;
      const int pix = pbase + prr[k];
      const bool ok = live && pl[k] >= 0 && pix >= 0 && pix < p.M;
      buf_lds16(rsa, inrange ? Ab + q * 1024 : zrow, ok ? ub + (unsigned)pl[k] : kOOB);
    }
  };
  auto wbase_of = [&](int T, int c) -> unsigned { return (unsigned)(((T % nnt) * BN * p.Kg + c * BK) * 2); };
  auto pbase_of = [&](int T) -> int { return (T / nnt) * BM - pre; };

  using acc_t = f32x16;
  acc_t acc[FM][FN];
  bf16x8 af[2][FM], bfr[2][FN];
  auto mma = [&](int buf) {
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[buf][i], bfr[buf][j], acc[i][j], 0, 0, 0);
  };

  // prologue: the first chunk's whole patch, then steps 0 .. NSTB-2 (a chunk has 9 >= NSTB-1 steps)
  int T = T_first, ca = item_ca(T), cb = item_cb(T);
  for (int q = wid; q < PINSTR; q += NW) buf_lds16(rsa, smem + q * 1024, patch_voff(pbase_of(T), q, ca * BK));
#pragma unroll
  for (int j = 0; j < NSTB - 1; ++j) issue_w(true, wbase_of(T, ca), j, j);

  int g = 0;               // global chunk ordinal: patch buffer g & 1
  int publish = -1;        // >= 0: flag of this block's partial, set at the next step-1 barrier
  for (;;) {
    // ---- item (T, [ca, cb)) ----
    set_rows((T / nnt) * BM);
    const bool tail = PK == 2 && ca > 0;  // stream-K: chunks 0 .. ca-1 were accumulated by block b-1
#ifdef PKX_NOTAIL
    if (false) {
#else
    if (tail) {
#endif
      // poll the producer's flag (one lane), then every wave loads its accumulators from the partial
      if (tid == 0) {
        int f;
        do {
          f = __hip_atomic_load(ha.cnt + (b - 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          if (!f) __builtin_amdgcn_s_sleep(2);
        } while (!f);
        __hip_atomic_store(ha.cnt + (b - 1), 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      __syncthreads();
      const __amdgpu_buffer_rsrc_t rsp = __builtin_amdgcn_make_buffer_rsrc(
          (void*)(ha.part + (size_t)(b - 1) * BM * BN), (short)0, (int)(BM * BN * 4), 0x00020000);
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j)
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const f32x4 v4 = load_wt16(rsp, (unsigned)((((wid * TM + i) * TN + j) * 4 + q) * 1024 + lane * 16));
#pragma unroll
            for (int e = 0; e < 4; ++e) acc[i][j][4 * q + e] = v4[e];
          }
    } else {
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j)
#pragma unroll
          for (int v = 0; v < 16; ++v) acc[i][j][v] = 0.f;
    }
    const bool last_item = T == T_last;
    const int Tn = T + T_step;  // the next item's tile (valid unless last_item)
    const int can = last_item ? 0 : item_ca(Tn);
    for (int c = ca; c < cb; ++c, ++g) {
      // the chunk after this one: (T, c+1), or the next item's first, or none
      const bool nx_live = c + 1 < cb || !last_item;
      const int nxT = c + 1 < cb ? T : Tn, nxc = c + 1 < cb ? c + 1 : can;
      const unsigned wb = wbase_of(T, c), nx_wb = wbase_of(nxT, nxc);
      const int nx_pb = pbase_of(nxT), nx_co = nxc * BK;
      const char* Ab = smem + (g & 1) * ABUF;
#pragma unroll
      for (int t = 0; t < 9; ++t) {
        const int stage = NSTB == 3 ? t % 3 : 0;
        static_assert(NSTB == 3, "stage = t % 3");
        // step s's weights have landed once only its own patch piece and steps s+1 .. s+NSTB-2 may be
        // outstanding (conv_halo_kernel's relaxed wait)
        int pieces = (t >= NSTB - 1) ? 1 : 0;
#pragma unroll
        for (int j = 1; j <= NSTB - 2; ++j) pieces += ((t + j) % 9 >= NSTB - 1) ? 1 : 0;
        constexpr int W0 = (NSTB - 2) * BR;
        if (pieces == 0)
          wait_vmcnt<W0>();
        else if (pieces == 1)
          wait_vmcnt<W0 + AP>();
        else
          wait_vmcnt<W0 + 2 * AP>();
        ring_barrier();
        if (PK == 2 && t == 1 && publish >= 0) {
          // every wave's partial stores are older than what its step-1 wait left outstanding: published
          if (tid == 0) __hip_atomic_store(ha.cnt + publish, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          publish = -1;
        }
        const char* Bs = smem + 2 * ABUF + stage * BSTAGE;
        auto load_frags = [&](int ks, int buf) {
#pragma unroll
          for (int i = 0; i < FM; ++i)
            af[buf][i] = *reinterpret_cast<const bf16x8*>(Ab + (arow[t][i] ^ (unsigned)(ks << 5)));
#pragma unroll
          for (int j = 0; j < FN; ++j) bfr[buf][j] = *reinterpret_cast<const bf16x8*>(Bs + boffs[j][ks]);
        };
        load_frags(0, 0);
        {  // step s + NSTB-1: tap t+2 of this chunk, or tap t-7 of the next one; pieces of the next chunk
          const int tn = t + NSTB - 1;
          const int st = (stage + NSTB - 1) % NSTB;
          if (tn < 9) {
            issue_w(true, wb, tn, st);
            issue_p(nx_live, nx_pb, nx_co, tn - (NSTB - 1), (g + 1) & 1);
          } else {
            issue_w(nx_live, nx_wb, tn - 9, st);
          }
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

    // ---- item epilogue ----
    const int mt = T / nnt, m0 = mt * BM, n0 = (T % nnt) * BN;
    if (PK == 2 && cb < nc) {
      // stream-K head: the fp32 partial in register order (write-through), published at the next step-1 barrier
      const __amdgpu_buffer_rsrc_t rsp = __builtin_amdgcn_make_buffer_rsrc(
          (void*)(ha.part + (size_t)b * BM * BN), (short)0, (int)(BM * BN * 4), 0x00020000);
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j)
#pragma unroll
          for (int q = 0; q < 4; ++q)
            store_wt16(rsp, (unsigned)((((wid * TM + i) * TN + j) * 4 + q) * 1024 + lane * 16),
                       f32x4{acc[i][j][4 * q], acc[i][j][4 * q + 1], acc[i][j][4 * q + 2], acc[i][j][4 * q + 3]});
      publish = b;
    } else {
      const int rows_valid = min(BM, p.M - m0);
      // lane terms from an opaque copy of the lane id (not hoisted out of the item loop: registers)
      int el = lane;
      asm volatile("" : "+v"(el));
      const int efr = el & (FR - 1), efh = el / FR;
      auto acc_row = [&](int i, int v) -> int { return wm * (BM / WM) + i * FR + (v & 3) + 8 * (v >> 2) + 4 * efh; };
#ifndef PKX_NOSTATS
      if (MODE == MODE_FWD && p.stats != nullptr && !(DBG & 2)) {
        // BN partial statistics of the tile (conv_halo_kernel's epilogue, same order: bitwise the same slots)
#pragma unroll
        for (int j = 0; j < FN; ++j) {
          float sm = 0.f;
#pragma unroll
          for (int i = 0; i < FM; ++i)
#pragma unroll
            for (int v = 0; v < 16; ++v)
              if (acc_row(i, v) < rows_valid) sm += acc[i][j][v];
#pragma unroll
          for (int o = FR; o < 64; o <<= 1) sm += __shfl_xor(sm, o, 64);
          if (efr == el) red[wm * BN + wn * (BN / WN) + j * FR + el] = sm;
        }
        __syncthreads();
#pragma unroll
        for (int j = 0; j < FN; ++j) {
          const int cc = wn * (BN / WN) + j * FR + efr;
          float tot = 0.f;
#pragma unroll
          for (int k = 0; k < WM; ++k) tot += red[k * BN + cc];
          const float mean = tot / (float)rows_valid;
          float q = 0.f;
#pragma unroll
          for (int i = 0; i < FM; ++i)
#pragma unroll
            for (int v = 0; v < 16; ++v) {
              const float d = acc[i][j][v] - mean;
              if (acc_row(i, v) < rows_valid) q += d * d;
            }
#pragma unroll
          for (int o = FR; o < 64; o <<= 1) q += __shfl_xor(q, o, 64);
          if (efr == el) red[WM * BN + wm * BN + cc] = q;
        }
        __syncthreads();
        bn_write_header(p.stats, nmt, 0, mt == 0 && n0 == 0);
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
        __syncthreads();  // the scratch is free for the next item's statistics
      }
#endif
      // outputs: each wave stages its 32 x 64 row blocks as bf16 in its own 4 KB slice of the patch buffer the item's
      // last chunk used (free until the next item's first barrier: the next patch streams into the other buffer),
      // lanes 2k, 2k+1 first swapping one value per row pair by DPP so each writes one dword (row v: c, c+1); then
      // every lane reads a 16-byte row chunk back and stores it, 8 lanes per 128-byte output row (+ add, masked:
      // bitwise conv_halo_kernel's epilogue).  The barrier: every wave has read its last fragments of the buffer.
      if (!(DBG & 1)) {
        __syncthreads();
        char* slice = smem + ((g - 1) & 1) * ABUF + wid * 4096;
        const bool odd = el & 1;
        const int rr0 = el >> 3, cch = el & 7;
#pragma unroll
        for (int i = 0; i < FM; ++i) {
#pragma unroll
          for (int j = 0; j < FN; ++j)
#pragma unroll
            for (int v = 0; v < 16; v += 2) {
              const float send = odd ? acc[i][j][v] : acc[i][j][v + 1];
              const float recv = __builtin_bit_cast(
                  float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, send), 0xB1, 0xF, 0xF, false));  // lane ^ 1
              const float lo = odd ? recv : acc[i][j][v], hi = odd ? acc[i][j][v + 1] : recv;
              const int r = (v & 3) + 8 * (v >> 2) + 4 * efh + (odd ? 1 : 0);
              *reinterpret_cast<unsigned*>(slice + r * 128 + (j * FR + (efr & ~1)) * 2) = pack2(lo, hi);
            }
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            const int rr = rr0 + 8 * k;
            u32x4 v = *reinterpret_cast<const u32x4*>(slice + rr * 128 + cch * 16);
            const int row = wm * (BM / WM) + i * FR + rr;
            // buffer stores/loads with 32-bit offsets (the host keeps M * Ng * 2 below 2 GiB); rows past M: out of range
            const unsigned eoff = (unsigned)((m0 + row) * p.Ng + n0 + wn * (BN / WN) + cch * 8);
            const unsigned boff = row < rows_valid ? eoff * 2 : kOOB;
            if (p.add != nullptr) {
              u32x4 a = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rs_add, boff, 0, 0));
              if (p.amask != nullptr)
                a = epi_mask8(a, __builtin_amdgcn_raw_buffer_load_b8(rs_am, row < rows_valid ? eoff >> 3 : kOOB, 0, 0));
              unsigned* vv = reinterpret_cast<unsigned*>(&v);
              const unsigned* aa = reinterpret_cast<const unsigned*>(&a);
#pragma unroll
              for (int e = 0; e < 4; ++e) vv[e] = pack2(bf2f(vv[e] & 0xffff) + bf2f(aa[e] & 0xffff),
                                                        bf2f(vv[e] >> 16) + bf2f(aa[e] >> 16));
            }
            __builtin_amdgcn_raw_buffer_store_b128(v, rs_out, boff, 0, 0);
          }
        }
      }
    }
    if (last_item) break;
    T = Tn;
    ca = can;
    cb = item_cb(T);
  }
  if (publish >= 0) {  // a head with no item after it (not planned: every range holds >= nc units)
    wait_vmcnt<0>();
    __syncthreads();
    if (tid == 0) __hip_atomic_store(ha.cnt + publish, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  wait_vmcnt<0>();
}
