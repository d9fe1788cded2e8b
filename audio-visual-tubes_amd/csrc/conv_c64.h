// Layer-1 3x3 / stride-1 / pad-1 convolution with 64 input and 64 output channels (fwd and dgrad),
// NHWC bf16, MFMA.  Included by conv_gemm.hip inside namespace avt (after conv_nt_pipe.h: wait_vmcnt,
// buf_lds16, kOOB, GemmNTParams, MODE_*).
//
// The layer-1 BasicBlocks (base_models.py:53-69 inside _forward_impl 195-210, both trunks) are the
// largest GEMMs of the step (M = N*56*56 vision, N*65*75 audio) but only 64 wide, so a tap-gather
// kernel streams its 128x64 weight tile and 9 tap copies of every input row through L2 -> LDS for
// each k-step and stays fill/LDS-bound (~400-550 TFLOP/s).  Here the whole weight operand
// ([64][9*64] bf16, 72 KiB) is loaded into LDS ONCE per block and stays resident; the block is
// persistent (one per CU) and walks 256-row tiles of consecutive output pixels.  Per tile only the
// input "patch" [m0 - W - 1, m0 + 256 + W + 1) moves, in two 32-channel halves (each 64-B row of a
// half is one LDS-DMA lane chunk set), double-buffered (each half-buffer followed by 16 zero rows
// that masked taps read): one half streams while the other multiplies.  Every per-k-step address is
// precomputed -- A: one VGPR per (tap, row block, k-step), the tile's border mask applied once per
// tile; B: one VGPR per (half, k-step, column block) + the tap as an immediate -- so the k loop is
// ds_read + MFMA only (address arithmetic between the MFMAs, not memory, was what bound a first
// version at ~30 % of the MFMA peak with one wave per SIMD).  4 waves, each a 64x64 sub-tile (2x2 32x32 accumulators): per 16-deep k-step
// 4 fragment reads feed 4 MFMAs.  Tiles are dealt XCD-contiguously (the 32 CUs of an XCD work on
// neighbouring tiles, whose halo rows meet in that XCD's L2).  Epilogue straight from the
// accumulators: BN partial statistics (fwd, as conv_nt_pipe_kernel: per 256-row tile sum / M2 /
// sum^2/n into fp64 slot accumulators) and bf16 pairs stored as 4-byte words (lane pairs swap one
// value so each lane holds two adjacent channels of one pixel), + add (optionally masked by the
// ReLU bits of an identity block's output) for the dgrad.
#pragma once

namespace c64 {
constexpr int BM = 256;                 // output pixels per tile
constexpr int NWMAX = 8;                // waves per block: 4 (64-row wave tiles) or 8 (32-row, two per SIMD)
constexpr int KTOT = 9 * 64;            // GEMM K: (tap, channel)
constexpr int WROW = KTOT * 2;          // bytes per resident weight row (1152)
constexpr int WBYTES = 64 * WROW;       // 73,728
constexpr int PRMAX = 416;              // patch rows a half-buffer holds: 256 + 2W + 2 <= 416 -> W <= 79
constexpr int RB = 64;                  // bytes per patch row of a 32-channel half
constexpr int PBYTES = PRMAX * RB;      // 26,624 patch bytes per half-buffer ...
constexpr int SLOT = PBYTES + 1024;     // ... + 16 zero rows (masked taps): 27,648
constexpr int PINSTR = PRMAX / 16;      // 26 LDS-DMA instructions (16 rows x 64 B) per half
constexpr int WOFF = 2 * SLOT;          // 55,296: resident weights (ds_read immediates stay < 64 KiB)
constexpr int ROFF = WOFF + WBYTES;     // [2][NW][64] floats: epilogue reduction scratch
constexpr int SMEM = ROFF + 2 * NWMAX * 64 * 4;    // 133,120 B
static_assert(PINSTR * 16 == PRMAX && SMEM <= 160 * 1024 && WOFF + 8 * 128 + 1024 < 65536, "LDS layout");
}  // namespace c64

struct C64Args {
  unsigned act_bytes, w_bytes;
  int W, H;              // image (= output) width / height
  int tiles;             // ceil(M / 256)
  int tap_dy[9], tap_dx[9];  // displacement of each tap (weight tap t): border mask
  int dbg;                   // A/B diagnostics (env AVT_C64_DBG): 1 = patch loads all out of range, 2 = no stores
};

// xor-1 lane exchange (DPP quad_perm [1,0,3,2]: no LDS crossbar)
__device__ __forceinline__ float c64_swap1(float v) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0xB1, 0xF, 0xF, true));
}

// ADD: 0 none, 1 dx = dgrad + add, 2 dx = dgrad + add * mask bits.  NWAVE 4: each wave a 64x64 sub-tile
// (TM = 2); NWAVE 8: 32x64 (TM = 1), two waves per SIMD to cover each other's non-MFMA issue
template <int MODE, int ADD, int NWAVE = 4>
__global__ __launch_bounds__(NWAVE * 64, 1) void conv_c64_kernel(GemmNTParams p, C64Args ca) {
  using namespace c64;
  constexpr int TM = 4 / (NWAVE / 2) ;     // 32-row accumulator blocks per wave: 2 (4 waves) / 1 (8 waves)
  constexpr int WR = TM * 32;              // rows per wave
  constexpr int PI = (PINSTR + NWAVE - 1) / NWAVE;  // DMA instructions per wave and half (past PINSTR: zeros)
  constexpr int SPW = TM * 2 * 8;          // epilogue stores per wave and tile (TM x 2 accumulators x 8 pairs)
  static_assert(TM * 32 * NWAVE == BM, "wave rows");
  __shared__ __attribute__((aligned(16))) char smem[SMEM];
  float* red = reinterpret_cast<float*>(smem + ROFF);

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int W = ca.W, H = ca.H, hw = W * H;
  const int pre = W + 1;  // patch row of output pixel m0
  const int frow = lane & 31, fhalf = lane >> 5;

  // ---- tiles of this block: XCD x = blockIdx % 8 (nbx blocks) owns a contiguous tile range in
  //      proportion to its blocks; its blocks take them round-robin (neighbouring tiles run at the same
  //      time on one XCD) ----
  const int nb = gridDim.x, b = blockIdx.x;
  const int xcd = b & 7, nbx = (nb >> 3) + ((nb & 7) > xcd ? 1 : 0), jb = b >> 3;
  const int cum0 = xcd * (nb >> 3) + min(xcd, nb & 7);  // blocks on XCDs before this one
  const int tlo = (int)((long long)ca.tiles * cum0 / nb), thi = (int)((long long)ca.tiles * (cum0 + nbx) / nb);

  const __amdgpu_buffer_rsrc_t rsa = __builtin_amdgcn_make_buffer_rsrc((void*)p.act, (short)0, (int)ca.act_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t rso =
      __builtin_amdgcn_make_buffer_rsrc((void*)p.out, (short)0, (int)((unsigned)p.M * 128u), 0x00020000);

  // ---- resident weights: row n (output channel of the GEMM), 16-B chunk q stored at q ^ ((n>>1)&7) ----
  for (int idx = tid; idx < 64 * (WROW / 16); idx += NWAVE * 64) {
    const int n = idx / (WROW / 16), q = idx - n * (WROW / 16);
    const u32x4 v = *reinterpret_cast<const u32x4*>(p.wmat + (size_t)n * KTOT + q * 8);
    *reinterpret_cast<u32x4*>(smem + WOFF + n * WROW + ((q ^ ((n >> 1) & 7)) << 4)) = v;
  }
  if (tid < 128) reinterpret_cast<u32x4*>(smem + PBYTES + (tid >> 6) * SLOT)[tid & 63] = u32x4{0u, 0u, 0u, 0u};

  // ---- patch DMA: instruction q of a half covers patch rows 16q..16q+15; lane -> (row, 16-B chunk).
  //      Source offset = tile base + a per-lane constant; rows before the tensor (negative offset) or
  //      past it land out of range and load zeros; rows past the patch are loaded but never read.
  //      Every wave issues exactly PI instructions per half. ----
  const int lrow = lane >> 2, pchunk = lane & 3;
  unsigned dma_off[PI];
#pragma unroll
  for (int i = 0; i < PI; ++i) {
    const int pr = (wid + NWAVE * i) * 16 + lrow;
    dma_off[i] = (unsigned)(pr * 128 + ((pchunk ^ ((pr >> 2) & 3)) << 4));
  }
  auto issue_half = [&](int tile, int half) {
    char* buf = smem + half * SLOT;
    const bool live = tile < thi && !(ca.dbg & 1);
    const unsigned base = live ? (unsigned)((tile * BM - pre) * 128 + half * 64) : kOOB;
#pragma unroll
    for (int i = 0; i < PI; ++i) {
      const int q = wid + NWAVE * i;  // wave-uniform
      buf_lds16(rsa, q < PINSTR ? buf + q * 1024 : buf + PBYTES, q < PINSTR ? base + dma_off[i] : kOOB);
    }
  };

  // ---- A addresses: rel[t][i][ks] = byte offset in a half-buffer of the 16-B fragment chunk of tap t,
  //      row block i, k-step ks (valid taps); masked taps read the zero rows at the same bank position ----
  unsigned relv[9][TM][2];
#pragma unroll
  for (int t = 0; t < 9; ++t)
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int pr = wid * WR + i * 32 + frow + pre + ca.tap_dy[t] * W + ca.tap_dx[t];
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) relv[t][i][ks] = (unsigned)(pr * RB + (((ks * 2 + fhalf) ^ ((pr >> 2) & 3)) << 4));
    }
  // ---- B addresses: weight row n = j*32 + frow, chunk q = 8t + 4half + 2ks + fhalf stored at q ^ f(n):
  //      = n*WROW + 128 t + ((4half + 2ks) ^ g) * 16 with g = fhalf ^ f(n); 128 t is a ds_read immediate ----
  unsigned bb[2][2][2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int n = j * 32 + frow;
    const int g = fhalf ^ ((n >> 1) & 7);
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) bb[h][ks][j] = (unsigned)(n * WROW + (((4 * h + 2 * ks) ^ g) << 4));
  }

  __syncthreads();  // weights + zero rows written (their global loads waited by the compiler)

  // Pipeline: half 1 of tile t streams while half 0 multiplies, half 0 of tile t+1 while half 1 multiplies
  // and the epilogue stores.  Wait before half 0 of tile t: issued after it are the previous tile's SPW
  // epilogue stores (buffer stores, issued unconditionally -- rows past M get an out-of-range offset --
  // so the count is exact; wave 0's statistics atomics only make its wait stricter); before half 1:
  // nothing.
  int tile = tlo + jb;
  double st_s = 0.0, st_m2 = 0.0, st_r = 0.0;  // BN partials of this block's tiles (threads < 64)
  issue_half(tile, 0);
  for (int it = 0; tile < thi; tile += nbx, ++it) {
    const int m0 = tile * BM;
    // border mask of this tile's fragment rows -> the A offsets of the tile
    unsigned rel[9][TM][2];
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int m = m0 + wid * WR + i * 32 + frow;
      const bool ok = m < p.M;
      const int mm = ok ? m : 0;
      const int n = mm / hw, rem = mm - n * hw;
      const int oh = rem / W, ow = rem - oh * W;
#pragma unroll
      for (int t = 0; t < 9; ++t) {
        const int y = oh + ca.tap_dy[t], x = ow + ca.tap_dx[t];
        const bool v = ok && y >= 0 && y < H && x >= 0 && x < W;
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) rel[t][i][ks] = v ? relv[t][i][ks] : ((relv[t][i][ks] & 1023u) | (unsigned)PBYTES);
      }
    }
    f32x16 acc[TM][2];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int v = 0; v < 16; ++v) acc[i][j][v] = 0.f;

#pragma unroll
    for (int half = 0; half < 2; ++half) {
      if (half == 1 || it == 0)
        wait_vmcnt<0>();    // this half landed
      else
        wait_vmcnt<SPW>();  // ... (the previous tile's stores may be in flight)
      ring_barrier();  // every wave's part landed; every wave is done with the other half-buffer
      if (half == 0)
        issue_half(tile, 1);
      else
        issue_half(tile + nbx, 0);
      // 18 k-steps (tap t, ks): k = t*64 + half*32 + ks*16; fragments of step s+1 read while step s multiplies
      bf16x8 af[2][TM], bfr[2][2];
      const char* abuf = smem + half * SLOT;
      auto load_frags = [&](int s, int buf) {
        const int t = s >> 1, ks = s & 1;
#pragma unroll
        for (int i = 0; i < TM; ++i) af[buf][i] = *reinterpret_cast<const bf16x8*>(abuf + rel[t][i][ks]);
#pragma unroll
        for (int j = 0; j < 2; ++j)
          bfr[buf][j] = *reinterpret_cast<const bf16x8*>(smem + WOFF + 128 * t + bb[half][ks][j]);
      };
      load_frags(0, 0);
#pragma unroll
      for (int s = 0; s < 18; ++s) {
        if (s + 1 < 18) {
          load_frags(s + 1, (s + 1) & 1);
          __builtin_amdgcn_sched_barrier(0);
        }
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[s & 1][i], bfr[s & 1][j], acc[i][j], 0, 0, 0);
        if (s + 1 < 18) __builtin_amdgcn_sched_barrier(0);
      }
    }
    const int rows_valid = min(BM, p.M - m0);
    // ---- epilogue ----
    if (MODE == MODE_FWD && p.stats != nullptr) {
      // per-column sum over this wave's valid rows -> tile mean -> M2 about it (conv_nt_pipe_kernel's scheme)
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        float s = 0.f;
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int v = 0; v < 16; ++v) {
            const int r = wid * WR + i * 32 + (v & 3) + 8 * (v >> 2) + 4 * fhalf;
            if (r < rows_valid) s += acc[i][j][v];
          }
        s += __shfl_xor(s, 32, 64);
        if (lane < 32) red[wid * 64 + j * 32 + lane] = s;
      }
      __syncthreads();
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int c = j * 32 + frow;
        float tot = 0.f;
#pragma unroll
        for (int k = 0; k < NWAVE; ++k) tot += red[k * 64 + c];
        const float mean = tot / (float)rows_valid;
        float q = 0.f;
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int v = 0; v < 16; ++v) {
            const int r = wid * WR + i * 32 + (v & 3) + 8 * (v >> 2) + 4 * fhalf;
            const float d = acc[i][j][v] - mean;
            if (r < rows_valid) q += d * d;
          }
        q += __shfl_xor(q, 32, 64);
        if (lane < 32) red[NWAVE * 64 + wid * 64 + c] = q;
      }
      __syncthreads();
      if (tid < 64) {
        double s = 0.0, m2 = 0.0;
#pragma unroll
        for (int k = 0; k < NWAVE; ++k) {
          s += (double)red[k * 64 + tid];
          m2 += (double)red[NWAVE * 64 + k * 64 + tid];
        }
        // the three terms are additive over tiles: summed per block, one set of atomics after the loop
        st_s += s;
        st_m2 += m2;
        st_r += s * s / (double)rows_valid;
      }
    }
    // bf16 pairs: lanes 2k / 2k+1 hold columns c / c+1 of the same rows; per pair of accumulator
    // values (v, v+1) = rows (r, r+1) the even lane stores row r (c, c+1), the odd lane row r+1 (c-1, c).
    // Per 32x32 accumulator the 8 `add` words (and mask bytes) are loaded together before any is used.
    const bool odd = lane & 1;
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int c = j * 32 + (frow & ~1);
        unsigned av[8], mv[8];
        size_t offs[8];
        bool okv[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          const int v = 2 * u;
          const int r = wid * WR + i * 32 + (v & 3) + 8 * (v >> 2) + 4 * fhalf + (odd ? 1 : 0);
          okv[u] = r < rows_valid;
          offs[u] = (size_t)(m0 + (okv[u] ? r : 0)) * 64 + c;  // element offset of the pair
          if (ADD) av[u] = *reinterpret_cast<const unsigned*>(p.add + offs[u]);
          if (ADD == 2) mv[u] = p.amask[offs[u] >> 3];
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          const float a0 = acc[i][j][2 * u], a1 = acc[i][j][2 * u + 1];
          const float r0 = c64_swap1(a0), r1 = c64_swap1(a1);
          unsigned o = odd ? pack2(r1, a1) : pack2(a0, r0);
          if (ADD) {
            unsigned a = av[u];
            if (ADD == 2) {
              const unsigned bits = mv[u] >> (c & 7);
              a &= (bits & 1u ? 0x0000ffffu : 0u) | (bits & 2u ? 0xffff0000u : 0u);
            }
            o = pack2(bf2f(o & 0xffff) + bf2f(a & 0xffff), bf2f(o >> 16) + bf2f(a >> 16));
          }
          __builtin_amdgcn_raw_buffer_store_b32(o, rso, okv[u] && !(ca.dbg & 2) ? (int)(offs[u] * 2) : (int)kOOB, 0, 0);
        }
      }
  }
  wait_vmcnt<0>();  // drain (the last iteration issued an all-out-of-range half 0)
  // BN partials per block (its tiles summed in tile order), stored in the block's own slot (avt_common.h;
  // a block without tiles stores zeros)
  if (MODE == MODE_FWD && p.stats != nullptr) {
    bn_write_header(p.stats, gridDim.x, 0);
    if (tid < 64) {
      double* a = bn_fwd_slots(p.stats) + ((size_t)blockIdx.x * p.Ng + tid) * 3;
      a[0] = st_s;
      a[1] = st_m2;
      a[2] = st_r;
    }
  }
}
