// 7x7 / stride 2 / pad 3 stem convolutions (models/base_models.py:135-138: the vision conv1 over
// 3 channels padded to 4, the audio conv1_a over 1 channel), 64 output channels, forward with the BN
// partial statistics of the other forward kernels.  Included by conv_gemm.hip inside namespace avt
// (needs the BN accumulator helpers of avt_common.h, f2bf).
//
// The stem is store-bound: 64 bf16 channels out per output pixel (205 MB vision / 317 MB audio at
// B = 128 against 51 / 20 MB of input), and the first versions of this kernel were VALU-bound on
// per-element work (PMC: ~550 VALU instructions per 32-pixel tile vs 28 MFMAs -- the masked BN sums,
// bf16 conversion and staging), so everything per element that can run on the matrix cores does:
//   * persistent: one block of kStemNW = 8 waves per CU; the 64 x K weight operand goes to LDS once;
//   * work unit = a wave tile of 32 output pixels of ONE output row (OW split into ceil(OW/32)
//     tiles: the idle rows of a short last tile cost MFMA time only); wave w of block b takes tiles
//     v*8 + w + k * 8 * gridDim, v = the XCD-grouped index of b (xcd_remap), so consecutive output
//     rows -- which share input rows -- meet in one XCD's L2; no block barrier in the main loop;
//   * the tile's input patch (7 input rows -- 8 for C = 1, whose dummy row r = 7 reads a zero row --
//     x 70 columns; buffer loads, zeros outside the image by an out-of-range offset) sits in one of
//     the wave's two LDS buffers; the patches of the next TWO tiles are in flight in registers;
//   * A fragments straight out of the patch:
//       C = 4: k = (r*8 + s)*4 + c (dummy tap s = 7, zero weight): a lane's 8 k values are taps
//              (r, s0), (r, s0+1) x 4 channels = two adjacent patch pixels = one ds_read_b128;
//              K = 224 (196 real), 14 MFMA k-steps;
//       C = 1: k = r*8 + s (dummy row r = 7 and tap s = 7): a lane's 8 k values are 8 adjacent
//              columns of one patch row; K = 64 (49 real), 4 k-steps;
//   * BN statistics on the MFMA pipe: the bf16 tile (v_cvt_pk_bf16_f32 pairs: a lane holds 16 pixels
//     of one channel -- exactly an MFMA operand with pixels as k) feeds, per 16-pixel k-step,
//       sum:   D_s += [1 (rows < 16) | 0] x Y_0 + [0 | 1 (rows >= 16)] x Y_1  (rows 0-15: channels
//              0-31 of Y_0, rows 16-31: channels 32-63)
//       sumsq: D_q[j] += Y_j^T x Y_j                                            (the diagonal)
//     accumulated over all of the wave's tiles in fp32 (~1000 terms per entry) -- the statistics of
//     the bf16 tensor that is stored (what bn1 normalises; the reference's bf16-autocast BatchNorm
//     sees the same rounded values); rows past the image edge are zeroed before;
//   * the bf16 tile goes out through the buffer the MFMAs just consumed, transposed: 4-pixel runs of
//     one channel as ds_write_b64 into [64 ch][32 px], back with ds_read_b64_tr_b16 as 8-channel
//     16-byte chunks of one pixel, 16-byte global stores;
//   * at the end each wave's (n, sum, M2 = sumsq - sum^2/n) merge (Chan, fp64) in LDS and each block
//     stores (sum, M2, sum^2/n) into slot blockIdx (the format avt_bn_finalize merges).
#pragma once

// orders a wave's own LDS writes before its later LDS reads of them (other lanes' data): a
// wavefront-scope fence -- no block barrier
__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

struct StemArgs {
  const bf16_t* x;  // [N][IH][IW][C]
  const bf16_t* w;  // [64][Kg], k' = (r*7+s)*C + c
  bf16_t* y;        // [N][OH][OW][64]
  double* stats;    // optional BN accumulator (avt_common.h): one slot per block
  unsigned x_bytes, y_bytes;
  int N, IH, IW, OH, OW, Kg;
  int tiles_per_row, total_tiles;
};

typedef short s16x8 __attribute__((ext_vector_type(8)));

constexpr int kStemPC = 70;    // patch columns of a 32-pixel tile: input x = 2*ow0 - 3 .. 2*ow0 + 66
constexpr int kStemNW = 8;     // waves per block (2 per SIMD)
constexpr int kStemTP = 72;    // bytes per channel row of the transposed output tile (64 + 8: banks)

template <int C>
struct StemCfg {
  static constexpr int KS = C == 4 ? 14 : 4;                 // MFMA k-steps
  static constexpr int ROWS = C == 4 ? 7 : 8;                // patch rows (C = 1: + the zero row)
  static constexpr int ROWB = kStemPC * C * 2;               // bytes per patch row
  static constexpr int LPL = (ROWS * kStemPC + 63) / 64;     // patch items (pixels) per lane
  static constexpr int PB0 = LPL * 64 * C * 2;               // patch bytes (whole lane rounds)
  static constexpr int PB = PB0 > 64 * kStemTP ? PB0 : 64 * kStemTP;  // buffer: patch, then out tile
  static constexpr int KP = KS * 16, BP = KP * 2 + 16;       // weight rows: K bf16 + 16 B (banks)
  static constexpr int WAVE_LDS = 2 * PB;                    // per wave: two buffers
  static constexpr int LDS = 64 * BP + kStemNW * WAVE_LDS;
  static_assert(kStemNW * WAVE_LDS >= kStemNW * 64 * 3 * 8, "the statistics merge reuses the wave regions");
};

template <int C>
__global__ __launch_bounds__(kStemNW * 64, 1) void conv_stem_fwd_kernel(StemArgs a) {
  using Cfg = StemCfg<C>;
  constexpr int NW = kStemNW, NTH = NW * 64;
  constexpr int KS = Cfg::KS, ROWS = Cfg::ROWS, ROWB = Cfg::ROWB, PB = Cfg::PB, LPL = Cfg::LPL;
  constexpr int KP = Cfg::KP, BP = Cfg::BP;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int frow = lane & 31, fhalf = lane >> 5;
  // LDS regions as offsets from smem (pointer arithmetic on smem keeps the LDS address space: an
  // array of LDS pointers indexed at run time lowers the fragment reads to flat loads)
  char* const Bs = smem;
  char* const wbase = smem + 64 * BP + wid * Cfg::WAVE_LDS;  // this wave's two buffers

  // ---- weights -> LDS once per block, in the kernel's k order: Bs [64][KP + 8] bf16 ----
  for (int u = tid; u < 64 * KP; u += NTH) {
    const int n = u / KP, k = u - n * KP;
    int kp = -1;  // packed index (r*7+s)*C + c, or none (dummy tap / row)
    if (C == 4) {
      const int rs = k >> 2, cc = k & 3, r = rs >> 3, s = rs & 7;
      if (s < 7) kp = (r * 7 + s) * 4 + cc;
    } else {
      const int r = k >> 3, s = k & 7;
      if (r < 7 && s < 7) kp = r * 7 + s;
    }
    *reinterpret_cast<bf16_t*>(Bs + n * BP + k * 2) = kp >= 0 ? a.w[(size_t)n * a.Kg + kp] : (bf16_t)0;
  }
  __syncthreads();  // the only block barrier before the statistics merge

  const __amdgpu_buffer_rsrc_t rsx = __builtin_amdgcn_make_buffer_rsrc((void*)a.x, (short)0, (int)a.x_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t rsy = __builtin_amdgcn_make_buffer_rsrc((void*)a.y, (short)0, (int)a.y_bytes, 0x00020000);
  typedef typename std::conditional<C == 4, u32x2, unsigned short>::type item_t;
  const int per_img = a.OH * a.tiles_per_row;
  // tile -> patch rows 2*oh-3 .. 2*oh+3 (+ the zero row), columns 2*ow0-3 .. 2*ow0+66
  // unconditional: a tile past the end loads zeros (out-of-range offsets), so every load and store
  // of the loop is issued in program order and the compiler's vmcnt waits stay counted (a
  // conditional load or store made it wait for everything, this tile's prefetch included)
  auto load_patch = [&](int t_in, item_t (&pre)[LPL]) {
    const bool live = t_in < a.total_tiles;
    const int t = live ? t_in : 0;
    const int img = t / per_img, rem = t - img * per_img;
    const int oh = rem / a.tiles_per_row, ow0 = (rem - oh * a.tiles_per_row) * 32;
    const int y0 = 2 * oh - 3, x0 = 2 * ow0 - 3;
    const int base = img * a.IH;
#pragma unroll
    for (int i = 0; i < LPL; ++i) {
      const int u = lane + 64 * i;
      const int g = u / kStemPC, col = u - g * kStemPC;
      const int yy = y0 + g, xx = x0 + col;
      const bool ok = live && g < 7 && (unsigned)yy < (unsigned)a.IH && (unsigned)xx < (unsigned)a.IW;
      const int off = ok ? ((base + yy) * a.IW + xx) * (C * 2) : (int)kOOB;
      if constexpr (C == 4)
        pre[i] = __builtin_bit_cast(u32x2, __builtin_amdgcn_raw_buffer_load_b64(rsx, off, 0, 0));
      else
        pre[i] = __builtin_amdgcn_raw_buffer_load_b16(rsx, off, 0, 0);
    }
  };
  auto store_patch = [&](int b, const item_t (&pre)[LPL]) {
#pragma unroll
    for (int i = 0; i < LPL; ++i) {
      const int u = lane + 64 * i;  // items past the patch land in the buffer's slack (never read)
      *reinterpret_cast<item_t*>(wbase + b * PB + u * C * 2) = pre[i];
    }
  };

  // statistics accumulators (see the header): D_s rows < 16 / >= 16 = channel sums of j = 0 / 1
  f32x16 dsum, dsq[2];
#pragma unroll
  for (int v = 0; v < 16; ++v) dsum[v] = dsq[0][v] = dsq[1][v] = 0.f;
  const __bf16 one = (__bf16)1.0f, zero = (__bf16)0.0f;
  const __bf16 s0v = frow < 16 ? one : zero, s1v = frow < 16 ? zero : one;
  const bf16x8 sel0 = {s0v, s0v, s0v, s0v, s0v, s0v, s0v, s0v};
  const bf16x8 sel1 = {s1v, s1v, s1v, s1v, s1v, s1v, s1v, s1v};
  int n_valid = 0;  // pixels this wave accounted (wave-uniform)

  const int P = a.OH * a.OW;
  const int stride = gridDim.x * NW;
  typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
  const int g4 = lane >> 4, t16 = lane & 15, q4 = t16 >> 2, pq = t16 & 3;

  // one tile: its patch is in buffer b; `nxt` holds the patch of tile t + stride (loaded one tile
  // earlier), `fut` receives tile t + 2 stride's -- two tiles of loads in flight per wave
  auto tile = [&](int t, int b, item_t (&nxt)[LPL], item_t (&fut)[LPL]) {
    load_patch(t + 2 * stride, fut);
    const int img = t / per_img, rem = t - img * per_img;
    const int oh = rem / a.tiles_per_row, ow0 = (rem - oh * a.tiles_per_row) * 32;
    const int rows_valid = min(32, a.OW - ow0);
    wave_lds_sync();  // this tile's patch (written by the whole wave) is complete
    const char* pb = wbase + b * PB + 2 * min(frow, rows_valid - 1) * C * 2;
    // fragment reads run two k-steps ahead of the MFMAs (sched_barrier fences keep the order; the
    // compiler alone waited for each read right before its MFMA: LDS latency on every k-step)
    auto frag_a = [&](int ks) -> bf16x8 {
      if constexpr (C == 4) {  // row ks/2, taps s0 = 4(ks&1) + 2 fhalf, s0 + 1
        return *reinterpret_cast<const bf16x8*>(pb + (ks >> 1) * ROWB + ((ks & 1) * 4 + 2 * fhalf) * 8);
      } else {  // row 2 ks + fhalf, columns 0..7
        const unsigned* q = reinterpret_cast<const unsigned*>(pb + (2 * ks + fhalf) * ROWB);
        u32x4 v;
        v.x = q[0];
        v.y = q[1];
        v.z = q[2];
        v.w = q[3];
        return __builtin_bit_cast(bf16x8, v);
      }
    };
    auto frag_b = [&](int ks, int j) -> bf16x8 {
      return *reinterpret_cast<const bf16x8*>(Bs + (j * 32 + frow) * BP + (16 * ks + 8 * fhalf) * 2);
    };
    constexpr int LA = 2;  // look-ahead in k-steps
    bf16x8 fa[LA + 1], fb[LA + 1][2];
#pragma unroll
    for (int ks = 0; ks < LA && ks < KS; ++ks) {
      fa[ks] = frag_a(ks);
      fb[ks][0] = frag_b(ks, 0);
      fb[ks][1] = frag_b(ks, 1);
    }
    f32x16 acc[2];
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      if (ks + LA < KS) {
        const int sl = (ks + LA) % (LA + 1);
        fa[sl] = frag_a(ks + LA);
        fb[sl][0] = frag_b(ks + LA, 0);
        fb[sl][1] = frag_b(ks + LA, 1);
      }
      __builtin_amdgcn_sched_barrier(0);
      const int sl = ks % (LA + 1);
#pragma unroll
      for (int j = 0; j < 2; ++j)
        acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[sl], fb[sl][j], ks == 0 ? f32x16{} : acc[j], 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);
    }
    // bf16 tile: pk[j][q] = rows (2q, 2q+1) of v order, channel j*32 + frow
    unsigned pk[2][8];
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int q = 0; q < 8; ++q) pk[j][q] = pack2(acc[j][2 * q], acc[j][2 * q + 1]);
    if (rows_valid < 32) {  // short last tile of a row: its clamped rows must not count
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const int r = ((2 * q) & 3) + 8 * ((2 * q) >> 2) + 4 * fhalf;
        const unsigned m = (r < rows_valid ? 0xffffu : 0u) | (r + 1 < rows_valid ? 0xffff0000u : 0u);
        pk[0][q] &= m;
        pk[1][q] &= m;
      }
    }
    n_valid += rows_valid;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const bf16x8 y0 = __builtin_bit_cast(bf16x8, u32x4{pk[0][4 * ks], pk[0][4 * ks + 1], pk[0][4 * ks + 2], pk[0][4 * ks + 3]});
      const bf16x8 y1 = __builtin_bit_cast(bf16x8, u32x4{pk[1][4 * ks], pk[1][4 * ks + 1], pk[1][4 * ks + 2], pk[1][4 * ks + 3]});
      dsum = __builtin_amdgcn_mfma_f32_32x32x16_bf16(sel0, y0, dsum, 0, 0, 0);
      dsum = __builtin_amdgcn_mfma_f32_32x32x16_bf16(sel1, y1, dsum, 0, 0, 0);
      dsq[0] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(y0, y0, dsq[0], 0, 0, 0);
      dsq[1] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(y1, y1, dsq[1], 0, 0, 0);
    }
    // the next tile's patch to the other buffer (its loads were issued a tile ago)
    store_patch(b ^ 1, nxt);
    // ---- the tile out, transposed through this (consumed) buffer: Tt [64 ch][32 px] ----
    char* const Tt = wbase + b * PB;
    wave_lds_sync();
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int g = 0; g < 4; ++g)  // pixels 8g + 4 fhalf .. + 3 of channel j*32 + frow
        *reinterpret_cast<u32x2*>(Tt + (j * 32 + frow) * kStemTP + (8 * g + 4 * fhalf) * 2) =
            u32x2{pk[j][2 * g], pk[j][2 * g + 1]};
    wave_lds_sync();
    const int ybase = (img * P + oh * a.OW + ow0) * 128;  // bytes
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      // 16-lane group g4 reads channels c0 .. c0+7 (two 4-row tr reads) of pixels p0 .. p0+15;
      // lane t16 then holds pixel p0 + t16's 16-byte chunk
      const int p0 = 16 * (i >> 1), c0 = 8 * (4 * (i & 1) + g4);
      const char* src = Tt + (c0 + q4) * kStemTP + (p0 + 4 * pq) * 2;
      const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(src));
      const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(src + 4 * kStemTP));
      const int px = p0 + t16;  // rows past the image edge: an out-of-range offset drops the store
      __builtin_amdgcn_raw_buffer_store_b128(
          __builtin_bit_cast(u32x4, s16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]}), rsy,
          px < rows_valid ? ybase + px * 128 + c0 * 2 : (int)kOOB, 0, 0);
    }
    wave_lds_sync();  // the tile read out before this buffer takes a patch again
  };

  // XCD-aware: consecutive virtual blocks (consecutive output rows, sharing input rows) on one XCD's L2
  int t = xcd_remap(blockIdx.x, gridDim.x) * NW + wid;
  item_t pa[LPL], pbuf[LPL];
  if (t < a.total_tiles) {
    load_patch(t, pa);
    store_patch(0, pa);
    load_patch(t + stride, pbuf);
  }
  for (; t < a.total_tiles; t += 2 * stride) {
    tile(t, 0, pbuf, pa);
    if (t + stride >= a.total_tiles) break;
    tile(t + stride, 1, pa, pbuf);
  }

  // ---- per-wave (n, sum, M2) -> LDS, Chan merge over the waves, publish ----
  if (a.stats != nullptr) {
    bn_write_header(a.stats, gridDim.x, 0);
    // channel frow of j: sum in dsum row 4 fhalf (j = 0) / 16 + 4 fhalf (j = 1) of column frow;
    // sumsq on the diagonal (row frow), held by the lane with fhalf = (frow >> 2) & 1
    const int vd = (frow & 3) + 4 * (frow >> 3);
    float q0 = 0.f, q1 = 0.f;
#pragma unroll
    for (int v = 0; v < 16; ++v) {
      q0 = v == vd ? dsq[0][v] : q0;
      q1 = v == vd ? dsq[1][v] : q1;
    }
    const float s0 = dsum[0], s1 = dsum[8];
    __syncthreads();  // every wave is done with its region: reuse the wave area
    double* red = reinterpret_cast<double*>(smem + 64 * BP);  // [NW waves][64 ch][3]
    if (fhalf == ((frow >> 2) & 1)) {
      const double n = (double)n_valid;
      const double sj[2] = {(double)s0, (double)s1}, qj[2] = {(double)q0, (double)q1};
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        double* q = red + ((size_t)wid * 64 + j * 32 + frow) * 3;
        q[0] = n;
        q[1] = sj[j];
        q[2] = n > 0.0 ? fmax(qj[j] - sj[j] * sj[j] / n, 0.0) : 0.0;
      }
    }
    __syncthreads();
    if (tid < 64) {
      double n = 0.0, s = 0.0, m2 = 0.0;
      for (int w = 0; w < NW; ++w) {
        const double* q = red + ((size_t)w * 64 + tid) * 3;
        const double nb = q[0];
        if (nb <= 0.0) continue;
        if (n > 0.0) {
          const double d = q[1] / nb - s / n;
          m2 += q[2] + d * d * n * nb / (n + nb);
        } else {
          m2 += q[2];
        }
        s += q[1];
        n += nb;
      }
      double* slot = bn_fwd_slots(a.stats) + ((size_t)blockIdx.x * 64 + tid) * 3;  // this block's own slot
      slot[0] = s;
      slot[1] = m2;
      slot[2] = n > 0.0 ? s * s / n : 0.0;
    }
  }
}

template <int C>
static size_t stem_lds_bytes() {
  return (size_t)StemCfg<C>::LDS;
}

template <int C>
static bool stem_fits(int OW) {
  return OW >= 1 && StemCfg<C>::LDS <= 160 * 1024;
}
