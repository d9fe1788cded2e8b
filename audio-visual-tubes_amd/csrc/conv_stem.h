// 7x7 / stride 2 / pad 3 stem convolutions (models/base_models.py:135-138: the vision conv1 over
// 3 channels padded to 4, the audio conv1_a over 1 channel), 64 output channels, forward with the BN
// partial statistics of the other forward kernels.  Included by conv_gemm.hip inside namespace avt
// (needs AVT_BN_SLOTS, f2bf).
//
// The stem is store-bound: 1 input channel-group in, 64 bf16 channels out per output pixel (205 MB
// vision / 317 MB audio at B = 128 against 51 / 20 MB of input), so the kernel is organised around
// keeping the output stream going:
//   * persistent: 512-thread blocks (8 waves) loop over 256-pixel chunks of one image (row-major
//     output pixels), so the 64 x K weight operand goes to LDS once per block (kept in registers it
//     spilled: 112 VGPRs of vision B fragments);
//   * the chunk's input rows (its "patch": 2*(rows spanned - 1) + 7 input rows, the 3-column padding
//     and out-of-image rows as zeros) sit in LDS, double-buffered: the next chunk's patch is loaded
//     into registers while this chunk multiplies and written to the other buffer after it, one
//     block barrier per chunk;
//   * each wave owns one 32-pixel M tile of the chunk: A fragments straight out of the patch,
//       C = 4: k = (r*8 + s)*4 + c (dummy tap s = 7, zero weight): a lane's 8 k values are taps
//              (r, s0), (r, s0+1) x 4 channels = two adjacent patch pixels = one ds_read_b128;
//              K = 224 (196 real), 14 MFMA k-steps;
//       C = 1: k = r*8 + s (dummy row r = 7 and tap s = 7): a lane's 8 k values are 8 adjacent
//              columns of one patch row = two ds_read2_b32; K = 64 (49 real), 4 k-steps;
//   * epilogue per chunk and wave: BN statistics of the 32-row tile (sum, and sum of squares about a
//     per-channel shift = the wave's first tile mean) accumulated per lane in fp64 -- no division in
//     the loop; M2 = Q - (S - n shift)^2 / n once at the end --, the bf16 tile through the wave's own
//     LDS region (no block barrier), four 16-byte stores per lane of the wave's contiguous 4 KB;
//     at the end the 8 waves' statistics merge in LDS and each block adds (sum, M2, sum^2/n) into
//     slot blockIdx % AVT_BN_SLOTS (the format avt_bn_finalize merges).
#pragma once

struct StemArgs {
  const bf16_t* x;  // [N][IH][IW][C]
  const bf16_t* w;  // [64][Kg], k' = (r*7+s)*C + c
  bf16_t* y;        // [N][OH][OW][64]
  double* stats;    // optional [AVT_BN_SLOTS][64][3]
  int N, IH, IW, OH, OW, Kg;
  int chunks_per_img, total_chunks;
};

constexpr int kStemCH = 256;     // output pixels per chunk (8 waves x 32)
constexpr int kStemCTP = 144;    // bytes per pixel row of a wave's staging tile (128 + 16 pad)

template <int C>
struct StemCfg {
  static constexpr int KS = C == 4 ? 14 : 4;  // MFMA k-steps
  static constexpr int MAXROWS = C == 4 ? 14 : 12;  // patch rows incl. one spare zero row
};

// patch geometry of a chunk
struct StemChunk {
  int img, p0, nvalid, oh_first, nrows;
};

__device__ __forceinline__ StemChunk stem_chunk(const StemArgs& a, int c) {
  StemChunk k;
  k.img = c / a.chunks_per_img;
  const int blk = c - k.img * a.chunks_per_img;
  const int P = a.OH * a.OW;
  k.p0 = blk * kStemCH;
  k.nvalid = min(kStemCH, P - k.p0);
  k.oh_first = k.p0 / a.OW;
  const int oh_last = (k.p0 + k.nvalid - 1) / a.OW;
  k.nrows = 2 * (oh_last - k.oh_first) + 8;  // + a zero row (the C = 1 dummy row r = 7 reads it)
  return k;
}

template <int C>
__global__ __launch_bounds__(512, 2) void conv_stem_fwd_kernel(StemArgs a) {
  using Cfg = StemCfg<C>;
  constexpr int KS = Cfg::KS, MAXROWS = Cfg::MAXROWS;
  const int PW = 2 * a.OW + 6;         // patch columns: input x = -3 .. 2*OW + 2
  const int ROWB = PW * C * 2;         // bytes per patch row
  const int PATCHB = MAXROWS * ROWB;   // bytes per patch buffer
  constexpr int KP = KS * 16, BP = KP * 2 + 16;  // weight rows: K bf16 + 16 B (bank spread)
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* Bs = smem;
  char* const patch0 = smem + 64 * BP;  // patch buffer b at patch0 + b * PATCHB (pointer arithmetic on
                                        // smem: an array of LDS pointers indexed at run time lowered
                                        // the fragment reads to flat loads)
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int frow = lane & 31, fhalf = lane >> 5;
  char* Ct = smem + 64 * BP + 2 * PATCHB + wid * 32 * kStemCTP;  // this wave's staging tile

  // ---- weights -> LDS once per block, in the kernel's k order: Bs [64][KP + 8] bf16 ----
  for (int u = tid; u < 64 * KP; u += 512) {
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

  // ---- patch loads: thread t covers items t, t + 512, ... of (row, column) (C = 4: 8-B pixels) ----
  constexpr int LPT = C == 4 ? 7 : 8;  // items per thread: 14 rows x 230 cols / 512; 12 x 306 / 512
  typedef typename std::conditional<C == 4, u32x2, unsigned short>::type item_t;
  item_t pre[LPT];
  auto load_patch = [&](const StemChunk& k) {
    const bf16_t* xi = a.x + (size_t)k.img * a.IH * a.IW * C;
    const int y0 = 2 * k.oh_first - 3;
    const int n_items = k.nrows * PW;
#pragma unroll
    for (int i = 0; i < LPT; ++i) {
      const int u = tid + i * 512;
      const int g = u / PW, col = u - g * PW;
      const int yy = y0 + g, xx = col - 3;
      const bool ok = u < n_items && g < k.nrows - 1 && yy >= 0 && yy < a.IH && xx >= 0 && xx < a.IW;
      if constexpr (C == 4) {
        pre[i] = ok ? *reinterpret_cast<const u32x2*>(xi + ((size_t)yy * a.IW + xx) * 4) : u32x2{0u, 0u};
      } else {
        pre[i] = ok ? xi[(size_t)yy * a.IW + xx] : (unsigned short)0;
      }
    }
  };
  auto store_patch = [&](const StemChunk& k, char* dst) {
    const int n_items = k.nrows * PW;
#pragma unroll
    for (int i = 0; i < LPT; ++i) {
      const int u = tid + i * 512;
      if (u < n_items) *reinterpret_cast<item_t*>(dst + (size_t)u * C * 2) = pre[i];
    }
  };

  // running BN statistics of this lane's two channels (j = 0, 1): rows n, sum, and the sum of squares
  // about a per-channel shift (the first tile's mean) -- no division in the chunk loop; the M2 about
  // the running mean is recovered once at the end (shifted-data variance)
  double st_n = 0.0, st_s[2] = {0.0, 0.0}, st_q[2] = {0.0, 0.0};
  float shift[2] = {0.f, 0.f};
  bool have_shift = false;

  int c = blockIdx.x;
  StemChunk cur{};
  if (c < a.total_chunks) {
    cur = stem_chunk(a, c);
    load_patch(cur);
    store_patch(cur, patch0);
  }
  int buf = 0;
  const int P = a.OH * a.OW;
  for (; c < a.total_chunks; c += gridDim.x) {
    __syncthreads();  // patch[buf] complete; every wave is past its reads of patch[buf ^ 1]
    const int cn = c + gridDim.x;
    StemChunk nxt{};
    if (cn < a.total_chunks) {
      nxt = stem_chunk(a, cn);
      load_patch(nxt);  // in flight during this chunk's MFMAs
    }
    // ---- this wave's 32-pixel tile ----
    const int row0 = wid * 32;  // first tile row within the chunk
    const int rows_valid = min(32, cur.nvalid - row0);
    if (rows_valid > 0) {
      const int p = cur.p0 + row0 + min(frow, rows_valid - 1);  // clamp: tail rows compute a valid pixel
      const int oh = p / a.OW, ow = p - oh * a.OW;
      const char* pb = patch0 + buf * PATCHB + (2 * (oh - cur.oh_first)) * ROWB + (2 * ow) * C * 2;
      f32x16 acc[2];
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int v = 0; v < 16; ++v) acc[j][v] = 0.f;
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        bf16x8 af;
        if constexpr (C == 4) {  // row ks/2, taps s0 = 4(ks&1) + 2 fhalf, s0 + 1
          af = *reinterpret_cast<const bf16x8*>(pb + (ks >> 1) * ROWB + ((ks & 1) * 4 + 2 * fhalf) * 8);
        } else {  // row 2 ks + fhalf, columns 0..7
          const unsigned* q = reinterpret_cast<const unsigned*>(pb + (2 * ks + fhalf) * ROWB);
          u32x4 v;
          v.x = q[0];
          v.y = q[1];
          v.z = q[2];
          v.w = q[3];
          af = __builtin_bit_cast(bf16x8, v);
        }
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const bf16x8 bf = *reinterpret_cast<const bf16x8*>(Bs + (j * 32 + frow) * BP + (16 * ks + 8 * fhalf) * 2);
          acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af, bf, acc[j], 0, 0, 0);
        }
      }
      // ---- BN statistics of the tile (fp32 values before rounding): sum and sum of squares about the
      //      channel's shift, accumulated in fp64 ----
      if (a.stats != nullptr) {
        if (!have_shift) {  // first tile of this wave: its mean becomes the shift
#pragma unroll
          for (int j = 0; j < 2; ++j) {
            float sm = 0.f;
#pragma unroll
            for (int v = 0; v < 16; ++v) {
              const int r = (v & 3) + 8 * (v >> 2) + 4 * fhalf;
              if (r < rows_valid) sm += acc[j][v];
            }
            sm += __shfl_xor(sm, 32, 64);
            shift[j] = sm / (float)rows_valid;
          }
          have_shift = true;
        }
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          float sm = 0.f, q = 0.f;
#pragma unroll
          for (int v = 0; v < 16; ++v) {
            const int r = (v & 3) + 8 * (v >> 2) + 4 * fhalf;
            const float d = acc[j][v] - shift[j];
            if (r < rows_valid) {
              sm += acc[j][v];
              q += d * d;
            }
          }
          sm += __shfl_xor(sm, 32, 64);
          q += __shfl_xor(q, 32, 64);
          st_s[j] += (double)sm;
          st_q[j] += (double)q;
        }
        st_n += (double)rows_valid;
      }
      // the next chunk's patch goes to LDS now, before this tile's stores: its wait for the
      // prefetch loads then does not also wait for the output stores (vmcnt counts both, in order)
      if (cn < a.total_chunks) store_patch(nxt, patch0 + (buf ^ 1) * PATCHB);
      // ---- bf16 tile through this wave's LDS region, then its contiguous 4 KB out ----
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int v = 0; v < 16; ++v) {
          const int r = (v & 3) + 8 * (v >> 2) + 4 * fhalf;
          *reinterpret_cast<bf16_t*>(Ct + r * kStemCTP + (j * 32 + frow) * 2) = f2bf(acc[j][v]);
        }
      // a wave's LDS accesses complete in order: its own tile is read back without a barrier
      bf16_t* yo = a.y + ((size_t)cur.img * P + cur.p0 + row0) * 64;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int u = lane + 64 * i;  // 256 chunks of 16 B: row u / 8, 16-B column u % 8
        const int r = u >> 3, cc = u & 7;
        if (r < rows_valid)
          *reinterpret_cast<u32x4*>(yo + (size_t)r * 64 + cc * 8) =
              *reinterpret_cast<const u32x4*>(Ct + r * kStemCTP + cc * 16);
      }
    } else if (cn < a.total_chunks) {
      store_patch(nxt, patch0 + (buf ^ 1) * PATCHB);
    }
    cur = nxt;
    buf ^= 1;
  }

  // ---- merge the 8 waves' statistics (lanes < 32 hold channels j*32 + frow) and publish ----
  if (a.stats != nullptr) {
    __syncthreads();  // the patch buffers are free: reuse them
    double* red = reinterpret_cast<double*>(smem + 64 * BP);  // [8 waves][64 ch][3]
    if (lane < 32) {
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        double* q = red + ((size_t)wid * 64 + j * 32 + frow) * 3;
        // M2 about this wave's mean: Q - (S - n c)^2 / n
        const double dc = st_n > 0.0 ? st_s[j] - st_n * (double)shift[j] : 0.0;
        q[0] = st_n;
        q[1] = st_s[j];
        q[2] = st_n > 0.0 ? fmax(st_q[j] - dc * dc / st_n, 0.0) : 0.0;
      }
    }
    __syncthreads();
    if (tid < 64) {
      double n = 0.0, s = 0.0, m2 = 0.0;
      for (int w = 0; w < 8; ++w) {
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
      if (n > 0.0) {
        double* slot = a.stats + ((size_t)(blockIdx.x % AVT_BN_SLOTS) * 64 + tid) * 3;
        atomicAdd(slot + 0, s);
        atomicAdd(slot + 1, m2);
        atomicAdd(slot + 2, s * s / n);
      }
    }
  }
}

template <int C>
static size_t stem_lds_bytes(int OW) {
  const size_t bs = (size_t)64 * (StemCfg<C>::KS * 16 * 2 + 16);
  const size_t patchb = (size_t)StemCfg<C>::MAXROWS * (2 * OW + 6) * C * 2;
  const size_t need = 2 * patchb + 8 * 32 * kStemCTP;
  const size_t red = (size_t)8 * 64 * 3 * sizeof(double);
  return bs + (need > red ? need : red);
}

// the chunk's rows must fit the patch: a 256-pixel chunk spans <= ceil(255 / OW) + 1 output rows
template <int C>
static bool stem_fits(int OW) {
  const int rows_spanned = (kStemCH - 1) / OW + 2;
  const int nrows = 2 * (rows_spanned - 1) + 8;
  const int PW = 2 * OW + 6;
  const int items_per_thread = C == 4 ? 7 : 8;
  return OW >= 8 && nrows <= StemCfg<C>::MAXROWS && nrows * PW <= items_per_thread * 512 &&
         stem_lds_bytes<C>(OW) <= 160 * 1024;
}

// blocks per CU of the persistent grid (~180 VGPRs: two waves per SIMD)
template <int C>
static int stem_blocks_per_cu() { return 1; }
