// 7x7 / stride 2 / pad 3 stem convolutions (models/base_models.py:135-138: the vision conv1 over
// 3 channels padded to 4, the audio conv1_a over 1 channel), K = 64 output channels, forward with
// the BN partial statistics of the other forward kernels.  Included by conv_gemm.hip inside
// namespace avt (needs AVT_BN_SLOTS, f2bf).
//
// The generic kernel gathers the stem's im2col one element at a time (C = 1 or 4 channels, 49 taps:
// 86-212 TFLOP/s).  Here a block owns kStemBM = 512 consecutive output pixels of ONE image, copies
// the input rows they read (with the 3-column padding) into an LDS patch once, and every A fragment
// is read straight out of the patch:
//   C = 4: k = (r*8 + s)*4 + c (a dummy 8th tap s = 7 with zero weight): a lane's 8 k values are
//          taps (r, s0), (r, s0+1) x 4 channels = two adjacent patch pixels = one ds_read_b128;
//          K = 7*8*4 = 224 (49*4 = 196 real), 14 MFMA k-steps.
//   C = 1: k = r*8 + s (dummy tap s = 7, dummy row r = 7): a lane's 8 k values are one patch row's
//          8 columns 2ow .. 2ow+7 = four ds_read_b32; K = 64 (49 real), 4 k-steps.
// The weights are re-laid out into that k order in LDS as the block starts (from the packed
// [64][Kg] operand of avt_pack_conv_weight, k = (r*7+s)*C + c).  4 waves x 128 rows (4 x 32-row
// MFMA tiles) x 64 columns; epilogue: BN partial statistics per 128-row wave tile (sum, M2 about the
// tile mean, sum^2/n: the format of the other conv epilogues), bf16 tile through LDS, 16-byte
// coalesced stores.  Bound: the 2 B per output element store (205 MB vision, 317 MB audio at
// B = 128) and the MFMA work of the padded K.
// Measured on MI355X (tools/stem_ab.sh, B = 128 step): conv fwd 3.42 ms/step here vs 3.16 ms on the
// generic kernel at 1 wave/SIMD (213 VGPR + 128 AGPR); with __launch_bounds__(256, 2) and the k loop
// unrolled by 2 (220 VGPR, 2 blocks per CU) 3.35 vs 3.30 ms -- a tie, so it stays OFF by default
// (AVT_STEM=1 / avt_set_stem_kernel(1) selects it).  What is left: one image per block leaves the
// last block of each image partly idle (OH*OW % 512), and the LDS patch fill is serialised ahead of
// the MFMA work (no double buffering) -- the store-bound floor (35-45 us per stem) is ~4x away.
#pragma once

struct StemArgs {
  const bf16_t* x;  // [N][IH][IW][C]
  const bf16_t* w;  // [64][Kg], k = (r*7+s)*C + c
  bf16_t* y;        // [N][OH][OW][64]
  double* stats;    // optional [AVT_BN_SLOTS][64][3]
  int IH, IW, OH, OW, Kg;
  int blocks_per_img;
};

constexpr int kStemBM = 512;
constexpr int kStemCT = 64 * 2 + 16;         // epilogue row pitch (bytes)
constexpr int kStemLds = 4 * 128 * kStemCT;  // 72 KB: the epilogue tiles; 2 blocks per CU

template <int C>
struct StemCfg {
  static constexpr int KP = C == 4 ? 224 : 64;  // LDS k extent
  static constexpr int KS = KP / 16;            // MFMA k-steps
  static constexpr int BP = KP * 2 + 16;        // LDS weight row pitch (bytes)
};

template <int C>
__global__ __launch_bounds__(256, 2) void conv_stem_fwd_kernel(StemArgs a) {
  using Cfg = StemCfg<C>;
  constexpr int KS = Cfg::KS, BP = Cfg::BP;
  __shared__ __attribute__((aligned(16))) char smem[kStemLds];
  char* Bs = smem;            // [64][BP]
  char* Ps = smem + 64 * BP;  // patch [nrows][PW][C] bf16
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int frow = lane & 31, fhalf = lane >> 5;
  const int img = blockIdx.x / a.blocks_per_img, blk = blockIdx.x - img * a.blocks_per_img;
  const int P = a.OH * a.OW;
  const int p0 = blk * kStemBM;
  const int oh_first = p0 / a.OW;
  const int oh_last = (min(p0 + kStemBM, P) - 1) / a.OW;
  const int nrows = 2 * (oh_last - oh_first) + 8;  // input rows 2*oh_first-3 ..; the last is a zero row
  const int PW = 2 * a.OW + 6;                     // input columns -3 .. 2*OW+2

  // ---- weights -> LDS in the kernel's k order ----
  if (C == 4) {
    for (int u = tid; u < 64 * 56; u += 256) {  // (n, r, s) units of 4 channels = 8 bytes
      const int n = u / 56, rs = u - n * 56, r = rs >> 3, s = rs & 7;
      u32x2 v = {0u, 0u};
      if (s < 7) v = *reinterpret_cast<const u32x2*>(a.w + (size_t)n * a.Kg + (r * 7 + s) * 4);
      *reinterpret_cast<u32x2*>(Bs + n * BP + rs * 8) = v;
    }
  } else {
    for (int u = tid; u < 64 * 64; u += 256) {
      const int n = u >> 6, rs = u & 63, r = rs >> 3, s = rs & 7;
      const bf16_t v = (r < 7 && s < 7) ? a.w[(size_t)n * a.Kg + r * 7 + s] : (bf16_t)0;
      *reinterpret_cast<bf16_t*>(Bs + n * BP + rs * 2) = v;
    }
  }
  // ---- input patch -> LDS (zeros outside the image and in the last row) ----
  const bf16_t* xi = a.x + (size_t)img * a.IH * a.IW * C;
  const int y0 = 2 * oh_first - 3;
  for (int u = tid; u < nrows * PW; u += 256) {
    const int g = u / PW, col = u - g * PW;
    const int y = y0 + g, x = col - 3;
    const bool ok = g < nrows - 1 && y >= 0 && y < a.IH && x >= 0 && x < a.IW;
    if (C == 4) {
      u32x2 v = {0u, 0u};
      if (ok) v = *reinterpret_cast<const u32x2*>(xi + ((size_t)y * a.IW + x) * 4);
      *reinterpret_cast<u32x2*>(Ps + u * 8) = v;
    } else {
      *reinterpret_cast<bf16_t*>(Ps + u * 2) = ok ? xi[(size_t)y * a.IW + x] : (bf16_t)0;
    }
  }
  __syncthreads();

  // ---- per m-tile patch offset of this lane's pixel (rows past the image end: the last pixel) ----
  int abase[4];
#pragma unroll
  for (int mt = 0; mt < 4; ++mt) {
    const int p = min(p0 + wid * 128 + mt * 32 + frow, P - 1);
    const int oh = p / a.OW, ow = p - oh * a.OW;
    abase[mt] = ((2 * (oh - oh_first)) * PW + 2 * ow) * C * 2;
  }
  f32x16 acc[4][2];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int v = 0; v < 16; ++v) acc[i][j][v] = 0.f;

#pragma unroll 2
  for (int ks = 0; ks < KS; ++ks) {
    bf16x8 bfr[2];
#pragma unroll
    for (int j = 0; j < 2; ++j)
      bfr[j] = *reinterpret_cast<const bf16x8*>(Bs + (j * 32 + frow) * BP + (16 * ks + 8 * fhalf) * 2);
#pragma unroll
    for (int mt = 0; mt < 4; ++mt) {
      bf16x8 af;
      if (C == 4) {  // taps t0 = 4ks + 2fhalf, t0+1: row ks/2, columns s0, s0+1
        const int off = ((ks >> 1) * PW + (4 * ks & 7) + 2 * fhalf) * 8;
        af = *reinterpret_cast<const bf16x8*>(Ps + abase[mt] + off);
      } else {  // row r = 2ks + fhalf, columns 0..7
        const char* q = Ps + abase[mt] + (2 * ks + fhalf) * PW * 2;
        u32x4 v;
        v.x = *reinterpret_cast<const unsigned*>(q + 0);
        v.y = *reinterpret_cast<const unsigned*>(q + 4);
        v.z = *reinterpret_cast<const unsigned*>(q + 8);
        v.w = *reinterpret_cast<const unsigned*>(q + 12);
        af = __builtin_bit_cast(bf16x8, v);
      }
#pragma unroll
      for (int j = 0; j < 2; ++j) acc[mt][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af, bfr[j], acc[mt][j], 0, 0, 0);
    }
  }

  // ---- BN partial statistics of this wave's 128-row tile (fp32 results, before rounding) ----
  const int rows_valid = min(128, P - (p0 + wid * 128));
  if (a.stats != nullptr && rows_valid > 0) {
    const size_t tile = ((size_t)img * a.blocks_per_img + blk) * 4 + wid;
    double* slot = a.stats + (tile % AVT_BN_SLOTS) * 64 * 3;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      float s = 0.f;
#pragma unroll
      for (int mt = 0; mt < 4; ++mt)
#pragma unroll
        for (int v = 0; v < 16; ++v) {
          const int r = mt * 32 + (v & 3) + 8 * (v >> 2) + 4 * fhalf;
          if (r < rows_valid) s += acc[mt][j][v];
        }
      s += __shfl_xor(s, 32, 64);
      const float mean = s / (float)rows_valid;
      float q = 0.f;
#pragma unroll
      for (int mt = 0; mt < 4; ++mt)
#pragma unroll
        for (int v = 0; v < 16; ++v) {
          const int r = mt * 32 + (v & 3) + 8 * (v >> 2) + 4 * fhalf;
          const float d = acc[mt][j][v] - mean;
          if (r < rows_valid) q += d * d;
        }
      q += __shfl_xor(q, 32, 64);
      if (lane < 32) {
        double* c3 = slot + (size_t)(j * 32 + frow) * 3;
        atomicAdd(c3 + 0, (double)s);
        atomicAdd(c3 + 1, (double)q);
        atomicAdd(c3 + 2, (double)s * (double)s / (double)rows_valid);
      }
    }
  }

  // ---- bf16 tile through LDS (each wave its own 128 x 64 region), 16-byte stores ----
  __syncthreads();  // every wave is done with the patch and the weights
  char* Ct = smem + wid * 128 * kStemCT;
#pragma unroll
  for (int mt = 0; mt < 4; ++mt)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int v = 0; v < 16; ++v) {
        const int r = mt * 32 + (v & 3) + 8 * (v >> 2) + 4 * fhalf;
        *reinterpret_cast<bf16_t*>(Ct + r * kStemCT + (j * 32 + frow) * 2) = f2bf(acc[mt][j][v]);
      }
  // a wave's LDS accesses complete in issue order: its own tile is read back without a barrier
  bf16_t* yo = a.y + ((size_t)img * P + p0 + wid * 128) * 64;
  for (int u = lane; u < 128 * 8; u += 64) {
    const int r = u >> 3, c = u & 7;
    if (r < rows_valid)
      *reinterpret_cast<u32x4*>(yo + (size_t)r * 64 + c * 8) =
          *reinterpret_cast<const u32x4*>(Ct + r * kStemCT + c * 16);
  }
}

// patch rows a block of kStemBM pixels can need (incl. the zero row)
static inline int stem_patch_rows(int OW) { return 2 * ((kStemBM - 1) / OW + 1) + 8; }

template <int C>
static bool stem_fits(int OW) {
  return 64 * StemCfg<C>::BP + (size_t)stem_patch_rows(OW) * (2 * OW + 6) * C * 2 <= (size_t)kStemLds;
}
