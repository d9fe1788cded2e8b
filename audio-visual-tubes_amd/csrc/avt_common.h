// Shared device/host helpers for libavt (gfx950 / CDNA4 only).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>
#include <stdio.h>

#include "avt.h"  // (include/, -I) the C-ABI: every extern "C" definition must match its declaration

typedef unsigned short bf16_t;  // storage type: raw bf16 bits
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));

#define AVT_OK 0
#define AVT_EINVAL -1
#define AVT_EHIP -2

namespace avt {

// ---- BatchNorm statistic accumulators (deterministic; include/avt.h "BatchNorm statistics") ----
// fp64 [kBnHdr header][bwd only: k1, k2 = 2C floats = C doubles][slot][C][W] (W = 3 fwd: sum, M2, sum^2/n;
// W = 2 bwd: sum g', sum g'*xhat).  Every slot is written by exactly ONE block of the accumulating launch, with
// plain stores (no atomics, no zeroing); header[0] = the slots that launch wrote, header[1] = slots a second
// launch appended after them (a stride-2 dgrad's downsample twin, conv_epi.h).  The finalize kernels sum
// the slots in slot order, so the statistics -- and everything downstream -- are the same bits on every
// run.  Capacity: one slot per 64 rows (the smallest row tile) + 520 (persistent / reduce grids <= 512).
constexpr int kBnHdr = 8;
__host__ __device__ inline long long bn_slot_cap(long long rows) { return (rows + 63) / 64 + 520; }
__device__ __forceinline__ double* bn_fwd_slots(double* acc) { return acc + kBnHdr; }
__device__ __forceinline__ double* bn_bwd_slots(double* acc, int C) { return acc + kBnHdr + C; }
// the launch's slot count, recorded by ONE block of it (`leader`: a block that surely reaches the call);
// append: after the slots of the launch it appends to -- header[0], written by that earlier launch on the same
// stream (bn_slot_base) -- into header[1]
__device__ __forceinline__ void bn_write_header(double* acc, int nslots, int append, bool leader) {
  if (leader && threadIdx.x == 0) {
    if (append) {
      acc[1] = (double)nslots;
    } else {
      acc[0] = (double)nslots;
      acc[1] = 0.0;
    }
  }
}
__device__ __forceinline__ void bn_write_header(double* acc, int nslots, int append) {
  bn_write_header(acc, nslots, append, blockIdx.x == 0);
}
__device__ __forceinline__ int bn_slot_base(const double* acc, int append) { return append ? (int)acc[0] : 0; }

// exact floor(n / d) for 32-bit n by a multiply-high and a shift (Granlund-Montgomery)
struct MagicDiv {  // exact floor(n / d) for 32-bit n (Granlund-Montgomery)
  unsigned m, l;
};

static inline MagicDiv make_magic(unsigned d) {
  unsigned l = 0;
  while ((1ull << l) < d) ++l;
  const unsigned long long m = ((1ull << 32) * ((1ull << l) - d)) / d + 1;
  return MagicDiv{(unsigned)m, l};
}

__device__ __forceinline__ unsigned magic_div(unsigned n, MagicDiv md) {
  if (md.l == 0) return n;  // d == 1
  const unsigned t = __umulhi(md.m, n);
  return (t + ((n - t) >> 1)) >> (md.l - 1);
}

void set_error(const char* fmt, ...);
int check_launch(const char* what);

__device__ __forceinline__ float bf2f(bf16_t h) { return __uint_as_float(((unsigned)h) << 16); }
__device__ __forceinline__ bf16_t f2bf(float f) {
  __bf16 b = (__bf16)f;  // v_cvt_pk_bf16_f32 (RNE) on gfx950
  return __builtin_bit_cast(bf16_t, b);
}
__device__ __forceinline__ unsigned pack2(float lo, float hi) {
  return (unsigned)f2bf(lo) | ((unsigned)f2bf(hi) << 16);
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Block-wide sum for blockDim.x <= 1024 (multiple of 64). `red` needs blockDim.x/64 floats.
__device__ __forceinline__ float block_sum(float v, float* red) {
  v = wave_sum(v);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
  __syncthreads();
  if (lane == 0) red[wid] = v;
  __syncthreads();
  float t = 0.f;
  for (int i = 0; i < nw; ++i) t += red[i];
  return t;
}

// Timing diagnostics, compiled only into the -DAVT_DIAG build (tools/build_variant.sh; avt_build_flags()
// reports it and bench.py refuses it): AVT_DIAG_SKIP bit mask of launches to leave out of a captured graph
// (1: forward bn_finalize, 2: backward bn finalize, 4: wgrad slab reduce, 8: backward BN reductions, 16: forward
// bn_apply; 32 / 64: the forward / backward BN finalizes launched TWICE -- a valid marginal cost of one finalize
// launch, every tensor keeping realistic values); results are WRONG when set.  Only the captured graph leaves them out.  The persistent BN accumulators
// keep what the eager warm-up wrote (bits 2, 8: the replays run on realistic statistics); the tensors a skipped
// launch would write inside the graph (bit 16) are graph-pool memory nobody wrote -- the data trap below.
// Caveat, measured: the step's speed depends on the data -- a graph whose BN statistics are never written
// normalises with uninitialised scale/shift, its activations collapse, and every MFMA kernel runs ~8-10 %
// faster (power/clock), which reads as a spurious ~1 ms "cost" of the finalize launches at B=128
// (DESIGN.md section 6).  The shipping build ignores the variable.
#ifdef AVT_DIAG
inline bool diag_skip(int bit, hipStream_t st) {
  static int v = -1;
  if (v < 0) v = getenv("AVT_DIAG_SKIP") ? atoi(getenv("AVT_DIAG_SKIP")) : 0;
  if (!(v & bit)) return false;
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  return hipStreamIsCapturing(st, &cs) == hipSuccess && cs == hipStreamCaptureStatusActive;
}
#else
inline bool diag_skip(int, hipStream_t) { return false; }
#endif

}  // namespace avt

#define AVT_REQUIRE(cond, ...)            \
  do {                                     \
    if (!(cond)) {                         \
      avt::set_error(__VA_ARGS__);         \
      return AVT_EINVAL;                   \
    }                                      \
  } while (0)
