// NT implicit-GEMM convolution, LDS-DMA pipeline (fwd / dgrad, C % 32 == 0).  Included by
// conv_gemm.hip inside namespace avt (needs GemmNTParams, swz64, MODE_*).
//
// Every operand chunk goes global -> LDS with `buffer_load_dwordx4 ... lds` (per-lane byte offset,
// lane-linear LDS image, XOR swizzle applied to the SOURCE chunk).  Out-of-image taps get an
// out-of-range offset, so the buffer unit writes zeros (no branches, no zero page).  The K loop
// walks an explicit tap list: all R*S taps, or — for the dgrad of a stride-2 conv — only the
// taps of one output parity class (rows are the pixels (2h'+ph, 2w'+pw) of that class), which
// removes the 3/4 of zero work a plain gather-dgrad would do.  Per lane and row the offset of the
// class origin and a bitmask of in-image taps are precomputed; a k-tile costs ~3 VALU per
// gathered row.  NST-stage ring, NST-1 tiles in flight, one counted vmcnt + raw s_barrier per
// k-tile (tiles past the end are issued as all-OOB dummies so the count is constant), XCD-aware
// tile order.
#pragma once
#include <type_traits>

template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

__device__ __forceinline__ int xcd_remap(int orig, int nwg) {
  const int xcd = orig & 7, q = nwg >> 3, r = nwg & 7;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (orig >> 3);
}

constexpr unsigned kOOB = 0x80000000u;  // beyond any activation buffer: the load returns zeros

typedef __attribute__((address_space(3))) void lds_void_t;

// The ring's barrier.  Every wave's LDS reads of the stage it is done with must have RETURNED before any
// wave passes the barrier and DMAs the next tile into that stage.  s_barrier is no memory fence to the
// compiler: it sinks a step's last MFMA below the barrier and with it the lgkmcnt wait for that MFMA's
// fragment read (seen in the gfx950 assembly: `s_waitcnt lgkmcnt(1); s_barrier; ... lgkmcnt(3); mfma`), so
// the read was still in flight while the other waves' DMA rewrote its stage -- rarely late enough to lose,
// which showed as run-to-run differences (a few launches in hundreds of the small-tile halo kernels;
// test_small_grid_conv_repeatable, tools/diag.py rep).  The explicit lgkmcnt(0) retires them first.
__device__ __forceinline__ void ring_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
}

// Issued as inline asm, not __builtin_amdgcn_raw_ptr_buffer_load_lds: the compiler treats every
// LDS read after a builtin LDS-DMA as possibly aliasing it and inserts `s_waitcnt vmcnt(0)` in
// front of the fragment reads, which drains ALL in-flight tiles each k-step and collapses the
// NST-stage ring to no overlap at all (seen in the gfx950 assembly of the TN and halo kernels).
// Opaque to the waitcnt pass, the loads are ordered only by the kernels' own counted
// wait_vmcnt + s_barrier, which is what the ring was designed around.  (vmcnt retires in issue
// order, so the compiler's waits for its own loads stay correct — at worst they over-wait.)
// m0 carries the wave's LDS base.  It is not listed as clobbered: LLVM ignores clobbers of reserved
// registers (with a warning per instantiation); the gfx950 code of these kernels has no other m0
// use (no movrel/sendmsg; checked in the --save-temps assembly), so nothing live is overwritten.
// The `s_nop 0` between the M0 write and the LDS-DMA is the required wait state (an SALU write of M0 ->
// an LDS-DMA reading it; hipcc pads nothing inside an asm string).  Without it an LDS-DMA could take the
// PREVIOUS M0 -- land on the previous instruction's LDS slot -- on some waves of some launches: run-to-run
// differences of a few launches in hundreds (the small-tile halo dgrad at 32 clips,
// test_small_grid_conv_repeatable / tools/diag.py rep), which no tolerance check of the results can see.
// lds_addr: the LDS byte address itself (an integer computed once from a shared-array base: converting a generic
// pointer per call costs a null check, 2 scalar instructions)
__device__ __forceinline__ void buf_lds16_at(__amdgpu_buffer_rsrc_t rs, unsigned lds_addr, unsigned voff) {
  const unsigned lds = __builtin_amdgcn_readfirstlane(lds_addr);
  asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, 0 offen lds" ::"s"(lds), "v"(voff),
               "s"(rs)
               : "memory");
}

// write-through (sc1) 16-byte stores / loads of the split-K partial tiles: the hand-off of
// MI355X_MICROARCH.md's table (sc1 stores, every storing wave's vmcnt(0), a barrier, one agent-scope
// atomic add per workgroup; the last adder reads with sc1 loads) -- no L2 write-back fence needed
__device__ __forceinline__ void store_wt16(__amdgpu_buffer_rsrc_t rs, unsigned off, f32x4 v) {
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), rs, off, 0, 16);
}
__device__ __forceinline__ f32x4 load_wt16(__amdgpu_buffer_rsrc_t rs, unsigned off) {
  return __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 16));
}

__device__ __forceinline__ void buf_lds16(__amdgpu_buffer_rsrc_t rs, char* lds_wave_base, unsigned voff) {
  // the low 32 bits of a generic address into the LDS aperture are the LDS address (the aperture base is the high
  // word): a truncation, where a cast to the LDS address space would add a null check per load
  const unsigned lds = __builtin_amdgcn_readfirstlane((unsigned)(size_t)lds_wave_base);
  asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, 0 offen lds" ::"s"(lds), "v"(voff),
               "s"(rs)
               : "memory");
}

constexpr int kMaxTaps = 49;  // 7x7 (the R3D stem as a 32-channel Conv2d); 3x3x3 Conv3d needs 27

template <int NTAPS>
struct NTPipeArgsT {
  unsigned act_bytes, w_bytes;
  int ntaps;              // taps in the K loop (<= NTAPS)
  int tap_w[NTAPS];       // weight tap index ((kt*R)+r)*S+s of each listed tap
  int tap_dt[NTAPS], tap_dy[NTAPS], tap_dx[NTAPS];  // source displacement of each tap relative to
                                                    // the row origin
  int cls;                // 1: rows are one parity class of a stride-2 dgrad output
  int ph, pw;             // that class
  int OHf, OWf;           // full output grid (class mode)
  // ncls > 1: the parity classes of a stride-2 dgrad in ONE launch.  Blocks [cls_start[k],
  // cls_start[k+1]) run class k; cls_meta[k] = ntaps | first tap << 4 | ph << 8 | pw << 9 (its taps
  // are tap_*[first tap ..]); class k's grid is ((OHf - ph + 1) / 2) x ((OWf - pw + 1) / 2) per sample.
  int ncls, batch;
  int cls_start[4], cls_meta[4];
  // row -> (n, oh, ow) divisors of the output grid (ncls > 1: per class k), set by launch_pipe_one: the
  // prologue's integer divisions were most of the short-K (1x1, strided) launches' instruction stream
  MagicDiv div_hw, div_ow, cdiv_hw[4], cdiv_ow[4];
};
typedef NTPipeArgsT<9> NTPipeArgs;          // Conv2d (3x3 and 1x1)
typedef NTPipeArgsT<kMaxTaps> NTPipeArgsV;  // Conv3d 3x3x3 and the folded 7x7 video stem

// the 2-D kernels take the 9-tap argument block (the larger one measured ~1.3 % slower on them)
inline NTPipeArgs narrow_args(const NTPipeArgsV& v) {
  NTPipeArgs a{};
  a.act_bytes = v.act_bytes;
  a.w_bytes = v.w_bytes;
  a.ntaps = v.ntaps;
  for (int t = 0; t < v.ntaps && t < 9; ++t) {
    a.tap_w[t] = v.tap_w[t];
    a.tap_dt[t] = v.tap_dt[t];
    a.tap_dy[t] = v.tap_dy[t];
    a.tap_dx[t] = v.tap_dx[t];
  }
  a.cls = v.cls;
  a.ph = v.ph;
  a.pw = v.pw;
  a.OHf = v.OHf;
  a.OWf = v.OWf;
  a.ncls = v.ncls;
  a.batch = v.batch;
  for (int k = 0; k < 4; ++k) {
    a.cls_start[k] = v.cls_start[k];
    a.cls_meta[k] = v.cls_meta[k];
    a.cdiv_hw[k] = v.cdiv_hw[k];
    a.cdiv_ow[k] = v.cdiv_ow[k];
  }
  a.div_hw = v.div_hw;
  a.div_ow = v.div_ow;
  return a;
}

// byte offset of 16-B chunk `chunk` of row `row` in a [rows][RB bytes] LDS image: the chunk is
// XOR-swizzled by the row so that the 32 rows of an MFMA fragment read hit distinct banks
template <int RB>
__device__ __forceinline__ int swz_rb(int row, int chunk) {
  if (RB == 64) return row * 64 + ((chunk ^ ((row >> 2) & 3)) << 4);
  return row * 128 + ((chunk ^ ((row >> 1) & 7)) << 4);
}

// 4 or 8 waves as WM x WN, each wave TM x TN tiles of 32x32: BM = WM*TM*32, BN = WN*TN*32; BK = k-tile
// depth (32 or 64 bf16: 64-B or whole 128-B lines per gathered row and tap).
// VID: rows carry a temporal coordinate and the tap list may exceed 32 taps (the Conv3d of the
// R3D-18 video trunk and its 49-tap stem); the Conv2d instances keep the 32-bit mask and 2-D row
// decode (measured: the general form costs the 2-D convs ~3.5 %).
// EPI: a dgrad with the BatchNorm-backward store epilogue (conv_epi.h; GemmNTParams::bx set).
template <int MODE, int WM, int WN, int TM, int TN, int NST, int BK = 32, bool VID = false, bool EPI = false>
__global__ __launch_bounds__(WM * WN * 64) void conv_nt_pipe_kernel(
    GemmNTParams p, typename std::conditional<VID, NTPipeArgsV, NTPipeArgs>::type ta) {
  typedef typename std::conditional<VID, unsigned long long, unsigned>::type mask_t;
  constexpr int NW = WM * WN, NT = NW * 64;  // waves, threads
  static_assert(NW == 4 || NW == 8, "4 or 8 waves");
  static_assert(BK == 32 || BK == 64, "BK");
  constexpr int BM = WM * TM * 32, BN = WN * TN * 32;
  constexpr int RB = BK * 2;                 // bytes per LDS row
  constexpr int CPR = RB / 16;               // 16-B chunks per row
  constexpr int RPI = 1024 / RB;             // rows per 1 KiB buffer-lds instruction
  constexpr int AR = BM / (NW * RPI), BR = BN / (NW * RPI);  // instructions per wave per tile
  static_assert(AR >= 1 && BR >= 1 && AR * NW * RPI == BM && BR * NW * RPI == BN, "tile/wave split");
  constexpr int LPT = AR + BR;
  constexpr int STAGE = (BM + BN) * RB;
  constexpr int CT_LD = BN + 8;
  constexpr int EPI_BYTES = BM * CT_LD * 2;
  constexpr int SMEM = (NST * STAGE > EPI_BYTES ? NST * STAGE : EPI_BYTES);
  __shared__ __attribute__((aligned(16))) char smem[SMEM + 2 * WM * BN * 4];
  float* red = reinterpret_cast<float*>(smem + SMEM);  // [2][WM][BN]

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid / WN, wn = wid % WN;
  const int nnt = p.Ng / BN;
  int bid, ntaps = ta.ntaps, tb = 0, cph = ta.ph, cpw = ta.pw;
  MagicDiv dhw = ta.div_hw, dow = ta.div_ow;
  if (!VID && MODE == MODE_DGRAD && ta.ncls > 1) {  // block-uniform: this block's parity class
    int k = 0;
#pragma unroll
    for (int j = 1; j < 4; ++j)
      if (j < ta.ncls && (int)blockIdx.x >= ta.cls_start[j]) k = j;
    const int meta = ta.cls_meta[k];
    ntaps = meta & 15;
    tb = (meta >> 4) & 15;
    cph = (meta >> 8) & 1;
    cpw = (meta >> 9) & 1;
    p.OH = (ta.OHf - cph + 1) >> 1;
    p.OW = (ta.OWf - cpw + 1) >> 1;
    p.M = ta.batch * p.OH * p.OW;
    dhw = ta.cdiv_hw[k];
    dow = ta.cdiv_ow[k];
    bid = (int)blockIdx.x - ta.cls_start[k];  // heavy classes first in dispatch order; no XCD remap
  } else {
    bid = xcd_remap(blockIdx.x, gridDim.x);
  }
  const int mt = bid / nnt, nt = bid - mt * nnt;
  const int m0 = mt * BM, n0 = nt * BN;

  const __amdgpu_buffer_rsrc_t rsa = __builtin_amdgcn_make_buffer_rsrc((void*)p.act, (short)0, (int)ta.act_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t rsb = __builtin_amdgcn_make_buffer_rsrc((void*)p.wmat, (short)0, (int)ta.w_bytes, 0x00020000);

  // ---- per-lane gather rows: instruction i of this wave covers rows (wid*AR + i)*RPI + lane/CPR ----
  const int lrow = lane / CPR, pchunk = lane % CPR;
  unsigned a_off0[AR];
  mask_t a_mask[AR];
  const int hw = p.OH * p.OW;
  const int thw = p.OT * hw;  // rows per sample: (t,) h, w  (OT = IT = 1 for Conv2d)
#pragma unroll
  for (int i = 0; i < AR; ++i) {
    const int row = (wid * AR + i) * RPI + lrow;
    const int lc = RB == 64 ? (pchunk ^ ((row >> 2) & 3)) : (pchunk ^ ((row >> 1) & 7));
    const int m = m0 + row;
    const bool ok = m < p.M;
    const int mm = ok ? m : 0;
    int n, ot, rem;
    if constexpr (VID) {
      n = mm / thw;
      const int rem0 = mm - n * thw;
      ot = rem0 / hw;  // temporal stride 1: the row origin's t is ot
      rem = rem0 - ot * hw;
    } else {
      n = (int)magic_div((unsigned)mm, dhw);
      ot = 0;
      rem = mm - n * hw;
    }
    const int oh = VID ? rem / p.OW : (int)magic_div((unsigned)rem, dow), ow = rem - oh * p.OW;
    int yb, xb;  // source coordinate of the row origin; tap t reads (yb + tap_dy[t], xb + tap_dx[t])
    if (MODE == MODE_FWD) {
      yb = oh * p.stride;
      xb = ow * p.stride;
    } else {
      yb = oh;  // class / stride-1 grids: displacements carry pad and parity
      xb = ow;
    }
    mask_t mask = 0;
    for (int t = 0; t < ntaps; ++t) {
      const int y = yb + ta.tap_dy[tb + t], x = xb + ta.tap_dx[tb + t];
      bool v = ok && y >= 0 && y < p.IH && x >= 0 && x < p.IW;
      if constexpr (VID) {
        const int tt = ot + ta.tap_dt[tb + t];
        v = v && tt >= 0 && tt < p.IT;
      }
      mask |= (v ? (mask_t)1 : (mask_t)0) << t;
    }
    a_mask[i] = mask;
    if constexpr (VID)
      a_off0[i] = (unsigned)(((((long long)n * p.IT + ot) * p.IH + yb) * p.IW + xb) * p.IC + lc * 8) * 2u;
    else  // 32-bit: the activation is < 2 GiB (act_bytes)
      a_off0[i] = (unsigned)(((n * p.IH + yb) * p.IW + xb) * p.IC + lc * 8) * 2u;
  }
  unsigned b_off[BR];
#pragma unroll
  for (int i = 0; i < BR; ++i) {
    const int row = (wid * BR + i) * RPI + lrow;
    const int lc = RB == 64 ? (pchunk ^ ((row >> 2) & 3)) : (pchunk ^ ((row >> 1) & 7));
    b_off[i] = (unsigned)(((size_t)(n0 + row) * p.Kg + lc * 8) * 2);
  }
  const int cpt = p.IC / BK;  // k-tiles per tap
  const int nkt = ntaps * cpt;

  // Tap table in VGPRs: lane t (< ntaps) holds tap t's activation and weight byte offsets; the
  // k loop reads them with v_readlane (no scalar-memory load, hence no lgkmcnt wait that would
  // also drain the LDS fragment reads, on the loop's critical path).
  int lane_tapoff = 0, lane_tapw = 0;
  if (lane < ntaps) {
    const int dt = VID ? ta.tap_dt[tb + lane] : 0;
    lane_tapoff = ((dt * p.IH + ta.tap_dy[tb + lane]) * p.IW + ta.tap_dx[tb + lane]) * p.IC * 2;
    lane_tapw = ta.tap_w[tb + lane] * p.IC * 2;
  }

  // incremental state of the next tile to issue (wave-uniform)
  int it_t = 0, it_c = 0, it_k = 0;
  auto issue = [&](int stage) {
    char* As = smem + stage * STAGE;
    char* Bs = As + BM * RB;
    const bool live = it_k < nkt;
    const int t = live ? it_t : 0;
    const int tapoff = __builtin_amdgcn_readlane(lane_tapoff, t) + it_c * 2;
    const unsigned boff = (unsigned)(__builtin_amdgcn_readlane(lane_tapw, t) + it_c * 2);  // Kg = R*S*IC
#pragma unroll
    for (int i = 0; i < AR; ++i) {
      const unsigned voff = a_off0[i] + (unsigned)tapoff;
      const bool valid = VID ? (a_mask[i] & (mask_t)1) != 0 : ((a_mask[i] >> t) & 1u) != 0;
      buf_lds16(rsa, As + (wid * AR + i) * 1024, (live && valid) ? voff : kOOB);
    }
#pragma unroll
    for (int i = 0; i < BR; ++i)
      buf_lds16(rsb, Bs + (wid * BR + i) * 1024, live ? b_off[i] + boff : kOOB);
    ++it_k;
    it_c += BK;
    if (it_c == p.IC) {
      it_c = 0;
      ++it_t;
      if constexpr (VID) {
#pragma unroll
        for (int i = 0; i < AR; ++i) a_mask[i] >>= 1;  // bit 0 = validity of the next tap
      }
    }
  };

  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int v = 0; v < 16; ++v) acc[i][j][v] = 0.f;

#pragma unroll
  for (int t = 0; t < NST - 1; ++t) issue(t);

  const int frow = lane & 31, fhalf = lane >> 5;
  constexpr int KS = BK / 16;
  bf16x8 af[2][TM], bfr[2][TN];  // fragments of k-step ks live in [ks & 1]
  auto load_frags = [&](const char* As, const char* Bs, int ks, int buf) {
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int row = wm * (BM / WM) + i * 32 + frow;
      af[buf][i] = *reinterpret_cast<const bf16x8*>(As + swz_rb<RB>(row, ks * 2 + fhalf));
    }
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int row = wn * (BN / WN) + j * 32 + frow;
      bfr[buf][j] = *reinterpret_cast<const bf16x8*>(Bs + swz_rb<RB>(row, ks * 2 + fhalf));
    }
  };
  for (int kt = 0; kt < nkt; ++kt) {
    wait_vmcnt<(NST - 2) * LPT>();  // tile kt has landed (NST-2 younger tiles may be in flight)
    ring_barrier();
    const char* As = smem + (kt % NST) * STAGE;
    const char* Bs = As + BM * RB;
    load_frags(As, Bs, 0, 0);
    issue((kt + NST - 1) % NST);  // the stage read in iteration kt-1; every wave has passed that
    // k-steps software-pipelined: the fragments of step ks+1 are read while step ks multiplies
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      if (ks + 1 < KS) {
        load_frags(As, Bs, ks + 1, (ks + 1) & 1);
        __builtin_amdgcn_sched_barrier(0);  // the next step's reads stay ahead of this step's MFMAs
      }
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[ks & 1][i], bfr[ks & 1][j], acc[i][j], 0, 0, 0);
      if (ks + 1 < KS) __builtin_amdgcn_sched_barrier(0);
    }
  }
  wait_vmcnt<0>();  // drain the dummy tail loads before the ring is reused
  __syncthreads();

  // ---- epilogue: BN partial statistics, then the bf16 tile through LDS ----
  const int rows_valid = min(BM, p.M - m0);
  if (MODE == MODE_FWD && p.stats != nullptr) {
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      float s = 0.f;
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int v = 0; v < 16; ++v) {
          const int r = wm * (BM / WM) + i * 32 + (v & 3) + 8 * (v >> 2) + 4 * fhalf;
          if (r < rows_valid) s += acc[i][j][v];
        }
      s += __shfl_xor(s, 32, 64);
      if (lane < 32) red[wm * BN + wn * (BN / WN) + j * 32 + lane] = s;
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int c = wn * (BN / WN) + j * 32 + frow;
      float tot = 0.f;
#pragma unroll
      for (int k = 0; k < WM; ++k) tot += red[k * BN + c];
      const float mean = tot / (float)rows_valid;
      float q = 0.f;
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int v = 0; v < 16; ++v) {
          const int r = wm * (BM / WM) + i * 32 + (v & 3) + 8 * (v >> 2) + 4 * fhalf;
          const float d = acc[i][j][v] - mean;
          if (r < rows_valid) q += d * d;
        }
      q += __shfl_xor(q, 32, 64);
      if (lane < 32) red[WM * BN + wm * BN + c] = q;
    }
    __syncthreads();
    // this row tile's own slot (avt_common.h): (M + BM - 1) / BM slots, plain stores
    bn_write_header(p.stats, (p.M + BM - 1) / BM, 0, mt == 0 && n0 == 0);
    double* acc_slot = bn_fwd_slots(p.stats) + (size_t)mt * p.Ng * 3;
    for (int c = tid; c < BN; c += NT) {
      double s = 0.0, m2 = 0.0;
#pragma unroll
      for (int k = 0; k < WM; ++k) {
        s += (double)red[k * BN + c];
        m2 += (double)red[WM * BN + k * BN + c];
      }
      double* a = acc_slot + (size_t)(n0 + c) * 3;
      a[0] = s;
      a[1] = m2;
      a[2] = s * s / (double)rows_valid;
    }
  }
  bf16_t* Ct = reinterpret_cast<bf16_t*>(smem);
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int v = 0; v < 16; ++v) {
        const int r = wm * (BM / WM) + i * 32 + (v & 3) + 8 * (v >> 2) + 4 * fhalf;
        const int c = wn * (BN / WN) + j * 32 + frow;
        Ct[r * CT_LD + c] = f2bf(acc[i][j][v]);
      }
  __syncthreads();
  // class mode: class row -> full output pixel (2h'+ph, 2w'+pw)
  auto orow = [&](int r) -> size_t {
    if (!ta.cls) return (size_t)(m0 + r);
    const int m = m0 + r;
    const int n = m / hw, rem = m - n * hw;
    const int oh = rem / p.OW, ow = rem - oh * p.OW;
    return ((size_t)n * ta.OHf + 2 * oh + cph) * ta.OWf + 2 * ow + cpw;
  };
  epi_store<NT, BM, BN, EPI>(p, Ct, CT_LD, n0, rows_valid, mt, (p.M + BM - 1) / BM, orow,
                             reinterpret_cast<float*>(smem));
}
