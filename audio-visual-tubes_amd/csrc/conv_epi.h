// Store epilogue of the NT conv kernels (conv_nt_pipe_kernel, conv_halo_kernel): the bf16 result
// tile, staged in LDS as Ct [BM][CT_LD], goes out as 16-byte rows (+ the optional `add` tensor), and
// -- for a dgrad carrying a BatchNorm-backward epilogue (GemmNTParams::bx) -- is first masked by that
// BN's ReLU and reduced into its backward statistics, so the separate reduction pass over
// (g, y, xc) of the reference's BatchNorm2d backward (base_models.py:46-49, 58-67) is not needed:
//   g' = g * [y > 0]  or  g * [fma(xc, scale, shift) > 0]          (the mask the forward produced)
//   acc[slot][c] = (sum g', sum g' * (xc - mean) * invstd)         (slot = the block's row tile, plain stores)
// and g' is what gets stored (it is also the residual branch's gradient of an identity block).
// Included by conv_gemm.hip inside namespace avt.
#pragma once

// zero the bf16 elements of v whose bit in `bits` is clear
__device__ __forceinline__ u32x4 epi_mask8(u32x4 v, unsigned bits) {
  unsigned* u = reinterpret_cast<unsigned*>(&v);
#pragma unroll
  for (int e = 0; e < 4; ++e)
    u[e] &= ((bits >> (2 * e)) & 1u ? 0x0000ffffu : 0u) | ((bits >> (2 * e + 1)) & 1u ? 0xffff0000u : 0u);
  return v;
}

__device__ __forceinline__ void epi_unpack8(const u32x4& v, float* f) {
  const unsigned* u = reinterpret_cast<const unsigned*>(&v);
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    f[2 * e] = bf2f(u[e] & 0xffff);
    f[2 * e + 1] = bf2f(u[e] >> 16);
  }
}

// NT threads; OCPR = BN / 8 16-byte chunks per tile row.  orow(r) -> output row of tile row r.
// `scratch`: LDS of >= NW * BN * 3 floats that may overwrite Ct once every thread has read it.
// mt / nrow_tiles: the block's row tile and the launch's row tiles -- the slot the block's columns n0 .. n0+BN-1
// of the statistics go to (every column tile of a row tile writes its own columns of that one slot)
template <int NT, int BM, int BN, int UMAX, typename OrowFn>
__device__ __forceinline__ void epi_store_bn(const GemmNTParams& p, const bf16_t* Ct, int ct_ld, int n0, int rows_valid,
                                             int mt, int nrow_tiles, OrowFn orow, float* scratch) {
  constexpr int OCPR = BN / 8;
  static_assert(NT % OCPR == 0 && 64 % OCPR == 0, "a thread keeps one channel chunk");
  const int tid = threadIdx.x;
  const bool bnb = p.bx != nullptr;
  const bool two = p.bx2 != nullptr;
  const int cc = tid % OCPR;  // this thread's 8 channels: n0 + cc*8 ..
  const int c0 = n0 + cc * 8;
  float s1[8], s2[8], s3[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) s1[e] = s2[e] = s3[e] = 0.f;
  // U rows per thread at a time: every global load of the group is issued before any is used, so
  // the epilogue's HBM reads (add, xc, y) overlap instead of paying one latency per row.  Register
  // footprint kept near the main loop's (an 8-wave tile at 190 VGPRs would lose half its occupancy):
  // U = 4 (measured faster than 2), the Ct rows read when used, the per-channel BN constants re-read
  // from L1 per group.
  constexpr int ITERS = BM * OCPR / NT;
  static_assert(ITERS * NT == BM * OCPR, "rows per thread");
  constexpr int U = ITERS < UMAX ? ITERS : UMAX;
  const bool has_add = p.add != nullptr, has_y = p.by != nullptr;
  for (int it0 = 0; it0 < ITERS; it0 += U) {
    u32x4 aa[U], xx[U], yy[U], x2[U];
    size_t off[U];
    bool ok[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int r = (tid + (it0 + u) * NT) / OCPR;
      ok[u] = r < rows_valid;
      off[u] = ok[u] ? orow(r) * (size_t)p.Ng + c0 : 0;
      if (ok[u] && has_add) {
        aa[u] = *reinterpret_cast<const u32x4*>(p.add + off[u]);
        if (p.amask) aa[u] = epi_mask8(aa[u], p.amask[off[u] >> 3]);
      }
      if (ok[u] && bnb) {
        xx[u] = *reinterpret_cast<const u32x4*>(p.bx + off[u]);
        if (has_y) yy[u] = *reinterpret_cast<const u32x4*>(p.by + off[u]);
        if (two) x2[u] = *reinterpret_cast<const u32x4*>(p.bx2 + off[u]);
      }
    }
    const float* bst = p.bst;
    const float* bst2 = p.bst2;
    asm volatile("" : "+v"(bst), "+v"(bst2));  // not loop-invariant to the compiler: re-read, not hoisted
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (!ok[u]) continue;
      const int r = (tid + (it0 + u) * NT) / OCPR;
      u32x4 v = *reinterpret_cast<const u32x4*>(Ct + r * ct_ld + cc * 8);
      if (has_add) {
        unsigned* vp = reinterpret_cast<unsigned*>(&v);
        const unsigned* ap = reinterpret_cast<const unsigned*>(&aa[u]);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float lo = bf2f(vp[e] & 0xffff) + bf2f(ap[e] & 0xffff);
          const float hi = bf2f(vp[e] >> 16) + bf2f(ap[e] >> 16);
          vp[e] = pack2(lo, hi);
        }
      }
      if (bnb) {
        float g[8], xc[8];
        epi_unpack8(v, g);
        epi_unpack8(xx[u], xc);
        if (has_y) {
          float y[8];
          epi_unpack8(yy[u], y);
#pragma unroll
          for (int e = 0; e < 8; ++e) g[e] = y[e] > 0.f ? g[e] : 0.f;
        } else {
#pragma unroll
          for (int e = 0; e < 8; ++e)
            g[e] = __builtin_fmaf(xc[e], bst[c0 + e], bst[p.Ng + c0 + e]) > 0.f ? g[e] : 0.f;
        }
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          s1[e] += g[e];
          s2[e] += g[e] * ((xc[e] - bst[2 * p.Ng + c0 + e]) * bst[3 * p.Ng + c0 + e]);
        }
        if (two) {
          float xb[8];
          epi_unpack8(x2[u], xb);
#pragma unroll
          for (int e = 0; e < 8; ++e)
            s3[e] += g[e] * ((xb[e] - bst2[2 * p.Ng + c0 + e]) * bst2[3 * p.Ng + c0 + e]);
        }
        unsigned* vp = reinterpret_cast<unsigned*>(&v);  // g' is exactly representable: masked bf16 values
#pragma unroll
        for (int e = 0; e < 4; ++e) vp[e] = pack2(g[2 * e], g[2 * e + 1]);
      }
      *reinterpret_cast<u32x4*>(p.out + off[u]) = v;
    }
  }
  if (!bnb) return;
  // lanes of a wave that share a channel chunk differ in the lane bits >= log2(OCPR)
#pragma unroll
  for (int m = OCPR; m < 64; m <<= 1)
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      s1[e] += __shfl_xor(s1[e], m, 64);
      s2[e] += __shfl_xor(s2[e], m, 64);
      if (two) s3[e] += __shfl_xor(s3[e], m, 64);
    }
  constexpr int NW = NT / 64;
  const int lane = tid & 63, wid = tid >> 6;
  __syncthreads();  // every thread is done reading Ct: scratch may overwrite it
  if (lane < OCPR) {
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      float* q = scratch + ((size_t)wid * BN + cc * 8 + e) * 3;
      q[0] = s1[e];
      q[1] = s2[e];
      q[2] = s3[e];
    }
  }
  __syncthreads();
  // this row tile's slot (avt_common.h): the call's earlier launches' slots come first (bslot_base), and an
  // appending call (a stride-2 block's downsample dgrad) starts after the slots of the call before it
  const int total = p.bslot_total ? p.bslot_total : nrow_tiles;
  bn_write_header(p.bacc, total, p.bappend);
  if (two) bn_write_header(p.bacc2, total, p.bappend);
  const size_t slot = (size_t)(p.bslot_base + bn_slot_base(p.bacc, p.bappend) + mt);
  const size_t slot2 = two ? (size_t)(p.bslot_base + bn_slot_base(p.bacc2, p.bappend) + mt) : 0;
  for (int c = tid; c < BN; c += NT) {
    float a = 0.f, b = 0.f, d = 0.f;
#pragma unroll
    for (int w = 0; w < NW; ++w) {
      const float* q = scratch + ((size_t)w * BN + c) * 3;
      a += q[0];
      b += q[1];
      d += q[2];
    }
    double* acc = bn_bwd_slots(p.bacc, p.Ng) + (slot * p.Ng + n0 + c) * 2;
    acc[0] = (double)a;
    acc[1] = (double)b;
    if (two) {
      double* acc2 = bn_bwd_slots(p.bacc2, p.Ng) + (slot2 * p.Ng + n0 + c) * 2;
      acc2[0] = (double)a;
      acc2[1] = (double)d;
    }
  }
}

// EPI = false: the plain store (+ add) -- the forward and plain-dgrad instantiations keep the register
// footprint of their main loop (the BN epilogue's load groups would raise it and cost occupancy).
template <int NT, int BM, int BN, bool EPI, typename OrowFn, int UMAX = 4>
__device__ __forceinline__ void epi_store(const GemmNTParams& p, const bf16_t* Ct, int ct_ld, int n0, int rows_valid,
                                          int mt, int nrow_tiles, OrowFn orow, float* scratch) {
  if constexpr (!EPI) {
    constexpr int OCPR = BN / 8;
    for (int idx = threadIdx.x; idx < BM * OCPR; idx += NT) {
      const int r = idx / OCPR, cc = idx - r * OCPR;
      if (r >= rows_valid) continue;
      u32x4 v = *reinterpret_cast<const u32x4*>(Ct + r * ct_ld + cc * 8);
      const size_t off = orow(r) * (size_t)p.Ng + n0 + cc * 8;
      if (p.add != nullptr) {
        u32x4 a = *reinterpret_cast<const u32x4*>(p.add + off);
        if (p.amask != nullptr) a = epi_mask8(a, p.amask[off >> 3]);
        unsigned* vv = reinterpret_cast<unsigned*>(&v);
        const unsigned* aa = reinterpret_cast<const unsigned*>(&a);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float lo = bf2f(vv[e] & 0xffff) + bf2f(aa[e] & 0xffff);
          const float hi = bf2f(vv[e] >> 16) + bf2f(aa[e] >> 16);
          vv[e] = pack2(lo, hi);
        }
      }
      *reinterpret_cast<u32x4*>(p.out + off) = v;
    }
    return;
  } else {
    epi_store_bn<NT, BM, BN, UMAX>(p, Ct, ct_ld, n0, rows_valid, mt, nrow_tiles, orow, scratch);
  }
}
