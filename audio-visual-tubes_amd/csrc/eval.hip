// Localisation metrics of the reference's test loops, batched on the device: one block per heatmap.
//
// Restates, per map (train_hardway_1frame.py:195-206 / train_hardway.py:152-163, test.py:97-130):
//   heatmap_now = cv2.resize(A[i,0], (S, S), INTER_LINEAR)        (fp32, half-pixel centres, edge clamp)
//   heatmap_now = normalize_img(-heatmap_now)                       (utils.py:234-239, min/max of the map)
//   pred = 1 - heatmap_now;  thr = sort(pred)[S*S/2]
//   pred[pred > thr] = 1;  pred[pred < 1] = 0
//   cIoU = sum(infer*gt) / (sum(gt) + sum(infer*(gt==0))),  infer = pred >= 0.5   (utils.py:209-214)
// and utils.mTC's consecutive-frame cIoU of the binarised maps (utils.py:311-318).
//
// Arithmetic: the resize takes cv2's INTER_LINEAR coefficients (fx = (x+0.5)*h/S - 0.5, floor, clamp
// to the edge with zero weight) and evaluates (S0*a0 + S1*a1) horizontally then vertically with
// separately rounded fp32 products and sums (no FMA contraction), so the oracle's numpy float32
// restatement reproduces it bit for bit; the median is an exact radix select over the order-
// preserving integer image of the fp32 pred values (4 passes of 8 bits, the map recomputed per
// pass: 50176 values do not fit in LDS); the cIoU sums are fp64 like numpy's.
#include "avt_common.h"

namespace avt {

constexpr int EV_T = 1024;
constexpr int EV_SMAX = 512;

__device__ __forceinline__ unsigned order_key(float f) {
  const unsigned u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}

struct EvalTabs {
  int sy[EV_SMAX], sx[EV_SMAX];
  float ay0[EV_SMAX], ay1[EV_SMAX], ax0[EV_SMAX], ax1[EV_SMAX];
};

// cv2 resize (INTER_LINEAR) source index / weights of destination coordinate d
__device__ __forceinline__ void lin_coef(int d, int src, int dst, int& s, float& a0, float& a1) {
  // cv2: fx = (float)((dx + 0.5) * scale_x - 0.5) with scale_x = (double)src / dst
  float f = (float)(((double)d + 0.5) * ((double)src / (double)dst) - 0.5);
  int i = (int)floorf(f);
  f = __fsub_rn(f, (float)i);
  if (i < 0) {
    f = 0.f;
    i = 0;
  }
  if (i >= src - 1) {
    f = 0.f;
    i = src - 1;
  }
  s = i;
  a0 = __fsub_rn(1.f, f);
  a1 = f;
}

__device__ __forceinline__ float resized(const float* __restrict__ m, int h, int w, const EvalTabs& tb, int y, int x) {
  const int sy = tb.sy[y], sx = tb.sx[x];
  const int sy1 = min(sy + 1, h - 1), sx1 = min(sx + 1, w - 1);
  const float r0 = __fadd_rn(__fmul_rn(m[sy * w + sx], tb.ax0[x]), __fmul_rn(m[sy * w + sx1], tb.ax1[x]));
  const float r1 = __fadd_rn(__fmul_rn(m[sy1 * w + sx], tb.ax0[x]), __fmul_rn(m[sy1 * w + sx1], tb.ax1[x]));
  return __fadd_rn(__fmul_rn(r0, tb.ay0[y]), __fmul_rn(r1, tb.ay1[y]));
}

// pred value of pixel (y, x) given the map's min/max (normalize_img of -heatmap, then 1 - .)
__device__ __forceinline__ float pred_at(const float* m, int h, int w, const EvalTabs& tb, int y, int x, float vmin,
                                         float vmax) {
  const float nh = -resized(m, h, w, tb, y, x);
  const float rng = __fsub_rn(vmax, vmin);
  const float v = rng != 0.f ? __fdiv_rn(__fsub_rn(nh, vmin), rng) : nh;
  return __fsub_rn(1.f, v);
}

__global__ __launch_bounds__(EV_T) void localize_ciou_kernel(const float* __restrict__ A, int h, int w, int S,
                                                             const float* __restrict__ gt, double* __restrict__ out,
                                                             unsigned char* __restrict__ pred_out) {
  __shared__ EvalTabs tb;
  __shared__ unsigned hist[256];
  __shared__ float fred[2][EV_T / 64];
  __shared__ double dred[3][EV_T / 64];
  __shared__ unsigned sel[2];  // prefix found so far, remaining rank
  const int img = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const float* m = A + (size_t)img * h * w;
  const int n = S * S;
  for (int d = tid; d < S; d += EV_T) {
    lin_coef(d, h, S, tb.sy[d], tb.ay0[d], tb.ay1[d]);
    lin_coef(d, w, S, tb.sx[d], tb.ax0[d], tb.ax1[d]);
  }
  __syncthreads();
  // min / max of -heatmap_now
  float mn = INFINITY, mx = -INFINITY;
  for (int i = tid; i < n; i += EV_T) {
    const float v = -resized(m, h, w, tb, i / S, i % S);
    mn = fminf(mn, v);
    mx = fmaxf(mx, v);
  }
  for (int o = 32; o >= 1; o >>= 1) {
    mn = fminf(mn, __shfl_xor(mn, o, 64));
    mx = fmaxf(mx, __shfl_xor(mx, o, 64));
  }
  if (lane == 0) {
    fred[0][wv] = mn;
    fred[1][wv] = mx;
  }
  if (tid == 0) {
    sel[0] = 0u;
    sel[1] = (unsigned)(n / 2);  // 0-based rank of the threshold: sort(pred)[S*S/2]
  }
  __syncthreads();
  float vmin = fred[0][0], vmax = fred[1][0];
  for (int k = 1; k < EV_T / 64; ++k) {
    vmin = fminf(vmin, fred[0][k]);
    vmax = fmaxf(vmax, fred[1][k]);
  }
  // radix select, most significant byte first
  for (int pass = 0; pass < 4; ++pass) {
    const int shift = 24 - 8 * pass;
    for (int b = tid; b < 256; b += EV_T) hist[b] = 0u;
    __syncthreads();
    const unsigned prefix = sel[0];
    const unsigned pmask = pass == 0 ? 0u : (0xFFFFFFFFu << (32 - 8 * pass));
    for (int i = tid; i < n; i += EV_T) {
      const unsigned key = order_key(pred_at(m, h, w, tb, i / S, i % S, vmin, vmax));
      if ((key & pmask) == prefix) atomicAdd(&hist[(key >> shift) & 255u], 1u);
    }
    __syncthreads();
    if (tid == 0) {
      unsigned rank = sel[1], b = 0;
      while (hist[b] <= rank) {
        rank -= hist[b];
        ++b;
      }
      sel[0] = prefix | (b << shift);
      sel[1] = rank;
    }
    __syncthreads();
  }
  const unsigned thr_key = sel[0];
  // binarise (pred > thr -> 1, then pred < 1 -> 0) and the cIoU sums against gt
  const float* g = gt ? gt + (size_t)img * n : nullptr;
  double s_ig = 0.0, s_g = 0.0, s_i0 = 0.0;
  for (int i = tid; i < n; i += EV_T) {
    const float p = pred_at(m, h, w, tb, i / S, i % S, vmin, vmax);
    const float q = order_key(p) > thr_key ? 1.f : p;
    const float b = q < 1.f ? 0.f : q;
    const double inf = b >= 0.5f ? 1.0 : 0.0;
    if (pred_out) pred_out[(size_t)img * n + i] = (unsigned char)(inf != 0.0);
    if (g) {
      const double gv = (double)g[i];
      s_ig += inf * gv;
      s_g += gv;
      s_i0 += inf * (gv == 0.0 ? 1.0 : 0.0);
    }
  }
  for (int o = 32; o >= 1; o >>= 1) {
    s_ig += __shfl_xor(s_ig, o, 64);
    s_g += __shfl_xor(s_g, o, 64);
    s_i0 += __shfl_xor(s_i0, o, 64);
  }
  if (lane == 0) {
    dred[0][wv] = s_ig;
    dred[1][wv] = s_g;
    dred[2][wv] = s_i0;
  }
  __syncthreads();
  if (tid == 0 && g) {
    double a = 0.0, b = 0.0, c = 0.0;
    for (int k = 0; k < EV_T / 64; ++k) {
      a += dred[0][k];
      b += dred[1][k];
      c += dred[2][k];
    }
    out[img * 3 + 0] = a / (b + c);
    out[img * 3 + 1] = a;
    out[img * 3 + 2] = b + c;
  }
}

// cal_CIOU(p[i], p[i+1], 0.5) of binary maps (utils.mTC): one block per pair
__global__ __launch_bounds__(EV_T) void pair_ciou_kernel(const unsigned char* __restrict__ p, int n,
                                                         double* __restrict__ out) {
  __shared__ double dred[3][EV_T / 64];
  const int k = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const unsigned char* a = p + (size_t)k * n;
  const unsigned char* b = a + n;
  double s_ig = 0.0, s_g = 0.0, s_i0 = 0.0;
  for (int i = tid; i < n; i += EV_T) {
    const double inf = a[i] ? 1.0 : 0.0, gv = b[i] ? 1.0 : 0.0;
    s_ig += inf * gv;
    s_g += gv;
    s_i0 += inf * (gv == 0.0 ? 1.0 : 0.0);
  }
  for (int o = 32; o >= 1; o >>= 1) {
    s_ig += __shfl_xor(s_ig, o, 64);
    s_g += __shfl_xor(s_g, o, 64);
    s_i0 += __shfl_xor(s_i0, o, 64);
  }
  if (lane == 0) {
    dred[0][wv] = s_ig;
    dred[1][wv] = s_g;
    dred[2][wv] = s_i0;
  }
  __syncthreads();
  if (tid == 0) {
    double x = 0.0, y = 0.0, z = 0.0;
    for (int j = 0; j < EV_T / 64; ++j) {
      x += dred[0][j];
      y += dred[1][j];
      z += dred[2][j];
    }
    out[k] = x / (y + z);
  }
}

}  // namespace avt

using namespace avt;

// A [N][h][w] fp32 heatmaps (AVENet's A), gt [N][S][S] fp32 ground-truth maps (or NULL), out [N][3]
// fp64 = (cIoU, intersection, denominator) (utils.Evaluator.cal_CIOU(pred, gt, 0.5) with the test
// loops' median binarisation), pred_out [N][S][S] u8 binary maps (or NULL).
extern "C" int avt_localize_ciou(const float* A, int N, int h, int w, int S, const float* gt, double* out,
                                 void* pred_out, void* stream) {
  AVT_REQUIRE(A && (gt == nullptr || out != nullptr), "localize_ciou: null pointer");
  AVT_REQUIRE(N >= 1 && h >= 1 && w >= 1 && S >= 2 && S <= EV_SMAX, "localize_ciou: bad shape N=%d h=%d w=%d S=%d",
              N, h, w, S);
  hipLaunchKernelGGL(localize_ciou_kernel, dim3(N), dim3(EV_T), 0, (hipStream_t)stream, A, h, w, S, gt, out,
                     (unsigned char*)pred_out);
  return check_launch("localize_ciou");
}

// out[k] = cal_CIOU(p[k], p[k+1], 0.5) for k < N-1 over binary maps p [N][n] u8 (utils.mTC).
extern "C" int avt_pair_ciou(const void* p, int N, int n, double* out, void* stream) {
  AVT_REQUIRE(p && out && N >= 2 && n >= 1, "pair_ciou: need N >= 2 maps");
  hipLaunchKernelGGL(pair_ciou_kernel, dim3(N - 1), dim3(EV_T), 0, (hipStream_t)stream, (const unsigned char*)p, n,
                     out);
  return check_launch("pair_ciou");
}
