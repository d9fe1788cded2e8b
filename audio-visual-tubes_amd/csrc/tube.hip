// Layout kernels of the 3-D tube path (FullModel, model.py:17-36; R3D-18 = models/resnet3D.py).
//
//  * Video stem as a 2-D conv.  The R3D stem Conv3d(3, 64, (7,7,7), stride (1,2,2), pad (3,3,3))
//    (resnet3D.py:122-127) has temporal stride 1, so folding its 7 temporal taps into channels,
//      X'[n][t][h][w][kt*4 + c] = x[n][c][t + kt - 3][h][w]   (0 outside the clip, c = 3 and
//                                                              channels 28..31 zero),
//    turns it into a Conv2d 7x7/s2/p3 with 32 channels over the N*T frames, which runs on the
//    same LDS-DMA MFMA kernel as every other conv (C % 32 == 0).  The weight is packed to match:
//      W'[k][(r*7 + s)*32 + kt*4 + c] = w[k][c][kt][r][s].
//  * Conv3d weight packing: fp32 OIDHW (the Parameter layout) -> bf16 [K][(kt,r,s,c)], the fwd
//    operand of avt_conv3d_fwd.
#include "avt_common.h"

namespace avt {

// one thread per output pixel (n, t, h, w): 32 channels = 64 contiguous bytes
__global__ __launch_bounds__(256) void video_stem_im2col_kernel(const float* __restrict__ x, bf16_t* __restrict__ out,
                                                                int N, int C, int T, int HW, int KT, int pad_t) {
  const long long npix = (long long)N * T * HW;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < npix;
       i += (long long)gridDim.x * blockDim.x) {
    const int hw = (int)(i % HW);
    const long long nt = i / HW;
    const int t = (int)(nt % T), n = (int)(nt / T);
    float v[32];
#pragma unroll
    for (int j = 0; j < 32; ++j) v[j] = 0.f;
#pragma unroll
    for (int kt = 0; kt < 8; ++kt) {
      if (kt >= KT) break;
      const int tt = t + kt - pad_t;
      if (tt < 0 || tt >= T) continue;
#pragma unroll
      for (int c = 0; c < 4; ++c)
        if (c < C) v[kt * 4 + c] = x[(((long long)n * C + c) * T + tt) * HW + hw];
    }
    u32x4* o = reinterpret_cast<u32x4*>(out + i * 32);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      u32x4 w;
      w[0] = pack2(v[q * 8 + 0], v[q * 8 + 1]);
      w[1] = pack2(v[q * 8 + 2], v[q * 8 + 3]);
      w[2] = pack2(v[q * 8 + 4], v[q * 8 + 5]);
      w[3] = pack2(v[q * 8 + 6], v[q * 8 + 7]);
      o[q] = w;
    }
  }
}

// fold = 0: out[k][((kt*R + r)*S + s)*C + c] = w[k][c][kt][r][s]            (Kg = KT*R*S*C)
// fold = 1: out[k][(r*S + s)*32 + kt*4 + c] = w[k][c][kt][r][s], zero padded (Kg = R*S*32)
__global__ __launch_bounds__(256) void pack_conv3d_kernel(const float* __restrict__ w, bf16_t* __restrict__ out, int K,
                                                          int C, int KT, int R, int S, int fold, long long total) {
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    const int kg = fold ? R * S * 32 : KT * R * S * C;
    const int k = (int)(i / kg), j = (int)(i % kg);
    int kt, r, s, c;
    bool ok = true;
    if (fold) {
      const int rs = j / 32, q = j % 32;
      r = rs / S;
      s = rs % S;
      kt = q / 4;
      c = q % 4;
      ok = kt < KT && c < C;
    } else {
      c = j % C;
      const int t = j / C;
      s = t % S;
      r = (t / S) % R;
      kt = t / (S * R);
    }
    const float v = ok ? w[((((long long)k * C + c) * KT + kt) * R + r) * S + s] : 0.f;
    out[i] = f2bf(v);
  }
}

// fold = 0 with the filter row in LDS: out[k] is the (C x T) -> (T x C) transpose of w[k] (T = KT*R*S taps): one block
// per output row, the fp32 row read into LDS with 16-byte loads, the bf16 row written 8 channels (16 bytes) per
// thread (both sides coalesced; the element kernel above reads with a T-float stride).  C % 8 == 0.  Same values as
// pack_conv3d_kernel.
__global__ __launch_bounds__(256) void pack_conv3d_rows_kernel(const float* __restrict__ w, bf16_t* __restrict__ out,
                                                               int K, int C, int T) {
  extern __shared__ __attribute__((aligned(16))) float row[];  // C * T floats
  const int n = C * T;
  for (int k = blockIdx.x; k < K; k += gridDim.x) {
    const float4* src = reinterpret_cast<const float4*>(w + (size_t)k * n);
    __syncthreads();
    for (int i = threadIdx.x; i < n / 4; i += blockDim.x) reinterpret_cast<float4*>(row)[i] = src[i];
    __syncthreads();
    u32x4* dst = reinterpret_cast<u32x4*>(out + (size_t)k * n);
    for (int j = threadIdx.x; j < n / 8; j += blockDim.x) {  // output elements 8j .. 8j + 7: tap t, channels c .. c + 7
      const int t = (8 * j) / C, c = 8 * j - t * C;
      const float* r0 = row + c * T + t;
      u32x4 o;
      o.x = pack2(r0[0], r0[T]);
      o.y = pack2(r0[2 * T], r0[3 * T]);
      o.z = pack2(r0[4 * T], r0[5 * T]);
      o.w = pack2(r0[6 * T], r0[7 * T]);
      dst[j] = o;
    }
  }
}

// Every non-stem Conv3d weight of the R3D trunk in ONE launch (blockIdx.y = conv): the filter-row transpose above per
// descriptor, its element form for a descriptor the 16-byte path cannot take (C % 8 != 0 or misaligned operands).
struct Pack3dDesc {
  const float* w;  // fp32 OIDHW [K][C][T]
  bf16_t* out;     // bf16 [K][T*C]
  int K, C, T, pad_;
};

__global__ __launch_bounds__(256) void pack_conv3d_batched_kernel(const Pack3dDesc* __restrict__ descs) {
  extern __shared__ __attribute__((aligned(16))) float row[];
  const Pack3dDesc d = descs[blockIdx.y];
  const int n = d.C * d.T;
  const bool vec = d.C % 8 == 0 && ((((uintptr_t)d.w) | ((uintptr_t)d.out)) & 15) == 0;
  for (int k = blockIdx.x; k < d.K; k += gridDim.x) {
    const float* wk = d.w + (size_t)k * n;
    bf16_t* ok = d.out + (size_t)k * n;
    if (!vec) {
      for (int j = threadIdx.x; j < n; j += blockDim.x) {
        const int t = j / d.C, c = j - t * d.C;
        ok[j] = f2bf(wk[c * d.T + t]);
      }
      continue;
    }
    __syncthreads();
    for (int i = threadIdx.x; i < n / 4; i += blockDim.x)
      reinterpret_cast<float4*>(row)[i] = reinterpret_cast<const float4*>(wk)[i];
    __syncthreads();
    for (int j = threadIdx.x; j < n / 8; j += blockDim.x) {
      const int t = (8 * j) / d.C, c = 8 * j - t * d.C;
      const float* r0 = row + c * d.T + t;
      u32x4 o;
      o.x = pack2(r0[0], r0[d.T]);
      o.y = pack2(r0[2 * d.T], r0[3 * d.T]);
      o.z = pack2(r0[4 * d.T], r0[5 * d.T]);
      o.w = pack2(r0[6 * d.T], r0[7 * d.T]);
      reinterpret_cast<u32x4*>(ok)[j] = o;
    }
  }
}

// out[(b*rep + k)][c] = in[b][c]  (the per-clip audio vector of each of its t frames)
__global__ __launch_bounds__(256) void repeat_rows_kernel(const float* __restrict__ in, float* __restrict__ out, int B,
                                                          int rep, int C) {
  const long long n = (long long)B * rep * C;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
    const int c = (int)(i % C);
    const long long row = i / C;
    out[i] = in[(row / rep) * C + c];
  }
}

// out[b][c] = sum_k in[(b*rep + k)][c]  (adjoint of repeat_rows_kernel)
__global__ __launch_bounds__(256) void sum_rep_rows_kernel(const float* __restrict__ in, float* __restrict__ out, int B,
                                                           int rep, int C) {
  const long long n = (long long)B * C;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
    const int c = (int)(i % C);
    const long long b = i / C;
    float a = 0.f;
    for (int k = 0; k < rep; ++k) a += in[(b * rep + k) * C + c];
    out[i] = a;
  }
}

// MaxPool3d(kernel_size=3, stride=2, padding=1) (resnet3D.py:129, applied after the stem's BN + ReLU when
// no_max_pool=False, :200-201) over bf16 NDHWC [N][T][H][W][C] -> [N][To][Ho][Wo][C], To = (T - 1) / 2 + 1 (same
// for H, W).  One thread per output pixel and 8 channels (16 B loads of the 27 taps); taps outside the clip are
// skipped (torch's -inf padding); the result is the winning input's bits, and a NaN tap wins, as in max_pool3d.
__global__ __launch_bounds__(256) void maxpool3d_k3s2p1_kernel(const bf16_t* __restrict__ x, bf16_t* __restrict__ y,
                                                               int N, int T, int H, int W, int C, int To, int Ho,
                                                               int Wo) {
  const int cv = C / 8;
  const long long total = (long long)N * To * Ho * Wo * cv;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    const int c8 = (int)(i % cv);
    long long r = i / cv;
    const int wo = (int)(r % Wo);
    r /= Wo;
    const int ho = (int)(r % Ho);
    r /= Ho;
    const int to = (int)(r % To);
    const int n = (int)(r / To);
    float m[8];
    unsigned short bits[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      m[e] = -__builtin_inff();
      bits[e] = 0xff80;  // -inf (never stored: every window holds at least its centre tap)
    }
    for (int dt = 0; dt < 3; ++dt) {
      const int t = 2 * to - 1 + dt;
      if (t < 0 || t >= T) continue;
      for (int dh = 0; dh < 3; ++dh) {
        const int h = 2 * ho - 1 + dh;
        if (h < 0 || h >= H) continue;
        for (int dw = 0; dw < 3; ++dw) {
          const int w = 2 * wo - 1 + dw;
          if (w < 0 || w >= W) continue;
          const u32x4 v = reinterpret_cast<const u32x4*>(x)[(((long long)n * T + t) * H + h) * (long long)W * cv +
                                                           (long long)w * cv + c8];
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            const unsigned short b = (unsigned short)((e & 1) ? (v[e >> 1] >> 16) : (v[e >> 1] & 0xffff));
            const float f = bf2f(b);
            if (f > m[e] || f != f) {
              if (m[e] == m[e]) {  // a NaN already taken stays
                m[e] = f;
                bits[e] = b;
              }
            }
          }
        }
      }
    }
    u32x4 o;
#pragma unroll
    for (int q = 0; q < 4; ++q) o[q] = (unsigned)bits[2 * q] | ((unsigned)bits[2 * q + 1] << 16);
    reinterpret_cast<u32x4*>(y)[i] = o;
  }
}

static int grid_for(long long n) {
  long long g = (n + 255) / 256;
  if (g > 8192) g = 8192;
  return (int)(g < 1 ? 1 : g);
}

}  // namespace avt

using namespace avt;

// x: fp32 NCDHW [N][C][T][H][W] (the reference's frames.float(), train_3D.py:131), C <= 4,
// KT <= 7 -> out: bf16 [N][T][H][W][32] (see the file comment).
extern "C" int avt_video_stem_im2col(const float* x, void* out, int N, int C, int T, int H, int W, int KT, int pad_t,
                                     void* stream) {
  AVT_REQUIRE(x && out, "video_stem_im2col: null pointer");
  AVT_REQUIRE(C >= 1 && C <= 4 && KT >= 1 && KT <= 7, "video_stem_im2col: need C <= 4 and KT <= 7");
  const long long npix = (long long)N * T * H * W;
  if (npix == 0) return AVT_OK;
  hipLaunchKernelGGL(video_stem_im2col_kernel, dim3(grid_for(npix)), dim3(256), 0, (hipStream_t)stream, x,
                     (bf16_t*)out, N, C, T, H * W, KT, pad_t);
  return check_launch("video_stem_im2col");
}

// w: fp32 OIDHW [K][C][KT][R][S] -> out bf16 [K][Kg] (fold: stem layout, Kg = R*S*32)
extern "C" int avt_pack_conv3d_weight(const float* w, void* out, int K, int C, int KT, int R, int S, int fold,
                                      void* stream) {
  AVT_REQUIRE(w && out, "pack_conv3d_weight: null pointer");
  AVT_REQUIRE(!fold || (C <= 4 && KT <= 8), "pack_conv3d_weight: stem fold needs C <= 4, KT <= 8");
  const long long total = (long long)K * (fold ? R * S * 32 : KT * R * S * C);
  const int T = KT * R * S;
  const size_t row_bytes = (size_t)C * T * sizeof(float);
  if (!fold && C % 8 == 0 && row_bytes <= 60 * 1024 && ((((uintptr_t)out) | ((uintptr_t)w)) & 15) == 0) {
    hipLaunchKernelGGL(pack_conv3d_rows_kernel, dim3(K < 2048 ? K : 2048), dim3(256), row_bytes, (hipStream_t)stream, w,
                       (bf16_t*)out, K, C, T);
    return check_launch("pack_conv3d_weight");
  }
  hipLaunchKernelGGL(pack_conv3d_kernel, dim3(grid_for(total)), dim3(256), 0, (hipStream_t)stream, w, (bf16_t*)out, K,
                     C, KT, R, S, fold, total);
  return check_launch("pack_conv3d_weight");
}

// x bf16 [N][T][H][W][C] (C % 8 == 0) -> y bf16 [N][(T-1)/2+1][(H-1)/2+1][(W-1)/2+1][C]: nn.MaxPool3d(3, 2, 1)
extern "C" int avt_maxpool3d_fwd(const void* x, void* y, int N, int T, int H, int W, int C, void* stream) {
  AVT_REQUIRE(x && y, "maxpool3d_fwd: null pointer");
  AVT_REQUIRE(N >= 0 && T >= 1 && H >= 1 && W >= 1 && C >= 8 && C % 8 == 0,
              "maxpool3d_fwd: N=%d T=%d H=%d W=%d C=%d (C a multiple of 8)", N, T, H, W, C);
  const int To = (T - 1) / 2 + 1, Ho = (H - 1) / 2 + 1, Wo = (W - 1) / 2 + 1;
  const long long n = (long long)N * To * Ho * Wo * (C / 8);
  if (n == 0) return AVT_OK;
  hipLaunchKernelGGL(maxpool3d_k3s2p1_kernel, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream, (const bf16_t*)x,
                     (bf16_t*)y, N, T, H, W, C, To, Ho, Wo);
  return check_launch("maxpool3d_fwd");
}

extern "C" size_t avt_pack3d_desc_bytes(void) { return sizeof(Pack3dDesc); }

// descs: device array of n records {const float* w; void* out; int K, C, T, pad} (avt_pack3d_desc_bytes() each):
// out[k][t*C + c] = bf16(w[k][c][t]) for every record in one launch; max_k = the largest K, max_row = the largest
// C*T (floats; <= 15360: one fp32 filter row in LDS)
extern "C" int avt_pack_conv3d_weights_batched(const void* descs, int n, int max_k, int max_row, void* stream) {
  AVT_REQUIRE(descs && n > 0 && max_k > 0, "pack_conv3d_weights_batched: bad arguments");
  AVT_REQUIRE(max_row > 0 && max_row <= 15360, "pack_conv3d_weights_batched: max_row=%d (<= 15360 floats)", max_row);
  hipLaunchKernelGGL(pack_conv3d_batched_kernel, dim3(max_k < 512 ? max_k : 512, n), dim3(256),
                     (size_t)max_row * sizeof(float), (hipStream_t)stream, (const Pack3dDesc*)descs);
  return check_launch("pack_conv3d_weights_batched");
}

// Audio de-duplication of the tube step (train_3D.py:128-130 repeats each clip's spectrogram t
// times): the audio trunk runs once per clip; its unit vector is repeated to the (b t) rows of the
// head, and the head's gradient is summed back over the t rows (exact: everything between is linear
// in the upstream gradient for the shared forward).
extern "C" int avt_repeat_rows_f32(const float* in, float* out, int B, int rep, int C, void* stream) {
  AVT_REQUIRE(in && out && B >= 0 && rep >= 1 && C >= 1, "repeat_rows_f32: bad arguments");
  const long long n = (long long)B * rep * C;
  if (n == 0) return AVT_OK;
  hipLaunchKernelGGL(repeat_rows_kernel, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream, in, out, B, rep, C);
  return check_launch("repeat_rows_f32");
}

extern "C" int avt_sum_rep_rows_f32(const float* in, float* out, int B, int rep, int C, void* stream) {
  AVT_REQUIRE(in && out && B >= 0 && rep >= 1 && C >= 1, "sum_rep_rows_f32: bad arguments");
  const long long n = (long long)B * C;
  if (n == 0) return AVT_OK;
  hipLaunchKernelGGL(sum_rep_rows_kernel, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream, in, out, B, rep, C);
  return check_launch("sum_rep_rows_f32");
}
