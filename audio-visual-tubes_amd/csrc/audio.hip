// Log-spectrogram of the reference's audio pipeline on the device (datasets/dataloader.py:86-96,
// 252-274):
//   resamples = clip(samples[:sr*10], -1, 1)
//   f, t, S = scipy.signal.spectrogram(resamples, sr, nperseg=512, noverlap=1)
//   spec = Normalize(0, 12)(ToTensor(log(S + 1e-7)))                      -> [1, 257, nseg]
// scipy's defaults: periodic Tukey(0.25) window, detrend='constant' (per-segment mean removed
// before windowing), one-sided PSD with scaling='density' (|X|^2 / (fs * sum w^2), bins 1..255
// doubled), segments of 512 samples every 511, no padding: nseg = (N - 512) / 511 + 1.
//
// One 256-thread block per (clip, run of SPB segments): the window, its energy and the 256 twiddles
// e^{-2 pi i q / 512} are built once per block (double precision, rounded to fp32); each segment is
// loaded (coalesced), clipped, de-meaned (fp64 block sum), windowed, and transformed by a radix-2
// Stockham FFT in LDS (9 stages, ping-pong float2 buffers); the 257 powers go to log(P + 1e-7)/12.
// HBM-bound: 4 B read per sample + 4 B written per (bin, segment); the FFT is ~14 kFLOP a segment.
#include "avt_common.h"

namespace avt {

constexpr int SG_N = 512;       // nperseg == nfft
constexpr int SG_BINS = SG_N / 2 + 1;
constexpr int SG_T = 256;
constexpr int SG_SPB = 8;       // segments per block

__device__ __forceinline__ float2 cmul(float2 a, float2 b) {
  return make_float2(a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x);
}

__global__ __launch_bounds__(SG_T) void spectrogram_kernel(const float* __restrict__ x, long long N, int nseg, int hop,
                                                           float fs, float* __restrict__ out) {
  __shared__ float2 buf[2][SG_N];
  __shared__ float2 tw[SG_N / 2];
  __shared__ float win[SG_N];
  __shared__ double dred[SG_T / 64];
  __shared__ float scale_s;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int clip = blockIdx.y;
  const int seg0 = blockIdx.x * SG_SPB;
  const double PI = 3.141592653589793238462643383279502884;
  // periodic Tukey(alpha = 0.25) of length 512 = the symmetric one of length 513, last point dropped
  const int M = SG_N + 1;
  const double alpha = 0.25;
  const int width = (int)floor(alpha * (M - 1) / 2.0);
  double e2 = 0.0;
  for (int i = tid; i < SG_N; i += SG_T) {
    double w = 1.0;
    if (i <= width)
      w = 0.5 * (1.0 + cos(PI * (-1.0 + 2.0 * i / alpha / (M - 1))));
    else if (i >= M - width - 1)
      w = 0.5 * (1.0 + cos(PI * (-2.0 / alpha + 1.0 + 2.0 * i / alpha / (M - 1))));
    win[i] = (float)w;
    e2 += w * w;
  }
  for (int q = tid; q < SG_N / 2; q += SG_T) {
    double s, c;
    sincospi(-2.0 * q / SG_N, &s, &c);
    tw[q] = make_float2((float)c, (float)s);
  }
  for (int o = 32; o >= 1; o >>= 1) e2 += __shfl_xor(e2, o, 64);
  if (lane == 0) dred[wv] = e2;
  __syncthreads();
  if (tid == 0) {
    double t = 0.0;
    for (int k = 0; k < SG_T / 64; ++k) t += dred[k];
    scale_s = (float)(1.0 / ((double)fs * t));  // scaling='density'
  }
  __syncthreads();
  const float scale = scale_s;
  const float* xc = x + (size_t)clip * N;
  for (int s = seg0; s < min(seg0 + SG_SPB, nseg); ++s) {
    const float* seg = xc + (size_t)s * hop;
    float v[2];
    double sum = 0.0;
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      v[r] = fminf(fmaxf(seg[tid + r * SG_T], -1.f), 1.f);  // dataloader.py:92-93
      sum += (double)v[r];
    }
    for (int o = 32; o >= 1; o >>= 1) sum += __shfl_xor(sum, o, 64);
    __syncthreads();  // the previous segment's readers of dred / buf are done
    if (lane == 0) dred[wv] = sum;
    __syncthreads();
    double tot = 0.0;
    for (int k = 0; k < SG_T / 64; ++k) tot += dred[k];
    const float mean = (float)(tot / SG_N);  // detrend='constant'
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      const int i = tid + r * SG_T;
      buf[0][i] = make_float2((v[r] - mean) * win[i], 0.f);
    }
    __syncthreads();
    // Stockham radix-2: Ns = 1, 2, ..., 256; thread j: butterfly (j, j + 256)
    int src = 0;
    for (int Ns = 1; Ns < SG_N; Ns <<= 1) {
      const int j = tid, k = j & (Ns - 1);
      float2 a = buf[src][j], b = buf[src][j + SG_N / 2];
      b = cmul(b, tw[k * (SG_N / 2 / Ns)]);
      const int d = ((j - k) << 1) + k;  // (j / Ns) * 2 Ns + j % Ns
      buf[src ^ 1][d] = make_float2(a.x + b.x, a.y + b.y);
      buf[src ^ 1][d + Ns] = make_float2(a.x - b.x, a.y - b.y);
      src ^= 1;
      __syncthreads();
    }
    float* o = out + (size_t)clip * SG_BINS * nseg + s;
    for (int kb = tid; kb < SG_BINS; kb += SG_T) {
      const float2 X = buf[src][kb];
      float p = (X.x * X.x + X.y * X.y) * scale;
      if (kb != 0 && kb != SG_N / 2) p *= 2.f;  // one-sided
      o[(size_t)kb * nseg] = logf(p + 1e-7f) / 12.f;
    }
  }
}

}  // namespace avt

using namespace avt;

extern "C" int avt_spectrogram_segments(long long n_samples, int hop) {
  if (n_samples < SG_N || hop < 1) return 0;
  return (int)((n_samples - SG_N) / hop + 1);
}

// x [B][N] fp32 waveforms -> out [B][1][257][nseg] fp32 normalised log-spectrograms
// (nseg = avt_spectrogram_segments(N, hop)); nperseg = nfft = 512, hop = nperseg - noverlap (511).
extern "C" int avt_spectrogram(const float* x, int B, long long N, int hop, float fs, float* out, void* stream) {
  AVT_REQUIRE(x && out, "spectrogram: null pointer");
  const int nseg = avt_spectrogram_segments(N, hop);
  AVT_REQUIRE(B >= 1 && nseg >= 1 && fs > 0.f, "spectrogram: need B >= 1, N >= 512 samples, fs > 0");
  dim3 grid((nseg + SG_SPB - 1) / SG_SPB, B);
  hipLaunchKernelGGL(spectrogram_kernel, grid, dim3(SG_T), 0, (hipStream_t)stream, x, N, nseg, hop, fs, out);
  return check_launch("spectrogram");
}
