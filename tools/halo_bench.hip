// (The DPP A-fragment shift variant measured in profiles/r5_halo_bench_shift.txt is in commit ee93575.)
// Standalone A/B bench of conv_halo_kernel variants (audio-visual-tubes_amd/csrc/conv_halo.h), built outside
// libavt so a variant compiles in seconds: per trunk shape and mode, the variants run on the same inputs, their
// outputs and BN slots are compared bit for bit with the first (baseline) variant, and each is timed with HIP
// events over alternating rounds of back-to-back launches (random data: the clock depends on the operands).
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -Iinclude -Iaudio-visual-tubes_amd/csrc -Itools tools/halo_bench.hip
//        -o tools/halo_bench        run: tools/halo_bench [B] [rounds] [launches]
#include "avt_common.h"

#include <vector>
#include <string>

namespace avt {
#include "conv_params.h"
#include "conv_epi.h"
#include "conv_nt_pipe.h"
#include "conv_halo.h"
#include "halo_pk.h"
void set_error(const char* fmt, ...) { (void)fmt; }
int check_launch(const char*) { return hipGetLastError() == hipSuccess ? AVT_OK : AVT_EHIP; }
}  // namespace avt
using namespace avt;

#define HIPCHECK(x)                                                                  \
  do {                                                                               \
    hipError_t e_ = (x);                                                             \
    if (e_ != hipSuccess) {                                                          \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(1);                                                                       \
    }                                                                                \
  } while (0)

__global__ void fill_bf16(bf16_t* p, size_t n, unsigned seed, float scale, int relu) {
  for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) {
    unsigned h = (unsigned)i * 2654435761u ^ seed;
    h ^= h >> 15; h *= 0x2c1b3c6du; h ^= h >> 12; h *= 0x297a2d39u; h ^= h >> 15;
    float v = ((h & 0xffffff) / 16777216.0f - 0.5f) * 2.f * scale;
    if (relu && v < 0.f) v = 0.f;
    p[i] = f2bf(v);
  }
}

struct Shape {
  const char* name;
  int N, H, W, C, K;
};

typedef void (*Launcher)(const GemmNTParams&, const HaloArgs&, int, hipStream_t);

template <int MODE, int WM, int WN, int TM, int TN, int NSTB, int PRMAX, int PREF, int OPT = 0>
void launch_v(const GemmNTParams& p, const HaloArgs& ha, int grid, hipStream_t st) {
  hipLaunchKernelGGL((conv_halo_kernel<MODE, WM, WN, TM, TN, NSTB, PRMAX, false, false, PREF, OPT>), dim3(grid),
                     dim3(WM * WN * 64), 0, st, p, ha);
}

template <int MODE, int WM, int WN, int TM, int TN, int NSTB, int PRMAX, int PK, int DBG = 0>
void launch_pk(const GemmNTParams& p, const HaloArgs& ha0, int grid, hipStream_t st) {
  HaloPkArgs ha;
  static_cast<HaloArgs&>(ha) = ha0;
  ha.div_hw = make_magic((unsigned)(ha0.W * ha0.H));
  ha.div_w = make_magic((unsigned)ha0.W);
  ha.pk = PK;
  static int ncu = 0;
  if (!ncu) {
    hipDeviceProp_t pr;
    (void)hipGetDeviceProperties(&pr, 0);
    ncu = getenv("HB_G") ? atoi(getenv("HB_G")) : pr.multiProcessorCount;
    fprintf(stderr, "multiProcessorCount %d, G %d\n", pr.multiProcessorCount, ncu);
  }
  int G = ncu;  // one block per CU
  if (PK == 1 && grid < G) G = grid;
  hipLaunchKernelGGL((conv_halo_pk_kernel<MODE, WM, WN, TM, TN, NSTB, PRMAX, PK, DBG>), dim3(G), dim3(WM * WN * 64), 0, st, p, ha);
}

struct Variant {
  std::string name;
  Launcher fn[2];  // fwd, dgrad
  int BM, BN, PRMAX;
  int pk;          // stream-K: needs >= nc units per block
  bool tps2;       // two taps per step: an even number of 64-channel chunks
};

template <int WM, int WN, int TM, int TN, int NSTB, int PRMAX, int PREF, int OPT = 0>
Variant make(const char* name) {
  return Variant{name,
                 {launch_v<MODE_FWD, WM, WN, TM, TN, NSTB, PRMAX, PREF, OPT>,
                  launch_v<MODE_DGRAD, WM, WN, TM, TN, NSTB, PRMAX, PREF, OPT>},
                 WM * TM * 32, WN * TN * 32, PRMAX, 0, (OPT & 2) != 0};
}
template <int WM, int WN, int TM, int TN, int NSTB, int PRMAX, int PK, int DBG = 0>
Variant make_pk(const char* name) {
  return Variant{name,
                 {launch_pk<MODE_FWD, WM, WN, TM, TN, NSTB, PRMAX, PK, DBG>, launch_pk<MODE_DGRAD, WM, WN, TM, TN, NSTB, PRMAX, PK, DBG>},
                 WM * TM * 32, WN * TN * 32, PRMAX, PK, false};
}

int main(int argc, char** argv) {
  const int B = argc > 1 ? atoi(argv[1]) : 128;
  const int rounds = argc > 2 ? atoi(argv[2]) : 3;
  const int launches = argc > 3 ? atoi(argv[3]) : 20;
  // the shapes the 8-wave 256 x 128 tile runs in the step (conv_gemm.hip launch_nt: W <= 39, K % 128 == 0)
  std::vector<Shape> shapes = {{"V.l2", B, 28, 28, 128, 128},  {"V.l3", B, 14, 14, 256, 256},
                               {"V.l4", B, 14, 14, 512, 512},  {"A.l2", B, 33, 38, 128, 128},
                               {"A.l4", B, 17, 19, 512, 512}};
  if (argc > 4 && !strcmp(argv[4], "sweep0"))  // fwd-only sweep shapes (dgrad = same GEMM: C = K)
    shapes = {{"s128x1", 256, 16, 16, 128, 128}, {"s512x1", 256, 16, 16, 512, 512}, {"s128x2", 512, 16, 16, 128, 128},
              {"s512x2", 512, 16, 16, 512, 512}};
  if (argc > 4 && !strcmp(argv[4], "sweep"))  // one / two rounds of 256 tiles (16 x 16 images), K = 18 / 36 / 72 steps
    shapes = {{"s128x1", 256, 16, 16, 128, 128}, {"s256x1", 256, 16, 16, 256, 128}, {"s512x1", 256, 16, 16, 512, 128},
              {"s128x2", 512, 16, 16, 128, 128}, {"s256x2", 512, 16, 16, 256, 128}, {"s512x2", 512, 16, 16, 512, 128}};
  std::vector<Variant> vars = {make<4, 2, 2, 2, 3, 336, 0>("base"), make<4, 2, 2, 2, 3, 336, 0, 1>("prio"),
                               make<4, 2, 2, 2, 2, 336, 0, 2>("tps2"), make<4, 2, 2, 2, 2, 336, 0, 3>("tps2p")};
  hipStream_t st;
  HIPCHECK(hipStreamCreate(&st));
  hipEvent_t e0, e1;
  HIPCHECK(hipEventCreate(&e0));
  HIPCHECK(hipEventCreate(&e1));
  int bad = 0;
  float* part;
  int* cnt;
  HIPCHECK(hipMalloc(&part, (size_t)256 * 256 * 128 * 4));
  HIPCHECK(hipMalloc(&cnt, 256 * 4));
  HIPCHECK(hipMemset(cnt, 0, 256 * 4));
  for (const Shape& s : shapes) {
    for (int mode = 0; mode < 2; ++mode) {
      const int IC = mode == 0 ? s.C : s.K, Ng = mode == 0 ? s.K : s.C;
      const long long M = (long long)s.N * s.H * s.W;
      const size_t act_n = (size_t)M * IC, w_n = (size_t)Ng * 9 * IC, out_n = (size_t)M * Ng;
      bf16_t *act, *w, *out;
      double* stats;
      const size_t stats_n = kBnHdr + bn_slot_cap(M) * Ng * 3;
      HIPCHECK(hipMalloc(&act, act_n * 2));
      HIPCHECK(hipMalloc(&w, w_n * 2));
      HIPCHECK(hipMalloc(&out, out_n * 2));
      HIPCHECK(hipMalloc(&stats, stats_n * 8));
      hipLaunchKernelGGL(fill_bf16, dim3(2048), dim3(256), 0, st, act, act_n, 17u + mode, 1.0f, mode == 0);
      hipLaunchKernelGGL(fill_bf16, dim3(2048), dim3(256), 0, st, w, w_n, 91u + mode, 0.05f, 0);
      GemmNTParams p{};
      p.act = act; p.wmat = w; p.out = out; p.add = nullptr;
      p.stats = mode == 0 ? stats : nullptr;
      p.M = (int)M; p.Ng = Ng; p.Kg = 9 * IC;
      p.IH = s.H; p.IW = s.W; p.IC = IC; p.OH = s.H; p.OW = s.W;
      p.IT = p.OT = p.KT = 1; p.R = p.S = 3; p.stride = 1; p.pad = 1;
      HaloArgs ha{};
      ha.ksplit = 1; ha.cps = IC / 64;
      ha.part = part; ha.cnt = cnt;
      ha.dbg = argc > 5 ? atoi(argv[5]) : 0;  // -DAVT_DIAG build only (conv_halo.h HALO_DBG; wrong results)
      ha.act_bytes = (unsigned)(act_n * 2);
      ha.w_bytes = (unsigned)(w_n * 2);
      ha.W = s.W; ha.H = s.H;
      for (int r = 0; r < 3; ++r)
        for (int c = 0; c < 3; ++c) {
          const int t = r * 3 + c;
          const int dy = mode == 0 ? r - 1 : 1 - r, dx = mode == 0 ? c - 1 : 1 - c;
          ha.tap_dy[t] = dy; ha.tap_dx[t] = dx; ha.tap_disp[t] = dy * s.W + dx; ha.tap_w[t] = t;
        }
      auto fits = [&](const Variant& V) {
        if (Ng % V.BN != 0 || V.BM + 2 * s.W + 2 > V.PRMAX) return false;
        if (V.tps2 && (IC / 64) % 2 != 0) return false;  // two taps per step: chunk pairs
        const long long tiles = (M + V.BM - 1) / V.BM * (Ng / V.BN);
        return V.pk != 2 || tiles >= 256;  // stream-K: >= nc units per block
      };
      std::vector<unsigned short> ref_out(out_n), got(out_n);
      std::vector<double> ref_st, got_st;
      std::vector<double> best(vars.size(), 1e30), sum(vars.size(), 0.0);
      for (size_t v = 0; v < vars.size(); ++v) {
        const Variant& V = vars[v];
        if (!fits(V)) continue;  // the variant does not fit the shape
        const int grid = (int)((M + V.BM - 1) / V.BM) * (Ng / V.BN);
        HIPCHECK(hipMemsetAsync(out, 0xff, out_n * 2, st));
        V.fn[mode](p, ha, grid, st);
        HIPCHECK(hipGetLastError());
        HIPCHECK(hipStreamSynchronize(st));
        HIPCHECK(hipMemcpy(v == 0 ? ref_out.data() : got.data(), out, out_n * 2, hipMemcpyDeviceToHost));
        if (mode == 0) {
          const size_t ns = kBnHdr + (size_t)((M + V.BM - 1) / V.BM) * Ng * 3;
          std::vector<double>& dst = v == 0 ? ref_st : got_st;
          dst.resize(ns);
          HIPCHECK(hipMemcpy(dst.data(), stats, ns * 8, hipMemcpyDeviceToHost));
        }
        if (v > 0) {
          size_t diff = 0;
          for (size_t i = 0; i < out_n; ++i) diff += ref_out[i] != got[i];
          size_t sdiff = 0;
          if (mode == 0 && vars[v].BM == vars[0].BM)
            for (size_t i = 0; i < ref_st.size(); ++i) sdiff += memcmp(&ref_st[i], &got_st[i], 8) != 0;
          if (diff || sdiff) {
            printf("MISMATCH %s %s %s: %zu output / %zu stat words differ\n", s.name, mode ? "dgrad" : "fwd",
                   V.name.c_str(), diff, sdiff);
            ++bad;
          }
        }
      }
      const double flop = 2.0 * M * Ng * 9.0 * IC;
      for (int r = 0; r < rounds; ++r)
        for (size_t v = 0; v < vars.size(); ++v) {
          const Variant& V = vars[v];
          if (!fits(V)) continue;
          const int grid = (int)((M + V.BM - 1) / V.BM) * (Ng / V.BN);
          for (int i = 0; i < 3; ++i) V.fn[mode](p, ha, grid, st);
          HIPCHECK(hipEventRecord(e0, st));
          for (int i = 0; i < launches; ++i) V.fn[mode](p, ha, grid, st);
          HIPCHECK(hipEventRecord(e1, st));
          HIPCHECK(hipEventSynchronize(e1));
          float ms;
          HIPCHECK(hipEventElapsedTime(&ms, e0, e1));
          const double us = ms * 1e3 / launches;
          best[v] = us < best[v] ? us : best[v];
          sum[v] += us;
        }
      printf("%-5s %-5s M=%7lld N=%4d K=%5d |", s.name, mode ? "dgrad" : "fwd", M, Ng, 9 * IC);
      for (size_t v = 0; v < vars.size(); ++v)
        if (sum[v] > 0)
          printf("  %s %7.1f us %5.0f TF/s", vars[v].name.c_str(), sum[v] / rounds, flop / (sum[v] / rounds * 1e-6) / 1e12);
      printf("\n");
      fflush(stdout);
      HIPCHECK(hipFree(act));
      HIPCHECK(hipFree(w));
      HIPCHECK(hipFree(out));
      HIPCHECK(hipFree(stats));
    }
  }
  printf(bad ? "FAILED: %d mismatches\n" : "all variants bitwise equal to base\n", bad);
  return bad ? 1 : 0;
}
