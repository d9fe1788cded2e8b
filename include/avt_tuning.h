/* libavt A/B knobs -- measurement only, NOT part of the drop-in boundary (include/avt.h).
 *
 * Each knob selects between kernel variants that were measured against each other; the
 * defaults are the measured winners, and every setting computes the same function (most bitwise, see
 * each).  They are process-global state, read by the launchers: set them once, before any launch, from
 * one thread -- the entry points of avt.h themselves are stateless and re-entrant per stream.  The
 * environment variables named below set the same defaults at first use (bench.py records every AVT_*
 * variable in its JSON line).
 */
#ifndef AVT_TUNING_H_
#define AVT_TUNING_H_

#ifdef __cplusplus
extern "C" {
#endif

/* conv kernel family for fwd/dgrad: 1 = LDS-DMA pipelined (default), 0 = register-staged
 * (the first implementation, kept for A/B measurement; env AVT_CONV_VARIANT sets the default) */
int avt_set_conv_variant(int variant);
/* weight-ring stages of the layer3/4 halo conv tiles: nst128 (128 x 128 tile) and nst64 (64 x 128
 * small-batch tile) in 2..5 (one block per CU from nst128 = 3 / nst64 = 4 on); all settings give bitwise-identical results (A/B knob) */
int avt_set_halo_stages(int nst128, int nst64);
/* tile config of the pipelined fwd/dgrad kernel when the GEMM N is 64 wide (-1 (default): 1, or 2 for a
 * Conv3d; 0: 256x64/4 stages, 1: 128x64/3 stages, 2: 128x64/4 stages, 3: 256x64/2 stages, 4: 128x64 k64/3 stages,
 * 5: 256x64 k64/2 stages, 6: 128x64 k64/2 stages, 7: 256x64 8 waves k64/3, 8: 256x64 8 waves k64/2)
 * — an A/B knob */
int avt_set_nt64_config(int cfg);
/* 1 (default; env AVT_HALO): 3x3 stride-1 fwd/dgrad with C % 64 == 0 and K % 128 == 0 run on the halo-reuse
 * kernel (each input pixel moved to LDS once per 64-channel chunk instead of once per tap): 4-wave 128x128
 * tiles for W <= 19 (layer3/4), 8-wave 256x128 tiles for W <= 79 (layer2); 0: tap-gather kernel everywhere;
 * 2: the 8-wave forms for every width (and 256x64 for K = 64) — an A/B knob */
int avt_set_halo(int on);
/* 1 (default; env AVT_HALO8): under avt_set_halo(1), layer3/4 shapes also take the 8-wave 256x128 halo
 * tile where it measured faster (C >= 512, or 256-row tiles fitting one wave of blocks); 0: the 4-wave
 * 128x128 tile for every W <= 19 shape; -1: back to the environment default — an A/B knob */
int avt_set_halo8(int on);
/* weight-ring stages of the 8-wave 256x128 halo tile: 3 (default) or 4 (150 KB of LDS, still one block per
 * CU); -1: the environment default (AVT_HALO8_NST) — an A/B knob (bitwise the same results) */
int avt_set_halo8_nst(int nst);
/* wave layout of the 256x128 halo tile: 0 (default) = 8 waves of 64x64, 1 = 4 waves of 128x64 (0.75 KB of
 * LDS reads per MFMA, one wave per SIMD); -1: the environment default (AVT_HALO8_FORM) — an A/B knob
 * (bitwise the same outputs; the BN statistics summed over another wave partition) */
int avt_set_halo8_form(int form);
/* 1 (default; env AVT_C64): 3x3 stride-1 fwd/dgrad with C = K = 64 (the layer-1 convs, image width <= 95)
 * run on the persistent kernel whose 64 x 576 weight operand stays resident in LDS (halo patch per
 * 256-pixel tile); 0: the tap-gather kernel (also off whenever avt_set_halo(0)) — an A/B knob */
int avt_set_c64(int on);
/* 1 (default; env AVT_S2_ONE): a stride-2 dgrad without the BN-backward epilogue runs its output parity
 * classes (each with only the taps that reach it) as ONE launch, blocks of the classes with the most taps
 * dispatched first; 0: one launch per class.  The results are bitwise identical (same tap order). */
int avt_set_s2_dgrad_one(int on);
/* ... and when the GEMM N is a multiple of 128 (-1: by GEMM M, 6 if M >= 65536 else 1 (default; a Conv3d
 * with K >= 3072 always 1);
 * 0: 128x128 k32/4 stages, 1: 128x128 k64/2, 2: 128x128 k64/3, 3: 256x128 k32/3, 4: 256x128 k64/2,
 * 5: 256x128 8 waves k64/2, 6: 256x128 8 waves k32/3) */
int avt_set_nt128_config(int cfg);
/* fwd/dgrad tiles of 64 rows (64x128 / 64x64; a 64x128 halo tile for layer3/4) when the 128-row tile
 * grid would give fewer than `waves` blocks per CU (small per-GPU batches); 0 = never, -1 = always, -2 = back to
 * the environment: AVT_SMALL_TILES (blocks per CU) or AVT_SMALL_TILES_PCT (% of the CUs; default 50) */
int avt_set_small_tiles(int waves);
/* wgrad split-K policy: target_blocks 0 = wave model (default), >0 = about that many blocks in total;
 * at least min_ktiles 32-pixel tiles per block */
int avt_set_wgrad_policy(int target_blocks, int min_ktiles);
/* wgrad split-K partials go through a slab + reduce up to max_splits splits (default: all -- deterministic;
 * beyond it fp32 atomics, whose summation order varies run to run; an A/B knob);
 * wave_cost = per-block fixed cost in k-tiles used by the wave model */
int avt_set_wgrad_slab_max(int max_splits, int wave_cost);
/* 1 (default): layer4 wgrads (K_out 512) use 8-wave 256-wide tiles; 0: 4-wave tiles of at most 128 — A/B knob */
int avt_set_wgrad_tiles(int big);
/* 3x3/s1 wgrads on the halo-reuse kernel -- 1: all 9 taps per block, 2: one filter row (3 taps) per
 * block, 3 (default): form 2 for the K = 64 (layer-1) convs and the tap-gather kernel elsewhere -- or all
 * on the tap-gather one (0); -1: back to env AVT_WGRAD_HALO.  Returns AVT_EINVAL outside -1..3 */
int avt_set_wgrad_halo(int on);
/* the one-filter-row form: k groups per 2-wave block pair (1, 2 or 4; env AVT_ROW3_KG, default 2), the floor
 * of k-tiles per split (env AVT_ROW3_MIN_KT, default 8), and (two k groups) the next tile's first fragments
 * read behind the current tile's MFMAs (1, env AVT_ROW3_PF, default) or after its barrier (0); -1 resets a value
 * to its environment default */
int avt_set_wgrad_row3(int kg, int min_kt, int pf);
/* the Conv3d 3x3x3 / stride 1 / pad 1 convs on the halo kernel's three-patch form -- 2 (default, env AVT_HALO3D): the
 * N % 128 == 0, W <= 79 ones (R3D-18 layer2-4) and the N = 64, W <= 115 ones (layer1); 1: the former only; 0: all on
 * the tap-gather kernel; -1: back to the environment default */
int avt_set_halo3d(int on);
/* A/B knob, 0 by default (env AVT_HALO_TPS2): 1 = the 8-wave 256 x 128 halo fwd/dgrad of the >= 8-chunk convs waits
 * and synchronises once per two taps (a 2-stage ring of two weight tiles) with waves 4-7 at s_setprio 1; -1: back to
 * the environment default.  Bitwise-equal results either way */
int avt_set_halo_tps2(int on);
/* A/B knob, avt_conv2d_wgrad_tk's in-kernel slab reduce: 1 = on where the other splits' partials of a tile are at most
 * max_kb KiB (env AVT_WGRAD_FUSED_MAX_KB, default 2048); 0 (default, env AVT_WGRAD_FUSED) = the separate reduce launch
 * (measured faster); -1: back to the environment default */
int avt_set_wgrad_fused(int on, int max_kb);
/* 1 (default, env AVT_STEM): the 7x7/s2 stem forwards (C 4 or 1, K 64) run on the per-wave LDS-patch
 * stem kernel (BN statistics of the stored bf16 tensor, on the MFMA pipe); 0: the generic gather kernel */
int avt_set_stem_kernel(int on);
/* 1 (default, env AVT_STEM_WGRAD): the 7x7/s2 stem wgrads (C 4 or 1, K 64) run on the per-wave
 * LDS-patch kernel (needs the avt_conv2d_wgrad_workspace() slab; deterministic); 0: the generic one */
int avt_set_stem_wgrad(int on);
int avt_set_halo_splitk(int ksplit, int target_blocks);
/* TN wgrad LDS ring depth: nst for the 4-wave tiles (4 default, 6, 8), nst_big for the 8-wave 256 x 256
 * tile (3 default, 4, 5) -- deeper rings keep more k-tiles in flight for a block alone on its CU */
int avt_set_wgrad_nst(int nst, int nst_big);
/* share of the chip's block slots the tap-gather wgrad's split-K planner assumes (the other trunk's kernels run
 * beside it): 0 auto (65 at batch <= 32, 75 at <= 64, else 100), 1-100 fixed, -1 env AVT_WGRAD_SLOTS_PCT (unset:
 * auto).  Workspace sizes follow the plan: query avt_conv2d_wgrad_workspace after changing it. */
int avt_set_wgrad_slots_pct(int pct);

#ifdef __cplusplus
}
#endif

#endif  /* AVT_TUNING_H_ */
