// The conv kernels' parameter blocks (NT fwd / dgrad, TN wgrad), shared by conv_gemm.hip and the standalone kernel
// benches under tools/ (included inside namespace avt).
#pragma once

// ------------------------------------------------------------------------------------------------
// NT kernel (fwd / dgrad)
// ------------------------------------------------------------------------------------------------
enum { MODE_FWD = 0, MODE_DGRAD = 1 };

struct GemmNTParams {
  const bf16_t* act;   // gather source: x [N][IH][IW][IC] (fwd) or dy [N][IH][IW][IC] (dgrad)
  const bf16_t* wmat;  // [Ng][Kg] bf16, K contiguous
  bf16_t* out;         // [M][Ng] bf16
  const bf16_t* add;   // optional [M][Ng] bf16 added to the result (may alias out)
  double* stats;       // optional BN accumulator (avt_common.h): per row tile t the fp32 results'
                       // (sum_t, M2_t about the tile mean, sum_t^2/n_t) are stored into slot t
  int M, Ng, Kg;
  int IH, IW, IC;      // source tensor geometry
  int OH, OW;          // pixel grid of the GEMM rows
  int IT, OT;          // temporal extent of source / rows (Conv3d, temporal stride 1; 1 for Conv2d)
  int KT, pad_t;       // temporal taps and padding (Conv3d; 1 / 0 for Conv2d)
  int R, S, stride, pad;
  // dgrad only -- fused BatchNorm-backward epilogue (conv_epi.h), active when bx != nullptr: the
  // result g (after `add`) is masked by the ReLU of the BN that produced the positions' activations,
  // g' = g * [by > 0] (by given: the block output) or g * [fma(bx, scale, shift) > 0] (BasicBlock.bn1),
  // stored as g', and that BN's backward reductions (sum g', sum g' * xhat), xhat = (bx - mean)*invstd,
  // are stored into slot bslot_base (+ bacc's header[0] when bappend) + the block's row tile of bacc (avt_common.h;
  // bslot_total: the slots of all launches of this call, 0 = this launch's row tiles); bx2/bst2/bacc2 optionally a second BN fed
  // by the same g' (the downsample BN of a first block: bn2 and downsample.1 share the ReLU).
  const bf16_t* bx;
  const bf16_t* by;
  const float* bst;    // [4][Ng]: scale, shift, mean, invstd
  double* bacc;
  const bf16_t* bx2;
  const float* bst2;
  double* bacc2;
  int bskip00;         // host side: a stride-2 dgrad's class-(0,0) launch stores plain g (another
                       // kernel -- the downsample dgrad -- adds to those pixels and applies the epilogue)
  int bslot_base, bslot_total, bappend;
  const unsigned char* amask;  // optional [M][Ng/8] bits: `add` enters masked, add * bit (an identity
                               // block's residual gradient g * [out > 0], from avt_bn_apply_mask's bits)
};

__device__ __forceinline__ int swz64(int row, int chunk) {  // byte offset in a [rows][32 bf16] tile
  return row * 64 + ((chunk ^ ((row >> 2) & 3)) << 4);
}

// wgrad ("TN"): dw[Mg][R*S*Creal] += sum over the Kred output pixels of dy[pix][Mg] * x[gathered pixel][(r,s,c)]
struct GemmTNParams {
  const bf16_t* dy;  // [Kred][Mg]
  const bf16_t* x;   // [N][H][W][Cp]
  float* dw;         // [Mg][R*S*Creal] fp32 (atomic accumulate)
  int Mg, Ng, Kred;  // Ng = padded patch width (multiple of BN)
  int H, W, Cp, Creal, P, Q, R, S, stride, pad;
  int kt_per_split;
};
