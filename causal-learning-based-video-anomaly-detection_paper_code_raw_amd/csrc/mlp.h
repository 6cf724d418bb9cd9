// Fused MLP chains (detector_net / direct_classifier) and the generic row-reduction weight gradient.
#pragma once
#include "common.h"

namespace vad {

constexpr int MLP_MAXW = 512;  // widest activation kept in LDS (layer-0 output)

struct MlpLayer {
  const float* W;  // [N][K]
  const float* b;  // [N]
  float* out;      // [M][N]
  int K, N;
  int relu, drop;
  uint64_t h1;
  uint32_t thr;
  float dscale;
};

// layers 1-4 on top of layer 0's finished output L[0].out (only L[0].out / L[0].N are read)
struct MlpTailArgs {
  int M;
  int64_t row0;        // global row of row 0 (dropout key)
  MlpLayer L[5];
  const float* WT[5];  // transposed weights WT[i][k][n] of layers 1-4
  // optional: layer 0 as split-K partial sums parts[nsplit][M][L[0].N] (dense_fwd_splitk); the kernel then finishes
  // layer 0 itself (fixed-order sum, bias, ReLU, dropout per L[0]) and writes L[0].out
  const float* parts;
  int nsplit;
};

struct MlpTransposeArgs {
  int n;
  const float* W[8];
  float* WT[8];
  int K[8], N[8];
};
int mlp_transpose(const MlpTransposeArgs& a, hipStream_t st);

// input-gradient chain: d[i-1] = (d_i W_i) * (h[i-1] > 0 ? gscale[i-1] : 0), d_4 = dout
struct MlpTailBwdArgs {
  int M;
  const float* dout;  // [M][N[4]]
  const float* W[5];
  int K[5], N[5];
  const float* h[4];   // forward outputs of layers 0..3 (post ReLU/dropout)
  float gscale[4];
  float* d[4];         // outputs: grads w.r.t. the pre-activations of layers 0..3
  const int* skip;     // nullable device flag: 0 -> no-op
};

extern int g_mlp_tail_wide;  // knob "mlp_tail_wide"
extern int g_mlp_tail_rb;    // knob "mlp_tail_rb"
int mlp_tail_fwd(const MlpTailArgs& a, hipStream_t st);
// Direct classifier (cad:525-538) with its loss-mode backward precomputed as an affine function of the causal score
// c (cad:655-676): with fin = 0.6 c + 0.4 p1 the upstream gradient of the logits is d_l[b] = A[b] + c[b] beta[b], and
// the classifier's input-gradient chain is linear in d_l, so it runs on the 2B stacked rows [A; beta] while the causal
// head computes c (B <= 8).  dir_mid runs layers 2-4 forward, the seed rows and the layer 4-1 input gradients in one block.
struct DirMidArgs {
  int B;
  const float *h0, *h1;                              // [B][512], [B][256] (layer 0 / 1 outputs, after dropout)
  const float *W1, *W2, *b2, *W3, *b3, *W4, *b4;     // [256][512], [128][256], [64][128], [2][64]
  float *h2, *h3, *logits;                           // [B][128], [B][64], [B][2]
  const int64_t* labels;                             // [B]
  float gs0, gs1;                                    // gate scales of layer 0 / 1 outputs (1 / (1 - p) in training)
  float *dl2, *d3, *d2, *d1, *d0;                    // [2B][2], [2B][64], [2B][128], [2B][256], [2B][512]
};
int dir_mid(const DirMidArgs& a, hipStream_t st);
// dst_s[b][k] = src_s[b][k] + c[b] src_s[B + b][k] for up to 6 segments (the stacked rows folded once c is known)
struct DirCombineArgs {
  int B, nseg;
  const float* c;
  const float* src[6];
  float* dst[6];
  int width[6];
};
int dir_combine(const DirCombineArgs& a, hipStream_t st);

int mlp_tail_bwd(const MlpTailBwdArgs& a, hipStream_t st);

// dW[o][i] = sum_r A[r][o] X[r][i], db[o] = sum_r A[r][o] for up to ROWS_WGRAD_MAXSEG Linear layers, one launch
constexpr int ROWS_WGRAD_MAXSEG = 6;
struct RowsWgradSeg {
  float* dW;
  float* db;  // nullable
  const float* A;  // [R][O]
  const float* X;  // [R][I]
  int O, I;
};
struct RowsWgradArgs {
  int R, nseg;
  RowsWgradSeg seg[ROWS_WGRAD_MAXSEG];
  const int* skip;
};
int rows_wgrad(const RowsWgradArgs& a, hipStream_t st);

}  // namespace vad
