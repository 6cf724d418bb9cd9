// Host-side launchers for the per-frame CNN (ResNetBackbone, causal_anomaly_detection.py:110-158) and the
// shared dense-layer GEMMs.  All tensors are fp32, activations NHWC, frames folded into the batch axis.
#pragma once
#include "common.h"

namespace vad {

// ---------------------------------------------------------------- conv1 (1 -> 32, 7x7, s2, p3) + BN stats
int conv1_fwd(const float* x, int NF, int H, int W, const float* w, const float* b, float* y, int OH, int OW,
              float* partials, int* nparts, hipStream_t st);
int conv1_num_parts(int NF, int OH);
// frozen-stem forward without the conv1 activation (stem.hip): conv1 + bias, its BN partial sums ([P][64], the
// conv1_fwd layout and P) and the 3x3/s2 pooling of the RAW output (max where gamma >= 0, min where gamma < 0);
// the consumer applies bn1+ReLU on load (exact: the affine+ReLU is monotone per channel)
extern int g_x3_dgrad_blocks;  // knob "conv_dgrad_blocks"
extern int g_x3_big;  // knob "conv_split_big"
extern int g_x3_pipe;  // knob "conv_split_pipe"
extern int g_x3_s2big;  // knob "conv_split_s2big"
extern int g_cad_dir_affine;  // knob "cad_dir_affine": the direct classifier's loss-mode backward precomputed in the forward
extern int g_cad_stem_early;
extern int g_cad_prep_stream, g_cad_wgrad_stream, g_cad_det_gate, g_cad_last_wgrad_main, g_cad_event_sysfence,
    g_cad_dy_per_layer, g_cad_l0_slab, g_cad_stream_prio;  // knobs "cad_prep_stream", "cad_wgrad_stream" (A/B)
extern int g_stem_fused;  // knob "stem_fused" (default 1)
bool stem_fused_ok(int OW);  // conv1 output width the fused stem handles
int stem_fused(const float* x, int NF, int H, int W, const float* w, const float* b, const float* gamma, int OH,
               int OW, float* pool, int HP, int WP, float* partials, int* nparts, hipStream_t st);
// stem backward: conv1 weight gradient (dW [32][49] torch layout; slab >= NF * ceil(OH/6) * 32 * 49 floats of
// per-block partials) and the MaxPool2d(3,2,1) backward over relu(bn1(y)) (first-maximum rule)
int conv1_wgrad(const float* x, int NF, int H, int W, const float* dy, int OH, int OW, float* slab,
                int64_t slab_cap, float* dw, hipStream_t st);
int maxpool3s2_bwd(const float* y, const float* stats, const float* dpool, int NF, int H, int W, int C, int OH,
                   int OW, float* dA, hipStream_t st);

// ---------------------------------------------------------------- BatchNorm (training mode)
// partials: [P][2*C] (sum | sumsq).  Writes mean/invstd/scale/shift [C] and updates running stats.
int bn_finalize(const float* partials, int P, int C, double count, const float* gamma, const float* beta,
                float* running_mean, float* running_var, float momentum, float eps, int training, float* stats,
                hipStream_t st, int cm = 0);  // cm: partials column-major [2C][P] (the fused stem's)
// stats layout per layer (BN_STATS_PER_C = 7): [0:C) mean, [C:2C) invstd, [2C:3C) scale, [3C:4C) shift,
//   [4C:5C) k (bwd), [5C:6C) mean(dZ), [6C:7C) mean(dZ*xhat)
int bn_bwd_reduce(const float* dA, const float* y, const float* stats, int M, int C, float* partials, int* nparts,
                  hipStream_t st, int cm = 0);  // cm: partials column-major [2C][P] (coalesced finalize reads)
// when dbias is given, also the gradient of the conv bias in front of the BN: the sum over pixels of dY (zero up to
// rounding in training mode)
int bn_bwd_finalize(const float* partials, int P, int C, double count, const float* gamma, float* stats,
                    float* dgamma, float* dbeta, int training, hipStream_t st, float* dbias = nullptr, int cm = 0);
// bias_partials may be null (the conv bias grad then comes from bn_bwd_finalize's dbias)
int bn_bwd_apply(const float* dA, const float* y, const float* stats, int M, int C, float* dY, float* bias_partials,
                 int* nparts, hipStream_t st);
// the same in place (dA == dY; fp32 activations: the training stem's backward)
int bn_bwd_apply_inplace(float* dAY, const float* y, const float* stats, int M, int C, hipStream_t st);
int bn_rows_parts(int M, int C);
// SyncBatchNorm: [P][2C] partials -> [2C] double sums (+ optional float copies of the two halves); finalize from
// (all-reduced) sums over `count` elements of the whole process group
int bn_sum_partials(const float* partials, int P, int C, double* sums, float* a_out, float* b_out, hipStream_t st,
                    int cm = 0);
int bn_finalize_sums(const double* sums, int C, double count, const float* gamma, const float* beta,
                     float* running_mean, float* running_var, float momentum, float eps, float* stats,
                     hipStream_t st);
int bn_bwd_finalize_sums(const double* sums, int C, double count, const float* gamma, float* stats, hipStream_t st,
                         float* dbias = nullptr);

// ---------------------------------------------------------------- pools
int maxpool3s2_bnrelu(const float* y, const float* stats, int NF, int H, int W, int C, float* out, int OH, int OW,
                      hipStream_t st);
// AdaptiveAvgPool2d((4,6)) of relu(bn(y)) -> features [NF][C*24] (torch flatten order) and the mean over T.
int avgpool_fwd(const float* y, const float* stats, int B, int T, int H, int W, int C, float* feats, float* pooled,
                hipStream_t st);
// dA of relu(bn(y)) from the feature grads dfeat [NF][C*24] (nullable) and the clip-mean grads dpooled [B][C*24]
// (nullable); with coef the clip-mean grads are dpooled[b] + coef[b] dpooled_c[b]
int avgpool_bwd(const float* dfeat, const float* dpooled, int B, int T, int H, int W, int C, float* dA,
                hipStream_t st, const float* dpooled_c = nullptr, const float* coef = nullptr);

// ---------------------------------------------------------------- 3x3 conv as implicit GEMM
struct Conv3Layer {
  int NF, Ci, Co, IH, IW, OH, OW, stride;
};
// weight relayout: W[co][ci][3][3] -> Wf[co][9][ci] and per-parity-class dgrad images Wd[ci][taps][co]
int conv3_prep_weights(const float* w, const Conv3Layer& L, float* wf, float* wd, hipStream_t st);
// the same for n <= 8 layers in one launch
// w3 (nullable, per layer nullable): also the pre-split bf16-plane Wd image of conv3_x3_dgrad_s2
int conv3_prep_weights_all(int n, const float* const* w, const Conv3Layer* L, float* const* wf, float* const* wd,
                           hipStream_t st, __bf16* const* w3 = nullptr);
int conv3_fwd(const Conv3Layer& L, const float* src, const float* src_stats /*nullable: BN+ReLU on load*/,
              const float* wf, const float* bias, float* y, float* partials, int* nparts, hipStream_t st,
              int* parts_cm = nullptr);  // parts_cm: in = accepted, out = 1 if written so
// the BN-backward reduce of the layer below fused into an input gradient's epilogue (split kernels only): y = that
// layer's raw output, stats = its BN state; per-block sums of dZ and dZ*xhat land column-major in parts (cap floats);
// *nparts = their block count, or 0 when the dispatched kernel does not fuse (the caller then runs bn_bwd_reduce)
struct BnBwdFuse {
  const float* y;
  const float* stats;
  float* parts;
  int64_t cap;
  int* nparts;
};
int conv3_dgrad(const Conv3Layer& L, const float* dY, const float* wd, float* dX, hipStream_t st,
                const BnBwdFuse* f = nullptr, const __bf16* w3 = nullptr);
// direct LDS-patch kernels (conv_patch.hip) for stride-1 layers; conv3_fwd / conv3_dgrad route there by default
bool conv3_patch_supported(const Conv3Layer& L, bool fwd);
extern int g_patch_persist;  // single-chunk (C == 32) stride-1 layers on the persistent patch kernel
int64_t conv3_patch_blocks(int NF, int OH, int OW);  // BN partial blocks of a patch forward
int conv3_patch_fwd(const Conv3Layer& L, const float* src, const float* src_stats, const float* wf, const float* bias,
                    float* y, float* partials, int* nparts, hipStream_t st);
int conv3_patch_dgrad(const Conv3Layer& L, const float* dY, const float* wd, float* dX, hipStream_t st);
// split-bf16 patch kernels (conv_x3.hip): fp32 operands as three bf16 planes, six bf16 MFMA products per K step
extern int g_conv_split;  // 0 disables them (f32 MFMA patch kernels)
extern int g_x3_nt;       // output channels per block: 0 auto, 1 -> 32, 2 -> 64
extern int g_x3_wres;     // 32-channel stride-1 layers: all split weights resident in LDS (1, default) or restaged
// bf16-operand mode of the split kernels (one plane, one bf16 product per K step, fp32 accumulation): BASELINE
// config 4's bf16 compute.  Thread-local, set for the duration of a plan call by ConvPrecision.
extern thread_local int g_conv_bf16;
struct ConvPrecision {
  int saved;
  explicit ConvPrecision(int bf16) : saved(g_conv_bf16) { g_conv_bf16 = bf16; }
  ~ConvPrecision() { g_conv_bf16 = saved; }
};
// bf16 activation storage (common.h ActT): the stem's pooled map, the raw conv outputs y, dA and dY hold bf16 (the
// float* arguments of the launchers below then point at bf16 data). Only with g_conv_bf16 (the split kernels'
// bf16 instantiations read and write it); BN statistics, partial sums, weights and grads stay fp32. Thread-local,
// set per plan call by ActStorage.
extern thread_local int g_act_bf16;
struct ActStorage {
  int saved;
  explicit ActStorage(int bf16) : saved(g_act_bf16) { g_act_bf16 = bf16; }
  ~ActStorage() { g_act_bf16 = saved; }
};
bool conv3_x3_supported(const Conv3Layer& L, bool fwd);
int conv3_x3_fwd(const Conv3Layer& L, const float* src, const float* src_stats, const float* wf, const float* bias,
                 float* y, float* partials, int* nparts, hipStream_t st, int* parts_cm = nullptr);
int conv3_x3_dgrad(const Conv3Layer& L, const float* dY, const float* wd, float* dX, hipStream_t st,
                   const BnBwdFuse* f = nullptr);
// stride-2 input gradient on the split-bf16 (or, with conv_bf16, bf16) MFMA: parity classes of a 16x16 dX tile
// sharing one dY patch; Wd in the plain [Ci][9][Co] layout (conv3_prep_weights with classes == 0)
extern int g_dgrad_s2_x3;  // knob "conv_dgrad_s2_x3"
bool conv3_x3_dgrad_s2_supported(const Conv3Layer& L);
// w3 (nullable): the Wd image pre-split into bf16 planes [Ci][9][Co/16][3][16] (conv3_prep_weights_all's w3 image):
// the weight staging copies it instead of splitting fp32 weights in every block
int conv3_x3_dgrad_s2(const Conv3Layer& L, const float* dY, const float* wd, float* dX, hipStream_t st,
                      const BnBwdFuse* f = nullptr, const __bf16* w3 = nullptr);
extern int g_dgrad_s2_w3, g_dgrad_s2_nt;  // knob "conv_dgrad_s2_w3": the plan pre-splits the stride-2 Wd images (1, default)
bool conv3_dgrad_w3_wanted(const Conv3Layer& L);
extern int g_wgrad_split;     // stride-1 weight gradients on the split-bf16 kernel (knob "conv_wgrad_split")
extern int g_wgrad_s1_nt, g_wgrad_s1_nt_blocks, g_wgrad_s1_nt_wide;  // knobs "conv_wgrad_s1_nt", "conv_wgrad_s1_nt_blocks"
extern int g_wgrad_s2_blocks;  // their target grid size (knob "conv_wgrad_s2_blocks")
extern int g_wgrad_split_s2;  // stride-2 weight gradients on the split-bf16 kernel (knob "conv_wgrad_split_s2")
bool conv3_wgrad_x3_supported(const Conv3Layer& L);
int conv3_wgrad_x3(const Conv3Layer& L, const float* dY, const float* src, const float* src_stats, float* slab,
                   int* nsplit, int64_t partial_cap, int target_blocks, hipStream_t st);
// fp32 weight gradients (both strides) on the split-bf16 MFMA with transposed LDS fragment reads (conv_x3w.hip)
extern int g_wgrad_tr, g_wgrad_tr_blocks, g_wgrad_tr_pft;  // knobs "conv_wgrad_tr", "conv_wgrad_tr_blocks", "conv_wgrad_tr_pft"
bool x3_wgrad_tr_supported(const Conv3Layer& L);
int x3_wgrad_tr(const Conv3Layer& L, const float* dY, const float* src, const float* src_stats, float* slab,
                int* nsplit, int64_t partial_cap, int target_blocks, hipStream_t st);
bool conv3_wgrad_patch_supported(const Conv3Layer& L);
int conv3_wgrad_patch(const Conv3Layer& L, const float* dY, const float* src, const float* src_stats, float* slab,
                      int* nsplit, int64_t partial_cap, int target_blocks, hipStream_t st);
// native bf16 kernels (conv_bf.hip; bf16 operands AND bf16 activation storage, i.e. config 4): forward and stride-1
// input gradient.  Their weights are the bf16 copies the prep writes behind the fp32 images (when conv_bf16 and
// act_bf16 are set), so in that mode a wf / wd buffer holds Co*Ci*9 floats + Co*Ci*9 bf16.
extern int g_bfc, g_bfc_blocks;  // knobs "conv_bfc", "conv_bfc_blocks"
extern int g_bfc_s2_ni2;         // knob "conv_bfc_s2_ni2"
bool bfc_supported(const Conv3Layer& L, bool fwd);
inline const __bf16* conv3_bf16_image(const float* img, const Conv3Layer& L) {
  return reinterpret_cast<const __bf16*>(img + (int64_t)L.Co * L.Ci * 9);
}
int bfc_fwd(const Conv3Layer& L, const __bf16* src, const float* src_stats, const __bf16* wfb, const float* bias,
            __bf16* y, float* partials, int64_t partial_cap, int* nparts, hipStream_t st);
int bfc_dgrad(const Conv3Layer& L, const __bf16* dY, const __bf16* wdb, __bf16* dX, hipStream_t st,
              const BnBwdFuse* f);
// weight gradient (both strides) into split-K slabs [S][Co][9 Ci] (conv3_wgrad_reduce)
extern int g_bfw_blocks;  // knob "conv_bfw_blocks"
bool bfc_wgrad_supported(const Conv3Layer& L);
int bfc_wgrad(const Conv3Layer& L, const __bf16* dY, const __bf16* src, const float* src_stats, float* slab,
              int* nsplit, int64_t partial_cap, hipStream_t st);
// which kernel family conv3_fwd (kind 0) / conv3_dgrad (1) / conv3_wgrad (2) dispatches to for this layer under the
// current knobs: 6 = split-bf16 (six bf16 products per K step), 2 = native bf16 (conv_bf.hip), 1 = bf16 operands on the
// split kernels, 0 = f32 MFMA kernels
int conv3_path(const Conv3Layer& L, int kind);
// every pass of this layer (forward, input gradient when dgrad, weight gradient) runs on a split kernel under the
// current knobs, i.e. can take bf16 activations
bool conv3_act_bf16_ok(const Conv3Layer& L, bool dgrad);
// alone: nothing else runs beside this weight gradient (the last layer's): the grid fills every CU
int conv3_wgrad(const Conv3Layer& L, const float* dY, const float* src, const float* src_stats, float* partial,
                int* nsplit, int64_t partial_cap, hipStream_t st, bool alone = false);
int conv3_wgrad_reduce(const Conv3Layer& L, const float* partial, int nsplit, const float* bias_partials,
                       int nbias_parts, float* dW, float* db, hipStream_t st);

// ---------------------------------------------------------------- dense layers  Y = act(X W^T + b)
struct DenseAct {
  int relu = 0;
  // dropout after the activation (keep iff u24 >= thr), keyed by (h1, global row, col)
  int drop = 0;
  uint64_t h1 = 0;
  uint32_t thr = 0;
  float dscale = 1.f;
  int64_t row0 = 0;
};
int dense_fwd(const float* X, int M, int K, const float* W, const float* b, int N, float* Y, const DenseAct& act,
              float* scratch, int64_t scratch_floats, hipStream_t st, int max_splits = 0);
// split-K partials only: scratch[S][M][N] (finished by mlp_tail_fwd)
int dense_fwd_splitk(const float* X, int M, int K, const float* W, int N, float* scratch, int64_t scratch_floats,
                     int* nsplit, hipStream_t st);
// dX = (dY W) * gate', where gate' = (gate > 0 ? gscale : 0) when gate != nullptr; gate_rows > 0: row m is gated by
// gate row m % gate_rows
// scratch (nullable): split-K slabs when the output has few tiles and the reduction is long
int dense_dgrad(const float* dY, int M, int N, const float* W, int K, float* dX, const float* gate, float gscale,
                const int* skip, hipStream_t st, int gate_rows = 0, float* scratch = nullptr,
                int64_t scratch_floats = 0);
// dW = dY^T X, db = colsum(dY) (written, not accumulated)
// target_blocks: split-K blocks to aim for (256: one per CU; tall-M weight gradients want several per CU to hide latency)
int dense_wgrad(const float* dY, int M, int N, const float* X, int K, float* dW, float* db, float* scratch,
                int64_t scratch_floats, const int* skip, hipStream_t st, int target_blocks = 256);

// ---------------------------------------------------------------- 4x4 / stride-2 / pad-1 convs (cad1's autoencoder)
// implicit GEMMs over NHWC frames, no im2col (backbone.hip: the layouts and the parity classes)
int conv4_prep(const float* w, int D0, int D1, float* wk, float* wc, hipStream_t st);  // wk / wc nullable
// scratch (nullable): split-K slabs for grids that leave most CUs idle
int conv4_fwd(const float* src, int NF, int H, int W, int C, const float* wk, const float* bias, int N, float* out,
              hipStream_t st, float* scratch = nullptr, int64_t scratch_floats = 0);
int conv4_cls(const float* src, int NF, int SH, int SW, int C, const float* wc, const float* bias, int N, float* out,
              hipStream_t st, float* scratch = nullptr, int64_t scratch_floats = 0);
int conv4_wgrad(const float* A, int R, const float* src, int C, int NF, int AH, int AW, float* part, int* nsplit,
                int64_t part_cap, int target_blocks, hipStream_t st);
int conv4_wgrad_reduce(const float* part, int S, int R, int C, float* dW, hipStream_t st);
// ---------------------------------------------------------------- Conv3d(k3, stride 2, p1) implicit GEMMs (a2)
// wk [Co][27 Ci]; wc: 8 parity-class images back to back (27 Ci Co floats in all); C % 4 == 0
int conv3s2_prep(const float* w, int Co, int Ci, float* wk, float* wc, hipStream_t st);
// taps of parity class cls (4 pd + 2 ph + pw) of a stride-2 3-D conv's input gradient
__device__ __host__ inline int c3_nt(int cls) { return (1 + ((cls >> 2) & 1)) * (1 + ((cls >> 1) & 1)) * (1 + (cls & 1)); }
// element i (torch layout [Co][Ci][27]) of conv3s2_prep, for fused preps (a2_plan.hip)
__device__ inline void conv3s2_prep_elem(const float* __restrict__ w, int Co, int Ci, float* __restrict__ wk,
                                  float* __restrict__ wc, int64_t i) {
  const int tap = (int)(i % 27), ci = (int)((i / 27) % Ci);
  const int64_t co = i / (27 * Ci);
  const float v = w[i];
  wk[co * 27 * Ci + tap * Ci + ci] = v;
  const int kd = tap / 9, kh = (tap / 3) % 3, kw = tap % 3;
  const int pd = kd == 1 ? 0 : 1, ph = kh == 1 ? 0 : 1, pw = kw == 1 ? 0 : 1;
  const int id = kd == 2 ? 1 : 0, ih = kh == 2 ? 1 : 0, iw = kw == 2 ? 1 : 0;  // index in the dim's tap list
  const int cls = 4 * pd + 2 * ph + pw, nh = 1 + ph, nw = 1 + pw, nt = c3_nt(cls);
  int64_t off = 0;
  for (int c = 0; c < cls; ++c) off += (int64_t)c3_nt(c) * Ci * Co;
  const int t = (id * nh + ih) * nw + iw;
  wc[off + ((int64_t)ci * nt + t) * Co + co] = v;
}

// scratch (nullable): split-K slabs when the output grid leaves most CUs idle (summed in order, bias + ReLU after)
int conv3s2_fwd(const float* src, int NF, int D, int H, int W, int C, const float* wk, const float* bias, int N,
                int relu, float* out, hipStream_t st, float* scratch = nullptr, int64_t scratch_floats = 0);
int conv3s2_dgrad(const float* dy, int NF, int Co, const float* wc, int Ci, float* dx, int D, int H, int W,
                  hipStream_t st, const float* gate = nullptr);
// db (nullable): the conv bias gradient (dY's column sums) from the same GEMM (a ones column)
int conv3s2_wgrad(const float* dy, int Co, const float* src, int Ci, int NF, int D, int H, int W, float* dW,
                  float* part, int64_t part_cap, int target_blocks, hipStream_t st, float* db = nullptr);
// scratch: 256 * N doubles
int col_sum(const float* x, int64_t M, int N, float* db, double* scratch, hipStream_t st);
// the single-channel ends, 32 channels on the other side, on the VALU: w = the [32][1][4][4] / [32][16] weight
int conv4_c1_fwd(const float* src, int NF, int H, int W, const float* w, const float* bias, float* out,
                 hipStream_t st);
int conv4_c1_tfwd(const float* src, int NF, int SH, int SW, const float* w, const float* bias, float* out,
                  hipStream_t st);
int conv4_c1_wgrad(const float* A, const float* src, int NF, int AH, int AW, float* dW, float* slab,
                   int64_t slab_floats, hipStream_t st);

// conv GEMM tuning knobs: conv_fwd_tile / conv_dgrad_tile / conv_wgrad_tile (tile id, -1 = heuristic),
// conv_wgrad_blocks, conv_wgrad_min_ktiles
int set_tuning(const char* key, int value);

}  // namespace vad
