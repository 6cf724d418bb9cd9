// 3-D building blocks shared by the clip-level 3-D CNNs (minicausal SimpleVideoAnomalyDetector mc:25-102, the a2
// CompactFeatureExtractor a2:27-35 and the bbox detector bbox:58-65).
//
// Convolutions run as im2col + f32 MFMA GEMM (backbone.h dense_fwd / dense_dgrad / dense_wgrad): with the column
// index k = ci*KD*KH*KW + (kd*KH + kh)*KW + kw the torch Conv3d weight [Co][Ci][KD][KH][KW] IS the row-major
// [Co][K] GEMM operand, so no weight re-layout is needed, and the weight + bias gradient is one GEMM with a ones
// column.  Activations are NDHWC (channels innermost); the clip input may be read in torch's NCDHW directly.
#pragma once
#include "common.h"

namespace vad {

struct Vol5 {
  int N, C, D, H, W;
  __host__ __device__ int64_t voxels() const { return (int64_t)N * D * H * W; }
  __host__ __device__ int64_t numel() const { return voxels() * C; }
};
// element (n, c, d, h, w) of a source tensor lives at n*n_ + c*c_ + d*d_ + h*h_ + w*w_
struct Strides5 {
  int64_t n, c, d, h, w;
};
inline Strides5 ndhwc_strides(const Vol5& v) {
  return {(int64_t)v.D * v.H * v.W * v.C, 1, (int64_t)v.H * v.W * v.C, (int64_t)v.W * v.C, v.C};
}
inline Strides5 ncdhw_strides(const Vol5& v) {
  return {(int64_t)v.C * v.D * v.H * v.W, (int64_t)v.D * v.H * v.W, (int64_t)v.H * v.W, v.W, 1};
}

struct Conv3dGeom {
  Vol5 in;   // source dims
  int Co;
  int kd, kh, kw, sd, sh, sw, pd, ph, pw;
  int OD, OH, OW;
  __host__ __device__ int K() const { return in.C * kd * kh * kw; }
  __host__ __device__ int64_t rows() const { return (int64_t)in.N * OD * OH * OW; }
  __host__ __device__ Vol5 out() const { return {in.N, Co, OD, OH, OW}; }
};
Conv3dGeom conv3d_geom(const Vol5& in, int Co, int k, int s_d, int s_h, int s_w, int pad);

// cols[rows][K]; optional relu(scale*x + shift) / relu(x) of the source applied on load (scale nullable)
int im2col3d(const float* src, const Strides5& s, const Conv3dGeom& g, const float* scale, const float* shift,
             int relu, float* cols, hipStream_t st);
// dsrc (NDHWC, in dims) = col2im(dcols) (+ bias[c] when bias != nullptr: a transposed conv's output)   (written,
// not accumulated)
int col2im3d(const float* dcols, const Conv3dGeom& g, float* dsrc, hipStream_t st, const float* bias = nullptr);

// Non-overlapping MaxPool3d (kernel == stride, floor mode) over act(y) where act = relu(scale*y + shift) when
// stats != nullptr (stats layout of bn_finalize) or relu(y) when relu, else identity.  out NDHWC.
int maxpool3d_fwd(const float* y, const float* stats, int relu, const Vol5& v, int kd, int kh, int kw, float* out,
                  hipStream_t st);
// dA (NDHWC, v dims) = grad w.r.t. act(y): the pooled grad routed to the FIRST max of each window (torch's scan
// order), zero elsewhere and outside complete windows.
int maxpool3d_bwd(const float* y, const float* stats, int relu, const Vol5& v, int kd, int kh, int kw,
                  const float* dout, float* dA, hipStream_t st);

// AdaptiveAvgPool3d((OD,OH,OW)) of act(x) (x NDHWC) -> out[n][c*OD*OH*OW + (od*OH + oh)*OW + ow] (torch flatten)
int adaptive_avgpool3d_fwd(const float* x, const float* stats, int relu, const Vol5& v, int OD, int OH, int OW,
                           float* out, hipStream_t st);
// dx (NDHWC) = backward of the average (act' is NOT applied: callers route through their ReLU/BN backward)
// gate (nullable, dx's layout): dx = 0 where !(gate > 0) -- the backward of a ReLU whose output is gate, fused
int adaptive_avgpool3d_bwd(const float* dout, const Vol5& v, int OD, int OH, int OW, float* dx, hipStream_t st,
                           const float* gate = nullptr);

// Conv3d k3 p1 s1 on NDHWC volumes (B clips x D slices x H x W x C) with split-bf16 MFMA (fp32-class numerics,
// conv_x3.hip): w3 = weights as [kd][N][kh*3+kw][C] (conv3d_prep_w3), out = conv + bias (no activation), NDHWC
int conv3d_x3_fwd(int B, int D, int H, int W, int C, int N, const float* src, const float* w3, const float* bias,
                  float* out, hipStream_t st);
// torch Conv3d weight [N][C][3][3][3] -> [3][N][9][C]
int conv3d_prep_w3(const float* w, int N, int C, float* w3, hipStream_t st);

// Direct Conv3d k3 s1 p1 for small channel counts (conv3d_direct.hip; fp32 FMA, no im2col).  Supported: Ci <= 16,
// Co in {8, 16, 32} (knob "conv3d_direct" off: false).  prep: torch weight [Co][Ci][27] -> wf [Ci][27][Co] (forward)
// and wd [Co][27][Ci] (flipped taps: the input gradient is conv3d_direct_fwd over dY with wd, CO = Ci).
extern int g_conv3d_direct, g_conv3d_wg_blocks;
bool conv3d_direct_supported(int Ci, int Co);
int conv3d_direct_prep(const float* w, int Co, int Ci, float* wf, float* wd, hipStream_t st);
// out (NDHWC, in's spatial dims, CO channels) = conv(src) + bias (nullable)
int conv3d_direct_fwd(const float* src, const Strides5& s, const Vol5& in, const float* w, int CO, const float* bias,
                      float* out, hipStream_t st);
// dW [Co][Ci][27] and db [Co] (nullable) written (not accumulated) from dY (NDHWC, CO channels) and the forward input
int conv3d_direct_wgrad(const float* dy, int CO, const float* src, const Strides5& s, const Vol5& in, float* dW,
                        float* db, float* slab, int64_t slab_floats, hipStream_t st);
int64_t conv3d_direct_wgrad_slab_floats(const Vol5& in, int CO);

// per-block column sums / sums of squares of Y[M][C] -> partials [P][2C] (bn_finalize layout)
int bn_fwd_partials(const float* y, int64_t M, int C, float* partials, int* nparts, hipStream_t st);
int64_t bn_fwd_partials_blocks(int64_t M);

}  // namespace vad
