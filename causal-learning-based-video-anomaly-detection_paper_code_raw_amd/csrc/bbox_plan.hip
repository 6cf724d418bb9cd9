// avenue_training_script_bbox.py clip scorer (config 5): CausalAnomalyDetector forward (bbox:51-101) as one device
// plan, eval mode (AnomalyVisualizer.predict_anomaly_for_clip, bbox:339-368).
//
//   Conv3d 3->32 (im2col + f32 MFMA GEMM, fused bias+ReLU) -> MaxPool3d(2) -> Conv3d 32->64 (+ReLU)
//   -> AdaptiveAvgPool3d(1,4,4) -> features (B,1024) -> causal_net GEMMs 1024->256 (ReLU) ->256, classifier GEMM
//   1024->128 (ReLU) -> tail kernel: sigmoid adjacency (B,16,16) and the 128->1 sigmoid score.
// There is no batch-coupled layer, so a batch of clips of one length T is exactly B independent clips; the host
// packs a mixed-T set into one plan per T (config 5's mixed-batch packing).
#include <string>

#include "../../include/vad.h"
#include "backbone.h"
#include "conv3d.h"
#include "plan_util.h"

namespace vad {

constexpr int BB_NSLOT = 12;
struct BbSlot {
  const char* name;
  int64_t numel;
};
// model.named_parameters() order (bbox:53-84)
static const BbSlot BB_SLOTS[BB_NSLOT] = {
    {"encoder.0.weight", 32 * 3 * 27},     {"encoder.0.bias", 32},
    {"encoder.3.weight", 64 * 32 * 27},    {"encoder.3.bias", 64},
    {"causal_net.0.weight", 256 * 1024},   {"causal_net.0.bias", 256},
    {"causal_net.2.weight", 256 * 256},    {"causal_net.2.bias", 256},
    {"classifier.0.weight", 128 * 1024},   {"classifier.0.bias", 128},
    {"classifier.3.weight", 128},          {"classifier.3.bias", 1},
};

struct BbOffsets {
  int64_t off[BB_NSLOT];
  int64_t total = 0;
  BbOffsets() {
    for (int i = 0; i < BB_NSLOT; ++i) {
      off[i] = total;
      total += (BB_SLOTS[i].numel + 255) / 256 * 256;
    }
  }
};
static const BbOffsets& bb_offsets() {
  static const BbOffsets o;
  return o;
}

// encoder[0:3] (bbox:58-60): Conv3d(3->32, k3, p1) + bias -> ReLU -> MaxPool3d(2), fused, exact fp32 on the VALU.
// x NCDHW (B, 3, T, H, W) -> pooled NDHWC (B, T/2, H/2, W/2, 32).  A block owns one pooled depth slice pd of one clip
// and an 8 x 8 tile of pooled voxels: the zero-padded input window (3 channels x 4 depths x 18 x 18) is staged in
// LDS once; lane (i, j) of every wave computes the 2 x 2 x 2 conv outputs under pooled voxel (i, j) for the wave's 8
// output channels (wave-uniform: the weights are scalar operands, wT[ci][tap][32]) and keeps relu(max + bias)
// (= max of relu(conv + bias): fl(a + b) and relu are monotone in a).
__global__ __launch_bounds__(256) void bbox_conv1_pool_kernel(const float* __restrict__ x, int T, int H, int W,
                                                              const float* __restrict__ wT,
                                                              const float* __restrict__ bias, int T2, int H2,
                                                              int W2, int tiles_w, float* __restrict__ pooled) {
  constexpr int PW = 18, PH = 18, PD = 4, CI = 3;
  __shared__ float xs[CI][PD][PH][PW + 1];
  const int tid = threadIdx.x;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
  const int tiles_per_slice = gridDim.x / (T2 > 0 ? T2 : 1);
  const int pd = blockIdx.x / tiles_per_slice, tr = blockIdx.x % tiles_per_slice;
  const int b = blockIdx.y;
  const int py0 = (tr / tiles_w) * 8, px0 = (tr % tiles_w) * 8;
  const int d0 = 2 * pd - 1, y0 = 2 * py0 - 1, x0 = 2 * px0 - 1;
  const float* xb = x + (int64_t)b * CI * T * H * W;
  for (int i = tid; i < CI * PD * PH * PW; i += 256) {
    const int xx = i % PW, yy = (i / PW) % PH, dd = (i / (PW * PH)) % PD, ci = i / (PW * PH * PD);
    const int d = d0 + dd, y = y0 + yy, xw = x0 + xx;
    float v = 0.f;
    if (d >= 0 && d < T && y >= 0 && y < H && xw >= 0 && xw < W) v = xb[(((int64_t)ci * T + d) * H + y) * W + xw];
    xs[ci][dd][yy][xx] = v;
  }
  __syncthreads();
  const int pi = lane >> 3, pj = lane & 7;  // pooled voxel (py0 + pi, px0 + pj)
  const int c0 = wave * 8;
  float acc[8][8];  // [conv output (a, bb, e)][channel]
#pragma unroll
  for (int v = 0; v < 8; ++v)
#pragma unroll
    for (int c = 0; c < 8; ++c) acc[v][c] = 0.f;
#pragma unroll 1
  for (int ci = 0; ci < CI; ++ci) {
    float in[4][4][4];
#pragma unroll
    for (int dd = 0; dd < 4; ++dd)
#pragma unroll
      for (int yy = 0; yy < 4; ++yy)
#pragma unroll
        for (int xx = 0; xx < 4; ++xx) in[dd][yy][xx] = xs[ci][dd][2 * pi + yy][2 * pj + xx];
#pragma unroll
    for (int t = 0; t < 27; ++t) {
      const int kd = t / 9, kh = (t / 3) % 3, kw = t % 3;
      const float* wt = wT + (ci * 27 + t) * 32 + c0;
      float wv[8];
#pragma unroll
      for (int c = 0; c < 8; ++c) wv[c] = wt[c];
#pragma unroll
      for (int v = 0; v < 8; ++v) {
        const float xv = in[(v >> 2) + kd][((v >> 1) & 1) + kh][(v & 1) + kw];
#pragma unroll
        for (int c = 0; c < 8; ++c) acc[v][c] = fmaf(wv[c], xv, acc[v][c]);
      }
    }
  }
  const int py = py0 + pi, px = px0 + pj;
  if (py < H2 && px < W2) {
    float o[8];
#pragma unroll
    for (int c = 0; c < 8; ++c) {
      float m = acc[0][c];
#pragma unroll
      for (int v = 1; v < 8; ++v) m = fmaxf(m, acc[v][c]);
      o[c] = relu_nan(m + bias[c0 + c]);
    }
    float* dst = pooled + ((((int64_t)b * T2 + pd) * H2 + py) * W2 + px) * 32 + c0;
    *reinterpret_cast<f32x4*>(dst) = f32x4{o[0], o[1], o[2], o[3]};
    *reinterpret_cast<f32x4*>(dst + 4) = f32x4{o[4], o[5], o[6], o[7]};
  }
}

// torch Conv3d weight [32][3][27] -> [3][27][32] (channel innermost: a wave's 8 channels are one scalar load)
__global__ void bbox_conv1_wT_kernel(const float* __restrict__ w, float* __restrict__ wT) {
  for (int i = threadIdx.x; i < 32 * 81; i += blockDim.x) {
    const int c = i % 32, k = i / 32;  // k = ci * 27 + tap
    wT[i] = w[c * 81 + k];
  }
}

// one block per clip: adj = sigmoid(logits); score = sigmoid(w . h + b)
__global__ __launch_bounds__(256) void bbox_tail_kernel(const float* __restrict__ logits, const float* __restrict__ hcl,
                                                        const float* __restrict__ w3, const float* __restrict__ b3,
                                                        float* __restrict__ adj, float* __restrict__ scores) {
  const int b = blockIdx.x, t = threadIdx.x;
  adj[b * 256 + t] = 1.f / (1.f + expf(-logits[b * 256 + t]));
  __shared__ float red[128];
  if (t < 128) red[t] = w3[t] * hcl[b * 128 + t];
  __syncthreads();
  if (t == 0) {
    float z = b3[0];
    for (int k = 0; k < 128; ++k) z += red[k];
    scores[b] = 1.f / (1.f + expf(-z));
  }
}

int g_bbox_im2col = 0;

struct BbPlanImpl {
  int B, T, H, W;
  Conv3dGeom g1, g2;
  Vol5 pool_vol;
  int64_t ws_bytes = 0;
  const float* params = nullptr;
  float *cols1, *y1, *pooled, *cols2, *y2, *feats, *hc, *logits, *hcl, *scratch, *wT1, *w3;
  int64_t scratch_floats = 0;

  BbPlanImpl(int B_, int T_, int H_, int W_) : B(B_), T(T_), H(H_), W(W_) {
    g1 = conv3d_geom({B, 3, T, H, W}, 32, 3, 1, 1, 1, 1);
    const Vol5 o1 = g1.out();
    pool_vol = {B, 32, o1.D / 2, o1.H / 2, o1.W / 2};
    g2 = conv3d_geom(pool_vol, 64, 3, 1, 1, 1, 1);
  }
  const float* P(int i) const { return params + bb_offsets().off[i]; }

  void carve(Ws& w) {
    cols1 = w.take<float>(g1.rows() * g1.K());
    y1 = w.take<float>(g1.out().numel());
    pooled = w.take<float>(pool_vol.numel());
    cols2 = w.take<float>(g2.rows() * g2.K());
    y2 = w.take<float>(g2.out().numel());
    feats = w.take<float>((int64_t)B * 1024);
    hc = w.take<float>((int64_t)B * 256);
    logits = w.take<float>((int64_t)B * 256);
    hcl = w.take<float>((int64_t)B * 128);
    scratch_floats = 8ll << 20;
    scratch = w.take<float>(scratch_floats);
    wT1 = w.take<float>(32 * 81);
    w3 = w.take<float>(64 * 32 * 27);
  }

  int forward(const float* x, float* scores, float* adj, float* features, hipStream_t st) {
    DenseAct relu;
    relu.relu = 1;
    float* f = features ? features : feats;
    if (g_bbox_im2col) {  // (knob "bbox_im2col": the round-2 path -- im2col columns + f32 MFMA GEMMs)
      VAD_TRY(im2col3d(x, ncdhw_strides(g1.in), g1, nullptr, nullptr, 0, cols1, st));
      VAD_TRY(dense_fwd(cols1, (int)g1.rows(), g1.K(), P(0), P(1), 32, y1, relu, scratch, scratch_floats, st));
      VAD_TRY(maxpool3d_fwd(y1, nullptr, 0, g1.out(), 2, 2, 2, pooled, st));
      VAD_TRY(im2col3d(pooled, ndhwc_strides(pool_vol), g2, nullptr, nullptr, 0, cols2, st));
      VAD_TRY(dense_fwd(cols2, (int)g2.rows(), g2.K(), P(2), P(3), 64, y2, relu, scratch, scratch_floats, st));
      VAD_TRY(adaptive_avgpool3d_fwd(y2, nullptr, 0, g2.out(), 1, 4, 4, f, st));
    } else {
      // encoder: fused conv1 + ReLU + MaxPool3d(2) (VALU, exact fp32) -> conv2 as the depth-tap instantiation of the
      // LDS-staged split-bf16 conv kernel (implicit GEMM, no im2col) -> ReLU + AdaptiveAvgPool3d(1,4,4) on load
      hipLaunchKernelGGL(bbox_conv1_wT_kernel, dim3(1), dim3(256), 0, st, P(0), wT1);
      VAD_LAUNCH_CHECK();
      VAD_TRY(conv3d_prep_w3(P(2), 64, 32, w3, st));
      const Vol5& pv = pool_vol;
      if (pv.D > 0 && pv.H > 0 && pv.W > 0) {
        const int tiles_w = (int)cdiv(pv.W, 8), tiles = (int)cdiv(pv.H, 8) * tiles_w;
        hipLaunchKernelGGL(bbox_conv1_pool_kernel, dim3(pv.D * tiles, B), dim3(256), 0, st, x, T, H, W, wT1, P(1),
                           pv.D, pv.H, pv.W, tiles_w, pooled);
        VAD_LAUNCH_CHECK();
      }
      VAD_TRY(conv3d_x3_fwd(B, pv.D, pv.H, pv.W, 32, 64, pooled, w3, P(3), y2, st));
      VAD_TRY(adaptive_avgpool3d_fwd(y2, nullptr, 1, g2.out(), 1, 4, 4, f, st));
    }
    VAD_TRY(dense_fwd(f, B, 1024, P(4), P(5), 256, hc, relu, scratch, scratch_floats, st));
    VAD_TRY(dense_fwd(hc, B, 256, P(6), P(7), 256, logits, DenseAct{}, scratch, scratch_floats, st));
    VAD_TRY(dense_fwd(f, B, 1024, P(8), P(9), 128, hcl, relu, scratch, scratch_floats, st));
    hipLaunchKernelGGL(bbox_tail_kernel, dim3(B), dim3(256), 0, st, logits, hcl, P(10), P(11), adj, scores);
    VAD_LAUNCH_CHECK();
    return 0;
  }
};

}  // namespace vad

using namespace vad;

struct vad_bbox_plan {
  vad_bbox_plan(int B, int T, int H, int W) : impl(B, T, H, W) {}
  BbPlanImpl impl;
};

extern "C" {

int vad_bbox_num_slots(void) { return BB_NSLOT; }
const char* vad_bbox_slot_name(int i) { return (i >= 0 && i < BB_NSLOT) ? BB_SLOTS[i].name : nullptr; }
int64_t vad_bbox_slot_numel(int i) { return (i >= 0 && i < BB_NSLOT) ? BB_SLOTS[i].numel : -1; }
int64_t vad_bbox_slot_offset(int i) { return (i >= 0 && i < BB_NSLOT) ? bb_offsets().off[i] : -1; }
int64_t vad_bbox_param_floats(void) { return bb_offsets().total; }

int vad_bbox_create(int B, int T, int H, int W, vad_bbox_plan** out) {
  VAD_CHECK(out != nullptr, "vad_bbox_create: out is null");
  VAD_CHECK(B >= 1 && T >= 2 && H >= 2 && W >= 2, "vad_bbox_create: unsupported shape (MaxPool3d(2) needs T,H,W >= 2)");
  auto* p = new vad_bbox_plan(B, T, H, W);
  Ws ws;
  p->impl.carve(ws);
  p->impl.ws_bytes = ws.off + 256;
  *out = p;
  return 0;
}
void vad_bbox_destroy(vad_bbox_plan* plan) { delete plan; }
int64_t vad_bbox_workspace_bytes(const vad_bbox_plan* p) { return p ? p->impl.ws_bytes : -1; }

int vad_bbox_bind(vad_bbox_plan* plan, void* workspace, const float* params) {
  VAD_CHECK(plan && workspace && params, "vad_bbox_bind: null argument");
  VAD_CHECK((reinterpret_cast<uintptr_t>(workspace) & 255) == 0, "vad_bbox_bind: workspace must be 256-B aligned");
  Ws ws;
  ws.base = reinterpret_cast<char*>(workspace);
  ws.dry = false;
  plan->impl.carve(ws);
  plan->impl.params = params;
  return 0;
}

int vad_bbox_forward(vad_bbox_plan* plan, const float* x, float* scores, float* adj, float* features, void* stream) {
  VAD_CHECK(plan && x && scores && adj, "vad_bbox_forward: null argument");
  VAD_CHECK(plan->impl.params != nullptr, "vad_bbox_forward: plan not bound");
  return plan->impl.forward(x, scores, adj, features, (hipStream_t)stream);
}

}  // extern "C"
