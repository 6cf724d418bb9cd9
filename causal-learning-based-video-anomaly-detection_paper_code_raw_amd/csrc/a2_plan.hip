// avenue_training_script2.py: the a2 CausalAnomalyDetector (a2:15-101), compute_improved_loss (a2:135-205) and
// the ImprovedMiniCausalVAD train step (a2:218-245) as one device plan.
//
//   forward   3 x [im2col3d -> f32 MFMA GEMM with fused bias+ReLU] (strides (1,2,2), 2, 2) -> AdaptiveAvgPool3d(4,4,4)
//             -> fc GEMM (4096 -> 16) with the keyed Dropout(0.3) -> one block-wide kernel for the causal-discovery
//             MLP (sigmoid adjacency, zero diagonal), graph encoder (Dropout .3) and predictor -> the loss kernel
//             (compute_improved_loss and its gradients w.r.t. scores and adjacency)
//   backward  loss + head backward in the same block-wide style (weight grads as fixed-order sums over the batch),
//             fc weight / input grads as GEMMs, avg-pool backward, then per stage ReLU gate -> weight+bias grad GEMM
//             over the saved columns -> input grad GEMM + col2im
//   update    clip_grad_norm_(0.5) (norm of per-parameter norms) -> AdamW (decoupled weight decay)
// losses[]: 0 total, 1 anomaly(focal), 2 acyclicity, 3 sparsity, 4 consistency, 5 structure, 6 edge_count,
//           7 sparsity_ratio, 8 grad total norm, 9 status (0 skipped: NaN loss, 2 stepped)
#include <cmath>
#include <string>
#include <vector>

#include "../../include/vad.h"
#include "backbone.h"
#include "conv3d.h"
#include "plan_util.h"

namespace vad {

int g_a2_head_clip = 1;  // knob "a2_head_clip": the head forward / backward one block per clip (0: one launch per layer)
int g_a2_direct = 1;  // knob "a2_direct": conv3d_1 direct on the VALU (latched per plan; 0: im2col + GEMM)

constexpr int A2_NSLOT = 20;
constexpr int A2_CO[3] = {16, 32, 64};
constexpr int A2_MAXB = 256;

struct A2Slot {
  const char* name;
  int64_t numel;
};
static const A2Slot A2_SLOTS[A2_NSLOT] = {
    {"feature_extractor.conv3d_1.weight", 16 * 3 * 27}, {"feature_extractor.conv3d_1.bias", 16},
    {"feature_extractor.conv3d_2.weight", 32 * 16 * 27}, {"feature_extractor.conv3d_2.bias", 32},
    {"feature_extractor.conv3d_3.weight", 64 * 32 * 27}, {"feature_extractor.conv3d_3.bias", 64},
    {"feature_extractor.fc.weight", 16 * 4096},          {"feature_extractor.fc.bias", 16},
    {"causal_discovery.causal_net.0.weight", 32 * 16},   {"causal_discovery.causal_net.0.bias", 32},
    {"causal_discovery.causal_net.2.weight", 256 * 32},  {"causal_discovery.causal_net.2.bias", 256},
    {"graph_encoder.0.weight", 128 * 256},               {"graph_encoder.0.bias", 128},
    {"graph_encoder.3.weight", 64 * 128},                {"graph_encoder.3.bias", 64},
    {"anomaly_predictor.0.weight", 32 * 80},             {"anomaly_predictor.0.bias", 32},
    {"anomaly_predictor.2.weight", 32},                  {"anomaly_predictor.2.bias", 1},
};
enum {
  S_C1W, S_C1B, S_C2W, S_C2B, S_C3W, S_C3B, S_FCW, S_FCB, S_CN0W, S_CN0B, S_CN2W, S_CN2B,
  S_GE0W, S_GE0B, S_GE3W, S_GE3B, S_AP0W, S_AP0B, S_AP2W, S_AP2B
};

struct A2Offsets {
  int64_t off[A2_NSLOT];
  int64_t total;
  A2Offsets() {
    total = 0;
    for (int i = 0; i < A2_NSLOT; ++i) {
      off[i] = total;
      total += (A2_SLOTS[i].numel + 255) / 256 * 256;
    }
  }
};
static const A2Offsets& a2_offsets() {
  static const A2Offsets o;
  return o;
}

// ------------------------------------------------------------------ head
// The head is a chain of small Linear layers over B rows (a2:27-101); each layer is one launch with one thread per
// output (out[b][n] = sum_k in[b][k] W[n][k] + bias[n], k in order), so the chain spreads over the CUs instead of one
// block walking it.
__device__ __forceinline__ float a2_dot(const float* __restrict__ x, const float* __restrict__ w, int K, float z) {
  for (int k = 0; k < K; ++k) z = fmaf(w[k], x[k], z);
  return z;
}
__device__ __forceinline__ float a2_sigmoid(float z) { return 1.f / (1.f + expf(-z)); }

struct A2HeadArgs {
  int B, training, with_loss;
  int64_t clip0;
  const float* P;  // params base
  const int64_t* off;
  float *f, *hc0, *sig, *adj, *g1, *g1d, *g2, *cat, *hp0, *s;  // saved activations
  uint64_t h_graph, h_pseudo;
  uint32_t thr_graph;
  float s_graph;
  float* losses;
  float* pseudo;  // [B]
  float* d_s;     // [B]  upstream grads written by the loss
  float* d_adj;   // [B][256]
  float* red;     // [256] scratch
  float* pairs;   // [B][B] mean |A_i - A_j| of the pseudo-normal pairs i < j
  float* lsc;     // [8] loss scalars between the loss launches: focal sum, acyclicity, edges, avg, csign, np
  // fc (a2:?: Linear(4096, 16) + Dropout(0.3) on the pooled features) inside the per-clip forward: pooled [B][4096]
  const float* pooled;  // null: f was written by dense_fwd (the per-layer launch path)
  uint64_t h_fc;
  uint32_t thr_fc;
  float s_fc;
};

// forward stage st: 0 causal_net.0 (+ReLU), 1 causal_net.2 (+sigmoid) -> sig, adj (zero diagonal), 2 graph_encoder.0
// (+ReLU, Dropout) -> g1, g1d, 3 graph_encoder.3 -> g2 and the predictor input cat = [f, g2], 4 anomaly_predictor.0
// (+ReLU), 5 anomaly_predictor.2 (+sigmoid) -> s
constexpr int A2_FWD_N[6] = {32, 256, 128, 64, 32, 1};

__global__ __launch_bounds__(256) void a2_head_fwd_kernel(A2HeadArgs a, int st) {
  const int B = a.B, idx = blockIdx.x * 256 + threadIdx.x;
  const float* P = a.P;
  const int64_t* o = a.off;
  switch (st) {
    case 0:
      if (idx < B * 32) {
        const int b = idx / 32, n = idx % 32;
        a.hc0[idx] = relu_nan(a2_dot(a.f + b * 16, P + o[S_CN0W] + n * 16, 16, P[o[S_CN0B] + n]));
      }
      break;
    case 1:
      if (idx < B * 256) {
        const int b = idx / 256, e = idx % 256;
        const float sg = a2_sigmoid(a2_dot(a.hc0 + b * 32, P + o[S_CN2W] + e * 32, 32, P[o[S_CN2B] + e]));
        a.sig[idx] = sg;
        a.adj[idx] = (e / 16 == e % 16) ? sg * 0.f : sg;  // * (1 - eye)
      }
      break;
    case 2:
      if (idx < B * 128) {
        const int b = idx / 128, n = idx % 128;
        float v = relu_nan(a2_dot(a.adj + b * 256, P + o[S_GE0W] + n * 256, 256, P[o[S_GE0B] + n]));
        a.g1[idx] = v;
        if (a.training)
          v = rng_u24(a.h_graph, (uint64_t)(a.clip0 + b), (uint64_t)n) >= a.thr_graph ? v * a.s_graph : 0.f;
        a.g1d[idx] = v;
      }
      break;
    case 3:
      if (idx < B * 64) {
        const int b = idx / 64, n = idx % 64;
        const float v = a2_dot(a.g1d + b * 128, P + o[S_GE3W] + n * 128, 128, P[o[S_GE3B] + n]);
        a.g2[idx] = v;
        a.cat[b * 80 + 16 + n] = v;
      }
      if (idx < B * 16) a.cat[(idx / 16) * 80 + idx % 16] = a.f[idx];
      break;
    case 4:
      if (idx < B * 32) {
        const int b = idx / 32, n = idx % 32;
        a.hp0[idx] = relu_nan(a2_dot(a.cat + b * 80, P + o[S_AP0W] + n * 80, 80, P[o[S_AP0B] + n]));
      }
      break;
    default:
      if (idx < B) a.s[idx] = a2_sigmoid(a2_dot(a.hp0 + idx * 32, P + o[S_AP2W], 32, P[o[S_AP2B]]));
  }
}

// The whole head of one clip per block (B blocks): the six stages above in order, each output computed by one thread
// with a2_dot's arithmetic (k in order) -- bit-identical to the per-stage launches -- with the stage inputs read from
// LDS; the saved activations still go to global memory for the backward.  One launch instead of six dependent ones.
__global__ __launch_bounds__(256) void a2_head_fwd_clip_kernel(A2HeadArgs a) {
  const int b = blockIdx.x, t = threadIdx.x;
  const float* P = a.P;
  const int64_t* o = a.off;
  __shared__ float sf[16], shc0[32], sadj[256], sg1d[128], scat[80], shp0[32];
  if (a.pooled) {
    // f = Dropout(fc(pooled)): output n by the 16 lanes of a row group (each 256 of the 4096 inputs, 16-B loads),
    // summed by butterflies within the group; the keyed dropout as dense_fwd's epilogue (row = clip0 + b, col = n)
    const int n = t >> 4, l = t & 15;
    const float* w = P + o[S_FCW] + (int64_t)n * 4096;
    const float* x = a.pooled + (int64_t)b * 4096;
    float acc = 0.f;
#pragma unroll 4
    for (int k = 4 * l; k < 4096; k += 64) {
      const f32x4 wv = *reinterpret_cast<const f32x4*>(w + k), xv = *reinterpret_cast<const f32x4*>(x + k);
      acc = fmaf(wv[0], xv[0], acc);
      acc = fmaf(wv[1], xv[1], acc);
      acc = fmaf(wv[2], xv[2], acc);
      acc = fmaf(wv[3], xv[3], acc);
    }
#pragma unroll
    for (int m = 8; m >= 1; m >>= 1) acc += __shfl_xor(acc, m, 16);
    if (l == 0) {
      float v = acc + P[o[S_FCB] + n];
      if (a.training) v = rng_u24(a.h_fc, (uint64_t)(a.clip0 + b), (uint64_t)n) >= a.thr_fc ? v * a.s_fc : 0.f;
      a.f[b * 16 + n] = v;
      sf[n] = scat[n] = v;
    }
  } else if (t < 16) {
    sf[t] = scat[t] = a.f[b * 16 + t];
  }
  __syncthreads();
  if (t < 32) shc0[t] = a.hc0[b * 32 + t] = relu_nan(a2_dot(sf, P + o[S_CN0W] + t * 16, 16, P[o[S_CN0B] + t]));
  __syncthreads();
  {
    const float sg = a2_sigmoid(a2_dot(shc0, P + o[S_CN2W] + t * 32, 32, P[o[S_CN2B] + t]));
    a.sig[b * 256 + t] = sg;
    sadj[t] = a.adj[b * 256 + t] = (t / 16 == t % 16) ? sg * 0.f : sg;  // * (1 - eye)
  }
  __syncthreads();
  if (t < 128) {
    float v = relu_nan(a2_dot(sadj, P + o[S_GE0W] + t * 256, 256, P[o[S_GE0B] + t]));
    a.g1[b * 128 + t] = v;
    if (a.training) v = rng_u24(a.h_graph, (uint64_t)(a.clip0 + b), (uint64_t)t) >= a.thr_graph ? v * a.s_graph : 0.f;
    sg1d[t] = a.g1d[b * 128 + t] = v;
  }
  __syncthreads();
  if (t < 64) {
    const float v = a2_dot(sg1d, P + o[S_GE3W] + t * 128, 128, P[o[S_GE3B] + t]);
    a.g2[b * 64 + t] = v;
    scat[16 + t] = a.cat[b * 80 + 16 + t] = v;
  }
  if (t < 16) a.cat[b * 80 + t] = sf[t];
  __syncthreads();
  if (t < 32) shp0[t] = a.hp0[b * 32 + t] = relu_nan(a2_dot(scat, P + o[S_AP0W] + t * 80, 80, P[o[S_AP0B] + t]));
  __syncthreads();
  if (t == 0) a.s[b] = a2_sigmoid(a2_dot(shp0, P + o[S_AP2W], 32, P[o[S_AP2B]]));
}

// compute_improved_loss (a2:135-205) on the saved scores / adjacency, plus d total / d scores and d total / d adj, as
// four launches: a2_loss_kernel (pseudo labels, focal BCE and d scores, mean adjacency, edge count: one block),
// a2_pairs_kernel (one wave per clip pair i < j: mean |A_i - A_j| over the 256 entries, fixed order),
// a2_loss_fin_kernel (the pair mean in fixed order, the loss terms) and a2_dadj_kernel (d total / d adj, one thread per
// entry)
__global__ __launch_bounds__(512) void a2_loss_kernel(A2HeadArgs a) {
  const int B = a.B;
  __shared__ float sh[512];
  __shared__ float sh2[512];
  const int t = threadIdx.x;
  if (t < B) {
    const float u = (float)rng_u24(a.h_pseudo, (uint64_t)(a.clip0 + t), 0) * (1.0f / 16777216.0f);
    a.pseudo[t] = u > 0.95f ? 1.f : 0.f;
  }
  __syncthreads();
  // focal BCE (mean over the batch) and its derivative w.r.t. the scores
  float focal = 0.f;
  for (int b = t; b < B; b += blockDim.x) {
    const float sv = a.s[b], p = a.pseudo[b];
    const float ce = -(p * fmaxf(logf(sv), -100.f) + (1.f - p) * fmaxf(log1pf(-sv), -100.f));
    const float pt = expf(-ce);
    focal += 0.25f * (1.f - pt) * (1.f - pt) * ce;
    const float dfdce = 0.25f * ((1.f - pt) * (1.f - pt) + 2.f * (1.f - pt) * pt * ce);
    const float dce = (sv - p) / fmaxf((1.f - sv) * sv, 1e-12f);
    a.d_s[b] = dfdce * dce / (float)B;
  }
  // mean adjacency, sparsity counts
  float acyc_part = 0.f, cnt = 0.f;
  for (int e = t; e < 256; e += blockDim.x) {
    float m = 0.f, mt = 0.f;
    const int i = e / 16, j = e % 16, et = j * 16 + i;
    for (int b = 0; b < B; ++b) {
      m += a.adj[b * 256 + e];
      mt += a.adj[b * 256 + et];
    }
    m /= (float)B;
    mt /= (float)B;
    a.red[e] = mt;  // mean_adj^T, for the acyclicity gradient
    acyc_part += m * mt;
  }
  for (int idx = t; idx < B * 256; idx += blockDim.x) cnt += a.adj[idx] > 0.1f ? 1.f : 0.f;
  sh[t] = focal + 0.f;
  sh2[t] = acyc_part;
  __syncthreads();
  for (int k = blockDim.x / 2; k > 0; k >>= 1) {
    if (t < k) {
      sh[t] += sh[t + k];
      sh2[t] += sh2[t + k];
    }
    __syncthreads();
  }
  const float focal_sum = sh[0], acyc = sh2[0];
  __syncthreads();
  sh[t] = cnt;
  __syncthreads();
  for (int k = blockDim.x / 2; k > 0; k >>= 1) {
    if (t < k) sh[t] += sh[t + k];
    __syncthreads();
  }
  if (t == 0) {
    a.lsc[0] = focal_sum;
    a.lsc[1] = acyc;
    a.lsc[2] = sh[0];
  }
}

__global__ __launch_bounds__(64) void a2_pairs_kernel(A2HeadArgs a) {
  const int B = a.B, i = blockIdx.x / B, j = blockIdx.x % B, lane = threadIdx.x;
  if (!(i < j && a.pseudo[i] == 0.f && a.pseudo[j] == 0.f)) {
    if (lane == 0) a.pairs[blockIdx.x] = 0.f;
    return;
  }
  float d = 0.f;
  for (int e = lane; e < 256; e += 64) d += fabsf(a.adj[i * 256 + e] - a.adj[j * 256 + e]);
  d = wave_sum(d);
  if (lane == 0) a.pairs[blockIdx.x] = d / 256.f;
}

__global__ __launch_bounds__(512) void a2_loss_fin_kernel(A2HeadArgs a) {
  const int B = a.B, t = threadIdx.x;
  __shared__ float sh[512];
  __shared__ int nn_s;
  if (t == 0) {
    int nn = 0;
    for (int b = 0; b < B; ++b) nn += a.pseudo[b] == 0.f;
    nn_s = nn;
  }
  float pd = 0.f;
  for (int q = t; q < B * B; q += blockDim.x) pd += a.pairs[q];
  sh[t] = pd;
  __syncthreads();
  for (int k = blockDim.x / 2; k > 0; k >>= 1) {
    if (t < k) sh[t] += sh[t + k];
    __syncthreads();
  }
  if (t == 0) {
    const int nn = nn_s, np = nn > 1 ? nn * (nn - 1) / 2 : 0;
    const float avg = np > 0 ? sh[0] / (float)np : 0.f;
    const float consistency = np > 0 ? fabsf(avg - 0.1f) : 0.f;
    const float csign = np > 0 ? (avg > 0.1f ? 1.f : (avg < 0.1f ? -1.f : 0.f)) : 0.f;
    const float focal_sum = a.lsc[0], acyc = a.lsc[1], edges = a.lsc[2];
    a.lsc[3] = csign;
    a.lsc[4] = (float)np;
    const float anomaly = focal_sum / (float)B;
    const float ratio = edges / (float)(B * 256);
    const float sparsity = fabsf(ratio - 0.3f);
    float structure = 0.f;
    if (edges < 10.f) structure = (10.f - edges) * 0.01f;
    else if (edges > 40.f) structure = (edges - 40.f) * 0.01f;
    const float total = anomaly + 0.01f * acyc + 0.001f * sparsity + 0.01f * consistency + 0.01f * structure;
    float* L = a.losses;
    L[0] = total; L[1] = anomaly; L[2] = acyc; L[3] = sparsity; L[4] = consistency; L[5] = structure;
    L[6] = edges; L[7] = ratio; L[8] = 0.f;
    L[9] = isnan(total) ? 0.f : 2.f;
  }
}

// d total / d adj: 0.01 * d acyc + 0.01 * d consistency  (sparsity / structure carry no gradient)
__global__ __launch_bounds__(256) void a2_dadj_kernel(A2HeadArgs a) {
  const int B = a.B, idx = blockIdx.x * 256 + threadIdx.x;
  if (idx >= B * 256) return;
  const int b = idx / 256, e = idx % 256;
  const float csign = a.lsc[3], np = a.lsc[4];
  float g = 0.01f * 2.f * a.red[e] / (float)B;
  if (np > 0.f && a.pseudo[b] == 0.f) {
    float sg = 0.f;
    for (int j = 0; j < B; ++j) {
      if (j == b || a.pseudo[j] != 0.f) continue;
      const float d = a.adj[idx] - a.adj[j * 256 + e];
      sg += d > 0.f ? 1.f : (d < 0.f ? -1.f : 0.f);
    }
    g += 0.01f * csign * sg / (np * 256.f);
  }
  a.d_adj[idx] = g;
}


struct A2HeadBwdArgs {
  A2HeadArgs f;
  const float* d_s;    // [B]
  const float* d_adj;  // [B][256] (nullable)
  const float* d_f;    // [B][16] external features grad (nullable)
  float* G;            // grads base
  float *dz_ap2, *dz_ap0, *dg2, *dz_ge0, *dz_cn2, *dz_cn0, *dfeat;  // scratch; dfeat = grad w.r.t. fc output
  uint64_t h_fc;
  uint32_t thr_fc;
  float s_fc;
  // per-clip path: fc's backward inside the head launches (pooled: the fc input; dpooled: its gradient, written by
  // a2_head_bwd_clip_kernel; nseg 7: fc's weight / bias grads as the 7th segment of stage 6); null / 6: dense GEMMs
  const float* pooled;
  float* dpooled;
  int nseg;
};

// Backward stages 0-5 of one clip per block (B blocks), the per-stage launches' arithmetic in the same order
// (bit-identical), stage inputs from LDS, every stage's output also written out for the weight-gradient launch (stage 6)
__global__ __launch_bounds__(256) void a2_head_bwd_clip_kernel(A2HeadBwdArgs a) {
  const A2HeadArgs& f = a.f;
  const int b = blockIdx.x, t = threadIdx.x;
  const float* P = f.P;
  const int64_t* o = f.off;
  __shared__ float sap0[32], sdg2[64], sdfeat[16], sge0[128], scn2[256], scn0[32];
  if (t < 32) {  // predictor: s = sigmoid(W2 hp0 + b), hp0 = relu(W0 cat + b)
    const float dz2 = a.d_s[b] * f.s[b] * (1.f - f.s[b]);
    if (t == 0) a.dz_ap2[b] = dz2;
    sap0[t] = a.dz_ap0[b * 32 + t] = f.hp0[b * 32 + t] > 0.f ? dz2 * P[o[S_AP2W] + t] : 0.f;
  }
  __syncthreads();
  if (t < 80) {
    float d = 0.f;
    for (int k = 0; k < 32; ++k) d = fmaf(sap0[k], P[o[S_AP0W] + k * 80 + t], d);
    if (t < 16) sdfeat[t] = d + (a.d_f ? a.d_f[b * 16 + t] : 0.f);
    else sdg2[t - 16] = a.dg2[b * 64 + t - 16] = d;
  }
  __syncthreads();
  if (t < 128) {  // graph encoder: g2 = W3 g1d + b; g1d = drop(relu(W0 adj + b))
    float d = 0.f;
    for (int k = 0; k < 64; ++k) d = fmaf(sdg2[k], P[o[S_GE3W] + k * 128 + t], d);
    if (f.training) d = rng_u24(f.h_graph, (uint64_t)(f.clip0 + b), (uint64_t)t) >= f.thr_graph ? d * f.s_graph : 0.f;
    sge0[t] = a.dz_ge0[b * 128 + t] = f.g1[b * 128 + t] > 0.f ? d : 0.f;
  }
  __syncthreads();
  {  // d adj -> d sig (zero diagonal) -> dz_cn2
    float d = a.d_adj ? a.d_adj[b * 256 + t] : 0.f;
    for (int k = 0; k < 128; ++k) d = fmaf(sge0[k], P[o[S_GE0W] + k * 256 + t], d);
    const float sg = f.sig[b * 256 + t];
    scn2[t] = a.dz_cn2[b * 256 + t] = (t / 16 == t % 16) ? 0.f : d * sg * (1.f - sg);
  }
  __syncthreads();
  if (t < 32) {
    float d = 0.f;
    for (int e = 0; e < 256; ++e) d = fmaf(scn2[e], P[o[S_CN2W] + e * 32 + t], d);
    scn0[t] = a.dz_cn0[b * 32 + t] = f.hc0[b * 32 + t] > 0.f ? d : 0.f;
  }
  __syncthreads();
  if (t < 16) {  // d features (fc output after dropout) += W_cn0^T dz_cn0, then the fc dropout backward
    float d = sdfeat[t];
    for (int k = 0; k < 32; ++k) d = fmaf(scn0[k], P[o[S_CN0W] + k * 16 + t], d);
    if (f.training) d = rng_u24(a.h_fc, (uint64_t)(f.clip0 + b), (uint64_t)t) >= a.thr_fc ? d * a.s_fc : 0.f;
    a.dfeat[b * 16 + t] = d;
    sdfeat[t] = d;
  }
  if (a.dpooled) {  // d pooled = W_fc^T d features (16-term dots, 16 of the 4096 inputs per thread)
    __syncthreads();
    const float* W = P + o[S_FCW];
#pragma unroll 4
    for (int k = t; k < 4096; k += 256) {
      float acc = 0.f;
#pragma unroll
      for (int n = 0; n < 16; ++n) acc = fmaf(sdfeat[n], W[n * 4096 + k], acc);
      a.dpooled[b * 4096 + k] = acc;
    }
  }
}

// backward stage st (the forward's mirror): 0 predictor output + anomaly_predictor.0 pre-activation grads, 1 d cat ->
// d g2 and the predictor's share of d features, 2 graph_encoder.0 pre-activation grads (dropout, ReLU), 3 d adj (graph
// encoder + loss) -> causal_net.2 pre-activation grads, 4 causal_net.0 pre-activation grads, 5 d features (fc output)
// incl. the fc dropout, 6 every head weight / bias grad (fixed-order sums over the batch, one thread per entry)
constexpr int A2_BWD_OUT[6] = {32, 80, 128, 256, 32, 16};
struct A2WSeg {
  int w, bias, N, K;
};
constexpr A2WSeg A2_WSEGS[7] = {{S_AP2W, S_AP2B, 1, 32},     {S_AP0W, S_AP0B, 32, 80},   {S_GE3W, S_GE3B, 64, 128},
                                {S_GE0W, S_GE0B, 128, 256}, {S_CN2W, S_CN2B, 256, 32}, {S_CN0W, S_CN0B, 32, 16},
                                {S_FCW, S_FCB, 16, 4096}};
constexpr int A2_WG_TOTAL = 1 * 33 + 32 * 81 + 64 * 129 + 128 * 257 + 256 * 33 + 32 * 17;
constexpr int A2_WG_TOTAL_FC = A2_WG_TOTAL + 16 * 4097;

__global__ __launch_bounds__(256) void a2_head_bwd_kernel(A2HeadBwdArgs a, int st) {
  const A2HeadArgs& f = a.f;
  const int B = f.B, idx = blockIdx.x * 256 + threadIdx.x;
  const float* P = f.P;
  const int64_t* o = f.off;
  switch (st) {
    case 0:  // predictor: s = sigmoid(W2 hp0 + b), hp0 = relu(W0 cat + b)
      if (idx < B * 32) {
        const int b = idx / 32, k = idx % 32;
        const float dz2 = a.d_s[b] * f.s[b] * (1.f - f.s[b]);
        if (k == 0) a.dz_ap2[b] = dz2;
        a.dz_ap0[idx] = f.hp0[idx] > 0.f ? dz2 * P[o[S_AP2W] + k] : 0.f;
      }
      break;
    case 1:
      if (idx < B * 80) {
        const int b = idx / 80, c = idx % 80;
        float d = 0.f;
        for (int k = 0; k < 32; ++k) d = fmaf(a.dz_ap0[b * 32 + k], P[o[S_AP0W] + k * 80 + c], d);
        if (c < 16) a.dfeat[b * 16 + c] = d + (a.d_f ? a.d_f[b * 16 + c] : 0.f);
        else a.dg2[b * 64 + c - 16] = d;
      }
      break;
    case 2:  // graph encoder: g2 = W3 g1d + b; g1d = drop(relu(W0 adj + b))
      if (idx < B * 128) {
        const int b = idx / 128, n = idx % 128;
        float d = 0.f;
        for (int k = 0; k < 64; ++k) d = fmaf(a.dg2[b * 64 + k], P[o[S_GE3W] + k * 128 + n], d);
        if (f.training) d = rng_u24(f.h_graph, (uint64_t)(f.clip0 + b), (uint64_t)n) >= f.thr_graph ? d * f.s_graph : 0.f;
        a.dz_ge0[idx] = f.g1[idx] > 0.f ? d : 0.f;
      }
      break;
    case 3:  // d adj -> d sig (zero diagonal) -> dz_cn2
      if (idx < B * 256) {
        const int b = idx / 256, e = idx % 256;
        float d = a.d_adj ? a.d_adj[idx] : 0.f;
        for (int k = 0; k < 128; ++k) d = fmaf(a.dz_ge0[b * 128 + k], P[o[S_GE0W] + k * 256 + e], d);
        const float sg = f.sig[idx];
        a.dz_cn2[idx] = (e / 16 == e % 16) ? 0.f : d * sg * (1.f - sg);
      }
      break;
    case 4:
      if (idx < B * 32) {
        const int b = idx / 32, k = idx % 32;
        float d = 0.f;
        for (int e = 0; e < 256; ++e) d = fmaf(a.dz_cn2[b * 256 + e], P[o[S_CN2W] + e * 32 + k], d);
        a.dz_cn0[idx] = f.hc0[idx] > 0.f ? d : 0.f;
      }
      break;
    case 5:  // d features (fc output after dropout) += W_cn0^T dz_cn0, then the fc dropout backward
      if (idx < B * 16) {
        const int b = idx / 16, c = idx % 16;
        float d = a.dfeat[idx];
        for (int k = 0; k < 32; ++k) d = fmaf(a.dz_cn0[b * 32 + k], P[o[S_CN0W] + k * 16 + c], d);
        if (f.training) d = rng_u24(a.h_fc, (uint64_t)(f.clip0 + b), (uint64_t)c) >= a.thr_fc ? d * a.s_fc : 0.f;
        a.dfeat[idx] = d;
      }
      break;
    default: {
      int r = idx, s = 0;
      for (; s < a.nseg; ++s) {
        const int len = A2_WSEGS[s].N * (A2_WSEGS[s].K + 1);
        if (r < len) break;
        r -= len;
      }
      if (s >= a.nseg) break;
      const A2WSeg g = A2_WSEGS[s];
      const float* dz = s == 0 ? a.dz_ap2 : s == 1 ? a.dz_ap0 : s == 2 ? a.dg2 : s == 3 ? a.dz_ge0 : s == 4 ? a.dz_cn2
                        : s == 5 ? a.dz_cn0 : a.dfeat;
      const float* x = s == 0 ? f.hp0 : s == 1 ? f.cat : s == 2 ? f.g1d : s == 3 ? f.adj : s == 4 ? f.hc0
                       : s == 5 ? f.f : a.pooled;
      const int n = r / (g.K + 1), k = r % (g.K + 1);
      float acc = 0.f;
      if (k < g.K) {
        for (int b = 0; b < B; ++b) acc = fmaf(dz[b * g.N + n], x[b * g.K + k], acc);
        a.G[o[g.w] + n * g.K + k] = acc;
      } else {
        for (int b = 0; b < B; ++b) acc += dz[b * g.N + n];
        a.G[o[g.bias] + n] = acc;
      }
    }
  }
}

// ------------------------------------------------------------------ conv3d_1 (3 -> 16, k3, stride (1, 2, 2), p1) direct
// (knob "a2_direct", latched per plan; 0: im2col + GEMM).  With 3 input channels the im2col matrix (K = 81) is 6.75x
// the clip and the GEMM runs 16-wide tiles, so the first conv and its weight gradient run on the VALU from the clip
// itself (NCDHW), over 2 x 8 x 16-voxel output tiles whose 3 x 4 x 17 x 33 input halo is staged in LDS (coalesced
// rows):
//   a2_conv1_fwd   one thread per output voxel: its 81 halo inputs x the [81][16] weights (LDS broadcast rows),
//                  + bias, ReLU, 16 channels out (NDHWC)
//   a2_conv1_wgrad thread (co, tap group) owns up to 6 of the 82 (ci, tap) / bias sums and walks the tile's 256 voxels
//                  (the gated dY tile in LDS beside the halo); per-block slabs summed in fixed order by
//                  a2_conv1_wgrad_reduce (64 lanes per entry)
constexpr int A2C1_TAPS = 81, A2T_D = 2, A2T_H = 8, A2T_W = 16;
constexpr int A2H_D = A2T_D + 2, A2H_H = 2 * A2T_H + 1, A2H_W = 2 * A2T_W + 1, A2_HALO = A2H_D * A2H_H * A2H_W;

struct A2Tiles {
  int T, H, W, OH, OW, td, th, tw;
  int64_t n;
  __host__ __device__ A2Tiles(int B, int T_, int H_, int W_) : T(T_), H(H_), W(W_) {
    OH = (H - 1) / 2 + 1;
    OW = (W - 1) / 2 + 1;
    td = (T + A2T_D - 1) / A2T_D;
    th = (OH + A2T_H - 1) / A2T_H;
    tw = (OW + A2T_W - 1) / A2T_W;
    n = (int64_t)B * td * th * tw;
  }
};

// the tile's input halo xs[ci][hd][hh][hw] = x[b][ci][d0 - 1 + hd][2 h0 - 1 + hh][2 w0 - 1 + hw] (0 outside)
__device__ __forceinline__ void a2_stage_halo(float* xs, const float* __restrict__ x, const A2Tiles& g, int64_t b,
                                              int d0, int h0, int w0) {
  for (int i = threadIdx.x; i < 3 * A2H_D * A2H_H * A2H_W; i += 256) {
    const int hw = i % A2H_W, r = i / A2H_W, hh = r % A2H_H, r2 = r / A2H_H, hd = r2 % A2H_D, ci = r2 / A2H_D;
    const int id = d0 - 1 + hd, ih = 2 * h0 - 1 + hh, iw = 2 * w0 - 1 + hw;
    float v = 0.f;
    if (id >= 0 && id < g.T && ih >= 0 && ih < g.H && iw >= 0 && iw < g.W)
      v = x[(((b * 3 + ci) * g.T + id) * g.H + ih) * (int64_t)g.W + iw];
    xs[i] = v;
  }
}

// The per-step weight images of the direct path in one launch: conv3d_2 / conv3d_3's GEMM and parity-class images
// (conv3s2_prep_elem) and conv3d_1's [ci*27 + tap][co] rows + its bias (w1t: a2_conv1_fwd_kernel copies them into LDS
// without transposing).
struct A2Prep {
  const float* w[3];
  float *wk[3], *wc[3];
  int Co[3], Ci[3];
  int64_t end[3];  // prefix sums of the element counts: conv3d_1 (16 * 81 + 16), conv3d_2, conv3d_3
  const float* b1;
  float* w1t;
};
__global__ __launch_bounds__(256) void a2_prep_kernel(const A2Prep p) {
  for (int64_t i = blockIdx.x * 256ll + threadIdx.x; i < p.end[2]; i += (int64_t)gridDim.x * 256) {
    if (i < p.end[0]) {
      if (i < 16 * A2C1_TAPS) {
        const int co = (int)(i / A2C1_TAPS), j = (int)(i % A2C1_TAPS);
        p.w1t[j * 16 + co] = p.w[0][i];
      } else {
        p.w1t[i] = p.b1[i - 16 * A2C1_TAPS];
      }
    } else {
      const int s = i < p.end[1] ? 1 : 2;
      conv3s2_prep_elem(p.w[s], p.Co[s], p.Ci[s], p.wk[s], p.wc[s], i - p.end[s - 1]);
    }
  }
}

__global__ __launch_bounds__(256) void a2_conv1_fwd_kernel(const float* __restrict__ x, int B, int T, int H, int W,
                                                           const float* __restrict__ w1t, float* __restrict__ y) {
  __shared__ __attribute__((aligned(16))) float ws[A2C1_TAPS + 1][16];  // [ci*27 + tap][co], then the bias row
  __shared__ float xs[3 * A2_HALO];
  __shared__ float os[256 * 17];
  for (int i = threadIdx.x; i < 16 * (A2C1_TAPS + 1); i += 256) ws[i / 16][i % 16] = w1t[i];
  const A2Tiles g(B, T, H, W);
  const int v = threadIdx.x, vd = v / (A2T_H * A2T_W), vh = (v / A2T_W) % A2T_H, vw = v % A2T_W;
  for (int64_t tile = blockIdx.x; tile < g.n; tile += gridDim.x) {
    const int bw = (int)(tile % g.tw);
    int64_t r = tile / g.tw;
    const int bh = (int)(r % g.th);
    r /= g.th;
    const int bd = (int)(r % g.td);
    const int64_t b = r / g.td;
    const int d0 = bd * A2T_D, h0 = bh * A2T_H, w0 = bw * A2T_W;
    __syncthreads();
    a2_stage_halo(xs, x, g, b, d0, h0, w0);
    __syncthreads();
    f32x4 acc[4];  // (voxels past the volume compute on zero halo and are not stored)
#pragma unroll
    for (int q = 0; q < 4; ++q) acc[q] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ci = 0; ci < 3; ++ci)
#pragma unroll
      for (int t = 0; t < 27; ++t) {
        const float xv = xs[((ci * A2H_D + vd + t / 9) * A2H_H + 2 * vh + (t / 3) % 3) * A2H_W + 2 * vw + t % 3];
#pragma unroll
        for (int q = 0; q < 4; ++q) {  // (LDS broadcast reads; weights through the scalar path measured 3.6x slower:
                                       // the waits on the scalar loads are exposed)
          const f32x4 wv = *reinterpret_cast<const f32x4*>(&ws[ci * 27 + t][4 * q]);
#pragma unroll
          for (int e = 0; e < 4; ++e) acc[q][e] = fmaf(xv, wv[e], acc[q][e]);
        }
      }
    // (through LDS: a voxel row of the output is 64 B, so per-voxel stores would leave every store instruction at a
    // 64-B lane stride; the tile's W-runs of 16 voxels x 16 channels = 1 KB are written back contiguous)
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
      for (int e = 0; e < 4; ++e) os[v * 17 + 4 * q + e] = relu_nan(acc[q][e] + ws[A2C1_TAPS][4 * q + e]);
    __syncthreads();
    for (int i = threadIdx.x; i < 256 * 4; i += 256) {  // (voxel, float4) in tile order: W-runs contiguous in y
      const int vv = i >> 2, c4 = (i & 3) * 4;
      const int ud = vv / (A2T_H * A2T_W), uh = (vv / A2T_W) % A2T_H, uw = vv % A2T_W;
      const int dd = d0 + ud, hh = h0 + uh, ww = w0 + uw;
      if (dd < T && hh < g.OH && ww < g.OW) {
        const f32x4 o4 = {os[vv * 17 + c4], os[vv * 17 + c4 + 1], os[vv * 17 + c4 + 2], os[vv * 17 + c4 + 3]};
        *reinterpret_cast<f32x4*>(y + (((b * T + dd) * g.OH + hh) * (int64_t)g.OW + ww) * 16 + c4) = o4;
      }
    }
  }
}

// thread = one (ci, tap) pair j = tid % 82 (pair 81 = the bias) x all 16 output channels, over one of three voxel
// groups vg = tid / 82 (voxels vg, vg + 3, ...; threads 246..255 idle): per voxel four 16-B reads of its dY row (the
// same row for every lane of a group: broadcast) and one halo read feed 16 FMAs (was 8 FMAs per 3 reads with 4 channels
// x 2 pairs per thread, a third of the pair slots empty); the three group sums are added in a fixed order
__global__ __launch_bounds__(256) void a2_conv1_wgrad_kernel(const float* __restrict__ dA, const float* __restrict__ x,
                                                             int B, int T, int H, int W, float* __restrict__ slab) {
  __shared__ float xs[3 * A2_HALO];
  __shared__ __attribute__((aligned(16))) float as[256][16];
  const A2Tiles g(B, T, H, W);
  const int tid = threadIdx.x, j = tid % (A2C1_TAPS + 1), vg = tid / (A2C1_TAPS + 1);
  int off = -1;  // the pair's halo offset at voxel (0, 0, 0); -1: the bias pair
  if (j < A2C1_TAPS) {
    const int ci = j / 27, t = j % 27;
    off = ((ci * A2H_D + t / 9) * A2H_H + (t / 3) % 3) * A2H_W + t % 3;
  }
  f32x4 acc[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) acc[k] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int64_t tile = blockIdx.x; tile < g.n; tile += gridDim.x) {
    const int bw = (int)(tile % g.tw);
    int64_t r = tile / g.tw;
    const int bh = (int)(r % g.th);
    r /= g.th;
    const int bd = (int)(r % g.td);
    const int64_t b = r / g.td;
    const int d0 = bd * A2T_D, h0 = bh * A2T_H, w0 = bw * A2T_W;
    __syncthreads();
    a2_stage_halo(xs, x, g, b, d0, h0, w0);
    {  // the gated dY rows of the tile's voxels (zero outside the volume)
      const int vd = tid / (A2T_H * A2T_W), vh = (tid / A2T_W) % A2T_H, vw = tid % A2T_W;
      const int d = d0 + vd, oh = h0 + vh, ow = w0 + vw;
      const bool ok = d < T && oh < g.OH && ow < g.OW;
      const float* row = dA + (((b * T + d) * g.OH + oh) * (int64_t)g.OW + ow) * 16;
#pragma unroll
      for (int k = 0; k < 4; ++k)
        *reinterpret_cast<f32x4*>(&as[tid][4 * k]) =
            ok ? *reinterpret_cast<const f32x4*>(row + 4 * k) : f32x4{0.f, 0.f, 0.f, 0.f};
    }
    __syncthreads();
    if (vg < 3) {
      for (int v = vg; v < 256; v += 3) {
        const int vd = v / (A2T_H * A2T_W), vh = (v / A2T_W) % A2T_H, vw = v % A2T_W;
        const int base = (vd * A2H_H + 2 * vh) * A2H_W + 2 * vw;
        const float xv = xs[max(off, 0) + base];
        const float xm = off < 0 ? 1.f : xv;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const f32x4 a = *reinterpret_cast<const f32x4*>(&as[v][4 * k]);
#pragma unroll
          for (int e = 0; e < 4; ++e) acc[k][e] = fmaf(a[e], xm, acc[k][e]);
        }
      }
    }
  }
  // the three voxel groups' sums, fixed order (rows vg * 82 + j of the dY staging array)
  __syncthreads();
  if (vg < 3)
#pragma unroll
    for (int k = 0; k < 4; ++k) *reinterpret_cast<f32x4*>(&as[tid][4 * k]) = acc[k];
  __syncthreads();
  if (vg == 0) {
#pragma unroll
    for (int c = 0; c < 16; ++c) {
      const float t = (as[j][c] + as[A2C1_TAPS + 1 + j][c]) + as[2 * (A2C1_TAPS + 1) + j][c];
      slab[((int64_t)blockIdx.x * 16 + c) * (A2C1_TAPS + 1) + j] = t;
    }
  }
}

// dW[co][ci*27 + tap] / db[co] = sum over the S slabs: 16 consecutive entries x 16 slab lanes per block (lane l adds
// slabs l, l + 16, ... in order, 8 loads in flight), the lane sums combined by a fixed tree
__global__ __launch_bounds__(256) void a2_conv1_wgrad_reduce_kernel(const float* __restrict__ slab, int S,
                                                                    float* __restrict__ dW, float* __restrict__ db) {
  constexpr int NE = 16 * (A2C1_TAPS + 1);
  __shared__ float red[16][17];
  const int e = threadIdx.x & 15, sl = threadIdx.x >> 4, i = blockIdx.x * 16 + e;
  float v = 0.f;
  if (i < NE) {
#pragma unroll 8
    for (int z = sl; z < S; z += 16) v += slab[(int64_t)z * NE + i];
  }
  red[sl][e] = v;
  __syncthreads();
  if (sl == 0 && i < NE) {
    float t[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) t[k] = red[2 * k][e] + red[2 * k + 1][e];
#pragma unroll
    for (int k = 0; k < 4; ++k) t[k] = t[2 * k] + t[2 * k + 1];
    const float r = (t[0] + t[1]) + (t[2] + t[3]);
    const int co = i / (A2C1_TAPS + 1), j = i % (A2C1_TAPS + 1);
    if (j < A2C1_TAPS) dW[co * A2C1_TAPS + j] = r;
    else db[co] = r;
  }
}

__global__ void relu_gate_kernel(float* __restrict__ d, const float* __restrict__ y, int64_t n) {
  for (int64_t i = blockIdx.x * 256ll + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256)
    if (!(y[i] > 0.f)) d[i] = 0.f;
}
static int relu_gate(float* d, const float* y, int64_t n, hipStream_t st) {
  hipLaunchKernelGGL(relu_gate_kernel, dim3((unsigned)std::min<int64_t>(cdiv(n, 256), 8192)), dim3(256), 0, st, d, y,
                     n);
  VAD_LAUNCH_CHECK();
  return 0;
}

// ------------------------------------------------------------------ AdamW with clip_grad_norm_(max_norm)
struct A2SlotTab {
  int64_t off[A2_NSLOT], numel[A2_NSLOT];
};
// per-slot squared sums in A2_SQ_CHUNKS fixed strided parts (block (slot, part)); a2_opt_prepare adds the parts in
// order and takes each slot's norm (torch's per-tensor norm, then the norm of norms)
constexpr int A2_SQ_CHUNKS = 16;
__global__ __launch_bounds__(256) void a2_sqsum_kernel(const float* __restrict__ g, A2SlotTab t, double* sqp) {
  const int s = blockIdx.x;
  __shared__ double red[256];
  double acc = 0.0;
  for (int64_t i = blockIdx.y * 256ll + threadIdx.x; i < t.numel[s]; i += 256ll * A2_SQ_CHUNKS) {
    const float v = g[t.off[s] + i];
    acc += (double)v * (double)v;
  }
  red[threadIdx.x] = acc;
  __syncthreads();
  for (int k = 128; k > 0; k >>= 1) {
    if (threadIdx.x < k) red[threadIdx.x] += red[threadIdx.x + k];
    __syncthreads();
  }
  if (threadIdx.x == 0) sqp[s * A2_SQ_CHUNKS + blockIdx.y] = red[0];
}
// ctrl: [0] step?, [1] clip coefficient, [2] -lr/bc1, [3] sqrt(bc2), [4] 1 - lr*wd
__global__ void a2_opt_prepare_kernel(const double* sqp, float* losses, int32_t* steps, float lr, float b1, float b2,
                                      float wd, float max_norm, float* ctrl, float* user_losses) {
  if (threadIdx.x != 0) return;
  ctrl[0] = 0.f;
  if (losses[9] < 1.f) return;
  double tot = 0.0;
  for (int s = 0; s < A2_NSLOT; ++s) {
    double q = 0.0;
    for (int c = 0; c < A2_SQ_CHUNKS; ++c) q += sqp[s * A2_SQ_CHUNKS + c];
    const float nrm = (float)sqrt(q);
    tot += (double)nrm * (double)nrm;
  }
  const float total = (float)sqrt(tot);
  losses[8] = total;
  if (user_losses) user_losses[8] = total;
  ctrl[1] = fminf(1.f, max_norm / (total + 1e-6f));
  const int step = steps[0] + 1;
  for (int s = 0; s < A2_NSLOT; ++s) steps[s] = step;
  const double bc1 = 1.0 - pow((double)b1, step), bc2 = 1.0 - pow((double)b2, step);
  ctrl[2] = (float)(-(double)lr / bc1);
  ctrl[3] = (float)sqrt(bc2);
  ctrl[4] = (float)(1.0 - (double)lr * (double)wd);
  ctrl[0] = 1.f;
}
__global__ __launch_bounds__(256) void a2_adamw_kernel(float* __restrict__ p, const float* __restrict__ g,
                                                       float* __restrict__ m, float* __restrict__ v, int64_t n,
                                                       const float* ctrl, float b1, float b2, float eps) {
  if (ctrl[0] == 0.f) return;
  const float coef = ctrl[1], step_size = ctrl[2], bc2s = ctrl[3], decay = ctrl[4];
  for (int64_t i = blockIdx.x * 256ll + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const float gv = g[i] * coef;
    const float pv = p[i] * decay;  // param.mul_(1 - lr * weight_decay)
    const float mv = m[i] + (1.f - b1) * (gv - m[i]);
    const float vv = fmaf(v[i], b2, (1.f - b2) * gv * gv);
    m[i] = mv;
    v[i] = vv;
    p[i] = fmaf(step_size, mv / (sqrtf(vv) / bc2s + eps), pv);
  }
}

// ------------------------------------------------------------------ the plan
struct A2PlanImpl {
  int B, T, H, W;
  Conv3dGeom g[3];
  int64_t ws_bytes = 0;
  float *params = nullptr, *grads = nullptr, *m = nullptr, *v = nullptr;
  int32_t* steps = nullptr;
  float *cols[3], *y[3], *pooled, *f, *hc0, *sig, *adj, *g1, *g1d, *g2, *cat, *hp0, *s, *losses, *pseudo, *d_s,
      *d_adj, *red, *pairs, *lsc, *dz_ap2, *dz_ap0, *dg2, *dz_ge0, *dz_cn2, *dz_cn0, *dfeat, *dpooled, *dA, *dcols,
      *scratch, *ctrl;
  double* sqp;
  int64_t* off_dev;
  float* xin = nullptr;  // (a2_direct) the forward's clip, kept for conv3d_1's weight gradient
  const float* xsrc = nullptr;  // the clip conv3d_1 reads: xin, or the caller's x itself with option borrow_input
  int borrow_input = 0;  // option: the caller keeps x unchanged until the backward (the fused step): no copy
  // (a2_direct) conv3d_2 / conv3d_3 weight images (conv3s2_prep: [Co][27 Ci] + the 8 parity-class images) and the
  // second input-gradient buffer
  float *wk3[3] = {}, *wc3[3] = {}, *dA2 = nullptr;
  float* w1t = nullptr;  // conv3d_1's [81][16] weight rows + bias (a2_prep_kernel)
  const int direct = g_a2_direct;
  int64_t scratch_floats = 0;
  int training = 1, with_loss = 0;
  uint64_t seed = 0, step = 0;
  int64_t clip0 = 0;

  A2PlanImpl(int B_, int T_, int H_, int W_) : B(B_), T(T_), H(H_), W(W_) {
    Vol5 in{B, 3, T, H, W};
    const int sd[3] = {1, 2, 2};
    for (int s = 0; s < 3; ++s) {
      g[s] = conv3d_geom(in, A2_CO[s], 3, sd[s], 2, 2, 1);
      in = g[s].out();
    }
  }
  float* P(int s) const { return params + a2_offsets().off[s]; }
  float* G(int s) const { return grads + a2_offsets().off[s]; }

  void carve(Ws& w) {
    int64_t max_y = 0, max_dcols = 1;
    xin = direct ? w.take<float>(g[0].in.numel()) : nullptr;
    for (int s = 0; s < 3; ++s) {
      cols[s] = direct ? nullptr : w.take<float>(g[s].rows() * g[s].K());
      if (direct && s > 0) {
        wk3[s] = w.take<float>((int64_t)27 * g[s].in.C * A2_CO[s]);
        wc3[s] = w.take<float>((int64_t)27 * g[s].in.C * A2_CO[s]);
      }
      if (direct && s == 0) w1t = w.take<float>(16 * (A2C1_TAPS + 1));
      y[s] = w.take<float>(g[s].out().numel());
      max_y = std::max(max_y, g[s].out().numel());
      if (s > 0 && !direct) max_dcols = std::max(max_dcols, g[s].rows() * g[s].K());
    }
    const int64_t b = B;
    pooled = w.take<float>(b * 4096);
    f = w.take<float>(b * 16);
    hc0 = w.take<float>(b * 32);
    sig = w.take<float>(b * 256);
    adj = w.take<float>(b * 256);
    g1 = w.take<float>(b * 128);
    g1d = w.take<float>(b * 128);
    g2 = w.take<float>(b * 64);
    cat = w.take<float>(b * 80);
    hp0 = w.take<float>(b * 32);
    s = w.take<float>(b);
    losses = w.take<float>(16);
    pseudo = w.take<float>(b);
    d_s = w.take<float>(b);
    d_adj = w.take<float>(b * 256);
    red = w.take<float>(256);
    pairs = w.take<float>((int64_t)b * b);
    lsc = w.take<float>(8);
    dz_ap2 = w.take<float>(b);
    dz_ap0 = w.take<float>(b * 32);
    dg2 = w.take<float>(b * 64);
    dz_ge0 = w.take<float>(b * 128);
    dz_cn2 = w.take<float>(b * 256);
    dz_cn0 = w.take<float>(b * 32);
    dfeat = w.take<float>(b * 16);
    dpooled = w.take<float>(b * 4096);
    dA = w.take<float>(max_y);
    dA2 = direct ? w.take<float>(max_y) : nullptr;
    dcols = w.take<float>(max_dcols);
    scratch_floats = 8ll << 20;
    scratch = w.take<float>(scratch_floats);
    sqp = w.take<double>(A2_NSLOT * A2_SQ_CHUNKS);
    ctrl = w.take<float>(8);
    off_dev = w.take<int64_t>(A2_NSLOT);
  }

  A2HeadArgs head_args() const {
    A2HeadArgs a{};
    a.B = B;
    a.training = training;
    a.with_loss = with_loss;
    a.clip0 = clip0;
    a.P = params;
    a.off = off_dev;
    a.f = f; a.hc0 = hc0; a.sig = sig; a.adj = adj; a.g1 = g1; a.g1d = g1d; a.g2 = g2; a.cat = cat; a.hp0 = hp0;
    a.s = s;
    a.h_graph = rng_h1(seed, S_A2_DROP_GRAPH, step);
    a.h_pseudo = rng_h1(seed, S_A2_PSEUDO, step);
    a.thr_graph = drop_threshold(0.3);
    a.s_graph = 1.0f / (float)(1.0 - 0.3);
    a.losses = losses;
    a.pseudo = pseudo;
    a.d_s = d_s;
    a.d_adj = d_adj;
    a.red = red;
    a.pairs = pairs;
    a.lsc = lsc;
    a.h_fc = rng_h1(seed, S_A2_DROP_FC, step);
    a.thr_fc = drop_threshold(0.3);
    a.s_fc = 1.0f / (float)(1.0 - 0.3);
    return a;
  }

  int forward(const float* x, hipStream_t st) {
    for (int s3 = 0; s3 < 3; ++s3) {
      if (direct && s3 == 0) {
        const int64_t n = g[0].in.numel();
        if (borrow_input) {
          xsrc = x;
        } else {
          VAD_HIP(hipMemcpyAsync(xin, x, sizeof(float) * n, hipMemcpyDeviceToDevice, st));
          xsrc = xin;
        }
        A2Prep pp{};
        int64_t acc = 16 * (A2C1_TAPS + 1);
        pp.end[0] = acc;
        pp.w[0] = P(S_C1W);
        pp.b1 = P(S_C1B);
        pp.w1t = w1t;
        for (int s = 1; s < 3; ++s) {
          pp.w[s] = P(2 * s);
          pp.wk[s] = wk3[s];
          pp.wc[s] = wc3[s];
          pp.Co[s] = A2_CO[s];
          pp.Ci[s] = g[s].in.C;
          acc += (int64_t)27 * g[s].in.C * A2_CO[s];
          pp.end[s] = acc;
        }
        hipLaunchKernelGGL(a2_prep_kernel, dim3((unsigned)std::min<int64_t>(cdiv(acc, 256), 1024)), dim3(256), 0, st, pp);
        VAD_LAUNCH_CHECK();
        const A2Tiles tl(B, T, H, W);
        hipLaunchKernelGGL(a2_conv1_fwd_kernel, dim3((unsigned)std::min<int64_t>(tl.n, 4096)), dim3(256), 0, st, xsrc, B,
                           T, H, W, w1t, y[0]);
        VAD_LAUNCH_CHECK();
        continue;
      }
      if (direct) {  // conv3d_2 / conv3d_3: implicit GEMM, bias + ReLU in the epilogue (images from a2_prep_kernel)
        const Vol5& in = g[s3].in;
        VAD_TRY(conv3s2_fwd(y[s3 - 1], B, in.D, in.H, in.W, in.C, wk3[s3], P(2 * s3 + 1), A2_CO[s3], 1, y[s3], st,
                            scratch, scratch_floats));
        continue;
      }
      const float* src = s3 == 0 ? x : y[s3 - 1];
      const Strides5 str = s3 == 0 ? ncdhw_strides(g[0].in) : ndhwc_strides(g[s3].in);
      VAD_TRY(im2col3d(src, str, g[s3], nullptr, nullptr, 0, cols[s3], st));
      DenseAct relu;
      relu.relu = 1;
      VAD_TRY(dense_fwd(cols[s3], (int)g[s3].rows(), g[s3].K(), P(2 * s3), P(2 * s3 + 1), A2_CO[s3], y[s3], relu,
                        scratch, scratch_floats, st));
    }
    VAD_TRY(adaptive_avgpool3d_fwd(y[2], nullptr, 0, g[2].out(), 4, 4, 4, pooled, st));
    DenseAct fc;
    if (training) {
      fc.drop = 1;
      fc.h1 = rng_h1(seed, S_A2_DROP_FC, step);
      fc.thr = drop_threshold(0.3);
      fc.dscale = 1.0f / (float)(1.0 - 0.3);
      fc.row0 = clip0;
    }
    A2HeadArgs ha = head_args();
    if (g_a2_head_clip) {  // (fc inside the per-clip kernel: no split-K GEMM + reduce launches)
      ha.pooled = pooled;
      hipLaunchKernelGGL(a2_head_fwd_clip_kernel, dim3((unsigned)B), dim3(256), 0, st, ha);
      VAD_LAUNCH_CHECK();
    } else {
      VAD_TRY(dense_fwd(pooled, B, 4096, P(S_FCW), P(S_FCB), 16, f, fc, scratch, scratch_floats, st));
      for (int s = 0; s < 6; ++s) {
        hipLaunchKernelGGL(a2_head_fwd_kernel, dim3((unsigned)cdiv(B * A2_FWD_N[s], 256)), dim3(256), 0, st, ha, s);
        VAD_LAUNCH_CHECK();
      }
    }
    if (with_loss) VAD_TRY(loss(st));
    return 0;
  }

  int loss(hipStream_t st) {
    with_loss = 1;
    const A2HeadArgs ha = head_args();
    hipLaunchKernelGGL(a2_loss_kernel, dim3(1), dim3(512), 0, st, ha);
    VAD_LAUNCH_CHECK();
    hipLaunchKernelGGL(a2_pairs_kernel, dim3((unsigned)(B * B)), dim3(64), 0, st, ha);
    VAD_LAUNCH_CHECK();
    hipLaunchKernelGGL(a2_loss_fin_kernel, dim3(1), dim3(512), 0, st, ha);
    VAD_LAUNCH_CHECK();
    hipLaunchKernelGGL(a2_dadj_kernel, dim3((unsigned)cdiv(B * 256, 256)), dim3(256), 0, st, ha);
    VAD_LAUNCH_CHECK();
    return 0;
  }

  int backward(const float* ext_ds, const float* ext_dadj, const float* ext_df, hipStream_t st) {
    const bool from_loss = !ext_ds && !ext_dadj && !ext_df;
    VAD_CHECK(!from_loss || with_loss, "vad_a2_backward: the forward computed no loss and no upstream grads given");
    if (!from_loss) {
      // external upstream grads replace the loss ones (zeros where absent)
      VAD_HIP(hipMemsetAsync(d_s, 0, sizeof(float) * B, st));
      VAD_HIP(hipMemsetAsync(d_adj, 0, sizeof(float) * B * 256, st));
      if (ext_ds) VAD_HIP(hipMemcpyAsync(d_s, ext_ds, sizeof(float) * B, hipMemcpyDeviceToDevice, st));
      if (ext_dadj) VAD_HIP(hipMemcpyAsync(d_adj, ext_dadj, sizeof(float) * B * 256, hipMemcpyDeviceToDevice, st));
    }
    A2HeadBwdArgs hb{};
    hb.f = head_args();
    hb.d_s = d_s;
    hb.d_adj = d_adj;
    hb.d_f = from_loss ? nullptr : ext_df;
    hb.G = grads;
    hb.dz_ap2 = dz_ap2; hb.dz_ap0 = dz_ap0; hb.dg2 = dg2; hb.dz_ge0 = dz_ge0; hb.dz_cn2 = dz_cn2; hb.dz_cn0 = dz_cn0;
    hb.dfeat = dfeat;
    hb.h_fc = rng_h1(seed, S_A2_DROP_FC, step);
    hb.thr_fc = drop_threshold(0.3);
    hb.s_fc = 1.0f / (float)(1.0 - 0.3);
    hb.nseg = 6;
    if (g_a2_head_clip) {  // (fc's backward inside these two launches: no dense weight / input gradient GEMMs)
      hb.pooled = pooled;
      hb.dpooled = dpooled;
      hb.nseg = 7;
      hipLaunchKernelGGL(a2_head_bwd_clip_kernel, dim3((unsigned)B), dim3(256), 0, st, hb);
      VAD_LAUNCH_CHECK();
    }
    for (int s = g_a2_head_clip ? 6 : 0; s < 7; ++s) {
      const int n = s < 6 ? B * A2_BWD_OUT[s] : (hb.nseg == 7 ? A2_WG_TOTAL_FC : A2_WG_TOTAL);
      hipLaunchKernelGGL(a2_head_bwd_kernel, dim3((unsigned)cdiv(n, 256)), dim3(256), 0, st, hb, s);
      VAD_LAUNCH_CHECK();
    }
    if (!g_a2_head_clip) {
      VAD_TRY(dense_wgrad(dfeat, B, 16, pooled, 4096, G(S_FCW), G(S_FCB), scratch, scratch_floats, nullptr, st));
      VAD_TRY(dense_dgrad(dfeat, B, 16, P(S_FCW), 4096, dpooled, nullptr, 1.f, nullptr, st));
    }
    // (direct: each ReLU backward is fused into the producer of its gradient -- the average-pool backward for
    // conv3d_3, the parity-class input gradients for conv3d_2 / conv3d_1 -- instead of a relu_gate pass)
    VAD_TRY(adaptive_avgpool3d_bwd(dpooled, g[2].out(), 4, 4, 4, dA, st, direct ? y[2] : nullptr));
    float* cur = dA;  // (direct: the input gradients ping-pong between dA and dA2)
    for (int s3 = 2; s3 >= 0; --s3) {
      const int64_t rows = g[s3].rows();
      float* const dg = cur;  // the gradient w.r.t. this stage's output (then its pre-activation)
      if (!direct) VAD_TRY(relu_gate(dg, y[s3], rows * A2_CO[s3], st));
      if (direct && s3 > 0) {  // conv3d_2 / conv3d_3 on the implicit GEMMs
        const Vol5& in = g[s3].in;
        float* nxt = dg == dA ? dA2 : dA;
        // (weight and bias gradients from one split-K GEMM: the bias is a column of ones beside the patch columns)
        VAD_TRY(conv3s2_wgrad(dg, A2_CO[s3], y[s3 - 1], in.C, B, in.D, in.H, in.W, G(2 * s3), scratch, scratch_floats,
                              1024, st, G(2 * s3 + 1)));
        VAD_TRY(conv3s2_dgrad(dg, B, A2_CO[s3], wc3[s3], in.C, nxt, in.D, in.H, in.W, st, y[s3 - 1]));
        cur = nxt;
        continue;
      }
      if (direct && s3 == 0) {
        const A2Tiles tl(B, T, H, W);
        const int64_t cap = scratch_floats / (16 * (A2C1_TAPS + 1));
        const int nb = (int)std::max<int64_t>(1, std::min<int64_t>({tl.n, 512, cap}));
        hipLaunchKernelGGL(a2_conv1_wgrad_kernel, dim3((unsigned)nb), dim3(256), 0, st, dg, xsrc, B, T, H, W, scratch);
        VAD_LAUNCH_CHECK();
        hipLaunchKernelGGL(a2_conv1_wgrad_reduce_kernel, dim3((unsigned)cdiv(16 * (A2C1_TAPS + 1), 16)), dim3(256), 0,
                           st, scratch, nb, G(S_C1W), G(S_C1B));
        VAD_LAUNCH_CHECK();
        continue;
      }
      VAD_TRY(dense_wgrad(dg, (int)rows, A2_CO[s3], cols[s3], g[s3].K(), G(2 * s3), G(2 * s3 + 1), scratch,
                          scratch_floats, nullptr, st, 1024));
      if (s3 > 0) {
        VAD_TRY(dense_dgrad(dg, (int)rows, A2_CO[s3], P(2 * s3), g[s3].K(), dcols, nullptr, 1.f, nullptr, st));
        VAD_TRY(col2im3d(dcols, g[s3], dg, st));
      }
    }
    return 0;
  }

  int optimizer(float lr, float b1, float b2, float eps, float wd, float max_norm, hipStream_t st,
                float* user_losses = nullptr) {
    A2SlotTab t{};
    for (int i = 0; i < A2_NSLOT; ++i) {
      t.off[i] = a2_offsets().off[i];
      t.numel[i] = A2_SLOTS[i].numel;
    }
    hipLaunchKernelGGL(a2_sqsum_kernel, dim3(A2_NSLOT, A2_SQ_CHUNKS), dim3(256), 0, st, grads, t, sqp);
    VAD_LAUNCH_CHECK();
    hipLaunchKernelGGL(a2_opt_prepare_kernel, dim3(1), dim3(64), 0, st, sqp, losses, steps, lr, b1, b2, wd,
                       max_norm, ctrl, user_losses);
    VAD_LAUNCH_CHECK();
    const int64_t n = a2_offsets().total;
    hipLaunchKernelGGL(a2_adamw_kernel, dim3((unsigned)std::min<int64_t>(cdiv(n, 256), 1024)), dim3(256), 0, st,
                       params, grads, m, v, n, ctrl, b1, b2, eps);
    VAD_LAUNCH_CHECK();
    return 0;
  }
};

}  // namespace vad

using namespace vad;

struct vad_a2_plan {
  vad_a2_plan(int B, int T, int H, int W) : impl(B, T, H, W) {}
  A2PlanImpl impl;
  float* user_losses = nullptr;
  // option "host_losses": a pinned (device-visible) 10-float host buffer the forward's copy kernel also writes, so a
  // caller waiting for the forward's event reads the losses without a copy-engine transfer on the stream
  float* host_losses = nullptr;
};

extern "C" {

int vad_a2_num_slots(void) { return A2_NSLOT; }
const char* vad_a2_slot_name(int i) { return (i >= 0 && i < A2_NSLOT) ? A2_SLOTS[i].name : nullptr; }
int64_t vad_a2_slot_numel(int i) { return (i >= 0 && i < A2_NSLOT) ? A2_SLOTS[i].numel : -1; }
int64_t vad_a2_slot_offset(int i) { return (i >= 0 && i < A2_NSLOT) ? a2_offsets().off[i] : -1; }
int64_t vad_a2_param_floats(void) { return a2_offsets().total; }

int vad_a2_create(int B, int T, int H, int W, vad_a2_plan** out) {
  VAD_CHECK(out != nullptr, "vad_a2_create: out is null");
  VAD_CHECK(B >= 2 && B <= A2_MAXB && T >= 1 && H >= 4 && W >= 4,
            "vad_a2_create: unsupported shape (2 <= B <= 256: the loss squeezes the scores to (B,))");
  auto* p = new vad_a2_plan(B, T, H, W);
  Ws ws;
  p->impl.carve(ws);
  p->impl.ws_bytes = ws.off + 256;
  *out = p;
  return 0;
}

void vad_a2_destroy(vad_a2_plan* plan) { delete plan; }
int64_t vad_a2_workspace_bytes(const vad_a2_plan* p) { return p ? p->impl.ws_bytes : -1; }

int vad_a2_bind(vad_a2_plan* plan, void* workspace, float* params, float* grads, float* exp_avg, float* exp_avg_sq,
                int32_t* steps) {
  VAD_CHECK(plan && workspace && params && grads && exp_avg && exp_avg_sq && steps, "vad_a2_bind: null argument");
  VAD_CHECK((reinterpret_cast<uintptr_t>(workspace) & 255) == 0, "vad_a2_bind: workspace must be 256-B aligned");
  A2PlanImpl& c = plan->impl;
  Ws ws;
  ws.base = reinterpret_cast<char*>(workspace);
  ws.dry = false;
  c.carve(ws);
  c.params = params; c.grads = grads; c.m = exp_avg; c.v = exp_avg_sq; c.steps = steps;
  VAD_HIP(hipMemcpy(c.off_dev, a2_offsets().off, sizeof(int64_t) * A2_NSLOT, hipMemcpyHostToDevice));
  return 0;
}

}  // extern "C"

namespace vad {
// the plan's small outputs handed to the caller's buffers in one launch (instead of one copy-engine blit each)
struct A2Copies {
  const float* src[5];
  float* dst[5];
  int n[5];
};
__global__ __launch_bounds__(256) void a2_copies_kernel(A2Copies c) {
  const int k = blockIdx.x;
  for (int i = threadIdx.x; i < c.n[k]; i += 256) c.dst[k][i] = c.src[k][i];
}
static int a2_copies(const A2Copies& c, int nseg, hipStream_t st) {
  if (nseg == 0) return 0;
  hipLaunchKernelGGL(a2_copies_kernel, dim3((unsigned)nseg), dim3(256), 0, st, c);
  VAD_LAUNCH_CHECK();
  return 0;
}
}  // namespace vad

extern "C" {

int vad_a2_set_option(vad_a2_plan* plan, const char* key, int64_t value) {
  VAD_CHECK(plan && key, "vad_a2_set_option: null argument");
  const std::string k(key);
  if (k == "borrow_input") plan->impl.borrow_input = value != 0;
  else if (k == "host_losses") plan->host_losses = reinterpret_cast<float*>(value);  // pinned 10 floats, 0 = none
  else {
    vad::set_error("vad_a2_set_option: unknown option " + k);
    return 1;
  }
  return 0;
}

int vad_a2_forward(vad_a2_plan* plan, const float* x, int training, uint64_t seed, uint64_t step, int64_t clip0,
                   int with_loss, float* scores, float* adj, float* features, float* losses, void* stream) {
  VAD_CHECK(plan && x, "vad_a2_forward: null argument");
  A2PlanImpl& c = plan->impl;
  VAD_CHECK(c.params != nullptr, "vad_a2_forward: plan not bound");
  hipStream_t st = (hipStream_t)stream;
  c.training = training;
  c.seed = seed;
  c.step = step;
  c.clip0 = clip0;
  c.with_loss = with_loss;
  VAD_TRY(c.forward(x, st));
  const int B = c.B;
  A2Copies cp{};
  int k = 0;
  auto add = [&](float* d, const float* s, int n) {
    if (d) {
      cp.dst[k] = d;
      cp.src[k] = s;
      cp.n[k++] = n;
    }
  };
  add(scores, c.s, B);
  add(adj, c.adj, B * 256);
  add(features, c.f, B * 16);
  plan->user_losses = losses;
  add(with_loss ? losses : nullptr, c.losses, 10);
  add(with_loss ? plan->host_losses : nullptr, c.losses, 10);
  return a2_copies(cp, k, st);
}

int vad_a2_loss(vad_a2_plan* plan, uint64_t seed, uint64_t step, int64_t clip0, float* losses, void* stream) {
  VAD_CHECK(plan != nullptr, "vad_a2_loss: null plan");
  A2PlanImpl& c = plan->impl;
  hipStream_t st = (hipStream_t)stream;
  c.seed = seed;
  c.step = step;
  c.clip0 = clip0;
  VAD_TRY(c.loss(st));
  plan->user_losses = losses;
  if (losses) VAD_HIP(hipMemcpyAsync(losses, c.losses, sizeof(float) * 10, hipMemcpyDeviceToDevice, st));
  return 0;
}

int vad_a2_loss_grads(vad_a2_plan* plan, float* d_scores, float* d_adj, void* stream) {
  VAD_CHECK(plan != nullptr, "vad_a2_loss_grads: null plan");
  A2PlanImpl& c = plan->impl;
  hipStream_t st = (hipStream_t)stream;
  A2Copies cp{};
  int k = 0;
  if (d_scores) {
    cp.dst[k] = d_scores; cp.src[k] = c.d_s; cp.n[k++] = c.B;
  }
  if (d_adj) {
    cp.dst[k] = d_adj; cp.src[k] = c.d_adj; cp.n[k++] = c.B * 256;
  }
  return a2_copies(cp, k, st);
}

int vad_a2_backward(vad_a2_plan* plan, const float* d_scores, const float* d_adj, const float* d_features,
                    void* stream) {
  VAD_CHECK(plan != nullptr, "vad_a2_backward: null plan");
  return plan->impl.backward(d_scores, d_adj, d_features, (hipStream_t)stream);
}

int vad_a2_optimizer_step(vad_a2_plan* plan, float lr, float beta1, float beta2, float eps, float weight_decay,
                          float max_norm, void* stream) {
  VAD_CHECK(plan != nullptr, "vad_a2_optimizer_step: null plan");
  A2PlanImpl& c = plan->impl;
  hipStream_t st = (hipStream_t)stream;
  // (the optimizer changes only the total grad norm, losses[8]: its prepare kernel writes it into the caller's buffer
  // too -- no copy launch)
  VAD_TRY(c.optimizer(lr, beta1, beta2, eps, weight_decay, max_norm, st, plan->user_losses));
  return 0;
}

}  // extern "C"
