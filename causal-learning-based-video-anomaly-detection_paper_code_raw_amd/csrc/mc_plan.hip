// minicausal_vad_complete3.py (config 1): SimpleVideoAnomalyDetector (mc:25-102) train/eval step and the
// StableTrainer update (mc:249-330) as one device plan.
//
//   forward   3 x [im2col3d -> f32 MFMA GEMM (torch Conv3d weight as-is) -> BN3d partial sums -> bn_finalize
//             (batch stats, running stats) -> fused BN+ReLU+MaxPool3d] -> AdaptiveAvgPool3d(1) -> classifier kernel
//             (Dropout .5 / .3 from the keyed RNG, Linear/ReLU x2, Linear, sigmoid) + BCE + finiteness status
//   backward  classifier kernel (BCE/sigmoid/ReLU/dropout backward, classifier weight grads over the batch)
//             -> avg-pool backward -> per stage: MaxPool3d gather backward -> BN3d backward (reduce / finalize /
//             apply) -> weight+bias grad GEMM over the saved im2col columns -> input-grad GEMM + col2im
//   update    per-slot squared norms (float64) and finiteness -> grad norm, clip to max_norm only when the norm
//             exceeds clip_above (mc:304-306) -> Adam with coupled L2 weight decay (torch.optim.Adam semantics)
// Status word (losses[3]): 0 = skipped before backward (non-finite outputs or loss, mc:281-291), 1 = counted but
// not stepped (non-finite grads: zero_grad() then a no-op step, mc:296-301), 2 = stepped.
#include <cmath>
#include <string>
#include <vector>

#include "../../include/vad.h"
#include "backbone.h"
#include "conv3d.h"
#include "plan_util.h"

namespace vad {

constexpr int MC_CO[3] = {8, 16, 32};
constexpr int MC_POOL[3][3] = {{1, 2, 2}, {2, 2, 2}, {2, 2, 2}};
constexpr int MC_FC[4] = {32, 16, 8, 1};
constexpr int MC_MAXB = 1024;

struct McSlot {
  std::string name;
  int64_t numel, offset;
};

struct McLayout {
  std::vector<McSlot> slots, bufs;
  int64_t param_floats = 0, buf_floats = 0;
  int conv_w[3], conv_b[3], bn_w[3], bn_b[3], fc_w[3], fc_b[3], rm[3], rv[3];
  explicit McLayout(int C) {
    auto add = [&](std::vector<McSlot>& v, const std::string& n, int64_t k) {
      v.push_back({n, k, 0});
      return (int)v.size() - 1;
    };
    int ci = C;
    for (int s = 0; s < 3; ++s) {
      const std::string c = "features." + std::to_string(4 * s), b = "features." + std::to_string(4 * s + 1);
      conv_w[s] = add(slots, c + ".weight", (int64_t)MC_CO[s] * ci * 27);
      conv_b[s] = add(slots, c + ".bias", MC_CO[s]);
      bn_w[s] = add(slots, b + ".weight", MC_CO[s]);
      bn_b[s] = add(slots, b + ".bias", MC_CO[s]);
      rm[s] = add(bufs, b + ".running_mean", MC_CO[s]);
      rv[s] = add(bufs, b + ".running_var", MC_CO[s]);
      ci = MC_CO[s];
    }
    const int fidx[3] = {1, 4, 6};
    for (int i = 0; i < 3; ++i) {
      const std::string f = "classifier." + std::to_string(fidx[i]);
      fc_w[i] = add(slots, f + ".weight", (int64_t)MC_FC[i + 1] * MC_FC[i]);
      fc_b[i] = add(slots, f + ".bias", MC_FC[i + 1]);
    }
    for (auto& s : slots) {
      s.offset = param_floats;
      param_floats += (s.numel + 255) / 256 * 256;
    }
    for (auto& b : bufs) {
      b.offset = buf_floats;
      buf_floats += (b.numel + 255) / 256 * 256;
    }
  }
};

// ------------------------------------------------------------------ classifier head
struct McHeadArgs {
  int B, training;
  int64_t clip0;
  const float* feats;  // [B][32]
  const float *W1, *b1, *W2, *b2, *W3, *b3;
  float *fd, *h1, *h1d, *h2, *o;  // saved activations
  float* scores;                  // [B]
  const float* labels;            // [B] nullable
  float* losses;                  // [4]
  int32_t* flags;                 // [4] nullable
  uint64_t hA, hB;                // dropout keys (mc classifier.0 / classifier.3)
  uint32_t thrA, thrB;
  float sA, sB;
};

__global__ __launch_bounds__(256) void mc_head_fwd_kernel(McHeadArgs a) {
  __shared__ float red[256];
  __shared__ int bad[256];
  float lsum = 0.f;
  int nonfin = 0;
  for (int b = threadIdx.x; b < a.B; b += 256) {
    const int64_t row = a.clip0 + b;
    float f[32], h1[16], h2[8];
    for (int c = 0; c < 32; ++c) {
      float v = a.feats[b * 32 + c];
      if (a.training) v = rng_u24(a.hA, (uint64_t)row, (uint64_t)c) >= a.thrA ? v * a.sA : 0.f;
      f[c] = v;
      a.fd[b * 32 + c] = v;
    }
    for (int k = 0; k < 16; ++k) {
      float z = a.b1[k];
      for (int c = 0; c < 32; ++c) z = fmaf(a.W1[k * 32 + c], f[c], z);
      z = relu_nan(z);
      a.h1[b * 16 + k] = z;
      if (a.training) z = rng_u24(a.hB, (uint64_t)row, (uint64_t)k) >= a.thrB ? z * a.sB : 0.f;
      h1[k] = z;
      a.h1d[b * 16 + k] = z;
    }
    for (int j = 0; j < 8; ++j) {
      float z = a.b2[j];
      for (int k = 0; k < 16; ++k) z = fmaf(a.W2[j * 16 + k], h1[k], z);
      h2[j] = relu_nan(z);
      a.h2[b * 8 + j] = h2[j];
    }
    float z = a.b3[0];
    for (int j = 0; j < 8; ++j) z = fmaf(a.W3[j], h2[j], z);
    const float o = 1.f / (1.f + expf(-z));
    a.o[b] = o;
    a.scores[b] = o;
    if (!isfinite(o)) nonfin = 1;
    if (a.labels) {
      // torch BCELoss: -(y * max(log(o), -100) + (1 - y) * max(log1p(-o), -100))
      const float y = a.labels[b];
      lsum += -(y * fmaxf(logf(o), -100.f) + (1.f - y) * fmaxf(log1pf(-o), -100.f));
    }
  }
  red[threadIdx.x] = lsum;
  bad[threadIdx.x] = nonfin;
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if (threadIdx.x < s) {
      red[threadIdx.x] += red[threadIdx.x + s];
      bad[threadIdx.x] |= bad[threadIdx.x + s];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    const float loss = red[0] / (float)a.B;
    const bool ok = !bad[0] && (!a.labels || isfinite(loss));
    a.losses[0] = a.labels ? loss : 0.f;
    a.losses[1] = 0.f;
    a.losses[2] = 0.f;
    a.losses[3] = ok ? 2.f : 0.f;
    if (a.flags) a.flags[0] = ok ? 2 : 0;
  }
}

struct McHeadBwdArgs {
  McHeadArgs f;
  const float* d_scores;  // nullable: BCE of the forward's labels
  float *gW1, *gb1, *gW2, *gb2, *gW3, *gb3;
  float *dz1, *dz2, *dz3;  // scratch [B][16], [B][8], [B]
  float* dfeat;            // [B][32]
};

__global__ __launch_bounds__(256) void mc_head_bwd_kernel(McHeadBwdArgs a) {
  const McHeadArgs& f = a.f;
  const int B = f.B;
  for (int b = threadIdx.x; b < B; b += 256) {
    const int64_t row = f.clip0 + b;
    const float o = f.o[b];
    float dout;
    if (a.d_scores) {
      dout = a.d_scores[b];
    } else {
      // torch binary_cross_entropy_backward (mean): (o - y) / max((1 - o) * o, 1e-12) / B
      dout = (o - f.labels[b]) / fmaxf((1.f - o) * o, 1e-12f) / (float)B;
    }
    const float dz3 = dout * (1.f - o) * o;
    a.dz3[b] = dz3;
    float dz2[8];
    for (int j = 0; j < 8; ++j) {
      dz2[j] = f.h2[b * 8 + j] > 0.f ? dz3 * f.W3[j] : 0.f;
      a.dz2[b * 8 + j] = dz2[j];
    }
    float dz1[16];
    for (int k = 0; k < 16; ++k) {
      float d = 0.f;
      for (int j = 0; j < 8; ++j) d = fmaf(dz2[j], f.W2[j * 16 + k], d);
      if (f.training) d = rng_u24(f.hB, (uint64_t)row, (uint64_t)k) >= f.thrB ? d * f.sB : 0.f;
      dz1[k] = f.h1[b * 16 + k] > 0.f ? d : 0.f;
      a.dz1[b * 16 + k] = dz1[k];
    }
    for (int c = 0; c < 32; ++c) {
      float d = 0.f;
      for (int k = 0; k < 16; ++k) d = fmaf(dz1[k], f.W1[k * 32 + c], d);
      if (f.training) d = rng_u24(f.hA, (uint64_t)row, (uint64_t)c) >= f.thrA ? d * f.sA : 0.f;
      a.dfeat[b * 32 + c] = d;
    }
  }
  __syncthreads();
  // classifier weight grads: fixed-order sums over the batch, one thread per weight element
  constexpr int N3 = 8 + 1, N2 = 8 * 16 + 8, N1 = 16 * 32 + 16;
  for (int e = threadIdx.x; e < N3 + N2 + N1; e += 256) {
    float s = 0.f;
    if (e < 8) {
      for (int b = 0; b < B; ++b) s = fmaf(a.dz3[b], f.h2[b * 8 + e], s);
      a.gW3[e] = s;
    } else if (e < N3) {
      for (int b = 0; b < B; ++b) s += a.dz3[b];
      a.gb3[0] = s;
    } else if (e < N3 + 128) {
      const int q = e - N3, j = q / 16, k = q % 16;
      for (int b = 0; b < B; ++b) s = fmaf(a.dz2[b * 8 + j], f.h1d[b * 16 + k], s);
      a.gW2[q] = s;
    } else if (e < N3 + N2) {
      const int j = e - N3 - 128;
      for (int b = 0; b < B; ++b) s += a.dz2[b * 8 + j];
      a.gb2[j] = s;
    } else if (e < N3 + N2 + 512) {
      const int q = e - N3 - N2, k = q / 32, c = q % 32;
      for (int b = 0; b < B; ++b) s = fmaf(a.dz1[b * 16 + k], f.fd[b * 32 + c], s);
      a.gW1[q] = s;
    } else {
      const int k = e - N3 - N2 - 512;
      for (int b = 0; b < B; ++b) s += a.dz1[b * 16 + k];
      a.gb1[k] = s;
    }
  }
}

// ------------------------------------------------------------------ update
struct McSlotTab {
  int n;
  int64_t off[24], numel[24];
};

__global__ __launch_bounds__(256) void mc_sqsum_kernel(const float* __restrict__ g, McSlotTab t, double* sq,
                                                       int* bad) {
  const int s = blockIdx.x;
  __shared__ double red[256];
  __shared__ int rb[256];
  double acc = 0.0;
  int nf = 0;
  for (int64_t i = threadIdx.x; i < t.numel[s]; i += 256) {
    const float v = g[t.off[s] + i];
    if (!isfinite(v)) nf = 1;
    acc += (double)v * (double)v;
  }
  red[threadIdx.x] = acc;
  rb[threadIdx.x] = nf;
  __syncthreads();
  for (int k = 128; k > 0; k >>= 1) {
    if (threadIdx.x < k) {
      red[threadIdx.x] += red[threadIdx.x + k];
      rb[threadIdx.x] |= rb[threadIdx.x + k];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    sq[s] = red[0];
    bad[s] = rb[0];
  }
}

// ctrl: [0] step? (1/0), [1] clip coefficient, [2] -lr / bias_correction1, [3] sqrt(bias_correction2)
__global__ void mc_opt_prepare_kernel(const double* sq, const int* bad, int n, float* losses, int32_t* steps,
                                      float lr, float b1, float b2, float clip_above, float max_norm, float* ctrl) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  ctrl[0] = 0.f;
  ctrl[1] = 1.f;
  if (losses[3] < 1.f) return;  // skipped before backward
  double tot = 0.0;
  int nonfin = 0;
  for (int s = 0; s < n; ++s) {
    tot += (double)(float)sqrt(sq[s]) * (double)(float)sqrt(sq[s]);  // host sum of per-param norm**2 (mc:302)
    nonfin |= bad[s];
  }
  if (nonfin) {
    losses[3] = 1.f;
    return;
  }
  const double gn = sqrt(tot);
  losses[1] = (float)gn;
  if (gn > (double)clip_above) {
    // clip_grad_norm_(params, max_norm): total = ||(||g_p||)||, coef = max_norm / (total + 1e-6), clamped to 1
    const float total = (float)gn;
    ctrl[1] = fminf(1.f, max_norm / (total + 1e-6f));
    losses[2] = 1.f;
  }
  const int step = steps[0] + 1;
  for (int s = 0; s < n; ++s) steps[s] = step;
  const double bc1 = 1.0 - pow((double)b1, step), bc2 = 1.0 - pow((double)b2, step);
  ctrl[0] = 1.f;
  ctrl[2] = (float)(-(double)lr / bc1);
  ctrl[3] = (float)sqrt(bc2);
  losses[3] = 2.f;
}

__global__ __launch_bounds__(256) void mc_adam_kernel(float* __restrict__ p, const float* __restrict__ g,
                                                      float* __restrict__ m, float* __restrict__ v, int64_t n,
                                                      const float* ctrl, float b1, float b2, float eps, float wd) {
  if (ctrl[0] == 0.f) return;
  const float coef = ctrl[1], step_size = ctrl[2], bc2s = ctrl[3];
  for (int64_t i = blockIdx.x * 256ll + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const float pv = p[i];
    const float gv = fmaf(wd, pv, g[i] * coef);            // grad.add(param, alpha=wd) after clipping
    const float mv = m[i] + (1.f - b1) * (gv - m[i]);       // exp_avg.lerp_(grad, 1 - beta1)
    const float vv = fmaf(v[i], b2, (1.f - b2) * gv * gv);  // exp_avg_sq.mul_(b2).addcmul_(g, g, 1 - b2)
    m[i] = mv;
    v[i] = vv;
    p[i] = fmaf(step_size, mv / (sqrtf(vv) / bc2s + eps), pv);
  }
}

__global__ void mc_nbt_kernel(int64_t* nbt, int n) {
  if (threadIdx.x < n) nbt[threadIdx.x] += 1;
}

// ------------------------------------------------------------------ the plan
struct McPlanImpl {
  int B, C, T, H, W;
  McLayout LY;
  Conv3dGeom g[3];
  Vol5 conv_out[3], pooled_vol[3];
  int64_t ws_bytes = 0;
  float *params = nullptr, *grads = nullptr, *bufs = nullptr, *m = nullptr, *v = nullptr;
  int64_t* nbt = nullptr;
  int32_t* steps = nullptr;
  // workspace
  float *cols[3], *y[3], *pooled[3], *stats[3], *wf[3], *wd[3], *xin;
  float *parts, *bparts, *feats, *fd, *h1, *h1d, *h2, *o, *dz1, *dz2, *dz3, *dfeat, *dpool, *dA, *dY, *dcols;
  float *scratch, *labels_copy, *losses, *ctrl;
  double* sq;
  int* bad;
  int32_t* flags = nullptr;
  int64_t parts_floats = 0, scratch_floats = 0;
  // per-call state
  int training = 1, direct_fwd = 0;
  uint64_t seed = 0, step = 0;
  int64_t clip0 = 0;
  bool have_labels = false;

  McPlanImpl(int B_, int C_, int T_, int H_, int W_) : B(B_), C(C_), T(T_), H(H_), W(W_), LY(C_) {
    Vol5 in{B, C, T, H, W};
    for (int s = 0; s < 3; ++s) {
      g[s] = conv3d_geom(in, MC_CO[s], 3, 1, 1, 1, 1);
      conv_out[s] = g[s].out();
      pooled_vol[s] = {B, MC_CO[s], conv_out[s].D / MC_POOL[s][0], conv_out[s].H / MC_POOL[s][1],
                       conv_out[s].W / MC_POOL[s][2]};
      in = pooled_vol[s];
    }
  }
  float* P(int s) const { return params + LY.slots[s].offset; }
  float* G(int s) const { return grads + LY.slots[s].offset; }
  float* RM(int s) const { return bufs + LY.bufs[LY.rm[s]].offset; }
  float* RV(int s) const { return bufs + LY.bufs[LY.rv[s]].offset; }

  void carve(Ws& w) {
    int64_t max_y = 0, max_pool = 0, max_dcols = 0;
    parts_floats = 1024;
    for (int s = 0; s < 3; ++s) {
      const int64_t V = conv_out[s].voxels(), Co = MC_CO[s];
      cols[s] = w.take<float>(g[s].rows() * g[s].K());
      y[s] = w.take<float>(V * Co);
      pooled[s] = w.take<float>(pooled_vol[s].numel());
      stats[s] = w.take<float>(BN_STATS_PER_C * Co);
      max_y = std::max(max_y, V * Co);
      max_pool = std::max(max_pool, pooled_vol[s].numel());
      if (s > 0) max_dcols = std::max(max_dcols, g[s].rows() * g[s].K());
      parts_floats = std::max<int64_t>(parts_floats, std::max<int64_t>(bn_fwd_partials_blocks(V), cdiv(V, 64)) * 2 * Co);
    }
    for (int s = 0; s < 3; ++s) {
      const int64_t n = (int64_t)MC_CO[s] * g[s].in.C * 27;
      wf[s] = w.take<float>(n);
      wd[s] = w.take<float>(n);
    }
    xin = w.take<float>(g[0].in.numel());  // (the forward input, kept for the direct weight gradient)
    max_pool = std::max(max_pool, g[1].in.numel());
    max_pool = std::max(max_pool, g[2].in.numel());
    parts = w.take<float>(parts_floats);
    bparts = w.take<float>(parts_floats);
    feats = w.take<float>((int64_t)B * 32);
    fd = w.take<float>((int64_t)B * 32);
    h1 = w.take<float>((int64_t)B * 16);
    h1d = w.take<float>((int64_t)B * 16);
    h2 = w.take<float>((int64_t)B * 8);
    o = w.take<float>(B);
    dz1 = w.take<float>((int64_t)B * 16);
    dz2 = w.take<float>((int64_t)B * 8);
    dz3 = w.take<float>(B);
    dfeat = w.take<float>((int64_t)B * 32);
    dpool = w.take<float>(max_pool);
    dA = w.take<float>(max_y);
    dY = w.take<float>(max_y);
    dcols = w.take<float>(std::max<int64_t>(max_dcols, 1));
    scratch_floats = 8ll << 20;
    scratch = w.take<float>(scratch_floats);
    labels_copy = w.take<float>(B);
    losses = w.take<float>(4);
    ctrl = w.take<float>(4);
    sq = w.take<double>(32);
    bad = w.take<int>(32);
  }

  McHeadArgs head_args() const {
    McHeadArgs a{};
    a.B = B;
    a.training = training;
    a.clip0 = clip0;
    a.feats = feats;
    a.W1 = P(LY.fc_w[0]); a.b1 = P(LY.fc_b[0]);
    a.W2 = P(LY.fc_w[1]); a.b2 = P(LY.fc_b[1]);
    a.W3 = P(LY.fc_w[2]); a.b3 = P(LY.fc_b[2]);
    a.fd = fd; a.h1 = h1; a.h1d = h1d; a.h2 = h2; a.o = o;
    a.labels = have_labels ? labels_copy : nullptr;
    a.losses = losses;
    a.flags = flags;
    a.hA = rng_h1(seed, S_MC_DROP1, step);
    a.hB = rng_h1(seed, S_MC_DROP2, step);
    a.thrA = drop_threshold(0.5);
    a.thrB = drop_threshold(0.3);
    a.sA = 1.0f / (float)(1.0 - 0.5);
    a.sB = 1.0f / (float)(1.0 - 0.3);
    return a;
  }

  bool direct(int s) const { return conv3d_direct_supported(g[s].in.C, MC_CO[s]); }

  int forward(const float* x, float* scores, hipStream_t st) {
    // direct convs (conv3d_direct.hip) keep the input for the weight gradient instead of the im2col columns
    direct_fwd = direct(0) && direct(1) && direct(2);
    if (direct_fwd)
      VAD_HIP(hipMemcpyAsync(xin, x, g[0].in.numel() * sizeof(float), hipMemcpyDeviceToDevice, st));
    for (int s = 0; s < 3; ++s) {
      const int Co = MC_CO[s];
      const int64_t V = conv_out[s].voxels();
      const float* src = s == 0 ? x : pooled[s - 1];
      const Strides5 str = s == 0 ? ncdhw_strides(g[0].in) : ndhwc_strides(g[s].in);
      if (direct_fwd) {
        VAD_TRY(conv3d_direct_prep(P(LY.conv_w[s]), Co, g[s].in.C, wf[s], wd[s], st));
        VAD_TRY(conv3d_direct_fwd(src, str, g[s].in, wf[s], Co, P(LY.conv_b[s]), y[s], st));
      } else {
        VAD_TRY(im2col3d(src, str, g[s], nullptr, nullptr, 0, cols[s], st));
        VAD_TRY(dense_fwd(cols[s], (int)g[s].rows(), g[s].K(), P(LY.conv_w[s]), P(LY.conv_b[s]), Co, y[s],
                          DenseAct{}, scratch, scratch_floats, st));
      }
      int np = 0;
      if (training) VAD_TRY(bn_fwd_partials(y[s], V, Co, parts, &np, st));
      VAD_TRY(bn_finalize(parts, np, Co, (double)V, P(LY.bn_w[s]), P(LY.bn_b[s]), RM(s), RV(s), 0.1f, 1e-5f,
                          training, stats[s], st));
      VAD_TRY(maxpool3d_fwd(y[s], stats[s], 1, conv_out[s], MC_POOL[s][0], MC_POOL[s][1], MC_POOL[s][2], pooled[s],
                            st));
    }
    VAD_TRY(adaptive_avgpool3d_fwd(pooled[2], nullptr, 0, pooled_vol[2], 1, 1, 1, feats, st));
    McHeadArgs a = head_args();
    a.scores = scores;
    hipLaunchKernelGGL(mc_head_fwd_kernel, dim3(1), dim3(256), 0, st, a);
    VAD_LAUNCH_CHECK();
    if (training && nbt) {
      hipLaunchKernelGGL(mc_nbt_kernel, dim3(1), dim3(64), 0, st, nbt, 3);
      VAD_LAUNCH_CHECK();
    }
    return 0;
  }

  int backward(const float* d_scores, hipStream_t st) {
    VAD_CHECK(d_scores || have_labels, "vad_mc_backward: no labels in the forward and no d_scores");
    McHeadBwdArgs hb{};
    hb.f = head_args();
    hb.d_scores = d_scores;
    hb.gW1 = G(LY.fc_w[0]); hb.gb1 = G(LY.fc_b[0]);
    hb.gW2 = G(LY.fc_w[1]); hb.gb2 = G(LY.fc_b[1]);
    hb.gW3 = G(LY.fc_w[2]); hb.gb3 = G(LY.fc_b[2]);
    hb.dz1 = dz1; hb.dz2 = dz2; hb.dz3 = dz3; hb.dfeat = dfeat;
    hipLaunchKernelGGL(mc_head_bwd_kernel, dim3(1), dim3(256), 0, st, hb);
    VAD_LAUNCH_CHECK();
    VAD_TRY(adaptive_avgpool3d_bwd(dfeat, pooled_vol[2], 1, 1, 1, dpool, st));
    for (int s = 2; s >= 0; --s) {
      const int Co = MC_CO[s];
      const int64_t V = conv_out[s].voxels();
      VAD_TRY(maxpool3d_bwd(y[s], stats[s], 1, conv_out[s], MC_POOL[s][0], MC_POOL[s][1], MC_POOL[s][2], dpool, dA,
                            st));
      int np = 0, nb = 0;
      VAD_TRY(bn_bwd_reduce(dA, y[s], stats[s], (int)V, Co, parts, &np, st));
      VAD_TRY(bn_bwd_finalize(parts, np, Co, (double)V, P(LY.bn_w[s]), stats[s], G(LY.bn_w[s]), G(LY.bn_b[s]),
                              training, st));
      VAD_TRY(bn_bwd_apply(dA, y[s], stats[s], (int)V, Co, dY, bparts, &nb, st));
      if (direct_fwd) {
        const float* src = s == 0 ? xin : pooled[s - 1];
        const Strides5 str = s == 0 ? ncdhw_strides(g[0].in) : ndhwc_strides(g[s].in);
        VAD_TRY(conv3d_direct_wgrad(dY, Co, src, str, g[s].in, G(LY.conv_w[s]), G(LY.conv_b[s]), scratch,
                                    scratch_floats, st));
        if (s > 0) {  // dX = conv(dY, flipped W^T): NDHWC over the layer's input grid
          const Vol5 vy{g[s].in.N, Co, g[s].in.D, g[s].in.H, g[s].in.W};
          VAD_TRY(conv3d_direct_fwd(dY, ndhwc_strides(vy), vy, wd[s], g[s].in.C, nullptr, dpool, st));
        }
      } else {
        VAD_TRY(dense_wgrad(dY, (int)V, Co, cols[s], g[s].K(), G(LY.conv_w[s]), G(LY.conv_b[s]), scratch,
                            scratch_floats, nullptr, st));
        if (s > 0) {
          VAD_TRY(dense_dgrad(dY, (int)V, Co, P(LY.conv_w[s]), g[s].K(), dcols, nullptr, 1.f, nullptr, st));
          VAD_TRY(col2im3d(dcols, g[s], dpool, st));
        }
      }
    }
    return 0;
  }

  int optimizer(float lr, float b1, float b2, float eps, float wd, float clip_above, float max_norm, hipStream_t st) {
    McSlotTab t{};
    t.n = (int)LY.slots.size();
    VAD_CHECK(t.n <= 24, "mc optimizer: slot table overflow");
    for (int i = 0; i < t.n; ++i) {
      t.off[i] = LY.slots[i].offset;
      t.numel[i] = LY.slots[i].numel;
    }
    hipLaunchKernelGGL(mc_sqsum_kernel, dim3(t.n), dim3(256), 0, st, grads, t, sq, bad);
    VAD_LAUNCH_CHECK();
    hipLaunchKernelGGL(mc_opt_prepare_kernel, dim3(1), dim3(64), 0, st, sq, bad, t.n, losses, steps, lr, b1, b2,
                       clip_above, max_norm, ctrl);
    VAD_LAUNCH_CHECK();
    const int64_t n = LY.param_floats;
    hipLaunchKernelGGL(mc_adam_kernel, dim3((unsigned)std::min<int64_t>(cdiv(n, 256), 1024)), dim3(256), 0, st,
                       params, grads, m, v, n, ctrl, b1, b2, eps, wd);
    VAD_LAUNCH_CHECK();
    return 0;
  }
};

}  // namespace vad

using namespace vad;

struct vad_mc_plan {
  explicit vad_mc_plan(int B, int C, int T, int H, int W) : impl(B, C, T, H, W) {}
  McPlanImpl impl;
  float* user_losses = nullptr;
};

extern "C" {

int vad_mc_create(int B, int C, int T, int H, int W, vad_mc_plan** out) {
  VAD_CHECK(out != nullptr, "vad_mc_create: out is null");
  VAD_CHECK(B >= 1 && B <= MC_MAXB && C >= 1 && C <= 64 && T >= 4 && H >= 8 && W >= 8,
            "vad_mc_create: unsupported shape (B<=1024, T>=4, H,W>=8 so every MaxPool3d window fits)");
  auto* p = new vad_mc_plan(B, C, T, H, W);
  for (int s = 0; s < 3; ++s)
    if (p->impl.pooled_vol[s].D < 1 || p->impl.pooled_vol[s].H < 1 || p->impl.pooled_vol[s].W < 1) {
      delete p;
      set_error("vad_mc_create: input too small for the three MaxPool3d stages");
      return 1;
    }
  Ws ws;
  p->impl.carve(ws);
  p->impl.ws_bytes = ws.off + 256;
  *out = p;
  return 0;
}

void vad_mc_destroy(vad_mc_plan* plan) { delete plan; }

int vad_mc_num_slots(const vad_mc_plan* p) { return p ? (int)p->impl.LY.slots.size() : -1; }
const char* vad_mc_slot_name(const vad_mc_plan* p, int i) {
  return (p && i >= 0 && i < vad_mc_num_slots(p)) ? p->impl.LY.slots[i].name.c_str() : nullptr;
}
int64_t vad_mc_slot_numel(const vad_mc_plan* p, int i) {
  return (p && i >= 0 && i < vad_mc_num_slots(p)) ? p->impl.LY.slots[i].numel : -1;
}
int64_t vad_mc_slot_offset(const vad_mc_plan* p, int i) {
  return (p && i >= 0 && i < vad_mc_num_slots(p)) ? p->impl.LY.slots[i].offset : -1;
}
int64_t vad_mc_param_floats(const vad_mc_plan* p) { return p ? p->impl.LY.param_floats : -1; }
int vad_mc_num_bufs(const vad_mc_plan* p) { return p ? (int)p->impl.LY.bufs.size() : -1; }
const char* vad_mc_buf_name(const vad_mc_plan* p, int i) {
  return (p && i >= 0 && i < vad_mc_num_bufs(p)) ? p->impl.LY.bufs[i].name.c_str() : nullptr;
}
int64_t vad_mc_buf_numel(const vad_mc_plan* p, int i) {
  return (p && i >= 0 && i < vad_mc_num_bufs(p)) ? p->impl.LY.bufs[i].numel : -1;
}
int64_t vad_mc_buf_offset(const vad_mc_plan* p, int i) {
  return (p && i >= 0 && i < vad_mc_num_bufs(p)) ? p->impl.LY.bufs[i].offset : -1;
}
int64_t vad_mc_buf_floats(const vad_mc_plan* p) { return p ? p->impl.LY.buf_floats : -1; }
int64_t vad_mc_workspace_bytes(const vad_mc_plan* p) { return p ? p->impl.ws_bytes : -1; }

int vad_mc_bind(vad_mc_plan* plan, void* workspace, float* params, float* grads, float* bufs, int64_t* nbt,
                float* exp_avg, float* exp_avg_sq, int32_t* steps) {
  VAD_CHECK(plan && workspace && params && grads && bufs && exp_avg && exp_avg_sq && steps,
            "vad_mc_bind: null argument");
  VAD_CHECK((reinterpret_cast<uintptr_t>(workspace) & 255) == 0, "vad_mc_bind: workspace must be 256-B aligned");
  McPlanImpl& c = plan->impl;
  Ws ws;
  ws.base = reinterpret_cast<char*>(workspace);
  ws.dry = false;
  c.carve(ws);
  c.params = params; c.grads = grads; c.bufs = bufs; c.nbt = nbt;
  c.m = exp_avg; c.v = exp_avg_sq; c.steps = steps;
  return 0;
}

int vad_mc_forward(vad_mc_plan* plan, const float* x, int training, uint64_t seed, uint64_t step, int64_t clip0,
                   const float* labels, float* scores, float* losses, int32_t* flags, void* stream) {
  VAD_CHECK(plan && x && scores, "vad_mc_forward: null argument");
  McPlanImpl& c = plan->impl;
  VAD_CHECK(c.params != nullptr, "vad_mc_forward: plan not bound");
  hipStream_t st = (hipStream_t)stream;
  c.training = training;
  c.seed = seed;
  c.step = step;
  c.clip0 = clip0;
  c.have_labels = labels != nullptr;
  c.flags = flags;
  if (labels) VAD_HIP(hipMemcpyAsync(c.labels_copy, labels, sizeof(float) * c.B, hipMemcpyDeviceToDevice, st));
  VAD_TRY(c.forward(x, scores, st));
  plan->user_losses = losses;
  if (losses) VAD_HIP(hipMemcpyAsync(losses, c.losses, 4 * sizeof(float), hipMemcpyDeviceToDevice, st));
  return 0;
}

int vad_mc_backward(vad_mc_plan* plan, const float* d_scores, void* stream) {
  VAD_CHECK(plan != nullptr, "vad_mc_backward: null plan");
  return plan->impl.backward(d_scores, (hipStream_t)stream);
}

int vad_mc_optimizer_step(vad_mc_plan* plan, float lr, float beta1, float beta2, float eps, float weight_decay,
                          float clip_above, float max_norm, void* stream) {
  VAD_CHECK(plan != nullptr, "vad_mc_optimizer_step: null plan");
  McPlanImpl& c = plan->impl;
  hipStream_t st = (hipStream_t)stream;
  VAD_TRY(c.optimizer(lr, beta1, beta2, eps, weight_decay, clip_above, max_norm, st));
  if (plan->user_losses)
    VAD_HIP(hipMemcpyAsync(plan->user_losses, c.losses, 4 * sizeof(float), hipMemcpyDeviceToDevice, st));
  return 0;
}

}  // extern "C"
