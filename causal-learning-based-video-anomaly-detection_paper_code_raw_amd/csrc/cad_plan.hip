// Orchestration of the CausalAnomalyDetector train step (causal_anomaly_detection.py:540-586, 609-690) on one
// HIP stream, plus the optimizer kernels and the extern "C" ABI declared in include/vad.h.
// The plan owns no device memory: PyTorch allocates the workspace and the flat parameter/grad/state buffers.
#include <algorithm>
#include <cstring>
#include <vector>

#include "../../include/vad.h"
#include "backbone.h"
#include "head.h"
#include "mlp.h"
#include "plan_util.h"

namespace vad {

// ------------------------------------------------------------------ parameter slot table (state_dict order)
enum Group { G_FROZEN = 0, G_ALWAYS = 1, G_DET = 2, G_STRUCT = 3, G_NEVER = 4 };
struct Slot {
  std::string name;
  int64_t numel;
  int group;
  int64_t offset;
};
struct BufSlot {
  std::string name;
  int64_t numel;
  int64_t offset;
};

constexpr int64_t ALIGN = 256;
static int64_t align_up(int64_t v) { return (v + ALIGN - 1) / ALIGN * ALIGN; }

struct CadLayout {
  std::vector<Slot> slots;
  std::vector<BufSlot> bufs;
  int64_t param_floats = 0, buf_floats = 0;
  // indices
  int conv1_w, conv1_b, bn1_w, bn1_b;
  int conv_w[8], conv_b[8], bn_w[8], bn_b[8];
  int det_w[5], det_b[5], dir_w[5], dir_b[5];
  int head0;  // first head slot (tracker.reid_net.0.weight)
  int rm[9], rv[9];
  CadLayout() {
    auto add = [&](const std::string& n, int64_t k, int g) {
      slots.push_back({n, k, g, 0});
      return (int)slots.size() - 1;
    };
    auto addb = [&](const std::string& n, int64_t k) {
      bufs.push_back({n, k, 0});
      return (int)bufs.size() - 1;
    };
    conv1_w = add("backbone.conv1.weight", 32 * 49, G_FROZEN);
    conv1_b = add("backbone.conv1.bias", 32, G_FROZEN);
    bn1_w = add("backbone.bn1.weight", 32, G_FROZEN);
    bn1_b = add("backbone.bn1.bias", 32, G_FROZEN);
    rm[0] = addb("backbone.bn1.running_mean", 32);
    rv[0] = addb("backbone.bn1.running_var", 32);
    const int cin[8] = {32, 32, 32, 64, 64, 128, 128, 256};
    const int cout[8] = {32, 32, 64, 64, 128, 128, 256, 256};
    for (int l = 0; l < 8; ++l) {
      const std::string L = "backbone.layer" + std::to_string(l / 2 + 1) + ".";
      const std::string c = L + (l % 2 == 0 ? "0" : "3"), b = L + (l % 2 == 0 ? "1" : "4");
      conv_w[l] = add(c + ".weight", (int64_t)cout[l] * cin[l] * 9, G_ALWAYS);
      conv_b[l] = add(c + ".bias", cout[l], G_ALWAYS);
      bn_w[l] = add(b + ".weight", cout[l], G_ALWAYS);
      bn_b[l] = add(b + ".bias", cout[l], G_ALWAYS);
      rm[l + 1] = addb(b + ".running_mean", cout[l]);
      rv[l + 1] = addb(b + ".running_var", cout[l]);
    }
    const int dims[6] = {6144, 512, 256, 128, 64, 20};
    const int didx[5] = {0, 3, 6, 8, 10};
    for (int i = 0; i < 5; ++i) {
      det_w[i] = add("detector.detector_net." + std::to_string(didx[i]) + ".weight", (int64_t)dims[i + 1] * dims[i],
                     G_DET);
      det_b[i] = add("detector.detector_net." + std::to_string(didx[i]) + ".bias", dims[i + 1], G_DET);
    }
    struct H { const char* n; int64_t k; int g; };
    const H head[H_NUM] = {
        {"tracker.reid_net.0.weight", 32 * 4, G_ALWAYS}, {"tracker.reid_net.0.bias", 32, G_ALWAYS},
        {"tracker.reid_net.2.weight", 64 * 32, G_ALWAYS}, {"tracker.reid_net.2.bias", 64, G_ALWAYS},
        {"tracker.reid_net.4.weight", 64 * 64, G_ALWAYS}, {"tracker.reid_net.4.bias", 64, G_ALWAYS},
        {"traj_encoder.gru.weight_ih_l0", 192 * 68, G_ALWAYS}, {"traj_encoder.gru.weight_hh_l0", 192 * 64, G_ALWAYS},
        {"traj_encoder.gru.bias_ih_l0", 192, G_ALWAYS}, {"traj_encoder.gru.bias_hh_l0", 192, G_ALWAYS},
        {"traj_encoder.encoder.weight", 32 * 64, G_ALWAYS}, {"traj_encoder.encoder.bias", 32, G_ALWAYS},
        {"causal_extractor.encoder.0.weight", 32 * 32, G_ALWAYS}, {"causal_extractor.encoder.0.bias", 32, G_ALWAYS},
        {"causal_extractor.encoder.2.weight", 32 * 32, G_ALWAYS}, {"causal_extractor.encoder.2.bias", 32, G_ALWAYS},
        {"causal_extractor.mu_head.weight", 6 * 32, G_ALWAYS}, {"causal_extractor.mu_head.bias", 6, G_ALWAYS},
        {"causal_extractor.logvar_head.weight", 6 * 32, G_ALWAYS}, {"causal_extractor.logvar_head.bias", 6, G_ALWAYS},
        {"structure_learner.structure_params", 36, G_NEVER},
        {"structure_learner.node_encoder.weight", 32 * 6, G_STRUCT}, {"structure_learner.node_encoder.bias", 32, G_STRUCT},
        {"structure_learner.edge_predictor.0.weight", 32 * 64, G_STRUCT},
        {"structure_learner.edge_predictor.0.bias", 32, G_STRUCT},
        {"structure_learner.edge_predictor.2.weight", 32, G_STRUCT},
        {"structure_learner.edge_predictor.2.bias", 1, G_STRUCT},
        {"dynamics_predictor.dynamics_net.0.weight", 32 * 6, G_ALWAYS}, {"dynamics_predictor.dynamics_net.0.bias", 32, G_ALWAYS},
        {"dynamics_predictor.dynamics_net.2.weight", 32 * 32, G_ALWAYS}, {"dynamics_predictor.dynamics_net.2.bias", 32, G_ALWAYS},
        {"dynamics_predictor.dynamics_net.4.weight", 6 * 32, G_ALWAYS}, {"dynamics_predictor.dynamics_net.4.bias", 6, G_ALWAYS},
        {"anomaly_scorer.causal_scorer.0.weight", 64 * 18, G_ALWAYS}, {"anomaly_scorer.causal_scorer.0.bias", 64, G_ALWAYS},
        {"anomaly_scorer.causal_scorer.3.weight", 32 * 64, G_ALWAYS}, {"anomaly_scorer.causal_scorer.3.bias", 32, G_ALWAYS},
        {"anomaly_scorer.causal_scorer.5.weight", 32, G_ALWAYS}, {"anomaly_scorer.causal_scorer.5.bias", 1, G_ALWAYS},
        {"anomaly_scorer.motion_scorer.0.weight", 32 * 12, G_ALWAYS}, {"anomaly_scorer.motion_scorer.0.bias", 32, G_ALWAYS},
        {"anomaly_scorer.motion_scorer.2.weight", 16 * 32, G_ALWAYS}, {"anomaly_scorer.motion_scorer.2.bias", 16, G_ALWAYS},
        {"anomaly_scorer.motion_scorer.4.weight", 16, G_ALWAYS}, {"anomaly_scorer.motion_scorer.4.bias", 1, G_ALWAYS},
        {"anomaly_scorer.temporal_scorer.0.weight", 32 * 6, G_ALWAYS}, {"anomaly_scorer.temporal_scorer.0.bias", 32, G_ALWAYS},
        {"anomaly_scorer.temporal_scorer.2.weight", 16 * 32, G_ALWAYS}, {"anomaly_scorer.temporal_scorer.2.bias", 16, G_ALWAYS},
        {"anomaly_scorer.temporal_scorer.4.weight", 16, G_ALWAYS}, {"anomaly_scorer.temporal_scorer.4.bias", 1, G_ALWAYS},
    };
    head0 = (int)slots.size();
    for (int i = 0; i < H_NUM; ++i) add(head[i].n, head[i].k, head[i].g);
    for (int i = 0; i < 5; ++i) {
      dir_w[i] = add("direct_classifier." + std::to_string(didx[i]) + ".weight",
                     (int64_t)(i == 4 ? 2 : dims[i + 1]) * dims[i], G_ALWAYS);
      dir_b[i] = add("direct_classifier." + std::to_string(didx[i]) + ".bias", i == 4 ? 2 : dims[i + 1], G_ALWAYS);
    }
    int64_t o = 0;
    for (auto& s : slots) {
      s.offset = o;
      o = align_up(o + s.numel);
    }
    param_floats = o;
    o = 0;
    for (auto& b : bufs) {
      b.offset = o;
      o = align_up(o + b.numel);
    }
    buf_floats = o;
  }
};

static const CadLayout& layout() {
  static CadLayout L;
  return L;
}

constexpr int64_t FLAG_FLOATS = 256;  // grad buffer tail: [0] det flag, [1] struct flag (summed under DP)

// ------------------------------------------------------------------ optimizer kernels
struct SlotTab {
  int64_t off[160];
  int32_t group[160];
  int nslots;
};

__device__ inline bool slot_active(int g, const float* flags, int stem) {
  return g == G_ALWAYS || (g == G_DET && flags[0] > 0.f) || (g == G_STRUCT && flags[1] > 0.f) ||
         (g == G_FROZEN && stem);
}

// sum of squared (scaled) grads: one 256-float chunk (slots are 256-aligned) per wave iteration, float4 per lane;
// chunks of slots without a grad this step (frozen, or the detector / structure learner when their flag is 0: zero)
// are skipped.  Per-lane float sums, block combine in double.
__global__ __launch_bounds__(256) void sqsum_kernel(const float* __restrict__ g, const int16_t* __restrict__ chunk_slot,
                                                    int64_t nchunks, SlotTab tab, const float* __restrict__ flags,
                                                    float scale, float* __restrict__ partials, int stem) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  float s = 0.f;
  for (int64_t c = (int64_t)blockIdx.x * 4 + wave; c < nchunks; c += (int64_t)gridDim.x * 4) {
    const int sl = chunk_slot[c];
    if (sl < 0 || !slot_active(tab.group[sl], flags, stem)) continue;
    const f32x4 v = *reinterpret_cast<const f32x4*>(g + c * 256 + lane * 4) * scale;
    s = fmaf(v[0], v[0], s);
    s = fmaf(v[1], v[1], s);
    s = fmaf(v[2], v[2], s);
    s = fmaf(v[3], v[3], s);
  }
  __shared__ double red[256];
  red[threadIdx.x] = s;
  __syncthreads();
  for (int k = 128; k > 0; k >>= 1) {
    if (threadIdx.x < k) red[threadIdx.x] += red[threadIdx.x + k];
    __syncthreads();
  }
  if (threadIdx.x == 0) partials[blockIdx.x] = (float)red[0];
}

// per-slot step bump + bias corrections; clip coefficient (torch clip_grad_norm_: coef = max/(norm+1e-6) <= 1)
__global__ void opt_prepare_kernel(const float* __restrict__ partials, int np, const float* __restrict__ flags,
                                   SlotTab tab, int32_t* steps, float beta1, float beta2, float max_norm,
                                   float* __restrict__ slot_info /* [nslots][4] */, float* clip_out,
                                   float* total_norm_out, int stem) {
  __shared__ double red[256];
  double s = 0.0;
  for (int i = threadIdx.x; i < np; i += 256) s += partials[i];
  red[threadIdx.x] = s;
  __syncthreads();
  for (int k = 128; k > 0; k >>= 1) {
    if (threadIdx.x < k) red[threadIdx.x] += red[threadIdx.x + k];
    __syncthreads();
  }
  const float norm = (float)sqrt(red[0]);
  if (threadIdx.x == 0) {
    float coef = max_norm / (norm + 1e-6f);
    clip_out[0] = coef < 1.f ? coef : 1.f;
    if (total_norm_out) total_norm_out[0] = norm;
  }
  for (int i = threadIdx.x; i < tab.nslots; i += 256) {
    const int g = tab.group[i];
    const bool active = slot_active(g, flags, stem);
    float st = 0.f, bc1 = 1.f, bc2s = 1.f;
    if (active) {
      const int step = steps[i] + 1;
      steps[i] = step;
      st = (float)step;
      bc1 = (float)(1.0 - pow((double)beta1, (double)step));
      bc2s = (float)sqrt(1.0 - pow((double)beta2, (double)step));
    }
    slot_info[i * 4 + 0] = active ? 1.f : 0.f;
    slot_info[i * 4 + 1] = bc1;
    slot_info[i * 4 + 2] = bc2s;
    slot_info[i * 4 + 3] = st;
  }
}

// torch.optim.AdamW single-tensor update, one 256-element chunk per block iteration (slots are 256-aligned)
__global__ __launch_bounds__(256) void adamw_kernel(float* __restrict__ p, const float* __restrict__ g,
                                                    float* __restrict__ m, float* __restrict__ v,
                                                    const int16_t* __restrict__ chunk_slot, int64_t nchunks,
                                                    const float* __restrict__ slot_info,
                                                    const float* __restrict__ clip, float grad_scale, float lr,
                                                    float beta1, float beta2, float eps, float wd) {
  const float coef = clip[0] * grad_scale;
  for (int64_t c = blockIdx.x; c < nchunks; c += gridDim.x) {
    const int s = chunk_slot[c];
    if (s < 0) continue;
    if (slot_info[s * 4] == 0.f) continue;
    const float bc1 = slot_info[s * 4 + 1], bc2s = slot_info[s * 4 + 2];
    const int64_t i = c * 256 + threadIdx.x;
    const float gr = g[i] * coef;
    float pv = p[i] * (1.f - lr * wd);
    const float mv = m[i] + (gr - m[i]) * (1.f - beta1);
    const float vv = v[i] * beta2 + gr * gr * (1.f - beta2);
    const float denom = sqrtf(vv) / bc2s + eps;
    pv = pv - (lr / bc1) * mv / denom;
    p[i] = pv;
    m[i] = mv;
    v[i] = vv;
  }
}

__global__ void nbt_bump_kernel(int64_t* nbt, int n) {
  if (threadIdx.x < n) nbt[threadIdx.x] += 1;
}

__global__ void rng_u24_kernel(uint64_t h1, int64_t row0, int64_t nrows, int64_t ncols, uint32_t* out) {
  const int64_t total = nrows * ncols;
  for (int64_t i = blockIdx.x * 256ll + threadIdx.x; i < total; i += (int64_t)gridDim.x * 256)
    out[i] = rng_u24(h1, (uint64_t)(row0 + i / ncols), (uint64_t)(i % ncols));
}

// mode 0: (u8 - 0.5)/0.5 (cad Normalize); mode 1: u8/255 (ToTensor range, mc:120 / bbox:411)
__global__ void synth_kernel(uint64_t h1, int64_t frame0, int64_t nframes, int64_t npix, int mode, float* out) {
  const int64_t total = nframes * npix;
  for (int64_t i = blockIdx.x * 256ll + threadIdx.x; i < total; i += (int64_t)gridDim.x * 256) {
    const uint32_t u8 = (uint32_t)(rng_hash(h1, (uint64_t)(frame0 + i / npix), (uint64_t)(i % npix)) >> 56);
    out[i] = mode == 0 ? ((float)u8 - 0.5f) / 0.5f : (float)u8 / 255.f;
  }
}

// ------------------------------------------------------------------ HIP-event timing of labelled launches
struct Profiler {
  bool on = false;
  std::string only;  // label prefix filter ("" = all)
  struct Rec { std::string label; hipEvent_t a, b; };
  std::vector<Rec> recs;
  std::vector<hipEvent_t> pool;
  size_t used = 0;
  hipEvent_t get() {
    if (used == pool.size()) {
      hipEvent_t e;
      // timing-only events: no system-scope fence (an L2 writeback per record would cost ~6 us of GPU time
      // and slow the next kernel)
      if (hipEventCreateWithFlags(&e, hipEventDisableSystemFence) != hipSuccess) return nullptr;
      pool.push_back(e);
    }
    return pool[used++];
  }
  // only: a label prefix, or several separated by '|'
  bool wants(const char* label) const {
    if (!on) return false;
    const std::string l(label);
    size_t s = 0;
    while (true) {
      const size_t e = only.find('|', s);
      const std::string pre = only.substr(s, e == std::string::npos ? std::string::npos : e - s);
      if (l.rfind(pre, 0) == 0) return true;
      if (e == std::string::npos) return false;
      s = e + 1;
    }
  }
  void reset() { recs.clear(); used = 0; }
  ~Profiler() {
    for (auto e : pool) (void)hipEventDestroy(e);
  }
};

// Labelled launch timing.  Breakdown mode (all labels): hipEventRecord around the op.  Family mode (a label
// prefix, bench.py's live roofline of the conv families): the op's kernel is dispatched with the events itself
// (VAD_KLAUNCH), so the timed steps carry no extra marker packets.
#define TIMED(label, expr)                                       \
  do {                                                           \
    const bool _w = prof.wants(label);                           \
    const bool _k = _w && !prof.only.empty();                    \
    hipEvent_t _a = nullptr, _b = nullptr;                       \
    if (_w) {                                                    \
      _a = prof.get();                                           \
      _b = prof.get();                                           \
      if (_k) {                                                  \
        ktimer().a = _a;                                         \
        ktimer().b = _b;                                         \
      } else {                                                   \
        VAD_HIP(hipEventRecord(_a, st));                         \
      }                                                          \
    }                                                            \
    VAD_TRY(expr);                                               \
    if (_k) {                                                    \
      if (ktimer().a == nullptr) prof.recs.push_back({std::string(label), _a, _b}); \
      ktimer().a = ktimer().b = nullptr;                         \
    } else if (_w) {                                             \
      VAD_HIP(hipEventRecord(_b, st));                           \
      prof.recs.push_back({std::string(label), _a, _b});         \
    }                                                            \
  } while (0)

// ------------------------------------------------------------------ the plan
struct CadPlanImpl {
  int B, T, H, W, NF;
  int H1, W1, HP, WP, HF, WF;
  Conv3Layer L[8];
  int64_t ws_bytes = 0;
  // bound buffers
  float *params = nullptr, *grads = nullptr, *bufs = nullptr, *m = nullptr, *v = nullptr;
  int64_t* nbt = nullptr;
  int32_t* steps = nullptr;
  // workspace carve
  float *y1, *pool, *y[8], *stats[9], *parts, *wf[8], *wd[8], *feats, *pooled;
  __bf16* w3[8] = {};  // the pre-split Wd planes the last prep wrote (stride-2 input gradients), per layer or null
  float *poolb[2] = {nullptr, nullptr}, *stats0b[2] = {nullptr, nullptr}, *parts_stem = nullptr;
  float *dh[5], *dlog, *gh[5], *glog;
  float* wt[5] = {};  // transposed detector_net weights of layers 1-4 (mlp_tail_fwd)
  float *head_ws, *head_rows;
  int* head_iws;
  float *probs, *finalv, *causal, *kl, *z, *adj, *boxes;
  int *counts, *nmax, *clip_flags, *flags;
  // detector gate (device word): the loss tail of the forward writes 1 when no box is in range (the detector then
  // gets no gradient, cad:221-226, and its input gradient into the backbone is the zero the forward cleared) and 0
  // otherwise; the side stream writes 1 once the detector's input gradient is final.  The backbone backward waits on
  // the word (hipStreamWaitValue64) instead of on the whole causal-head backward.
  uint64_t* det_gate = nullptr;
  int grads_zeroed = 0;  // the last forward cleared the grad buffer for the backward that follows it
  float *d_causal, *d_kl, *d_glog, *d_dlog, *slabs, *d_feat_det, *d_pooled, *dense_scratch, *dense_scratch2;
  float *dg[5], *ddh[5];
  // the direct classifier's affine loss-mode backward (knob "cad_dir_affine", B <= 8): the forward with labels leaves
  // the input-gradient chain of the stacked rows [A; beta] (d_logits = A + c beta) in dl2 / dg2 / dpool2 while the side
  // stream runs the causal head; a loss-mode backward folds in c (dir_pre).  tail_pre: the forward's loss tail also
  // wrote the loss-mode upstream grads, so the backward's tail launch is skipped once.  dir_used: stage 0 took the
  // affine path (stage 1 then reads the stacked clip-mean grads).
  float *dl2 = nullptr, *dg2[4] = {}, *dpool2 = nullptr;
  int dir_pre = 0, tail_pre = 0, dir_used = 0;
  // wpart0: layer 0's split-K slab (frozen stem: its weight gradient runs on the caller's stream while the weight-gradient
  // stream may still be reducing layer 1's slab)
  float *dA, *dY, *dY2, *wpart, *wpart0, *stem_d;  // stem_d: [NF][H1][W1][32], the stem backward's dA / dY (stem_grad only)
  // per-layer dY buffers (option "dy_per_layer", default on): layer l's BN backward writes dYL[l], which only layer l's
  // weight and input gradients read, so the compute stream never waits for the weight-gradient stream to release a
  // shared dY buffer (one cross-queue barrier per layer less); ~2x the dY memory (≈210 MB at config 2)
  float* dYL[8] = {};
  int dy_per_layer = 1;
  float *sq_parts, *slot_info, *clip;
  int16_t* chunk_slot;
  int64_t parts_floats, dense_scratch_floats, wpart_floats, wpart0_floats, slab_len, act_max;
  int64_t clip0 = 0;
  // SyncBatchNorm (option): per-layer [2C] double sums are handed to the caller's callback (an all-reduce over the
  // process group) between the partial-sum reduction and the finalize, forward and backward
  vad_bn_sync_fn sync_fn = nullptr;
  void* sync_user = nullptr;
  int sync_world = 1;
  double* bnsync = nullptr;
  // backward-stage bookkeeping: forward resets it, stage 0 (or the whole backward) sets it; stage 1 requires it
  // (stage 1 reads d_feat_det / d_pooled and the zeroed grads that stage 0 leaves)
  int bwd_state = 0;
  int debug_stop_layer = -1;  // backward returns after this backbone layer (debug introspection)
  Profiler prof;
  // side stream: the detector + causal head chain runs beside the direct classifier (forward and backward); the
  // two chains share only their inputs (features / the loss tail's upstream grads) and meet again at the loss tail
  // and at the backbone backward (fork / join through events on the caller's stream)
  hipStream_t st2 = nullptr;
  hipEvent_t ev_fork = nullptr, ev_join = nullptr, ev_det = nullptr;
  // weight-gradient stream: in the backbone backward, layer l's weight gradient (+ split-K reduce) runs here
  // concurrently with its input gradient and the next layer's BN backward on the caller's stream.  dY alternates
  // between two buffers: ev_dy[b] = "dYb[b] written" (caller's stream), ev_wg[b] = "the weight gradient reading
  // dYb[b] is done" (st3)
  hipStream_t st3 = nullptr;
  hipEvent_t ev_dy[2] = {nullptr, nullptr}, ev_wg[2] = {nullptr, nullptr}, ev_wgj = nullptr, ev_prep = nullptr;
  // ev_layer[l]: every grad of backbone layer l (conv weight + bias, BN gamma / beta) is final -- recorded after the
  // layer's split-K reduce on the queue that ran it (layer 0: also after the stem backward), for per-layer
  // data-parallel gradient buckets (vad_cad_wait_layer_grads)
  hipEvent_t ev_layer[8] = {};
  // early stem (vad_cad_input_ready): the frozen stem of the armed forward runs on the weight-gradient stream (behind
  // the previous step's weight gradients of layers 7..1) once the inputs are ready (ev_input), beside what the
  // caller's stream still has queued (layer 0's weight gradient, the optimizer); its outputs (pool, bn1's state
  // stats[0]) alternate between two sets, set p free again once the backward of the forward that used it has read
  // layer 0's input (ev_stem_free[p]).  (A stream of its own measured 2x slower steps at config 2 -- 3.46 vs 1.72 ms
  // -- whatever GPU_MAX_HW_QUEUES; the side stream 1.77 ms, behind the prep's wait for the previous step)
  hipEvent_t ev_input = nullptr, ev_stem = nullptr, ev_stem_free[2] = {nullptr, nullptr};
  int input_armed = 0, spar = 0;
  int wgrad_stream = 1;  // option "wgrad_stream" (0: weight gradients on the caller's stream)
  int streams() {
    if (!st2) {
      // the plan's events only order its own queues on this device (stream waits, never host inspection): an
      // agent-scope release suffices, so the system-scope fence at each record is dropped (knob
      // "cad_event_sysfence" = 1 restores it)
      const unsigned evf = hipEventDisableTiming | (g_cad_event_sysfence ? 0u : (unsigned)hipEventDisableSystemFence);
      // knob "cad_stream_prio": the side stream (the detector / causal-head chain, on the forward's critical path) at
      // the device's greatest priority, the weight-gradient stream (slack beside the input gradients) at its least
      int lo = 0, hi = 0;
      if (g_cad_stream_prio) VAD_HIP(hipDeviceGetStreamPriorityRange(&lo, &hi));
      VAD_HIP(hipStreamCreateWithPriority(&st2, hipStreamNonBlocking, g_cad_stream_prio ? hi : 0));
      VAD_HIP(hipEventCreateWithFlags(&ev_fork, evf));
      VAD_HIP(hipEventCreateWithFlags(&ev_join, evf));
      VAD_HIP(hipEventCreateWithFlags(&ev_det, evf));
      VAD_HIP(hipStreamCreateWithPriority(&st3, hipStreamNonBlocking, g_cad_stream_prio ? lo : 0));
      for (int b = 0; b < 2; ++b) {
        VAD_HIP(hipEventCreateWithFlags(&ev_dy[b], evf));
        VAD_HIP(hipEventCreateWithFlags(&ev_wg[b], evf));
      }
      VAD_HIP(hipEventCreateWithFlags(&ev_wgj, evf));
      VAD_HIP(hipEventCreateWithFlags(&ev_prep, evf));
      for (int l = 0; l < 8; ++l) VAD_HIP(hipEventCreateWithFlags(&ev_layer[l], evf));
      VAD_HIP(hipEventCreateWithFlags(&ev_input, evf));
      VAD_HIP(hipEventCreateWithFlags(&ev_stem, evf));
      for (int b = 0; b < 2; ++b) VAD_HIP(hipEventCreateWithFlags(&ev_stem_free[b], evf));
    }
    return 0;
  }
  int fork(hipStream_t st) {
    VAD_TRY(streams());
    VAD_HIP(hipEventRecord(ev_fork, st));
    VAD_HIP(hipStreamWaitEvent(st2, ev_fork, 0));
    return 0;
  }
  // orders `st` after everything queued so far on the side stream (the stage-2 backward's head / detector grads)
  int wait_side(hipStream_t st) {
    VAD_TRY(streams());
    VAD_HIP(hipEventRecord(ev_join, st2));
    VAD_HIP(hipStreamWaitEvent(st, ev_join, 0));
    return 0;
  }
  int join(hipStream_t st) {
    VAD_HIP(hipEventRecord(ev_join, st2));
    VAD_HIP(hipStreamWaitEvent(st, ev_join, 0));
    return 0;
  }
  ~CadPlanImpl() {
    if (ev_fork) (void)hipEventDestroy(ev_fork);
    if (ev_join) (void)hipEventDestroy(ev_join);
    if (ev_det) (void)hipEventDestroy(ev_det);
    for (int b = 0; b < 2; ++b) {
      if (ev_dy[b]) (void)hipEventDestroy(ev_dy[b]);
      if (ev_wg[b]) (void)hipEventDestroy(ev_wg[b]);
    }
    if (ev_wgj) (void)hipEventDestroy(ev_wgj);
    if (ev_prep) (void)hipEventDestroy(ev_prep);
    for (int l = 0; l < 8; ++l)
      if (ev_layer[l]) (void)hipEventDestroy(ev_layer[l]);
    if (ev_input) (void)hipEventDestroy(ev_input);
    if (ev_stem) (void)hipEventDestroy(ev_stem);
    for (int b = 0; b < 2; ++b)
      if (ev_stem_free[b]) (void)hipEventDestroy(ev_stem_free[b]);
    if (st3) (void)hipStreamDestroy(st3);
    if (st2) (void)hipStreamDestroy(st2);
  }
  char lbl[64];
  const char* L_(const char* base, int l) {
    snprintf(lbl, sizeof(lbl), "%s/L%d", base, l);
    return lbl;
  }
  int training = 1;
  bool have_labels = false;
  uint64_t seed = 0, step = 0;
  const int64_t* labels = nullptr;

  // workspace carved for the options set before vad_cad_workspace_bytes: the training stem's buffers (y1, stem_d:
  // 0.2-0.5 GB at configs 2/4) only when the stem trains or the fused frozen stem cannot run, and either the per-layer
  // dY buffers or the shared pair.  A forward / backward needing a buffer the carve left out fails loudly (the Python
  // engine builds a new plan when the stem's requires_grad turns on).
  int ws_stem = 1, ws_dy_shared = 1, bound = 0;
  void carve_options() {
    ws_stem = stem_grad || !g_stem_fused || !stem_fused_ok(W1);
    ws_dy_shared = !(dy_per_layer && g_cad_dy_per_layer);
  }
  void carve(Ws& w) {
    const int64_t nf = NF;
    y1 = ws_stem ? w.take<float>(nf * H1 * W1 * 32) : nullptr;
    poolb[0] = pool = w.take<float>(nf * HP * WP * 32);
    // (the early stem's second set: only for the fused frozen stem)
    poolb[1] = ws_stem ? nullptr : w.take<float>(nf * HP * WP * 32);
    act_max = nf * HP * WP * 32;
    for (int l = 0; l < 8; ++l) {
      y[l] = w.take<float>(nf * L[l].OH * L[l].OW * L[l].Co);
      // (fp32 image + its bf16 copy: conv3_bf16_image)
      wf[l] = w.take<float>((int64_t)L[l].Co * L[l].Ci * 9 * 3 / 2);
      wd[l] = w.take<float>((int64_t)L[l].Co * L[l].Ci * 9 * 5 / 2);  // fp32 | bf16 copy or 3 bf16 planes
      act_max = std::max<int64_t>(act_max, nf * L[l].OH * L[l].OW * L[l].Co);
    }
    const int cs[9] = {32, 32, 32, 64, 64, 128, 128, 256, 256};
    for (int l = 0; l < 9; ++l) stats[l] = w.take<float>(BN_STATS_PER_C * cs[l]);
    stats0b[0] = stats[0];
    stats0b[1] = w.take<float>(BN_STATS_PER_C * 32);
    spar = 0;
    parts_floats = std::max<int64_t>((int64_t)conv1_num_parts(NF, H1) * 64, 1024);
    // (the training stem's bn1 backward reduces over all NF * H1 * W1 conv1 outputs: bn_rows_parts <= cdiv(M, 64))
    parts_floats = std::max<int64_t>(parts_floats, cdiv((int64_t)nf * H1 * W1, 64) * 2 * 32);
    for (int l = 0; l < 8; ++l) {
      const int64_t M = nf * L[l].OH * L[l].OW;
      parts_floats = std::max<int64_t>(parts_floats, cdiv(M, 64) * 2 * L[l].Co);
      parts_floats = std::max<int64_t>(parts_floats, conv3_patch_blocks(nf, L[l].OH, L[l].OW) * 2 * L[l].Co);
    }
    parts = w.take<float>(parts_floats);
    parts_stem = ws_stem ? nullptr : w.take<float>(std::max<int64_t>((int64_t)conv1_num_parts(NF, H1) * 64, 1024));
    feats = w.take<float>(nf * 6144);
    pooled = w.take<float>((int64_t)B * 6144);
    const int dd[5] = {512, 256, 128, 64, 20};
    const int gd[5] = {512, 256, 128, 64, 2};
    for (int i = 0; i < 4; ++i) dh[i] = w.take<float>(nf * dd[i]);
    dlog = w.take<float>(nf * 20);
    for (int i = 0; i < 4; ++i) gh[i] = w.take<float>((int64_t)B * gd[i]);
    glog = w.take<float>((int64_t)B * 2);
    for (int i = 1; i < 5; ++i) wt[i] = w.take<float>((int64_t)dd[i - 1] * dd[i]);
    head_ws = w.take<float>((int64_t)B * head_ws_floats(T));
    head_rows = w.take<float>(head_rows_floats(B, T));
    head_iws = w.take<int>((int64_t)B * head_iws_ints(T));
    probs = w.take<float>(B * 2);
    finalv = w.take<float>(B);
    causal = w.take<float>(B);
    kl = w.take<float>(B);
    z = w.take<float>(B * 30);
    adj = w.take<float>(B * 36);
    boxes = w.take<float>(nf * 20);
    counts = w.take<int>(nf);
    nmax = w.take<int>(B);
    clip_flags = w.take<int>(B * 2);
    flags = w.take<int>(4);
    det_gate = w.take<uint64_t>(1);
    d_causal = w.take<float>(B);
    d_kl = w.take<float>(B);
    d_glog = w.take<float>(B * 2);
    d_dlog = w.take<float>(nf * 20);
    const CadLayout& LY = layout();
    slab_len = LY.slots[LY.dir_w[0]].offset - LY.slots[LY.head0].offset;
    slabs = w.take<float>((int64_t)B * slab_len);
    d_feat_det = w.take<float>(nf * 6144);
    d_pooled = w.take<float>((int64_t)B * 6144);
    for (int i = 0; i < 4; ++i) {
      ddh[i] = w.take<float>(nf * dd[i]);
      dg[i] = w.take<float>((int64_t)B * gd[i]);
      dg2[i] = w.take<float>(2ll * B * gd[i]);
    }
    dl2 = w.take<float>(2ll * B * 2);
    dpool2 = w.take<float>(2ll * B * 6144);
    dense_scratch_floats = std::max<int64_t>(512ll * 6145, 16ll * nf * 512);
    dense_scratch_floats = std::max<int64_t>(dense_scratch_floats, 16ll * B * 512);
    dense_scratch = w.take<float>(dense_scratch_floats);
    dense_scratch2 = w.take<float>(dense_scratch_floats);  // the side stream's (detector) split-K scratch
    dA = w.take<float>(act_max);
    dY = ws_dy_shared ? w.take<float>(act_max) : nullptr;
    dY2 = ws_dy_shared ? w.take<float>(act_max) : nullptr;
    for (int l = 0; l < 8; ++l) dYL[l] = ws_dy_shared ? nullptr : w.take<float>(nf * L[l].OH * L[l].OW * L[l].Co);
    stem_d = ws_stem ? w.take<float>(nf * H1 * W1 * 32) : nullptr;
    wpart_floats = 16ll << 20;
    wpart = w.take<float>(wpart_floats);
    wpart0_floats = std::max<int64_t>(8ll << 20, (int64_t)L[0].Co * 9 * L[0].Ci);
    wpart0 = w.take<float>(wpart0_floats);
    sq_parts = w.take<float>(1024);
    bnsync = w.take<double>(2 * 256);
    slot_info = w.take<float>(4 * 160);
    clip = w.take<float>(4);
    chunk_slot = w.take<int16_t>(LY.param_floats / 256 + 1);
  }

  float* P(int slot) const { return params + layout().slots[slot].offset; }
  float* G(int slot) const { return grads + layout().slots[slot].offset; }
  float* RM(int i) const { return bufs + layout().bufs[layout().rm[i]].offset; }
  float* RV(int i) const { return bufs + layout().bufs[layout().rv[i]].offset; }

  HeadArgs head_args() const {
    const CadLayout& LY = layout();
    HeadArgs a{};
    a.B = B;
    a.T = T;
    a.clip0 = clip0;
    a.training = training;
    a.h1_eps = rng_h1(seed, S_EPS, step);
    a.h1_drop = rng_h1(seed, S_SCORER_DROP, step);
    a.thr_drop = drop_threshold(0.2);
    a.pbase = params;
    for (int i = 0; i < H_NUM; ++i) a.off[i] = LY.slots[LY.head0 + i].offset;
    a.head_begin = LY.slots[LY.head0].offset;
    int64_t numel[H_NUM];
    for (int i = 0; i < H_NUM; ++i) numel[i] = LY.slots[LY.head0 + i].numel;
    head_pack_weights(a, numel);  // sizes are fixed by the architecture; checked once in create()
    a.ws = head_ws;
    a.ws_stride = head_ws_floats(T);
    a.iws = head_iws;
    a.iws_stride = head_iws_ints(T);
    a.rows = head_rows;
    a.grad = grads;
    return a;
  }
  HeadOut head_out() const { return HeadOut{causal, kl, z, adj, boxes, counts, nmax, clip_flags}; }

  // layers 1-4 of a 5-layer MLP chain (widths wd[0..5]) on top of h[0]; layer outputs h[1..3] and the logits
  MlpTailArgs mlp_args(int M, int64_t row0, const int* wd, const int* wslot, const int* bslot, float* const* h,
                       float* logits, int drop2, float* const* wtr) const {
    MlpTailArgs m{};
    m.M = M;
    m.row0 = row0;
    for (int i = 0; i < 5; ++i) {
      const DenseAct a = act(i < 4, i == 1 ? drop2 : 0, 0.2, row0);
      MlpLayer& L = m.L[i];
      L.W = P(wslot[i]);
      L.b = P(bslot[i]);
      L.out = i < 4 ? h[i] : logits;
      L.K = wd[i];
      L.N = wd[i + 1];
      L.relu = a.relu;
      L.drop = a.drop;
      L.h1 = a.h1;
      L.thr = a.thr;
      L.dscale = a.dscale;
      m.WT[i] = i >= 1 ? wtr[i] : nullptr;
    }
    return m;
  }
  MlpTransposeArgs mlp_transpose_args() const {
    const CadLayout& LY = layout();
    const int dd[6] = {6144, 512, 256, 128, 64, 20};
    MlpTransposeArgs t{};
    for (int i = 1; i < 5; ++i, ++t.n) {
      t.W[t.n] = P(LY.det_w[i]);
      t.WT[t.n] = wt[i];
      t.K[t.n] = dd[i];
      t.N[t.n] = dd[i + 1];
    }
    return t;
  }
  // dropout after layers 0 and 1 (p = 0.3, 0.2): their gates carry the 1/(1-p) scale in training
  MlpTailBwdArgs mlp_bwd_args(int M, const float* dout, const int* wd, const int* wslot, float* const* h,
                              float* const* d, const int* skip) const {
    MlpTailBwdArgs b{};
    b.M = M;
    b.dout = dout;
    for (int i = 0; i < 5; ++i) {
      b.W[i] = P(wslot[i]);
      b.K[i] = wd[i];
      b.N[i] = wd[i + 1];
    }
    const double gp[4] = {0.3, 0.2, 0.0, 0.0};
    for (int i = 0; i < 4; ++i) {
      b.h[i] = h[i];
      b.d[i] = d[i];
      b.gscale[i] = (training && gp[i] > 0) ? (float)(1.0 / (1.0 - gp[i])) : 1.f;
    }
    b.skip = skip;
    return b;
  }
  RowsWgradArgs mlp_wgrad_args(int M, const float* dout, const int* wd, const int* wslot, const int* bslot,
                               float* const* h, float* const* d, const int* skip) const {
    RowsWgradArgs r{};
    r.R = M;
    r.nseg = 4;
    for (int i = 4; i >= 1; --i) {
      RowsWgradSeg& sg = r.seg[4 - i];
      sg.dW = G(wslot[i]);
      sg.db = G(bslot[i]);
      sg.A = i == 4 ? dout : d[i];
      sg.X = h[i - 1];
      sg.O = wd[i + 1];
      sg.I = wd[i];
    }
    r.skip = skip;
    return r;
  }

  DenseAct act(bool relu, int stream_id, double p, int64_t row0) const {
    DenseAct a;
    a.relu = relu ? 1 : 0;
    if (training && stream_id > 0) {
      a.drop = 1;
      a.h1 = rng_h1(seed, (uint32_t)stream_id, step);
      a.thr = drop_threshold(p);
      a.dscale = 1.0f / (float)(1.0 - p);
      a.row0 = row0;
    }
    return a;
  }

  int conv_bf16 = 0;  // option "conv_bf16": 3x3 convs on bf16 operands (BASELINE config 4)
  // option "act_bf16" (default on): with conv_bf16, the backbone activations (pooled stem map, conv outputs y, dA,
  // dY) are stored as bf16 -- half the bytes of every memory-bound pass. act_bf16: the last forward ran so (the
  // frozen fused stem and split kernels for every pass are required; the backward follows the forward)
  int act_bf16_opt = 1, act_bf16 = 0;
  // option "stem_grad": backbone.conv1 / bn1 train (the reference's module without apply_memory_efficient_training);
  // stem_active: the last backward wrote their grads (the fused optimizer then steps them too)
  int stem_grad = 0, stem_active = 0;
  int y1_fresh = 0;  // the last forward wrote conv1's output y1 (the stem backward reads it)
  // BN state layer1.0 applies on load to `pool`: bn1's (fused stem: `pool` holds the raw pooled conv1 output) or none
  const float* pool_stats = nullptr;

  // batch statistics of BN layer i (0 = bn1) from the `np` partials in `parts`: local (default) or, with a sync
  // callback in training mode, over the whole process group (torch.nn.SyncBatchNorm semantics)
  int bn_fwd_stats(int i, int np, int C, double count, const float* gamma, const float* beta, hipStream_t st,
                   int cm = 0, const float* pparts = nullptr) {
    if (sync_fn == nullptr || !training) {
      TIMED("bn_fin", bn_finalize(pparts ? pparts : parts, np, C, count, gamma, beta, RM(i), RV(i), 0.1f, 1e-5f, training, stats[i],
                                  st, cm));
      return 0;
    }
    TIMED("bn_fin", bn_sum_partials(parts, np, C, bnsync, nullptr, nullptr, st, cm));
    VAD_CHECK(sync_fn(sync_user, i, 0, 2 * C, st) == 0, "BatchNorm sync callback failed (forward)");
    TIMED("bn_fin", bn_finalize_sums(bnsync, C, count * sync_world, gamma, beta, RM(i), RV(i), 0.1f, 1e-5f, stats[i],
                                     st));
    return 0;
  }
  // backward of BN layer i: dgamma/dbeta from this rank's sums (the grad all-reduce adds the ranks), the mean terms
  // from the group's sums when synchronised; the partials are column-major [2C][P] (bn_bwd_reduce with cm = 1)
  int bn_bwd_stats(int i, int np, int C, double count, const float* gamma, float* dgamma, float* dbeta,
                   float* dbias, hipStream_t st) {
    if (sync_fn == nullptr || !training) {
      TIMED("bn_bwd_fin", bn_bwd_finalize(parts, np, C, count, gamma, stats[i], dgamma, dbeta, training, st, dbias,
                                          1));
      return 0;
    }
    TIMED("bn_bwd_fin", bn_sum_partials(parts, np, C, bnsync, dbeta, dgamma, st, 1));
    VAD_CHECK(sync_fn(sync_user, i, 1, 2 * C, st) == 0, "BatchNorm sync callback failed (backward)");
    TIMED("bn_bwd_fin", bn_bwd_finalize_sums(bnsync, C, count * sync_world, gamma, stats[i], st, dbias));
    return 0;
  }

  const float* x_last = nullptr;  // the last forward's input (the stem backward's conv1 weight gradient reads it)

  int forward(const float* x, hipStream_t st) {
    const hipStream_t st0 = st;
    VAD_TRY(join_open_stage2(st));
    ConvPrecision prec(conv_bf16);
    x_last = x;
    const CadLayout& LY = layout();
    y1_fresh = !(g_stem_fused && !stem_grad && stem_fused_ok(W1));
    VAD_CHECK(!y1_fresh || y1, "forward: the workspace was carved without the training stem's buffers (option stem_grad "
                               "or knob stem_fused changed after vad_cad_bind): create a new plan");
    act_bf16 = conv_bf16 && act_bf16_opt && !y1_fresh;
    for (int l = 0; l < 8; ++l) act_bf16 = act_bf16 && conv3_act_bf16_ok(L[l], l > 0);
    ActStorage abf(act_bf16);
    // weight relayouts (conv images -- with bf16 storage also their bf16 copies --, the detector's transposed layers)
    // on the side stream, beside the stem
    VAD_TRY(fork(st));
    {
      hipStream_t st = g_cad_prep_stream ? st2 : st0;
      const float* w8[8];
      for (int l = 0; l < 8; ++l) w8[l] = P(LY.conv_w[l]);
      for (int l = 0; l < 8; ++l)
        w3[l] = conv3_dgrad_w3_wanted(L[l]) ? reinterpret_cast<__bf16*>(wd[l] + (int64_t)L[l].Co * L[l].Ci * 9) : nullptr;
      TIMED("prep", conv3_prep_weights_all(8, w8, L, wf, wd, st, w3));
      TIMED("prep", mlp_transpose(mlp_transpose_args(), st));
      VAD_HIP(hipEventRecord(ev_prep, st));
    }
    int np = 0;
    bwd_state = 0;
    // early stem: armed by vad_cad_input_ready, frozen fused stem, per-rank BN statistics
    const bool early = g_cad_stem_early && input_armed && !y1_fresh && poolb[1] && (sync_fn == nullptr || !training);
    // (armed but not early: the inputs may still be in flight on the arming stream, so the stem waits for them)
    if (input_armed && !early) VAD_HIP(hipStreamWaitEvent(st0, ev_input, 0));
    input_armed = 0;
    if (early) {
      spar ^= 1;
      pool = poolb[spar];
      stats[0] = stats0b[spar];
    }
    if (!y1_fresh) {
      // frozen stem (the training default): conv1 + BN sums + pooling of the raw output in one pass (stem.hip);
      // `pool` then holds the pooled conv1 output and layer1.0 applies bn1 + ReLU on load
      hipStream_t st = early ? st3 : st0;
      float* sp = early ? parts_stem : parts;
      if (early) {
        VAD_HIP(hipStreamWaitEvent(st, ev_input, 0));
        VAD_HIP(hipStreamWaitEvent(st, ev_stem_free[spar], 0));
      }
      TIMED("conv1", stem_fused(x, NF, H, W, P(LY.conv1_w), P(LY.conv1_b), P(LY.bn1_w), H1, W1, pool, HP, WP, sp,
                                &np, st));
      VAD_TRY(bn_fwd_stats(0, np, 32, (double)NF * H1 * W1, P(LY.bn1_w), P(LY.bn1_b), st, 1, sp));  // column-major
      if (early) {
        VAD_HIP(hipEventRecord(ev_stem, st));
        VAD_HIP(hipStreamWaitEvent(st0, ev_stem, 0));
      }
      pool_stats = stats[0];
    } else {
      // training stem: the backward's MaxPool / bn1 / conv1 gradients read conv1's output y1
      TIMED("conv1", conv1_fwd(x, NF, H, W, P(LY.conv1_w), P(LY.conv1_b), y1, H1, W1, parts, &np, st));
      VAD_TRY(bn_fwd_stats(0, np, 32, (double)NF * H1 * W1, P(LY.bn1_w), P(LY.bn1_b), st));
      TIMED("maxpool", maxpool3s2_bnrelu(y1, stats[0], NF, H1, W1, 32, pool, HP, WP, st));
      pool_stats = nullptr;
    }
    VAD_HIP(hipStreamWaitEvent(st, ev_prep, 0));  // layer1.0 reads the prepared weight images
    const float* src = pool;
    const float* sst = pool_stats;
    for (int l = 0; l < 8; ++l) {
      int cm = 1;  // the split kernels write the partials column-major (coalesced finalize reads)
      TIMED(L_("conv_fwd", l), conv3_fwd(L[l], src, sst, wf[l], P(LY.conv_b[l]), y[l], parts, &np, st, &cm));
      VAD_TRY(bn_fwd_stats(l + 1, np, L[l].Co, (double)NF * L[l].OH * L[l].OW, P(LY.bn_w[l]), P(LY.bn_b[l]), st, cm));
      src = y[l];
      sst = stats[l + 1];
    }
    TIMED("avgpool", avgpool_fwd(y[7], stats[8], B, T, HF, WF, 256, feats, pooled, st));
    const int64_t f0 = clip0 * T;
    const int dd[6] = {6144, 512, 256, 128, 64, 20};
    const int gd[6] = {6144, 512, 256, 128, 64, 2};
    // The detector + causal head chain (the longer one, which the loss tail waits for) stays on the caller's stream,
    // the direct classifier and the buffer clears go to the side stream: a cross-stream hand-off costs ~8 us from the
    // producer's end to the consumer's start (tools/exp/xstream_probe.hip), a same-stream one ~1 us, so only the
    // shorter chain pays the fork and the join finds it finished
    VAD_TRY(fork(st));
    dir_pre = tail_pre = 0;
    // (train-mode forwards with grads bound only: an eval / probe forward with labels is followed by no loss backward)
    const bool affine = labels != nullptr && training && grads != nullptr && g_cad_dir_affine != 0 && B <= 8;
    {  // side stream: direct_classifier on the mean over T (cad:525-538, 568-570)
      // (B rows only: one block per 64 columns, so the chain runs layer by layer on many CUs; layers 1-4 unsplit)
      // With labels (and B <= 8) layers 2-4 run in dir_mid together with the loss-mode input-gradient chain of the
      // stacked rows [A; beta], layers 1 and 0 of that chain follow: the backward then only folds in the causal score
      hipStream_t st = st2;
      const float* in = pooled;
      for (int i = 0; i < (affine ? 2 : 5); ++i) {
        float* out = i < 4 ? gh[i] : glog;
        const int sid = i == 0 ? S_DIRECT_DROP1 : (i == 1 ? S_DIRECT_DROP2 : 0);
        TIMED("dir_fwd", dense_fwd(in, B, gd[i], P(LY.dir_w[i]), P(LY.dir_b[i]), gd[i + 1], out,
                                   act(i < 4, sid, i == 0 ? 0.3 : 0.2, clip0), dense_scratch, dense_scratch_floats, st,
                                   i == 0 ? 0 : 1));
        in = out;
      }
      if (affine) {
        const float gs0 = training ? (float)(1.0 / (1.0 - 0.3)) : 1.f;
        const float gs1 = training ? (float)(1.0 / (1.0 - 0.2)) : 1.f;
        DirMidArgs da{};
        da.B = B;
        da.h0 = gh[0];
        da.h1 = gh[1];
        da.W1 = P(LY.dir_w[1]);
        da.W2 = P(LY.dir_w[2]); da.b2 = P(LY.dir_b[2]);
        da.W3 = P(LY.dir_w[3]); da.b3 = P(LY.dir_b[3]);
        da.W4 = P(LY.dir_w[4]); da.b4 = P(LY.dir_b[4]);
        da.h2 = gh[2]; da.h3 = gh[3]; da.logits = glog;
        da.labels = labels;
        da.gs0 = gs0;
        da.gs1 = gs1;
        da.dl2 = dl2; da.d3 = dg2[3]; da.d2 = dg2[2]; da.d1 = dg2[1]; da.d0 = dg2[0];
        TIMED("dir_fwd", dir_mid(da, st));
        TIMED("dir_pre", dense_dgrad(dg2[0], 2 * B, 512, P(LY.dir_w[0]), 6144, dpool2, nullptr, 1.f, nullptr, st));
        dir_pre = tail_pre = 1;
      }
      // the detector's input gradient buffer is zero unless its backward writes it (the backward skips it on device
      // when no box was in range)
      VAD_HIP(hipMemsetAsync(d_feat_det, 0, sizeof(float) * (size_t)NF * 6144, st));
      // (train mode: the backward's grad buffer is cleared here too, off its critical path; the backward clears it
      // itself when the forward did not)
      grads_zeroed = 0;
      if (training && grads) {
        VAD_HIP(hipMemsetAsync(grads, 0, sizeof(float) * layout().param_floats, st));
        grads_zeroed = 1;
      }
    }
    // caller's stream: detector_net (cad:167-179; layer 0 as a split-K GEMM, layers 1-4 fused per row block), then
    // the causal head on the detections
    // (layer 0's split-K partials are summed and finished inside the layer 1-4 kernel: one launch less)
    {
      int ns = 0;
      TIMED("det_fwd", dense_fwd_splitk(feats, NF, 6144, P(LY.det_w[0]), 512, dense_scratch2, dense_scratch_floats,
                                        &ns, st));
      MlpTailArgs m = mlp_args(NF, f0, dd, LY.det_w, LY.det_b, dh, dlog, S_DET_DROP2, wt);
      const DenseAct a0 = act(true, S_DET_DROP1, 0.3, f0);
      m.L[0].relu = a0.relu;
      m.L[0].drop = a0.drop;
      m.L[0].h1 = a0.h1;
      m.L[0].thr = a0.thr;
      m.L[0].dscale = a0.dscale;
      m.parts = dense_scratch2;
      m.nsplit = ns;
      TIMED("det_fwd", mlp_tail_fwd(m, st));
    }
    TIMED("head_rows", head_rows_fwd(head_args(), dlog, head_out(), st));
    TIMED("head_seq", head_seq_fwd(head_args(), head_out(), st));
    VAD_TRY(join(st));
    TailArgs t = tail_args(nullptr, nullptr, nullptr, nullptr);
    t.fwd_bwd = tail_pre;
    if (training && nbt) {  // num_batches_tracked of the 9 BN layers (bumped by the tail kernel)
      t.nbt = nbt;
      t.nbt_n = 9;
    }
    TIMED("tail", cad_tail_fwd(t, st));
    return 0;
  }

  TailArgs tail_args(const float* dfin, const float* dprobs, const float* dcaus, const float* dkl) const {
    TailArgs t{};
    t.B = B;
    t.direct_logits = glog;
    t.causal = causal;
    t.kl = kl;
    t.clip_flags = clip_flags;
    t.probs = probs;
    t.final_scores = finalv;
    t.flags = flags;
    t.det_gate = det_gate;
    t.flags_f = grads ? grads + layout().param_floats : nullptr;
    t.labels = labels;
    t.losses = losses_ptr;
    t.ext_d_final = dfin;
    t.ext_d_probs = dprobs;
    t.ext_d_causal = dcaus;
    t.ext_d_kl = dkl;
    t.d_causal = d_causal;
    t.d_kl = d_kl;
    t.d_direct_logits = d_glog;
    return t;
  }
  float* losses_ptr = nullptr;

  // stage -1: the whole backward.  stage 0: loss tail, causal head, direct classifier and detector (every
  // non-backbone grad is final when it returns); stage 1: the backbone.  Splitting lets a data-parallel caller
  // all-reduce the head grads while the backbone backward runs.
  int backward(bool use_loss, const float* dfin, const float* dprobs, const float* dcaus, const float* dkl,
               const float* dz, const float* dadj, hipStream_t st, int stage = -1, const float* dboxes = nullptr) {
    ConvPrecision prec(conv_bf16);
    ActStorage abf(act_bf16);
    const CadLayout& LY = layout();
    VAD_CHECK(grads != nullptr, "backward: grads not bound");
    VAD_CHECK(!use_loss || labels != nullptr, "backward(use_loss): forward ran without labels");
    VAD_CHECK(stage >= -1 && stage <= 2, "backward: stage must be -1, 0, 1 or 2");
    VAD_CHECK(bwd_state != 0 || stage != 1, "backward stage 1: stage 0 has not run for the current forward");
    // detector gate: knob "cad_det_gate" (0: the backbone waits for the side stream's event as before)
    const bool gate = g_cad_det_gate != 0 && det_gate != nullptr;
    if (stage != 1) {
    // grads of frozen / never-used slots stay zero
    if (!grads_zeroed) VAD_HIP(hipMemsetAsync(grads, 0, sizeof(float) * LY.param_floats, st));
    grads_zeroed = 0;
    TailArgs t = use_loss ? tail_args(nullptr, nullptr, nullptr, nullptr) : tail_args(dfin, dprobs, dcaus, dkl);
    if (!use_loss) t.labels = nullptr;
    // (the forward's loss tail already wrote the loss-mode upstream grads and armed the gate: skipped once)
    if (!(use_loss && tail_pre)) TIMED("tail", cad_tail_bwd(t, st));
    tail_pre = 0;
    const bool aff = use_loss && dir_pre;
    dir_used = aff ? 1 : 0;
    const int gd[6] = {6144, 512, 256, 128, 64, 2};
    const int dd[6] = {6144, 512, 256, 128, 64, 20};
    VAD_TRY(fork(st));
    {  // side stream: causal head backward, then the detector chain (skipped on device when no box was in range: no
       // grads reach it, cad:221-226)
      hipStream_t st = st2;
      HeadUp up{d_causal, d_kl, dz, dadj, dboxes};
      TIMED("head_bwd", head_bwd(head_args(), dlog, head_out(), up, slabs, slab_len, d_dlog, st));
    }
    // direct classifier chain (B rows): per-layer input-gradient GEMMs spread over many CUs, the layer 1-4 weight
    // grads in one launch, layer 0 GEMMs.  (Affine path: the forward ran the input-gradient chain; the weight grads
    // follow the detector chain on the side stream.)
    if (!aff) {
      const double gp[4] = {0.3, 0.2, 0.0, 0.0};
      const float* dcur = d_glog;
      for (int i = 4; i >= 1; --i) {
        const float gs = (training && gp[i - 1] > 0) ? (float)(1.0 / (1.0 - gp[i - 1])) : 1.f;
        TIMED("dir_bwd", dense_dgrad(dcur, B, gd[i + 1], P(LY.dir_w[i]), gd[i], dg[i - 1], gh[i - 1], gs, nullptr,
                                     st));
        dcur = dg[i - 1];
      }
      TIMED("dir_bwd", rows_wgrad(mlp_wgrad_args(B, d_glog, gd, LY.dir_w, LY.dir_b, gh, dg, nullptr), st));
      TIMED("dir_bwd", dense_wgrad(dg[0], B, 512, pooled, 6144, G(LY.dir_w[0]), G(LY.dir_b[0]), dense_scratch,
                                   dense_scratch_floats, nullptr, st));
      TIMED("dir_bwd", dense_dgrad(dg[0], B, 512, P(LY.dir_w[0]), 6144, d_pooled, nullptr, 1.f, nullptr, st));
    }
    // side stream, continued: the detector chain (it feeds the backbone: event ev_det / the gate word), then the
    // head's weight grads, which only the optimizer / the grad all-reduce wait for.  (It must be queued BEFORE the
    // compute stream's wait on the gate: streams share a few hardware queues, and a wait queued ahead of the work
    // that releases it on the same hardware queue never completes -- measured: a hang in the forced regime.)
    VAD_TRY(side_det_chain(st2));
    if (aff) {  // the stacked rows folded with the causal score, then the classifier's weight grads (side stream)
      hipStream_t st = st2;
      DirCombineArgs ca{};
      ca.B = B;
      ca.c = causal;
      // (four segments: the clip-mean grads are not folded here -- stage 1's avgpool_bwd reads dpool2 + c dpool2[B:]
      // itself, so d_pooled is not written on this path; debug_buffer "d_pooled" is the non-affine path's)
      ca.nseg = 4;
      for (int i = 0; i < 4; ++i) {
        ca.src[i] = dg2[i];
        ca.dst[i] = dg[i];
        ca.width[i] = gd[i + 1];
      }
      TIMED("dir_bwd", dir_combine(ca, st));
      TIMED("dir_bwd", rows_wgrad(mlp_wgrad_args(B, d_glog, gd, LY.dir_w, LY.dir_b, gh, dg, nullptr), st));
      TIMED("dir_bwd", dense_wgrad(dg[0], B, 512, pooled, 6144, G(LY.dir_w[0]), G(LY.dir_b[0]), dense_scratch,
                                   dense_scratch_floats, nullptr, st));
    }
    // stage 0: every non-backbone grad is final on the caller's stream when it returns.  Stage 2 (= stage 0 for a
    // caller that orders its own consumer after the side stream with vad_cad_wait_side): the head / detector chain
    // keeps running on the side stream and the backbone (stage 1) waits only for the detector input gradient
    if (stage == 0) VAD_TRY(join(st));
    else if (gate) VAD_HIP(hipStreamWaitValue64(st, det_gate, 1, hipStreamWaitValueEq, ~0ull));
    else VAD_HIP(hipStreamWaitEvent(st, ev_det, 0));
    }
    if (stage != 1) bwd_state = stage == 2 ? 2 : 1;
    if (stage == 0 || stage == 2) return 0;
    // backbone (BatchNorm backward as streaming passes: the conv kernels are MFMA/LDS-bound and slowed down more by
    // extra loads than the separate 6 TB/s passes cost -- DESIGN.md §6, BN-backward fusion experiment)
    if (dir_used)  // clip-mean grads A + c beta, folded while spreading them over the map
      TIMED("avgpool_bwd", avgpool_bwd(d_feat_det, dpool2, B, T, HF, WF, 256, dA, st, dpool2 + (int64_t)B * 6144,
                                       causal));
    else
      TIMED("avgpool_bwd", avgpool_bwd(d_feat_det, d_pooled, B, T, HF, WF, 256, dA, st));
    VAD_TRY(streams());
    const bool wgs = wgrad_stream != 0 && g_cad_wgrad_stream;
    bool st3_joined = false;
    int fused_np = 0;  // layer l's BN-backward partial sums, already written by layer l+1's input gradient
    for (int l = 7; l >= 0; --l) {
      const int64_t M = (int64_t)NF * L[l].OH * L[l].OW;
      const int C = L[l].Co;
      int np = fused_np, nb = 0;
      const bool perl = dy_per_layer != 0 && g_cad_dy_per_layer != 0;
      float* dYl = perl ? dYL[l] : ((l & 1) ? dY2 : dY);
      VAD_CHECK(dYl != nullptr, "backward: dY buffers carved for the other dy_per_layer setting: create a new plan");
      VAD_CHECK((int64_t)bn_rows_parts((int)M, C) * 2 * C <= parts_floats, "backward: BN partial buffer too small");
      if (np == 0) TIMED(L_("bn_bwd_reduce", l), bn_bwd_reduce(dA, y[l], stats[l + 1], (int)M, C, parts, &np, st, 1));
      VAD_TRY(bn_bwd_stats(l + 1, np, C, (double)M, P(LY.bn_w[l]), G(LY.bn_w[l]), G(LY.bn_b[l]), G(LY.conv_b[l]), st));
      // dYl was last read by layer l+2's weight gradient
      if (wgs && l + 2 <= 7 && !perl) VAD_HIP(hipStreamWaitEvent(st, ev_wg[l & 1], 0));
      TIMED(L_("bn_bwd_apply", l), bn_bwd_apply(dA, y[l], stats[l + 1], (int)M, C, dYl, nullptr, &nb, st));
      const float* src = l == 0 ? pool : y[l - 1];
      const float* sst = l == 0 ? pool_stats : stats[l];
      {
        // layer 0 with the frozen stem: nothing follows its weight gradient on the caller's stream, so it runs there
        // (after layer 1's weight gradient has released the slab) -- no cross-queue hand-off of dY0 and no join
        // behind it before the optimizer
        const bool on_main = wgs && l == 0 && !stem_grad && g_cad_last_wgrad_main;
        hipStream_t wst = st;
        if (wgs && !on_main) {
          VAD_HIP(hipEventRecord(ev_dy[l & 1], st));
          VAD_HIP(hipStreamWaitEvent(st3, ev_dy[l & 1], 0));
          wst = st3;
        }
        // layer 0 on the caller's stream: on a slab of its own (knob cad_l0_slab) it starts right after its BN backward,
        // beside the end of layer 1's weight gradient (the stream join after the loop orders the optimizer after both);
        // on the shared slab it waits for layer 1's slab reduce
        const bool own = on_main && g_cad_l0_slab;
        if (on_main && !own) {
          VAD_HIP(hipStreamWaitEvent(st, ev_wg[1], 0));  // layer 1's weight gradient + slab reduce are done
          st3_joined = true;  // (the weight-gradient stream's last work)
        }
        float* slab = own ? wpart0 : wpart;
        const int64_t slab_cap = own ? wpart0_floats : wpart_floats;
        hipStream_t st = wst;
        int ns = 0;
        // (layer 0 with the frozen stem: little runs beside its weight gradient)
        TIMED(L_("conv_wgrad", l), conv3_wgrad(L[l], dYl, src, sst, slab, &ns, slab_cap, st, l == 0 && !stem_grad));
        TIMED(L_("wgrad_reduce", l), conv3_wgrad_reduce(L[l], slab, ns, nullptr, 0, G(LY.conv_w[l]), nullptr, st));
        if (wgs && !on_main) VAD_HIP(hipEventRecord(ev_wg[l & 1], st));
        // (layer 0: recorded after the join below -- its data-parallel bucket also holds layers 1-3, whose weight
        // gradients may still run on the weight-gradient stream when layer 0's runs on the caller's)
        if (l > 0) VAD_HIP(hipEventRecord(ev_layer[l], st));
        if (l == 0) VAD_HIP(hipEventRecord(ev_stem_free[spar], st));  // (layer 0's input read: set spar free)
      }
      fused_np = 0;
      if (l > 0) {
        // its epilogue also reduces layer l-1's BN backward (dZ = dA masked by layer l-1's ReLU, dZ * xhat)
        const BnBwdFuse fu{y[l - 1], stats[l], parts, parts_floats, &fused_np};
        TIMED(L_("conv_dgrad", l), conv3_dgrad(L[l], dYl, wd[l], dA, st, &fu, w3[l]));
      }
      if (l == debug_stop_layer) break;
    }
    if (wgs && !st3_joined) {  // every weight gradient is final before the stem backward / optimizer
      VAD_HIP(hipEventRecord(ev_wgj, st3));
      VAD_HIP(hipStreamWaitEvent(st, ev_wgj, 0));
    }
    // frozen stem: every backbone grad is final on the caller's stream here (the stem's own are recorded below)
    if (!stem_grad) VAD_HIP(hipEventRecord(ev_layer[0], st));
    stem_active = 0;
    if (stem_grad && debug_stop_layer < 0) {
      VAD_CHECK(y1_fresh, "stem backward: the forward ran with the stem frozen (set option stem_grad before it)");
      // the stem (cad:145-147): input gradient of layer1.0 into the pooled map, MaxPool2d backward, bn1 backward (in
      // place), conv1 weight gradient (its bias gradient comes from the bn1 finalize)
      TIMED("stem_bwd", conv3_dgrad(L[0], (dy_per_layer && g_cad_dy_per_layer) ? dYL[0] : dY, wd[0], dA, st));
      TIMED("stem_bwd", maxpool3s2_bwd(y1, stats[0], dA, NF, H1, W1, 32, HP, WP, stem_d, st));
      const int64_t M1 = (int64_t)NF * H1 * W1;
      int np = 0;
      VAD_CHECK((int64_t)bn_rows_parts((int)M1, 32) * 64 <= parts_floats, "stem backward: BN partial buffer too small");
      TIMED("stem_bwd", bn_bwd_reduce(stem_d, y1, stats[0], (int)M1, 32, parts, &np, st, 1));
      VAD_TRY(bn_bwd_stats(0, np, 32, (double)M1, P(LY.bn1_w), G(LY.bn1_w), G(LY.bn1_b), G(LY.conv1_b), st));
      TIMED("stem_bwd", bn_bwd_apply_inplace(stem_d, y1, stats[0], (int)M1, 32, st));
      TIMED("stem_bwd", conv1_wgrad(x_last, NF, H, W, stem_d, H1, W1, wpart, wpart_floats, G(LY.conv1_w), st));
      stem_active = 1;
      VAD_HIP(hipEventRecord(ev_layer[0], st));  // (layer 0's bucket holds the stem's grads too)
    }
    if (stage == -1 || bwd_state == 2) {
      VAD_TRY(join(st));  // the head's weight grads (side stream)
      bwd_state = 1;      // (joined: a following forward / optimizer step need not join again)
    }
    return 0;
  }
  // a stage-2 backward leaves the head / detector grads running on the side stream until stage 1 joins them; a forward
  // or an optimizer step issued without stage 1 must not overwrite what that work still reads or writes
  int join_open_stage2(hipStream_t st) {
    if (bwd_state == 2) {
      VAD_TRY(join(st));
      bwd_state = 1;
    }
    return 0;
  }

  // the detector's backward (input gradient first: the backbone waits for d_feat_det; its weight grads after it)
  // and the head's weight-grad reductions, on the side stream
  int side_det_chain(hipStream_t st) {
    const CadLayout& LY = layout();
    const int dd[6] = {6144, 512, 256, 128, 64, 20};
    const bool gate = g_cad_det_gate != 0 && det_gate != nullptr;
    TIMED("det_bwd", mlp_tail_bwd(mlp_bwd_args(NF, d_dlog, dd, LY.det_w, dh, ddh, flags), st));
    TIMED("det_bwd", dense_dgrad(ddh[0], NF, 512, P(LY.det_w[0]), 6144, d_feat_det, nullptr, 1.f, flags, st));
    VAD_HIP(hipEventRecord(ev_det, st));
    if (gate) VAD_HIP(hipStreamWriteValue64(st, det_gate, 1, 0));
    TIMED("det_bwd", rows_wgrad(mlp_wgrad_args(NF, d_dlog, dd, LY.det_w, LY.det_b, dh, ddh, flags), st));
    TIMED("det_bwd", dense_wgrad(ddh[0], NF, 512, feats, 6144, G(LY.det_w[0]), G(LY.det_b[0]), dense_scratch2,
                                 dense_scratch_floats, flags, st));
    TIMED("head_bwd", head_slab_reduce(slabs, B, slab_len, grads + LY.slots[LY.head0].offset, st));
    TIMED("head_bwd", head_rows_wgrad(head_args(), st));
    return 0;
  }

  int optimizer(float lr, float b1, float b2, float eps, float wd_, float max_norm, float gscale, float* tn,
                hipStream_t st) {
    const CadLayout& LY = layout();
    VAD_CHECK(m && v && steps, "optimizer: state buffers not bound");
    VAD_TRY(join_open_stage2(st));
    const bool pw = prof.wants("optimizer");
    hipEvent_t pa = nullptr, pb = nullptr;
    if (pw) {
      pa = prof.get();
      pb = prof.get();
      VAD_HIP(hipEventRecord(pa, st));
    }
    SlotTab tab{};
    tab.nslots = (int)LY.slots.size();
    VAD_CHECK(tab.nslots <= 160, "too many slots");
    for (int i = 0; i < tab.nslots; ++i) {
      tab.off[i] = LY.slots[i].offset;
      tab.group[i] = LY.slots[i].group;
    }
    const int nb = 1024;  // (<= the 1024-float sq_parts)
    hipLaunchKernelGGL(sqsum_kernel, dim3(nb), dim3(256), 0, st, grads, chunk_slot, LY.param_floats / 256, tab,
                       grads + LY.param_floats, gscale, sq_parts, stem_active);
    VAD_LAUNCH_CHECK();
    hipLaunchKernelGGL(opt_prepare_kernel, dim3(1), dim3(256), 0, st, sq_parts, nb, grads + LY.param_floats, tab,
                       steps, b1, b2, max_norm, slot_info, clip, tn, stem_active);
    VAD_LAUNCH_CHECK();
    const int64_t nchunks = LY.param_floats / 256;
    hipLaunchKernelGGL(adamw_kernel, dim3((unsigned)std::min<int64_t>(nchunks, 4096)), dim3(256), 0, st, params,
                       grads, m, v, chunk_slot, nchunks, slot_info, clip, gscale, lr, b1, b2, eps, wd_);
    VAD_LAUNCH_CHECK();
    if (pw) {
      VAD_HIP(hipEventRecord(pb, st));
      prof.recs.push_back({"optimizer", pa, pb});
    }
    return 0;
  }
};

}  // namespace vad

struct vad_cad_plan {
  vad::CadPlanImpl impl;
  std::vector<int16_t> chunk_host;
  bool chunk_uploaded = false;
};

using namespace vad;

extern "C" {

int vad_abi_version(void) { return VAD_ABI_VERSION; }
const char* vad_last_error(void) { return vad::last_error(); }

int vad_rng_u24(uint64_t seed, uint32_t stream_id, uint64_t step, int64_t row0, int64_t nrows, int64_t ncols,
                uint32_t* out, void* stream) {
  const int64_t total = nrows * ncols;
  if (total <= 0) return 0;
  hipLaunchKernelGGL(rng_u24_kernel, dim3((unsigned)std::min<int64_t>(cdiv(total, 256), 4096)), dim3(256), 0,
                     (hipStream_t)stream, rng_h1(seed, stream_id, step), row0, nrows, ncols, out);
  VAD_LAUNCH_CHECK();
  return 0;
}

int vad_synth_frames(uint64_t seed, uint64_t step, int64_t frame0, int64_t nframes, int64_t npix, int mode,
                     float* out, void* stream) {
  const int64_t total = nframes * npix;
  if (total <= 0) return 0;
  hipLaunchKernelGGL(synth_kernel, dim3((unsigned)std::min<int64_t>(cdiv(total, 256), 8192)), dim3(256), 0,
                     (hipStream_t)stream, rng_h1(seed, S_INPUT, step), frame0, nframes, npix, mode, out);
  VAD_LAUNCH_CHECK();
  return 0;
}

int vad_cad_num_slots(void) { return (int)layout().slots.size(); }
const char* vad_cad_slot_name(int i) {
  return (i >= 0 && i < vad_cad_num_slots()) ? layout().slots[i].name.c_str() : nullptr;
}
int64_t vad_cad_slot_numel(int i) { return (i >= 0 && i < vad_cad_num_slots()) ? layout().slots[i].numel : -1; }
int64_t vad_cad_slot_offset(int i) { return (i >= 0 && i < vad_cad_num_slots()) ? layout().slots[i].offset : -1; }
int vad_cad_slot_group(int i) { return (i >= 0 && i < vad_cad_num_slots()) ? layout().slots[i].group : -1; }
int64_t vad_cad_param_floats(void) { return layout().param_floats; }
int vad_cad_num_bufs(void) { return (int)layout().bufs.size(); }
const char* vad_cad_buf_name(int i) {
  return (i >= 0 && i < vad_cad_num_bufs()) ? layout().bufs[i].name.c_str() : nullptr;
}
int64_t vad_cad_buf_numel(int i) { return (i >= 0 && i < vad_cad_num_bufs()) ? layout().bufs[i].numel : -1; }
int64_t vad_cad_buf_offset(int i) { return (i >= 0 && i < vad_cad_num_bufs()) ? layout().bufs[i].offset : -1; }
int64_t vad_cad_buf_floats(void) { return layout().buf_floats; }
int vad_cad_num_bn(void) { return 9; }

int vad_cad_create(int B, int T, int H, int W, vad_cad_plan** out) {
  VAD_CHECK(out != nullptr, "vad_cad_create: out is null");
  VAD_CHECK(B >= 1 && T >= 1 && T <= 256 && H >= 16 && W >= 16, "vad_cad_create: unsupported shape");
  {
    HeadArgs probe{};
    int64_t numel[H_NUM];
    for (int i = 0; i < H_NUM; ++i) numel[i] = layout().slots[layout().head0 + i].numel;
    VAD_CHECK(head_pack_weights(probe, numel) == 0, "vad_cad_create: head weight image exceeds its LDS capacity");
  }
  auto* p = new vad_cad_plan();
  CadPlanImpl& c = p->impl;
  c.B = B; c.T = T; c.H = H; c.W = W; c.NF = B * T;
  c.H1 = (H - 1) / 2 + 1; c.W1 = (W - 1) / 2 + 1;
  c.HP = (c.H1 - 1) / 2 + 1; c.WP = (c.W1 - 1) / 2 + 1;
  const int cin[8] = {32, 32, 32, 64, 64, 128, 128, 256};
  const int cout[8] = {32, 32, 64, 64, 128, 128, 256, 256};
  const int strd[8] = {1, 1, 2, 1, 2, 1, 2, 1};
  int h = c.HP, w = c.WP;
  for (int l = 0; l < 8; ++l) {
    const int oh = (h - 1) / strd[l] + 1, ow = (w - 1) / strd[l] + 1;
    c.L[l] = Conv3Layer{c.NF, cin[l], cout[l], h, w, oh, ow, strd[l]};
    h = oh;
    w = ow;
  }
  c.HF = h; c.WF = w;
  const CadLayout& LY = layout();
  p->chunk_host.assign(LY.param_floats / 256 + 1, (int16_t)-1);
  for (int i = 0; i < (int)LY.slots.size(); ++i) {
    const auto& s = LY.slots[i];
    for (int64_t q = s.offset / 256; q < cdiv(s.offset + s.numel, 256); ++q) p->chunk_host[q] = (int16_t)i;
  }
  *out = p;
  return 0;
}

void vad_cad_destroy(vad_cad_plan* plan) { delete plan; }

int64_t vad_cad_workspace_bytes(const vad_cad_plan* plan) {
  if (!plan) return -1;
  CadPlanImpl& c = const_cast<vad_cad_plan*>(plan)->impl;
  if (!c.bound) {  // sized for the options set so far (carve_options); fixed once bound
    c.carve_options();
    Ws ws;
    c.carve(ws);
    c.ws_bytes = ws.off + 256;
  }
  return c.ws_bytes;
}

int vad_cad_bind(vad_cad_plan* plan, void* workspace, float* params, float* grads, float* bufs, int64_t* nbt,
                 float* exp_avg, float* exp_avg_sq, int32_t* steps) {
  VAD_CHECK(plan && workspace && params && bufs, "vad_cad_bind: null argument");
  VAD_CHECK((reinterpret_cast<uintptr_t>(workspace) & 255) == 0, "vad_cad_bind: workspace must be 256-B aligned");
  CadPlanImpl& c = plan->impl;
  if (!c.bound) vad_cad_workspace_bytes(plan);  // (fixes the carve options)
  Ws ws;
  ws.base = reinterpret_cast<char*>(workspace);
  ws.dry = false;
  c.carve(ws);
  c.bound = 1;
  c.params = params; c.grads = grads; c.bufs = bufs; c.nbt = nbt;
  c.m = exp_avg; c.v = exp_avg_sq; c.steps = steps;
  VAD_HIP(hipMemcpy(c.chunk_slot, plan->chunk_host.data(), plan->chunk_host.size() * sizeof(int16_t),
                    hipMemcpyHostToDevice));
  return 0;
}

namespace {
struct CopyList {
  uint32_t* dst[10];
  const uint32_t* src[10];
  int words[10];
  int n;
};
// one block per entry; every entry is a whole number of 4-byte words (fp32 / int32 arrays)
__global__ void __launch_bounds__(256) copy_list_kernel(CopyList L) {
  const int e = blockIdx.x;
  uint32_t* d = L.dst[e];
  const uint32_t* s = L.src[e];
  for (int i = threadIdx.x; i < L.words[e]; i += 256) d[i] = s[i];
}
}  // namespace

int vad_cad_forward(vad_cad_plan* plan, const float* x, int training, uint64_t seed, uint64_t step, int64_t clip0,
                    const int64_t* labels, float* final_scores, float* probs, float* causal, float* kl, float* z,
                    float* adj, int32_t* nmax, float* boxes, int32_t* counts, float* losses, int32_t* flags,
                    void* stream) {
  VAD_CHECK(plan && x, "vad_cad_forward: null argument");
  CadPlanImpl& c = plan->impl;
  VAD_CHECK(c.params != nullptr, "vad_cad_forward: plan not bound");
  hipStream_t st = (hipStream_t)stream;
  c.training = training;
  c.seed = seed;
  c.step = step;
  c.clip0 = clip0;
  c.labels = labels;
  c.losses_ptr = losses ? losses : c.sq_parts;  // scratch when not requested
  VAD_TRY(c.forward(x, st));
  // the ten small result arrays leave the plan in one launch (one block per array) instead of ten copy kernels
  const int B = c.B, NF = c.NF;
  CopyList L{};
  auto cp = [&](void* dst, const void* src, size_t bytes) {
    if (!dst) return;
    L.dst[L.n] = (uint32_t*)dst;
    L.src[L.n] = (const uint32_t*)src;
    L.words[L.n] = (int)(bytes / 4);
    ++L.n;
  };
  cp(final_scores, c.finalv, B * 4);
  cp(probs, c.probs, B * 8);
  cp(causal, c.causal, B * 4);
  cp(kl, c.kl, B * 4);
  cp(z, c.z, B * 30 * 4);
  cp(adj, c.adj, B * 36 * 4);
  cp(nmax, c.nmax, B * 4);
  cp(boxes, c.boxes, (size_t)NF * 80);
  cp(counts, c.counts, (size_t)NF * 4);
  cp(flags, c.flags, 8);
  if (L.n > 0) {
    hipLaunchKernelGGL(copy_list_kernel, dim3(L.n), dim3(256), 0, st, L);
    VAD_HIP(hipGetLastError());
  }
  return 0;
}

int vad_cad_backward(vad_cad_plan* plan, int use_loss, const float* d_final, const float* d_probs,
                     const float* d_causal, const float* d_kl, const float* d_z, const float* d_adj, void* stream) {
  VAD_CHECK(plan != nullptr, "vad_cad_backward: null plan");
  return plan->impl.backward(use_loss != 0, d_final, d_probs, d_causal, d_kl, d_z, d_adj, (hipStream_t)stream);
}

int vad_cad_backward_stage(vad_cad_plan* plan, int stage, int use_loss, const float* d_final, const float* d_probs,
                           const float* d_causal, const float* d_kl, const float* d_z, const float* d_adj,
                           void* stream) {
  VAD_CHECK(plan != nullptr, "vad_cad_backward_stage: null plan");
  return plan->impl.backward(use_loss != 0, d_final, d_probs, d_causal, d_kl, d_z, d_adj, (hipStream_t)stream,
                             stage);
}

int vad_cad_wait_side(vad_cad_plan* plan, void* stream) {
  VAD_CHECK(plan != nullptr, "vad_cad_wait_side: null plan");
  return plan->impl.wait_side((hipStream_t)stream);
}

int vad_cad_input_ready(vad_cad_plan* plan, void* stream) {
  VAD_CHECK(plan != nullptr, "vad_cad_input_ready: null plan");
  CadPlanImpl& c = plan->impl;
  VAD_TRY(c.streams());
  VAD_HIP(hipEventRecord(c.ev_input, (hipStream_t)stream));
  c.input_armed = 1;
  return 0;
}

int vad_cad_wait_layer_grads(vad_cad_plan* plan, int layer, void* stream) {
  VAD_CHECK(plan != nullptr && layer >= 0 && layer < 8, "vad_cad_wait_layer_grads: null plan or layer outside 0..7");
  CadPlanImpl& c = plan->impl;
  VAD_CHECK(c.ev_layer[layer] != nullptr, "vad_cad_wait_layer_grads: no backbone backward has been queued");
  VAD_HIP(hipStreamWaitEvent((hipStream_t)stream, c.ev_layer[layer], 0));
  return 0;
}

int vad_cad_backward_ext(vad_cad_plan* plan, int stage, int use_loss, const float* d_final, const float* d_probs,
                         const float* d_causal, const float* d_kl, const float* d_z, const float* d_adj,
                         const float* d_boxes, void* stream) {
  VAD_CHECK(plan != nullptr, "vad_cad_backward_ext: null plan");
  return plan->impl.backward(use_loss != 0, d_final, d_probs, d_causal, d_kl, d_z, d_adj, (hipStream_t)stream,
                             stage, d_boxes);
}

int vad_cad_optimizer_step(vad_cad_plan* plan, float lr, float beta1, float beta2, float eps, float weight_decay,
                           float max_norm, float grad_scale, float* total_norm, void* stream) {
  VAD_CHECK(plan != nullptr, "vad_cad_optimizer_step: null plan");
  return plan->impl.optimizer(lr, beta1, beta2, eps, weight_decay, max_norm, grad_scale, total_norm,
                              (hipStream_t)stream);
}

int vad_cad_debug_buffer(vad_cad_plan* plan, const char* name, int idx, void** ptr, int64_t* nfloats) {
  VAD_CHECK(plan && name && ptr && nfloats, "vad_cad_debug_buffer: null argument");
  CadPlanImpl& c = plan->impl;
  const std::string n(name);
  const int64_t NF = c.NF;
  auto act = [&](int l) { return NF * c.L[l].OH * c.L[l].OW * c.L[l].Co; };
  const int cs[9] = {32, 32, 32, 64, 64, 128, 128, 256, 256};
  if (n == "y1") { *ptr = c.y1; *nfloats = NF * c.H1 * c.W1 * 32; }
  else if (n == "pool") { *ptr = c.pool; *nfloats = NF * c.HP * c.WP * 32; }
  else if (n == "y" && idx >= 0 && idx < 8) { *ptr = c.y[idx]; *nfloats = act(idx); }
  else if (n == "stats" && idx >= 0 && idx < 9) { *ptr = c.stats[idx]; *nfloats = BN_STATS_PER_C * cs[idx]; }
  else if (n == "feats") { *ptr = c.feats; *nfloats = NF * 6144; }
  else if (n == "pooled") { *ptr = c.pooled; *nfloats = (int64_t)c.B * 6144; }
  else if (n == "dA") { *ptr = c.dA; *nfloats = c.act_max; }
  else if (n == "dY") {
    const int l = c.debug_stop_layer;
    const bool perl = c.dy_per_layer && g_cad_dy_per_layer && l >= 0 && l < 8;
    *ptr = perl ? c.dYL[l] : ((l & 1) ? c.dY2 : c.dY);
    *nfloats = perl ? (int64_t)c.NF * c.L[l].OH * c.L[l].OW * c.L[l].Co : c.act_max;
  }
  else if (n == "act_bf16") { *ptr = nullptr; *nfloats = c.act_bf16; }  // storage of pool / y / dA / dY
  else if (n == "d_pooled") { *ptr = c.d_pooled; *nfloats = (int64_t)c.B * 6144; }
  else if (n == "d_feat_det") { *ptr = c.d_feat_det; *nfloats = NF * 6144; }
  else if (n == "det_logits") { *ptr = c.dlog; *nfloats = NF * 20; }
  else if (n == "dir_h" && idx >= 0 && idx < 4) {  // direct classifier hidden layer idx (post ReLU / dropout)
    const int w[4] = {512, 256, 128, 64};
    *ptr = c.gh[idx];
    *nfloats = (int64_t)c.B * w[idx];
  }
  else if (n == "bn_sync") { *ptr = c.bnsync; *nfloats = 2 * 2 * 256; }  // double [2*256]: 1024 float words
  else { vad::set_error("vad_cad_debug_buffer: unknown buffer " + n); return 1; }
  VAD_CHECK(*ptr != nullptr || n == "act_bf16", "vad_cad_debug_buffer: " + n + " is not carved under this plan's options");
  return 0;
}

int vad_cad_set_debug(vad_cad_plan* plan, const char* key, int64_t value) {
  VAD_CHECK(plan && key, "vad_cad_set_debug: null argument");
  if (std::string(key) == "stop_layer") plan->impl.debug_stop_layer = (int)value;
  else { vad::set_error("vad_cad_set_debug: unknown key"); return 1; }
  return 0;
}

int vad_cad_set_option(vad_cad_plan* plan, const char* key, int64_t value) {
  VAD_CHECK(plan && key, "vad_cad_set_option: null argument");
  if (std::string(key) == "conv_bf16") plan->impl.conv_bf16 = value ? 1 : 0;
  else if (std::string(key) == "stem_grad") plan->impl.stem_grad = value ? 1 : 0;
  else if (std::string(key) == "wgrad_stream") plan->impl.wgrad_stream = value ? 1 : 0;
  else if (std::string(key) == "dy_per_layer") plan->impl.dy_per_layer = value ? 1 : 0;
  else if (std::string(key) == "act_bf16") plan->impl.act_bf16_opt = value ? 1 : 0;
  else if (std::string(key) == "input_armed" && value == 0) plan->impl.input_armed = 0;  // (arming: vad_cad_input_ready)
  else { vad::set_error("vad_cad_set_option: unknown key"); return 1; }
  return 0;
}

int vad_cad_set_bn_sync(vad_cad_plan* plan, vad_bn_sync_fn fn, void* user, int world) {
  VAD_CHECK(plan != nullptr, "vad_cad_set_bn_sync: null plan");
  VAD_CHECK(fn == nullptr || world >= 1, "vad_cad_set_bn_sync: world must be >= 1");
  plan->impl.sync_fn = fn;
  plan->impl.sync_user = user;
  plan->impl.sync_world = fn ? world : 1;
  return 0;
}

int vad_cad_conv_path(vad_cad_plan* plan, int layer, int kind) {
  if (!plan || layer < 0 || layer >= 8 || kind < 0 || kind > 2) {
    vad::set_error("vad_cad_conv_path: bad argument");
    return -1;
  }
  ConvPrecision prec(plan->impl.conv_bf16);
  return conv3_path(plan->impl.L[layer], kind);
}

int vad_cad_profile(vad_cad_plan* plan, int enable, const char* only_prefix) {
  VAD_CHECK(plan != nullptr, "vad_cad_profile: null plan");
  Profiler& p = plan->impl.prof;
  // enable: 0 off (records kept), 1 on after clearing the records, 2 on, appending to the records
  p.on = enable != 0;
  if (enable) p.only = only_prefix ? only_prefix : "";
  if (enable == 1) p.reset();
  return 0;
}

/* aggregates the recorded launches by label (after the stream has been synchronised). Returns the number of
 * distinct labels; fills at most cap entries: labels (64 chars each), total ms, launch counts. */
int vad_cad_profile_read(vad_cad_plan* plan, char* labels, double* total_ms, int* counts, int cap) {
  VAD_CHECK(plan != nullptr, "vad_cad_profile_read: null plan");
  Profiler& p = plan->impl.prof;
  std::vector<std::string> names;
  std::vector<double> tot;
  std::vector<int> cnt;
  for (auto& r : p.recs) {
    float ms = 0.f;
    VAD_HIP(hipEventSynchronize(r.b));
    VAD_HIP(hipEventElapsedTime(&ms, r.a, r.b));
    size_t i = 0;
    while (i < names.size() && names[i] != r.label) ++i;
    if (i == names.size()) {
      names.push_back(r.label);
      tot.push_back(0.0);
      cnt.push_back(0);
    }
    tot[i] += ms;
    cnt[i] += 1;
  }
  for (size_t i = 0; i < names.size() && (int)i < cap; ++i) {
    strncpy(labels + 64 * i, names[i].c_str(), 63);
    labels[64 * i + 63] = 0;
    total_ms[i] = tot[i];
    counts[i] = cnt[i];
  }
  return (int)names.size();
}

/* the recorded launches one by one, in record order: label, start and end in ms after the first record's start (the
 * post-backbone chain measurement: start of avgpool_bwd minus end of the last forward conv).  Returns the number of
 * records; fills at most cap. */
int vad_cad_profile_marks(vad_cad_plan* plan, char* labels, double* t0_ms, double* t1_ms, int cap) {
  VAD_CHECK(plan != nullptr, "vad_cad_profile_marks: null plan");
  Profiler& p = plan->impl.prof;
  for (size_t i = 0; i < p.recs.size() && (int)i < cap; ++i) {
    const auto& r = p.recs[i];
    float a = 0.f, b = 0.f;
    VAD_HIP(hipEventSynchronize(r.b));
    VAD_HIP(hipEventElapsedTime(&a, p.recs[0].a, r.a));
    VAD_HIP(hipEventElapsedTime(&b, p.recs[0].a, r.b));
    strncpy(labels + 64 * i, r.label.c_str(), 63);
    labels[64 * i + 63] = 0;
    t0_ms[i] = a;
    t1_ms[i] = b;
  }
  return (int)p.recs.size();
}

int vad_debug_d2h(void* host, const void* dev, int64_t bytes) {
  VAD_HIP(hipDeviceSynchronize());
  VAD_HIP(hipMemcpy(host, dev, (size_t)bytes, hipMemcpyDeviceToHost));
  return 0;
}

}  // extern "C"
