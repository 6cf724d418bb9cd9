// causal_anomaly_detection1.py (cad1): the memory-bank VideoAutoEncoder (cad1:124-321) and its train_model
// iteration (cad1:372-431) as one device plan.
//
// Frames are folded n = t*B + b.  The reference runs its encoder once per frame index t on the B clips
// (encode_sequence, cad1:226-231), so each t is its own train-mode BatchNorm batch: the encoder's BN statistics are
// per group t, a contiguous row range in this order.  The decoder is called T times on the same sequence feature
// (decode_sequence, cad1:254-258); the calls are identical, so it runs once per clip and only its BN running
// statistics take the T updates.
//   encoder   4 x [Conv2d(4, s2, p1) as an implicit f32 MFMA GEMM over the NHWC frames (backbone.hip conv4_fwd; the
//             first, 1-channel layer on the VALU, conv4_c1_fwd: 32 outputs per pixel from its 4x4 window) -> per-t BN
//             partial sums
//             -> grouped finalize (running stats updated once per t, in t order) -> BN + LeakyReLU(0.1); layer 4
//             straight into the NCHW flatten order] -> Linear(2048, 64) GEMM -> tanh, NaN -> 0
//   LSTM      input projection of all B*T frames as one GEMM; the recurrence one block per clip with the W_hh rows
//             in registers and h broadcast from LDS; gates, cell states and h_{t-1} kept for BPTT
//   decoder   Linear(64, 2048) GEMM -> LeakyReLU into NHWC -> 3 x [ConvTranspose2d as four parity-class implicit
//             GEMMs with the bias in the epilogue (conv4_cls) -> BN + LeakyReLU] -> ConvTranspose2d(32, 1) -> sigmoid
//   loss      MSE of the T identical reconstructions against the T frames (cad1:340-344) and d MSE / d logits in
//             one pass; per-clip errors (cad1:545-546)
//   memory    cosine min-distance to the ring (cad1:262-301), then the ring update (cad1:201-219), both on the
//             device-resident memory_ptr
//   backward  mirror image: Conv2d input grads as parity-class GEMMs over dY, ConvTranspose2d input grads as the
//             16-tap gather over dY, weight grads as split-K correlations of the two operands (conv4_wgrad; the
//             1-channel ends -- encoder layer 0's weight grad, the last ConvTranspose2d's grads -- on the VALU,
//             conv4_c1_wgrad / conv4_c1_fwd), grouped BN backward through the LeakyReLU, BPTT one block per clip
// (knob "ae_direct" = 0 at plan creation: every conv, the 1-channel ends included, on im2col / col2im columns + dense
// GEMMs with K = 16 for the 1-channel layer -- the round-4 path, kept as the cross-check of the direct kernels:
// tests/test_ae_gpu.py::test_ae_direct_and_im2col_paths_agree)
//   update    non-finite-grad skip + clip_grad_norm_(0.1) + Adam with coupled L2 (optim.h)
// Status word (losses[3]): 0 = skipped before backward (train-loop mode: a non-finite input, cad1:385-387 -- the BN
// running stats, counters and the memory ring stay untouched, as the reference's `continue` before the forward -- or
// a non-finite loss), 1 = non-finite grads, no step, 2 = stepped.
#include <algorithm>
#include <cmath>
#include <string>
#include <vector>

#include "../../include/vad.h"
#include "backbone.h"
#include "conv3d.h"
#include "optim.h"
#include "plan_util.h"

namespace vad {

int g_ae_direct = 1;  // knob "ae_direct" (latched per plan)
// knob "ae_wgrad_stream" (latched per plan, direct mode): the backward's weight gradients run on a low-priority stream
// of the plan beside the input-gradient chain, on their own split-K scratch, with dY alternating between two buffers
int g_ae_wgrad_stream = 1;

constexpr int AE_HW = 64;  // frame side: the encoder's Linear(128 * 4 * 4) fixes 64x64 frames (cad1:151)
constexpr int AE_PIX = AE_HW * AE_HW;
constexpr int AE_CHUNKS = AE_PIX / 256;
constexpr int AE_LAT = 64;  // latent_dim: LSTM input and hidden size
constexpr int AE_GATES = 4 * AE_LAT;
constexpr int AE_FLAT = 128 * 16;
constexpr int AE_MEM = 500;  // memory_size (cad1:191-193)
constexpr float AE_SLOPE = 0.1f;
constexpr int AE_ST = 8;  // floats per channel of one BN group's stats block
constexpr int AE_NBN = 7;
int g_ae_wgrad_blocks = 1024;  // knob "ae_wgrad_blocks": split-K target grid of the implicit-GEMM weight gradients
                               // (sweep: 1024 3.149, 2048 3.206, 4096 3.202 ms, profiles/r05_cad1_direct.json)
constexpr int ENC_CI[4] = {1, 32, 64, 128}, ENC_CO[4] = {32, 64, 128, 128}, ENC_IN[4] = {64, 32, 16, 8};
constexpr int DEC_CI[4] = {128, 128, 64, 32}, DEC_CO[4] = {128, 64, 32, 1}, DEC_IN[4] = {4, 8, 16, 32};

struct AeSlot {
  std::string name;
  int64_t numel, offset;
};

// model.named_parameters() and BN running-stat order (cad1:129-188)
struct AeLayout {
  std::vector<AeSlot> slots, bufs;
  int64_t param_floats = 0, buf_floats = 0;
  int enc_w[4], enc_b[4], ebn_w[4], ebn_b[4], efc_w, efc_b;
  int dfc_w, dfc_b, dec_w[4], dec_b[4], dbn_w[3], dbn_b[3];
  int wih, whh, bih, bhh;
  int erm[4], erv[4], drm[3], drv[3];
  AeLayout() {
    auto add = [](std::vector<AeSlot>& v, const std::string& n, int64_t k) {
      v.push_back({n, k, 0});
      return (int)v.size() - 1;
    };
    for (int l = 0; l < 4; ++l) {
      const std::string c = "encoder." + std::to_string(3 * l), b = "encoder." + std::to_string(3 * l + 1);
      enc_w[l] = add(slots, c + ".weight", (int64_t)ENC_CO[l] * ENC_CI[l] * 16);
      enc_b[l] = add(slots, c + ".bias", ENC_CO[l]);
      ebn_w[l] = add(slots, b + ".weight", ENC_CO[l]);
      ebn_b[l] = add(slots, b + ".bias", ENC_CO[l]);
      erm[l] = add(bufs, b + ".running_mean", ENC_CO[l]);
      erv[l] = add(bufs, b + ".running_var", ENC_CO[l]);
    }
    efc_w = add(slots, "encoder.13.weight", (int64_t)AE_LAT * AE_FLAT);
    efc_b = add(slots, "encoder.13.bias", AE_LAT);
    dfc_w = add(slots, "decoder.0.weight", (int64_t)AE_FLAT * AE_LAT);
    dfc_b = add(slots, "decoder.0.bias", AE_FLAT);
    for (int j = 0; j < 4; ++j) {
      const std::string c = "decoder." + std::to_string(3 * j + 3), b = "decoder." + std::to_string(3 * j + 4);
      dec_w[j] = add(slots, c + ".weight", (int64_t)DEC_CI[j] * DEC_CO[j] * 16);
      dec_b[j] = add(slots, c + ".bias", DEC_CO[j]);
      if (j < 3) {
        dbn_w[j] = add(slots, b + ".weight", DEC_CO[j]);
        dbn_b[j] = add(slots, b + ".bias", DEC_CO[j]);
        drm[j] = add(bufs, b + ".running_mean", DEC_CO[j]);
        drv[j] = add(bufs, b + ".running_var", DEC_CO[j]);
      }
    }
    wih = add(slots, "temporal_encoder.weight_ih_l0", (int64_t)AE_GATES * AE_LAT);
    whh = add(slots, "temporal_encoder.weight_hh_l0", (int64_t)AE_GATES * AE_LAT);
    bih = add(slots, "temporal_encoder.bias_ih_l0", AE_GATES);
    bhh = add(slots, "temporal_encoder.bias_hh_l0", AE_GATES);
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
static const AeLayout& ae_layout() {
  static const AeLayout L;
  return L;
}

__device__ __forceinline__ float leaky(float v) { return v > 0.f ? v : v * AE_SLOPE; }
__device__ __forceinline__ float nan0(float v) { return v != v ? 0.f : v; }

static dim3 grid_for(int64_t n) {
  return dim3((unsigned)std::max<int64_t>(1, std::min<int64_t>(cdiv(n, 256), 8192)));
}

// Conv2d(C -> Co, 4, stride 2, padding 1) over NHWC frames, as a depth-1 3-D conv for conv3d.h's im2col / col2im
static Conv3dGeom ae_geom(int N, int C, int hw, int Co) {
  Conv3dGeom g{};
  g.in = {N, C, 1, hw, hw};
  g.Co = Co;
  g.kd = 1;
  g.kh = g.kw = 4;
  g.sd = 1;
  g.sh = g.sw = 2;
  g.pd = 0;
  g.ph = g.pw = 1;
  g.OD = 1;
  g.OH = g.OW = hw / 2;
  return g;
}

// ------------------------------------------------------------------ input frames
// xf[t*B + b] = frame t of clip b with NaN -> 0 (check_and_fix_nan of the input, cad1:304); *bad |= any NaN / Inf
__global__ __launch_bounds__(256) void ae_frames_kernel(const float* __restrict__ x, int B, int T,
                                                        float* __restrict__ xf, int* bad) {
  constexpr int Q = AE_PIX / 4;
  const int64_t total = (int64_t)B * T * Q;
  int nonfin = 0;
  for (int64_t i = blockIdx.x * 256ll + threadIdx.x; i < total; i += (int64_t)gridDim.x * 256) {
    const int64_t bt = i / Q;
    const int p = (int)(i - bt * Q) * 4;
    const int b = (int)(bt / T), t = (int)(bt - (int64_t)b * T);
    f32x4 v = *reinterpret_cast<const f32x4*>(x + bt * AE_PIX + p);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      if (!isfinite(v[e])) nonfin = 1;
      v[e] = nan0(v[e]);
    }
    *reinterpret_cast<f32x4*>(xf + ((int64_t)t * B + b) * AE_PIX + p) = v;
  }
  if (nonfin) atomicOr(bad, 1);
}

// ------------------------------------------------------------------ grouped train-mode BatchNorm + LeakyReLU(0.1)
// Y[M][C] (NHWC rows); rows [g*Mg, (g+1)*Mg) are BN batch g.  Per-group stats block [AE_ST][C]: 0 mean, 1 invstd,
// 2 scale, 3 shift, 4 k = gamma*invstd, 5 mean(dZ), 6 mean(dZ*xhat).  Reductions run on a (P row tiles, G) grid.
struct Gbn {
  int G, C, P, R;
  int64_t Mg;
};
static Gbn gbn(int G, int64_t Mg, int C) {
  Gbn q{G, C, 0, 256, Mg};
  q.P = (int)cdiv(Mg, q.R);
  return q;
}

// fixed-order block combine of per-thread [sum | sum2] channel quads (thread = row lane x channel quad)
__device__ inline void ae_block_store(float (&v)[2][4], int C, float* out) {
  __shared__ float red[8 * 256];
  const int t = threadIdx.x;
#pragma unroll
  for (int s = 0; s < 2; ++s)
#pragma unroll
    for (int e = 0; e < 4; ++e) red[(s * 4 + e) * 256 + t] = v[s][e];
  __syncthreads();
  const int nq = C / 4, lanes = 256 / nq;
  for (int idx = t; idx < 2 * C; idx += 256) {
    const int s = idx / C, c = idx % C, q = c / 4, e = c % 4;
    float acc = 0.f;
    for (int g = 0; g < lanes; ++g) acc += red[(s * 4 + e) * 256 + g * nq + q];
    out[idx] = acc;
  }
}

__global__ __launch_bounds__(256) void gbn_partials_kernel(const float* __restrict__ y, Gbn q,
                                                           float* __restrict__ parts) {
  const int C = q.C, nq = C / 4, lanes = 256 / nq;
  const int c = (threadIdx.x % nq) * 4, rl = threadIdx.x / nq;
  const float* yg = y + (int64_t)blockIdx.y * q.Mg * C;
  const int64_t r0 = (int64_t)blockIdx.x * q.R, r1 = min(q.Mg, r0 + q.R);
  float v[2][4] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
  // (4 rows in flight per thread: the loads of an unrolled group issue before its arithmetic; same summation order)
#pragma unroll 4
  for (int64_t r = r0 + rl; r < r1; r += lanes) {
    const f32x4 a = *reinterpret_cast<const f32x4*>(yg + r * C + c);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      v[0][e] += a[e];
      v[1][e] = fmaf(a[e], a[e], v[1][e]);
    }
  }
  ae_block_store(v, C, parts + ((int64_t)blockIdx.y * q.P + blockIdx.x) * 2 * C);
}

// batch statistics per group (double combine); running stats updated `repeat` times per group, in group order
// (momentum 0.1, unbiased variance), not at all when *skip; eval mode normalises with the running stats
// BN group sums of one channel: 16 lanes per group (groups g0 .. g0 + 15 per pass), each lane adding the partial rows
// p = lane, lane + 16, ... in order, then a fixed xor butterfly over the 16 lanes (double)
__device__ inline double gbn_sum16(double v) {
#pragma unroll
  for (int o = 8; o > 0; o >>= 1) v += __shfl_xor(v, o, 16);
  return v;
}

__global__ __launch_bounds__(256) void gbn_finalize_kernel(const float* __restrict__ parts, Gbn q,
                                                           const float* __restrict__ gamma,
                                                           const float* __restrict__ beta, float* running_mean,
                                                           float* running_var, int training, int repeat,
                                                           const int* skip, float* __restrict__ stats) {
  const int c = blockIdx.x, C = q.C, lane = threadIdx.x & 15, gl = threadIdx.x >> 4;
  __shared__ double red[2][16];
  const double count = (double)q.Mg, mom = 0.1;
  const bool upd = training && !(skip && *skip);
  float rm = running_mean[c], rv = running_var[c];
  for (int g0 = 0; g0 < q.G; g0 += 16) {
    const int g = g0 + gl;
    double a = 0.0, b = 0.0;
    if (training && g < q.G)
#pragma unroll 4
      for (int p = lane; p < q.P; p += 16) {
        const float* pp = parts + ((int64_t)g * q.P + p) * 2 * C;
        a += (double)pp[c];
        b += (double)pp[C + c];
      }
    a = gbn_sum16(a);
    b = gbn_sum16(b);
    if (lane == 0) {
      red[0][gl] = a;
      red[1][gl] = b;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      // (running stats updated once per group, in group order)
      for (int k = 0; k < 16 && g0 + k < q.G; ++k) {
        double mean = rm, var = rv;
        if (training) {
          mean = red[0][k] / count;
          var = red[1][k] / count - mean * mean;
          if (var < 0) var = 0;
          if (upd)
            for (int r = 0; r < repeat; ++r) {
              rm = (float)((1.0 - mom) * rm + mom * mean);
              rv = (float)((1.0 - mom) * rv + mom * var * count / (count - 1.0));
            }
        }
        const double invstd = 1.0 / sqrt(var + 1e-5), scale = (double)gamma[c] * invstd;
        float* s = stats + (int64_t)(g0 + k) * AE_ST * C;
        s[c] = (float)mean;
        s[C + c] = (float)invstd;
        s[2 * C + c] = (float)scale;
        s[3 * C + c] = (float)((double)beta[c] - mean * scale);
      }
    }
    __syncthreads();
  }
  if (threadIdx.x == 0 && upd) {
    running_mean[c] = rm;
    running_var[c] = rv;
  }
}

// A = LeakyReLU(scale_g * Y + shift_g); hw_perm > 0 writes A in the per-frame NCHW flatten order (hw_perm pixels
// per frame: the encoder's Flatten, cad1:150)
__global__ __launch_bounds__(256) void gbn_act_kernel(const float* __restrict__ y, const float* __restrict__ stats,
                                                      int64_t M, int64_t Mg, int C, int hw_perm,
                                                      float* __restrict__ out) {
  const int nq = C / 4;
  const int64_t total = M * nq;
  for (int64_t i = blockIdx.x * 256ll + threadIdx.x; i < total; i += (int64_t)gridDim.x * 256) {
    const int64_t r = i / nq;
    const int c = (int)(i - r * nq) * 4;
    const float* s = stats + (r / Mg) * AE_ST * C;
    const f32x4 a = *reinterpret_cast<const f32x4*>(y + r * C + c);
    f32x4 o;
#pragma unroll
    for (int e = 0; e < 4; ++e) o[e] = leaky(fmaf(a[e], s[2 * C + c + e], s[3 * C + c + e]));
    if (!hw_perm) {
      *reinterpret_cast<f32x4*>(out + r * C + c) = o;
    } else {
      const int64_t n = r / hw_perm;
      const int px = (int)(r - n * hw_perm);
#pragma unroll
      for (int e = 0; e < 4; ++e) out[(n * C + c + e) * hw_perm + px] = o[e];
    }
  }
}

// backward through LeakyReLU(BN(y)) (LeakyReLU'(z) = 1 for z > 0, else 0.1): per group sum(dZ), sum(dZ*xhat)
__global__ __launch_bounds__(256) void gbn_bwd_reduce_kernel(const float* __restrict__ dA, const float* __restrict__ y,
                                                             const float* __restrict__ stats, Gbn q,
                                                             float* __restrict__ parts) {
  const int C = q.C, nq = C / 4, lanes = 256 / nq;
  const int c = (threadIdx.x % nq) * 4, rl = threadIdx.x / nq;
  const float* s = stats + (int64_t)blockIdx.y * AE_ST * C;
  const f32x4 mean = *reinterpret_cast<const f32x4*>(s + c), inv = *reinterpret_cast<const f32x4*>(s + C + c);
  const f32x4 sc = *reinterpret_cast<const f32x4*>(s + 2 * C + c), sh = *reinterpret_cast<const f32x4*>(s + 3 * C + c);
  const int64_t base = (int64_t)blockIdx.y * q.Mg * C;
  const int64_t r0 = (int64_t)blockIdx.x * q.R, r1 = min(q.Mg, r0 + q.R);
  float v[2][4] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
  // (4 rows in flight per thread: the loads of an unrolled group issue before its arithmetic; same summation order)
#pragma unroll 4
  for (int64_t r = r0 + rl; r < r1; r += lanes) {
    const f32x4 a = *reinterpret_cast<const f32x4*>(dA + base + r * C + c);
    const f32x4 yy = *reinterpret_cast<const f32x4*>(y + base + r * C + c);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float z = fmaf(yy[e], sc[e], sh[e]);
      const float dz = z > 0.f ? a[e] : a[e] * AE_SLOPE;
      v[0][e] += dz;
      v[1][e] = fmaf(dz, (yy[e] - mean[e]) * inv[e], v[1][e]);
    }
  }
  ae_block_store(v, C, parts + ((int64_t)blockIdx.y * q.P + blockIdx.x) * 2 * C);
}

// per group k = gamma * invstd, mean(dZ), mean(dZ * xhat); dgamma / dbeta summed over the groups (the reference
// accumulates the grads of its per-t calls)
__global__ __launch_bounds__(256) void gbn_bwd_finalize_kernel(const float* __restrict__ parts, Gbn q,
                                                               const float* __restrict__ gamma, int training,
                                                               float* __restrict__ stats, float* dgamma,
                                                               float* dbeta) {
  const int c = blockIdx.x, C = q.C, lane = threadIdx.x & 15, gl = threadIdx.x >> 4;
  __shared__ double red[2][16];
  const double count = (double)q.Mg;
  double tz = 0.0, tzx = 0.0;
  for (int g0 = 0; g0 < q.G; g0 += 16) {
    const int g = g0 + gl;
    double a = 0.0, b = 0.0;
    if (g < q.G)
#pragma unroll 4
      for (int p = lane; p < q.P; p += 16) {
        const float* pp = parts + ((int64_t)g * q.P + p) * 2 * C;
        a += (double)pp[c];
        b += (double)pp[C + c];
      }
    a = gbn_sum16(a);
    b = gbn_sum16(b);
    if (lane == 0) {
      red[0][gl] = a;
      red[1][gl] = b;
    }
    __syncthreads();
    if (threadIdx.x == 0)
      for (int k = 0; k < 16 && g0 + k < q.G; ++k) {
        float* s = stats + (int64_t)(g0 + k) * AE_ST * C;
        s[4 * C + c] = gamma[c] * s[C + c];
        // eval mode: BN is the affine map of the running stats, no batch-mean terms in its backward
        s[5 * C + c] = training ? (float)(red[0][k] / count) : 0.f;
        s[6 * C + c] = training ? (float)(red[1][k] / count) : 0.f;
        tz += red[0][k];
        tzx += red[1][k];
      }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    dgamma[c] = (float)tzx;
    dbeta[c] = (float)tz;
  }
}

// dY = k * (dZ - mean(dZ) - xhat * mean(dZ * xhat)); bparts (nullable): per-block sums of dY (conv-bias grads)
__global__ __launch_bounds__(256) void gbn_bwd_apply_kernel(const float* __restrict__ dA, const float* __restrict__ y,
                                                            const float* __restrict__ stats, Gbn q,
                                                            float* __restrict__ dY, float* __restrict__ bparts) {
  const int C = q.C, nq = C / 4, lanes = 256 / nq;
  const int c = (threadIdx.x % nq) * 4, rl = threadIdx.x / nq;
  const float* s = stats + (int64_t)blockIdx.y * AE_ST * C;
  const f32x4 mean = *reinterpret_cast<const f32x4*>(s + c), inv = *reinterpret_cast<const f32x4*>(s + C + c);
  const f32x4 sc = *reinterpret_cast<const f32x4*>(s + 2 * C + c), sh = *reinterpret_cast<const f32x4*>(s + 3 * C + c);
  const f32x4 k = *reinterpret_cast<const f32x4*>(s + 4 * C + c);
  const f32x4 mdz = *reinterpret_cast<const f32x4*>(s + 5 * C + c), mdzx = *reinterpret_cast<const f32x4*>(s + 6 * C + c);
  const int64_t base = (int64_t)blockIdx.y * q.Mg * C;
  const int64_t r0 = (int64_t)blockIdx.x * q.R, r1 = min(q.Mg, r0 + q.R);
  float v[2][4] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
  // (4 rows in flight per thread: the loads of an unrolled group issue before its arithmetic; same summation order)
#pragma unroll 4
  for (int64_t r = r0 + rl; r < r1; r += lanes) {
    const f32x4 a = *reinterpret_cast<const f32x4*>(dA + base + r * C + c);
    const f32x4 yy = *reinterpret_cast<const f32x4*>(y + base + r * C + c);
    f32x4 o;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float z = fmaf(yy[e], sc[e], sh[e]);
      const float dz = z > 0.f ? a[e] : a[e] * AE_SLOPE;
      const float xh = (yy[e] - mean[e]) * inv[e];
      o[e] = k[e] * (dz - mdz[e] - xh * mdzx[e]);
      v[0][e] += o[e];
    }
    *reinterpret_cast<f32x4*>(dY + base + r * C + c) = o;
  }
  if (bparts) ae_block_store(v, C, bparts + ((int64_t)blockIdx.y * q.P + blockIdx.x) * 2 * C);
}

// db[c] = sum over blocks of parts[blk][c] (the first half of each block's [2][C] record): one block per channel,
// thread t adding blocks t, t + 256, ... in order, then a fixed tree (double)
__global__ __launch_bounds__(256) void ae_bias_reduce_kernel(const float* __restrict__ parts, int nblk, int C,
                                                             float* __restrict__ db) {
  const int c = blockIdx.x;
  __shared__ double red[256];
  double s = 0.0;
  for (int i = threadIdx.x; i < nblk; i += 256) s += (double)parts[(int64_t)i * 2 * C + c];
  red[threadIdx.x] = s;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) db[c] = (float)red[0];
}

// out[0] = sum of x[0, n) (one block, fixed order): the bias grad of the single-channel last ConvTranspose2d
// sum of n floats in two fixed-order passes: AE_SUM_BLOCKS block partials (double), then one block adds them
constexpr int AE_SUM_BLOCKS = 256;

__global__ __launch_bounds__(256) void ae_sum_parts_kernel(const float* __restrict__ x, int64_t n,
                                                           double* __restrict__ parts) {
  __shared__ double red[256];
  double s = 0.0;
  for (int64_t i = blockIdx.x * 256ll + threadIdx.x; i < n; i += (int64_t)AE_SUM_BLOCKS * 256) s += (double)x[i];
  red[threadIdx.x] = s;
  __syncthreads();
  for (int k = 128; k > 0; k >>= 1) {
    if (threadIdx.x < k) red[threadIdx.x] += red[threadIdx.x + k];
    __syncthreads();
  }
  if (threadIdx.x == 0) parts[blockIdx.x] = red[0];
}

__global__ __launch_bounds__(256) void ae_sum_kernel(const double* __restrict__ parts, float* __restrict__ out) {
  __shared__ double red[AE_SUM_BLOCKS];
  red[threadIdx.x] = parts[threadIdx.x];
  __syncthreads();
  for (int k = AE_SUM_BLOCKS / 2; k > 0; k >>= 1) {
    if (threadIdx.x < k) red[threadIdx.x] += red[threadIdx.x + k];
    __syncthreads();
  }
  if (threadIdx.x == 0) out[0] = (float)red[0];
}

// ------------------------------------------------------------------ latents, layout changes
// frame latents lat = tanh(z) with NaN -> 0 (cad1:152, 230, 234); frame_features (B, T, 64) when ff != nullptr
__global__ __launch_bounds__(256) void ae_latent_kernel(const float* __restrict__ z, int B, int T,
                                                        float* __restrict__ lat, float* __restrict__ ff) {
  const int64_t total = (int64_t)B * T * AE_LAT;
  for (int64_t i = blockIdx.x * 256ll + threadIdx.x; i < total; i += (int64_t)gridDim.x * 256) {
    const float v = nan0(tanhf(z[i]));
    lat[i] = v;
    if (ff) {
      const int64_t n = i / AE_LAT;
      const int t = (int)(n / B), b = (int)(n - (int64_t)t * B), k = (int)(i - n * AE_LAT);
      ff[((int64_t)b * T + t) * AE_LAT + k] = v;
    }
  }
}

// dz = (d lat + d frame_features) * (1 - lat^2); 0 where z was NaN (the NaN fix passes no gradient)
__global__ __launch_bounds__(256) void ae_latent_bwd_kernel(const float* __restrict__ dlat,
                                                            const float* __restrict__ dff,
                                                            const float* __restrict__ lat,
                                                            const float* __restrict__ z, int B, int T,
                                                            float* __restrict__ dz) {
  const int64_t total = (int64_t)B * T * AE_LAT;
  for (int64_t i = blockIdx.x * 256ll + threadIdx.x; i < total; i += (int64_t)gridDim.x * 256) {
    float d = dlat[i];
    if (dff) {
      const int64_t n = i / AE_LAT;
      const int t = (int)(n / B), b = (int)(n - (int64_t)t * B), k = (int)(i - n * AE_LAT);
      d += dff[((int64_t)b * T + t) * AE_LAT + k];
    }
    const float l = lat[i];
    dz[i] = z[i] != z[i] ? 0.f : d * (1.f - l * l);
  }
}

// Linear(64, 2048) output u[b][c*16 + p] -> LeakyReLU -> NHWC x0[b*16 + p][c] (Unflatten(1, (128, 4, 4)), cad1:157-159)
__global__ __launch_bounds__(256) void ae_dec_in_kernel(const float* __restrict__ u, int B, float* __restrict__ x0) {
  const int64_t total = (int64_t)B * AE_FLAT;
  for (int64_t i = blockIdx.x * 256ll + threadIdx.x; i < total; i += (int64_t)gridDim.x * 256) {
    const int64_t b = i / AE_FLAT;
    const int r = (int)(i - b * AE_FLAT), p = r / 128, c = r % 128;
    x0[i] = leaky(u[b * AE_FLAT + c * 16 + p]);
  }
}

__global__ __launch_bounds__(256) void ae_dec_in_bwd_kernel(const float* __restrict__ dx0, const float* __restrict__ u,
                                                            int B, float* __restrict__ du) {
  const int64_t total = (int64_t)B * AE_FLAT;
  for (int64_t i = blockIdx.x * 256ll + threadIdx.x; i < total; i += (int64_t)gridDim.x * 256) {
    const int64_t b = i / AE_FLAT;
    const int r = (int)(i - b * AE_FLAT), c = r / 16, p = r % 16;
    const float g = dx0[(b * 16 + p) * 128 + c];
    du[i] = u[i] > 0.f ? g : g * AE_SLOPE;
  }
}

// per-frame NCHW flatten order -> NHWC rows: dst[n*hw + p][c] = src[n][c*hw + p]
__global__ __launch_bounds__(256) void ae_unflatten_kernel(const float* __restrict__ src, int64_t N, int C, int hw,
                                                           float* __restrict__ dst) {
  const int64_t per = (int64_t)hw * C, total = N * per;
  for (int64_t i = blockIdx.x * 256ll + threadIdx.x; i < total; i += (int64_t)gridDim.x * 256) {
    const int64_t n = i / per;
    const int r = (int)(i - n * per), p = r / C, c = r % C;
    dst[i] = src[n * per + (int64_t)c * hw + p];
  }
}

__global__ __launch_bounds__(256) void ae_seq_in_kernel(const float* __restrict__ src, int n, float* __restrict__ seq,
                                                        float* __restrict__ out) {
  for (int i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256) {
    const float v = nan0(src[i]);
    seq[i] = v;
    if (out) out[i] = v;
  }
}

__global__ __launch_bounds__(256) void ae_add_kernel(float* __restrict__ a, const float* __restrict__ b, int64_t n) {
  for (int64_t i = blockIdx.x * 256ll + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) a[i] += b[i];
}

// ------------------------------------------------------------------ LSTM(64, 64) (cad1:182-188, 236-240)
// One block per clip: thread j owns gate row j of W_hh (64 registers), h is broadcast from LDS.  torch gate order
// i, f, g, o; gx = x W_ih^T + b_ih for all frames (one GEMM).  Keeps post-activation gates, c_t and h_{t-1}.
__global__ __launch_bounds__(256) void ae_lstm_fwd_kernel(const float* __restrict__ gx, const float* __restrict__ whh,
                                                          const float* __restrict__ bhh, int B, int T,
                                                          float* __restrict__ gates, float* __restrict__ cs,
                                                          float* __restrict__ hprev, float* __restrict__ seq,
                                                          float* __restrict__ seq_out) {
  __shared__ float h[AE_LAT], act[AE_GATES];
  const int b = blockIdx.x, j = threadIdx.x;
  float w[AE_LAT];
#pragma unroll
  for (int k = 0; k < AE_LAT; k += 4) {
    const f32x4 q = *reinterpret_cast<const f32x4*>(whh + (int64_t)j * AE_LAT + k);
    w[k] = q[0];
    w[k + 1] = q[1];
    w[k + 2] = q[2];
    w[k + 3] = q[3];
  }
  const float bj = bhh[j];
  float c = 0.f;
  if (j < AE_LAT) h[j] = 0.f;
  __syncthreads();
  for (int t = 0; t < T; ++t) {
    const int64_t n = (int64_t)t * B + b;
    float acc = bj;
#pragma unroll
    for (int k = 0; k < AE_LAT; ++k) acc = fmaf(w[k], h[k], acc);
    const float pre = gx[n * AE_GATES + j] + acc;
    const float a = (j >= 2 * AE_LAT && j < 3 * AE_LAT) ? tanhf(pre) : 1.f / (1.f + expf(-pre));
    act[j] = a;
    gates[n * AE_GATES + j] = a;
    if (j < AE_LAT) hprev[n * AE_LAT + j] = h[j];
    __syncthreads();
    if (j < AE_LAT) {
      c = act[AE_LAT + j] * c + act[j] * act[2 * AE_LAT + j];
      cs[n * AE_LAT + j] = c;
      h[j] = act[3 * AE_LAT + j] * tanhf(c);
    }
    __syncthreads();
  }
  if (j < AE_LAT) {
    const float v = nan0(h[j]);  // check_and_fix_nan(sequence_feature), cad1:240
    seq[b * AE_LAT + j] = v;
    if (seq_out) seq_out[b * AE_LAT + j] = v;
  }
}

// BPTT, one block per clip in reverse time: thread (q, k) holds column k of W_hh rows [64q, 64q + 64) for
// d h_{t-1} = W_hh^T d gates.  dG = d pre-activation gates per frame (for the W_ih / W_hh / bias GEMMs)
__global__ __launch_bounds__(256) void ae_lstm_bwd_kernel(const float* __restrict__ gates, const float* __restrict__ cs,
                                                          const float* __restrict__ whh,
                                                          const float* __restrict__ dseq, int B, int T,
                                                          float* __restrict__ dG) {
  __shared__ float dg[AE_GATES], part[4][AE_LAT];
  const int b = blockIdx.x, k = threadIdx.x & 63, q = threadIdx.x >> 6;
  float w[AE_LAT];
#pragma unroll
  for (int jj = 0; jj < AE_LAT; ++jj) w[jj] = whh[(int64_t)(q * AE_LAT + jj) * AE_LAT + k];
  float dh = q == 0 ? dseq[b * AE_LAT + k] : 0.f, dc = 0.f;
  for (int t = T - 1; t >= 0; --t) {
    const int64_t n = (int64_t)t * B + b;
    if (q == 0) {
      const float* g = gates + n * AE_GATES;
      const float gi = g[k], gf = g[AE_LAT + k], gg = g[2 * AE_LAT + k], go = g[3 * AE_LAT + k];
      const float c = cs[n * AE_LAT + k];
      const float cp = t > 0 ? cs[(n - B) * AE_LAT + k] : 0.f;
      const float tc = tanhf(c);
      const float dct = dc + dh * go * (1.f - tc * tc);
      const float di = dct * gg * gi * (1.f - gi);
      const float df = dct * cp * gf * (1.f - gf);
      const float dgg = dct * gi * (1.f - gg * gg);
      const float dgo = dh * tc * go * (1.f - go);
      dc = dct * gf;
      dg[k] = di;
      dg[AE_LAT + k] = df;
      dg[2 * AE_LAT + k] = dgg;
      dg[3 * AE_LAT + k] = dgo;
      float* o = dG + n * AE_GATES;
      o[k] = di;
      o[AE_LAT + k] = df;
      o[2 * AE_LAT + k] = dgg;
      o[3 * AE_LAT + k] = dgo;
    }
    __syncthreads();
    float s = 0.f;
#pragma unroll
    for (int jj = 0; jj < AE_LAT; ++jj) s = fmaf(w[jj], dg[q * AE_LAT + jj], s);
    part[q][k] = s;
    __syncthreads();
    if (q == 0) dh = (part[0][k] + part[1][k]) + (part[2][k] + part[3][k]);
  }
}

// ------------------------------------------------------------------ reconstruction loss
// One block per (clip b, 256-pixel chunk): r = sigmoid(y3) with NaN -> 0 (cad1:256); block sums of
// sum_t (r - x_t)^2; with dy, d MSE / d y3 = r (1 - r) * scale * sum_t (r - x_t), scale = 2 / (B*T*4096): the T
// stacked copies of the reconstruction (cad1:258-259, 340-344)
__global__ __launch_bounds__(256) void ae_loss_kernel(const float* __restrict__ y3, const float* __restrict__ xf,
                                                      int B, int T, float scale, float* __restrict__ recon,
                                                      float* __restrict__ dy, float* __restrict__ part) {
  __shared__ float red[256];
  const int b = blockIdx.x / AE_CHUNKS, p = (blockIdx.x % AE_CHUNKS) * 256 + threadIdx.x;
  const float r0 = 1.f / (1.f + expf(-y3[(int64_t)b * AE_PIX + p]));
  const bool isn = r0 != r0;
  const float r = isn ? 0.f : r0;
  float sq = 0.f, sd = 0.f;
  if (xf)
    for (int t = 0; t < T; ++t) {
      const float d = r - xf[((int64_t)t * B + b) * AE_PIX + p];
      sq = fmaf(d, d, sq);
      sd += d;
    }
  if (recon)
    for (int t = 0; t < T; ++t) recon[((int64_t)b * T + t) * AE_PIX + p] = r;
  if (dy) dy[(int64_t)b * AE_PIX + p] = isn ? 0.f : r * (1.f - r) * (sd * scale);
  red[threadIdx.x] = sq;
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if (threadIdx.x < s) red[threadIdx.x] += red[threadIdx.x + s];
    __syncthreads();
  }
  if (threadIdx.x == 0) part[blockIdx.x] = red[0];
}

// losses[0] = MSE, per-clip errors, status 2 (0 when the loss is not finite or a train-loop input was bad)
__global__ __launch_bounds__(256) void ae_loss_finalize_kernel(const float* __restrict__ part, int B, int T,
                                                               const int* bad, int with_loss,
                                                               float* __restrict__ losses,
                                                               float* __restrict__ recon_err) {
  __shared__ double red[256];
  double tot = 0.0;
  for (int b = threadIdx.x; b < B; b += 256) {
    double s = 0.0;
    for (int c = 0; c < AE_CHUNKS; ++c) s += (double)part[b * AE_CHUNKS + c];
    if (recon_err) recon_err[b] = (float)(s / ((double)T * AE_PIX));
    tot += s;
  }
  red[threadIdx.x] = tot;
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if (threadIdx.x < s) red[threadIdx.x] += red[threadIdx.x + s];
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    const float loss = (float)(red[0] / ((double)B * T * AE_PIX));
    const bool ok = !with_loss || (isfinite(loss) && !(bad && *bad));
    losses[0] = with_loss ? loss : 0.f;
    losses[1] = 0.f;
    losses[2] = 0.f;
    losses[3] = ok ? 2.f : 0.f;
  }
}

// module backward: d logits = r (1 - r) * sum_t d_recon[b][t] (the T stacked copies); 0 where r was NaN
__global__ __launch_bounds__(256) void ae_recon_bwd_kernel(const float* __restrict__ y3, const float* __restrict__ drec,
                                                           int B, int T, float* __restrict__ dy) {
  const int64_t total = (int64_t)B * AE_PIX;
  for (int64_t i = blockIdx.x * 256ll + threadIdx.x; i < total; i += (int64_t)gridDim.x * 256) {
    const int64_t b = i / AE_PIX, p = i - b * AE_PIX;
    const float r = 1.f / (1.f + expf(-y3[i]));
    float s = 0.f;
    if (drec)
      for (int t = 0; t < T; ++t) s += drec[(b * T + t) * AE_PIX + p];
    dy[i] = r != r ? 0.f : r * (1.f - r) * s;
  }
}

// ------------------------------------------------------------------ memory ring (cad1:201-219, 262-301)
// one block per sequence feature: min over the first memory_ptr rows of 1 - clamp(cos, -1, 1), clamped to [0, 2],
// halved; 0 while fewer than 10 rows are filled
__global__ __launch_bounds__(256) void ae_memory_score_kernel(const float* __restrict__ memory,
                                                              const int64_t* __restrict__ mptr,
                                                              const float* __restrict__ seq,
                                                              float* __restrict__ scores) {
  __shared__ float sn[AE_LAT];
  __shared__ float red[256];
  const int b = blockIdx.x;
  const int64_t n = min((int64_t)AE_MEM, max((int64_t)0, *mptr));
  if (n < 10) {
    if (threadIdx.x == 0) scores[b] = 0.f;
    return;
  }
  if (threadIdx.x < AE_LAT) {
    const float v = nan0(seq[b * AE_LAT + threadIdx.x]);
    const float nrm = sqrtf(wave_sum(v * v));
    sn[threadIdx.x] = v / fmaxf(nrm, 1e-8f);
  }
  __syncthreads();
  float best = INFINITY;
  for (int64_t m = threadIdx.x; m < n; m += 256) {
    const float* row = memory + m * AE_LAT;
    float ss = 0.f;
    for (int k = 0; k < AE_LAT; ++k) ss = fmaf(row[k], row[k], ss);
    const float nm = fmaxf(sqrtf(ss), 1e-8f);
    float dot = 0.f;
    for (int k = 0; k < AE_LAT; ++k) dot = fmaf(sn[k], row[k] / nm, dot);
    best = fminf(best, 1.f - fminf(fmaxf(dot, -1.f), 1.f));
  }
  red[threadIdx.x] = best;
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if (threadIdx.x < s) red[threadIdx.x] = fminf(red[threadIdx.x], red[threadIdx.x + s]);
    __syncthreads();
  }
  if (threadIdx.x == 0) scores[b] = fminf(fmaxf(red[0], 0.f), 2.f) / 2.f;
}

// ring write of n features at memory_ptr with wrap-around; skipped when status says the batch was skipped
__global__ __launch_bounds__(256) void ae_memory_update_kernel(float* __restrict__ memory, int64_t* mptr,
                                                               const float* __restrict__ f, int n,
                                                               const float* status) {
  if (status && status[3] < 1.f) return;
  const int64_t p = min((int64_t)AE_MEM - 1, max((int64_t)0, *mptr));
  for (int i = threadIdx.x; i < n * AE_LAT; i += 256) {
    const int r = i / AE_LAT, k = i - r * AE_LAT;
    int64_t dst = p + r;
    if (dst >= AE_MEM) dst -= AE_MEM;
    memory[dst * AE_LAT + k] = nan0(f[i]);
  }
  __syncthreads();
  if (threadIdx.x == 0) *mptr = p + n <= AE_MEM ? (p + n) % AE_MEM : p + n - AE_MEM;
}

// num_batches_tracked: + T per train forward for the encoder BNs [0, 4) (one call per t) and the decoder BNs [4, 7)
__global__ void ae_nbt_kernel(int64_t* nbt, int enc, int dec, int add, const int* skip) {
  if (skip && *skip) return;
  const int i = threadIdx.x;
  if (i < AE_NBN && ((i < 4 && enc) || (i >= 4 && dec))) nbt[i] += add;
}

// ------------------------------------------------------------------ the plan
struct AePlanImpl {
  int B, T, NF;
  Conv3dGeom ge[4], gd[4];
  int64_t ws_bytes = 0;
  float *params = nullptr, *grads = nullptr, *bufs = nullptr, *m = nullptr, *v = nullptr, *memory = nullptr;
  int64_t *nbt = nullptr, *mptr = nullptr;
  int32_t* steps = nullptr;
  // workspace
  float *xf, *ecols[4], *ey[4], *ea[4], *est[4], *z, *lat, *gx, *gates, *cs, *hprev, *seq;
  float *u, *dx[4], *dy[4], *dst[3], *dylast, *parts, *bparts, *bparts2 = nullptr, *lpart, *losses, *bufA, *bufB, *bcols;
  float *dG, *dlat, *dz, *da3, *dseq, *dU, *scratch, *bufC = nullptr, *scratch2 = nullptr;
  // implicit-GEMM weight images (conv4_prep): encoder layers 1-3 [Co][16 Ci] (forward) / [4][Ci][4 Co] (input grad),
  // decoder layers [4][Co][4 Ci] (forward) / [Ci][16 Co] (input grad, layers 0-2)
  float *ewk[4] = {}, *ewc[4] = {}, *dwk[4] = {}, *dwc[4] = {};
  const int direct = g_ae_direct;
  const int side = g_ae_direct && g_ae_wgrad_stream;
  hipStream_t sw = nullptr;  // weight-gradient stream (side)
  hipEvent_t ev_fork = nullptr, ev_join = nullptr, ev_wg[2] = {nullptr, nullptr};
  int wg_pending[2] = {0, 0};
  int* bad;
  double* sum_parts;
  AdamWs aws{};
  int64_t scratch_floats = 0;
  // per-call state
  int training = 1, loss_mode = 0, have_fwd = 0;

  AePlanImpl(int B_, int T_) : B(B_), T(T_), NF(B_ * T_) {
    for (int l = 0; l < 4; ++l) ge[l] = ae_geom(NF, ENC_CI[l], ENC_IN[l], ENC_CO[l]);
    // the conv whose input gradient is ConvTranspose2d j: input = the ConvT output (Co channels, 2x size)
    for (int j = 0; j < 4; ++j) gd[j] = ae_geom(B, DEC_CO[j], 2 * DEC_IN[j], DEC_CI[j]);
  }
  float* P(int s) const { return params + ae_layout().slots[s].offset; }
  float* G(int s) const { return grads + ae_layout().slots[s].offset; }
  float* RB(int b) const { return bufs + ae_layout().bufs[b].offset; }
  ~AePlanImpl() {
    for (hipEvent_t e : {ev_fork, ev_join, ev_wg[0], ev_wg[1]})
      if (e) (void)hipEventDestroy(e);
    if (sw) (void)hipStreamDestroy(sw);
  }
  // the weight-gradient stream, ordered after everything queued so far on st (st itself without the side stream)
  int fork(hipStream_t st, hipStream_t* out) {
    *out = st;
    if (!side) return 0;
    if (!sw) {
      int lo = 0, hi = 0;
      VAD_HIP(hipDeviceGetStreamPriorityRange(&lo, &hi));
      VAD_HIP(hipStreamCreateWithPriority(&sw, hipStreamNonBlocking, lo));
      const unsigned evf = hipEventDisableTiming | (unsigned)hipEventDisableSystemFence;
      for (hipEvent_t* e : {&ev_fork, &ev_join, &ev_wg[0], &ev_wg[1]}) VAD_HIP(hipEventCreateWithFlags(e, evf));
    }
    VAD_HIP(hipEventRecord(ev_fork, st));
    VAD_HIP(hipStreamWaitEvent(sw, ev_fork, 0));
    *out = sw;
    return 0;
  }
  // dY buffer k: the side stream's reads of it are queued (mark), st must not overwrite it before they end (reuse)
  int wg_mark(int k) {
    if (!side) return 0;
    VAD_HIP(hipEventRecord(ev_wg[k], sw));
    wg_pending[k] = 1;
    return 0;
  }
  int wg_reuse(int k, hipStream_t st) {
    if (side && wg_pending[k]) VAD_HIP(hipStreamWaitEvent(st, ev_wg[k], 0));
    wg_pending[k] = 0;
    return 0;
  }
  int join(hipStream_t st) {
    if (!side || !sw) return 0;
    VAD_HIP(hipEventRecord(ev_join, sw));
    VAD_HIP(hipStreamWaitEvent(st, ev_join, 0));
    wg_pending[0] = wg_pending[1] = 0;
    return 0;
  }
  Gbn enc_bn(int l) const { return gbn(T, ge[l].rows() / T, ENC_CO[l]); }
  Gbn dec_bn(int j) const { return gbn(1, gd[j].in.voxels(), DEC_CO[j]); }

  void carve(Ws& w) {
    int64_t max_act = (int64_t)NF * AE_FLAT, max_cols = 1, max_parts = 1;
    auto parts_of = [](const Gbn& q) { return (int64_t)q.G * q.P * 2 * q.C; };
    xf = w.take<float>((int64_t)NF * AE_PIX);
    for (int l = 0; l < 4; ++l) {
      const int64_t M = ge[l].rows(), Co = ENC_CO[l];
      ecols[l] = direct ? nullptr : w.take<float>(M * ge[l].K());
      ey[l] = w.take<float>(M * Co);
      ea[l] = w.take<float>(M * Co);
      est[l] = w.take<float>((int64_t)T * AE_ST * Co);
      max_act = std::max(max_act, M * Co);
      if (l > 0 && !direct) max_cols = std::max(max_cols, M * ge[l].K());
      if (direct && l > 0) {
        ewk[l] = w.take<float>(16 * Co * ENC_CI[l]);
        ewc[l] = w.take<float>(16 * Co * ENC_CI[l]);
      }
      max_parts = std::max(max_parts, parts_of(enc_bn(l)));
    }
    z = w.take<float>((int64_t)NF * AE_LAT);
    lat = w.take<float>((int64_t)NF * AE_LAT);
    gx = w.take<float>((int64_t)NF * AE_GATES);
    gates = w.take<float>((int64_t)NF * AE_GATES);
    cs = w.take<float>((int64_t)NF * AE_LAT);
    hprev = w.take<float>((int64_t)NF * AE_LAT);
    seq = w.take<float>((int64_t)B * AE_LAT);
    u = w.take<float>((int64_t)B * AE_FLAT);
    for (int j = 0; j < 4; ++j) {
      const int64_t rows = gd[j].rows();
      dx[j] = w.take<float>(rows * DEC_CI[j]);
      dy[j] = w.take<float>(gd[j].in.numel());
      max_act = std::max(max_act, std::max(gd[j].in.numel(), rows * DEC_CI[j]));
      if (!direct) max_cols = std::max(max_cols, rows * gd[j].K());
      if (direct && j < 3) {
        dwc[j] = w.take<float>(16 * DEC_CI[j] * DEC_CO[j]);
        dwk[j] = w.take<float>(16 * DEC_CI[j] * DEC_CO[j]);
      }
      if (j < 3) {
        dst[j] = w.take<float>((int64_t)AE_ST * DEC_CO[j]);
        max_parts = std::max(max_parts, parts_of(dec_bn(j)));
      }
    }
    dylast = w.take<float>((int64_t)B * AE_PIX);
    parts = w.take<float>(max_parts);
    bparts = w.take<float>(max_parts);
    if (side) bparts2 = w.take<float>(max_parts);
    lpart = w.take<float>((int64_t)B * AE_CHUNKS);
    losses = w.take<float>(4);
    bufA = w.take<float>(max_act);
    bufB = w.take<float>(max_act);
    if (side) bufC = w.take<float>(max_act);
    bcols = w.take<float>(max_cols);
    dG = w.take<float>((int64_t)NF * AE_GATES);
    dlat = w.take<float>((int64_t)NF * AE_LAT);
    dz = w.take<float>((int64_t)NF * AE_LAT);
    da3 = w.take<float>((int64_t)NF * AE_FLAT);
    dseq = w.take<float>((int64_t)B * AE_LAT);
    dU = w.take<float>((int64_t)B * AE_FLAT);
    scratch_floats = 32ll << 20;  // (split-K slabs of the weight gradients: 128 MB)
    scratch = w.take<float>(scratch_floats);
    if (side) scratch2 = w.take<float>(scratch_floats);
    bad = w.take<int>(4);
    aws.sq = w.take<double>(ADAM_MAX_SLOTS * ADAM_SQ_CHUNKS);
    aws.bad = w.take<int>(ADAM_MAX_SLOTS * ADAM_SQ_CHUNKS);
    sum_parts = w.take<double>(AE_SUM_BLOCKS);
    aws.ctrl = w.take<float>(4);
  }

  // train-mode statistics (+ running stats) or eval-mode affine, then A = LeakyReLU(BN(y))
  int bn_fwd(const float* y, const Gbn& q, int gw, int gb, int rm, int rv, int repeat, const int* skip,
             float* stats, float* act, int hw_perm, hipStream_t st) {
    if (training) {
      hipLaunchKernelGGL(gbn_partials_kernel, dim3(q.P, q.G), dim3(256), 0, st, y, q, parts);
      VAD_LAUNCH_CHECK();
    }
    hipLaunchKernelGGL(gbn_finalize_kernel, dim3(q.C), dim3(256), 0, st, parts, q, P(gw), P(gb), RB(rm), RB(rv),
                       training, repeat, skip, stats);
    VAD_LAUNCH_CHECK();
    const int64_t M = (int64_t)q.G * q.Mg;
    hipLaunchKernelGGL(gbn_act_kernel, grid_for(M * q.C / 4), dim3(256), 0, st, y, stats, M, q.Mg, q.C, hw_perm,
                       act);
    VAD_LAUNCH_CHECK();
    return 0;
  }

  // dY = grad through LeakyReLU(BN(y)) given dA; gamma / beta grads into slots gw / gb; dbias (nullable) = sum(dY)
  // kb: the dY buffer's index -- with the side stream the conv-bias sum (dbias) runs there, on bparts / bparts2 by kb
  // (the same reuse event as the dY buffer: the side stream's weight gradient of dY is queued after it)
  int bn_bwd(const float* dA, const float* y, const Gbn& q, int gw, int gb, float* stats, float* dY, float* dbias,
             hipStream_t st, int kb = 0) {
    float* const bp = side && kb ? bparts2 : bparts;
    hipLaunchKernelGGL(gbn_bwd_reduce_kernel, dim3(q.P, q.G), dim3(256), 0, st, dA, y, stats, q, parts);
    VAD_LAUNCH_CHECK();
    hipLaunchKernelGGL(gbn_bwd_finalize_kernel, dim3(q.C), dim3(256), 0, st, parts, q, P(gw), training, stats, G(gw),
                       G(gb));
    VAD_LAUNCH_CHECK();
    hipLaunchKernelGGL(gbn_bwd_apply_kernel, dim3(q.P, q.G), dim3(256), 0, st, dA, y, stats, q, dY,
                       dbias ? bp : nullptr);
    VAD_LAUNCH_CHECK();
    if (dbias) {
      hipStream_t bs = st;
      VAD_TRY(fork(st, &bs));
      hipLaunchKernelGGL(ae_bias_reduce_kernel, dim3((unsigned)q.C), dim3(256), 0, bs, bp, q.G * q.P, q.C, dbias);
      VAD_LAUNCH_CHECK();
    }
    return 0;
  }

  int forward(const float* x, const float* seq_in, int stages, float* recon, float* seq_out, float* ff,
              float* scores, float* recon_err, hipStream_t st) {
    const AeLayout& L = ae_layout();
    const bool enc = stages & 1, dec = stages & 2;
    const int* skip = loss_mode == 2 ? bad : nullptr;
    bool dec_prepped = false, prep_wait = false;
    const DenseAct none{};
    VAD_HIP(hipMemsetAsync(bad, 0, sizeof(int), st));
    if (enc) {
      hipLaunchKernelGGL(ae_frames_kernel, grid_for((int64_t)NF * AE_PIX / 4), dim3(256), 0, st, x, B, T, xf, bad);
      VAD_LAUNCH_CHECK();
      if (direct) {  // the weight images on the side stream, beside the first layer (waited for before layer 1)
        hipStream_t ps = st;
        VAD_TRY(fork(st, &ps));
        for (int l = 1; l < 4; ++l) VAD_TRY(conv4_prep(P(L.enc_w[l]), ENC_CO[l], ENC_CI[l], ewk[l], ewc[l], ps));
        if (dec)
          for (int j = 0; j < 3; ++j) VAD_TRY(conv4_prep(P(L.dec_w[j]), DEC_CI[j], DEC_CO[j], dwk[j], dwc[j], ps));
        dec_prepped = dec;
        if (ps != st) {
          VAD_HIP(hipEventRecord(ev_join, ps));
          prep_wait = true;
        }
      }
      for (int l = 0; l < 4; ++l) {
        const int64_t M = ge[l].rows();
        if (direct && l == 0) {
          VAD_TRY(conv4_c1_fwd(xf, NF, AE_HW, AE_HW, P(L.enc_w[0]), P(L.enc_b[0]), ey[0], st));
        } else if (direct) {
          if (prep_wait) VAD_HIP(hipStreamWaitEvent(st, ev_join, 0));
          prep_wait = false;
          VAD_TRY(conv4_fwd(ea[l - 1], NF, ENC_IN[l], ENC_IN[l], ENC_CI[l], ewk[l], P(L.enc_b[l]), ENC_CO[l], ey[l],
                            st, scratch, scratch_floats));
        } else {
          VAD_TRY(im2col3d(l == 0 ? xf : ea[l - 1], ndhwc_strides(ge[l].in), ge[l], nullptr, nullptr, 0, ecols[l],
                           st));
          VAD_TRY(dense_fwd(ecols[l], (int)M, ge[l].K(), P(L.enc_w[l]), P(L.enc_b[l]), ENC_CO[l], ey[l], none,
                            scratch, scratch_floats, st));
        }
        VAD_TRY(bn_fwd(ey[l], enc_bn(l), L.ebn_w[l], L.ebn_b[l], L.erm[l], L.erv[l], 1, skip, est[l], ea[l],
                       l == 3 ? 16 : 0, st));
      }
      VAD_TRY(dense_fwd(ea[3], NF, AE_FLAT, P(L.efc_w), P(L.efc_b), AE_LAT, z, none, scratch, scratch_floats, st));
      hipLaunchKernelGGL(ae_latent_kernel, grid_for((int64_t)NF * AE_LAT), dim3(256), 0, st, z, B, T, lat, ff);
      VAD_LAUNCH_CHECK();
      VAD_TRY(dense_fwd(lat, NF, AE_LAT, P(L.wih), P(L.bih), AE_GATES, gx, none, scratch, scratch_floats, st));
      hipLaunchKernelGGL(ae_lstm_fwd_kernel, dim3(B), dim3(AE_GATES), 0, st, gx, P(L.whh), P(L.bhh), B, T, gates,
                         cs, hprev, seq, seq_out);
      VAD_LAUNCH_CHECK();
    } else {
      hipLaunchKernelGGL(ae_seq_in_kernel, grid_for((int64_t)B * AE_LAT), dim3(256), 0, st, seq_in, B * AE_LAT, seq,
                         seq_out);
      VAD_LAUNCH_CHECK();
    }
    if (scores) {
      hipLaunchKernelGGL(ae_memory_score_kernel, dim3(B), dim3(256), 0, st, memory, mptr, seq, scores);
      VAD_LAUNCH_CHECK();
    }
    if (dec) {
      VAD_TRY(dense_fwd(seq, B, AE_LAT, P(L.dfc_w), P(L.dfc_b), AE_FLAT, u, none, scratch, scratch_floats, st));
      hipLaunchKernelGGL(ae_dec_in_kernel, grid_for((int64_t)B * AE_FLAT), dim3(256), 0, st, u, B, dx[0]);
      VAD_LAUNCH_CHECK();
      if (direct && !dec_prepped)
        for (int j = 0; j < 3; ++j) VAD_TRY(conv4_prep(P(L.dec_w[j]), DEC_CI[j], DEC_CO[j], dwk[j], dwc[j], st));
      for (int j = 0; j < 4; ++j) {
        if (direct && j == 3) {  // ConvTranspose2d(32, 1): 128 MACs per output pixel on the VALU
          VAD_TRY(conv4_c1_tfwd(dx[3], B, DEC_IN[3], DEC_IN[3], P(L.dec_w[3]), P(L.dec_b[3]), dy[3], st));
        } else if (direct) {  // ConvTranspose2d j: four parity-class GEMMs, bias in the epilogue
          VAD_TRY(conv4_cls(dx[j], B, DEC_IN[j], DEC_IN[j], DEC_CI[j], dwc[j], P(L.dec_b[j]), DEC_CO[j], dy[j], st,
                            scratch, scratch_floats));
        } else {
          // columns = X_j Wt (the transposed conv's GEMM), col2im + bias
          VAD_TRY(dense_dgrad(dx[j], (int)gd[j].rows(), DEC_CI[j], P(L.dec_w[j]), gd[j].K(), bcols, nullptr, 1.f,
                              nullptr, st));
          VAD_TRY(col2im3d(bcols, gd[j], dy[j], st, P(L.dec_b[j])));
        }
        if (j < 3)
          VAD_TRY(bn_fwd(dy[j], dec_bn(j), L.dbn_w[j], L.dbn_b[j], L.drm[j], L.drv[j], T, skip, dst[j], dx[j + 1], 0,
                         st));
      }
      const bool lossy = loss_mode != 0 && enc;
      hipLaunchKernelGGL(ae_loss_kernel, dim3(B * AE_CHUNKS), dim3(256), 0, st, dy[3], lossy ? xf : nullptr, B, T,
                         (float)(2.0 / ((double)B * T * AE_PIX)), recon,
                         (loss_mode == 2 && training) ? dylast : nullptr, lpart);
      VAD_LAUNCH_CHECK();
      hipLaunchKernelGGL(ae_loss_finalize_kernel, dim3(1), dim3(256), 0, st, lpart, B, T, skip, lossy ? 1 : 0, losses,
                         lossy ? recon_err : nullptr);
      VAD_LAUNCH_CHECK();
    }
    if (training) {
      hipLaunchKernelGGL(ae_nbt_kernel, dim3(1), dim3(64), 0, st, nbt, enc ? 1 : 0, dec ? 1 : 0, T, skip);
      VAD_LAUNCH_CHECK();
    }
    if (loss_mode == 2) {  // after the score: the reference scores against the ring before updating it
      hipLaunchKernelGGL(ae_memory_update_kernel, dim3(1), dim3(256), 0, st, memory, mptr, seq, B, losses);
      VAD_LAUNCH_CHECK();
    }
    have_fwd = stages == 3;
    return 0;
  }

  int backward(int use_loss, const float* d_recon, const float* d_seq, const float* d_ff, hipStream_t st) {
    const AeLayout& L = ae_layout();
    const DenseAct none{};
    VAD_CHECK(have_fwd, "vad_ae_backward: needs a preceding full forward (stages 3) of this plan");
    VAD_CHECK(!use_loss || (loss_mode == 2 && training),
              "vad_ae_backward: use_loss needs the train_model forward (loss_mode 2, training)");
    if (!use_loss) {
      hipLaunchKernelGGL(ae_recon_bwd_kernel, grid_for((int64_t)B * AE_PIX), dim3(256), 0, st, dy[3], d_recon, B, T,
                         dylast);
      VAD_LAUNCH_CHECK();
    }
    // direct mode with the side stream: weight gradients (and their split-K reduces) on sw with scratch2, dY of the
    // BN backwards alternating between bufB / bufC so the next layer's dY never overwrites one still being read
    float* const dyb[2] = {bufB, side ? bufC : bufB};
    int kb = 1;
    auto next_dy = [&](hipStream_t s) -> float* {
      kb ^= side;
      if (wg_reuse(kb, s)) return nullptr;
      return dyb[kb];
    };
    float* const scr2 = side ? scratch2 : scratch;
    hipStream_t ws = st;
    VAD_TRY(fork(st, &ws));
    hipLaunchKernelGGL(ae_sum_parts_kernel, dim3(AE_SUM_BLOCKS), dim3(256), 0, ws, dylast, (int64_t)B * AE_PIX,
                       sum_parts);
    VAD_LAUNCH_CHECK();
    hipLaunchKernelGGL(ae_sum_kernel, dim3(1), dim3(AE_SUM_BLOCKS), 0, ws, sum_parts, G(L.dec_b[3]));
    VAD_LAUNCH_CHECK();
    // decoder, last ConvTranspose2d first: dX_j = im2col(dY_j) Wt^T, dWt = X_j^T im2col(dY_j)
    const float* dcur = dylast;
    for (int j = 3; j >= 0; --j) {
      const int M = (int)gd[j].rows(), K = gd[j].K(), Ci = DEC_CI[j];
      if (direct && j == 3) {
        VAD_TRY(conv4_c1_wgrad(dx[3], dcur, B, DEC_IN[3], DEC_IN[3], G(L.dec_w[3]), scr2, scratch_floats, ws));
        VAD_TRY(conv4_c1_fwd(dcur, B, 2 * DEC_IN[3], 2 * DEC_IN[3], P(L.dec_w[3]), nullptr, bufA, st));
      } else if (direct) {
        int ns = 0;
        VAD_TRY(fork(st, &ws));
        VAD_TRY(conv4_wgrad(dx[j], Ci, dcur, DEC_CO[j], B, DEC_IN[j], DEC_IN[j], scr2, &ns, scratch_floats,
                            g_ae_wgrad_blocks, ws));
        VAD_TRY(conv4_wgrad_reduce(scr2, ns, Ci, DEC_CO[j], G(L.dec_w[j]), ws));
        VAD_TRY(wg_mark(kb));
        VAD_TRY(conv4_fwd(dcur, B, 2 * DEC_IN[j], 2 * DEC_IN[j], DEC_CO[j], dwk[j], nullptr, Ci, bufA, st, scratch,
                          scratch_floats));
      } else {
        VAD_TRY(im2col3d(dcur, ndhwc_strides(gd[j].in), gd[j], nullptr, nullptr, 0, bcols, st));
        VAD_TRY(dense_wgrad(dx[j], M, Ci, bcols, K, G(L.dec_w[j]), nullptr, scratch, scratch_floats, nullptr, st));
        VAD_TRY(dense_fwd(bcols, M, K, P(L.dec_w[j]), nullptr, Ci, bufA, none, scratch, scratch_floats, st));
      }
      if (j > 0) {
        // X_j = LeakyReLU(BN_{j-1}(y_{j-1})); sum(dY_{j-1}) is the bias grad of ConvTranspose2d j-1
        float* dY = next_dy(st);
        VAD_CHECK(dY != nullptr, "vad_ae_backward: stream wait failed");
        VAD_TRY(bn_bwd(bufA, dy[j - 1], dec_bn(j - 1), L.dbn_w[j - 1], L.dbn_b[j - 1], dst[j - 1], dY,
                       G(L.dec_b[j - 1]), st, kb));
        dcur = dY;
      }
    }
    hipLaunchKernelGGL(ae_dec_in_bwd_kernel, grid_for((int64_t)B * AE_FLAT), dim3(256), 0, st, bufA, u, B, dU);
    VAD_LAUNCH_CHECK();
    VAD_TRY(fork(st, &ws));
    VAD_TRY(dense_wgrad(dU, B, AE_FLAT, seq, AE_LAT, G(L.dfc_w), G(L.dfc_b), scr2, scratch_floats, nullptr, ws));
    VAD_TRY(dense_dgrad(dU, B, AE_FLAT, P(L.dfc_w), AE_LAT, dseq, nullptr, 1.f, nullptr, st, 0, scratch,
                        scratch_floats));
    if (d_seq) {
      hipLaunchKernelGGL(ae_add_kernel, grid_for((int64_t)B * AE_LAT), dim3(256), 0, st, dseq, d_seq,
                         (int64_t)B * AE_LAT);
      VAD_LAUNCH_CHECK();
    }
    // LSTM BPTT, then the W_ih / W_hh / bias grads and d latents as GEMMs over all frames
    hipLaunchKernelGGL(ae_lstm_bwd_kernel, dim3(B), dim3(AE_GATES), 0, st, gates, cs, P(L.whh), dseq, B, T, dG);
    VAD_LAUNCH_CHECK();
    VAD_TRY(fork(st, &ws));
    VAD_TRY(dense_wgrad(dG, NF, AE_GATES, lat, AE_LAT, G(L.wih), G(L.bih), scr2, scratch_floats, nullptr, ws));
    VAD_TRY(dense_wgrad(dG, NF, AE_GATES, hprev, AE_LAT, G(L.whh), G(L.bhh), scr2, scratch_floats, nullptr, ws));
    VAD_TRY(dense_dgrad(dG, NF, AE_GATES, P(L.wih), AE_LAT, dlat, nullptr, 1.f, nullptr, st));
    hipLaunchKernelGGL(ae_latent_bwd_kernel, grid_for((int64_t)NF * AE_LAT), dim3(256), 0, st, dlat, d_ff, lat, z, B,
                       T, dz);
    VAD_LAUNCH_CHECK();
    VAD_TRY(fork(st, &ws));
    VAD_TRY(dense_wgrad(dz, NF, AE_LAT, ea[3], AE_FLAT, G(L.efc_w), G(L.efc_b), scr2, scratch_floats, nullptr, ws));
    VAD_TRY(dense_dgrad(dz, NF, AE_LAT, P(L.efc_w), AE_FLAT, da3, nullptr, 1.f, nullptr, st));
    hipLaunchKernelGGL(ae_unflatten_kernel, grid_for((int64_t)NF * AE_FLAT), dim3(256), 0, st, da3, (int64_t)NF, 128,
                       16, bufA);
    VAD_LAUNCH_CHECK();
    // encoder, last layer first
    for (int l = 3; l >= 0; --l) {
      const int M = (int)ge[l].rows(), K = ge[l].K(), Co = ENC_CO[l];
      if (direct && l == 0) {  // Conv2d(1, 32): weight grad on the VALU, the bias grad from the BN backward
        float* dY = next_dy(st);
        VAD_CHECK(dY != nullptr, "vad_ae_backward: stream wait failed");
        VAD_TRY(bn_bwd(bufA, ey[0], enc_bn(0), L.ebn_w[0], L.ebn_b[0], est[0], dY, G(L.enc_b[0]), st, kb));
        VAD_TRY(fork(st, &ws));
        VAD_TRY(conv4_c1_wgrad(dY, xf, NF, ENC_IN[0] / 2, ENC_IN[0] / 2, G(L.enc_w[0]), scr2, scratch_floats, ws));
        continue;
      }
      if (direct) {  // (the conv bias grad = sum of dY, from the BN backward's apply pass)
        const int OH = ENC_IN[l] / 2;
        int ns = 0;
        float* dY = next_dy(st);
        VAD_CHECK(dY != nullptr, "vad_ae_backward: stream wait failed");
        VAD_TRY(bn_bwd(bufA, ey[l], enc_bn(l), L.ebn_w[l], L.ebn_b[l], est[l], dY, G(L.enc_b[l]), st, kb));
        VAD_TRY(fork(st, &ws));
        VAD_TRY(conv4_wgrad(dY, Co, ea[l - 1], ENC_CI[l], NF, OH, OH, scr2, &ns, scratch_floats, g_ae_wgrad_blocks,
                            ws));
        VAD_TRY(conv4_wgrad_reduce(scr2, ns, Co, ENC_CI[l], G(L.enc_w[l]), ws));
        VAD_TRY(wg_mark(kb));
        VAD_TRY(conv4_cls(dY, NF, OH, OH, Co, ewc[l], nullptr, ENC_CI[l], bufA, st, scratch, scratch_floats));
        continue;
      }
      VAD_TRY(bn_bwd(bufA, ey[l], enc_bn(l), L.ebn_w[l], L.ebn_b[l], est[l], bufB, nullptr, st));
      VAD_TRY(dense_wgrad(bufB, M, Co, ecols[l], K, G(L.enc_w[l]), G(L.enc_b[l]), scratch, scratch_floats, nullptr,
                          st));
      if (l > 0) {
        VAD_TRY(dense_dgrad(bufB, M, Co, P(L.enc_w[l]), K, bcols, nullptr, 1.f, nullptr, st));
        VAD_TRY(col2im3d(bcols, ge[l], bufA, st));
      }
    }
    return join(st);
  }

  int optimizer(float lr, float b1, float b2, float eps, float wd, float max_norm, float grad_scale, hipStream_t st) {
    const AeLayout& L = ae_layout();
    AdamSlots t{};
    t.n = (int)L.slots.size();
    VAD_CHECK(t.n <= ADAM_MAX_SLOTS, "vad_ae_optimizer_step: slot table overflow");
    for (int i = 0; i < t.n; ++i) {
      t.off[i] = L.slots[i].offset;
      t.numel[i] = L.slots[i].numel;
    }
    // clip_grad_norm_(max_norm) on every step (cad1:424): clip_above < 0
    return adam_clip_step(t, params, grads, m, v, L.param_floats, steps, losses, aws, lr, b1, b2, eps, wd, -1.f,
                          max_norm, grad_scale, st);
  }
};

}  // namespace vad

using namespace vad;

struct vad_ae_plan {
  vad_ae_plan(int B, int T) : impl(B, T) {}
  AePlanImpl impl;
  float* user_losses = nullptr;
};

extern "C" {

int vad_ae_num_slots(void) { return (int)ae_layout().slots.size(); }
const char* vad_ae_slot_name(int i) {
  return (i >= 0 && i < vad_ae_num_slots()) ? ae_layout().slots[i].name.c_str() : nullptr;
}
int64_t vad_ae_slot_numel(int i) { return (i >= 0 && i < vad_ae_num_slots()) ? ae_layout().slots[i].numel : -1; }
int64_t vad_ae_slot_offset(int i) { return (i >= 0 && i < vad_ae_num_slots()) ? ae_layout().slots[i].offset : -1; }
int64_t vad_ae_param_floats(void) { return ae_layout().param_floats; }
int vad_ae_num_bufs(void) { return (int)ae_layout().bufs.size(); }
const char* vad_ae_buf_name(int i) {
  return (i >= 0 && i < vad_ae_num_bufs()) ? ae_layout().bufs[i].name.c_str() : nullptr;
}
int64_t vad_ae_buf_numel(int i) { return (i >= 0 && i < vad_ae_num_bufs()) ? ae_layout().bufs[i].numel : -1; }
int64_t vad_ae_buf_offset(int i) { return (i >= 0 && i < vad_ae_num_bufs()) ? ae_layout().bufs[i].offset : -1; }
int64_t vad_ae_buf_floats(void) { return ae_layout().buf_floats; }

int vad_ae_create(int B, int T, vad_ae_plan** out) {
  VAD_CHECK(out != nullptr, "vad_ae_create: out is null");
  VAD_CHECK(B >= 1 && B <= AE_MEM && T >= 1 && T <= 4096,
            "vad_ae_create: unsupported shape (1 <= B <= 500: update_memory writes B rows of the 500-row ring)");
  auto* p = new vad_ae_plan(B, T);
  Ws ws;
  p->impl.carve(ws);
  p->impl.ws_bytes = ws.off + 256;
  *out = p;
  return 0;
}

void vad_ae_destroy(vad_ae_plan* plan) { delete plan; }
int64_t vad_ae_workspace_bytes(const vad_ae_plan* p) { return p ? p->impl.ws_bytes : -1; }

int vad_ae_bind(vad_ae_plan* plan, void* workspace, float* params, float* grads, float* bufs, int64_t* nbt,
                float* memory, int64_t* memory_ptr, float* exp_avg, float* exp_avg_sq, int32_t* steps) {
  VAD_CHECK(plan && workspace && params && grads && bufs && nbt && memory && memory_ptr, "vad_ae_bind: null argument");
  VAD_CHECK((reinterpret_cast<uintptr_t>(workspace) & 255) == 0, "vad_ae_bind: workspace must be 256-B aligned");
  AePlanImpl& c = plan->impl;
  Ws ws;
  ws.base = reinterpret_cast<char*>(workspace);
  ws.dry = false;
  c.carve(ws);
  c.params = params;
  c.grads = grads;
  c.bufs = bufs;
  c.nbt = nbt;
  c.memory = memory;
  c.mptr = memory_ptr;
  c.m = exp_avg;
  c.v = exp_avg_sq;
  c.steps = steps;
  return 0;
}

int vad_ae_forward(vad_ae_plan* plan, const float* x, const float* seq_in, int stages, int training, int loss_mode,
                   float* recon, float* seq, float* frame_feats, float* scores, float* recon_err, float* losses,
                   void* stream) {
  VAD_CHECK(plan != nullptr, "vad_ae_forward: null plan");
  AePlanImpl& c = plan->impl;
  VAD_CHECK(c.params != nullptr, "vad_ae_forward: plan not bound");
  VAD_CHECK(stages >= 1 && stages <= 3, "vad_ae_forward: stages must be 1 (encode), 2 (decode) or 3 (both)");
  VAD_CHECK(!(stages & 1) || (x && (reinterpret_cast<uintptr_t>(x) & 15) == 0),
            "vad_ae_forward: x must be a 16-byte aligned device pointer");
  VAD_CHECK(stages != 2 || seq_in != nullptr, "vad_ae_forward: decode-only needs seq_in");
  VAD_CHECK(loss_mode >= 0 && loss_mode <= 2 && (loss_mode == 0 || stages == 3),
            "vad_ae_forward: loss_mode 1/2 needs the full forward (stages 3)");
  VAD_CHECK(loss_mode != 2 || training, "vad_ae_forward: the train_model iteration (loss_mode 2) runs in training mode");
  VAD_CHECK(recon_err == nullptr || loss_mode != 0, "vad_ae_forward: recon_err needs loss_mode 1 or 2");
  VAD_CHECK(scores == nullptr || stages == 3, "vad_ae_forward: scores need the full forward");
  hipStream_t st = (hipStream_t)stream;
  c.training = training ? 1 : 0;
  c.loss_mode = loss_mode;
  VAD_TRY(c.forward(x, seq_in, stages, recon, seq, frame_feats, scores, recon_err, st));
  plan->user_losses = losses;
  if (losses) VAD_HIP(hipMemcpyAsync(losses, c.losses, 4 * sizeof(float), hipMemcpyDeviceToDevice, st));
  return 0;
}

int vad_ae_backward(vad_ae_plan* plan, int use_loss, const float* d_recon, const float* d_seq,
                    const float* d_frame_feats, void* stream) {
  VAD_CHECK(plan != nullptr, "vad_ae_backward: null plan");
  return plan->impl.backward(use_loss, d_recon, d_seq, d_frame_feats, (hipStream_t)stream);
}

int vad_ae_optimizer_step(vad_ae_plan* plan, float lr, float beta1, float beta2, float eps, float weight_decay,
                          float max_norm, float grad_scale, void* stream) {
  VAD_CHECK(plan != nullptr, "vad_ae_optimizer_step: null plan");
  AePlanImpl& c = plan->impl;
  hipStream_t st = (hipStream_t)stream;
  VAD_TRY(c.optimizer(lr, beta1, beta2, eps, weight_decay, max_norm, grad_scale, st));
  if (plan->user_losses)
    VAD_HIP(hipMemcpyAsync(plan->user_losses, c.losses, 4 * sizeof(float), hipMemcpyDeviceToDevice, st));
  return 0;
}

int vad_ae_debug_buffer(vad_ae_plan* plan, const char* name, int idx, void** ptr, int64_t* nfloats) {
  VAD_CHECK(plan && name && ptr && nfloats, "vad_ae_debug_buffer: null argument");
  AePlanImpl& c = plan->impl;
  const std::string n(name);
  if (n == "ey" && idx >= 0 && idx < 4) { *ptr = c.ey[idx]; *nfloats = c.ge[idx].rows() * ENC_CO[idx]; }
  else if (n == "est" && idx >= 0 && idx < 4) { *ptr = c.est[idx]; *nfloats = (int64_t)c.T * AE_ST * ENC_CO[idx]; }
  else if (n == "dy" && idx >= 0 && idx < 3) { *ptr = c.dy[idx]; *nfloats = c.gd[idx].in.numel(); }
  else if (n == "dst" && idx >= 0 && idx < 3) { *ptr = c.dst[idx]; *nfloats = (int64_t)AE_ST * DEC_CO[idx]; }
  else if (n == "u") { *ptr = c.u; *nfloats = (int64_t)c.B * AE_FLAT; }
  else { vad::set_error("vad_ae_debug_buffer: unknown buffer " + n); return 1; }
  return 0;
}

int vad_ae_update_memory(float* memory, int64_t* memory_ptr, const float* features, int n, void* stream) {
  VAD_CHECK(memory && memory_ptr && features && n >= 0 && n <= AE_MEM,
            "vad_ae_update_memory: bad arguments (at most 500 features of 64)");
  if (n == 0) return 0;
  hipLaunchKernelGGL(ae_memory_update_kernel, dim3(1), dim3(256), 0, (hipStream_t)stream, memory, memory_ptr,
                     features, n, nullptr);
  VAD_LAUNCH_CHECK();
  return 0;
}

int vad_ae_memory_score(const float* memory, const int64_t* memory_ptr, const float* seq, int n, float* scores,
                        void* stream) {
  VAD_CHECK(memory && memory_ptr && seq && scores && n >= 0, "vad_ae_memory_score: bad arguments");
  if (n == 0) return 0;
  hipLaunchKernelGGL(ae_memory_score_kernel, dim3(n), dim3(256), 0, (hipStream_t)stream, memory, memory_ptr, seq,
                     scores);
  VAD_LAUNCH_CHECK();
  return 0;
}

}  // extern "C"
