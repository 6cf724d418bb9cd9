// Per-frame CNN kernels for gfx950: conv1 (direct, VALU), 3x3 convs (implicit GEMM on f32 MFMA),
// train-mode BatchNorm forward/backward, max/adaptive-avg pooling, and the dense-layer GEMMs.
// Reference semantics: ResNetBackbone (causal_anomaly_detection.py:110-158), nn.BatchNorm2d train mode,
// nn.MaxPool2d(3,2,1), nn.AdaptiveAvgPool2d((4,6)), nn.Linear / ReLU / Dropout stacks (cad:167-179, 525-538).
#include <type_traits>

#include "backbone.h"
#include "conv3d.h"
#include "mlp.h"
#include "gemm.h"
#include "head.h"

namespace vad {

int g_cad_prep_stream = 1;   // knob "cad_prep_stream": weight relayouts on the plan's side stream (A/B measurement)
int g_cad_last_wgrad_main = 1;  // knob "cad_last_wgrad_main": layer 0's weight gradient on the caller's stream
int g_cad_event_sysfence = 0;  // knob "cad_event_sysfence": system-scope fence on the plan's stream-order events
int g_cad_dy_per_layer = 1;  // knob "cad_dy_per_layer" (A/B of the plan option dy_per_layer)
int g_cad_stem_early = 1;  // knob "cad_stem_early": an armed forward (vad_cad_input_ready) runs its stem early (0: off)
int g_cad_det_gate = 1;      // knob "cad_det_gate": the backbone backward waits on the device detector gate
int g_cad_dir_affine = 1;  // knob "cad_dir_affine": direct classifier backward as A + c beta, precomputed in the forward
int g_cad_wgrad_stream = 1;  // knob "cad_wgrad_stream": backbone weight gradients on their own stream
// knob "bn_bwd_fuse": the BN-backward reduce in the input gradients' epilogues -- bit 0 the stride-1 kernels, bit 1 the
// stride-2 one (A/B at config 2: both 1.922 -> 1.893 ms, stride-1 only 1.927 -> 1.922, profiles/r03_bnfuse_ab.json)
int g_bn_bwd_fuse = 3;
int g_cad_stream_prio = 1;  // knob "cad_stream_prio" (cad_plan.hip streams(); A/B profiles/r03_prio_ab.json)
int g_cad_l0_slab = 1;  // knob "cad_l0_slab": layer 0's weight gradient on a split-K slab of its own (no wait for layer 1's)

// =====================================================================================================
// conv1: 1 -> 32 channels, 7x7, stride 2, pad 3, as a K=49 (padded to 56) GEMM on f32 MFMA.
// One block = one frame x a band of C1_RB output rows.  The zero-padded input band is staged in LDS; each wave
// walks 32-pixel tiles of the band: lane (i, h) gathers its A operand patch[2*oy+kh][2*ox+kw] straight from LDS
// (k = 8*kk + 4*h + s), its B operand (weights of channel lane&31) lives in 28 registers for the whole block.
// Epilogue: +bias, NHWC store (one 128-B row per pixel), per-block BN partial sums (deterministic).
// =====================================================================================================
constexpr int C1_RB = 6;  // 114 output rows at 227x227 = 19 full bands; 2432 blocks balance over 256 CUs
constexpr int C1_CO = 32;
constexpr int C1_K = 56;  // 49 taps padded to 7 MFMA sub-steps of 8

__global__ __launch_bounds__(256) void conv1_kernel(const float* __restrict__ x, int H, int W,
                                                    const float* __restrict__ w, const float* __restrict__ bias,
                                                    float* __restrict__ y, int OH, int OW, int bands,
                                                    float* __restrict__ partials) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int img = blockIdx.x / bands, band = blockIdx.x % bands;
  const int r0 = band * C1_RB;
  const int PW = 2 * OW + 6;  // padded band width
  const int PH = 2 * C1_RB + 5;
  float* patch = sm;  // [PH][PW]
  const float* xi = x + (int64_t)img * H * W;
  for (int i = threadIdx.x; i < PH * PW; i += 256) {
    const int pr = i / PW, pc = i - pr * PW;
    const int ih = 2 * r0 - 3 + pr, iw = pc - 3;
    patch[i] = (ih >= 0 && ih < H && iw >= 0 && iw < W) ? xi[(int64_t)ih * W + iw] : 0.f;
  }
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int j = lane & 31, h = lane >> 5;
  // B operand: w[j][k] for k = 8*kk + 4*h + s, zero for k >= 49.  The A operand's patch offset of tap k,
  // (k/7)*PW + k%7, is rebuilt per MFMA from compile-time row/col constants selected by h (no 28-register
  // offset table: 4 instead of 3 waves per SIMD)
  float wr[28];
#pragma unroll
  for (int kk = 0; kk < 7; ++kk)
#pragma unroll
    for (int s4 = 0; s4 < 4; ++s4) {
      const int k = kk * 8 + 4 * h + s4;
      wr[kk * 4 + s4] = k < 49 ? w[j * 49 + k] : 0.f;
    }
  const float bj = bias[j];
  __syncthreads();
  const int rows = min(C1_RB, OH - r0);
  const int npix = rows * OW;
  float s1 = 0.f, s2 = 0.f;
  for (int t0 = wave * 32; t0 < npix; t0 += 4 * 32) {
    // this lane's pixel for the A operand: i = lane & 31
    const int pa = t0 + (lane & 31);
    const int pac = pa < npix ? pa : npix - 1;
    const int oy = pac / OW, ox = pac - oy * OW;
    const float* pp = patch + (2 * oy) * PW + 2 * ox;
    f32x16 acc;
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[r] = 0.f;
#pragma unroll
    for (int q = 0; q < 28; ++q) {
      const int k0 = (q >> 2) * 8 + (q & 3), k1 = k0 + 4;  // tap of lane half 0 / 1
      const int kr = h ? (k1 < 49 ? k1 / 7 : 0) : (k0 < 49 ? k0 / 7 : 0);
      const int kc = h ? (k1 < 49 ? k1 % 7 : 0) : (k0 < 49 ? k0 % 7 : 0);
      acc = mfma32(pp[kr * PW + kc], wr[q], acc);
    }
    // the band's output pixels are contiguous in NHWC: the store address is linear in pi (no per-element divide)
    float* yb = y + (((int64_t)img * OH + r0) * OW) * C1_CO + j;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int pi = t0 + (r & 3) + 8 * (r >> 2) + 4 * h;
      if (pi < npix) {
        const float v = acc[r] + bj;
        yb[(int64_t)pi * C1_CO] = v;
        s1 += v;
        s2 = fmaf(v, v, s2);
      }
    }
  }
  s1 += __shfl_xor(s1, 32, 64);
  s2 += __shfl_xor(s2, 32, 64);
  __syncthreads();
  float* red = sm;  // [4 waves][2][32]
  if (lane < 32) {
    red[wave * 64 + lane] = s1;
    red[wave * 64 + 32 + lane] = s2;
  }
  __syncthreads();
  if (threadIdx.x < 64) {
    const int t = threadIdx.x;
    const float v = red[t] + red[64 + t] + red[128 + t] + red[192 + t];
    partials[(int64_t)blockIdx.x * 2 * C1_CO + t] = v;  // [P][2*C]: sums then sums of squares
  }
}

int conv1_num_parts(int NF, int OH) { return NF * (int)cdiv(OH, C1_RB); }

// =====================================================================================================
// Stem backward (only when backbone.conv1 / bn1 train: the module API without apply_memory_efficient_training,
// cad:115-116,145-147; train_model freezes them, cad:592-598)
// =====================================================================================================
// conv1 weight gradient: dW[c][tap] = sum over output pixels of dY[p][c] * xpad[patch_p + tap], as f32 MFMA with
// M = 32 channels, K = pixels (two per MFMA), N = taps (two tiles: 0..31, 32..48).  One block per (frame, band of
// C1_RB output rows), the zero-padded input band staged in LDS as in the forward; the 4 waves take interleaved
// pixel pairs and are combined in a fixed order; each block writes its [32][49] partial to slab[blockIdx.x].
__global__ __launch_bounds__(256) void conv1_wgrad_kernel(const float* __restrict__ x, int H, int W,
                                                          const float* __restrict__ dy, int OH, int OW, int bands,
                                                          float* __restrict__ slab) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int img = blockIdx.x / bands, band = blockIdx.x % bands;
  const int r0 = band * C1_RB;
  const int PW = 2 * OW + 6, PH = 2 * C1_RB + 5;
  float* patch = sm;
  float* red = sm + ((PH * PW + 3) & ~3);  // [4 waves][2 tiles][16][64]
  const float* xi = x + (int64_t)img * H * W;
  for (int i = threadIdx.x; i < PH * PW; i += 256) {
    const int pr = i / PW, pc = i - pr * PW;
    const int ih = 2 * r0 - 3 + pr, iw = pc - 3;
    patch[i] = (ih >= 0 && ih < H && iw >= 0 && iw < W) ? xi[(int64_t)ih * W + iw] : 0.f;
  }
  __syncthreads();
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int j = lane & 31, h = lane >> 5;
  const int rows = min(C1_RB, OH - r0), npix = rows * OW;
  const float* dyb = dy + (((int64_t)img * OH + r0) * OW) * C1_CO;
  const int t1 = 32 + j;
  const int off0 = (j / 7) * PW + j % 7;
  const int off1 = t1 < 49 ? (t1 / 7) * PW + t1 % 7 : 0;
  f32x16 acc0, acc1;
#pragma unroll
  for (int r = 0; r < 16; ++r) acc0[r] = acc1[r] = 0.f;
  for (int p0 = wave * 2; p0 < npix; p0 += 8) {
    const int p = p0 + h;
    const bool ok = p < npix;
    const int pc = ok ? p : npix - 1;
    const float a = ok ? dyb[(int64_t)pc * C1_CO + j] : 0.f;  // A[c = j][k = h]
    const int oy = pc / OW, ox = pc - oy * OW;
    const float* pp = patch + (2 * oy) * PW + 2 * ox;
    acc0 = mfma32(a, pp[off0], acc0);
    acc1 = mfma32(a, t1 < 49 ? pp[off1] : 0.f, acc1);
  }
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    red[((wave * 2 + 0) * 16 + r) * 64 + lane] = acc0[r];
    red[((wave * 2 + 1) * 16 + r) * 64 + lane] = acc1[r];
  }
  __syncthreads();
  for (int e = threadIdx.x; e < 2 * 16 * 64; e += 256) {
    const int tile = e / 1024, r = (e / 64) % 16, l = e % 64;
    const float v = (red[((0 * 2 + tile) * 16 + r) * 64 + l] + red[((1 * 2 + tile) * 16 + r) * 64 + l]) +
                    (red[((2 * 2 + tile) * 16 + r) * 64 + l] + red[((3 * 2 + tile) * 16 + r) * 64 + l]);
    const int c = (r & 3) + 8 * (r >> 2) + 4 * (l >> 5), tap = tile * 32 + (l & 31);
    if (tap < 49) slab[(int64_t)blockIdx.x * 32 * 49 + c * 49 + tap] = v;
  }
}

// dW (torch [32][1][7][7]) = sum of the blocks' partials, fixed order: 64 elements x 4 slab lanes per block
__global__ __launch_bounds__(256) void conv1_wgrad_reduce_kernel(const float* __restrict__ slab, int S,
                                                                 float* __restrict__ dw) {
  __shared__ float red[4][64];
  const int e = blockIdx.x * 64 + (threadIdx.x & 63), g = threadIdx.x >> 6;
  float s0 = 0.f, s1 = 0.f;
  if (e < 32 * 49) {
    int s = g;
    for (; s + 4 < S; s += 8) {
      s0 += slab[(int64_t)s * 32 * 49 + e];
      s1 += slab[(int64_t)(s + 4) * 32 * 49 + e];
    }
    for (; s < S; s += 4) s0 += slab[(int64_t)s * 32 * 49 + e];
  }
  red[g][threadIdx.x & 63] = s0 + s1;
  __syncthreads();
  if (threadIdx.x < 64 && e < 32 * 49)
    dw[e] = (red[0][threadIdx.x] + red[1][threadIdx.x]) + (red[2][threadIdx.x] + red[3][threadIdx.x]);
}

int conv1_wgrad(const float* x, int NF, int H, int W, const float* dy, int OH, int OW, float* slab,
                int64_t slab_cap, float* dw, hipStream_t st) {
  const int bands = (int)cdiv(OH, C1_RB);
  const int S = NF * bands;
  VAD_CHECK((int64_t)S * 32 * 49 <= slab_cap, "conv1_wgrad: slab buffer too small");
  const size_t patch = ((size_t)(2 * C1_RB + 5) * (2 * OW + 6) + 3) & ~(size_t)3;
  const size_t lds = (patch + 4 * 2 * 16 * 64) * sizeof(float);
  VAD_CHECK(lds <= 160 * 1024, "conv1_wgrad: frame too wide for the LDS band");
  hipLaunchKernelGGL(conv1_wgrad_kernel, dim3(S), dim3(256), lds, st, x, H, W, dy, OH, OW, bands, slab);
  VAD_LAUNCH_CHECK();
  hipLaunchKernelGGL(conv1_wgrad_reduce_kernel, dim3((unsigned)cdiv(32 * 49, 64)), dim3(256), 0, st, slab, S, dw);
  VAD_LAUNCH_CHECK();
  return 0;
}

// MaxPool2d(3, 2, 1) backward over relu(bn1(y)): dA[p] = sum of dpool over the (1, 2 or 4) windows whose first
// maximum in scan order (torch CPU max_pool2d's index rule) is p; recomputed from y instead of stored indices.
__global__ __launch_bounds__(256) void maxpool_bwd_kernel(const float* __restrict__ y, const float* __restrict__ stats,
                                                          const float* __restrict__ dpool, int NF, int H, int W,
                                                          int C, int OH, int OW, float* __restrict__ dA) {
  const int nq = C / 4;
  const int64_t total = (int64_t)NF * H * W * nq;
  for (int64_t i = blockIdx.x * 256ll + threadIdx.x; i < total; i += (int64_t)gridDim.x * 256) {
    const int q = (int)(i % nq);
    int64_t p = i / nq;
    const int ix = (int)(p % W);
    p /= W;
    const int iy = (int)(p % H);
    const int img = (int)(p / H);
    const int c = q * 4;
    const f32x4 sc = *reinterpret_cast<const f32x4*>(stats + 2 * C + c);
    const f32x4 sh = *reinterpret_cast<const f32x4*>(stats + 3 * C + c);
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    const int oy0 = max(0, iy / 2), oy1 = min(OH - 1, (iy + 1) / 2);
    const int ox0 = max(0, ix / 2), ox1 = min(OW - 1, (ix + 1) / 2);
    for (int oy = oy0; oy <= oy1; ++oy)
      for (int ox = ox0; ox <= ox1; ++ox) {
        f32x4 best = {-INFINITY, -INFINITY, -INFINITY, -INFINITY};
        int first[4] = {-1, -1, -1, -1};
        for (int dyy = -1; dyy <= 1; ++dyy) {
          const int yy = 2 * oy + dyy;
          if (yy < 0 || yy >= H) continue;
          for (int dxx = -1; dxx <= 1; ++dxx) {
            const int xx = 2 * ox + dxx;
            if (xx < 0 || xx >= W) continue;
            const f32x4 v = *reinterpret_cast<const f32x4*>(y + (((int64_t)img * H + yy) * W + xx) * C + c);
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              const float z = fmaxf(fmaf(v[e], sc[e], sh[e]), 0.f);
              if (z > best[e]) {
                best[e] = z;
                first[e] = yy * W + xx;
              }
            }
          }
        }
        const f32x4 g = *reinterpret_cast<const f32x4*>(dpool + (((int64_t)img * OH + oy) * OW + ox) * C + c);
#pragma unroll
        for (int e = 0; e < 4; ++e)
          if (first[e] == iy * W + ix) acc[e] += g[e];
      }
    *reinterpret_cast<f32x4*>(dA + (((int64_t)img * H + iy) * W + ix) * C + c) = acc;
  }
}

int maxpool3s2_bwd(const float* y, const float* stats, const float* dpool, int NF, int H, int W, int C, int OH,
                   int OW, float* dA, hipStream_t st) {
  VAD_CHECK(!g_act_bf16, "stem: the unfused stem keeps fp32 activations");
  VAD_CHECK(OH == (H - 1) / 2 + 1 && OW == (W - 1) / 2 + 1 && C % 4 == 0, "maxpool_bwd: bad dims");
  const int64_t total = (int64_t)NF * H * W * (C / 4);
  const int grid = (int)std::min<int64_t>(cdiv(total, 256), 16384);
  hipLaunchKernelGGL(maxpool_bwd_kernel, dim3(grid), dim3(256), 0, st, y, stats, dpool, NF, H, W, C, OH, OW, dA);
  VAD_LAUNCH_CHECK();
  return 0;
}

int conv1_fwd(const float* x, int NF, int H, int W, const float* w, const float* b, float* y, int OH, int OW,
              float* partials, int* nparts, hipStream_t st) {
  VAD_CHECK(!g_act_bf16, "stem: the unfused stem keeps fp32 activations");
  VAD_CHECK(OH == (H - 1) / 2 + 1 && OW == (W - 1) / 2 + 1, "conv1: bad output dims");
  const int bands = (int)cdiv(OH, C1_RB);
  const size_t lds = (size_t)(2 * C1_RB + 5) * (2 * OW + 6) * sizeof(float);
  VAD_CHECK(lds <= 160 * 1024, "conv1: frame too wide for the LDS band");
  VAD_KLAUNCH(conv1_kernel, dim3(NF * bands), dim3(256), lds, st, x, H, W, w, b, y, OH, OW, bands, partials);
  VAD_LAUNCH_CHECK();
  *nparts = NF * bands;
  return 0;
}

// =====================================================================================================
// BatchNorm finalize: combine partial sums in double; batch stats, affine folding, running-stat update
// (momentum 0.1, unbiased variance for running_var; nn.BatchNorm2d train semantics).
// =====================================================================================================
template <typename PT>
__global__ __launch_bounds__(256) void bn_finalize_kernel(const PT* __restrict__ partials, int P, int C,
                                                          double count, const float* __restrict__ gamma,
                                                          const float* __restrict__ beta, float* running_mean,
                                                          float* running_var, float momentum, float eps,
                                                          int training, float* __restrict__ stats, int cm) {
  const int c = blockIdx.x;
  double a = 0.0, b = 0.0;
  // partials row-major [P][2C], or column-major [2C][P] (cm: the fused stem's layout, coalesced here)
  const int64_t rs = cm ? 1 : 2 * C, ia = cm ? (int64_t)c * P : c, ib = cm ? (int64_t)(C + c) * P : C + c;
  if (training) {
#pragma unroll 4
    for (int p = threadIdx.x; p < P; p += 256) {
      a += (double)partials[p * rs + ia];
      b += (double)partials[p * rs + ib];
    }
  }
  block_sum2_256(a, b);
  if (threadIdx.x == 0) {
    double mean, var;
    if (training) {
      mean = a / count;
      var = b / count - mean * mean;
      if (var < 0) var = 0;
      running_mean[c] = (float)((1.0 - momentum) * running_mean[c] + momentum * mean);
      running_var[c] = (float)((1.0 - momentum) * running_var[c] + momentum * var * count / (count - 1.0));
    } else {
      mean = running_mean[c];
      var = running_var[c];
    }
    const double invstd = 1.0 / sqrt(var + (double)eps);
    const double scale = (double)gamma[c] * invstd;
    stats[c] = (float)mean;
    stats[C + c] = (float)invstd;
    stats[2 * C + c] = (float)scale;
    stats[3 * C + c] = (float)((double)beta[c] - mean * scale);
  }
}

int bn_finalize(const float* partials, int P, int C, double count, const float* gamma, const float* beta,
                float* running_mean, float* running_var, float momentum, float eps, int training, float* stats,
                hipStream_t st, int cm) {
  hipLaunchKernelGGL(bn_finalize_kernel<float>, dim3(C), dim3(256), 0, st, partials, P, C, count, gamma, beta,
                     running_mean, running_var, momentum, eps, training, stats, cm);
  VAD_LAUNCH_CHECK();
  return 0;
}

int bn_finalize_sums(const double* sums, int C, double count, const float* gamma, const float* beta,
                     float* running_mean, float* running_var, float momentum, float eps, float* stats,
                     hipStream_t st) {
  hipLaunchKernelGGL(bn_finalize_kernel<double>, dim3(C), dim3(256), 0, st, sums, 1, C, count, gamma, beta,
                     running_mean, running_var, momentum, eps, 1, stats, 0);
  VAD_LAUNCH_CHECK();
  return 0;
}

// SyncBatchNorm support: fold a layer's [P][2C] float partials into [2C] double sums (the buffer the caller
// all-reduces across ranks); optionally also writes them as float to a_out / b_out (the local dbeta / dgamma)
__global__ __launch_bounds__(256) void bn_sum_partials_kernel(const float* __restrict__ partials, int P, int C,
                                                              double* __restrict__ sums, float* a_out,
                                                              float* b_out, int cm) {
  const int c = blockIdx.x;
  double a = 0.0, b = 0.0;
  const int64_t rs = cm ? 1 : 2 * C, ia = cm ? (int64_t)c * P : c, ib = cm ? (int64_t)(C + c) * P : C + c;
#pragma unroll 4
  for (int p = threadIdx.x; p < P; p += 256) {
    a += (double)partials[p * rs + ia];
    b += (double)partials[p * rs + ib];
  }
  block_sum2_256(a, b);
  if (threadIdx.x == 0) {
    sums[c] = a;
    sums[C + c] = b;
    if (a_out) a_out[c] = (float)a;
    if (b_out) b_out[c] = (float)b;
  }
}

int bn_sum_partials(const float* partials, int P, int C, double* sums, float* a_out, float* b_out, hipStream_t st,
                    int cm) {
  hipLaunchKernelGGL(bn_sum_partials_kernel, dim3(C), dim3(256), 0, st, partials, P, C, sums, a_out, b_out, cm);
  VAD_LAUNCH_CHECK();
  return 0;
}

// =====================================================================================================
// BatchNorm backward (through the ReLU that follows it):  dZ = dA * [scale*y+shift > 0]
//   reduce: per-channel sum(dZ), sum(dZ*xhat)          -> partials
//   finalize: dgamma = sum(dZ*xhat), dbeta = sum(dZ), k = gamma*invstd, means
//   apply: dY = k * (dZ - mean(dZ) - xhat*mean(dZ*xhat)), plus per-block sum(dY) for the conv bias grad
// Thread layout over [M][C] rows: thread -> (row offset, channel quad); 1024 rows per block.
// =====================================================================================================
// rows per block: 1024, lowered (down to 64) until the grid has >= 1024 blocks.  Callers size partial buffers for
// the worst case ceil(M/64) blocks (CadPlanImpl::carve).
static int bn_rows(int M) {
  int r = 1024;
  while (r > 64 && cdiv(M, r) < 1024) r >>= 1;
  return r;
}

int bn_rows_parts(int M, int C) {
  (void)C;
  return (int)cdiv(M, bn_rows(M));
}

// out: this block's [2C] row (row-major partials), or with cs > 0 element j at out[j * cs] (column-major [2C][P])
__device__ inline void bn_block_reduce_store(float (&v)[2][4], int C, float* out, int64_t cs = 0) {
  // threads sharing a channel quad: tid % (C/4) equal.  Reduce through LDS.
  __shared__ float red[256 * 8];
  const int t = threadIdx.x;
#pragma unroll
  for (int s = 0; s < 2; ++s)
#pragma unroll
    for (int e = 0; e < 4; ++e) red[(s * 4 + e) * 256 + t] = v[s][e];
  __syncthreads();
  const int nq = C / 4, groups = 256 / nq;
  for (int idx = t; idx < 2 * C; idx += 256) {
    const int s = idx / C, c = idx % C, q = c / 4, e = c % 4;
    float acc = 0.f;
    for (int g = 0; g < groups; ++g) acc += red[(s * 4 + e) * 256 + g * nq + q];
    out[cs ? (int64_t)(s * C + c) * cs : s * C + c] = acc;
  }
}

template <bool AB>
__global__ __launch_bounds__(256) void bn_bwd_reduce_kernel(const act_t<AB>* __restrict__ dA,
                                                            const act_t<AB>* __restrict__ y,
                                                            const float* __restrict__ stats, int M, int C,
                                                            float* __restrict__ partials, int BN_ROWS, int cm) {
  const int nq = C / 4, groups = 256 / nq;
  const int q = threadIdx.x % nq, g = threadIdx.x / nq;
  const int c = q * 4;
  const f32x4 mean = *reinterpret_cast<const f32x4*>(stats + c);
  const f32x4 inv = *reinterpret_cast<const f32x4*>(stats + C + c);
  const f32x4 sc = *reinterpret_cast<const f32x4*>(stats + 2 * C + c);
  const f32x4 sh = *reinterpret_cast<const f32x4*>(stats + 3 * C + c);
  float v[2][4] = {{0, 0, 0, 0}, {0, 0, 0, 0}};
  const int r0 = blockIdx.x * BN_ROWS;
  const int r1 = min(M, r0 + BN_ROWS);
  for (int r = r0 + g; r < r1; r += groups) {
    const f32x4 a = act_f4(act_ld4(dA + (int64_t)r * C + c));
    const f32x4 yy = act_f4(act_ld4(y + (int64_t)r * C + c));
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float z = fmaf(yy[e], sc[e], sh[e]);
      const float dz = z > 0.f ? a[e] : 0.f;
      v[0][e] += dz;
      v[1][e] = fmaf(dz, (yy[e] - mean[e]) * inv[e], v[1][e]);
    }
  }
  if (cm) bn_block_reduce_store(v, C, partials + blockIdx.x, gridDim.x);
  else bn_block_reduce_store(v, C, partials + (int64_t)blockIdx.x * 2 * C);
}

int bn_bwd_reduce(const float* dA, const float* y, const float* stats, int M, int C, float* partials, int* nparts,
                  hipStream_t st, int cm) {
  VAD_CHECK(C % 4 == 0 && C <= 1024 && 256 % (C / 4) == 0, "bn_bwd_reduce: unsupported C");
  const int P = bn_rows_parts(M, C);
  if (g_act_bf16)
    hipLaunchKernelGGL(bn_bwd_reduce_kernel<true>, dim3(P), dim3(256), 0, st, reinterpret_cast<const __bf16*>(dA),
                       reinterpret_cast<const __bf16*>(y), stats, M, C, partials, bn_rows(M), cm);
  else
    hipLaunchKernelGGL(bn_bwd_reduce_kernel<false>, dim3(P), dim3(256), 0, st, dA, y, stats, M, C, partials,
                       bn_rows(M), cm);
  VAD_LAUNCH_CHECK();
  *nparts = P;
  return 0;
}

template <typename PT>
__global__ __launch_bounds__(256) void bn_bwd_finalize_kernel(const PT* __restrict__ partials, int P, int C,
                                                              double count, const float* __restrict__ gamma,
                                                              float* __restrict__ stats, float* dgamma,
                                                              float* dbeta, int training, float* dbias, int cm) {
  const int c = blockIdx.x;
  double a = 0.0, b = 0.0;
  // partials row-major [P][2C] or column-major [2C][P] (cm)
  const int64_t rs = cm ? 1 : 2 * C, ia = cm ? (int64_t)c * P : c, ib = cm ? (int64_t)(C + c) * P : C + c;
#pragma unroll 4
  for (int p = threadIdx.x; p < P; p += 256) {
    a += (double)partials[p * rs + ia];
    b += (double)partials[p * rs + ib];
  }
  block_sum2_256(a, b);
  if (threadIdx.x == 0) {
    const double sdz = a, sdzx = b;
    if (dgamma) dgamma[c] = (float)sdzx;
    if (dbeta) dbeta[c] = (float)sdz;
    const double inv = stats[C + c];
    const double k = (double)gamma[c] * inv;
    stats[4 * C + c] = gamma[c] * stats[C + c];
    // eval mode: BN is the affine map of the running stats, no batch-mean terms in its backward
    const double mdz = training ? sdz / count : 0.0, mdzx = training ? sdzx / count : 0.0;
    stats[5 * C + c] = (float)mdz;
    stats[6 * C + c] = (float)mdzx;
    // conv bias grad = sum of dY = k (sum dZ - count mean(dZ)) - k invstd mean(dZ xhat) sum(y - mean); the last
    // sum is zero by the definition of the mean, the first vanishes in training mode up to rounding
    if (dbias) dbias[c] = (float)(k * (sdz - count * mdz));
  }
}

int bn_bwd_finalize(const float* partials, int P, int C, double count, const float* gamma, float* stats,
                    float* dgamma, float* dbeta, int training, hipStream_t st, float* dbias, int cm) {
  hipLaunchKernelGGL(bn_bwd_finalize_kernel<float>, dim3(C), dim3(256), 0, st, partials, P, C, count, gamma, stats,
                     dgamma, dbeta, training, dbias, cm);
  VAD_LAUNCH_CHECK();
  return 0;
}

int bn_bwd_finalize_sums(const double* sums, int C, double count, const float* gamma, float* stats, hipStream_t st,
                         float* dbias) {
  hipLaunchKernelGGL(bn_bwd_finalize_kernel<double>, dim3(C), dim3(256), 0, st, sums, 1, C, count, gamma, stats,
                     nullptr, nullptr, 1, dbias, 0);
  VAD_LAUNCH_CHECK();
  return 0;
}

// dY = k (dZ - mean(dZ) - xhat mean(dZ xhat)), dZ = dA where relu(fma(y, scale, shift)) > 0.  The body takes plain
// pointers: bn_bwd_apply_kernel adds __restrict__ (distinct buffers), bn_bwd_apply_inplace_kernel does not (the
// training stem's backward applies it in place, dY == dA: every thread reads an element before it writes it)
template <bool AB>
__device__ __forceinline__ void bn_bwd_apply_body(const act_t<AB>* dA, const act_t<AB>* y, const float* stats, int M,
                                                  int C, act_t<AB>* dY, float* bparts, int BN_ROWS) {
  const int nq = C / 4, groups = 256 / nq;
  const int q = threadIdx.x % nq, g = threadIdx.x / nq;
  const int c = q * 4;
  const f32x4 mean = *reinterpret_cast<const f32x4*>(stats + c);
  const f32x4 inv = *reinterpret_cast<const f32x4*>(stats + C + c);
  const f32x4 sc = *reinterpret_cast<const f32x4*>(stats + 2 * C + c);
  const f32x4 sh = *reinterpret_cast<const f32x4*>(stats + 3 * C + c);
  const f32x4 k = *reinterpret_cast<const f32x4*>(stats + 4 * C + c);
  const f32x4 mdz = *reinterpret_cast<const f32x4*>(stats + 5 * C + c);
  const f32x4 mdzx = *reinterpret_cast<const f32x4*>(stats + 6 * C + c);
  float v[2][4] = {{0, 0, 0, 0}, {0, 0, 0, 0}};
  const int r0 = blockIdx.x * BN_ROWS;
  const int r1 = min(M, r0 + BN_ROWS);
  for (int r = r0 + g; r < r1; r += groups) {
    const f32x4 a = act_f4(act_ld4(dA + (int64_t)r * C + c));
    const f32x4 yy = act_f4(act_ld4(y + (int64_t)r * C + c));
    f32x4 o;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float z = fmaf(yy[e], sc[e], sh[e]);
      const float dz = z > 0.f ? a[e] : 0.f;
      const float xh = (yy[e] - mean[e]) * inv[e];
      o[e] = k[e] * (dz - mdz[e] - xh * mdzx[e]);
      v[0][e] += o[e];
    }
    act_st4(dY + (int64_t)r * C + c, o);
  }
  if (bparts) bn_block_reduce_store(v, C, bparts + (int64_t)blockIdx.x * 2 * C);
}

template <bool AB>
__global__ __launch_bounds__(256) void bn_bwd_apply_kernel(const act_t<AB>* __restrict__ dA,
                                                           const act_t<AB>* __restrict__ y,
                                                           const float* __restrict__ stats, int M, int C,
                                                           act_t<AB>* __restrict__ dY, float* __restrict__ bparts,
                                                           int BN_ROWS) {
  bn_bwd_apply_body<AB>(dA, y, stats, M, C, dY, bparts, BN_ROWS);
}

__global__ __launch_bounds__(256) void bn_bwd_apply_inplace_kernel(float* dAY, const float* __restrict__ y,
                                                                   const float* __restrict__ stats, int M, int C,
                                                                   int BN_ROWS) {
  bn_bwd_apply_body<false>(dAY, y, stats, M, C, dAY, nullptr, BN_ROWS);
}

typedef unsigned u32x4v __attribute__((ext_vector_type(4)));
struct f32x8v {
  f32x4 lo, hi;
};
__device__ inline void vload8(u32x4v r, float (&v)[8]) {
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    v[2 * e] = __uint_as_float(r[e] << 16);
    v[2 * e + 1] = __uint_as_float(r[e] & 0xffff0000u);
  }
}
__device__ inline void vload8(const f32x8v& r, float (&v)[8]) {
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    v[e] = r.lo[e];
    v[4 + e] = r.hi[e];
  }
}
template <typename V>
__device__ inline V vstore8(const float (&v)[8]);
template <>
__device__ inline u32x4v vstore8<u32x4v>(const float (&v)[8]) {
  typedef __bf16 b8 __attribute__((ext_vector_type(8)));
  b8 b;
#pragma unroll
  for (int e = 0; e < 8; ++e) b[e] = (__bf16)v[e];
  return __builtin_bit_cast(u32x4v, b);
}
template <>
__device__ inline f32x8v vstore8<f32x8v>(const float (&v)[8]) {
  f32x8v o;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    o.lo[e] = v[e];
    o.hi[e] = v[4 + e];
  }
  return o;
}

int bn_bwd_apply_inplace(float* dAY, const float* y, const float* stats, int M, int C, hipStream_t st) {
  VAD_CHECK(!g_act_bf16, "bn_bwd_apply_inplace: fp32 activations only");
  hipLaunchKernelGGL(bn_bwd_apply_inplace_kernel, dim3(bn_rows_parts(M, C)), dim3(256), 0, st, dAY, y, stats, M, C,
                     bn_rows(M));
  VAD_LAUNCH_CHECK();
  return 0;
}

// Streaming form (no conv-bias partial sums): thread = 8 consecutive channels of a row (16 B per operand in bf16, 32 B in
// fp32), U rows per iteration with every load issued before the arithmetic (the 4-channel row loop above keeps one 8-B
// load per operand in flight per thread and reaches ~3.5 TB/s), grid-stride over the row groups.
template <bool AB, int U>
__global__ __launch_bounds__(256) void bn_bwd_apply_v_kernel(const act_t<AB>* __restrict__ dA,
                                                           const act_t<AB>* __restrict__ y,
                                                           const float* __restrict__ stats, int M, int C,
                                                           act_t<AB>* __restrict__ dY) {
  using V = typename std::conditional<AB, u32x4v, f32x8v>::type;  // 8 channels
  const int tpr = C / 8, rpp = 256 / tpr;                         // threads per row, rows per pass
  const int q = threadIdx.x % tpr, c = q * 8;
  float mean[8], inv[8], sc[8], sh[8], k[8], mdz[8], mdzx[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    mean[e] = stats[c + e];
    inv[e] = stats[C + c + e];
    sc[e] = stats[2 * C + c + e];
    sh[e] = stats[3 * C + c + e];
    k[e] = stats[4 * C + c + e];
    mdz[e] = stats[5 * C + c + e];
    mdzx[e] = stats[6 * C + c + e];
  }
  const int64_t step = (int64_t)gridDim.x * rpp * U;
  for (int64_t r0 = ((int64_t)blockIdx.x * U) * rpp + threadIdx.x / tpr; r0 < M; r0 += step) {
    V a[U], yy[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t r = min(r0 + (int64_t)u * rpp, (int64_t)M - 1);
      a[u] = *reinterpret_cast<const V*>(dA + r * C + c);
      yy[u] = *reinterpret_cast<const V*>(y + r * C + c);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t r = r0 + (int64_t)u * rpp;
      if (r >= M) break;
      float af[8], yf[8], o[8];
      vload8(a[u], af);
      vload8(yy[u], yf);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float dz = fmaf(yf[e], sc[e], sh[e]) > 0.f ? af[e] : 0.f;
        const float xh = (yf[e] - mean[e]) * inv[e];
        o[e] = k[e] * (dz - mdz[e] - xh * mdzx[e]);
      }
      *reinterpret_cast<V*>(dY + r * C + c) = vstore8<V>(o);
    }
  }
}

int g_bn_apply_v = 1;  // knob "bn_apply_v": the streaming apply kernel (0: the 4-channel row loop)
int g_bn_apply_u = 4;          // knob "bn_apply_u": rows in flight per thread (2, 4, 8)
int g_bn_apply_blocks = 2048;  // knob "bn_apply_blocks": grid cap (grid-stride beyond it)

int bn_bwd_apply(const float* dA, const float* y, const float* stats, int M, int C, float* dY, float* bias_partials,
                 int* nparts, hipStream_t st) {
  const int P = bn_rows_parts(M, C);
  if (g_bn_apply_v && !bias_partials && C % 8 == 0 && C >= 8 && C <= 2048 && 256 % (C / 8) == 0) {
    const int U = g_bn_apply_u == 8 ? 8 : (g_bn_apply_u == 2 ? 2 : 4);
    const int rpp = 256 / (C / 8);
    const int blocks = (int)std::max<int64_t>(1, std::min<int64_t>(cdiv(M, (int64_t)rpp * U), g_bn_apply_blocks));
#define VAD_BNA(AB, UU, T)                                                                                            \
  hipLaunchKernelGGL((bn_bwd_apply_v_kernel<AB, UU>), dim3(blocks), dim3(256), 0, st, reinterpret_cast<const T*>(dA), \
                     reinterpret_cast<const T*>(y), stats, M, C, reinterpret_cast<T*>(dY))
    if (g_act_bf16) {
      if (U == 8) VAD_BNA(true, 8, __bf16);
      else if (U == 2) VAD_BNA(true, 2, __bf16);
      else VAD_BNA(true, 4, __bf16);
    } else {
      if (U == 8) VAD_BNA(false, 8, float);
      else if (U == 2) VAD_BNA(false, 2, float);
      else VAD_BNA(false, 4, float);
    }
#undef VAD_BNA
    VAD_LAUNCH_CHECK();
    *nparts = 0;
    return 0;
  }
  if (g_act_bf16)
    hipLaunchKernelGGL(bn_bwd_apply_kernel<true>, dim3(P), dim3(256), 0, st, reinterpret_cast<const __bf16*>(dA),
                       reinterpret_cast<const __bf16*>(y), stats, M, C, reinterpret_cast<__bf16*>(dY), bias_partials,
                       bn_rows(M));
  else
    hipLaunchKernelGGL(bn_bwd_apply_kernel<false>, dim3(P), dim3(256), 0, st, dA, y, stats, M, C, dY, bias_partials,
                       bn_rows(M));
  VAD_LAUNCH_CHECK();
  *nparts = P;
  return 0;
}

// =====================================================================================================
// MaxPool 3x3 s2 p1 over relu(bn1(y)) (the frozen stem: forward only).
// =====================================================================================================
__global__ __launch_bounds__(256) void maxpool_kernel(const float* __restrict__ y, const float* __restrict__ stats,
                                                      int NF, int H, int W, int C, float* __restrict__ out, int OH,
                                                      int OW) {
  const int nq = C / 4;
  const int64_t total = (int64_t)NF * OH * OW * nq;
  for (int64_t i = blockIdx.x * 256ll + threadIdx.x; i < total; i += (int64_t)gridDim.x * 256) {
    const int q = (int)(i % nq);
    int64_t p = i / nq;
    const int ox = (int)(p % OW);
    p /= OW;
    const int oy = (int)(p % OH);
    const int img = (int)(p / OH);
    const int c = q * 4;
    const f32x4 sc = *reinterpret_cast<const f32x4*>(stats + 2 * C + c);
    const f32x4 sh = *reinterpret_cast<const f32x4*>(stats + 3 * C + c);
    f32x4 m = {-INFINITY, -INFINITY, -INFINITY, -INFINITY};
    for (int dy = -1; dy <= 1; ++dy) {
      const int iy = 2 * oy + dy;
      if (iy < 0 || iy >= H) continue;
      for (int dx = -1; dx <= 1; ++dx) {
        const int ix = 2 * ox + dx;
        if (ix < 0 || ix >= W) continue;
        const f32x4 v = *reinterpret_cast<const f32x4*>(y + (((int64_t)img * H + iy) * W + ix) * C + c);
#pragma unroll
        for (int e = 0; e < 4; ++e) m[e] = fmaxf(m[e], fmaxf(fmaf(v[e], sc[e], sh[e]), 0.f));
      }
    }
    *reinterpret_cast<f32x4*>(out + (((int64_t)img * OH + oy) * OW + ox) * C + c) = m;
  }
}

int maxpool3s2_bnrelu(const float* y, const float* stats, int NF, int H, int W, int C, float* out, int OH, int OW,
                      hipStream_t st) {
  VAD_CHECK(!g_act_bf16, "stem: the unfused stem keeps fp32 activations");
  VAD_CHECK(OH == (H - 1) / 2 + 1 && OW == (W - 1) / 2 + 1 && C % 4 == 0, "maxpool: bad dims");
  const int64_t total = (int64_t)NF * OH * OW * (C / 4);
  const int grid = (int)std::min<int64_t>(cdiv(total, 256), 8192);
  hipLaunchKernelGGL(maxpool_kernel, dim3(grid), dim3(256), 0, st, y, stats, NF, H, W, C, out, OH, OW);
  VAD_LAUNCH_CHECK();
  return 0;
}

// =====================================================================================================
// AdaptiveAvgPool2d((4,6)) on relu(bn(y)) + flatten (c*24 + i*6 + j) + mean over T, and its backward.
// torch bins: start = floor(i*In/Out), end = ceil((i+1)*In/Out).
// =====================================================================================================
__device__ inline int ap_start(int i, int in, int out) { return (i * in) / out; }
__device__ inline int ap_end(int i, int in, int out) { return ((i + 1) * in + out - 1) / out; }

// AdaptiveAvgPool2d((4, 6)) of relu(bn(y)) and its mean over the clip (cad:560-568) in one pass: thread (clip b, bin
// (i, j), channel c) walks the bin's pixels of the T images in (t, row, column) order -- loads in chunks of 16 from
// clamped addresses, so a chunk costs one memory round trip -- and writes each image's bin mean and the clip mean
// (same summation order as a per-image pass followed by a mean over T)
template <bool AB>
__global__ __launch_bounds__(256) void avgpool_fwd_kernel(const act_t<AB>* __restrict__ y,
                                                          const float* __restrict__ stats, int T, int H, int W, int C,
                                                          float* __restrict__ feats, float* __restrict__ pooled) {
  const int b = blockIdx.y, i = blockIdx.z / 6, j = blockIdx.z % 6;
  const int c = blockIdx.x * 256 + threadIdx.x;
  if (c >= C) return;
  const float sc = stats[2 * C + c], sh = stats[3 * C + c];
  const int h0 = ap_start(i, H, 4), h1 = ap_end(i, H, 4), w0 = ap_start(j, W, 6), w1 = ap_end(j, W, 6);
  const int wn = w1 - w0, n = (h1 - h0) * wn, total = T * n;
  const float fn = (float)n;
  const act_t<AB>* yb = y + (int64_t)b * T * H * W * C + c;
  float cur = 0.f, pool = 0.f;
  int curt = 0;
  for (int base = 0; base < total; base += 16) {
    float v[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      const int q = min(base + k, total - 1), t = q / n, p = q - t * n;
      const int hh = h0 + p / wn, ww = w0 + p % wn;
      v[k] = act_ld(yb + (((int64_t)t * H + hh) * W + ww) * C);
    }
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      const int q = base + k;
      if (q < total) {
        const int t = q / n;
        if (t != curt) {
          const float f = cur / fn;
          feats[((int64_t)b * T + curt) * C * 24 + c * 24 + i * 6 + j] = f;
          pool += f;
          curt = t;
          cur = 0.f;
        }
        cur += fmaxf(fmaf(v[k], sc, sh), 0.f);
      }
    }
  }
  const float f = cur / fn;
  feats[((int64_t)b * T + curt) * C * 24 + c * 24 + i * 6 + j] = f;
  pool += f;
  pooled[(int64_t)b * C * 24 + c * 24 + i * 6 + j] = pool / (float)T;
}

int avgpool_fwd(const float* y, const float* stats, int B, int T, int H, int W, int C, float* feats, float* pooled,
                hipStream_t st) {
  const dim3 grid((unsigned)cdiv(C, 256), B, 24);
  if (g_act_bf16)
    VAD_KLAUNCH(avgpool_fwd_kernel<true>, grid, dim3(256), 0, st, reinterpret_cast<const __bf16*>(y), stats, T, H, W,
                C, feats, pooled);
  else
    VAD_KLAUNCH(avgpool_fwd_kernel<false>, grid, dim3(256), 0, st, y, stats, T, H, W, C, feats, pooled);
  VAD_LAUNCH_CHECK();
  return 0;
}

// one block per (image, output row hh): thread c spreads the bins covering row hh over the W pixels of the row
// (1024 blocks at config 2 instead of one 64-pixel loop per channel over 128 blocks).  coef != null: the clip-mean
// gradient is dpooled[b] + coef[b] dpooled_c[b] (the direct classifier's affine backward, mlp.h DirMidArgs)
template <bool AB>
__global__ __launch_bounds__(256) void avgpool_bwd_kernel(const float* __restrict__ dfeat,
                                                          const float* __restrict__ dpooled,
                                                          const float* __restrict__ dpooled_c,
                                                          const float* __restrict__ coef, int B, int T, int H,
                                                          int W, int C, act_t<AB>* __restrict__ dA) {
  const int img = blockIdx.x, hh = blockIdx.y;
  const int b = img / T;
  const float invT = 1.f / (float)T;
  const float cb = coef ? coef[b] : 0.f;
  for (int c = threadIdx.x; c < C; c += 256) {
    float g[4][6];  // (up to 4 row bins cover hh when H < 4)
    int ni = 0, iv[4] = {0, 0, 0, 0};
#pragma unroll
    for (int i = 0; i < 4; ++i)
      if (hh >= ap_start(i, H, 4) && hh < ap_end(i, H, 4)) iv[ni++] = i;
    for (int q = 0; q < ni; ++q) {
      const int i = iv[q];
      const float hn = (float)(ap_end(i, H, 4) - ap_start(i, H, 4));
#pragma unroll
      for (int j = 0; j < 6; ++j) {
        float v = dfeat ? dfeat[(int64_t)img * C * 24 + c * 24 + i * 6 + j] : 0.f;
        if (dpooled) {
          const int64_t o = (int64_t)b * C * 24 + c * 24 + i * 6 + j;
          v += (coef ? fmaf(cb, dpooled_c[o], dpooled[o]) : dpooled[o]) * invT;
        }
        g[q][j] = v / (hn * (float)(ap_end(j, W, 6) - ap_start(j, W, 6)));
      }
    }
    for (int ww = 0; ww < W; ++ww) {
      float s = 0.f;
      for (int q = 0; q < ni; ++q)
#pragma unroll
        for (int j = 0; j < 6; ++j)
          if (ww >= ap_start(j, W, 6) && ww < ap_end(j, W, 6)) s += g[q][j];
      act_st(dA + (((int64_t)img * H + hh) * W + ww) * C + c, s);
    }
  }
}

int avgpool_bwd(const float* dfeat, const float* dpooled, int B, int T, int H, int W, int C, float* dA,
                hipStream_t st, const float* dpooled_c, const float* coef) {
  VAD_CHECK(!coef || (dpooled && dpooled_c), "avgpool_bwd: the affine form needs both parts");
  const dim3 grid((unsigned)(B * T), (unsigned)H);
  if (g_act_bf16)
    VAD_KLAUNCH(avgpool_bwd_kernel<true>, grid, dim3(256), 0, st, dfeat, dpooled, dpooled_c, coef, B, T, H, W, C,
                reinterpret_cast<__bf16*>(dA));
  else
    VAD_KLAUNCH(avgpool_bwd_kernel<false>, grid, dim3(256), 0, st, dfeat, dpooled, dpooled_c, coef, B, T, H, W, C, dA);
  VAD_LAUNCH_CHECK();
  return 0;
}

// =====================================================================================================
// GEMM epilogues
// =====================================================================================================
struct EpiConvFwd {  // y = acc + bias (NHWC rows), plus per-block BN partial sums
  static constexpr int SCRATCH = 2 * 4 * 256;
  struct Params { float* y; const float* bias; int C; float* partials; };
  template <class Cfg>
  static __device__ void apply(const Params& P, f32x16 (&acc)[Cfg::TM][Cfg::TN], int m0, int n0, int wm, int wn,
                               int lane, int M, int N, float* lds) {
    float s1[Cfg::TN], s2[Cfg::TN];
#pragma unroll
    for (int j = 0; j < Cfg::TN; ++j) {
      s1[j] = s2[j] = 0.f;
      const int col = n0 + acc_col<Cfg>(wn, j, lane);
      const float bj = col < N ? P.bias[col] : 0.f;
#pragma unroll
      for (int i = 0; i < Cfg::TM; ++i)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int row = m0 + acc_row<Cfg>(wm, i, r, lane);
          if (row < M && col < N) {
            const float v = acc[i][j][r] + bj;
            P.y[(int64_t)row * P.C + col] = v;
            s1[j] += v;
            s2[j] = fmaf(v, v, s2[j]);
          }
        }
      s1[j] += __shfl_xor(s1[j], 32, 64);
      s2[j] += __shfl_xor(s2[j], 32, 64);
    }
    // lds is free: the main loop ended with a barrier
    constexpr int BN = Cfg::BN;
    if (lane < 32) {
#pragma unroll
      for (int j = 0; j < Cfg::TN; ++j) {
        const int c = (wn * Cfg::TN + j) * 32 + lane;
        lds[wm * BN + c] = s1[j];
        lds[Cfg::WM * BN + wm * BN + c] = s2[j];
      }
    }
    __syncthreads();
    for (int c = threadIdx.x; c < BN; c += 256) {
      float a = 0.f, b = 0.f;
#pragma unroll
      for (int w = 0; w < Cfg::WM; ++w) {
        a += lds[w * BN + c];
        b += lds[Cfg::WM * BN + w * BN + c];
      }
      if (n0 + c < N) {
        P.partials[(int64_t)blockIdx.x * 2 * P.C + n0 + c] = a;
        P.partials[(int64_t)blockIdx.x * 2 * P.C + P.C + n0 + c] = b;
      }
    }
  }
};

struct EpiConvDgrad {  // scatter rows of a (parity-class) grid back to the full NHWC input gradient (+ bias)
  static constexpr int SCRATCH = 0;
  struct Params { float* dst; int GA, GB, ra, pa, rb, pb, DH, DW, C; const float* bias; };
  template <class Cfg>
  static __device__ void apply(const Params& P, f32x16 (&acc)[Cfg::TM][Cfg::TN], int m0, int n0, int wm, int wn,
                               int lane, int M, int N, float*) {
#pragma unroll
    for (int i = 0; i < Cfg::TM; ++i)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = m0 + acc_row<Cfg>(wm, i, r, lane);
        if (row >= M) continue;
        const int img = row / (P.GA * P.GB);
        const int rem = row - img * P.GA * P.GB;
        const int a = rem / P.GB, b = rem - a * P.GB;
        const int64_t base = (((int64_t)img * P.DH + a * P.ra + P.pa) * P.DW + b * P.rb + P.pb) * P.C;
#pragma unroll
        for (int j = 0; j < Cfg::TN; ++j) {
          const int col = n0 + acc_col<Cfg>(wn, j, lane);
          if (col < N) P.dst[base + col] = acc[i][j][r] + (P.bias ? P.bias[col] : 0.f);
        }
      }
  }
};

struct EpiPartial {  // split-K slab: part[z][row][col]
  static constexpr int SCRATCH = 0;
  struct Params { float* part; int64_t ld; };
  template <class Cfg>
  static __device__ void apply(const Params& P, f32x16 (&acc)[Cfg::TM][Cfg::TN], int m0, int n0, int wm, int wn,
                               int lane, int M, int N, float*) {
    float* base = P.part + (int64_t)blockIdx.z * M * P.ld;
#pragma unroll
    for (int i = 0; i < Cfg::TM; ++i)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = m0 + acc_row<Cfg>(wm, i, r, lane);
        if (row >= M) continue;
#pragma unroll
        for (int j = 0; j < Cfg::TN; ++j) {
          const int col = n0 + acc_col<Cfg>(wn, j, lane);
          if (col < N) base[(int64_t)row * P.ld + col] = acc[i][j][r];
        }
      }
  }
};

struct DenseEpiArgs {
  float* out; int64_t ldc; const float* bias; int relu; int drop; uint64_t h1; uint32_t thr; float dscale;
  int64_t row0; const float* gate; float gscale;
  int gmod;  // gate row = row % gmod when > 0 (the stacked rows of the direct classifier's affine backward)
};

__device__ inline float dense_finish(const DenseEpiArgs& P, int row, int col, float v) {
  if (P.bias) v += P.bias[col];
  if (P.relu) v = relu_nan(v);
  if (P.drop) v = (rng_u24(P.h1, (uint64_t)(P.row0 + row), (uint64_t)col) >= P.thr) ? v * P.dscale : 0.f;
  if (P.gate) v = P.gate[(int64_t)(P.gmod > 0 ? row % P.gmod : row) * P.ldc + col] > 0.f ? v * P.gscale : 0.f;
  return v;
}

struct EpiDense {
  static constexpr int SCRATCH = 0;
  using Params = DenseEpiArgs;
  template <class Cfg>
  static __device__ void apply(const Params& P, f32x16 (&acc)[Cfg::TM][Cfg::TN], int m0, int n0, int wm, int wn,
                               int lane, int M, int N, float*) {
#pragma unroll
    for (int i = 0; i < Cfg::TM; ++i)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = m0 + acc_row<Cfg>(wm, i, r, lane);
        if (row >= M) continue;
#pragma unroll
        for (int j = 0; j < Cfg::TN; ++j) {
          const int col = n0 + acc_col<Cfg>(wn, j, lane);
          if (col < N) P.out[(int64_t)row * P.ldc + col] = dense_finish(P, row, col, acc[i][j][r]);
        }
      }
  }
};

// sum_{z < S} p[z * stride] in z order, 8 loads in flight (clamped, unconditional): the slab sums of the split-K
// reduces (a plain loop leaves one dependent load round trip per slab)
__device__ __forceinline__ float slab_sum(const float* __restrict__ p, int S, int64_t stride) {
  float s = 0.f;
  for (int z0 = 0; z0 < S; z0 += 8) {
    float u[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) u[k] = p[(int64_t)min(z0 + k, S - 1) * stride];
#pragma unroll
    for (int k = 0; k < 8; ++k)
      if (z0 + k < S) s += u[k];
  }
  return s;
}

__global__ __launch_bounds__(256) void dense_splitk_reduce_kernel(const float* __restrict__ part, int S, int M, int N,
                                                                  DenseEpiArgs P, const int* skip) {
  if (skip && *skip == 0) return;
  const int64_t total = (int64_t)M * N;
  for (int64_t i = blockIdx.x * 256ll + threadIdx.x; i < total; i += (int64_t)gridDim.x * 256) {
    const float s = slab_sum(part + i, S, total);
    const int row = (int)(i / N), col = (int)(i % N);
    P.out[(int64_t)row * P.ldc + col] = dense_finish(P, row, col, s);
  }
}

// weight grad of a Linear: part[S][N][K+1] -> dW[N][K], db[N]
__global__ __launch_bounds__(256) void dense_wgrad_reduce_kernel(const float* __restrict__ part, int S, int N, int K,
                                                                 float* __restrict__ dW, float* __restrict__ db,
                                                                 const int* skip) {
  if (skip && *skip == 0) return;
  const int64_t ld = K + 1;
  const int64_t total = (int64_t)N * ld;
  for (int64_t i = blockIdx.x * 256ll + threadIdx.x; i < total; i += (int64_t)gridDim.x * 256) {
    const float s = slab_sum(part + i, S, total);
    const int row = (int)(i / ld), col = (int)(i % ld);
    if (col < K) dW[(int64_t)row * K + col] = s;
    else if (db) db[row] = s;
  }
}

// =====================================================================================================
// launch helpers
// =====================================================================================================
template <class Cfg, template <int> class LA, template <int> class LB, class Epi>
static int launch_gemm(const typename LA<Cfg::BM>::Params& pa, const typename LB<Cfg::BN>::Params& pb,
                       const typename Epi::Params& pe, int M, int N, int K, int splits, const int* skip,
                       hipStream_t st, int* used_splits = nullptr) {
  if (M <= 0 || N <= 0) return 0;
  splits = std::max(1, splits);
  int kps = (int)(cdiv(cdiv(K, splits), BK) * BK);
  if (kps <= 0) kps = BK;
  splits = (int)cdiv(K, kps);
  if (splits < 1) splits = 1;
  dim3 grid((unsigned)cdiv(M, Cfg::BM), (unsigned)cdiv(N, Cfg::BN), (unsigned)splits);
  VAD_KLAUNCH((gemm_kernel<Cfg, LA<Cfg::BM>, LB<Cfg::BN>, Epi>), grid, dim3(256), 0, st, pa, pb, pe, M, N, K,
                     kps, skip);
  VAD_LAUNCH_CHECK();
  if (used_splits) *used_splits = splits;
  return 0;
}

using T128x32 = TileCfg<4, 1, 1, 1>;
using T128x64 = TileCfg<2, 2, 2, 1>;
using T64x64 = TileCfg<2, 2, 1, 1>;
using T128x128 = TileCfg<2, 2, 2, 2>;
using T32x128 = TileCfg<1, 4, 1, 1>;

// runtime-selectable tile shapes for the conv GEMMs (tuning / sweeps); id -> TileCfg
template <class F>
static int with_tile(int id, F&& f) {
  switch (id) {
    case 0: return f(TileCfg<4, 1, 1, 1>{});  // 128 x 32
    case 1: return f(TileCfg<4, 1, 2, 1>{});  // 256 x 32
    case 2: return f(TileCfg<2, 2, 1, 1>{});  //  64 x 64
    case 3: return f(TileCfg<2, 2, 2, 1>{});  // 128 x 64
    case 4: return f(TileCfg<2, 2, 1, 2>{});  //  64 x 128
    case 5: return f(TileCfg<2, 2, 2, 2>{});  // 128 x 128
    case 6: return f(TileCfg<4, 1, 2, 2>{});  // 256 x 64
    case 7: return f(TileCfg<1, 4, 1, 1>{});  //  32 x 128
    case 8: return f(TileCfg<1, 4, 1, 2>{});  //  32 x 256
    case 9: return f(TileCfg<2, 2, 1, 4>{});  //  64 x 256
    default: set_error("unknown tile id"); return 1;
  }
}
static int tile_bm(int id) {
  static const int bm[10] = {128, 256, 64, 128, 64, 128, 256, 32, 32, 64};
  return (id >= 0 && id < 10) ? bm[id] : 64;
}

struct ConvTuning {
  int fwd = -1, dgrad = -1, wgrad = -1;  // forced tile ids (-1: heuristic)
  int wgrad_blocks = 1024;               // target grid size of the split-K weight gradient
  int wgrad_min_ktiles = 16;             // minimum BK-slices per split
  int patch = 1;                         // stride-1 fwd/dgrad on the LDS-patch kernels
  int wgrad_patch = 1;                   // weight gradients on the LDS-patch kernel: 1 stride-1 layers, 2 all
  int wgrad_alone_blocks = 448;          // the same for a weight gradient nothing else runs beside (the last layer's;
                                         // 512 / 1024 measured no faster)
  int wgrad_patch_blocks = 448;          // its target grid size (below 2 per CU: the weight gradients share the GPU with the input gradients, own stream)
};
static ConvTuning g_tune;

extern int g_bbox_im2col;  // bbox_plan.hip
extern int g_maxpool_bwd_win;  // conv3d.hip
extern int g_ae_direct, g_ae_wgrad_blocks, g_ae_wgrad_stream;  // ae_plan.hip
extern int g_conv4_cls_batch_min, g_conv4_split_tiles;
extern int g_a2_direct, g_a2_head_clip;     // a2_plan.hip
extern int g_conv3s2_fwd_blocks;
int set_tuning(const char* key, int value) {
  const std::string k(key);
  if (k == "conv_fwd_tile") g_tune.fwd = value;
  else if (k == "conv_dgrad_tile") g_tune.dgrad = value;
  else if (k == "conv_wgrad_tile") g_tune.wgrad = value;
  else if (k == "conv_wgrad_blocks") g_tune.wgrad_blocks = value;
  else if (k == "conv_wgrad_min_ktiles") g_tune.wgrad_min_ktiles = value;
  else if (k == "conv_patch") g_tune.patch = value;
  else if (k == "conv_patch_persist") g_patch_persist = value;
  else if (k == "conv_split") g_conv_split = value;
  else if (k == "conv_split_nt") g_x3_nt = value;
  else if (k == "conv_split_wres") g_x3_wres = value;
  else if (k == "conv_wgrad_patch") g_tune.wgrad_patch = value;
  else if (k == "conv_wgrad_split") g_wgrad_split = value;
  else if (k == "conv_wgrad_split_s2") g_wgrad_split_s2 = value;
  else if (k == "conv_wgrad_tr") g_wgrad_tr = value;
  else if (k == "conv_wgrad_tr_blocks") g_wgrad_tr_blocks = value;
  else if (k == "conv_wgrad_tr_pft") g_wgrad_tr_pft = value;
  else if (k == "conv_wgrad_s2_blocks") g_wgrad_s2_blocks = value;
  else if (k == "stem_fused") g_stem_fused = value;
  else if (k == "conv_dgrad_s2_x3") g_dgrad_s2_x3 = value;
  else if (k == "conv_dgrad_blocks") g_x3_dgrad_blocks = value;
  else if (k == "conv_split_big") g_x3_big = value;
  else if (k == "conv_split_s2big") g_x3_s2big = value;
  else if (k == "bbox_im2col") g_bbox_im2col = value;
  else if (k == "ae_direct") g_ae_direct = value;
  else if (k == "ae_wgrad_blocks") g_ae_wgrad_blocks = value;
  else if (k == "ae_wgrad_stream") g_ae_wgrad_stream = value;
  else if (k == "conv4_cls_batch_min") g_conv4_cls_batch_min = value;
  else if (k == "conv4_split_tiles") g_conv4_split_tiles = value;
  else if (k == "a2_direct") g_a2_direct = value;
  else if (k == "a2_head_clip") g_a2_head_clip = value;
  else if (k == "cad_prep_stream") g_cad_prep_stream = value;
  else if (k == "conv3s2_fwd_blocks") g_conv3s2_fwd_blocks = value;
  else if (k == "cad_wgrad_stream") g_cad_wgrad_stream = value;
  else if (k == "cad_dir_affine") g_cad_dir_affine = value;
  else if (k == "cad_det_gate") g_cad_det_gate = value;
  else if (k == "cad_stem_early") g_cad_stem_early = value;
  else if (k == "cad_dy_per_layer") g_cad_dy_per_layer = value;
  else if (k == "cad_event_sysfence") g_cad_event_sysfence = value;
  else if (k == "mlp_tail_wide") g_mlp_tail_wide = value;
  else if (k == "mlp_tail_rb") g_mlp_tail_rb = value;
  else if (k == "cad_last_wgrad_main") g_cad_last_wgrad_main = value;
  else if (k == "cad_l0_slab") g_cad_l0_slab = value;
  else if (k == "cad_stream_prio") g_cad_stream_prio = value;
  else if (k == "conv_split_pipe") g_x3_pipe = value;
  else if (k == "bn_bwd_fuse") g_bn_bwd_fuse = value;
  else if (k == "bn_apply_v") g_bn_apply_v = value;
  else if (k == "conv_wgrad_s1_nt") g_wgrad_s1_nt = value;
  else if (k == "conv_wgrad_s1_nt_wide") g_wgrad_s1_nt_wide = value;
  else if (k == "conv_wgrad_s1_nt_blocks") g_wgrad_s1_nt_blocks = value;
  else if (k == "conv_bf16") g_conv_bf16 = value;  // ops API only (calling thread); plans use their own option
  else if (k == "act_bf16") g_act_bf16 = value;    // ops API only: bf16 activation storage for the calling thread
  else if (k == "conv_bfc") g_bfc = value;
  else if (k == "conv_bfc_blocks") g_bfc_blocks = value;
  else if (k == "conv_bfc_s2_ni2") g_bfc_s2_ni2 = value;
  else if (k == "conv3d_direct") g_conv3d_direct = value;
  else if (k == "maxpool3d_bwd_win") g_maxpool_bwd_win = value;
  else if (k == "conv3d_wgrad_blocks") g_conv3d_wg_blocks = value;
  else if (k == "conv_dgrad_s2_w3") g_dgrad_s2_w3 = value;
  else if (k == "conv_dgrad_s2_nt") g_dgrad_s2_nt = value;
  else if (k == "bn_apply_u") g_bn_apply_u = value;
  else if (k == "bn_apply_blocks") g_bn_apply_blocks = value;
  else if (k == "conv_bfw_blocks") g_bfw_blocks = value;
  else if (k == "conv_wgrad_patch_blocks") g_tune.wgrad_patch_blocks = value;
  else if (k == "conv_wgrad_alone_blocks") g_tune.wgrad_alone_blocks = value;
  else {
    set_error("unknown tuning key " + k);
    return 1;
  }
  return 0;
}

// heuristics (fallback when no tile is forced); BM >= 64 keeps the forward BN partial count within bounds
static int pick_fwd_tile(int M, int N) {
  if (g_tune.fwd >= 0 && tile_bm(g_tune.fwd) >= 64) return g_tune.fwd;
  if (N == 32) return 0;
  return M >= 64 * 1024 ? 3 : 2;
}
static int pick_dgrad_tile(int M, int N) {
  if (g_tune.dgrad >= 0) return g_tune.dgrad;
  if (N <= 32) return 0;  // (128 x 32: a2's 16-channel input gradient wastes half a tile instead of three quarters)
  return M >= 64 * 1024 ? 3 : 2;
}
static int pick_wgrad_tile(int M, int N) {
  (void)N;
  if (g_tune.wgrad >= 0) return g_tune.wgrad;
  return M == 32 ? 7 : 2;
}

// =====================================================================================================
// 3x3 convs
// =====================================================================================================
static void fwd_taps(TapTable& t) {
  t.ntaps = 9;
  for (int k = 0; k < 9; ++k) {
    t.dh[k] = (int8_t)(k / 3 - 1);
    t.dw[k] = (int8_t)(k % 3 - 1);
  }
}

// dgrad parity classes.  stride 1: one class, all taps, src offset = 1 - k.  stride 2: class (ph,pw) uses
// taps kh with (ph+1-kh) even, src offset (ph+1-kh)/2.
struct DgradClass {
  int ph, pw, nrt, nct;
  int kh[2], dh[2], kw[2], dw[2];
};
static int dgrad_classes(int stride, DgradClass* cls) {
  if (stride == 1) return 0;
  int n = 0;
  for (int ph = 0; ph < 2; ++ph)
    for (int pw = 0; pw < 2; ++pw) {
      DgradClass c{};
      c.ph = ph; c.pw = pw; c.nrt = c.nct = 0;
      for (int k = 0; k < 3; ++k) {
        if (((ph + 1 - k) & 1) == 0) { c.kh[c.nrt] = k; c.dh[c.nrt] = (ph + 1 - k) / 2; ++c.nrt; }
        if (((pw + 1 - k) & 1) == 0) { c.kw[c.nct] = k; c.dw[c.nct] = (pw + 1 - k) / 2; ++c.nct; }
      }
      cls[n++] = c;
    }
  return n;
}

// dgrad weight images: stride 1 and the stride-2 patch kernel -> Wd[ci][t=kh*3+kw][co]; stride-2 GEMM path -> per
// class, concatenated, Wd_c[ci][ri*nct+cj][co] for taps (kh[ri], kw[cj]).
__global__ void conv3_prep_kernel(const float* __restrict__ w, int Ci, int Co, int classes, float* __restrict__ wf,
                                  float* __restrict__ wd) {
  const int64_t total = (int64_t)Co * Ci * 9;
  for (int64_t i = blockIdx.x * 256ll + threadIdx.x; i < total; i += (int64_t)gridDim.x * 256) {
    const int t = (int)(i % 9);
    const int ci = (int)((i / 9) % Ci);
    const int co = (int)(i / (9 * Ci));
    const float v = w[i];
    wf[((int64_t)co * 9 + t) * Ci + ci] = v;
    const int kh = t / 3, kw = t % 3;
    if (!classes) {
      wd[((int64_t)ci * 9 + t) * Co + co] = v;
    } else {
      // class (ph,pw): kh valid iff (ph+1-kh) even -> ph = (kh+1)&1; its index among the class's row taps
      const int ph = (kh + 1) & 1, pw = (kw + 1) & 1;
      const int ri = (ph == 0) ? 0 : (kh == 0 ? 0 : 1);
      const int cj = (pw == 0) ? 0 : (kw == 0 ? 0 : 1);
      const int nrt = ph == 0 ? 1 : 2, nct = pw == 0 ? 1 : 2;
      int64_t off = 0;  // classes in order (0,0),(0,1),(1,0),(1,1)
      for (int c = 0; c < ph * 2 + pw; ++c) {
        const int r = (c >> 1) == 0 ? 1 : 2, q = (c & 1) == 0 ? 1 : 2;
        off += (int64_t)r * q * Ci * Co;
      }
      wd[off + ((int64_t)ci * (nrt * nct) + ri * nct + cj) * Co + co] = v;
    }
  }
}

struct PrepTab {
  const float* w[8];
  float* wf[8];
  float* wd[8];
  __bf16* w3[8];  // nullable: pre-split bf16 planes of Wd, [ci][tap][co / 16][3][16]
  int Ci[8], Co[8], classes[8];
  int64_t end[8];  // inclusive prefix sums of Co*Ci*9
  int n;
  int bf16;  // also the bf16 copies of the plain images (conv3_bf16_image: behind the fp32 image)
};

__global__ void conv3_prep_all_kernel(const PrepTab t) {
  const int64_t total = t.end[t.n - 1];
  for (int64_t g = blockIdx.x * 256ll + threadIdx.x; g < total; g += (int64_t)gridDim.x * 256) {
    int l = 0;
    while (g >= t.end[l]) ++l;
    const int64_t i = g - (l ? t.end[l - 1] : 0);
    const int Ci = t.Ci[l], Co = t.Co[l];
    const int tap = (int)(i % 9);
    const int ci = (int)((i / 9) % Ci);
    const int co = (int)(i / (9 * Ci));
    const float v = t.w[l][i];
    t.wf[l][((int64_t)co * 9 + tap) * Ci + ci] = v;
    if (t.bf16) {
      const int64_t tot = (int64_t)Co * Ci * 9;
      reinterpret_cast<__bf16*>(t.wf[l] + tot)[((int64_t)co * 9 + tap) * Ci + ci] = (__bf16)v;
      reinterpret_cast<__bf16*>(t.wd[l] + tot)[((int64_t)ci * 9 + tap) * Co + co] = (__bf16)v;
    }
    if (t.w3[l]) {  // (the split of put_planes / split3: hi, mid, lo)
      const __bf16 h = (__bf16)v;
      const float r = v - (float)h;
      const __bf16 m = (__bf16)r;
      __bf16* d = t.w3[l] + ((((int64_t)ci * 9 + tap) * (Co / 16) + co / 16) * 3) * 16 + co % 16;
      d[0] = h;
      d[16] = m;
      d[32] = (__bf16)(r - (float)m);
    }
    if (!t.classes[l]) {
      t.wd[l][((int64_t)ci * 9 + tap) * Co + co] = v;
    } else {
      const int kh = tap / 3, kw = tap % 3;
      const int ph = (kh + 1) & 1, pw = (kw + 1) & 1;
      const int ri = (ph == 0) ? 0 : (kh == 0 ? 0 : 1);
      const int cj = (pw == 0) ? 0 : (kw == 0 ? 0 : 1);
      const int nrt = ph == 0 ? 1 : 2, nct = pw == 0 ? 1 : 2;
      int64_t off = 0;
      for (int c = 0; c < ph * 2 + pw; ++c) {
        const int r = (c >> 1) == 0 ? 1 : 2, q = (c & 1) == 0 ? 1 : 2;
        off += (int64_t)r * q * Ci * Co;
      }
      t.wd[l][off + ((int64_t)ci * (nrt * nct) + ri * nct + cj) * Co + co] = v;
    }
  }
}

int conv3_prep_weights_all(int n, const float* const* w, const Conv3Layer* L, float* const* wf, float* const* wd,
                           hipStream_t st, __bf16* const* w3) {
  VAD_CHECK(n >= 1 && n <= 8, "conv3_prep_weights_all: 1..8 layers");
  PrepTab t{};
  t.n = n;
  t.bf16 = g_conv_bf16 && g_act_bf16;
  int64_t acc = 0;
  for (int l = 0; l < n; ++l) {
    t.w[l] = w[l];
    t.wf[l] = wf[l];
    t.wd[l] = wd[l];
    t.w3[l] = w3 ? w3[l] : nullptr;
    VAD_CHECK(!t.w3[l] || L[l].Co % 16 == 0, "conv3_prep_weights_all: pre-split Wd needs Co % 16 == 0");
    t.Ci[l] = L[l].Ci;
    t.Co[l] = L[l].Co;
    t.classes[l] = L[l].stride == 2 && !(g_tune.patch && conv3_patch_supported(L[l], false));
    acc += (int64_t)L[l].Co * L[l].Ci * 9;
    t.end[l] = acc;
  }
  hipLaunchKernelGGL(conv3_prep_all_kernel, dim3((unsigned)std::min<int64_t>(cdiv(acc, 256), 4096)), dim3(256), 0, st,
                     t);
  VAD_LAUNCH_CHECK();
  return 0;
}

int conv3_prep_weights(const float* w, const Conv3Layer& L, float* wf, float* wd, hipStream_t st) {
  return conv3_prep_weights_all(1, &w, &L, &wf, &wd, st);
}

int conv3_fwd(const Conv3Layer& L, const float* src, const float* src_stats, const float* wf, const float* bias,
              float* y, float* partials, int* nparts, hipStream_t st, int* parts_cm) {
  if (parts_cm) *parts_cm = 0;
  if (bfc_supported(L, true)) {  // native bf16 kernels (config 4): column-major partials
    if (parts_cm) *parts_cm = 1;
    return bfc_fwd(L, reinterpret_cast<const __bf16*>(src), src_stats, conv3_bf16_image(wf, L), bias,
                   reinterpret_cast<__bf16*>(y), partials, conv3_patch_blocks(L.NF, L.OH, L.OW) * 2 * L.Co, nparts, st);
  }
  VAD_CHECK(L.Ci % 32 == 0, "conv3_fwd: Ci must be a multiple of 32");
  // (the patch grid may exceed ceil(M/64) BN partial blocks on tiny images: those stay on the GEMM path)
  if (g_tune.patch && conv3_patch_blocks(L.NF, L.OH, L.OW) <= cdiv((int64_t)L.NF * L.OH * L.OW, 64)) {
    if (conv3_x3_supported(L, true))
      return conv3_x3_fwd(L, src, src_stats, wf, bias, y, partials, nparts, st, parts_cm);
    VAD_CHECK(!g_act_bf16, "conv3_fwd: bf16 activations need the split kernels");
    if (conv3_patch_supported(L, true)) return conv3_patch_fwd(L, src, src_stats, wf, bias, y, partials, nparts, st);
  }
  VAD_CHECK(!g_act_bf16, "conv3_fwd: bf16 activations need the split kernels");
  ConvGeom g{L.NF, L.OH, L.OW, L.stride, L.stride, L.IH, L.IW, L.Ci};
  TapTable taps;
  fwd_taps(taps);
  const int M = L.NF * L.OH * L.OW, N = L.Co, K = 9 * L.Ci;
  EpiConvFwd::Params pe{y, bias, L.Co, partials};
  const int id = pick_fwd_tile(M, N);
  return with_tile(id, [&](auto cfg) -> int {
    using C = decltype(cfg);
    VAD_CHECK(gather_fits((int64_t)g.imgs * g.SH * g.SW * g.C), "conv gather: source over 2 GB");
    typename ConvGatherKC<C::BM>::Params pa{src, g, taps, src_stats ? src_stats + 2 * L.Ci : nullptr,
                                            src_stats ? src_stats + 3 * L.Ci : nullptr};
    typename DenseKC<C::BN>::Params pb{wf, K, N, K};
    VAD_TRY((launch_gemm<C, ConvGatherKC, DenseKC, EpiConvFwd>(pa, pb, pe, M, N, K, 1, nullptr, st)));
    *nparts = (int)cdiv(M, C::BM);
    return 0;
  });
}

static int dgrad_launch(const ConvGeom& g, const TapTable& taps, const float* dY, const float* wd, int N,
                        const EpiConvDgrad::Params& pe, hipStream_t st) {
  const int M = g.imgs * g.GA * g.GB, K = taps.ntaps * g.C;
  return with_tile(pick_dgrad_tile(M, N), [&](auto cfg) -> int {
    using C = decltype(cfg);
    VAD_CHECK(gather_fits((int64_t)g.imgs * g.SH * g.SW * g.C), "conv gather: source over 2 GB");
    typename ConvGatherKC<C::BM>::Params pa{dY, g, taps, nullptr, nullptr};
    typename DenseKC<C::BN>::Params pb{wd, K, N, K};
    return launch_gemm<C, ConvGatherKC, DenseKC, EpiConvDgrad>(pa, pb, pe, M, N, K, 1, nullptr, st);
  });
}

int conv3_dgrad(const Conv3Layer& L, const float* dY, const float* wd, float* dX, hipStream_t st,
                const BnBwdFuse* f, const __bf16* w3) {
  VAD_CHECK(L.Co % 32 == 0, "conv3_dgrad: Co must be a multiple of 32");
  const int N = L.Ci;
  if (f) *f->nparts = 0;
  if (bfc_supported(L, false))
    return bfc_dgrad(L, reinterpret_cast<const __bf16*>(dY), conv3_bf16_image(wd, L), reinterpret_cast<__bf16*>(dX), st,
                     (g_bn_bwd_fuse & 1) ? f : nullptr);
  if (g_tune.patch && conv3_x3_supported(L, false))
    return conv3_x3_dgrad(L, dY, wd, dX, st, (g_bn_bwd_fuse & 1) ? f : nullptr);
  // (the split kernel reads the plain Wd layout, which the prep writes exactly when the f32 patch kernel is usable)
  if (g_tune.patch && conv3_patch_supported(L, false) && conv3_x3_dgrad_s2_supported(L))
    return conv3_x3_dgrad_s2(L, dY, wd, dX, st, (g_bn_bwd_fuse & 2) ? f : nullptr, w3);
  VAD_CHECK(!g_act_bf16, "conv3_dgrad: bf16 activations need the split kernels");
  if (g_tune.patch && conv3_patch_supported(L, false)) return conv3_patch_dgrad(L, dY, wd, dX, st);
  if (L.stride == 1) {
    ConvGeom g{L.NF, L.IH, L.IW, 1, 1, L.OH, L.OW, L.Co};
    TapTable taps;
    taps.ntaps = 9;
    for (int k = 0; k < 9; ++k) {
      taps.dh[k] = (int8_t)(1 - k / 3);
      taps.dw[k] = (int8_t)(1 - k % 3);
    }
    EpiConvDgrad::Params pe{dX, L.IH, L.IW, 1, 0, 1, 0, L.IH, L.IW, L.Ci};
    return dgrad_launch(g, taps, dY, wd, N, pe, st);
  }
  DgradClass cls[4];
  const int nc = dgrad_classes(2, cls);
  int64_t off = 0;
  for (int ci = 0; ci < nc; ++ci) {
    const DgradClass& c = cls[ci];
    const int GA = (L.IH - c.ph + 1) / 2, GB = (L.IW - c.pw + 1) / 2;
    ConvGeom g{L.NF, GA, GB, 1, 1, L.OH, L.OW, L.Co};
    TapTable taps;
    taps.ntaps = c.nrt * c.nct;
    for (int r = 0; r < c.nrt; ++r)
      for (int q = 0; q < c.nct; ++q) {
        taps.dh[r * c.nct + q] = (int8_t)c.dh[r];
        taps.dw[r * c.nct + q] = (int8_t)c.dw[q];
      }
    EpiConvDgrad::Params pe{dX, GA, GB, 2, c.ph, 2, c.pw, L.IH, L.IW, L.Ci};
    VAD_TRY(dgrad_launch(g, taps, dY, wd + off, N, pe, st));
    off += (int64_t)taps.ntaps * L.Ci * L.Co;
  }
  return 0;
}

bool conv3_act_bf16_ok(const Conv3Layer& L, bool dgrad) {
  {
    ActStorage abf(1);  // (the native bf16 kernels exist for bf16 storage only)
    if (bfc_supported(L, true) && (!dgrad || bfc_supported(L, false) || conv3_x3_dgrad_s2_supported(L)) &&
        (bfc_wgrad_supported(L) || (g_tune.wgrad_patch && conv3_wgrad_x3_supported(L))))
      return true;
  }
  const bool fwd = g_tune.patch && conv3_patch_blocks(L.NF, L.OH, L.OW) <= cdiv((int64_t)L.NF * L.OH * L.OW, 64) &&
                   conv3_x3_supported(L, true);
  const bool dg = !dgrad || (g_tune.patch && (conv3_x3_supported(L, false) ||
                                              (conv3_patch_supported(L, false) && conv3_x3_dgrad_s2_supported(L))));
  const bool wg = g_tune.wgrad_patch && conv3_wgrad_x3_supported(L);
  return fwd && dg && wg;
}

int conv3_path(const Conv3Layer& L, int kind) {
  if (kind < 2 ? bfc_supported(L, kind == 0) : bfc_wgrad_supported(L)) return 2;
  bool x3 = false;
  if (kind == 1 && L.stride == 2)  // stride-2 input gradients: the parity-class split kernel when supported
    x3 = g_tune.patch && conv3_patch_supported(L, false) && conv3_x3_dgrad_s2_supported(L);
  else if (kind == 0)
    x3 = g_tune.patch && conv3_patch_blocks(L.NF, L.OH, L.OW) <= cdiv((int64_t)L.NF * L.OH * L.OW, 64) &&
         conv3_x3_supported(L, true);
  else if (kind == 1)
    x3 = g_tune.patch && conv3_x3_supported(L, false);
  else
    x3 = g_tune.wgrad_patch && (x3_wgrad_tr_supported(L) || conv3_wgrad_x3_supported(L));
  return x3 ? (g_conv_bf16 ? 1 : 6) : 0;
}

int conv3_wgrad(const Conv3Layer& L, const float* dY, const float* src, const float* src_stats, float* partial,
                int* nsplit, int64_t partial_cap, hipStream_t st, bool alone) {
  if (bfc_wgrad_supported(L))
    return bfc_wgrad(L, reinterpret_cast<const __bf16*>(dY), reinterpret_cast<const __bf16*>(src), src_stats, partial,
                     nsplit, partial_cap, st);
  if (g_tune.wgrad_patch && x3_wgrad_tr_supported(L))
    return x3_wgrad_tr(L, dY, src, src_stats, partial, nsplit, partial_cap, alone ? g_tune.wgrad_alone_blocks : 0, st);
  if (g_tune.wgrad_patch && conv3_wgrad_x3_supported(L))
    return conv3_wgrad_x3(L, dY, src, src_stats, partial, nsplit, partial_cap,
                          alone ? g_tune.wgrad_alone_blocks : g_tune.wgrad_patch_blocks, st);
  VAD_CHECK(!g_act_bf16, "conv3_wgrad: bf16 activations need the split kernels");
  if (g_tune.wgrad_patch && conv3_wgrad_patch_supported(L) && (L.stride == 1 || g_tune.wgrad_patch == 2))
    return conv3_wgrad_patch(L, dY, src, src_stats, partial, nsplit, partial_cap, g_tune.wgrad_patch_blocks, st);
  const int M = L.Co, N = 9 * L.Ci, K = L.NF * L.OH * L.OW;
  return with_tile(pick_wgrad_tile(M, N), [&](auto cfg) -> int {
    using C = decltype(cfg);
    const int tiles = (int)(cdiv(M, C::BM) * cdiv(N, C::BN));
    int splits = (int)std::max<int64_t>(
        1, std::min<int64_t>(cdiv(g_tune.wgrad_blocks, tiles), cdiv(K, (int64_t)g_tune.wgrad_min_ktiles * BK)));
    while ((int64_t)splits * M * N > partial_cap && splits > 1) splits /= 2;
    VAD_CHECK(gather_fits((int64_t)K * L.Co), "dense gather: operand over 2 GB");
    typename DenseKM<C::BM>::Params pa{dY, L.Co, L.Co, K, -1};
    VAD_CHECK(gather_fits((int64_t)L.NF * L.IH * L.IW * L.Ci), "conv patch: source over 2 GB");
    typename ConvPatchKM<C::BN>::Params pb{src, L.NF, L.OH, L.OW, L.stride, 1, L.IH, L.IW, L.Ci, 3, N,
                                           src_stats ? src_stats + 2 * L.Ci : nullptr,
                                           src_stats ? src_stats + 3 * L.Ci : nullptr};
    EpiPartial::Params pe{partial, N};
    return launch_gemm<C, DenseKM, ConvPatchKM, EpiPartial>(pa, pb, pe, M, N, K, splits, nullptr, st, nsplit);
  });
}

// Split-K slab reduction of the conv weight gradient.  Block = 256/SL float4 columns x SL split lanes; lane sl sums
// slabs sl, sl + SL, ... in order with 8 loads in flight (unconditional, from clamped slab indices), and the SL lanes
// of a column are combined through LDS in a fixed order.  SL = the smallest of 1, 2, 4, 8, 16 that leaves each lane
// <= 16 slabs (the wide layers have 12-48 slabs: one lane per column reads them all; the 32-channel layers up to
// 512: 16 lanes) -- a fixed function of S, so the summation order is fixed per layer.  Slab layout [S][co][t*Ci + ci];
// dW is torch [co][ci][kh][kw].  Extra blocks after the first wblocks reduce the conv bias (one block per channel).
template <int SL>
__global__ __launch_bounds__(256) void conv3_wgrad_reduce_kernel(const float* __restrict__ part, int S, int Co, int Ci,
                                                                 const float* __restrict__ bparts, int NB,
                                                                 float* __restrict__ dW, float* __restrict__ db,
                                                                 int wblocks) {
  constexpr int NCOL = 256 / SL;
  __shared__ f32x4 red[SL > 1 ? SL : 1][NCOL + 1];
  const int64_t ldp = 9 * Ci;
  const int64_t total = (int64_t)Co * ldp;
  if ((int)blockIdx.x >= wblocks) {  // conv bias: one block per channel, 256-way strided sum + tree
    const int c = blockIdx.x - wblocks;
    float s = 0.f;
    for (int p = threadIdx.x; p < NB; p += 256) s += bparts[(int64_t)p * 2 * Co + c];
    s = wave_sum(s);
    __shared__ float r0[4];
    if ((threadIdx.x & 63) == 0) r0[threadIdx.x >> 6] = s;
    __syncthreads();
    if (threadIdx.x == 0) db[c] = (r0[0] + r0[1]) + (r0[2] + r0[3]);
    return;
  }
  const int e = threadIdx.x % NCOL, sl = threadIdx.x / NCOL;
  const int64_t i = ((int64_t)blockIdx.x * NCOL + e) * 4;  // total % 4 == 0 (Ci % 4 == 0)
  f32x4 a0 = {0.f, 0.f, 0.f, 0.f};
  if (i < total) {
    const int n = S > sl ? (S - sl + SL - 1) / SL : 0;
    for (int k0 = 0; k0 < n; k0 += 8) {
      f32x4 v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u)
        v[u] = *reinterpret_cast<const f32x4*>(part + (int64_t)(sl + SL * min(k0 + u, n - 1)) * total + i);
#pragma unroll
      for (int u = 0; u < 8; ++u)
        if (k0 + u < n) a0 += v[u];
    }
  }
  f32x4 s = a0;
  if constexpr (SL > 1) {
    red[sl][e] = a0;
    __syncthreads();
    if (sl != 0) return;
    // pairwise tree over the SL lanes, fixed order
    f32x4 q[SL];
#pragma unroll
    for (int u = 0; u < SL; ++u) q[u] = red[u][e];
#pragma unroll
    for (int w = 1; w < SL; w <<= 1)
#pragma unroll
      for (int u = 0; u < SL; u += 2 * w) q[u] += q[u + w];
    s = q[0];
  }
  if (i < total) {
    const int64_t co = i / ldp, r = i - co * ldp;
    const int t = (int)(r / Ci), ci = (int)(r - (int64_t)t * Ci);
#pragma unroll
    for (int u = 0; u < 4; ++u) dW[(co * Ci + ci + u) * 9 + t] = s[u];
  }
}

int conv3_wgrad_reduce(const Conv3Layer& L, const float* partial, int nsplit, const float* bias_partials,
                       int nbias_parts, float* dW, float* db, hipStream_t st) {
  const int64_t total = (int64_t)L.Co * L.Ci * 9;
  VAD_CHECK(L.Ci % 4 == 0, "conv3_wgrad_reduce: Ci % 4");
  int sl = 1;
  while (sl < 16 && cdiv(nsplit, sl) > 16) sl *= 2;
  const int wblocks = (int)cdiv(total, 4 * (256 / sl));
  const int bblocks = db ? L.Co : 0;
  const dim3 grid((unsigned)(wblocks + bblocks));
  switch (sl) {
    case 1: VAD_KLAUNCH(conv3_wgrad_reduce_kernel<1>, grid, dim3(256), 0, st, partial, nsplit, L.Co, L.Ci, bias_partials, nbias_parts, dW, db, wblocks); break;
    case 2: VAD_KLAUNCH(conv3_wgrad_reduce_kernel<2>, grid, dim3(256), 0, st, partial, nsplit, L.Co, L.Ci, bias_partials, nbias_parts, dW, db, wblocks); break;
    case 4: VAD_KLAUNCH(conv3_wgrad_reduce_kernel<4>, grid, dim3(256), 0, st, partial, nsplit, L.Co, L.Ci, bias_partials, nbias_parts, dW, db, wblocks); break;
    case 8: VAD_KLAUNCH(conv3_wgrad_reduce_kernel<8>, grid, dim3(256), 0, st, partial, nsplit, L.Co, L.Ci, bias_partials, nbias_parts, dW, db, wblocks); break;
    default: VAD_KLAUNCH(conv3_wgrad_reduce_kernel<16>, grid, dim3(256), 0, st, partial, nsplit, L.Co, L.Ci, bias_partials, nbias_parts, dW, db, wblocks); break;
  }
  VAD_LAUNCH_CHECK();
  return 0;
}

// =====================================================================================================
// dense layers
// =====================================================================================================
// Few-row layers (M <= 16: the direct classifier runs on the B clips of a rank, cad:568-570) are bound by the weight
// read and by launch latency, not by FLOPs: they use row-streaming kernels instead of the MFMA GEMM tiles, whose K
// loop over 64-row tiles would leave most of the chip idle.
constexpr int kSkinnyRows = 16;
static bool skinny_ok(int M, int K) { return M >= 1 && M <= kSkinnyRows && K % 4 == 0; }

// Y[m][n] = finish(sum_k X[m][k] W[n][k]): a block owns 4 output columns; its 512 threads stride over K in float4
// steps (coalesced W rows, X from L2) with the loads of up to 4 steps in flight, then the 4*MR partial sums are
// combined through LDS in a fixed order.
template <int MR>
__global__ __launch_bounds__(512) void skinny_fwd_kernel(const float* __restrict__ X, int M, int K,
                                                         const float* __restrict__ W, int N, DenseEpiArgs P) {
  constexpr int NT = 512, NO = 4 * MR, G = NT / NO, U = 4;
  __shared__ float red[NT][NO + 1];
  const int tid = threadIdx.x, n0 = blockIdx.x * 4, K4 = K / 4;
  float acc[4][MR];
#pragma unroll
  for (int c = 0; c < 4; ++c)
#pragma unroll
    for (int m = 0; m < MR; ++m) acc[c][m] = 0.f;
  // (all loads unconditional from clamped addresses, out-of-range terms zeroed afterwards: a predicated load makes the
  // compiler wait for the previous one, i.e. one memory round trip per load)
  for (int kb = 0; kb < K4; kb += NT * U) {
    f32x4 w[U][4];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int k4 = min(kb + u * NT + tid, K4 - 1);
#pragma unroll
      for (int c = 0; c < 4; ++c)
        w[u][c] = *reinterpret_cast<const f32x4*>(W + (int64_t)min(n0 + c, N - 1) * K + 4 * k4);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int k4 = kb + u * NT + tid;
      if (k4 >= K4) break;
      f32x4 xv[MR];
#pragma unroll
      for (int m = 0; m < MR; ++m) xv[m] = *reinterpret_cast<const f32x4*>(X + (int64_t)min(m, M - 1) * K + 4 * k4);
#pragma unroll
      for (int m = 0; m < MR; ++m) {
        const f32x4 x = m < M ? xv[m] : f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int c = 0; c < 4; ++c)
          acc[c][m] = fmaf(x[3], w[u][c][3], fmaf(x[2], w[u][c][2], fmaf(x[1], w[u][c][1], fmaf(x[0], w[u][c][0], acc[c][m]))));
      }
    }
  }
#pragma unroll
  for (int c = 0; c < 4; ++c)
#pragma unroll
    for (int m = 0; m < MR; ++m) red[tid][c * MR + m] = acc[c][m];
  __syncthreads();
  const int o = tid / G, part = tid % G;
  float v = 0.f;
  for (int r = part; r < NT; r += G) v += red[r][o];
#pragma unroll
  for (int off = 1; off < G; off <<= 1) v += __shfl_xor(v, off, 64);
  const int c = o / MR, m = o % MR;
  if (part == 0 && m < M && n0 + c < N) P.out[(int64_t)m * P.ldc + n0 + c] = dense_finish(P, m, n0 + c, v);
}

// dX[m][k] = gate(sum_n dY[m][n] W[n][k]): a block owns 64 consecutive k (one per lane), its 16 waves split N (up to 32
// W loads in flight per lane); dY is staged in LDS as [n][MR] (broadcast reads), the waves are combined in a fixed order
// (wave q + wave q + 8, then the 8 pair sums in order: an 8-wave combine buffer, so 16 rows fit N <= 512 in 64 KB).
template <int MR>
__global__ __launch_bounds__(1024) void skinny_dgrad_kernel(const float* __restrict__ dY, int M, int N,
                                                            const float* __restrict__ W, int K, DenseEpiArgs P,
                                                            const int* skip) {
  if (skip && *skip == 0) return;
  constexpr int NW = 16, U = 32;  // (a wave's whole n range in one batch of loads when N <= 512)
  extern __shared__ __attribute__((aligned(16))) float dsm[];  // [N][MR] then [NW / 2][MR][64]
  float* dys = dsm;
  float* red = dsm + (int64_t)N * MR;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  for (int i0 = 0; i0 < N * MR; i0 += 4 * 64 * NW) {  // 4 clamped loads in flight per thread, zeroed after
    float v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int i = min(i0 + u * 64 * NW + tid, N * MR - 1), n = i / MR, m = i % MR;
      v[u] = dY[(int64_t)min(m, M - 1) * N + n];
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int i = i0 + u * 64 * NW + tid;
      if (i < N * MR) dys[i] = i % MR < M ? v[u] : 0.f;
    }
  }
  __syncthreads();
  const int k = blockIdx.x * 64 + lane;
  const int nq = (N + NW - 1) / NW, nb = wave * nq, ne = min(N, nb + nq);
  float acc[MR];
#pragma unroll
  for (int m = 0; m < MR; ++m) acc[m] = 0.f;
  if (k < K) {
    for (int n0 = nb; n0 < ne; n0 += U) {
      float w[U];
#pragma unroll
      for (int u = 0; u < U; ++u) w[u] = W[(int64_t)min(n0 + u, ne - 1) * K + k];  // (clamped: see skinny_fwd)
#pragma unroll
      for (int u = 0; u < U; ++u) {
        if (n0 + u >= ne) break;
#pragma unroll
        for (int m4 = 0; m4 < MR; m4 += 4) {
          const f32x4 d = *reinterpret_cast<const f32x4*>(dys + (n0 + u) * MR + m4);
#pragma unroll
          for (int e = 0; e < 4; ++e) acc[m4 + e] = fmaf(d[e], w[u], acc[m4 + e]);
        }
      }
    }
  }
  if (wave >= NW / 2) {
#pragma unroll
    for (int m = 0; m < MR; ++m) red[((wave - NW / 2) * MR + m) * 64 + lane] = acc[m];
  }
  __syncthreads();
  if (wave < NW / 2) {
#pragma unroll
    for (int m = 0; m < MR; ++m) red[(wave * MR + m) * 64 + lane] += acc[m];
  }
  __syncthreads();
  if (wave == 0 && k < K) {
    for (int m = 0; m < M; ++m) {
      float v = 0.f;
#pragma unroll
      for (int q = 0; q < NW / 2; ++q) v += red[(q * MR + m) * 64 + lane];
      P.out[(int64_t)m * P.ldc + k] = dense_finish(P, m, k, v);
    }
  }
}

// dW[n][k] = sum_m dY[m][n] X[m][k] (written), db[n] = sum_m dY[m][n]: a thread owns 4 columns n x one float4 of k.
__global__ __launch_bounds__(256) void skinny_wgrad_kernel(const float* __restrict__ dY, int M, int N,
                                                           const float* __restrict__ X, int K, float* __restrict__ dW,
                                                           float* __restrict__ db, const int* skip) {
  if (skip && *skip == 0) return;
  const int k4 = blockIdx.x * 256 + threadIdx.x, n0 = blockIdx.y * 4;
  if (db && blockIdx.x == 0 && threadIdx.x < 4 && n0 + (int)threadIdx.x < N) {
    float s = 0.f;
    for (int m = 0; m < M; ++m) s += dY[(int64_t)m * N + n0 + threadIdx.x];
    db[n0 + threadIdx.x] = s;
  }
  if (k4 >= K / 4) return;
  f32x4 acc[4];
#pragma unroll
  for (int c = 0; c < 4; ++c) acc[c] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int m = 0; m < M; ++m) {
    const f32x4 x = *reinterpret_cast<const f32x4*>(X + (int64_t)m * K + 4 * k4);
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const float d = n0 + c < N ? dY[(int64_t)m * N + n0 + c] : 0.f;
#pragma unroll
      for (int e = 0; e < 4; ++e) acc[c][e] = fmaf(d, x[e], acc[c][e]);
    }
  }
#pragma unroll
  for (int c = 0; c < 4; ++c)
    if (n0 + c < N) *reinterpret_cast<f32x4*>(dW + (int64_t)(n0 + c) * K + 4 * k4) = acc[c];
}

int dense_fwd(const float* X, int M, int K, const float* W, const float* b, int N, float* Y, const DenseAct& act,
              float* scratch, int64_t scratch_floats, hipStream_t st, int max_splits) {
  using C = T64x64;
  DenseEpiArgs pe{Y, N, b, act.relu, act.drop, act.h1, act.thr, act.dscale, act.row0, nullptr, 1.f};
  if (skinny_ok(M, K)) {
    const dim3 grid((unsigned)cdiv(N, 4));
    if (M <= 8) VAD_KLAUNCH(skinny_fwd_kernel<8>, grid, dim3(512), 0, st, X, M, K, W, N, pe);
    else VAD_KLAUNCH(skinny_fwd_kernel<16>, grid, dim3(512), 0, st, X, M, K, W, N, pe);
    VAD_LAUNCH_CHECK();
    return 0;
  }
  DenseKC<C::BM>::Params pa{X, K, M, K};
  DenseKC<C::BN>::Params pb{W, K, N, K};
  const int tiles = (int)(cdiv(M, C::BM) * cdiv(N, C::BN));
  int splits = (int)std::min<int64_t>(cdiv(256, tiles), cdiv(K, 4 * BK));
  if (max_splits > 0) splits = std::min(splits, max_splits);
  while (splits > 1 && (int64_t)splits * M * N > scratch_floats) splits /= 2;
  if (splits <= 1) return launch_gemm<C, DenseKC, DenseKC, EpiDense>(pa, pb, pe, M, N, K, 1, nullptr, st);
  EpiPartial::Params pp{scratch, N};
  int used = 1;
  VAD_TRY((launch_gemm<C, DenseKC, DenseKC, EpiPartial>(pa, pb, pp, M, N, K, splits, nullptr, st, &used)));
  const int64_t total = (int64_t)M * N;
  hipLaunchKernelGGL(dense_splitk_reduce_kernel, dim3((unsigned)std::min<int64_t>(cdiv(total, 256), 1024)), dim3(256),
                     0, st, scratch, used, M, N, pe, nullptr);
  VAD_LAUNCH_CHECK();
  return 0;
}

int dense_fwd_splitk(const float* X, int M, int K, const float* W, int N, float* scratch, int64_t scratch_floats,
                     int* nsplit, hipStream_t st) {
  using C = T64x64;
  DenseKC<C::BM>::Params pa{X, K, M, K};
  DenseKC<C::BN>::Params pb{W, K, N, K};
  const int tiles = (int)(cdiv(M, C::BM) * cdiv(N, C::BN));
  int splits = (int)std::max<int64_t>(1, std::min<int64_t>(cdiv(256, tiles), cdiv(K, 4 * BK)));
  while (splits > 1 && (int64_t)splits * M * N > scratch_floats) splits /= 2;
  VAD_CHECK((int64_t)M * N <= scratch_floats, "dense_fwd_splitk: scratch too small");
  EpiPartial::Params pp{scratch, N};
  return launch_gemm<C, DenseKC, DenseKC, EpiPartial>(pa, pb, pp, M, N, K, splits, nullptr, st, nsplit);
}

int dense_dgrad(const float* dY, int M, int N, const float* W, int K, float* dX, const float* gate, float gscale,
                const int* skip, hipStream_t st, int gate_rows, float* scratch, int64_t scratch_floats) {
  // dX[m][k] = sum_n dY[m][n] W[n][k]: A = dY (KC over n), B(row k, red n) = W[n][k] (KM, ld K)
  using C = T64x64;
  DenseEpiArgs pe{dX, K, nullptr, 0, 0, 0, 0, 1.f, 0, gate, gscale, gate_rows};
  if (skinny_ok(M, N) && (int64_t)(N + 512) * (M <= 8 ? 8 : 16) * 4 <= 65536) {  // dY + combine buffer in LDS
    const dim3 grid((unsigned)cdiv(K, 64));
    if (M <= 8)
      VAD_KLAUNCH(skinny_dgrad_kernel<8>, grid, dim3(1024), sizeof(float) * (N * 8 + 8 * 8 * 64), st, dY, M, N,
                         W, K, pe, skip);
    else
      VAD_KLAUNCH(skinny_dgrad_kernel<16>, grid, dim3(1024), sizeof(float) * (N * 16 + 8 * 16 * 64), st, dY, M,
                         N, W, K, pe, skip);
    VAD_LAUNCH_CHECK();
    return 0;
  }
  DenseKC<C::BM>::Params pa{dY, N, M, N};
  VAD_CHECK(gather_fits((int64_t)N * K), "dense gather: operand over 2 GB");
  DenseKM<C::BN>::Params pb{W, K, K, N, -1};
  // few output tiles and a long reduction (e.g. cad1's Linear(64, 2048) input gradient: one tile, N = 2048): split-K
  // slabs in scratch when the caller gives one, summed in order with the gate by dense_splitk_reduce
  const int64_t tiles = cdiv(M, C::BM) * cdiv(K, C::BN);
  if (scratch && tiles < 64 && N >= 8 * BK) {
    int splits = (int)std::min<int64_t>(cdiv(256, tiles), N / (4 * BK));
    while (splits > 1 && (int64_t)splits * M * K > scratch_floats) splits /= 2;
    if (splits > 1) {
      int used = 1;
      EpiPartial::Params pp{scratch, K};
      VAD_TRY((launch_gemm<C, DenseKC, DenseKM, EpiPartial>(pa, pb, pp, M, K, N, splits, skip, st, &used)));
      const int64_t total = (int64_t)M * K;
      hipLaunchKernelGGL(dense_splitk_reduce_kernel, dim3((unsigned)std::min<int64_t>(cdiv(total, 256), 1024)),
                         dim3(256), 0, st, scratch, used, M, K, pe, skip);
      VAD_LAUNCH_CHECK();
      return 0;
    }
  }
  return launch_gemm<C, DenseKC, DenseKM, EpiDense>(pa, pb, pe, M, K, N, 1, skip, st);
}

int dense_wgrad(const float* dY, int M, int N, const float* X, int K, float* dW, float* db, float* scratch,
                int64_t scratch_floats, const int* skip, hipStream_t st, int target_blocks) {
  // GEMM rows = out feature n, cols = in feature k (+ ones column for the bias), reduction over m
  using C = T64x64;
  if (skinny_ok(M, K)) {
    hipLaunchKernelGGL(skinny_wgrad_kernel, dim3((unsigned)cdiv(K / 4, 256), (unsigned)cdiv(N, 4)), dim3(256), 0, st, dY,
                       M, N, X, K, dW, db, skip);
    VAD_LAUNCH_CHECK();
    return 0;
  }
  const int GN = K + 1;
  VAD_CHECK(gather_fits((int64_t)M * N) && gather_fits((int64_t)M * K), "dense gather: operand over 2 GB");
  DenseKM<C::BM>::Params pa{dY, N, N, M, -1};
  DenseKM<C::BN>::Params pb{X, K, K, M, K};
  const int tiles = (int)(cdiv(N, C::BM) * cdiv(GN, C::BN));
  int splits = (int)std::min<int64_t>(std::max<int64_t>(1, cdiv(target_blocks, tiles)), cdiv(M, 4 * BK));
  while (splits > 1 && (int64_t)splits * N * GN > scratch_floats) splits /= 2;
  VAD_CHECK((int64_t)N * GN <= scratch_floats, "dense_wgrad: scratch too small");
  EpiPartial::Params pp{scratch, GN};
  int used = 1;
  VAD_TRY((launch_gemm<C, DenseKM, DenseKM, EpiPartial>(pa, pb, pp, N, GN, M, splits, skip, st, &used)));
  const int64_t total = (int64_t)N * GN;
  hipLaunchKernelGGL(dense_wgrad_reduce_kernel, dim3((unsigned)std::min<int64_t>(cdiv(total, 256), 2048)), dim3(256),
                     0, st, scratch, used, N, K, dW, db, skip);
  VAD_LAUNCH_CHECK();
  return 0;
}

// =====================================================================================================
// Conv2d(kernel 4, stride 2, padding 1) and ConvTranspose2d(4, 2, 1) as implicit GEMMs over NHWC frames (cad1's
// VideoAutoEncoder, causal_anomaly_detection1.py:129-188): the im2col / col2im columns are never written.
//   conv4_fwd   out[p][n] = sum_{tap, c} src[2a - 1 + ky][2b - 1 + kx][c] wk[n][tap C + c] (+ bias): the 16-tap
//               gather (Conv2d forward; ConvTranspose2d input gradient with src = dY)
//   conv4_cls   the transposed direction, one GEMM per output parity class (py, px): rows 2a + py take ky in {1, 3}
//               (py = 0: source rows a, a - 1) or {0, 2} (py = 1: source rows a + 1, a), 2 x 2 taps scattered to
//               (2a + py, 2b + px) (+ bias) (Conv2d input gradient with src = dY; ConvTranspose2d forward)
//   conv4_wgrad the correlation sum over A's pixels p of A[p][r] src[2a - 1 + ky][2b - 1 + kx][c] into split-K slabs
//               [S][R][16 C] (Conv2d: A = dY, src = X; ConvTranspose2d: A = X, src = dY), summed by
//               conv4_wgrad_reduce into torch's [R][C][4][4] (Conv2d [Co][Ci], ConvTranspose2d [Ci][Co])
// =====================================================================================================
__global__ __launch_bounds__(256) void conv4_prep_kernel(const float* __restrict__ w, int D0, int D1,
                                                         float* __restrict__ wk, float* __restrict__ wc) {
  const int64_t total = (int64_t)D0 * D1 * 16;
  for (int64_t i = blockIdx.x * 256ll + threadIdx.x; i < total; i += (int64_t)gridDim.x * 256) {
    const int tap = (int)(i % 16), d1 = (int)((i / 16) % D1);
    const int64_t d0 = i / (16 * D1);
    const float v = w[i];
    if (wk) wk[d0 * 16 * D1 + tap * D1 + d1] = v;
    if (wc) {
      const int ky = tap / 4, kx = tap % 4;
      const int py = (ky & 1) ? 0 : 1, px = (kx & 1) ? 0 : 1;  // (odd ky: class row 0)
      const int r = ky >> 1, q = kx >> 1;                      // index among the class's 2 x 2 taps
      wc[((int64_t)(2 * py + px) * D1 + d1) * 4 * D0 + (2 * r + q) * D0 + d0] = v;
    }
  }
}

int conv4_prep(const float* w, int D0, int D1, float* wk, float* wc, hipStream_t st) {
  const int64_t total = (int64_t)D0 * D1 * 16;
  hipLaunchKernelGGL(conv4_prep_kernel, dim3((unsigned)std::min<int64_t>(cdiv(total, 256), 1024)), dim3(256), 0, st, w,
                     D0, D1, wk, wc);
  VAD_LAUNCH_CHECK();
  return 0;
}

// split-K when the tile grid leaves most CUs idle (the decoder's 4x4 / 8x8 frames): slabs [S][M][N] in scratch, summed
// in order (+ bias) by dense_splitk_reduce / conv4_cls_reduce
// knob "conv4_split_tiles": implicit-GEMM convs with fewer 64 x 64 output tiles than this split K (slabs + a reduce)
int g_conv4_split_tiles = 512;
static int conv4_splits(int M, int N, int K, int64_t scratch_floats) {
  const int64_t tiles = cdiv(M, 64) * cdiv(N, 64);
  if (tiles >= g_conv4_split_tiles || scratch_floats <= 0) return 1;
  int s = (int)std::min<int64_t>(cdiv(1024, tiles), K / (2 * BK));
  while (s > 1 && (int64_t)s * M * N > scratch_floats) s /= 2;
  return std::max(1, s);
}

int conv4_fwd(const float* src, int NF, int H, int W, int C, const float* wk, const float* bias, int N, float* out,
              hipStream_t st, float* scratch, int64_t scratch_floats) {
  VAD_CHECK(C % 32 == 0 && H % 2 == 0 && W % 2 == 0 && N >= 1, "conv4_fwd: C % 32 == 0, even frames");
  const int OH = H / 2, OW = W / 2;
  const ConvGeom g{NF, OH, OW, 2, 2, H, W, C};
  TapTable taps;
  taps.ntaps = 16;
  for (int k = 0; k < 16; ++k) {
    taps.dh[k] = (int8_t)(k / 4 - 1);
    taps.dw[k] = (int8_t)(k % 4 - 1);
  }
  const int M = NF * OH * OW, K = 16 * C;
  const DenseEpiArgs pe{out, N, bias, 0, 0, 0, 0, 1.f, 0, nullptr, 1.f};
  const int splits = conv4_splits(M, N, K, scratch_floats);
  if (splits > 1) {
    int used = 1;
    VAD_CHECK(gather_fits((int64_t)g.imgs * g.SH * g.SW * g.C), "conv gather: source over 2 GB");
    typename ConvGatherKC<64>::Params pa{src, g, taps, nullptr, nullptr};
    typename DenseKC<64>::Params pb{wk, K, N, K};
    const EpiPartial::Params pp{scratch, N};
    VAD_TRY((launch_gemm<T64x64, ConvGatherKC, DenseKC, EpiPartial>(pa, pb, pp, M, N, K, splits, nullptr, st, &used)));
    const int64_t total = (int64_t)M * N;
    hipLaunchKernelGGL(dense_splitk_reduce_kernel, dim3((unsigned)std::min<int64_t>(cdiv(total, 256), 1024)),
                       dim3(256), 0, st, scratch, used, M, N, pe, nullptr);
    VAD_LAUNCH_CHECK();
    return 0;
  }
  return with_tile(pick_fwd_tile(M, N), [&](auto cfg) -> int {
    using Cf = decltype(cfg);
    VAD_CHECK(gather_fits((int64_t)g.imgs * g.SH * g.SW * g.C), "conv gather: source over 2 GB");
    typename ConvGatherKC<Cf::BM>::Params pa{src, g, taps, nullptr, nullptr};
    typename DenseKC<Cf::BN>::Params pb{wk, K, N, K};
    return launch_gemm<Cf, ConvGatherKC, DenseKC, EpiDense>(pa, pb, pe, M, N, K, 1, nullptr, st);
  });
}

struct EpiConv3DgradCls {  // EpiConv3Dgrad for the class-batched GEMM: class = blockIdx.z, its own grid
  static constexpr int SCRATCH = 0;
  struct Params {
    float* dst; int imgs; int GD[8], GA[8], GB[8]; int DD, DH, DW, C; const float* bias;
    const float* gate;  // nullable, dst's layout: dst = 0 where !(gate > 0) (the producing ReLU's backward, fused)
    int rev;            // blockIdx.z = 7 - class (the heaviest classes dispatched first); the tables are in z order
  };
  template <class Cfg>
  static __device__ void apply(const Params& P, f32x16 (&acc)[Cfg::TM][Cfg::TN], int m0, int n0, int wm, int wn,
                               int lane, int, int N, float*) {
    const int z = blockIdx.z, cls = P.rev ? 7 - z : z, pd = (cls >> 2) & 1, ph = (cls >> 1) & 1, pw = cls & 1;
    const int GD = P.GD[z], GA = P.GA[z], GB = P.GB[z], per = GD * GA * GB;
    if (per == 0) return;
    // a lane's 16 rows come in 4 runs of 4 consecutive rows (acc_row): the first row of a run is decomposed into
    // (img, a, b, c) by division, the next three by a carrying +1 (the divisions by the class grid were most of the
    // kernel's VALU work: 38 VALU per MFMA)
#pragma unroll
    for (int i = 0; i < Cfg::TM; ++i)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int row0 = m0 + acc_row<Cfg>(wm, i, 4 * q, lane);
        int img = row0 / per;
        const int rem = row0 - img * per;
        int a = rem / (GA * GB);
        const int r2 = rem - a * GA * GB;
        int b = r2 / GB, c = r2 - b * GB;
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          if (u > 0) {  // row0 + u: c + 1 with carries into b, a, img
            ++c;
            const bool cb = c == GB;
            c = cb ? 0 : c;
            b += cb;
            const bool ca = b == GA;
            b = ca ? 0 : b;
            a += ca;
            const bool ci = a == GD;
            a = ci ? 0 : a;
            img += ci;
          }
          if (img >= P.imgs) continue;
          const int64_t base = ((((int64_t)img * P.DD + 2 * a + pd) * P.DH + 2 * b + ph) * P.DW + 2 * c + pw) * P.C;
          const int r = 4 * q + u;
#pragma unroll
          for (int j = 0; j < Cfg::TN; ++j) {
            const int col = n0 + acc_col<Cfg>(wn, j, lane);
            if (col < N) {
              const float v = acc[i][j][r] + (P.bias ? P.bias[col] : 0.f);
              P.dst[base + col] = (P.gate && !(P.gate[base + col] > 0.f)) ? 0.f : v;
            }
          }
        }
      }
  }
};

// out[img][2a + py][2b + px][n] = bias[n] + sum over the slabs of part[s][(img SH + a) SW + b][n]
__global__ __launch_bounds__(256) void conv4_cls_reduce_kernel(const float* __restrict__ part, int S, int M, int SH,
                                                               int SW, int N, int py, int px,
                                                               const float* __restrict__ bias, float* __restrict__ out) {
  const int64_t total = (int64_t)M * N;
  for (int64_t i = blockIdx.x * 256ll + threadIdx.x; i < total; i += (int64_t)gridDim.x * 256) {
    const float v = slab_sum(part + i, S, total);
    const int n = (int)(i % N);
    const int64_t m = i / N;
    const int b = (int)(m % SW);
    const int64_t ia = m / SW;
    const int a = (int)(ia % SH);
    const int64_t img = ia / SH;
    out[((img * 2 * SH + 2 * a + py) * 2 * SW + 2 * b + px) * N + n] = v + (bias ? bias[n] : 0.f);
  }
}

// knob "conv4_cls_batch_min": the four parity classes go to one batched launch (whole K per block, bias in the
// epilogue) from this many 64 x 64 class tiles up; below it, per-class split-K launches with a reduce each
int g_conv4_cls_batch_min = 0;  // (sweep at cad1: 512 1.845-1.850, 128 1.813-1.817, 0 1.785-1.795 ms)
int conv4_cls(const float* src, int NF, int SH, int SW, int C, const float* wc, const float* bias, int N, float* out,
              hipStream_t st, float* scratch, int64_t scratch_floats) {
  VAD_CHECK(C % 32 == 0 && N >= 1, "conv4_cls: C % 32 == 0");
  const int Mc = NF * SH * SW;
  if (cdiv(Mc, 64) * cdiv(N, 64) * 4 >= g_conv4_cls_batch_min || scratch_floats <= 0) {
    // the four classes in one launch (blockIdx.z = class, the 3-D class-batched GEMM with a depth of 1)
    Conv3ClsGeom g{};
    g.imgs = NF; g.SD = 1; g.SH = SH; g.SW = SW; g.C = C;
    EpiConv3DgradCls::Params pe{};
    pe.dst = out; pe.imgs = NF; pe.DD = 1; pe.DH = 2 * SH; pe.DW = 2 * SW; pe.C = N; pe.bias = bias;
    for (int cls = 0; cls < 4; ++cls) {
      const int py = cls >> 1, px = cls & 1;
      g.GD[cls] = pe.GD[cls] = 1;
      g.GA[cls] = pe.GA[cls] = SH;
      g.GB[cls] = pe.GB[cls] = SW;
      TapTable3& taps = g.taps[cls];
      taps.ntaps = 4;
      for (int r = 0; r < 2; ++r)
        for (int q = 0; q < 2; ++q) {
          taps.dd[2 * r + q] = 0;
          taps.dh[2 * r + q] = (int8_t)(py == 0 ? -r : 1 - r);
          taps.dw[2 * r + q] = (int8_t)(px == 0 ? -q : 1 - q);
        }
    }
    const int K = 4 * C;
    return with_tile(pick_dgrad_tile(Mc, N), [&](auto cfg) -> int {
      using Cf = decltype(cfg);
      VAD_CHECK(gather_fits((int64_t)g.imgs * g.SD * g.SH * g.SW * g.C), "conv gather: source over 2 GB");
      typename ConvGather3ClsKC<Cf::BM>::Params pa{src, g};
      typename DenseKCz<Cf::BN>::Params pb{wc, {}, {}, N};
      for (int c = 0; c < 4; ++c) {
        pb.off[c] = (int64_t)c * N * K;
        pb.kdim[c] = K;
      }
      const dim3 grid((unsigned)cdiv(Mc, Cf::BM), (unsigned)cdiv(N, Cf::BN), 4u);
      VAD_KLAUNCH((gemm_kernel<Cf, ConvGather3ClsKC<Cf::BM>, DenseKCz<Cf::BN>, EpiConv3DgradCls>), grid, dim3(256), 0,
                  st, pa, pb, pe, Mc, N, K, -1, nullptr);
      VAD_LAUNCH_CHECK();
      return 0;
    });
  }
  for (int cls = 0; cls < 4; ++cls) {
    const int py = cls >> 1, px = cls & 1;
    const ConvGeom g{NF, SH, SW, 1, 1, SH, SW, C};
    TapTable taps;
    taps.ntaps = 4;
    for (int r = 0; r < 2; ++r)
      for (int q = 0; q < 2; ++q) {
        taps.dh[2 * r + q] = (int8_t)(py == 0 ? -r : 1 - r);
        taps.dw[2 * r + q] = (int8_t)(px == 0 ? -q : 1 - q);
      }
    const int M = NF * SH * SW, K = 4 * C;
    const int splits = conv4_splits(M, N, K, scratch_floats);
    if (splits > 1) {
      int used = 1;
      VAD_CHECK(gather_fits((int64_t)g.imgs * g.SH * g.SW * g.C), "conv gather: source over 2 GB");
      typename ConvGatherKC<64>::Params pa{src, g, taps, nullptr, nullptr};
      typename DenseKC<64>::Params pb{wc + (int64_t)cls * N * 4 * C, K, N, K};
      const EpiPartial::Params pp{scratch, N};
      VAD_TRY((launch_gemm<T64x64, ConvGatherKC, DenseKC, EpiPartial>(pa, pb, pp, M, N, K, splits, nullptr, st,
                                                                     &used)));
      const int64_t total = (int64_t)M * N;
      hipLaunchKernelGGL(conv4_cls_reduce_kernel, dim3((unsigned)std::min<int64_t>(cdiv(total, 256), 1024)),
                         dim3(256), 0, st, scratch, used, M, SH, SW, N, py, px, bias, out);
      VAD_LAUNCH_CHECK();
      continue;
    }
    const EpiConvDgrad::Params pe{out, SH, SW, 2, py, 2, px, 2 * SH, 2 * SW, N, bias};
    VAD_TRY(dgrad_launch(g, taps, src, wc + (int64_t)cls * N * 4 * C, N, pe, st));
  }
  return 0;
}

int conv4_wgrad(const float* A, int R, const float* src, int C, int NF, int AH, int AW, float* part, int* nsplit,
                int64_t part_cap, int target_blocks, hipStream_t st) {
  VAD_CHECK(C % 4 == 0 && R % 4 == 0, "conv4_wgrad: channel counts % 4 == 0");
  const int M = R, N = 16 * C, K = NF * AH * AW;
  VAD_CHECK((int64_t)M * N <= part_cap, "conv4_wgrad: slab too small");
  return with_tile(pick_wgrad_tile(M, N), [&](auto cfg) -> int {
    using Cf = decltype(cfg);
    const int tiles = (int)(cdiv(M, Cf::BM) * cdiv(N, Cf::BN));
    int splits = (int)std::max<int64_t>(1, std::min<int64_t>(cdiv(target_blocks, tiles), cdiv(K, 16 * BK)));
    while ((int64_t)splits * M * N > part_cap && splits > 1) splits /= 2;
    VAD_CHECK(gather_fits((int64_t)K * R), "dense gather: operand over 2 GB");
    typename DenseKM<Cf::BM>::Params pa{A, R, R, K, -1};
    VAD_CHECK(gather_fits((int64_t)NF * 2 * AH * 2 * AW * C), "conv patch: source over 2 GB");
    typename ConvPatchKM<Cf::BN>::Params pb{src, NF, AH, AW, 2, 1, 2 * AH, 2 * AW, C, 4, N, nullptr, nullptr};
    const EpiPartial::Params pe{part, N};
    return launch_gemm<Cf, DenseKM, ConvPatchKM, EpiPartial>(pa, pb, pe, M, N, K, splits, nullptr, st, nsplit);
  });
}

// dW[r][c][tap] = sum over the S slabs, in order, of part[s][r][tap C + c] (NT taps: 16 for the 4x4 convs, 27 for
// the 3-D ones)
// (slab rows of ld floats: the NT C weight columns, then with db the bias column NT C)
__global__ __launch_bounds__(256) void conv4_wgrad_reduce_kernel(const float* __restrict__ part, int S, int R, int C,
                                                                 int NT, int ld, float* __restrict__ dW,
                                                                 float* __restrict__ db) {
  const int W1 = NT * C + (db ? 1 : 0);
  const int64_t total = (int64_t)R * W1, slab = (int64_t)R * ld;
  for (int64_t i = blockIdx.x * 256ll + threadIdx.x; i < total; i += (int64_t)gridDim.x * 256) {
    const int64_t r = i / W1;
    const int col = (int)(i - r * W1);
    const float s = slab_sum(part + r * ld + col, S, slab);
    if (col == NT * C) {
      db[r] = s;
    } else {
      const int c = col % C, tap = col / C;
      dW[(r * C + c) * NT + tap] = s;
    }
  }
}

// the same for many slabs: 64 consecutive entries x 4 slab lanes per block (lane l adds slabs l, l + 4, ... in order
// with 8 loads in flight, coalesced across the 64 entries), the 4 lane sums combined in a fixed order
__global__ __launch_bounds__(256) void conv4_wgrad_reduce_small_kernel(const float* __restrict__ part, int S, int R,
                                                                       int C, int NT, int ld, float* __restrict__ dW,
                                                                       float* __restrict__ db) {
  __shared__ float red[4][64];
  const int W1 = NT * C + (db ? 1 : 0);
  const int64_t total = (int64_t)R * W1, slab = (int64_t)R * ld;
  const int e = threadIdx.x & 63, sl = threadIdx.x >> 6;
  const int64_t i = (int64_t)blockIdx.x * 64 + e;
  const int64_t row = i / W1, col = i - row * W1, pi = row * ld + col;
  float v = 0.f;
  if (i < total) {
    const int n = S > sl ? (S - sl + 3) / 4 : 0;
    for (int k0 = 0; k0 < n; k0 += 8) {
      float u[8];
#pragma unroll
      for (int q = 0; q < 8; ++q) u[q] = part[(int64_t)(sl + 4 * min(k0 + q, n - 1)) * slab + pi];
#pragma unroll
      for (int q = 0; q < 8; ++q)
        if (k0 + q < n) v += u[q];
    }
  }
  red[sl][e] = v;
  __syncthreads();
  if (sl == 0 && i < total) {
    const float t = (red[0][e] + red[1][e]) + (red[2][e] + red[3][e]);
    if (col == NT * C) {
      db[row] = t;
    } else {
      const int c = (int)(col % C), tap = (int)(col / C);
      dW[(row * C + c) * NT + tap] = t;
    }
  }
}

// slabs [S][R][ld] -> dW (torch [R][C][taps]) and, with db, the bias column NT C of each row
static int taps_wgrad_reduce(const float* part, int S, int R, int C, int NT, float* dW, hipStream_t st, int ld = 0,
                             float* db = nullptr) {
  if (ld <= 0) ld = NT * C;
  const int64_t total = (int64_t)R * (NT * C + (db ? 1 : 0));
  if (S >= 16) {
    hipLaunchKernelGGL(conv4_wgrad_reduce_small_kernel, dim3((unsigned)cdiv(total, 64)), dim3(256), 0, st, part, S, R, C,
                       NT, ld, dW, db);
    VAD_LAUNCH_CHECK();
    return 0;
  }
  hipLaunchKernelGGL(conv4_wgrad_reduce_kernel, dim3((unsigned)std::min<int64_t>(cdiv(total, 256), 2048)), dim3(256), 0,
                     st, part, S, R, C, NT, ld, dW, db);
  VAD_LAUNCH_CHECK();
  return 0;
}

int conv4_wgrad_reduce(const float* part, int S, int R, int C, float* dW, hipStream_t st) {
  return taps_wgrad_reduce(part, S, R, C, 16, dW, st);
}

// ---------------------------------------------------------------- the single-channel ends (cad1:131, cad1:185)
// conv4_c1_fwd  out[p][n] = sum_tap src[2a - 1 + ky][2b - 1 + kx] w[n][tap] (+ bias[n]), 1-channel NHWC source, 32
//               outputs per pixel on the VALU (Conv2d(1, 32) forward; ConvTranspose2d(32, 1) input gradient with
//               src = dY, w = the [32][1][4][4] weight)
// conv4_c1_tfwd out[2a + py][2b + px] = bias + sum over the class taps and the 32 source channels (ConvTranspose2d(32,
//               1) forward)
// conv4_c1_wgrad slab[block][r][tap] = sum over the block's pixels p of A[p][r] src[2a - 1 + ky][2b - 1 + kx] (r < 32;
//               Conv2d(1, 32): A = dY; ConvTranspose2d(32, 1): A = X, src = dY)
__global__ __launch_bounds__(256) void conv4_c1_fwd_kernel(const float* __restrict__ src, int NF, int H, int W,
                                                           const float* __restrict__ w, const float* __restrict__ bias,
                                                           float* __restrict__ out) {
  __shared__ __attribute__((aligned(16))) float ws[16][32];  // [tap][n]
  __shared__ __attribute__((aligned(16))) float os[256 * 33];  // the block's 256 output rows, written back coalesced
  for (int i = threadIdx.x; i < 512; i += 256) ws[i % 16][i / 16] = w[i];
  const int OH = H / 2, OW = W / 2;
  const int64_t total = (int64_t)NF * OH * OW;
  for (int64_t p0 = blockIdx.x * 256ll; p0 < total; p0 += (int64_t)gridDim.x * 256) {
    __syncthreads();
    const int64_t p = p0 + threadIdx.x;
    if (p < total) {
      const int ox = (int)(p % OW);
      const int64_t r = p / OW;
      const int oy = (int)(r % OH);
      const float* img = src + (r / OH) * H * W;
      float x[16];
#pragma unroll
      for (int t = 0; t < 16; ++t) {
        const int iy = 2 * oy - 1 + t / 4, ix = 2 * ox - 1 + t % 4;
        x[t] = (iy >= 0 && iy < H && ix >= 0 && ix < W) ? img[iy * W + ix] : 0.f;
      }
#pragma unroll
      for (int n4 = 0; n4 < 8; ++n4) {
        f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int t = 0; t < 16; ++t) {
          const f32x4 wv = *reinterpret_cast<const f32x4*>(&ws[t][4 * n4]);
#pragma unroll
          for (int e = 0; e < 4; ++e) acc[e] = fmaf(x[t], wv[e], acc[e]);
        }
#pragma unroll
        for (int e = 0; e < 4; ++e) os[threadIdx.x * 33 + 4 * n4 + e] = acc[e] + (bias ? bias[4 * n4 + e] : 0.f);
      }
    }
    __syncthreads();
    const int64_t nrow = min((int64_t)256, total - p0);
    for (int i = threadIdx.x; i < nrow * 8; i += 256) {  // 8 float4 per output row, consecutive lanes -> consecutive
      const int row = i >> 3, c4 = (i & 7) * 4;
      const f32x4 v = {os[row * 33 + c4], os[row * 33 + c4 + 1], os[row * 33 + c4 + 2], os[row * 33 + c4 + 3]};
      *reinterpret_cast<f32x4*>(out + (p0 + row) * 32 + c4) = v;
    }
  }
}

__global__ __launch_bounds__(256) void conv4_c1_tfwd_kernel(const float* __restrict__ src, int NF, int SH, int SW,
                                                            const float* __restrict__ w, const float* __restrict__ bias,
                                                            float* __restrict__ out) {
  __shared__ __attribute__((aligned(16))) float ws[16][32];  // [tap][source channel]
  for (int i = threadIdx.x; i < 512; i += 256) ws[i % 16][i / 16] = w[i];
  __syncthreads();
  const int OH = 2 * SH, OW = 2 * SW;
  const int64_t total = (int64_t)NF * OH * OW;
  const float b0 = bias ? bias[0] : 0.f;
  for (int64_t p = blockIdx.x * 256ll + threadIdx.x; p < total; p += (int64_t)gridDim.x * 256) {
    const int ox = (int)(p % OW);
    const int64_t r = p / OW;
    const int oy = (int)(r % OH);
    const int64_t img = r / OH;
    const int py = oy & 1, px = ox & 1, a = oy >> 1, b = ox >> 1;
    float acc = 0.f;
#pragma unroll
    for (int rr = 0; rr < 2; ++rr)
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        const int sy = a + (py == 0 ? -rr : 1 - rr), sx = b + (px == 0 ? -q : 1 - q);
        if (sy < 0 || sy >= SH || sx < 0 || sx >= SW) continue;
        const int ky = py == 0 ? 1 + 2 * rr : 2 * rr, kx = px == 0 ? 1 + 2 * q : 2 * q;
        const float* xs = src + ((img * SH + sy) * SW + sx) * 32;
        const float* wt = ws[ky * 4 + kx];
#pragma unroll
        for (int c4 = 0; c4 < 8; ++c4) {
          const f32x4 xv = *reinterpret_cast<const f32x4*>(xs + 4 * c4);
          const f32x4 wv = *reinterpret_cast<const f32x4*>(wt + 4 * c4);
#pragma unroll
          for (int e = 0; e < 4; ++e) acc = fmaf(xv[e], wv[e], acc);
        }
      }
    out[p] = acc + b0;
  }
}

// conv4_c1_wgrad: a block walks tiles of 256 consecutive A pixels (256 / AW whole rows of one image); the tile's A rows
// (256 x 32) and its 1-channel source halo ((2 TR + 2) x (2 AW + 2)) in LDS, thread (channel r, tap pair) sums over the
// tile's pixels (three LDS reads, two FMAs per pixel)
constexpr int C1_TILE = 256;

// thread = 4 output channels (quad q) x 2 taps (pair p) over one wave's share of the tile's pixel rows (wave w takes
// rows w, w + 4, ...): per pixel one 16-B read of the dY quad and two halo reads feed 8 FMAs; the four waves' sums are
// combined in a fixed order at the end
__global__ __launch_bounds__(256) void conv4_c1_wgrad_kernel(const float* __restrict__ A, const float* __restrict__ src,
                                                             int NF, int AH, int AW, float* __restrict__ slab) {
  __shared__ __attribute__((aligned(16))) float as[C1_TILE][32];
  __shared__ float xs[(2 * C1_TILE / 8 + 2) * (2 * 64 + 2)];  // (AW >= 8, AW <= 64)
  __shared__ float red[4][512];
  const int H = 2 * AH, W = 2 * AW, TR = C1_TILE / AW, XW = 2 * AW + 2, XR = 2 * TR + 2;
  const int64_t ntiles = (int64_t)NF * AH / TR;
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6, q = lane & 7, p = lane >> 3;
  const int k0 = 2 * p, k1 = 2 * p + 1;
  const int o0 = (k0 / 4) * XW + k0 % 4, o1 = (k1 / 4) * XW + k1 % 4;  // tap offsets in the halo
  f32x4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
  for (int64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    const int64_t img = tile / (AH / TR);
    const int y0 = (int)(tile % (AH / TR)) * TR;  // first A row of the tile
    __syncthreads();
    const float* arow = A + ((img * AH + y0) * (int64_t)AW) * 32;
    for (int i = t; i < C1_TILE * 8; i += 256)
      *reinterpret_cast<f32x4*>(&as[i >> 3][(i & 7) * 4]) = *reinterpret_cast<const f32x4*>(arow + (int64_t)i * 4);
    const float* simg = src + img * (int64_t)H * W;
    for (int i = t; i < XR * XW; i += 256) {
      const int hy = i / XW, hx = i - hy * XW;
      const int iy = 2 * y0 - 1 + hy, ix = hx - 1;
      xs[i] = (iy >= 0 && iy < H && ix >= 0 && ix < W) ? simg[(int64_t)iy * W + ix] : 0.f;
    }
    __syncthreads();
    for (int vy = wv; vy < TR; vy += 4) {  // (pixel v = vy * AW + vx, walked without divisions)
      const float* xrow = xs + 2 * vy * XW;
#pragma unroll 4
      for (int vx = 0; vx < AW; ++vx) {
        const f32x4 a = *reinterpret_cast<const f32x4*>(&as[vy * AW + vx][4 * q]);
        const float x0 = xrow[2 * vx + o0], x1 = xrow[2 * vx + o1];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          acc0[e] = fmaf(a[e], x0, acc0[e]);
          acc1[e] = fmaf(a[e], x1, acc1[e]);
        }
      }
    }
  }
  __syncthreads();
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    red[wv][(4 * q + e) * 16 + k0] = acc0[e];
    red[wv][(4 * q + e) * 16 + k1] = acc1[e];
  }
  __syncthreads();
  for (int i = t; i < 512; i += 256)
    slab[(int64_t)blockIdx.x * 512 + i] = (red[0][i] + red[1][i]) + (red[2][i] + red[3][i]);
}

int conv4_c1_fwd(const float* src, int NF, int H, int W, const float* w, const float* bias, float* out,
                 hipStream_t st) {
  VAD_CHECK(H % 2 == 0 && W % 2 == 0, "conv4_c1_fwd: even frames");
  const int64_t total = (int64_t)NF * (H / 2) * (W / 2);
  hipLaunchKernelGGL(conv4_c1_fwd_kernel, dim3((unsigned)std::min<int64_t>(cdiv(total, 256), 4096)), dim3(256), 0, st,
                     src, NF, H, W, w, bias, out);
  VAD_LAUNCH_CHECK();
  return 0;
}

int conv4_c1_tfwd(const float* src, int NF, int SH, int SW, const float* w, const float* bias, float* out,
                  hipStream_t st) {
  const int64_t total = (int64_t)NF * 4 * SH * SW;
  hipLaunchKernelGGL(conv4_c1_tfwd_kernel, dim3((unsigned)std::min<int64_t>(cdiv(total, 256), 4096)), dim3(256), 0, st,
                     src, NF, SH, SW, w, bias, out);
  VAD_LAUNCH_CHECK();
  return 0;
}

int conv4_c1_wgrad(const float* A, const float* src, int NF, int AH, int AW, float* dW, float* slab,
                   int64_t slab_floats, hipStream_t st) {
  VAD_CHECK(AW >= 8 && AW <= 64 && C1_TILE % AW == 0 && AH % (C1_TILE / AW) == 0,
            "conv4_c1_wgrad: 256 / AW whole rows per tile");
  const int64_t ntiles = (int64_t)NF * AH * AW / C1_TILE;
  const int blocks = (int)std::max<int64_t>(1, std::min<int64_t>({ntiles, 512, slab_floats / 512}));
  hipLaunchKernelGGL(conv4_c1_wgrad_kernel, dim3((unsigned)blocks), dim3(256), 0, st, A, src, NF, AH, AW, slab);
  VAD_LAUNCH_CHECK();
  return conv4_wgrad_reduce(slab, blocks, 32, 1, dW, st);
}

// =====================================================================================================
// Conv3d(kernel 3, stride 2, padding 1) as implicit GEMMs over NDHWC volumes (a2's conv3d_2 / conv3d_3,
// avenue_training_script2.py:20-21): no im2col / col2im columns.
//   conv3s2_fwd    out[p][n] = act(sum_{tap, c} src[2a - 1 + kd][2b - 1 + kh][2c - 1 + kw][c] wk[n][tap C + c] + bias)
//   conv3s2_dgrad  the input gradient as 8 parity-class GEMMs over dY: along each dim an even input index takes k = 1
//                  (dY index = its half), an odd one k = 0 (half + 1) and k = 2 (half); scattered to (2a + pd, ...)
//   conv3s2_wgrad  split-K correlation dY x patch3(src) into slabs, summed into torch's [Co][Ci][27] layout
// Weight images (conv3s2_prep) of torch [Co][Ci][27]: wk [Co][27 Ci]; wc = the 8 class images [Ci][nt Co] back to back
// (class cls = 4 pd + 2 ph + pw, nt = its tap count 1 / 2 / 4 / 8, taps d-major over the per-dim lists).
// =====================================================================================================

__global__ __launch_bounds__(256) void conv3s2_prep_kernel(const float* __restrict__ w, int Co, int Ci,
                                                           float* __restrict__ wk, float* __restrict__ wc) {
  const int64_t total = (int64_t)Co * Ci * 27;
  for (int64_t i = blockIdx.x * 256ll + threadIdx.x; i < total; i += (int64_t)gridDim.x * 256)
    conv3s2_prep_elem(w, Co, Ci, wk, wc, i);
}

int conv3s2_prep(const float* w, int Co, int Ci, float* wk, float* wc, hipStream_t st) {
  const int64_t total = (int64_t)Co * Ci * 27;
  hipLaunchKernelGGL(conv3s2_prep_kernel, dim3((unsigned)std::min<int64_t>(cdiv(total, 256), 1024)), dim3(256), 0, st,
                     w, Co, Ci, wk, wc);
  VAD_LAUNCH_CHECK();
  return 0;
}

int g_conv3s2_fwd_blocks = 512;  // knob "conv3s2_fwd_blocks": split K until the grid reaches this many blocks
int conv3s2_fwd(const float* src, int NF, int D, int H, int W, int C, const float* wk, const float* bias, int N,
                int relu, float* out, hipStream_t st, float* scratch, int64_t scratch_floats) {
  VAD_CHECK(C % 4 == 0 && N >= 1, "conv3s2_fwd: C % 4 == 0");
  const int OD = (D - 1) / 2 + 1, OH = (H - 1) / 2 + 1, OW = (W - 1) / 2 + 1;
  ConvGeom3 g{NF, OD, OH, OW, 2, 2, 2, D, H, W, C};
  TapTable3 taps;
  taps.ntaps = 27;
  for (int t = 0; t < 27; ++t) {
    taps.dd[t] = (int8_t)(t / 9 - 1);
    taps.dh[t] = (int8_t)((t / 3) % 3 - 1);
    taps.dw[t] = (int8_t)(t % 3 - 1);
  }
  const int M = NF * OD * OH * OW, K = 27 * C;
  const DenseEpiArgs pe{out, N, bias, relu, 0, 0, 0, 1.f, 0, nullptr, 1.f};
  return with_tile(pick_fwd_tile(M, N), [&](auto cfg) -> int {
    using Cf = decltype(cfg);
    VAD_CHECK(gather_fits((int64_t)g.imgs * g.SD * g.SH * g.SW * g.C), "conv gather: source over 2 GB");
    typename ConvGather3KC<Cf::BM>::Params pa{src, g, taps};
    typename DenseKC<Cf::BN>::Params pb{wk, K, N, K};
    // (conv3d_3 at B = 32: 64 output tiles of 27 K slices each -- split K four ways, slabs summed in order by
    // dense_splitk_reduce, which applies the bias and the ReLU)
    const int tiles = (int)(cdiv(M, Cf::BM) * cdiv(N, Cf::BN));
    int splits = (int)std::min<int64_t>(cdiv(g_conv3s2_fwd_blocks, tiles), cdiv(K, 4 * BK));
    while (splits > 1 && (int64_t)splits * M * N > scratch_floats) splits /= 2;
    if (!scratch || splits <= 1) return launch_gemm<Cf, ConvGather3KC, DenseKC, EpiDense>(pa, pb, pe, M, N, K, 1, nullptr, st);
    EpiPartial::Params pp{scratch, N};
    int used = 1;
    VAD_TRY((launch_gemm<Cf, ConvGather3KC, DenseKC, EpiPartial>(pa, pb, pp, M, N, K, splits, nullptr, st, &used)));
    const int64_t total = (int64_t)M * N;
    hipLaunchKernelGGL(dense_splitk_reduce_kernel, dim3((unsigned)std::min<int64_t>(cdiv(total, 256), 1024)), dim3(256),
                       0, st, scratch, used, M, N, pe, nullptr);
    VAD_LAUNCH_CHECK();
    return 0;
  });
}

struct EpiConv3Dgrad {  // scatter the rows of a parity-class grid to the NDHWC input gradient
  static constexpr int SCRATCH = 0;
  struct Params { float* dst; int GD, GA, GB, pd, ph, pw, DD, DH, DW, C; };
  template <class Cfg>
  static __device__ void apply(const Params& P, f32x16 (&acc)[Cfg::TM][Cfg::TN], int m0, int n0, int wm, int wn,
                               int lane, int M, int N, float*) {
    const int per = P.GD * P.GA * P.GB;
#pragma unroll
    for (int i = 0; i < Cfg::TM; ++i)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = m0 + acc_row<Cfg>(wm, i, r, lane);
        if (row >= M) continue;
        const int img = row / per, rem = row - img * per;
        const int a = rem / (P.GA * P.GB), r2 = rem - a * P.GA * P.GB;
        const int b = r2 / P.GB, c = r2 - b * P.GB;
        const int64_t base =
            ((((int64_t)img * P.DD + 2 * a + P.pd) * P.DH + 2 * b + P.ph) * P.DW + 2 * c + P.pw) * P.C;
#pragma unroll
        for (int j = 0; j < Cfg::TN; ++j) {
          const int col = n0 + acc_col<Cfg>(wn, j, lane);
          if (col < N) P.dst[base + col] = acc[i][j][r];
        }
      }
  }
};

int conv3s2_dgrad(const float* dy, int NF, int Co, const float* wc, int Ci, float* dx, int D, int H, int W,
                  hipStream_t st, const float* gate) {
  VAD_CHECK(Co % 4 == 0, "conv3s2_dgrad: Co % 4 == 0");
  const int OD = (D - 1) / 2 + 1, OH = (H - 1) / 2 + 1, OW = (W - 1) / 2 + 1;
  // the 8 parity classes in one launch (blockIdx.z = 7 - class: the 8-tap class first, the 1-tap class last, so the
  // longest blocks are dispatched first; each block's K loop stops at its class's own taps x Co)
  Conv3ClsGeom g{};
  g.imgs = NF; g.SD = OD; g.SH = OH; g.SW = OW; g.C = Co;
  typename DenseKCz<64>::Params pb0{};
  EpiConv3DgradCls::Params pe{};
  pe.dst = dx; pe.imgs = NF; pe.DD = D; pe.DH = H; pe.DW = W; pe.C = Ci; pe.gate = gate; pe.rev = 1;
  int64_t off = 0;
  int Mmax = 0;
  for (int cls = 0; cls < 8; ++cls) {
    const int pd = (cls >> 2) & 1, ph = (cls >> 1) & 1, pw = cls & 1, nt = c3_nt(cls), z = 7 - cls;
    g.GD[z] = pe.GD[z] = std::max(0, (D - pd + 1) / 2);
    g.GA[z] = pe.GA[z] = std::max(0, (H - ph + 1) / 2);
    g.GB[z] = pe.GB[z] = std::max(0, (W - pw + 1) / 2);
    Mmax = std::max(Mmax, NF * g.GD[z] * g.GA[z] * g.GB[z]);
    TapTable3& taps = g.taps[z];
    taps.ntaps = nt;
    const int nh = 1 + ph, nw = 1 + pw;
    for (int t = 0; t < nt; ++t) {
      const int id = t / (nh * nw), ih = (t / nw) % nh, iw = t % nw;
      // even parity: k = 1, offset 0; odd: k = 0 -> offset +1, k = 2 -> offset 0
      taps.dd[t] = (int8_t)(pd == 0 ? 0 : (id == 0 ? 1 : 0));
      taps.dh[t] = (int8_t)(ph == 0 ? 0 : (ih == 0 ? 1 : 0));
      taps.dw[t] = (int8_t)(pw == 0 ? 0 : (iw == 0 ? 1 : 0));
    }
    pb0.off[z] = off;
    pb0.kdim[z] = nt * Co;
    off += (int64_t)nt * Ci * Co;
  }
  if (Mmax == 0) return 0;
  const int K = 8 * Co;
  return with_tile(pick_dgrad_tile(Mmax, Ci), [&](auto cfg) -> int {
    using Cf = decltype(cfg);
    VAD_CHECK(gather_fits((int64_t)g.imgs * g.SD * g.SH * g.SW * g.C), "conv gather: source over 2 GB");
    typename ConvGather3ClsKC<Cf::BM>::Params pa{dy, g};
    typename DenseKCz<Cf::BN>::Params pb{wc, {}, {}, Ci};
    for (int c = 0; c < 8; ++c) {
      pb.off[c] = pb0.off[c];
      pb.kdim[c] = pb0.kdim[c];
    }
    const dim3 grid((unsigned)cdiv(Mmax, Cf::BM), (unsigned)cdiv(Ci, Cf::BN), 8u);
    VAD_KLAUNCH((gemm_kernel<Cf, ConvGather3ClsKC<Cf::BM>, DenseKCz<Cf::BN>, EpiConv3DgradCls>), grid, dim3(256), 0, st,
                pa, pb, pe, Mmax, Ci, K, -1, nullptr);
    VAD_LAUNCH_CHECK();
    return 0;
  });
}

int conv3s2_wgrad(const float* dy, int Co, const float* src, int Ci, int NF, int D, int H, int W, float* dW,
                  float* part, int64_t part_cap, int target_blocks, hipStream_t st, float* db) {
  VAD_CHECK(Ci % 4 == 0 && Co % 4 == 0, "conv3s2_wgrad: channel counts % 4 == 0");
  const int OD = (D - 1) / 2 + 1, OH = (H - 1) / 2 + 1, OW = (W - 1) / 2 + 1;
  // (db: the bias gradient = dY's column sums, as one more GEMM column of ones beside the 27 Ci patch columns)
  const int M = Co, N = 27 * Ci + (db ? 1 : 0), K = NF * OD * OH * OW;
  VAD_CHECK((int64_t)M * N <= part_cap, "conv3s2_wgrad: slab too small");
  int used = 1;
  VAD_TRY(with_tile(pick_wgrad_tile(M, N), [&](auto cfg) -> int {
    using Cf = decltype(cfg);
    const int tiles = (int)(cdiv(M, Cf::BM) * cdiv(N, Cf::BN));
    int splits = (int)std::max<int64_t>(1, std::min<int64_t>(cdiv(target_blocks, tiles), cdiv(K, 8 * BK)));
    while ((int64_t)splits * M * N > part_cap && splits > 1) splits /= 2;
    VAD_CHECK(gather_fits((int64_t)K * Co), "dense gather: operand over 2 GB");
    typename DenseKM<Cf::BM>::Params pa{dy, Co, Co, K, -1};
    VAD_CHECK(gather_fits((int64_t)NF * D * H * W * Ci), "conv patch: source over 2 GB");
    typename ConvPatch3KM<Cf::BN>::Params pb{src, NF, OD, OH, OW, 2, 2, 2, 1, D, H, W, Ci, 27 * Ci, db ? 1 : 0};
    const EpiPartial::Params pe{part, N};
    return launch_gemm<Cf, DenseKM, ConvPatch3KM, EpiPartial>(pa, pb, pe, M, N, K, splits, nullptr, st, &used);
  }));
  return taps_wgrad_reduce(part, used, Co, Ci, 27, dW, st, N, db);
}

// db[n] = sum over the M rows of x[m][n], fixed order, two passes: block b sums the rows of its contiguous range with
// 256 / N row lanes per column (coalesced rows), lanes combined by a fixed tree -> part[b][n]; then one block adds the
// block sums in order (double).  N divides 256.
__global__ __launch_bounds__(256) void col_sum_part_kernel(const float* __restrict__ x, int64_t M, int N, int64_t rows,
                                                           double* __restrict__ part) {
  __shared__ double red[256];
  const int n = threadIdx.x % N, lane = threadIdx.x / N, lanes = 256 / N;
  const int64_t r0 = (int64_t)blockIdx.x * rows, r1 = min(M, r0 + rows);
  double s = 0.0;
#pragma unroll 4
  for (int64_t m = r0 + lane; m < r1; m += lanes) s += (double)x[m * N + n];
  red[threadIdx.x] = s;
  __syncthreads();
  for (int o = lanes / 2; o > 0; o >>= 1) {
    if (lane < o) red[threadIdx.x] += red[threadIdx.x + o * N];
    __syncthreads();
  }
  if (lane == 0) part[(int64_t)blockIdx.x * N + n] = red[n];
}
// 256 / N lanes per column each add a strided subset of the P block sums (loads independent, in flight together),
// then the same fixed tree as the first pass
__global__ __launch_bounds__(256) void col_sum_fin_kernel(const double* __restrict__ part, int P, int N,
                                                          float* __restrict__ db) {
  __shared__ double red[256];
  const int n = threadIdx.x % N, lane = threadIdx.x / N, lanes = 256 / N;
  double s = 0.0;
#pragma unroll 8
  for (int p = lane; p < P; p += lanes) s += part[(int64_t)p * N + n];
  red[threadIdx.x] = s;
  __syncthreads();
  for (int o = lanes / 2; o > 0; o >>= 1) {
    if (lane < o) red[threadIdx.x] += red[threadIdx.x + o * N];
    __syncthreads();
  }
  if (lane == 0) db[n] = (float)red[n];
}

int col_sum(const float* x, int64_t M, int N, float* db, double* scratch, hipStream_t st) {
  VAD_CHECK(N >= 1 && N <= 256 && 256 % N == 0, "col_sum: N divides 256");
  const int64_t rows = std::max<int64_t>(256 / N, cdiv(M, 256));
  const int P = (int)cdiv(M, rows);
  hipLaunchKernelGGL(col_sum_part_kernel, dim3((unsigned)P), dim3(256), 0, st, x, M, N, rows, scratch);
  VAD_LAUNCH_CHECK();
  hipLaunchKernelGGL(col_sum_fin_kernel, dim3(1), dim3(256), 0, st, scratch, P, N, db);
  VAD_LAUNCH_CHECK();
  return 0;
}

}  // namespace vad
