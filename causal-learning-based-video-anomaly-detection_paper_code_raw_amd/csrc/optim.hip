// Adam + gated clip for the Adam-trained autoencoder plan (optim.h).
#include <algorithm>
#include <cmath>

#include "optim.h"

namespace vad {

// block (slot s, chunk c): squared L2 norm (double accumulation) and finiteness of one contiguous chunk of the slot's
// grad -> partial [s][c]; adam_prepare_kernel sums a slot's chunks in order (one block per slot took 0.4 ms on the
// autoencoder's largest weight)
__global__ __launch_bounds__(256) void adam_sqsum_kernel(const float* __restrict__ g, AdamSlots t, double* sq,
                                                         int* bad) {
  const int s = blockIdx.x, c = blockIdx.y;
  const int64_t len = (t.numel[s] + ADAM_SQ_CHUNKS - 1) / ADAM_SQ_CHUNKS;
  const int64_t i0 = c * len, i1 = min(t.numel[s], i0 + len);
  __shared__ double red[256];
  __shared__ int rb[256];
  double acc = 0.0;
  int nf = 0;
  for (int64_t i = i0 + threadIdx.x; i < i1; i += 256) {
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
    sq[s * ADAM_SQ_CHUNKS + c] = red[0];
    bad[s * ADAM_SQ_CHUNKS + c] = rb[0];
  }
}

// ctrl: [0] step? (1/0), [1] grad multiplier (clip coefficient x grad_scale), [2] -lr / bias_correction1,
//       [3] sqrt(bias_correction2)
__global__ void adam_prepare_kernel(const double* sq, const int* bad, int n, float* status, int32_t* steps, float lr,
                                    float b1, float b2, float clip_above, float max_norm, float grad_scale,
                                    float* ctrl) {
  // thread s adds slot s's chunk partials in order; thread 0 then goes on alone
  __shared__ double slot_sq[ADAM_MAX_SLOTS];
  __shared__ int slot_bad[ADAM_MAX_SLOTS];
  for (int s = threadIdx.x; s < n; s += blockDim.x) {
    double ss = 0.0;
    int nf = 0;
    for (int c = 0; c < ADAM_SQ_CHUNKS; ++c) {
      ss += sq[s * ADAM_SQ_CHUNKS + c];
      nf |= bad[s * ADAM_SQ_CHUNKS + c];
    }
    slot_sq[s] = ss;
    slot_bad[s] = nf;
  }
  __syncthreads();
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  ctrl[0] = 0.f;
  ctrl[1] = grad_scale;
  status[2] = 0.f;
  if (status[3] < 1.f) return;  // skipped before backward
  double tot = 0.0;
  int nonfin = 0;
  for (int s = 0; s < n; ++s) {
    const double ns = (double)(float)(sqrt(slot_sq[s]) * (double)grad_scale);  // per-param norm (float), squared
    tot += ns * ns;
    nonfin |= slot_bad[s];
  }
  if (nonfin) {
    status[3] = 1.f;
    return;
  }
  const double gn = sqrt(tot);
  status[1] = (float)gn;
  if (clip_above < 0.f || gn > (double)clip_above) {
    // clip_grad_norm_(params, max_norm): total = ||(||g_p||)||, coef = max_norm / (total + 1e-6), clamped to 1
    const float total = (float)gn;
    ctrl[1] = fminf(1.f, max_norm / (total + 1e-6f)) * grad_scale;
    status[2] = 1.f;
  }
  const int step = steps[0] + 1;
  for (int s = 0; s < n; ++s) steps[s] = step;
  const double bc1 = 1.0 - pow((double)b1, step), bc2 = 1.0 - pow((double)b2, step);
  ctrl[0] = 1.f;
  ctrl[2] = (float)(-(double)lr / bc1);
  ctrl[3] = (float)sqrt(bc2);
  status[3] = 2.f;
}

// torch.optim.Adam single-tensor step (weight decay coupled into the grad, torch/optim/adam.py)
__global__ __launch_bounds__(256) void adam_kernel(float* __restrict__ p, const float* __restrict__ g,
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

int adam_clip_step(const AdamSlots& t, float* params, const float* grads, float* exp_avg, float* exp_avg_sq,
                   int64_t nfloats, int32_t* steps, float* status, const AdamWs& w, float lr, float b1, float b2,
                   float eps, float wd, float clip_above, float max_norm, float grad_scale, hipStream_t st) {
  VAD_CHECK(t.n >= 1 && t.n <= ADAM_MAX_SLOTS, "adam_clip_step: slot table size");
  VAD_CHECK(exp_avg && exp_avg_sq && steps, "adam_clip_step: optimizer state not bound");
  hipLaunchKernelGGL(adam_sqsum_kernel, dim3(t.n, ADAM_SQ_CHUNKS), dim3(256), 0, st, grads, t, w.sq, w.bad);
  VAD_LAUNCH_CHECK();
  hipLaunchKernelGGL(adam_prepare_kernel, dim3(1), dim3(64), 0, st, w.sq, w.bad, t.n, status, steps, lr, b1, b2,
                     clip_above, max_norm, grad_scale, w.ctrl);
  VAD_LAUNCH_CHECK();
  hipLaunchKernelGGL(adam_kernel, dim3((unsigned)std::min<int64_t>(cdiv(nfloats, 256), 1024)), dim3(256), 0, st,
                     params, grads, exp_avg, exp_avg_sq, nfloats, w.ctrl, b1, b2, eps, wd);
  VAD_LAUNCH_CHECK();
  return 0;
}

}  // namespace vad
