// torch.optim.Adam (coupled L2 weight decay) behind a finiteness-gated, optionally norm-gated clip_grad_norm_, over
// one flat parameter / grad / moment buffer split into slots (= named_parameters()).  Used by the cad1 memory
// autoencoder's train step (cad1:413-425); the minicausal plan carries the same sequence inline (mc_plan.hip).
//
// Status word (status[3], float): < 1 on entry = the step was skipped before backward (nothing happens); on exit
// 1 = non-finite grads (no step: the reference's skip), 2 = stepped.  status[1] = grad norm sqrt(sum_p ||g_p||^2)
// (per-slot norms rounded to float, summed in double, as torch's clip_grad_norm_), status[2] = 1 when clipped.
#pragma once
#include "common.h"

namespace vad {

constexpr int ADAM_MAX_SLOTS = 64;
constexpr int ADAM_SQ_CHUNKS = 64;  // blocks per slot of the squared-norm pass (fixed-order partials)

struct AdamSlots {
  int n;
  int64_t off[ADAM_MAX_SLOTS], numel[ADAM_MAX_SLOTS];
};

struct AdamWs {
  double* sq;   // [ADAM_MAX_SLOTS][ADAM_SQ_CHUNKS]
  int* bad;     // [ADAM_MAX_SLOTS][ADAM_SQ_CHUNKS]
  float* ctrl;  // [4]
};

// clip_grad_norm_(max_norm) only when norm > clip_above (clip_above < 0: always, plain torch semantics), then Adam
// (lr, betas, eps, coupled weight_decay) over params[0, nfloats); steps: int32 per slot (torch per-param counters).
// grad_scale multiplies the grads first (1/world after a data-parallel sum).
int adam_clip_step(const AdamSlots& t, float* params, const float* grads, float* exp_avg, float* exp_avg_sq,
                   int64_t nfloats, int32_t* steps, float* status, const AdamWs& w, float lr, float b1, float b2,
                   float eps, float wd, float clip_above, float max_norm, float grad_scale, hipStream_t st);

}  // namespace vad
