// Stand-alone entry points for single building blocks (dense layer, 3x3 conv) used by the kernel unit tests.
#include "../../include/vad.h"
#include "backbone.h"

using namespace vad;

extern "C" {

int vad_dense_forward(const float* X, int M, int K, const float* W, const float* b, int N, float* Y, int relu,
                      float* scratch, int64_t scratch_floats, void* stream) {
  DenseAct a;
  a.relu = relu;
  return dense_fwd(X, M, K, W, b, N, Y, a, scratch, scratch_floats, (hipStream_t)stream);
}

int vad_conv3x3_forward(const float* x_nhwc, int NF, int Ci, int IH, int IW, const float* w, const float* bias,
                        int Co, int stride, float* y_nhwc, float* wf_scratch, float* wd_scratch, float* partials,
                        void* stream) {
  Conv3Layer L{NF, Ci, Co, IH, IW, (IH - 1) / stride + 1, (IW - 1) / stride + 1, stride};
  if (w) VAD_TRY(conv3_prep_weights(w, L, wf_scratch, wd_scratch, (hipStream_t)stream));  // w == NULL: prepared
  int np = 0;
  return conv3_fwd(L, x_nhwc, nullptr, wf_scratch, bias, y_nhwc, partials, &np, (hipStream_t)stream);
}

int vad_conv3x3_dgrad(const float* dy_nhwc, int NF, int Ci, int IH, int IW, const float* w, int Co, int stride,
                      float* dx_nhwc, float* wf_scratch, float* wd_scratch, void* stream) {
  Conv3Layer L{NF, Ci, Co, IH, IW, (IH - 1) / stride + 1, (IW - 1) / stride + 1, stride};
  if (w) VAD_TRY(conv3_prep_weights(w, L, wf_scratch, wd_scratch, (hipStream_t)stream));  // w == NULL: prepared
  return conv3_dgrad(L, dy_nhwc, wd_scratch, dx_nhwc, (hipStream_t)stream);
}

}  // extern "C"

extern "C" int vad_conv3x3_wgrad(const float* x_nhwc, const float* dy_nhwc, int NF, int Ci, int IH, int IW, int Co,
                                 int stride, float* dW, float* partial, int64_t partial_floats, void* stream) {
  Conv3Layer L{NF, Ci, Co, IH, IW, (IH - 1) / stride + 1, (IW - 1) / stride + 1, stride};
  int ns = 0;
  VAD_TRY(conv3_wgrad(L, dy_nhwc, x_nhwc, nullptr, partial, &ns, partial_floats, (hipStream_t)stream));
  return conv3_wgrad_reduce(L, partial, ns, nullptr, 0, dW, nullptr, (hipStream_t)stream);
}

extern "C" int vad_set_tuning(const char* key, int value) { return vad::set_tuning(key, value); }

// The BN backward apply pass alone (measurement / tests): dY = k (dZ - mean dZ - xhat mean(dZ xhat)), dZ = dA masked by
// the ReLU of s y + t; stats = the layer's [7 C] BN state; bf16: dA / y / dY stored as bf16 (config 4).
extern "C" int vad_bn_bwd_apply(const void* dA, const void* y, const float* stats, int M, int C, void* dY, int bf16,
                                void* stream) {
  ActStorage abf(bf16);
  int nb = 0;
  return bn_bwd_apply(reinterpret_cast<const float*>(dA), reinterpret_cast<const float*>(y), stats, M, C,
                      reinterpret_cast<float*>(dY), nullptr, &nb, (hipStream_t)stream);
}
