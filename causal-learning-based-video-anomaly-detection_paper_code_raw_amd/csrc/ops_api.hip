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
  if (x3_wgrad_dma_supported(L)) {  // (knob conv_wgrad_dma) the operand planes live at the end of the scratch
    const int64_t mo = (int64_t)L.NF * L.OH * L.OW * L.Co, mi = (int64_t)L.NF * L.IH * L.IW * L.Ci;
    const int64_t pf = (3 * (mo + mi) + 1) / 2 + 64;
    VAD_CHECK(partial_floats > pf, "vad_conv3x3_wgrad: scratch too small for the operand planes");
    __bf16* pdy = reinterpret_cast<__bf16*>(partial + (partial_floats - pf) / 64 * 64);
    __bf16* px = pdy + 3 * mo;
    VAD_TRY(planes_split(dy_nhwc, nullptr, mo / L.Co, L.Co, pdy, (hipStream_t)stream));
    VAD_TRY(planes_split(x_nhwc, nullptr, mi / L.Ci, L.Ci, px, (hipStream_t)stream));
    VAD_TRY(x3_wgrad_dma(L, pdy, px, partial, &ns, (partial_floats - pf) / 64 * 64, 0, (hipStream_t)stream));
    return conv3_wgrad_reduce(L, partial, ns, nullptr, 0, dW, nullptr, (hipStream_t)stream);
  }
  VAD_TRY(conv3_wgrad(L, dy_nhwc, x_nhwc, nullptr, partial, &ns, partial_floats, (hipStream_t)stream));
  return conv3_wgrad_reduce(L, partial, ns, nullptr, 0, dW, nullptr, (hipStream_t)stream);
}

extern "C" int vad_set_tuning(const char* key, int value) { return vad::set_tuning(key, value); }

extern "C" int vad_conv3x3_dgrad_planes(const float* dy_nhwc, int NF, int Ci, int IH, int IW, const float* w, int Co,
                                        int stride, float* dx_nhwc, float* scratch, int64_t scratch_floats,
                                        void* stream) {
  Conv3Layer L{NF, Ci, Co, IH, IW, (IH - 1) / stride + 1, (IW - 1) / stride + 1, stride};
  VAD_CHECK((stride == 2 && dgrad_s2_dma_supported(L)) || (stride == 1 && dgrad_s1_dma_supported(L)),
            "vad_conv3x3_dgrad_planes: unsupported shape (or knob conv_dgrad_s1_dma / conv_dgrad_s2_dma off)");
  const int64_t nw = (int64_t)9 * Ci * Co, mo = (int64_t)NF * L.OH * L.OW * Co;
  VAD_CHECK(scratch_floats >= 4 * nw + (3 * mo + 1) / 2 + 1024, "vad_conv3x3_dgrad_planes: scratch too small");
  float* wf = scratch;
  float* wd = scratch + nw;  // fp32 Wd, then its bf16 planes (1.5 nw floats)
  __bf16* w3 = reinterpret_cast<__bf16*>(wd + nw);
  __bf16* pdy = reinterpret_cast<__bf16*>(scratch + (4 * nw + 63) / 64 * 64);
  const hipStream_t st = (hipStream_t)stream;
  const float* w1[1] = {w};
  float* wf1[1] = {wf};
  float* wd1[1] = {wd};
  __bf16* w31[1] = {w3};
  VAD_TRY(conv3_prep_weights_all(1, w1, &L, wf1, wd1, st, w31));
  VAD_TRY(planes_split(dy_nhwc, nullptr, mo / Co, Co, pdy, st));
  return stride == 2 ? dgrad_s2_dma(L, pdy, w3, dx_nhwc, st, nullptr) : dgrad_s1_dma(L, pdy, w3, dx_nhwc, st, nullptr);
}
