// Host data path: u8 frames staged in pinned host memory are copied to HBM as u8 (a quarter of
// the fp32 bytes over PCIe) and turned into the model's fp32 clip tensor on the device; frame resizing on the host.
//   vad_u8_to_clip  : dst = (u8 - 0.5) / 0.5   (mode 0: cad's Normalize([0.5],[0.5]) over raw 0..255 pixels,
//                                                causal_anomaly_detection.py:92-96, 1177-1179)
//                     dst = u8 / 255           (mode 1: ToTensor range, minicausal:120, bbox:409-411)
//                     -- the same float expressions as the synthetic-clip generator (bit-identical results)
//   vad_host_device_ptr: the device address of pinned (page-locked, mapped) host memory, so vad_u8_to_clip can read a
//                     staged batch straight over PCIe (ClipStager's direct mode: no copy engine, no u8 device slot)
//   vad_resize_u8   : bilinear resize with half-pixel centres, border clamping and 11-bit fixed-point weights
//                     (the scheme of cv2.resize INTER_LINEAR on u8 images that UCSDped2Dataset.__getitem__ calls,
//                     cad:88-89; restated from its published algorithm, cv2 itself is absent here: parity unpinned
//                     except for the identity case, which UCSD Ped2's native 360x240 frames hit)
#include <math.h>

#include <algorithm>
#include <vector>

#include "../../include/vad.h"
#include "common.h"

namespace vad {

typedef unsigned u32x4d __attribute__((ext_vector_type(4)));

__device__ __forceinline__ float u8_pixel(uint32_t u, int mode) {
  const float f = (float)u;
  return mode == 0 ? (f - 0.5f) / 0.5f : f / 255.f;
}

// 16 pixels per lane and iteration (one 16-B load, four 16-B stores): the source may be pinned host memory read over
// PCIe (vad_host_device_ptr), where wide requests matter; n16 = n / 16 full groups, the tail pixel by pixel
__global__ __launch_bounds__(256) void u8_to_clip_kernel(const uint8_t* __restrict__ src, int64_t n, int mode,
                                                         float* __restrict__ dst) {
  const int64_t n16 = n / 16;
  for (int64_t i = blockIdx.x * 256ll + threadIdx.x; i < n16; i += (int64_t)gridDim.x * 256) {
    const u32x4d w = reinterpret_cast<const u32x4d*>(src)[i];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      f32x4 o;
#pragma unroll
      for (int e = 0; e < 4; ++e) o[e] = u8_pixel((w[q] >> (8 * e)) & 0xffu, mode);
      reinterpret_cast<f32x4*>(dst)[4 * i + q] = o;
    }
  }
  for (int64_t i = n16 * 16 + blockIdx.x * 256ll + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256)
    dst[i] = u8_pixel(src[i], mode);
}

}  // namespace vad

using namespace vad;

extern "C" {

int vad_u8_to_clip(const uint8_t* src, int64_t n, int mode, float* dst, void* stream) {
  VAD_CHECK(mode == 0 || mode == 1, "vad_u8_to_clip: mode 0 (Normalize 0.5/0.5) or 1 (u8/255)");
  VAD_CHECK((reinterpret_cast<uintptr_t>(src) & 15) == 0 && (reinterpret_cast<uintptr_t>(dst) & 15) == 0,
            "vad_u8_to_clip: src and dst must be 16-byte aligned");
  if (n <= 0) return 0;
  // (1024 blocks keep ~4 MB of 16-B requests in flight: enough for HBM, and for PCIe when src is mapped host memory)
  hipLaunchKernelGGL(u8_to_clip_kernel, dim3((unsigned)std::min<int64_t>(cdiv(n / 16 + 1, 256), 1024)), dim3(256), 0,
                     (hipStream_t)stream, src, n, mode, dst);
  VAD_LAUNCH_CHECK();
  return 0;
}

int vad_host_device_ptr(const void* host, void** dev) {
  VAD_CHECK(host != nullptr && dev != nullptr, "vad_host_device_ptr: null argument");
  VAD_HIP(hipHostGetDevicePointer(dev, const_cast<void*>(host), 0));
  return 0;
}

int vad_resize_u8(const uint8_t* src, int sh, int sw, uint8_t* dst, int dh, int dw) {
  VAD_CHECK(src && dst && sh > 0 && sw > 0 && dh > 0 && dw > 0, "vad_resize_u8: bad arguments");
  constexpr int ONE = 2048;  // INTER_RESIZE_COEF_SCALE
  // per destination column / row: source index and the two 11-bit weights (rounded like saturate_cast<short>)
  auto table = [&](int dn, int sn, std::vector<int>& ofs, std::vector<int>& c0, std::vector<int>& c1) {
    ofs.resize(dn);
    c0.resize(dn);
    c1.resize(dn);
    const double scale = (double)sn / dn;
    for (int d = 0; d < dn; ++d) {
      float f = (float)((d + 0.5) * scale - 0.5);
      int s = (int)floorf(f);
      f -= (float)s;
      if (s < 0) {
        f = 0.f;
        s = 0;
      }
      if (s >= sn - 1) {
        f = 0.f;
        s = sn - 1;
      }
      ofs[d] = s;
      c0[d] = (int)lrintf((1.f - f) * ONE);
      c1[d] = (int)lrintf(f * ONE);
    }
  };
  std::vector<int> xo, xa, xb, yo, ya, yb;
  table(dw, sw, xo, xa, xb);
  table(dh, sh, yo, ya, yb);
  std::vector<int> r0(dw), r1(dw);
  auto hrow = [&](int sy, std::vector<int>& r) {
    const uint8_t* s = src + (int64_t)sy * sw;
    for (int x = 0; x < dw; ++x) {
      const int sx = xo[x];
      r[x] = sx + 1 < sw ? s[sx] * xa[x] + s[sx + 1] * xb[x] : s[sx] * ONE;
    }
  };
  for (int y = 0; y < dh; ++y) {
    const int sy = yo[y];
    hrow(sy, r0);
    hrow(std::min(sy + 1, sh - 1), r1);
    uint8_t* d = dst + (int64_t)y * dw;
    for (int x = 0; x < dw; ++x) {
      const int64_t v = ((int64_t)ya[y] * r0[x] + (int64_t)yb[y] * r1[x] + (1 << 21)) >> 22;
      d[x] = (uint8_t)std::min<int64_t>(255, std::max<int64_t>(0, v));
    }
  }
  return 0;
}

}  // extern "C"
