// Direct 3x3 convolution over an LDS-resident input patch, on f32 MFMA (v_mfma_f32_32x32x2_f32).
//
// The implicit GEMM (gemm.h) re-gathers the input from L2 for every one of the 9 taps and synchronises every
// 32-wide K slice.  Here a block owns 128 output pixels (NI images x TH x TW) x 32 output channels and walks the
// reduction channels in chunks of 32: per chunk it stages the input patch (tile + 1-pixel halo, BN+ReLU of the
// producing layer applied while staging, zero padding) and the 32 x (9 taps x 32) weight slice in LDS once, then
// every wave issues 9 x 4 x 4 = 144 MFMAs on its 32 pixels with only LDS reads in between (one ds_read_b128 of A
// and one of B feed 4 MFMAs; rows padded to 36 / 292 floats so the 16-lane read groups are conflict-free).
// Used for stride-1 forward convs (BN statistics in the epilogue) and stride-1 input gradients (flipped taps).
#include "backbone.h"
#include "gemm.h"

namespace vad {

constexpr int PC = 32;            // reduction channels per chunk
constexpr int PROW = PC + 4;      // patch row stride (floats)
constexpr int WROW = 9 * PC + 4;  // weight row stride (floats)

struct PatchArgs {
  const float* src;    // NHWC [NF][IH][IW][C]
  const float* scale;  // BN+ReLU on load (forward), nullable
  const float* shift;
  const float* w;      // prepared B operand [N][9][C]
  const float* bias;   // forward only
  float* out;          // NHWC [NF][OH][OW][N]
  float* partials;     // forward: [gridDim.x][2N] BN partial sums
  int NF, IH, IW, C, OH, OW, N;
  int tiles_h, tiles_w;
};

template <int NI, int TH, int TW, bool FWD>
__global__ __launch_bounds__(256, 2) void conv3x3_patch_kernel(const PatchArgs p) {
  static_assert(NI * TH * TW == 128, "a block owns 128 output pixels");
  constexpr int PH = TH + 2, PW = TW + 2, PROWS = NI * PH * PW;
  __shared__ __attribute__((aligned(16))) float sm[PROWS * PROW + 32 * WROW];
  float* patch = sm;
  float* wl = sm + PROWS * PROW;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int tiles_per_img = p.tiles_h * p.tiles_w;
  const int img0 = (blockIdx.x / tiles_per_img) * NI;
  const int trem = blockIdx.x % tiles_per_img;
  const int oy0 = (trem / p.tiles_w) * TH, ox0 = (trem % p.tiles_w) * TW;
  const int n0 = blockIdx.y * 32;

  // this lane's A pixel (MFMA row i = lane & 31) inside the block tile
  const int m = wave * 32 + (lane & 31);
  const int mi = m / (TH * TW), mr = m % (TH * TW);
  const int py = mr / TW, px = mr % TW;
  const int arow = (mi * PH + py) * PW + px;  // patch row of tap (0,0)
  const int h = lane >> 5;
  const int j = lane & 31;  // B column (output channel n0 + j)

  f32x16 acc;
#pragma unroll
  for (int r = 0; r < 16; ++r) acc[r] = 0.f;

  // staging: thread tid always handles channel quad c4 = (tid % 8) * 4 (256 % 8 == 0), so BN scale/shift are
  // per-thread constants; all global loads of a chunk are issued back to back into registers, the chunk after
  // the current one is fetched while the current one is multiplied.
  constexpr int PQ = PROWS * (PC / 4), PIT = (PQ + 255) / 256;
  constexpr int WQ = 32 * 9 * (PC / 4), WIT = WQ / 256;
  static_assert(WQ % 256 == 0, "weight staging is exact");
  const int c4 = (tid % (PC / 4)) * 4;
  f32x4 pv[PIT], wv[WIT];
  auto fetch = [&](int c0) {
#pragma unroll
    for (int it = 0; it < PIT; ++it) {
      const int q = tid + it * 256;
      const int row = q / (PC / 4);
      const int im = row / (PH * PW), rr = row % (PH * PW);
      const int iy = oy0 - 1 + rr / PW, ix = ox0 - 1 + rr % PW;
      const int img = img0 + im;
      pv[it] = f32x4{0.f, 0.f, 0.f, 0.f};
      if (q < PQ && img < p.NF && iy >= 0 && iy < p.IH && ix >= 0 && ix < p.IW)
        pv[it] = *reinterpret_cast<const f32x4*>(p.src + (((int64_t)img * p.IH + iy) * p.IW + ix) * p.C + c0 + c4);
    }
#pragma unroll
    for (int it = 0; it < WIT; ++it) {
      const int q = tid + it * 256;
      const int n = q / (9 * PC / 4), t = (q % (9 * PC / 4)) / (PC / 4);
      const int tw = FWD ? t : 8 - t;
      wv[it] = f32x4{0.f, 0.f, 0.f, 0.f};
      if (n0 + n < p.N) wv[it] = *reinterpret_cast<const f32x4*>(p.w + ((int64_t)(n0 + n) * 9 + tw) * p.C + c0 + c4);
    }
  };
  auto stash = [&](int c0) {
    f32x4 sc = {1.f, 1.f, 1.f, 1.f}, sh = {0.f, 0.f, 0.f, 0.f};
    const bool bn = FWD && p.scale;
    if (bn) {
      sc = *reinterpret_cast<const f32x4*>(p.scale + c0 + c4);
      sh = *reinterpret_cast<const f32x4*>(p.shift + c0 + c4);
    }
#pragma unroll
    for (int it = 0; it < PIT; ++it) {
      const int q = tid + it * 256;
      if (q < PQ) {
        const int row = q / (PC / 4);
        f32x4 v = pv[it];
        if (bn) {
          // zero padding stays zero: padded taps read 0 in the reference's relu(bn(y)) zero-padded input
          const int im = row / (PH * PW), rr = row % (PH * PW);
          const int iy = oy0 - 1 + rr / PW, ix = ox0 - 1 + rr % PW;
          if (img0 + im < p.NF && iy >= 0 && iy < p.IH && ix >= 0 && ix < p.IW) {
#pragma unroll
            for (int e = 0; e < 4; ++e) v[e] = fmaxf(fmaf(v[e], sc[e], sh[e]), 0.f);
          }
        }
        *reinterpret_cast<f32x4*>(patch + row * PROW + c4) = v;
      }
    }
#pragma unroll
    for (int it = 0; it < WIT; ++it) {
      const int q = tid + it * 256;
      const int n = q / (9 * PC / 4), t = (q % (9 * PC / 4)) / (PC / 4);
      *reinterpret_cast<f32x4*>(wl + n * WROW + t * PC + c4) = wv[it];
    }
  };

  fetch(0);
  for (int c0 = 0; c0 < p.C; c0 += PC) {
    __syncthreads();
    stash(c0);
    __syncthreads();
    if (c0 + PC < p.C) fetch(c0 + PC);
    // 36 steps of (one A quad, one B quad) -> 4 MFMAs; the next step's quads are read before this step's MFMAs
    const float* abase = patch + arow * PROW + 4 * h;
    const float* bbase = wl + j * WROW + 4 * h;
    f32x4 a4 = *reinterpret_cast<const f32x4*>(abase);
    f32x4 b4 = *reinterpret_cast<const f32x4*>(bbase);
#pragma unroll
    for (int s = 0; s < 36; ++s) {
      f32x4 an = a4, bn = b4;
      if (s + 1 < 36) {
        const int t = (s + 1) >> 2, kk = (s + 1) & 3;
        an = *reinterpret_cast<const f32x4*>(abase + ((t / 3) * PW + (t % 3)) * PROW + kk * 8);
        bn = *reinterpret_cast<const f32x4*>(bbase + t * PC + kk * 8);
      }
      acc = mfma32(a4[0], b4[0], acc);
      acc = mfma32(a4[1], b4[1], acc);
      acc = mfma32(a4[2], b4[2], acc);
      acc = mfma32(a4[3], b4[3], acc);
      a4 = an;
      b4 = bn;
    }
  }

  // epilogue: row = pixel (r&3) + 8(r>>2) + 4h of the wave's 32, column = channel n0 + j
  const int col = n0 + j;
  const float bj = (FWD && col < p.N) ? p.bias[col] : 0.f;
  float s1 = 0.f, s2 = 0.f;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int pm = wave * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
    const int qi = pm / (TH * TW), qr = pm % (TH * TW);
    const int oy = oy0 + qr / TW, ox = ox0 + qr % TW, img = img0 + qi;
    if (img < p.NF && oy < p.OH && ox < p.OW && col < p.N) {
      const float v = acc[r] + bj;
      p.out[(((int64_t)img * p.OH + oy) * p.OW + ox) * p.N + col] = v;
      if (FWD) {
        s1 += v;
        s2 = fmaf(v, v, s2);
      }
    }
  }
  if (FWD) {
    s1 += __shfl_xor(s1, 32, 64);
    s2 += __shfl_xor(s2, 32, 64);
    __syncthreads();
    float* red = sm;  // [4 waves][2][32]
    if (lane < 32) {
      red[wave * 64 + lane] = s1;
      red[wave * 64 + 32 + lane] = s2;
    }
    __syncthreads();
    if (tid < 64) {
      const int c = tid & 31, which = tid >> 5;
      const float v = red[which * 32 + c] + red[64 + which * 32 + c] + red[128 + which * 32 + c] +
                      red[192 + which * 32 + c];
      if (n0 + c < p.N) p.partials[(int64_t)blockIdx.x * 2 * p.N + which * p.N + n0 + c] = v;
    }
  }
}

template <int NI, int TH, int TW, bool FWD>
static int launch_patch(PatchArgs a, hipStream_t st, int* nparts) {
  a.tiles_h = (int)cdiv(a.OH, TH);
  a.tiles_w = (int)cdiv(a.OW, TW);
  const int64_t gx = cdiv(a.NF, NI) * a.tiles_h * a.tiles_w;
  dim3 grid((unsigned)gx, (unsigned)cdiv(a.N, 32));
  hipLaunchKernelGGL((conv3x3_patch_kernel<NI, TH, TW, FWD>), grid, dim3(256), 0, st, a);
  VAD_LAUNCH_CHECK();
  if (nparts) *nparts = (int)gx;
  return 0;
}

// tile geometry per output size (128 pixels per block): 0 -> 2 images x 8x8, 1 -> 8x16, 2 -> 4x32
static int patch_geom(int OH, int OW) { return (OH <= 8 && OW <= 8) ? 0 : (OW <= 16 ? 1 : 2); }

template <bool FWD>
static int dispatch_patch(const PatchArgs& a, hipStream_t st, int* nparts) {
  switch (patch_geom(a.OH, a.OW)) {
    case 0: return launch_patch<2, 8, 8, FWD>(a, st, nparts);
    case 1: return launch_patch<1, 8, 16, FWD>(a, st, nparts);
    default: return launch_patch<1, 4, 32, FWD>(a, st, nparts);
  }
}

int64_t conv3_patch_blocks(int NF, int OH, int OW) {
  switch (patch_geom(OH, OW)) {
    case 0: return cdiv(NF, 2) * cdiv(OH, 8) * cdiv(OW, 8);
    case 1: return (int64_t)NF * cdiv(OH, 8) * cdiv(OW, 16);
    default: return (int64_t)NF * cdiv(OH, 4) * cdiv(OW, 32);
  }
}

bool conv3_patch_supported(const Conv3Layer& L, bool fwd) {
  return L.stride == 1 && (fwd ? L.Ci : L.Co) % PC == 0;
}

int conv3_patch_fwd(const Conv3Layer& L, const float* src, const float* src_stats, const float* wf, const float* bias,
                    float* y, float* partials, int* nparts, hipStream_t st) {
  VAD_CHECK(conv3_patch_supported(L, true), "conv3_patch_fwd: stride-1, Ci % 32 == 0 only");
  PatchArgs a{};
  a.src = src;
  a.scale = src_stats ? src_stats + 2 * L.Ci : nullptr;
  a.shift = src_stats ? src_stats + 3 * L.Ci : nullptr;
  a.w = wf;
  a.bias = bias;
  a.out = y;
  a.partials = partials;
  a.NF = L.NF; a.IH = L.IH; a.IW = L.IW; a.C = L.Ci; a.OH = L.OH; a.OW = L.OW; a.N = L.Co;
  return dispatch_patch<true>(a, st, nparts);
}

int conv3_patch_dgrad(const Conv3Layer& L, const float* dY, const float* wd, float* dX, hipStream_t st) {
  VAD_CHECK(conv3_patch_supported(L, false), "conv3_patch_dgrad: stride-1, Co % 32 == 0 only");
  PatchArgs a{};
  a.src = dY;
  a.w = wd;
  a.out = dX;
  a.NF = L.NF; a.IH = L.OH; a.IW = L.OW; a.C = L.Co; a.OH = L.IH; a.OW = L.IW; a.N = L.Ci;
  return dispatch_patch<false>(a, st, nullptr);
}

}  // namespace vad
