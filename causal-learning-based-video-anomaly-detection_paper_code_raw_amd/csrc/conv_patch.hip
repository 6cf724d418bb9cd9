// Direct 3x3 convolutions over an LDS-resident input patch, on f32 MFMA (v_mfma_f32_32x32x2_f32).
//
// The implicit GEMM (gemm.h) re-gathers the input from L2 for every one of the 9 taps and synchronises every
// 32-wide K slice.  Here a block owns 128 output pixels (NI images x TH x TW) x 32 output channels and walks the
// reduction channels in chunks of PC: per chunk it stages the input patch (tile + halo, BN+ReLU of the producing
// layer applied while staging, zero padding) and the 32 x (9 taps x PC) weight slice in LDS once, then every
// wave issues 9 x PC/2 MFMAs on its 32 pixels with only LDS reads in between (one ds_read_b128 of A and one of
// B feed 4 MFMAs; rows padded to PC+4 / 9PC+4 floats so the 16-lane read groups cover all 64 banks).
// Global loads of chunk c+1 are issued into registers before chunk c is multiplied.
//   conv3x3_patch_kernel        stride-1/2 forward (BN statistics in the epilogue), stride-1 input gradient
//   conv3x3_dgrad_s2_kernel     stride-2 input gradient: 4 parity classes of a 16x16 dX tile share one dY patch
//   conv3x3_wgrad_patch_kernel  weight gradient (split-K over pixel tiles)
// Stride-2 patches store their columns de-interleaved by parity so consecutive output pixels read consecutive
// patch rows.
#include <algorithm>

#include "backbone.h"
#include "gemm.h"

namespace vad {

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

// Stage one chunk of a weight slice [32 n][9 taps][PC] into LDS rows of 9*PC+4 floats (tap order = LDS order;
// FLIP reverses the taps, i.e. the stride-1 input gradient's rotated kernel).
template <int PC, bool FLIP>
struct WeightStage {
  static constexpr int CQ = PC / 4, WQ = 32 * 9 * CQ, WIT = (WQ + 255) / 256, WROW = 9 * PC + 4;
  f32x4 v[WIT];
  __device__ void fetch(const PatchArgs& p, int n0, int c0, int tid) {
#pragma unroll
    for (int it = 0; it < WIT; ++it) {
      const int q = tid + it * 256;
      const int n = q / (9 * CQ), t = (q % (9 * CQ)) / CQ, c4 = (q % CQ) * 4;
      v[it] = f32x4{0.f, 0.f, 0.f, 0.f};
      if (q < WQ && n0 + n < p.N)
        v[it] = *reinterpret_cast<const f32x4*>(p.w + ((int64_t)(n0 + n) * 9 + (FLIP ? 8 - t : t)) * p.C + c0 + c4);
    }
  }
  __device__ void stash(float* wl, int tid) const {
#pragma unroll
    for (int it = 0; it < WIT; ++it) {
      const int q = tid + it * 256;
      const int n = q / (9 * CQ), t = (q % (9 * CQ)) / CQ, c4 = (q % CQ) * 4;
      if (q < WQ) *reinterpret_cast<f32x4*>(wl + n * WROW + t * PC + c4) = v[it];
    }
  }
};

template <int S, int NI, int TH, int TW, int PC, bool FWD>
__global__ __launch_bounds__(256, 2) void conv3x3_patch_kernel(const PatchArgs p) {
  static_assert(NI * TH * TW == 128, "a block owns 128 output pixels");
  static_assert(FWD || S == 1, "strided input gradients use conv3x3_dgrad_s2_kernel");
  constexpr int PROW = PC + 4, WROW = 9 * PC + 4, CQ = PC / 4;
  constexpr int PH = (TH - 1) * S + 3, PW = (TW - 1) * S + 3, PROWS = NI * PH * PW, PWE = (PW + 1) / 2;
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
  const int h = lane >> 5;
  const int j = lane & 31;  // B column (output channel n0 + j)
  const float* abase = patch + ((mi * PH + py * S) * PW + px) * PROW + 4 * h;
  const float* bbase = wl + j * WROW + 4 * h;

  f32x16 acc;
#pragma unroll
  for (int r = 0; r < 16; ++r) acc[r] = 0.f;

  // staging: thread tid always handles channel quad c4 = (tid % CQ) * 4, so BN scale/shift are per-thread
  // constants
  constexpr int PQ = PROWS * CQ, PIT = (PQ + 255) / 256;
  const int c4 = (tid % CQ) * 4;
  f32x4 pv[PIT];
  WeightStage<PC, !FWD> ws;
  auto fetch = [&](int c0) {
#pragma unroll
    for (int it = 0; it < PIT; ++it) {
      const int q = tid + it * 256;
      const int row = q / CQ;
      const int im = row / (PH * PW), rr = row % (PH * PW);
      const int iy = oy0 * S - 1 + rr / PW, ix = ox0 * S - 1 + rr % PW;
      const int img = img0 + im;
      pv[it] = f32x4{0.f, 0.f, 0.f, 0.f};
      if (q < PQ && img < p.NF && iy >= 0 && iy < p.IH && ix >= 0 && ix < p.IW)
        pv[it] = *reinterpret_cast<const f32x4*>(p.src + (((int64_t)img * p.IH + iy) * p.IW + ix) * p.C + c0 + c4);
    }
    ws.fetch(p, n0, c0, tid);
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
        const int row = q / CQ;
        const int im = row / (PH * PW), rr = row % (PH * PW);
        const int ry = rr / PW, rx = rr % PW;
        f32x4 v = pv[it];
        if (bn) {
          // zero padding stays zero: padded taps read 0 in the reference's relu(bn(y)) zero-padded input
          const int iy = oy0 * S - 1 + ry, ix = ox0 * S - 1 + rx;
          if (img0 + im < p.NF && iy >= 0 && iy < p.IH && ix >= 0 && ix < p.IW) {
#pragma unroll
            for (int e = 0; e < 4; ++e) v[e] = fmaxf(fmaf(v[e], sc[e], sh[e]), 0.f);
          }
        }
        const int col = S == 1 ? rx : ((rx & 1) ? PWE + (rx >> 1) : (rx >> 1));
        *reinterpret_cast<f32x4*>(patch + ((im * PH + ry) * PW + col) * PROW + c4) = v;
      }
    }
    ws.stash(wl, tid);
  };

  fetch(0);
  for (int c0 = 0; c0 < p.C; c0 += PC) {
    __syncthreads();
    stash(c0);
    __syncthreads();
    if (c0 + PC < p.C) fetch(c0 + PC);
    // 9*PC/8 steps of (one A quad, one B quad) -> 4 MFMAs
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      const int kh = t / 3, kw = t % 3;
      const int kwo = S == 1 ? kw : ((kw & 1) ? PWE + (kw >> 1) : (kw >> 1));
      const float* ap = abase + (kh * PW + kwo) * PROW;
      const float* bp = bbase + t * PC;
#pragma unroll
      for (int kk = 0; kk < PC / 8; ++kk) {
        const f32x4 a4 = *reinterpret_cast<const f32x4*>(ap + kk * 8);
        const f32x4 b4 = *reinterpret_cast<const f32x4*>(bp + kk * 8);
        acc = mfma32(a4[0], b4[0], acc);
        acc = mfma32(a4[1], b4[1], acc);
        acc = mfma32(a4[2], b4[2], acc);
        acc = mfma32(a4[3], b4[3], acc);
      }
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

// Stride-2 input gradient.  dX pixel (2i+ph, 2j+pw) only sees the taps whose parity matches (ph, pw):
// rows kh=1 (dY row i) for ph=0, kh=0 (row i+1) and kh=2 (row i) for ph=1; same for columns.  A block owns the
// 16x16 dX tile of class pixels i in [i0, i0+8), j in [j0, j0+8): all four classes read the same 9x9 dY patch.
// Work per (class, half of the 8x8 class tile) = its tap count (1/2/2/4 x 32 pixels); the waves take
// (11,00), (11,00), (01,10), (01,10) pairs -> 5/5/4/4 taps.
template <int PC, int CPH, int CPW>
__device__ __forceinline__ void dgrad_s2_class(f32x16& acc, const float* pbase, const float* bbase) {
  constexpr int PROW = PC + 4;
#pragma unroll
  for (int a = 0; a < (CPH ? 2 : 1); ++a) {
    const int kh = CPH ? (a == 0 ? 0 : 2) : 1, dh = (CPH && a == 0) ? 1 : 0;
#pragma unroll
    for (int b = 0; b < (CPW ? 2 : 1); ++b) {
      const int kw = CPW ? (b == 0 ? 0 : 2) : 1, dw = (CPW && b == 0) ? 1 : 0;
      const float* ap = pbase + (dh * 9 + dw) * PROW;
      const float* bp = bbase + (kh * 3 + kw) * PC;
#pragma unroll
      for (int kk = 0; kk < PC / 8; ++kk) {
        const f32x4 a4 = *reinterpret_cast<const f32x4*>(ap + kk * 8);
        const f32x4 b4 = *reinterpret_cast<const f32x4*>(bp + kk * 8);
        acc = mfma32(a4[0], b4[0], acc);
        acc = mfma32(a4[1], b4[1], acc);
        acc = mfma32(a4[2], b4[2], acc);
        acc = mfma32(a4[3], b4[3], acc);
      }
    }
  }
}

// p.src = dY [NF][IH=OHy][IW=OWy][C=Co], p.w = Wd [Ci][9][Co], p.out = dX [NF][OH=XH][OW=XW][N=Ci]
template <int PC>
__global__ __launch_bounds__(256, 2) void conv3x3_dgrad_s2_kernel(const PatchArgs p) {
  constexpr int PROW = PC + 4, WROW = 9 * PC + 4, CQ = PC / 4, PROWS = 81;
  __shared__ __attribute__((aligned(16))) float sm[PROWS * PROW + 32 * WROW];
  float* patch = sm;
  float* wl = sm + PROWS * PROW;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int tiles_per_img = p.tiles_h * p.tiles_w;
  const int img = blockIdx.x / tiles_per_img;
  const int trem = blockIdx.x % tiles_per_img;
  const int i0 = (trem / p.tiles_w) * 8, j0 = (trem % p.tiles_w) * 8;
  const int n0 = blockIdx.y * 32;
  const int h = lane >> 5, j = lane & 31;
  const int g = wave & 1;  // half of the 8x8 class tile (class rows 4g..4g+3)
  const float* pbase = patch + ((4 * g + (lane & 31) / 8) * 9 + (lane & 31) % 8) * PROW + 4 * h;
  const float* bbase = wl + j * WROW + 4 * h;

  f32x16 acc0, acc1;
#pragma unroll
  for (int r = 0; r < 16; ++r) acc0[r] = acc1[r] = 0.f;

  constexpr int PQ = PROWS * CQ, PIT = (PQ + 255) / 256;
  const int c4 = (tid % CQ) * 4;
  f32x4 pv[PIT];
  WeightStage<PC, false> ws;
  auto fetch = [&](int c0) {
#pragma unroll
    for (int it = 0; it < PIT; ++it) {
      const int q = tid + it * 256;
      const int row = q / CQ;
      const int y = i0 + row / 9, x = j0 + row % 9;
      pv[it] = f32x4{0.f, 0.f, 0.f, 0.f};
      if (q < PQ && y < p.IH && x < p.IW)
        pv[it] = *reinterpret_cast<const f32x4*>(p.src + (((int64_t)img * p.IH + y) * p.IW + x) * p.C + c0 + c4);
    }
    ws.fetch(p, n0, c0, tid);
  };
  fetch(0);
  for (int c0 = 0; c0 < p.C; c0 += PC) {
    __syncthreads();
#pragma unroll
    for (int it = 0; it < PIT; ++it) {
      const int q = tid + it * 256;
      if (q < PQ) *reinterpret_cast<f32x4*>(patch + (q / CQ) * PROW + c4) = pv[it];
    }
    ws.stash(wl, tid);
    __syncthreads();
    if (c0 + PC < p.C) fetch(c0 + PC);
    if (wave < 2) {
      dgrad_s2_class<PC, 1, 1>(acc0, pbase, bbase);
      dgrad_s2_class<PC, 0, 0>(acc1, pbase, bbase);
    } else {
      dgrad_s2_class<PC, 0, 1>(acc0, pbase, bbase);
      dgrad_s2_class<PC, 1, 0>(acc1, pbase, bbase);
    }
  }

  const int col = n0 + j;
  const int ph0 = wave < 2 ? 1 : 0, pw0 = 1;  // acc0 class: (1,1) or (0,1)
  const int ph1 = wave < 2 ? 0 : 1, pw1 = 0;  // acc1 class: (0,0) or (1,0)
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int pm = (r & 3) + 8 * (r >> 2) + 4 * h;
    const int ci_ = i0 + 4 * g + pm / 8, cj = j0 + pm % 8;
    const int y0 = 2 * ci_ + ph0, x0 = 2 * cj + pw0;
    if (y0 < p.OH && x0 < p.OW && col < p.N) p.out[(((int64_t)img * p.OH + y0) * p.OW + x0) * p.N + col] = acc0[r];
    const int y1 = 2 * ci_ + ph1, x1 = 2 * cj + pw1;
    if (y1 < p.OH && x1 < p.OW && col < p.N) p.out[(((int64_t)img * p.OH + y1) * p.OW + x1) * p.N + col] = acc1[r];
  }
}

// Single-chunk stride-1 layers (C == 32: layer1.0 / layer1.1 forward, layer1.1 input gradient).  The weight slice
// is the same for every pixel tile, so a persistent block stages it once, then walks a contiguous range of tiles
// (neighbours share halo rows in the same L2): the next tile's patch is loaded into registers while the current
// one is multiplied, and the BN partial sums accumulate across the block's tiles (one partial row per block).
template <int NI, int TH, int TW, bool FWD>
__global__ __launch_bounds__(256, 2) void conv3x3_patch_persist_kernel(const PatchArgs p, int tpb, int ntiles) {
  constexpr int PC = 32, PROW = PC + 4, WROW = 9 * PC + 4, CQ = PC / 4;
  constexpr int PH = TH + 2, PW = TW + 2, PROWS = NI * PH * PW;
  __shared__ __attribute__((aligned(16))) float sm[PROWS * PROW + 32 * WROW];
  float* patch = sm;
  float* wl = sm + PROWS * PROW;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int tiles_per_img = p.tiles_h * p.tiles_w;
  const int n0 = blockIdx.y * 32;
  const int t0 = blockIdx.x * tpb, t1 = min(ntiles, t0 + tpb);
  const int m = wave * 32 + (lane & 31);
  const int mi = m / (TH * TW), mr = m % (TH * TW);
  const int py = mr / TW, px = mr % TW;
  const int h = lane >> 5, j = lane & 31;
  const float* abase = patch + ((mi * PH + py) * PW + px) * PROW + 4 * h;
  const float* bbase = wl + j * WROW + 4 * h;
  const int c4 = (tid % CQ) * 4;
  constexpr int PQ = PROWS * CQ, PIT = (PQ + 255) / 256;

  {  // the weight slice, once
    WeightStage<PC, !FWD> ws;
    ws.fetch(p, n0, 0, tid);
    ws.stash(wl, tid);
  }
  f32x4 sc = {1.f, 1.f, 1.f, 1.f}, sh = {0.f, 0.f, 0.f, 0.f};
  const bool bn = FWD && p.scale;
  if (bn) {
    sc = *reinterpret_cast<const f32x4*>(p.scale + c4);
    sh = *reinterpret_cast<const f32x4*>(p.shift + c4);
  }
  f32x4 pv[PIT];
  auto origin = [&](int tile, int& img0, int& oy0, int& ox0) {
    img0 = (tile / tiles_per_img) * NI;
    const int tr = tile % tiles_per_img;
    oy0 = (tr / p.tiles_w) * TH;
    ox0 = (tr % p.tiles_w) * TW;
  };
  auto fetch = [&](int tile) {
    int img0, oy0, ox0;
    origin(tile, img0, oy0, ox0);
#pragma unroll
    for (int it = 0; it < PIT; ++it) {
      const int q = tid + it * 256;
      const int row = q / CQ;
      const int im = row / (PH * PW), rr = row % (PH * PW);
      const int iy = oy0 - 1 + rr / PW, ix = ox0 - 1 + rr % PW, img = img0 + im;
      pv[it] = f32x4{0.f, 0.f, 0.f, 0.f};
      if (q < PQ && img < p.NF && iy >= 0 && iy < p.IH && ix >= 0 && ix < p.IW)
        pv[it] = *reinterpret_cast<const f32x4*>(p.src + (((int64_t)img * p.IH + iy) * p.IW + ix) * p.C + c4);
    }
  };
  auto stash = [&](int tile) {
    int img0, oy0, ox0;
    origin(tile, img0, oy0, ox0);
#pragma unroll
    for (int it = 0; it < PIT; ++it) {
      const int q = tid + it * 256;
      if (q < PQ) {
        const int row = q / CQ;
        f32x4 v = pv[it];
        if (bn) {
          const int im = row / (PH * PW), rr = row % (PH * PW);
          const int iy = oy0 - 1 + rr / PW, ix = ox0 - 1 + rr % PW;
          if (img0 + im < p.NF && iy >= 0 && iy < p.IH && ix >= 0 && ix < p.IW) {
#pragma unroll
            for (int e = 0; e < 4; ++e) v[e] = relu_nan(fmaf(v[e], sc[e], sh[e]));
          }
        }
        *reinterpret_cast<f32x4*>(patch + row * PROW + c4) = v;
      }
    }
  };

  const int col = n0 + j;
  const float bj = (FWD && col < p.N) ? p.bias[col] : 0.f;
  float s1 = 0.f, s2 = 0.f;
  if (t0 < t1) fetch(t0);
  for (int tile = t0; tile < t1; ++tile) {
    __syncthreads();  // weights staged / the previous tile's reads of the patch are done
    stash(tile);
    __syncthreads();
    if (tile + 1 < t1) fetch(tile + 1);
    f32x16 acc;
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[r] = 0.f;
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      const float* ap = abase + ((t / 3) * PW + (t % 3)) * PROW;
      const float* bp = bbase + t * PC;
#pragma unroll
      for (int kk = 0; kk < PC / 8; ++kk) {
        const f32x4 a4 = *reinterpret_cast<const f32x4*>(ap + kk * 8);
        const f32x4 b4 = *reinterpret_cast<const f32x4*>(bp + kk * 8);
        acc = mfma32(a4[0], b4[0], acc);
        acc = mfma32(a4[1], b4[1], acc);
        acc = mfma32(a4[2], b4[2], acc);
        acc = mfma32(a4[3], b4[3], acc);
      }
    }
    int img0, oy0, ox0;
    origin(tile, img0, oy0, ox0);
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
  }
  if (FWD) {
    s1 += __shfl_xor(s1, 32, 64);
    s2 += __shfl_xor(s2, 32, 64);
    __syncthreads();
    float* red = sm;
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
static int launch_patch_persist(PatchArgs a, hipStream_t st, int* nparts) {
  a.tiles_h = (int)cdiv(a.OH, TH);
  a.tiles_w = (int)cdiv(a.OW, TW);
  const int ntiles = (int)(cdiv(a.NF, NI) * a.tiles_h * a.tiles_w);
  const int ny = (int)cdiv(a.N, 32);
  const int target = std::max(1, 512 / ny);  // 2 resident blocks per CU over 256 CUs
  const int tpb = (int)cdiv(ntiles, target);
  const int gx = (int)cdiv(ntiles, tpb);
  VAD_KLAUNCH((conv3x3_patch_persist_kernel<NI, TH, TW, FWD>), dim3(gx, ny), dim3(256), 0, st, a, tpb, ntiles);
  VAD_LAUNCH_CHECK();
  if (nparts) *nparts = gx;
  return 0;
}

template <int S, int NI, int TH, int TW, int PC, bool FWD>
static int launch_patch(PatchArgs a, hipStream_t st, int* nparts) {
  a.tiles_h = (int)cdiv(a.OH, TH);
  a.tiles_w = (int)cdiv(a.OW, TW);
  const int64_t gx = cdiv(a.NF, NI) * a.tiles_h * a.tiles_w;
  dim3 grid((unsigned)gx, (unsigned)cdiv(a.N, 32));
  VAD_KLAUNCH((conv3x3_patch_kernel<S, NI, TH, TW, PC, FWD>), grid, dim3(256), 0, st, a);
  VAD_LAUNCH_CHECK();
  if (nparts) *nparts = (int)gx;
  return 0;
}

int g_patch_persist = 1;  // tuning knob "conv_patch_persist"

// tile geometry per output size (128 pixels per block): 0 -> 2 images x 8x8, 1 -> 8x16, 2 -> 4x32
static int patch_geom(int OH, int OW) { return (OH <= 8 && OW <= 8) ? 0 : (OW <= 16 ? 1 : 2); }

// stride 1: 32-channel chunks; stride 2 (4x the patch pixels): 16-channel chunks keep 2 blocks per CU
template <int S, bool FWD>
static int dispatch_patch(const PatchArgs& a, hipStream_t st, int* nparts) {
  constexpr int PC = S == 1 ? 32 : 16;
  if (S == 1 && a.C == 32 && g_patch_persist) {
    switch (patch_geom(a.OH, a.OW)) {
      case 0: return launch_patch_persist<2, 8, 8, FWD>(a, st, nparts);
      case 1: return launch_patch_persist<1, 8, 16, FWD>(a, st, nparts);
      default: return launch_patch_persist<1, 4, 32, FWD>(a, st, nparts);
    }
  }
  switch (patch_geom(a.OH, a.OW)) {
    case 0: return launch_patch<S, 2, 8, 8, PC, FWD>(a, st, nparts);
    case 1: return launch_patch<S, 1, 8, 16, PC, FWD>(a, st, nparts);
    default: return launch_patch<S, 1, 4, 32, PC, FWD>(a, st, nparts);
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
  if (L.stride != 1 && L.stride != 2) return false;
  return fwd ? L.Ci % 16 == 0 && (L.stride == 2 || L.Ci % 32 == 0) : L.Co % 32 == 0;
}

int conv3_patch_fwd(const Conv3Layer& L, const float* src, const float* src_stats, const float* wf, const float* bias,
                    float* y, float* partials, int* nparts, hipStream_t st) {
  VAD_CHECK(conv3_patch_supported(L, true), "conv3_patch_fwd: unsupported stride / channel count");
  PatchArgs a{};
  a.src = src;
  a.scale = src_stats ? src_stats + 2 * L.Ci : nullptr;
  a.shift = src_stats ? src_stats + 3 * L.Ci : nullptr;
  a.w = wf;
  a.bias = bias;
  a.out = y;
  a.partials = partials;
  a.NF = L.NF; a.IH = L.IH; a.IW = L.IW; a.C = L.Ci; a.OH = L.OH; a.OW = L.OW; a.N = L.Co;
  return L.stride == 1 ? dispatch_patch<1, true>(a, st, nparts) : dispatch_patch<2, true>(a, st, nparts);
}

// wd: [Ci][9][Co] with the original tap order (conv3_prep_weights writes this layout for every stride while the
// patch path is on)
int conv3_patch_dgrad(const Conv3Layer& L, const float* dY, const float* wd, float* dX, hipStream_t st) {
  VAD_CHECK(conv3_patch_supported(L, false), "conv3_patch_dgrad: unsupported stride / channel count");
  PatchArgs a{};
  a.src = dY;
  a.w = wd;
  a.out = dX;
  a.NF = L.NF; a.IH = L.OH; a.IW = L.OW; a.C = L.Co; a.OH = L.IH; a.OW = L.IW; a.N = L.Ci;
  if (L.stride == 1) return dispatch_patch<1, false>(a, st, nullptr);
  a.tiles_h = (int)cdiv(cdiv(L.IH, 2), 8);
  a.tiles_w = (int)cdiv(cdiv(L.IW, 2), 8);
  dim3 grid((unsigned)((int64_t)L.NF * a.tiles_h * a.tiles_w), (unsigned)cdiv(L.Ci, 32));
  VAD_KLAUNCH((conv3x3_dgrad_s2_kernel<32>), grid, dim3(256), 0, st, a);
  VAD_LAUNCH_CHECK();
  return 0;
}

// =====================================================================================================
// Weight gradient: dW[co][t][ci] = sum_p dY[p][co] * relu(bn(x))[p + off_t][ci].
// Block = (32 co) x (9 taps x 32 ci) over a strided subset of 128-pixel tiles (split-K over pixels, split index
// blockIdx.z).  Per tile it stages dY [128 px][32 co] and the input patch [patch px][32 ci] (BN+ReLU on load)
// in LDS; wave w takes pixels [32w, 32w+32) as the MFMA K dimension (2 per step) and keeps all 9 tap tiles in
// registers (one A read feeds 9 MFMAs).  The 4 waves are combined in a fixed order through LDS and the block's
// sum lands in slab z of the [S][co][t*Ci + ci] split-K layout that conv3_wgrad_reduce consumes.
// Stride 2: patch columns are stored de-interleaved by parity so consecutive output pixels read consecutive
// patch rows (conflict-free b32 reads).
// =====================================================================================================
struct WgradPatchArgs {
  const float* dY;     // [NF][OH][OW][Co]
  const float* src;    // [NF][IH][IW][Ci]
  const float* scale;  // BN+ReLU on load, nullable
  const float* shift;
  float* slab;         // [S][Co][9*Ci]
  int NF, IH, IW, Ci, OH, OW, Co;
  int tiles_h, tiles_w, ntiles;
};

template <int S, int NI, int TH, int TW, int WPX>
__global__ __launch_bounds__(256, 2) void conv3x3_wgrad_patch_kernel(const WgradPatchArgs p) {
  static_assert(NI * TH * TW == 4 * WPX, "a tile holds 4 waves x WPX output pixels");
  constexpr int TPX = 4 * WPX;  // pixels per tile
  constexpr int PH = (TH - 1) * S + 3, PW = (TW - 1) * S + 3, PROWS = NI * PH * PW;
  constexpr int PWE = (PW + 1) / 2;  // stride 2: even columns first
  constexpr int XF = PROWS * 32, YF = TPX * 32, RF = 2 * 9 * 16 * 64;
  constexpr int LF = (XF + YF) > RF ? (XF + YF) : RF;
  __shared__ __attribute__((aligned(16))) float sm[LF];
  float* xs = sm;
  float* ys = sm + XF;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int co0 = blockIdx.x * 32, ci0 = blockIdx.y * 32;
  const int h = lane >> 5, j = lane & 31;
  const int tiles_per_img = p.tiles_h * p.tiles_w;
  const int c4 = (tid & 7) * 4;

  f32x16 acc[9];
#pragma unroll
  for (int t = 0; t < 9; ++t)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[t][r] = 0.f;

  constexpr int PIT = (PROWS * 8 + 255) / 256, YIT = TPX * 8 / 256;
  f32x4 pv[PIT], yv[YIT];
  int img0 = 0, oy0 = 0, ox0 = 0;
  auto tile_origin = [&](int tile, int& i0, int& y0, int& x0) {
    i0 = (tile / tiles_per_img) * NI;
    const int tr = tile % tiles_per_img;
    y0 = (tr / p.tiles_w) * TH;
    x0 = (tr % p.tiles_w) * TW;
  };
  auto fetch = [&](int tile) {
    int i0, y0, x0;
    tile_origin(tile, i0, y0, x0);
#pragma unroll
    for (int it = 0; it < YIT; ++it) {
      const int m = (tid >> 3) + it * 32;
      const int mi = m / (TH * TW), mr = m % (TH * TW);
      const int oy = y0 + mr / TW, ox = x0 + mr % TW, img = i0 + mi;
      yv[it] = f32x4{0.f, 0.f, 0.f, 0.f};
      if (img < p.NF && oy < p.OH && ox < p.OW)
        yv[it] = *reinterpret_cast<const f32x4*>(p.dY + (((int64_t)img * p.OH + oy) * p.OW + ox) * p.Co + co0 + c4);
    }
#pragma unroll
    for (int it = 0; it < PIT; ++it) {
      const int row = (tid >> 3) + it * 32;
      const int im = row / (PH * PW), rr = row % (PH * PW);
      const int iy = y0 * S - 1 + rr / PW, ix = x0 * S - 1 + rr % PW, img = i0 + im;
      pv[it] = f32x4{0.f, 0.f, 0.f, 0.f};
      if (row < PROWS && img < p.NF && iy >= 0 && iy < p.IH && ix >= 0 && ix < p.IW)
        pv[it] = *reinterpret_cast<const f32x4*>(p.src + (((int64_t)img * p.IH + iy) * p.IW + ix) * p.Ci + ci0 + c4);
    }
  };
  f32x4 sc = {1.f, 1.f, 1.f, 1.f}, sh = {0.f, 0.f, 0.f, 0.f};
  if (p.scale) {
    sc = *reinterpret_cast<const f32x4*>(p.scale + ci0 + c4);
    sh = *reinterpret_cast<const f32x4*>(p.shift + ci0 + c4);
  }
  auto stash = [&]() {
#pragma unroll
    for (int it = 0; it < YIT; ++it) *reinterpret_cast<f32x4*>(ys + ((tid >> 3) + it * 32) * 32 + c4) = yv[it];
#pragma unroll
    for (int it = 0; it < PIT; ++it) {
      const int row = (tid >> 3) + it * 32;
      if (row < PROWS) {
        const int im = row / (PH * PW), rr = row % (PH * PW);
        const int py = rr / PW, px = rr % PW;
        const int iy = oy0 * S - 1 + py, ix = ox0 * S - 1 + px;
        f32x4 v = pv[it];
        if (p.scale && img0 + im < p.NF && iy >= 0 && iy < p.IH && ix >= 0 && ix < p.IW) {
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] = fmaxf(fmaf(v[e], sc[e], sh[e]), 0.f);
        }
        const int col = S == 1 ? px : ((px & 1) ? PWE + (px >> 1) : (px >> 1));
        *reinterpret_cast<f32x4*>(xs + ((im * PH + py) * PW + col) * 32 + c4) = v;
      }
    }
  };

  int tile = blockIdx.z;
  if (tile < p.ntiles) fetch(tile);
  for (; tile < p.ntiles; tile += gridDim.z) {
    tile_origin(tile, img0, oy0, ox0);
    __syncthreads();
    stash();
    __syncthreads();
    if (tile + (int)gridDim.z < p.ntiles) fetch(tile + gridDim.z);
#pragma unroll 4
    for (int s2 = 0; s2 < WPX / 2; ++s2) {
      const int m = wave * WPX + 2 * s2 + h;
      const int mi = m / (TH * TW), mr = m % (TH * TW);
      const int py = mr / TW, px = mr % TW;
      const float a = ys[m * 32 + j];
      const float* xb = xs + ((mi * PH + py * S) * PW) * 32 + j;
#pragma unroll
      for (int t = 0; t < 9; ++t) {
        const int kh = t / 3, kw = t % 3;
        const int col = S == 1 ? px + kw : ((kw & 1) ? PWE + px + (kw >> 1) : px + (kw >> 1));
        const float b = xb[(kh * PW + col) * 32];
        acc[t] = mfma32(a, b, acc[t]);
      }
    }
  }

  // fixed-order combine of the 4 waves: (2,3) -> (0,1), then 1 -> 0
  __syncthreads();
  float* red = sm;
  if (wave >= 2) {
#pragma unroll
    for (int t = 0; t < 9; ++t)
#pragma unroll
      for (int r = 0; r < 16; ++r) red[(((wave - 2) * 9 + t) * 16 + r) * 64 + lane] = acc[t][r];
  }
  __syncthreads();
  if (wave < 2) {
#pragma unroll
    for (int t = 0; t < 9; ++t)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[t][r] += red[((wave * 9 + t) * 16 + r) * 64 + lane];
  }
  __syncthreads();
  if (wave == 1) {
#pragma unroll
    for (int t = 0; t < 9; ++t)
#pragma unroll
      for (int r = 0; r < 16; ++r) red[(t * 16 + r) * 64 + lane] = acc[t][r];
  }
  __syncthreads();
  if (wave == 0) {
    float* out = p.slab + (int64_t)blockIdx.z * p.Co * 9 * p.Ci;
#pragma unroll
    for (int t = 0; t < 9; ++t)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int co = co0 + (r & 3) + 8 * (r >> 2) + 4 * h;
        out[(int64_t)co * 9 * p.Ci + t * p.Ci + ci0 + j] = acc[t][r] + red[(t * 16 + r) * 64 + lane];
      }
  }
}

template <int S, int NI, int TH, int TW, int WPX = 32>
static int launch_wgrad_patch(WgradPatchArgs a, int target_blocks, int64_t partial_cap, hipStream_t st,
                              int* nsplit) {
  a.tiles_h = (int)cdiv(a.OH, TH);
  a.tiles_w = (int)cdiv(a.OW, TW);
  a.ntiles = (int)(cdiv(a.NF, NI) * a.tiles_h * a.tiles_w);
  const int pairs = (a.Co / 32) * (a.Ci / 32);
  int64_t z = std::max<int64_t>(1, std::min<int64_t>(cdiv(target_blocks, pairs), a.ntiles));
  z = std::min<int64_t>(z, std::max<int64_t>(1, partial_cap / ((int64_t)a.Co * 9 * a.Ci)));
  dim3 grid((unsigned)(a.Co / 32), (unsigned)(a.Ci / 32), (unsigned)z);
  VAD_KLAUNCH((conv3x3_wgrad_patch_kernel<S, NI, TH, TW, WPX>), grid, dim3(256), 0, st, a);
  VAD_LAUNCH_CHECK();
  *nsplit = (int)z;
  return 0;
}

bool conv3_wgrad_patch_supported(const Conv3Layer& L) {
  return (L.stride == 1 || L.stride == 2) && L.Ci % 32 == 0 && L.Co % 32 == 0;
}

int conv3_wgrad_patch(const Conv3Layer& L, const float* dY, const float* src, const float* src_stats, float* slab,
                      int* nsplit, int64_t partial_cap, int target_blocks, hipStream_t st) {
  VAD_CHECK(conv3_wgrad_patch_supported(L), "conv3_wgrad_patch: stride 1/2, Ci and Co multiples of 32");
  VAD_CHECK(partial_cap >= (int64_t)L.Co * 9 * L.Ci, "conv3_wgrad_patch: slab capacity below one split");
  WgradPatchArgs a{};
  a.dY = dY;
  a.src = src;
  a.scale = src_stats ? src_stats + 2 * L.Ci : nullptr;
  a.shift = src_stats ? src_stats + 3 * L.Ci : nullptr;
  a.slab = slab;
  a.NF = L.NF; a.IH = L.IH; a.IW = L.IW; a.Ci = L.Ci; a.OH = L.OH; a.OW = L.OW; a.Co = L.Co;
  const int g = patch_geom(L.OH, L.OW);
  if (L.stride == 1) {
    if (g == 0) return launch_wgrad_patch<1, 2, 8, 8>(a, target_blocks, partial_cap, st, nsplit);
    if (g == 1) return launch_wgrad_patch<1, 1, 8, 16>(a, target_blocks, partial_cap, st, nsplit);
    return launch_wgrad_patch<1, 1, 4, 32>(a, target_blocks, partial_cap, st, nsplit);
  }
  // stride 2: 64-pixel tiles (16 per wave) keep the ~4x larger input patch at 2 waves per SIMD
  if (g == 0) return launch_wgrad_patch<2, 1, 8, 8, 16>(a, target_blocks, partial_cap, st, nsplit);
  if (g == 1) return launch_wgrad_patch<2, 1, 4, 16, 16>(a, target_blocks, partial_cap, st, nsplit);
  return launch_wgrad_patch<2, 1, 2, 32, 16>(a, target_blocks, partial_cap, st, nsplit);
}

}  // namespace vad
