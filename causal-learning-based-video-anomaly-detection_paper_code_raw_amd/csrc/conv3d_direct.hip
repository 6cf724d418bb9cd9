// Direct Conv3d (kernel 3, stride 1, padding 1) for the small-channel 3-D CNNs (minicausal SimpleVideoAnomalyDetector,
// mc:36-57: 1 -> 8 -> 16 -> 32 channels).  With 1-16 input and 8-32 output channels an im2col matrix is 27x the
// activation it is built from and the GEMM over it runs 8-32-wide MFMA tiles mostly empty; these kernels read the
// activation once into LDS instead and accumulate on the vector ALUs (fp32 FMA, exact-f32 products like the GEMM).
//
//   conv3d_direct_fwd   : block = 2 x 8 x 16 output voxels (one per thread) x all CO output channels; the 4 x 10 x 18
//                         input halo of 8 input channels at a time in LDS channel-major (lanes read consecutive
//                         voxels: no bank conflicts) and that chunk's [ci][tap][co] weights (16-B broadcast reads).
//                         The input gradient is the same kernel over dY with the flipped, transposed weights.
//   conv3d_direct_wgrad : block = the same voxel tiles, persistent; each thread owns one (ci, tap) pair (or the bias
//                         pair) x all CO, the dY tile's rows are broadcast reads; per-block partials in a slab, summed
//                         over blocks in a fixed order by a second kernel (deterministic).
#include <algorithm>

#include "conv3d.h"

namespace vad {

int g_conv3d_direct = 1;  // knob "conv3d_direct": the minicausal convs on these kernels (0: im2col + GEMM)
int g_conv3d_wg_blocks = 512;  // knob "conv3d_wgrad_blocks": weight-gradient blocks (512: config 1 3.06 -> 3.01 ms over 256, profiles/r04_conv3d_wgrad_blocks_ab.json)

constexpr int DT_D = 2, DT_H = 8, DT_W = 16;                                   // output tile: 256 voxels
constexpr int HD = DT_D + 2, HH = DT_H + 2, HW = DT_W + 2, HALO = HD * HH * HW;  // 4 x 10 x 18 = 720
constexpr int CIB = 8;                                                          // input channels per chunk
constexpr int WG_CI = 16;                                                       // weight gradient: Ci <= 16

struct DirectArgs {
  const float* src;
  Strides5 s;
  Vol5 in;            // in.C = input channels
  const float* w;     // [Ci][27][CoT]
  const float* bias;  // [CoT] (nullable)
  float* out;         // NDHWC [N][D][H][W][CoT]
  int CoT;            // output channels in all; block row blockIdx.y computes [CO * y, CO * y + CO)
  int tiles_d, tiles_h, tiles_w, ntiles;
};

__device__ __forceinline__ void tile_origin(int tile, int tiles_d, int tiles_h, int tiles_w, int& n, int& d0, int& h0,
                                            int& w0) {
  const int bw = tile % tiles_w;
  int r = tile / tiles_w;
  const int bh = r % tiles_h;
  r /= tiles_h;
  const int bd = r % tiles_d;
  n = r / tiles_d;
  d0 = bd * DT_D;
  h0 = bh * DT_H;
  w0 = bw * DT_W;
}

// stage channels [c0, c0 + cn) of the tile's input halo into xs[ci][HALO] (zero outside the volume)
__device__ __forceinline__ void stage_halo(float* xs, const float* src, const Strides5& s, const Vol5& in, int n,
                                           int d0, int h0, int w0, int c0, int cn, int tid) {
  const bool cl = s.c == 1;  // channels-last source: channel fastest across lanes (coalesced)
  for (int q = tid; q < cn * HALO; q += 256) {
    const int ci = cl ? q % cn : q / HALO, hv = cl ? q / cn : q % HALO;
    const int hd = hv / (HH * HW), hh = (hv / HW) % HH, hw = hv % HW;
    const int d = d0 - 1 + hd, h = h0 - 1 + hh, w = w0 - 1 + hw;
    float v = 0.f;
    if (d >= 0 && d < in.D && h >= 0 && h < in.H && w >= 0 && w < in.W)
      v = src[n * s.n + (int64_t)(c0 + ci) * s.c + d * s.d + h * s.h + w * s.w];
    xs[ci * HALO + hv] = v;
  }
}

template <int CO>
__global__ __launch_bounds__(256) void conv3d_direct_kernel(const DirectArgs p) {
  __shared__ float xs[CIB * HALO];
  __shared__ __attribute__((aligned(16))) float ws[CIB * 27 * CO];
  const int tid = threadIdx.x;
  const int tw = tid % DT_W, th = (tid / DT_W) % DT_H, td = tid / (DT_W * DT_H);
  const int Ci = p.in.C, co0 = blockIdx.y * CO;
  for (int tile = blockIdx.x; tile < p.ntiles; tile += gridDim.x) {
    int n, d0, h0, w0;
    tile_origin(tile, p.tiles_d, p.tiles_h, p.tiles_w, n, d0, h0, w0);
    float acc[CO];
#pragma unroll
    for (int c = 0; c < CO; ++c) acc[c] = 0.f;
    for (int c0 = 0; c0 < Ci; c0 += CIB) {
      const int cn = min(CIB, Ci - c0);
      __syncthreads();  // the previous chunk's (or tile's) LDS reads are done
      stage_halo(xs, p.src, p.s, p.in, n, d0, h0, w0, c0, cn, tid);
      for (int q = tid; q < cn * 27 * CO; q += 256)
        ws[q] = p.w[(int64_t)(c0 * 27 + q / CO) * p.CoT + co0 + q % CO];  // ([ci][tap] rows of CO)
      __syncthreads();
      for (int ci = 0; ci < cn; ++ci) {
        const float* xb = xs + ci * HALO + (td * HH + th) * HW + tw;
        const float* wb = ws + ci * 27 * CO;
#pragma unroll
        for (int t = 0; t < 27; ++t) {
          const float x = xb[((t / 9) * HH + (t / 3) % 3) * HW + t % 3];
#pragma unroll
          for (int c4 = 0; c4 < CO; c4 += 4) {
            const f32x4 w4 = *reinterpret_cast<const f32x4*>(wb + t * CO + c4);
#pragma unroll
            for (int e = 0; e < 4; ++e) acc[c4 + e] = fmaf(x, w4[e], acc[c4 + e]);
          }
        }
      }
    }
    const int d = d0 + td, h = h0 + th, w = w0 + tw;
    if (d < p.in.D && h < p.in.H && w < p.in.W) {
      float* o = p.out + ((((int64_t)n * p.in.D + d) * p.in.H + h) * p.in.W + w) * p.CoT + co0;
#pragma unroll
      for (int c4 = 0; c4 < CO; c4 += 4) {
        f32x4 v = {acc[c4], acc[c4 + 1], acc[c4 + 2], acc[c4 + 3]};
        if (p.bias) {
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] += p.bias[co0 + c4 + e];
        }
        *reinterpret_cast<f32x4*>(o + c4) = v;
      }
    }
  }
}

// torch Conv3d weight [Co][Ci][27] -> wf [Ci][27][Co] (forward) and wd [Co][27][Ci] with the taps flipped (the input
// gradient as a forward conv over dY)
__global__ __launch_bounds__(256) void conv3d_direct_prep_kernel(const float* __restrict__ w, int Co, int Ci,
                                                                 float* __restrict__ wf, float* __restrict__ wd) {
  const int total = Co * Ci * 27;
  for (int i = blockIdx.x * 256 + threadIdx.x; i < total; i += gridDim.x * 256) {
    const int co = i / (Ci * 27), rem = i % (Ci * 27), ci = rem / 27, t = rem % 27;
    const float v = w[i];
    wf[(ci * 27 + t) * Co + co] = v;
    wd[(co * 27 + 26 - t) * Ci + ci] = v;
  }
}

struct DirectWgradArgs {
  const float* dy;  // NDHWC [N][D][H][W][CO]
  const float* src;
  Strides5 s;
  Vol5 in;      // the forward input (in.C = Ci <= WG_CI)
  float* slab;  // [gridDim.x][(Ci*27 + 1) * CO]
  int tiles_d, tiles_h, tiles_w, ntiles;
};

// pairs = Ci*27 + 1 bias pair; more than 256: block row blockIdx.y owns pairs [256 y, 256 y + 256)
template <int CO>
__global__ __launch_bounds__(256) void conv3d_direct_wgrad_kernel(const DirectWgradArgs p) {
  constexpr int MP = 1;
  __shared__ float xs[WG_CI * HALO];
  __shared__ __attribute__((aligned(16))) float dys[256 * CO];
  const int tid = threadIdx.x;
  const int Ci = p.in.C, P = Ci * 27 + 1;
  const int S = P <= 256 ? 256 / P : 1;      // voxel slices (threads of slice k own the pairs, voxels v % S == k)
  const int slice = P <= 256 ? tid / P : 0;  // (slice >= S: idle thread)
  int xoff[MP];                              // per owned pair: ci*HALO + tap offset, -1 = bias pair, -2 = none
#pragma unroll
  for (int m = 0; m < MP; ++m) {
    const int pair = P <= 256 ? tid % P : tid + 256 * (int)blockIdx.y;
    if (slice >= S || pair >= P) xoff[m] = -2;
    else if (pair == P - 1) xoff[m] = -1;
    else {
      const int ci = pair / 27, t = pair % 27;
      xoff[m] = ci * HALO + ((t / 9) * HH + (t / 3) % 3) * HW + t % 3;
    }
  }
  float acc[MP][CO];
#pragma unroll
  for (int m = 0; m < MP; ++m)
#pragma unroll
    for (int c = 0; c < CO; ++c) acc[m][c] = 0.f;
  for (int tile = blockIdx.x; tile < p.ntiles; tile += gridDim.x) {
    int n, d0, h0, w0;
    tile_origin(tile, p.tiles_d, p.tiles_h, p.tiles_w, n, d0, h0, w0);
    __syncthreads();
    stage_halo(xs, p.src, p.s, p.in, n, d0, h0, w0, 0, Ci, tid);
    {
      const int td = tid / (DT_W * DT_H), th = (tid / DT_W) % DT_H, tw = tid % DT_W;
      const int d = d0 + td, h = h0 + th, w = w0 + tw;
      const bool ok = d < p.in.D && h < p.in.H && w < p.in.W;
      const float* row = p.dy + ((((int64_t)n * p.in.D + d) * p.in.H + h) * p.in.W + w) * CO;
#pragma unroll
      for (int c4 = 0; c4 < CO; c4 += 4)
        *reinterpret_cast<f32x4*>(dys + tid * CO + c4) =
            ok ? *reinterpret_cast<const f32x4*>(row + c4) : f32x4{0.f, 0.f, 0.f, 0.f};
    }
    __syncthreads();
    if (slice < S) {
      for (int v = slice; v < 256; v += S) {
        const int base = ((v / (DT_W * DT_H)) * HH + (v / DT_W) % DT_H) * HW + v % DT_W;
        f32x4 g[CO / 4];
#pragma unroll
        for (int c4 = 0; c4 < CO / 4; ++c4) g[c4] = *reinterpret_cast<const f32x4*>(dys + v * CO + 4 * c4);
#pragma unroll
        for (int m = 0; m < MP; ++m) {
          const float x = xoff[m] >= 0 ? xs[xoff[m] + base] : (xoff[m] == -1 ? 1.f : 0.f);
#pragma unroll
          for (int c4 = 0; c4 < CO / 4; ++c4)
#pragma unroll
            for (int e = 0; e < 4; ++e) acc[m][4 * c4 + e] = fmaf(x, g[c4][e], acc[m][4 * c4 + e]);
        }
      }
    }
  }
  float* slab = p.slab + (int64_t)blockIdx.x * P * CO;
  if (S == 1) {
#pragma unroll
    for (int m = 0; m < MP; ++m) {
      const int pair = P <= 256 ? tid : tid + 256 * (int)blockIdx.y;
      if (xoff[m] != -2)
#pragma unroll
        for (int c = 0; c < CO; ++c) slab[pair * CO + c] = acc[m][c];
    }
    return;
  }
  // several slices: their partials combine in slice order through LDS ([slice][pair][co] in the dY tile's space)
  __syncthreads();
  if (slice < S)
#pragma unroll
    for (int c = 0; c < CO; ++c) dys[(slice * P + tid % P) * CO + c] = acc[0][c];
  __syncthreads();
  for (int q = tid; q < P * CO; q += 256) {
    float v = 0.f;
    for (int k = 0; k < S; ++k) v += dys[k * P * CO + q];
    slab[q] = v;
  }
}

// dW[co][ci][t] = sum over blocks of slab[b][(ci*27 + t)*CO + co]; db[co] likewise from the bias pair.  Block =
// 64 outputs x 4 block groups (group g sums blocks g, g + 4, ...), the 4 group sums added in order (deterministic)
__global__ __launch_bounds__(256) void conv3d_direct_wgrad_reduce_kernel(const float* __restrict__ slab, int nblk,
                                                                         int Ci, int CO, float* __restrict__ dW,
                                                                         float* __restrict__ db) {
  __shared__ float red[4][64];
  const int P = Ci * 27 + 1, total = P * CO;
  const int q = blockIdx.x * 64 + threadIdx.x % 64, grp = threadIdx.x / 64;
  float v = 0.f;
  if (q < total) {  // blocks grp, grp + 4, ... in order, 8 loads in flight (clamped indices, unconditional loads)
    const int n = nblk > grp ? (nblk - grp + 3) / 4 : 0;
    for (int k0 = 0; k0 < n; k0 += 8) {
      float u[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) u[k] = slab[(int64_t)(grp + 4 * min(k0 + k, n - 1)) * total + q];
#pragma unroll
      for (int k = 0; k < 8; ++k)
        if (k0 + k < n) v += u[k];
    }
  }
  red[grp][threadIdx.x % 64] = v;
  __syncthreads();
  if (grp == 0 && q < total) {
    const int l = threadIdx.x;
    v = (red[0][l] + red[1][l]) + (red[2][l] + red[3][l]);
    const int pair = q / CO, co = q % CO;
    if (pair == P - 1) {
      if (db) db[co] = v;
    } else {
      dW[(co * Ci + pair / 27) * 27 + pair % 27] = v;
    }
  }
}

static void direct_tiles(const Vol5& v, int& td, int& th, int& tw, int& nt) {
  td = (int)cdiv(v.D, DT_D);
  th = (int)cdiv(v.H, DT_H);
  tw = (int)cdiv(v.W, DT_W);
  nt = v.N * td * th * tw;
}

bool conv3d_direct_supported(int Ci, int Co) {
  return g_conv3d_direct && Ci >= 1 && Ci <= WG_CI && (Co == 8 || Co == 16 || Co == 32);
}

int conv3d_direct_prep(const float* w, int Co, int Ci, float* wf, float* wd, hipStream_t st) {
  const int total = Co * Ci * 27;
  hipLaunchKernelGGL(conv3d_direct_prep_kernel, dim3((unsigned)std::min<int64_t>(cdiv(total, 256), 256)), dim3(256), 0,
                     st, w, Co, Ci, wf, wd);
  VAD_LAUNCH_CHECK();
  return 0;
}

int conv3d_direct_fwd(const float* src, const Strides5& s, const Vol5& in, const float* w, int CO, const float* bias,
                      float* out, hipStream_t st) {
  VAD_CHECK(CO == 8 || CO == 16 || CO == 32, "conv3d_direct_fwd: output channels 8, 16 or 32");
  VAD_CHECK(in.C >= 1 && in.numel() < (1ll << 31) && in.voxels() * CO < (1ll << 31),
            "conv3d_direct_fwd: volume too large for 32-bit voxel offsets");
  DirectArgs a{};
  a.src = src;
  a.s = s;
  a.in = in;
  a.w = w;
  a.bias = bias;
  a.out = out;
  a.CoT = CO;
  direct_tiles(in, a.tiles_d, a.tiles_h, a.tiles_w, a.ntiles);
  if (a.ntiles == 0) return 0;
  // few tiles (small volumes): the output channels split over block rows so the grid still covers the CUs
  const int split = (a.ntiles < 256 && CO >= 16) ? 2 : 1, cb = CO / split;
  const dim3 grid((unsigned)std::min(a.ntiles, 2048), (unsigned)split);
  if (cb == 8) hipLaunchKernelGGL(conv3d_direct_kernel<8>, grid, dim3(256), 0, st, a);
  else if (cb == 16) hipLaunchKernelGGL(conv3d_direct_kernel<16>, grid, dim3(256), 0, st, a);
  else hipLaunchKernelGGL(conv3d_direct_kernel<32>, grid, dim3(256), 0, st, a);
  VAD_LAUNCH_CHECK();
  return 0;
}

int64_t conv3d_direct_wgrad_slab_floats(const Vol5& in, int CO) {
  int td, th, tw, nt;
  direct_tiles(in, td, th, tw, nt);
  return (int64_t)std::min(nt, std::max(1, g_conv3d_wg_blocks)) * (in.C * 27 + 1) * CO;
}

int conv3d_direct_wgrad(const float* dy, int CO, const float* src, const Strides5& s, const Vol5& in, float* dW,
                        float* db, float* slab, int64_t slab_floats, hipStream_t st) {
  VAD_CHECK(in.C >= 1 && in.C <= WG_CI && (CO == 8 || CO == 16 || CO == 32),
            "conv3d_direct_wgrad: Ci <= 16 and Co in {8, 16, 32}");
  VAD_CHECK(in.voxels() * CO < (1ll << 31), "conv3d_direct_wgrad: volume too large for 32-bit voxel offsets");
  DirectWgradArgs a{};
  a.dy = dy;
  a.src = src;
  a.s = s;
  a.in = in;
  a.slab = slab;
  direct_tiles(in, a.tiles_d, a.tiles_h, a.tiles_w, a.ntiles);
  const int nblk = std::min(a.ntiles, std::max(1, g_conv3d_wg_blocks));
  const int P = in.C * 27 + 1;
  VAD_CHECK((int64_t)nblk * P * CO <= slab_floats, "conv3d_direct_wgrad: slab too small");
  if (nblk == 0) return 0;
  VAD_CHECK(P <= 1024, "conv3d_direct_wgrad: more than 1024 (ci, tap) pairs");
  const dim3 grid((unsigned)nblk, (unsigned)(P > 256 ? cdiv(P, 256) : 1));
  if (CO == 8) hipLaunchKernelGGL(conv3d_direct_wgrad_kernel<8>, grid, dim3(256), 0, st, a);
  else if (CO == 16) hipLaunchKernelGGL(conv3d_direct_wgrad_kernel<16>, grid, dim3(256), 0, st, a);
  else hipLaunchKernelGGL(conv3d_direct_wgrad_kernel<32>, grid, dim3(256), 0, st, a);
  VAD_LAUNCH_CHECK();
  hipLaunchKernelGGL(conv3d_direct_wgrad_reduce_kernel, dim3((unsigned)cdiv(P * CO, 64)), dim3(256), 0, st, slab, nblk,
                     in.C, CO, dW, db);
  VAD_LAUNCH_CHECK();
  return 0;
}

}  // namespace vad
