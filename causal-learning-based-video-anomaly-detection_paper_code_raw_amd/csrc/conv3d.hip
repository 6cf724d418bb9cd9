// 3-D building blocks (see conv3d.h): im2col / col2im, fused act + MaxPool3d and its gather backward, adaptive
// average pooling, BatchNorm forward partial sums.  All are HBM-streaming kernels with one thread per written
// element (coalesced writes, gathered reads that hit L2 for the 27-tap windows).
#include <algorithm>

#include "conv3d.h"

namespace vad {

Conv3dGeom conv3d_geom(const Vol5& in, int Co, int k, int s_d, int s_h, int s_w, int pad) {
  Conv3dGeom g{};
  g.in = in;
  g.Co = Co;
  g.kd = g.kh = g.kw = k;
  g.sd = s_d;
  g.sh = s_h;
  g.sw = s_w;
  g.pd = g.ph = g.pw = pad;
  g.OD = (in.D + 2 * pad - k) / s_d + 1;
  g.OH = (in.H + 2 * pad - k) / s_h + 1;
  g.OW = (in.W + 2 * pad - k) / s_w + 1;
  return g;
}

__device__ __forceinline__ float act_of(float v, const float* scale, const float* shift, int relu, int c) {
  if (scale) v = fmaf(v, scale[c], shift[c]);
  return (relu || scale) ? relu_nan(v) : v;
}

// one thread per column element; k fastest so the cols writes are coalesced.  I = int when every index fits 31 bits
// (the index arithmetic is most of this kernel's work: 64-bit divisions cost several times the 32-bit ones)
template <typename I>
__global__ __launch_bounds__(256) void im2col3d_kernel(const float* __restrict__ src, Strides5 s, Conv3dGeom g,
                                                       const float* __restrict__ scale,
                                                       const float* __restrict__ shift, int relu,
                                                       float* __restrict__ cols) {
  const int K = g.K(), taps = g.kd * g.kh * g.kw, khw = g.kh * g.kw;
  const I total = (I)(g.rows() * K);
  for (I i = blockIdx.x * 256 + threadIdx.x; i < total; i += (I)gridDim.x * 256) {
    const I row = i / K;
    const int k = (int)(i - row * K);
    const int ci = k / taps, t = k - ci * taps;
    const int kd = t / khw, kh = (t - kd * khw) / g.kw, kw = t % g.kw;
    I r = row;
    const int ow = (int)(r % g.OW);
    r /= g.OW;
    const int oh = (int)(r % g.OH);
    r /= g.OH;
    const int od = (int)(r % g.OD);
    const int n = (int)(r / g.OD);
    const int d = od * g.sd - g.pd + kd, h = oh * g.sh - g.ph + kh, w = ow * g.sw - g.pw + kw;
    float v = 0.f;
    if (d >= 0 && d < g.in.D && h >= 0 && h < g.in.H && w >= 0 && w < g.in.W)
      v = act_of(src[n * s.n + ci * s.c + d * s.d + h * s.h + w * s.w], scale, shift, relu, ci);
    cols[i] = v;
  }
}

int im2col3d(const float* src, const Strides5& s, const Conv3dGeom& g, const float* scale, const float* shift,
             int relu, float* cols, hipStream_t st) {
  const int64_t total = g.rows() * g.K();
  if (total == 0) return 0;
  const dim3 grid((unsigned)std::min<int64_t>(cdiv(total, 256), 16384));
  if (total + (int64_t)grid.x * 256 < (1ll << 31))
    hipLaunchKernelGGL(im2col3d_kernel<int>, grid, dim3(256), 0, st, src, s, g, scale, shift, relu, cols);
  else
    hipLaunchKernelGGL(im2col3d_kernel<int64_t>, grid, dim3(256), 0, st, src, s, g, scale, shift, relu, cols);
  VAD_LAUNCH_CHECK();
  return 0;
}

// one thread per source element (NDHWC): gather the taps that read it
template <typename I>
__global__ __launch_bounds__(256) void col2im3d_kernel(const float* __restrict__ dcols, Conv3dGeom g,
                                                       const float* __restrict__ bias, float* __restrict__ dsrc) {
  const int K = g.K(), taps = g.kd * g.kh * g.kw, C = g.in.C;
  const I total = (I)g.in.numel();
  for (I i = blockIdx.x * 256 + threadIdx.x; i < total; i += (I)gridDim.x * 256) {
    const int c = (int)(i % C);
    I r = i / C;
    const int w = (int)(r % g.in.W);
    r /= g.in.W;
    const int h = (int)(r % g.in.H);
    r /= g.in.H;
    const int d = (int)(r % g.in.D);
    const int n = (int)(r / g.in.D);
    float acc = 0.f;
    for (int kd = 0; kd < g.kd; ++kd) {
      const int td = d + g.pd - kd;
      if (td < 0 || td % g.sd) continue;
      const int od = td / g.sd;
      if (od >= g.OD) continue;
      for (int kh = 0; kh < g.kh; ++kh) {
        const int th = h + g.ph - kh;
        if (th < 0 || th % g.sh) continue;
        const int oh = th / g.sh;
        if (oh >= g.OH) continue;
        for (int kw = 0; kw < g.kw; ++kw) {
          const int tw = w + g.pw - kw;
          if (tw < 0 || tw % g.sw) continue;
          const int ow = tw / g.sw;
          if (ow >= g.OW) continue;
          const I row = (((I)n * g.OD + od) * g.OH + oh) * g.OW + ow;
          acc += dcols[row * K + c * taps + (kd * g.kh + kh) * g.kw + kw];
        }
      }
    }
    dsrc[i] = bias ? acc + bias[c] : acc;
  }
}

int col2im3d(const float* dcols, const Conv3dGeom& g, float* dsrc, hipStream_t st, const float* bias) {
  const int64_t total = g.in.numel();
  if (total == 0) return 0;
  const dim3 grid((unsigned)std::min<int64_t>(cdiv(total, 256), 16384));
  if (g.rows() * g.K() < (1ll << 31) && total + (int64_t)grid.x * 256 < (1ll << 31))
    hipLaunchKernelGGL(col2im3d_kernel<int>, grid, dim3(256), 0, st, dcols, g, bias, dsrc);
  else
    hipLaunchKernelGGL(col2im3d_kernel<int64_t>, grid, dim3(256), 0, st, dcols, g, bias, dsrc);
  VAD_LAUNCH_CHECK();
  return 0;
}

__global__ __launch_bounds__(256) void conv3d_prep_w3_kernel(const float* __restrict__ w, int N, int C,
                                                             float* __restrict__ w3) {
  const int64_t total = (int64_t)N * C * 27;
  for (int64_t i = blockIdx.x * 256ll + threadIdx.x; i < total; i += (int64_t)gridDim.x * 256) {
    const int c = (int)(i % C);
    int64_t r = i / C;
    const int t = (int)(r % 9);
    r /= 9;
    const int n = (int)(r % N);
    const int kd = (int)(r / N);
    w3[i] = w[((int64_t)n * C + c) * 27 + kd * 9 + t];
  }
}

int conv3d_prep_w3(const float* w, int N, int C, float* w3, hipStream_t st) {
  const int64_t total = (int64_t)N * C * 27;
  hipLaunchKernelGGL(conv3d_prep_w3_kernel, dim3((unsigned)std::min<int64_t>(cdiv(total, 256), 2048)), dim3(256), 0,
                     st, w, N, C, w3);
  VAD_LAUNCH_CHECK();
  return 0;
}

// ------------------------------------------------------------------ MaxPool3d (kernel == stride)
__device__ __forceinline__ float pool_act(const float* y, const float* stats, int relu, int C, int c, int64_t idx) {
  float v = y[idx];
  if (stats) return relu_nan(fmaf(v, stats[2 * C + c], stats[3 * C + c]));
  return relu ? relu_nan(v) : v;
}

__global__ __launch_bounds__(256) void maxpool3d_fwd_kernel(const float* __restrict__ y,
                                                            const float* __restrict__ stats, int relu, Vol5 v, int kd,
                                                            int kh, int kw, float* __restrict__ out) {
  const int OD = v.D / kd, OH = v.H / kh, OW = v.W / kw, C = v.C;
  const int64_t total = (int64_t)v.N * OD * OH * OW * C;
  for (int64_t i = blockIdx.x * 256ll + threadIdx.x; i < total; i += (int64_t)gridDim.x * 256) {
    const int c = (int)(i % C);
    int64_t r = i / C;
    const int ow = (int)(r % OW);
    r /= OW;
    const int oh = (int)(r % OH);
    r /= OH;
    const int od = (int)(r % OD);
    const int n = (int)(r / OD);
    float m = -INFINITY;
    for (int a = 0; a < kd; ++a)
      for (int b = 0; b < kh; ++b)
        for (int e = 0; e < kw; ++e) {
          const int64_t idx = ((((int64_t)n * v.D + od * kd + a) * v.H + oh * kh + b) * v.W + ow * kw + e) * C + c;
          const float val = pool_act(y, stats, relu, C, c, idx);
          if (val > m || isnan(val)) m = val;
        }
    out[i] = m;
  }
}

int maxpool3d_fwd(const float* y, const float* stats, int relu, const Vol5& v, int kd, int kh, int kw, float* out,
                  hipStream_t st) {
  const int64_t total = (int64_t)v.N * (v.D / kd) * (v.H / kh) * (v.W / kw) * v.C;
  if (total == 0) return 0;
  hipLaunchKernelGGL(maxpool3d_fwd_kernel, dim3((unsigned)std::min<int64_t>(cdiv(total, 256), 16384)), dim3(256), 0,
                     st, y, stats, relu, v, kd, kh, kw, out);
  VAD_LAUNCH_CHECK();
  return 0;
}

template <typename I>
__global__ __launch_bounds__(256) void maxpool3d_bwd_kernel(const float* __restrict__ y,
                                                            const float* __restrict__ stats, int relu, Vol5 v, int kd,
                                                            int kh, int kw, const float* __restrict__ dout,
                                                            float* __restrict__ dA) {
  const int OD = v.D / kd, OH = v.H / kh, OW = v.W / kw, C = v.C;
  const I total = (I)v.numel();
  for (I i = blockIdx.x * 256 + threadIdx.x; i < total; i += (I)gridDim.x * 256) {
    const int c = (int)(i % C);
    I r = i / C;
    const int w = (int)(r % v.W);
    r /= v.W;
    const int h = (int)(r % v.H);
    r /= v.H;
    const int d = (int)(r % v.D);
    const int n = (int)(r / v.D);
    const int od = d / kd, oh = h / kh, ow = w / kw;
    float g = 0.f;
    if (od < OD && oh < OH && ow < OW) {
      // first max of the window in (d, h, w) scan order (torch max_pool3d CPU: val > max || isnan(val))
      float m = -INFINITY;
      I arg = -1;
      for (int a = 0; a < kd; ++a)
        for (int b = 0; b < kh; ++b)
          for (int e = 0; e < kw; ++e) {
            const I idx = ((((I)n * v.D + od * kd + a) * v.H + oh * kh + b) * v.W + ow * kw + e) * C + c;
            const float val = pool_act(y, stats, relu, C, c, idx);
            if (arg < 0 || val > m || isnan(val)) {
              m = val;
              arg = idx;
            }
          }
      if (arg == i) g = dout[((((I)n * OD + od) * OH + oh) * OW + ow) * C + c];
    }
    dA[i] = g;
  }
}

// The same backward with one thread per pooling window (output): the window's first max found once, its kd kh kw
// input gradients written together (dout at the max, 0 elsewhere) -- every y value read once instead of once per
// element of its window (the per-element kernel above re-scans the window kd kh kw times).  Input elements outside
// every window (extents not divisible by the window) are cleared first.
template <typename I>
__global__ __launch_bounds__(256) void maxpool3d_bwd_win_kernel(const float* __restrict__ y,
                                                                const float* __restrict__ stats, int relu, Vol5 v,
                                                                int kd, int kh, int kw,
                                                                const float* __restrict__ dout,
                                                                float* __restrict__ dA) {
  const int OD = v.D / kd, OH = v.H / kh, OW = v.W / kw, C = v.C;
  const I total = (I)v.N * OD * OH * OW * C;
  for (I i = blockIdx.x * 256 + threadIdx.x; i < total; i += (I)gridDim.x * 256) {
    const int c = (int)(i % C);
    I r = i / C;
    const int ow = (int)(r % OW);
    r /= OW;
    const int oh = (int)(r % OH);
    r /= OH;
    const int od = (int)(r % OD);
    const int n = (int)(r / OD);
    // first max of the window in (d, h, w) scan order (torch max_pool3d CPU: val > max || isnan(val))
    float m = -INFINITY;
    int arg = -1;
    for (int a = 0; a < kd; ++a)
      for (int b = 0; b < kh; ++b)
        for (int e = 0; e < kw; ++e) {
          const I idx = ((((I)n * v.D + od * kd + a) * v.H + oh * kh + b) * v.W + ow * kw + e) * C + c;
          const float val = pool_act(y, stats, relu, C, c, idx);
          if (arg < 0 || val > m || isnan(val)) {
            m = val;
            arg = (a * kh + b) * kw + e;
          }
        }
    const float g = dout[i];
    for (int a = 0; a < kd; ++a)
      for (int b = 0; b < kh; ++b)
        for (int e = 0; e < kw; ++e) {
          const I idx = ((((I)n * v.D + od * kd + a) * v.H + oh * kh + b) * v.W + ow * kw + e) * C + c;
          dA[idx] = (a * kh + b) * kw + e == arg ? g : 0.f;
        }
  }
}

int g_maxpool_bwd_win = 1;  // knob "maxpool3d_bwd_win": one thread per window (0: one per input element)

int maxpool3d_bwd(const float* y, const float* stats, int relu, const Vol5& v, int kd, int kh, int kw,
                  const float* dout, float* dA, hipStream_t st) {
  const int64_t total = v.numel();
  if (total == 0) return 0;
  if (g_maxpool_bwd_win) {
    const int OD = v.D / kd, OH = v.H / kh, OW = v.W / kw;
    if (OD * kd != v.D || OH * kh != v.H || OW * kw != v.W)
      VAD_HIP(hipMemsetAsync(dA, 0, sizeof(float) * (size_t)total, st));
    const int64_t nw = (int64_t)v.N * OD * OH * OW * v.C;
    if (nw == 0) return 0;
    const dim3 g2((unsigned)std::min<int64_t>(cdiv(nw, 256), 16384));
    if (total + (int64_t)g2.x * 256 < (1ll << 31))
      hipLaunchKernelGGL(maxpool3d_bwd_win_kernel<int>, g2, dim3(256), 0, st, y, stats, relu, v, kd, kh, kw, dout, dA);
    else
      hipLaunchKernelGGL(maxpool3d_bwd_win_kernel<int64_t>, g2, dim3(256), 0, st, y, stats, relu, v, kd, kh, kw, dout,
                         dA);
    VAD_LAUNCH_CHECK();
    return 0;
  }
  const dim3 grid((unsigned)std::min<int64_t>(cdiv(total, 256), 16384));
  if (total + (int64_t)grid.x * 256 < (1ll << 31))
    hipLaunchKernelGGL(maxpool3d_bwd_kernel<int>, grid, dim3(256), 0, st, y, stats, relu, v, kd, kh, kw, dout, dA);
  else
    hipLaunchKernelGGL(maxpool3d_bwd_kernel<int64_t>, grid, dim3(256), 0, st, y, stats, relu, v, kd, kh, kw, dout, dA);
  VAD_LAUNCH_CHECK();
  return 0;
}

// ------------------------------------------------------------------ AdaptiveAvgPool3d
__device__ __forceinline__ int bin_start(int i, int in, int out) { return (int)(((int64_t)i * in) / out); }
__device__ __forceinline__ int bin_end(int i, int in, int out) {
  return (int)(((int64_t)(i + 1) * in + out - 1) / out);
}

// one thread per output (n, c, od, oh, ow); the bin's voxels are summed in (d, h, w) order
__global__ __launch_bounds__(256) void adaptive_avgpool3d_fwd_kernel(const float* __restrict__ x,
                                                                     const float* __restrict__ stats, int relu, Vol5 v,
                                                                     int OD, int OH, int OW, float* __restrict__ out) {
  const int C = v.C, per = OD * OH * OW;
  const int64_t total = (int64_t)v.N * C * per;
  for (int64_t i = blockIdx.x * 256ll + threadIdx.x; i < total; i += (int64_t)gridDim.x * 256) {
    const int n = (int)(i / ((int64_t)C * per));
    const int rem = (int)(i % ((int64_t)C * per));
    const int c = rem / per, o = rem % per;
    const int od = o / (OH * OW), oh = (o / OW) % OH, ow = o % OW;
    const int d0 = bin_start(od, v.D, OD), d1 = bin_end(od, v.D, OD);
    const int h0 = bin_start(oh, v.H, OH), h1 = bin_end(oh, v.H, OH);
    const int w0 = bin_start(ow, v.W, OW), w1 = bin_end(ow, v.W, OW);
    float s = 0.f;
    for (int d = d0; d < d1; ++d)
      for (int h = h0; h < h1; ++h)
        for (int w = w0; w < w1; ++w)
          s += pool_act(x, stats, relu, C, c, ((((int64_t)n * v.D + d) * v.H + h) * v.W + w) * C + c);
    out[i] = s / (float)((d1 - d0) * (h1 - h0) * (w1 - w0));
  }
}

// one block per output bin (n, od, oh, ow): 64 channel lanes x 4 voxel groups, the NDHWC channel rows read
// coalesced; each thread sums every 4th voxel of the bin in (d, h, w) order, the 4 partial sums combine in a fixed
// order (large bins: the one-thread-per-output kernel above reads a stride-C column per thread)
__global__ __launch_bounds__(256) void adaptive_avgpool3d_bin_kernel(const float* __restrict__ x,
                                                                     const float* __restrict__ stats, int relu,
                                                                     Vol5 v, int OD, int OH, int OW,
                                                                     float* __restrict__ out) {
  const int per = OD * OH * OW, C = v.C;
  const int n = blockIdx.x / per, o = blockIdx.x % per;
  const int od = o / (OH * OW), oh = (o / OW) % OH, ow = o % OW;
  const int d0 = bin_start(od, v.D, OD), d1 = bin_end(od, v.D, OD);
  const int h0 = bin_start(oh, v.H, OH), h1 = bin_end(oh, v.H, OH);
  const int w0 = bin_start(ow, v.W, OW), w1 = bin_end(ow, v.W, OW);
  const int nh = h1 - h0, nw = w1 - w0, nvox = (d1 - d0) * nh * nw;
  const int lane = threadIdx.x & 63, vg = threadIdx.x >> 6;
  __shared__ float red[4][64];
  for (int cb = 0; cb < C; cb += 64) {
    const int c = cb + lane;
    float s = 0.f;
    if (c < C)
      for (int k = vg; k < nvox; k += 4) {
        const int d = d0 + k / (nh * nw), h = h0 + (k / nw) % nh, w = w0 + k % nw;
        s += pool_act(x, stats, relu, C, c, ((((int64_t)n * v.D + d) * v.H + h) * v.W + w) * C + c);
      }
    red[vg][lane] = s;
    __syncthreads();
    if (vg == 0 && c < C)
      out[(int64_t)n * C * per + (int64_t)c * per + o] =
          ((red[0][lane] + red[1][lane]) + (red[2][lane] + red[3][lane])) / (float)nvox;
    __syncthreads();
  }
}

int adaptive_avgpool3d_fwd(const float* x, const float* stats, int relu, const Vol5& v, int OD, int OH, int OW,
                           float* out, hipStream_t st) {
  const int64_t total = (int64_t)v.N * v.C * OD * OH * OW;
  if (total == 0) return 0;
  if ((int64_t)v.D * v.H * v.W >= 64LL * OD * OH * OW) {  // large bins: a block per bin
    hipLaunchKernelGGL(adaptive_avgpool3d_bin_kernel, dim3((unsigned)((int64_t)v.N * OD * OH * OW)), dim3(256), 0, st,
                       x, stats, relu, v, OD, OH, OW, out);
  } else {
    hipLaunchKernelGGL(adaptive_avgpool3d_fwd_kernel, dim3((unsigned)std::min<int64_t>(cdiv(total, 256), 16384)),
                       dim3(256), 0, st, x, stats, relu, v, OD, OH, OW, out);
  }
  VAD_LAUNCH_CHECK();
  return 0;
}

__global__ __launch_bounds__(256) void adaptive_avgpool3d_bwd_kernel(const float* __restrict__ dout, Vol5 v, int OD,
                                                                     int OH, int OW, float* __restrict__ dx,
                                                                     const float* __restrict__ gate) {
  const int C = v.C, per = OD * OH * OW;
  const int64_t total = v.numel();
  for (int64_t i = blockIdx.x * 256ll + threadIdx.x; i < total; i += (int64_t)gridDim.x * 256) {
    const int c = (int)(i % C);
    int64_t r = i / C;
    const int w = (int)(r % v.W);
    r /= v.W;
    const int h = (int)(r % v.H);
    r /= v.H;
    const int d = (int)(r % v.D);
    const int n = (int)(r / v.D);
    float g = 0.f;
    // bins are monotone in the input index: scan the (at most 2) candidates per axis
    for (int od = (int)(((int64_t)d * OD) / v.D); od < OD && bin_start(od, v.D, OD) <= d; ++od) {
      if (d >= bin_end(od, v.D, OD)) continue;
      const int dn = bin_end(od, v.D, OD) - bin_start(od, v.D, OD);
      for (int oh = (int)(((int64_t)h * OH) / v.H); oh < OH && bin_start(oh, v.H, OH) <= h; ++oh) {
        if (h >= bin_end(oh, v.H, OH)) continue;
        const int hn = bin_end(oh, v.H, OH) - bin_start(oh, v.H, OH);
        for (int ow = (int)(((int64_t)w * OW) / v.W); ow < OW && bin_start(ow, v.W, OW) <= w; ++ow) {
          if (w >= bin_end(ow, v.W, OW)) continue;
          const int wn = bin_end(ow, v.W, OW) - bin_start(ow, v.W, OW);
          g += dout[(int64_t)n * C * per + (int64_t)c * per + (od * OH + oh) * OW + ow] / (float)(dn * hn * wn);
        }
      }
    }
    dx[i] = (gate && !(gate[i] > 0.f)) ? 0.f : g;  // (gate: the ReLU backward of gate = y fused)
  }
}

int adaptive_avgpool3d_bwd(const float* dout, const Vol5& v, int OD, int OH, int OW, float* dx, hipStream_t st,
                           const float* gate) {
  const int64_t total = v.numel();
  if (total == 0) return 0;
  hipLaunchKernelGGL(adaptive_avgpool3d_bwd_kernel, dim3((unsigned)std::min<int64_t>(cdiv(total, 256), 16384)),
                     dim3(256), 0, st, dout, v, OD, OH, OW, dx, gate);
  VAD_LAUNCH_CHECK();
  return 0;
}

// ------------------------------------------------------------------ BatchNorm forward partial sums
// Block b sums rows [b*R, (b+1)*R) of Y[M][C]; thread -> (row group, channel quad); fixed-order LDS combine.
__global__ __launch_bounds__(256) void bn_fwd_partials_kernel(const float* __restrict__ y, int64_t M, int C,
                                                              int64_t R, float* __restrict__ partials) {
  __shared__ float red[8][256];
  const int nq = C / 4, groups = 256 / nq;
  const int q = threadIdx.x % nq, g = threadIdx.x / nq, c = q * 4;
  float s1[4] = {0, 0, 0, 0}, s2[4] = {0, 0, 0, 0};
  const int64_t r0 = blockIdx.x * R, r1 = min(M, r0 + R);
  for (int64_t r = r0 + g; r < r1; r += groups) {
    const f32x4 v = *reinterpret_cast<const f32x4*>(y + r * C + c);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      s1[e] += v[e];
      s2[e] = fmaf(v[e], v[e], s2[e]);
    }
  }
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    red[e][threadIdx.x] = s1[e];
    red[4 + e][threadIdx.x] = s2[e];
  }
  __syncthreads();
  for (int idx = threadIdx.x; idx < 2 * C; idx += 256) {
    const int s = idx / C, cc = idx % C, qq = cc / 4, e = cc % 4;
    float acc = 0.f;
    for (int gg = 0; gg < groups; ++gg) acc += red[s * 4 + e][gg * nq + qq];
    partials[(int64_t)blockIdx.x * 2 * C + idx] = acc;
  }
}

static int64_t bn_fwd_rows(int64_t M) { return std::max<int64_t>(256, cdiv(M, 2048)); }
int64_t bn_fwd_partials_blocks(int64_t M) { return cdiv(M, bn_fwd_rows(M)); }

int bn_fwd_partials(const float* y, int64_t M, int C, float* partials, int* nparts, hipStream_t st) {
  VAD_CHECK(C % 4 == 0 && C <= 1024 && 256 % (C / 4) == 0, "bn_fwd_partials: unsupported C");
  const int64_t P = bn_fwd_partials_blocks(M);
  hipLaunchKernelGGL(bn_fwd_partials_kernel, dim3((unsigned)P), dim3(256), 0, st, y, M, C, bn_fwd_rows(M), partials);
  VAD_LAUNCH_CHECK();
  *nparts = (int)P;
  return 0;
}

}  // namespace vad
