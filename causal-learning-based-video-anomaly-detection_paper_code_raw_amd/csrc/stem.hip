// Frozen-stem forward without the conv1 activation round trip (the training default: train_model freezes
// backbone.conv1 / bn1, cad:592-598, so nothing downstream needs conv1's output, only maxpool(relu(bn1(.))).
//
// One pass: conv1 (1 -> 32, 7x7, s2, p3) + bias, the BN partial sums, and the 3x3 / stride-2 pooling of the RAW
// output y, taken per channel as a max where bn1's gamma >= 0 and as a min where gamma < 0.  bn1+ReLU is applied
// on load by layer1.0's kernels (as for every other layer): z = relu(fma(y, scale, shift)) is monotone in y,
// non-decreasing for scale = gamma * invstd >= 0 and non-increasing for scale < 0, so
//   maxpool(relu(fma(y, s, t))) == relu(fma(gamma >= 0 ? maxpool(y) : minpool(y), s, t))
// exactly (rounding is monotone too), while the batch statistics that set s and t are still being accumulated.
// The 114x114x32 activation (213 MB at config 2) is neither written nor read: the stem reads the input once
// (26 MB) and writes the pooled map (53 MB).
//
// conv1 runs on the bf16 MFMA with both operands split three ways (hi + mid + lo, six products: fp32-class
// numerics, see conv_x3.hip) as a GEMM M = 32 output pixels, N = 32 channels, K = 8 kernel rows x 8 columns (row 7
// and column 7 zero): K step ks covers kernel rows 2ks (lane half 0) and 2ks+1 (half 1), so a lane's 8 A values are
// input columns 2ox-3 .. 2ox+4 of one input row -- four consecutive dwords of a bf16 LDS row (x is staged once per
// band as 3 bf16 planes).  The weights live in 48 registers.  A wave's 32 pixels are conv columns c0-1 .. c0+30 of
// one row (c0 = 30 * tile): a wave folds the three conv rows of a pooled row in registers, and after swapping the
// lane halves every lane holds all 32 values of its channel and takes the 15 horizontal windows (columns 2px-1 ..
// 2px+1) in registers -- no LDS round trip for the pooling.
#include <algorithm>

#include "backbone.h"

namespace vad {

typedef __bf16 bf16x8s __attribute__((ext_vector_type(8)));
typedef unsigned u32x4s __attribute__((ext_vector_type(4)));

namespace {

__device__ __forceinline__ void split3s(float v, __bf16& h, __bf16& m, __bf16& l) {
  h = (__bf16)v;
  const float r = v - (float)h;
  m = (__bf16)r;
  l = (__bf16)(r - (float)m);
}

// B fragments: w[co = lane & 31][kh = 2ks + (lane >> 5)][kw = 0..7], zero outside the 7x7 kernel
__device__ __forceinline__ void stem_weights(const float* __restrict__ w, bf16x8s (&b)[4][3]) {
  const int lane = threadIdx.x & 63, j = lane & 31, h = lane >> 5;
#pragma unroll
  for (int ks = 0; ks < 4; ++ks) {
    const int kh = 2 * ks + h;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float v = (kh < 7 && e < 7) ? w[j * 49 + kh * 7 + e] : 0.f;
      __bf16 hi, mid, lo;
      split3s(v, hi, mid, lo);
      b[ks][0][e] = hi;
      b[ks][1][e] = mid;
      b[ks][2][e] = lo;
    }
  }
}

// staging of input rows [2*c0 - 3, 2*c0 - 3 + rows) x columns [-3, PWb - 3) of a frame as 3 bf16 planes (zero
// padding), in two halves so the global loads of the next band can be in flight during the current one's MFMAs:
// item q = column pair m of row pr, held by thread q % 256 in register slot q / 256
template <int N>  // register slots: rows * PWb / 2 <= N * 256
struct StemRegs {
  static constexpr int items = N;
  float v[N][2];
};

template <class R>
__device__ __forceinline__ void stem_fetch(const float* __restrict__ xi, int H, int W, int c0, int rows, int PWb,
                                           R& r) {
  constexpr int ST_ITEMS = R::items;
  const int half = PWb / 2;
  // q / half by a float reciprocal: q + 0.5 sits >= 0.5 / half away from a multiple of half, far above the
  // rounding error of q * (1 / half) for q < 2^12
  const float inv = 1.f / (float)half;
  // branch-free: clamped (always in-bounds) addresses, out-of-frame taps zeroed by a select, so all loads issue
  // back to back
#pragma unroll
  for (int k = 0; k < ST_ITEMS; ++k) {
    const int q = threadIdx.x + k * 256;
    const int pr = (int)(((float)q + 0.5f) * inv), m = q - pr * half;
    const int ih = 2 * c0 - 3 + pr, iw = 2 * m - 3;
    const bool rok = pr < rows && ih >= 0 && ih < H;
    const int64_t rowo = (int64_t)min(max(ih, 0), H - 1) * W;
    const float a0 = xi[rowo + min(max(iw, 0), W - 1)];
    const float a1 = xi[rowo + min(max(iw + 1, 0), W - 1)];
    r.v[k][0] = (rok && iw >= 0 && iw < W) ? a0 : 0.f;
    r.v[k][1] = (rok && iw + 1 >= 0 && iw + 1 < W) ? a1 : 0.f;
  }
}

template <int NP, class R>
__device__ __forceinline__ void stem_store(const R& r, int rows, int PWb, __bf16* xs) {
  constexpr int ST_ITEMS = R::items;
  typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
  const int half = PWb / 2, plane2 = rows * half;  // plane stride in bf16 pairs
  bf16x2* d = reinterpret_cast<bf16x2*>(xs);
#pragma unroll
  for (int k = 0; k < ST_ITEMS; ++k) {
    const int q = threadIdx.x + k * 256;
    if (q < rows * half) {
      __bf16 h0, m0, l0, h1, m1, l1;
      split3s(r.v[k][0], h0, m0, l0);
      split3s(r.v[k][1], h1, m1, l1);
      const bf16x2 hi = {h0, h1}, mid = {m0, m1}, lo = {l0, l1};
      d[q] = hi;  // q = pr * half + m
      if constexpr (NP == 3) {
        d[q + plane2] = mid;
        d[q + 2 * plane2] = lo;
      }
    }
  }
}

// block = (frame, band of ST_PB pooled rows): conv rows 2*py0-1 .. 2*py1-1 (the first one is the previous band's
// last and is recomputed; rows 2*py0 .. 2*py1-1 are this band's own for the BN sums), per conv row ceil(WP/15)
// tiles of 32 columns.
constexpr int ST_PB = 3;
constexpr int ST_SLOTS = 12;  // input staging register slots: (2 * (2 * ST_PB + 1) + 6) rows * PWb / 2 <= 12 * 256

// NP = 3: split-bf16 operands (fp32 numerics, the default); NP = 1: bf16 operands (conv_bf16, BASELINE config 4);
// AB: the pooled map is stored as bf16 (bf16 activation storage)
//
// A wave item is (pooled row py, tile of 15 pooled columns): the wave computes the tile's 32 conv columns of conv
// rows 2py-1, 2py, 2py+1 (row 2py-1 is also the previous pooled row's; recomputing it is cheaper than sharing it
// through LDS atomics), folds them with a running max in registers, takes the 15 horizontal windows after the lane
// half swap, and writes the pooled values straight to the map (lane = channel: 128 contiguous bytes per column).
// BN sums: rows 2py and 2py+1 are pooled row py's own.
template <int NP, bool AB = false>
__global__ __launch_bounds__(256, 4) void stem_fused_kernel(const float* __restrict__ x, int H, int W,
                                                            const float* __restrict__ w,
                                                            const float* __restrict__ bias,
                                                            const float* __restrict__ gamma, int OH, int OW, int HP,
                                                            int WP, int nbands, int PWb, float* __restrict__ pool,
                                                            float* __restrict__ partials) {
  extern __shared__ __attribute__((aligned(16))) __bf16 smb[];
  constexpr int C = 32;
  const int img = blockIdx.x / nbands, band = blockIdx.x % nbands;
  const int py0 = band * ST_PB, py1 = min(HP, py0 + ST_PB);
  const int c_lo = max(2 * py0 - 1, 0), c_hi = min(2 * py1 - 1, OH - 1), n = c_hi - c_lo + 1;
  const int rows = 2 * n + 6;
  __bf16* xs = smb;
  __shared__ float red[4 * 64];  // [4 waves][2][32] BN partial sums
  bf16x8s b[4][3];
  stem_weights(w, b);
  {
    StemRegs<ST_SLOTS> sr;
    stem_fetch(x + (int64_t)img * H * W, H, W, c_lo, rows, PWb, sr);
    // every input load is issued before the first is consumed: left to itself the scheduler interleaved the split
    // and LDS stores of early slots with the loads of later ones, waiting on the memory system a dozen times
    __builtin_amdgcn_sched_barrier(0);
    stem_store<NP>(sr, rows, PWb, xs);
  }
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, h = lane >> 5, j = lane & 31;
  const float bj = bias[j];
  const float sgn = gamma[j] < 0.f ? -1.f : 1.f;  // this channel pools the minimum (as the maximum of -y)
  const int ntr = (WP + 14) / 15;                  // tiles per pooled row
  act_t<AB>* poolp = reinterpret_cast<act_t<AB>*>(pool);
  __syncthreads();
  float s1 = 0.f, s2 = 0.f;
  const int plane2 = rows * PWb / 2;
  for (int t = wave; t < (py1 - py0) * ntr; t += 4) {
    const int pyl = t / ntr, c0 = 30 * (t - pyl * ntr), py = py0 + pyl;
    // lane pixel: conv column c0 - 1 + (lane & 31) (address clamped; out-of-map columns excluded)
    const int col = c0 - 1 + (lane & 31), colc = min(max(col, 0), OW - 1);
    // D row i (pixel = column c0 - 1 + i) of register r in lane half h: i = (r & 3) + 8 (r >> 2) + 4 h.  Valid
    // columns are i <= ihi (and i >= 1 on the first tile); this tile's own columns for the BN sums are i = 1 .. 30
    const int ihi = min(30, OW - c0), ilo = c0 == 0 ? 1 : 0;
    float v[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) v[r] = -INFINITY;
    for (int dr = -1; dr <= 1; ++dr) {
      const int crow = 2 * py + dr;
      if (crow < 0 || crow >= OH) continue;
      const int rl = crow - c_lo;
      f32x16 acc;
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[r] = 0.f;
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) {
        const unsigned* rowp = reinterpret_cast<const unsigned*>(xs + (2 * rl + 2 * ks + h) * PWb) + colc;
        bf16x8s a[NP];
#pragma unroll
        for (int q = 0; q < NP; ++q) {
          const unsigned* sp = rowp + q * plane2;
          const u32x4s d = {sp[0], sp[1], sp[2], sp[3]};
          a[q] = __builtin_bit_cast(bf16x8s, d);
        }
        if constexpr (NP == 3) {
          acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[2], b[ks][0], acc, 0, 0, 0);
          acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[1], b[ks][1], acc, 0, 0, 0);
          acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], b[ks][2], acc, 0, 0, 0);
          acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[1], b[ks][0], acc, 0, 0, 0);
          acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], b[ks][1], acc, 0, 0, 0);
        }
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], b[ks][0], acc, 0, 0, 0);
      }
      const float own = dr >= 0 ? 1.f : 0.f;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int i = (r & 3) + 8 * (r >> 2) + 4 * h;
        const float y = acc[r] + bj;
        const float m = (i >= 1 && i <= ihi) ? own : 0.f;
        s1 = fmaf(y, m, s1);
        s2 = fmaf(y * y, m, s2);
        v[r] = fmaxf(v[r], (i >= ilo && i <= ihi) ? y * sgn : -INFINITY);  // a max of y (gamma >= 0) or of -y
      }
    }
    // v_permlane32_swap of (v[r], v[r+8]): lane half 0 gets pixels 0..15 in X/Y (its windows 0..7 also need pixel
    // 16 = its own v[8], kept aside), lane half 1 pixels 16..31 -- the same registers for local pixel 16h + l:
    // l -> ((l >> 2) & 1 ? Y : X)[(l & 3) + 4 (l >> 3)], so both halves run one window code path
    const float p16 = v[8];
    float X[8], Y[8];
#pragma unroll
    for (int r = 0; r < 8; ++r) {
      const auto sw = __builtin_amdgcn_permlane32_swap(__float_as_uint(v[r]), __float_as_uint(v[r + 8]), false, false);
      X[r] = __uint_as_float(sw[0]);
      Y[r] = __uint_as_float(sw[1]);
    }
    auto loc = [&](int l) { return l == 16 ? p16 : (((l >> 2) & 1) ? Y : X)[(l & 3) + 4 * (l >> 3)]; };
    const int pxb = 15 * (c0 / 30) + 8 * h;  // window k of this half = pooled column pxb + k
    act_t<AB>* dst = poolp + (((int64_t)img * HP + py) * WP + pxb) * C + j;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const float m = fmaxf(fmaxf(loc(2 * k), loc(2 * k + 1)), loc(2 * k + 2));
      if (k < 8 - h && pxb + k < WP) act_st(dst + k * C, m * sgn);
    }
  }
  s1 += __shfl_xor(s1, 32, 64);
  s2 += __shfl_xor(s2, 32, 64);
  if (lane < 32) {
    red[wave * 64 + lane] = s1;
    red[wave * 64 + 32 + lane] = s2;
  }
  __syncthreads();
  if (threadIdx.x < 64) {
    const int t = threadIdx.x;
    // column-major [64][P] (P = gridDim.x): the finalize then reads each channel's P sums contiguously
    partials[(int64_t)t * gridDim.x + blockIdx.x] = (red[t] + red[64 + t]) + (red[128 + t] + red[192 + t]);
  }
}

}  // namespace

int g_stem_fused = 1;  // tuning knob "stem_fused": the frozen stem's forward without the conv1 activation

static int stem_pitch(int OW) { return (int)cdiv(2 * OW + 6, 8) * 8; }
static size_t stem_lds(int OW) { return (size_t)3 * (2 * (2 * ST_PB + 1) + 6) * stem_pitch(OW) * sizeof(__bf16); }

bool stem_fused_ok(int OW) {
  return OW >= 2 && (2 * (2 * ST_PB + 1) + 6) * stem_pitch(OW) / 2 <= ST_SLOTS * 256 && stem_lds(OW) <= 160 * 1024;
}

int stem_fused(const float* x, int NF, int H, int W, const float* w, const float* b, const float* gamma, int OH,
               int OW, float* pool, int HP, int WP, float* partials, int* nparts, hipStream_t st) {
  VAD_CHECK(OH == (H - 1) / 2 + 1 && OW == (W - 1) / 2 + 1 && HP == (OH - 1) / 2 + 1 && WP == (OW - 1) / 2 + 1,
            "stem_fused: bad dims");
  VAD_CHECK(stem_fused_ok(OW), "stem_fused: frame width");
  const int nbands = (int)cdiv(HP, ST_PB);
  // (the partial rows fit the conv1_fwd layout: ceil(ceil(OH/2)/3) == ceil(OH/6))
  VAD_CHECK(nbands == (int)cdiv(OH, 6) && (int64_t)NF * nbands == conv1_num_parts(NF, OH), "stem_fused: partials");
  VAD_CHECK(!g_act_bf16 || g_conv_bf16, "stem_fused: bf16 activations need conv_bf16");
  if (g_conv_bf16 && g_act_bf16)
    VAD_KLAUNCH((stem_fused_kernel<1, true>), dim3(NF * nbands), dim3(256), stem_lds(OW), st, x, H, W, w, b, gamma, OH,
                OW, HP, WP, nbands, stem_pitch(OW), pool, partials);
  else if (g_conv_bf16)
    VAD_KLAUNCH(stem_fused_kernel<1>, dim3(NF * nbands), dim3(256), stem_lds(OW), st, x, H, W, w, b, gamma, OH, OW,
                HP, WP, nbands, stem_pitch(OW), pool, partials);
  else
    VAD_KLAUNCH(stem_fused_kernel<3>, dim3(NF * nbands), dim3(256), stem_lds(OW), st, x, H, W, w, b, gamma, OH, OW,
                HP, WP, nbands, stem_pitch(OW), pool, partials);
  VAD_LAUNCH_CHECK();
  *nparts = NF * nbands;
  return 0;
}

}  // namespace vad
