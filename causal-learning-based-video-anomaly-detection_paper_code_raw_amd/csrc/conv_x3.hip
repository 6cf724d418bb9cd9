// Direct 3x3 convolutions (forward, stride-1 input gradient) on the bf16 MFMA with fp32 operands split three ways.
//
// Every fp32 operand v is staged in LDS as three bf16 planes hi + mid + lo (hi = bf16(v), mid = bf16(v - hi),
// lo = bf16(v - hi - mid): 24 significant bits, the residuals are exact in fp32).  Per 16-deep K step a wave
// issues the six partial products whose magnitude reaches fp32 resolution (lo*hi, mid*mid, hi*lo, mid*hi,
// hi*mid, hi*hi, smallest first) into one fp32 accumulator; the three dropped products are below 2^-26 of
// |a||b|, so the result carries fp32-level error (each bf16 product is exact, the MFMA sums in fp32).  The bf16
// MFMA (v_mfma_f32_32x32x16_bf16, 32 cycles for 32x32x16) runs 16x the f32 MFMA rate, so six of them deliver
// 2.67x the f32 MFMA throughput at the same numerics class.
//
// Structure (same geometry as conv_patch.hip): a block owns 128 output pixels (NI images x TH x TW) x 32*NT output
// channels and walks its contiguous range of tiles and, per tile, the reduction channels in chunks of PC: per
// (tile, chunk) it stages the input patch (tile + halo, BN+ReLU on load, zero padding) and the weight slice
// [32*NT][9 taps][PC] as split planes, then wave w multiplies pixels [32w, 32w+32) against all 32*NT channels
// with only LDS reads between MFMAs.  LDS rows are padded to an odd number of 16-B units so the b128 fragment
// reads of 16 lanes cover all 64 banks.  The next (tile, chunk)'s global loads are issued before the current one
// is multiplied; single-chunk layers stage the weights once per block.
#include <algorithm>

#include "backbone.h"

namespace vad {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

struct X3Args {
  const float* src;    // NHWC [NF][IH][IW][C]
  const float* scale;  // BN+ReLU on load (forward), nullable
  const float* shift;
  const float* w;      // [N][9][C]
  const float* bias;   // forward only
  float* out;          // NHWC [NF][OH][OW][N]
  float* partials;     // forward: [gridDim.x][2N] BN partial sums
  int NF, IH, IW, C, OH, OW, N;
  int tiles_h, tiles_w, ntiles, tpb;
  int dbg;  // measurement only (knob "conv_split_dbg"): 1 no weight restaging, 2 no patch split, 4 no MFMA,
            // 8 no patch loads -- results are wrong with any bit set
};

__device__ __forceinline__ void split3(const float* v, bf16x8& hi, bf16x8& mid, bf16x8& lo) {
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const __bf16 h = (__bf16)v[e];
    const float r = v[e] - (float)h;
    const __bf16 m = (__bf16)r;
    hi[e] = h;
    mid[e] = m;
    lo[e] = (__bf16)(r - (float)m);
  }
}

__device__ __forceinline__ f32x16 mfma_x3(const bf16x8* a, const bf16x8* b, f32x16 c) {
  c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[2], b[0], c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[1], b[1], c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], b[2], c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[1], b[0], c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], b[1], c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], b[0], c, 0, 0, 0);
  return c;
}

template <int S, int NI, int TH, int TW, int NT, int PC, bool FWD>
__global__ __launch_bounds__(256, 2) void conv3x3_x3_kernel(const X3Args p) {
  static_assert(NI * TH * TW == 128, "a block owns 128 output pixels");
  static_assert(FWD || S == 1, "stride-2 input gradients use conv3x3_dgrad_s2_kernel");
  static_assert(PC % 16 == 0, "16-deep K steps");
  constexpr int NC = 32 * NT, G8 = PC / 8;
  constexpr int PH = (TH - 1) * S + 3, PW = (TW - 1) * S + 3, PROWS = NI * PH * PW, PWE = (PW + 1) / 2;
  constexpr int RP = 3 * PC + 8;   // patch row: 3 planes x PC + 16 B pad (odd number of 16-B units)
  constexpr int WP = 27 * PC + 8;  // weight row: 9 taps x 3 planes x PC + pad
  static_assert(((RP * 2 / 16) & 1) && ((WP * 2 / 16) & 1), "odd 16-B row pitch");
  __shared__ __attribute__((aligned(16))) __bf16 sm[PROWS * RP + NC * WP];
  __bf16* patch = sm;
  __bf16* wl = sm + PROWS * RP;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int h = lane >> 5, j = lane & 31;
  const int tiles_per_img = p.tiles_h * p.tiles_w;
  const int n0 = blockIdx.y * NC;
  const int t0 = blockIdx.x * p.tpb, t1 = min(p.ntiles, t0 + p.tpb);
  const int nch = p.C / PC;

  // this lane's A pixel (MFMA row lane & 31) inside the tile
  const int m = wave * 32 + j;
  const int mi = m / (TH * TW), mr = m % (TH * TW);
  const int py = mr / TW, px = mr % TW;
  const int arow0 = (mi * PH + py * S) * PW;
  const __bf16* bbase = wl + j * WP + 8 * h;

  // staging: thread tid always handles the channel group g8 = tid % G8 (256 % G8 == 0)
  constexpr int PQ = PROWS * G8, PIT = (PQ + 255) / 256;
  constexpr int WQ = NC * 9 * G8, WIT = (WQ + 255) / 256;
  const int g8 = tid % G8;
  f32x4 pv[PIT][2], wv[WIT][2];
  auto origin = [&](int tile, int& img0, int& oy0, int& ox0) {
    img0 = (tile / tiles_per_img) * NI;
    const int tr = tile % tiles_per_img;
    oy0 = (tr / p.tiles_w) * TH;
    ox0 = (tr % p.tiles_w) * TW;
  };
  auto fetch = [&](int tile, int c0, bool weights) {
    int img0, oy0, ox0;
    origin(tile, img0, oy0, ox0);
#pragma unroll
    for (int it = 0; it < PIT; ++it) {
      const int q = tid + it * 256;
      const int row = q / G8;
      const int im = row / (PH * PW), rr = row % (PH * PW);
      const int iy = oy0 * S - 1 + rr / PW, ix = ox0 * S - 1 + rr % PW, img = img0 + im;
      pv[it][0] = pv[it][1] = f32x4{0.f, 0.f, 0.f, 0.f};
      if (!(p.dbg & 8) && q < PQ && img < p.NF && iy >= 0 && iy < p.IH && ix >= 0 && ix < p.IW) {
        const float* s = p.src + (((int64_t)img * p.IH + iy) * p.IW + ix) * p.C + c0 + g8 * 8;
        pv[it][0] = *reinterpret_cast<const f32x4*>(s);
        pv[it][1] = *reinterpret_cast<const f32x4*>(s + 4);
      }
    }
    if (weights) {
#pragma unroll
      for (int it = 0; it < WIT; ++it) {
        const int q = tid + it * 256;
        const int n = q / (9 * G8), t = (q / G8) % 9;
        wv[it][0] = wv[it][1] = f32x4{0.f, 0.f, 0.f, 0.f};
        if (q < WQ && n0 + n < p.N) {
          const float* s = p.w + ((int64_t)(n0 + n) * 9 + (FWD ? t : 8 - t)) * p.C + c0 + g8 * 8;
          wv[it][0] = *reinterpret_cast<const f32x4*>(s);
          wv[it][1] = *reinterpret_cast<const f32x4*>(s + 4);
        }
      }
    }
  };
  auto stash = [&](int tile, int c0, bool weights) {
    int img0, oy0, ox0;
    origin(tile, img0, oy0, ox0);
    const bool bn = FWD && p.scale;
    f32x4 sc[2] = {{1.f, 1.f, 1.f, 1.f}, {1.f, 1.f, 1.f, 1.f}}, sh[2] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
    if (bn) {
      sc[0] = *reinterpret_cast<const f32x4*>(p.scale + c0 + g8 * 8);
      sc[1] = *reinterpret_cast<const f32x4*>(p.scale + c0 + g8 * 8 + 4);
      sh[0] = *reinterpret_cast<const f32x4*>(p.shift + c0 + g8 * 8);
      sh[1] = *reinterpret_cast<const f32x4*>(p.shift + c0 + g8 * 8 + 4);
    }
#pragma unroll
    for (int it = 0; it < PIT; ++it) {
      const int q = tid + it * 256;
      if (q < PQ) {
        const int row = q / G8;
        const int im = row / (PH * PW), rr = row % (PH * PW);
        const int ry = rr / PW, rx = rr % PW;
        float v[8];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          v[e] = pv[it][0][e];
          v[4 + e] = pv[it][1][e];
        }
        if (bn) {
          // zero padding stays zero: padded taps read 0 in the reference's zero-padded relu(bn(y))
          const int iy = oy0 * S - 1 + ry, ix = ox0 * S - 1 + rx;
          if (img0 + im < p.NF && iy >= 0 && iy < p.IH && ix >= 0 && ix < p.IW) {
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              v[e] = relu_nan(fmaf(v[e], sc[0][e], sh[0][e]));
              v[4 + e] = relu_nan(fmaf(v[4 + e], sc[1][e], sh[1][e]));
            }
          }
        }
        const int col = S == 1 ? rx : ((rx & 1) ? PWE + (rx >> 1) : (rx >> 1));
        bf16x8 hi, mid, lo;
        if (p.dbg & 2) {
#pragma unroll
          for (int e = 0; e < 8; ++e) hi[e] = mid[e] = lo[e] = (__bf16)v[e];
        } else {
          split3(v, hi, mid, lo);
        }
        __bf16* d = patch + ((im * PH + ry) * PW + col) * RP + g8 * 8;
        *reinterpret_cast<bf16x8*>(d) = hi;
        *reinterpret_cast<bf16x8*>(d + PC) = mid;
        *reinterpret_cast<bf16x8*>(d + 2 * PC) = lo;
      }
    }
    if (weights) {
#pragma unroll
      for (int it = 0; it < WIT; ++it) {
        const int q = tid + it * 256;
        if (q < WQ) {
          const int n = q / (9 * G8), t = (q / G8) % 9;
          float v[8];
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            v[e] = wv[it][0][e];
            v[4 + e] = wv[it][1][e];
          }
          bf16x8 hi, mid, lo;
          split3(v, hi, mid, lo);
          __bf16* d = wl + n * WP + t * 3 * PC + g8 * 8;
          *reinterpret_cast<bf16x8*>(d) = hi;
          *reinterpret_cast<bf16x8*>(d + PC) = mid;
          *reinterpret_cast<bf16x8*>(d + 2 * PC) = lo;
        }
      }
    }
  };

  float bj[NT], s1[NT], s2[NT];
#pragma unroll
  for (int nt = 0; nt < NT; ++nt) {
    const int col = n0 + nt * 32 + j;
    bj[nt] = (FWD && col < p.N) ? p.bias[col] : 0.f;
    s1[nt] = s2[nt] = 0.f;
  }
  f32x16 acc[NT];
  const int nitems = (t1 - t0) * nch;
  if (nitems > 0) fetch(t0, 0, true);
  for (int item = 0; item < nitems; ++item) {
    const int tile = t0 + item / nch, ch = item % nch, c0 = ch * PC;
    const bool wnow = (nch > 1 && !(p.dbg & 1)) || item == 0;
    __syncthreads();  // the previous item's fragment reads are done
    stash(tile, c0, wnow);
    __syncthreads();
    if (item + 1 < nitems) {
      const int nx = item + 1;
      fetch(t0 + nx / nch, (nx % nch) * PC, nch > 1 && !(p.dbg & 1));
    }
    if (ch == 0) {
#pragma unroll
      for (int nt = 0; nt < NT; ++nt)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[nt][r] = 0.f;
    }
#pragma unroll
    for (int t = 0; t < ((p.dbg & 4) ? 0 : 9); ++t) {
      const int kh = t / 3, kw = t % 3;
      const int col = S == 1 ? px + kw : ((kw & 1) ? PWE + px + (kw >> 1) : px + (kw >> 1));
      const __bf16* ap = patch + (arow0 + kh * PW + col) * RP + 8 * h;
#pragma unroll
      for (int kk = 0; kk < PC / 16; ++kk) {
        bf16x8 a[3], b[NT][3];
#pragma unroll
        for (int q = 0; q < 3; ++q) a[q] = *reinterpret_cast<const bf16x8*>(ap + q * PC + kk * 16);
#pragma unroll
        for (int nt = 0; nt < NT; ++nt)
#pragma unroll
          for (int q = 0; q < 3; ++q)
            b[nt][q] = *reinterpret_cast<const bf16x8*>(bbase + nt * 32 * WP + (t * 3 + q) * PC + kk * 16);
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) acc[nt] = mfma_x3(a, b[nt], acc[nt]);
      }
    }
    if (ch == nch - 1) {
      // row = pixel (r&3) + 8(r>>2) + 4h of the wave's 32, column = channel n0 + 32 nt + j
      int img0, oy0, ox0;
      origin(tile, img0, oy0, ox0);
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int pm = wave * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
        const int qi = pm / (TH * TW), qr = pm % (TH * TW);
        const int oy = oy0 + qr / TW, ox = ox0 + qr % TW, img = img0 + qi;
        if (img < p.NF && oy < p.OH && ox < p.OW) {
          float* o = p.out + (((int64_t)img * p.OH + oy) * p.OW + ox) * p.N + n0 + j;
#pragma unroll
          for (int nt = 0; nt < NT; ++nt) {
            if (n0 + nt * 32 + j < p.N) {
              const float v = acc[nt][r] + bj[nt];
              o[nt * 32] = v;
              if (FWD) {
                s1[nt] += v;
                s2[nt] = fmaf(v, v, s2[nt]);
              }
            }
          }
        }
      }
    }
  }
  if (FWD) {
    __syncthreads();
    float* red = reinterpret_cast<float*>(sm);  // [4 waves][2][NC]
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) {
      const float a1 = s1[nt] + __shfl_xor(s1[nt], 32, 64);
      const float a2 = s2[nt] + __shfl_xor(s2[nt], 32, 64);
      if (lane < 32) {
        red[(wave * 2 + 0) * NC + nt * 32 + lane] = a1;
        red[(wave * 2 + 1) * NC + nt * 32 + lane] = a2;
      }
    }
    __syncthreads();
    for (int q = tid; q < 2 * NC; q += 256) {
      const int which = q / NC, c = q % NC;
      const float v = red[which * NC + c] + red[(2 + which) * NC + c] + red[(4 + which) * NC + c] +
                      red[(6 + which) * NC + c];
      if (n0 + c < p.N) p.partials[(int64_t)blockIdx.x * 2 * p.N + which * p.N + n0 + c] = v;
    }
  }
}

template <int S, int NI, int TH, int TW, int NT, int PC, bool FWD>
static int launch_x3(X3Args a, int max_blocks, hipStream_t st, int* nparts) {
  a.tiles_h = (int)cdiv(a.OH, TH);
  a.tiles_w = (int)cdiv(a.OW, TW);
  a.ntiles = (int)(cdiv(a.NF, NI) * a.tiles_h * a.tiles_w);
  const int ny = (int)cdiv(a.N, 32 * NT);
  const int target = std::max(1, std::min(max_blocks, 512 / ny));  // 2 resident blocks per CU over 256 CUs
  a.tpb = (int)cdiv(a.ntiles, target);
  a.dbg = g_x3_dbg;
  const int gx = (int)cdiv(a.ntiles, a.tpb);
  hipLaunchKernelGGL((conv3x3_x3_kernel<S, NI, TH, TW, NT, PC, FWD>), dim3(gx, ny), dim3(256), 0, st, a);
  VAD_LAUNCH_CHECK();
  if (nparts) *nparts = gx;
  return 0;
}

int g_conv_split = 1;  // tuning knob "conv_split": 1 = split-bf16 patch kernels where supported, 0 = f32 MFMA
int g_x3_nt = 0;       // tuning knob "conv_split_nt": 0 = auto, 1 / 2 = force 32 / 64 output channels per block
int g_x3_dbg = 0;      // knob "conv_split_dbg" (measurement only, see X3Args::dbg)

template <int S, bool FWD, int NT>
static int dispatch_x3_nt(const X3Args& a, int max_blocks, hipStream_t st, int* nparts) {
  const int OH = a.OH, OW = a.OW;
  if (OH <= 8 && OW <= 8) return launch_x3<S, 2, 8, 8, NT, 16, FWD>(a, max_blocks, st, nparts);
  if (OW <= 16) return launch_x3<S, 1, 8, 16, NT, 16, FWD>(a, max_blocks, st, nparts);
  return launch_x3<S, 1, 4, 32, NT, 16, FWD>(a, max_blocks, st, nparts);
}

template <int S, bool FWD>
static int dispatch_x3(const X3Args& a, int max_blocks, hipStream_t st, int* nparts) {
  int nt = g_x3_nt;
  if (nt == 0) {
    // 64 channels per block halves the fragment reads per MFMA; keep 32 when that would leave the chip underfull
    const int64_t tiles = conv3_patch_blocks(a.NF, a.OH, a.OW);
    nt = (a.N % 64 == 0 && tiles * (a.N / 64) >= 512) ? 2 : 1;
  }
  return nt == 2 ? dispatch_x3_nt<S, FWD, 2>(a, max_blocks, st, nparts)
                 : dispatch_x3_nt<S, FWD, 1>(a, max_blocks, st, nparts);
}

bool conv3_x3_supported(const Conv3Layer& L, bool fwd) {
  if (!g_conv_split) return false;
  if (fwd) return (L.stride == 1 || L.stride == 2) && L.Ci % 16 == 0;
  return L.stride == 1 && L.Co % 16 == 0;
}

int conv3_x3_fwd(const Conv3Layer& L, const float* src, const float* src_stats, const float* wf, const float* bias,
                 float* y, float* partials, int* nparts, hipStream_t st) {
  VAD_CHECK(conv3_x3_supported(L, true), "conv3_x3_fwd: unsupported layer");
  X3Args a{};
  a.src = src;
  a.scale = src_stats ? src_stats + 2 * L.Ci : nullptr;
  a.shift = src_stats ? src_stats + 3 * L.Ci : nullptr;
  a.w = wf;
  a.bias = bias;
  a.out = y;
  a.partials = partials;
  a.NF = L.NF; a.IH = L.IH; a.IW = L.IW; a.C = L.Ci; a.OH = L.OH; a.OW = L.OW; a.N = L.Co;
  // BN partial rows are bounded by conv3_patch_blocks (the caller's partial buffer)
  const int max_blocks = (int)std::min<int64_t>(conv3_patch_blocks(L.NF, L.OH, L.OW), 1 << 20);
  return L.stride == 1 ? dispatch_x3<1, true>(a, max_blocks, st, nparts) : dispatch_x3<2, true>(a, max_blocks, st, nparts);
}

int conv3_x3_dgrad(const Conv3Layer& L, const float* dY, const float* wd, float* dX, hipStream_t st) {
  VAD_CHECK(conv3_x3_supported(L, false), "conv3_x3_dgrad: unsupported layer");
  X3Args a{};
  a.src = dY;
  a.w = wd;
  a.out = dX;
  a.NF = L.NF; a.IH = L.OH; a.IW = L.OW; a.C = L.Co; a.OH = L.IH; a.OW = L.IW; a.N = L.Ci;
  return dispatch_x3<1, false>(a, 1 << 20, st, nullptr);
}

}  // namespace vad
