// Weight gradient of the backbone's 3x3 convs (causal_anomaly_detection.py:128-139) for the fp32 configs on the
// split-bf16 MFMA, built on transposed LDS reads:
//   dW[co][tap][ci] = sum_p dY[p][co] * relu(bn(x))[p + off(tap)][ci]   (zero padding, stride 1 or 2).
// GEMM view per tap: M = output channels (A = dY^T), N = input channels (B = the shifted input), K = output pixels;
// fp32 operands are split three ways (hi + mid + lo bf16 planes, the six products whose magnitude reaches fp32
// resolution, smallest first: conv_x3.hip's numerics).  Both operands need 8 consecutive pixels of one channel per
// lane -- the transpose of the NHWC rows the loads deliver -- so the LDS images keep NHWC order, [pixel][32 channels]
// per plane (64-B rows), and the fragments are read with ds_read_b64_tr_b16 (per 16-lane group 4 rows x 16 columns
// delivered column-major), two reads per plane fragment: the staging is one 16-B load + BN/ReLU + split + three 8-B
// LDS stores per 4 channels, no register transposition (conv_x3.hip's weight-gradient kernels spend ~10 VALU per MFMA
// on the transposition and the unaligned column shifts).
// MFMA shape 16x16x32 (K = 32 pixels, 8 per 16-lane group): a wave owns 32 co x 16 ci x 9 taps = 72 accumulator
// registers (a 32x32 tile over 9 taps would take 144 and leave no room for the register prefetch of the next tile at
// 2 waves per SIMD).  Each 16-channel half of a plane is an image of its own with 32-B rows, and group g of a K step
// takes pixels 16 (g >> 1) + 4 (g & 1) + {0..3} (first read) and + 8 (second read): the two groups of a 32-lane half
// then read 8 consecutive rows of one image, 256 contiguous bytes -- conflict-free with no swizzle, so every tap's
// fragment is a constant offset (the ds_read immediate) from one base per K step.  Stride 2: patch columns stored
// parity-split ([even | odd]), so 4 consecutive output pixels read 4 consecutive LDS rows for every tap.
// A block owns NCO co tiles of 32 x 32 input channels and a strided set of pixel tiles (2 blocks per CU); wave w takes
// ci half w & 1 and either co tile w >> 1 (NCO = 2) or K half w >> 1 (NCO = 1, summed in a fixed order).  The block's
// sum lands in split-K slab blockIdx.z ([S][Co][9 Ci], conv3_wgrad_reduce).
#include <algorithm>

#include "backbone.h"

namespace vad {

namespace {

typedef float f32x4w __attribute__((ext_vector_type(4)));
typedef __bf16 bfv8w __attribute__((ext_vector_type(8)));
typedef __bf16 bfv4w __attribute__((ext_vector_type(4)));
typedef short s16x4w __attribute__((ext_vector_type(4)));

__device__ __forceinline__ bfv8w trf(const __bf16* a0, const __bf16* a1) {
  typedef __attribute__((address_space(3))) s16x4w lds_s16x4;
  const s16x4w u = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(a0));
  const s16x4w v = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(a1));
  const bfv4w x = __builtin_bit_cast(bfv4w, u), y = __builtin_bit_cast(bfv4w, v);
  return bfv8w{x[0], x[1], x[2], x[3], y[0], y[1], y[2], y[3]};
}

// 4 fp32 values -> hi / mid / lo bf16 planes (8 B each)
__device__ __forceinline__ void split4(const f32x4 v, bfv4w& hi, bfv4w& mid, bfv4w& lo) {
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const __bf16 h = (__bf16)v[e];
    const float r = v[e] - (float)h;
    const __bf16 m = (__bf16)r;
    hi[e] = h;
    mid[e] = m;
    lo[e] = (__bf16)(r - (float)m);
  }
}

__device__ __forceinline__ void lds_bar() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

}  // namespace

struct TrwArgs {
  const float* dY;     // [NF][OH][OW][Co]
  const float* src;    // [NF][IH][IW][Ci]
  const float* scale;  // BN + ReLU on load (nullable)
  const float* shift;
  float* slab;         // [S][Co][9 Ci]
  int NF, IH, IW, Ci, OH, OW, Co;
  int tiles_h, tiles_w, ntiles;
  int dy_bytes, x_bytes;  // buffer extents (< 2^31)
};

template <int S, int NI, int TH, int TW, int NCO, bool PFT = false>
__global__ __launch_bounds__(256, 2) void x3_wgrad_tr_kernel(const TrwArgs p) {
  constexpr int TPX = NI * TH * TW, KS = TPX / 32, KSW = NCO == 2 ? KS : KS / 2;
  static_assert(TW % 8 == 0 && TPX % 32 == 0 && KS % (3 - NCO) == 0 && (NCO == 1 || NCO == 2), "whole K steps");
  constexpr int PH = (TH - 1) * S + 3, PW = (TW - 1) * S + 3, PWE = (PW + 1) / 2, PROWS = NI * PH * PW;
  // one (16-channel half, plane) image; + 128 B so that the two halves of a store phase land on different banks when
  // that still leaves two blocks per CU (input images: + a junk row for the staging pieces past the patch)
  constexpr int PAD = 12 * (NCO * (TPX * 16 + 64) + (PROWS + 1) * 16 + 64) <= 81920 ? 64 : 0;
  constexpr int YH = TPX * 16 + PAD, XH = (PROWS + 1) * 16 + PAD;
  static_assert(12 * (NCO * YH + XH) <= 81920, "two blocks per CU");
  __shared__ __attribute__((aligned(16))) __bf16 sm[6 * (NCO * YH + XH)];
  __bf16* const ys = sm;                  // [co tile][half][plane][TPX][16]
  __bf16* const xs = sm + 6 * NCO * YH;   // [half][plane][PROWS + 1][16]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int grp = lane >> 4, q4 = (lane & 15) >> 2, p4 = lane & 3;  // transposed-read roles
  const int co0 = blockIdx.x * 32 * NCO, ci0 = blockIdx.y * 32;
  const int tiles_per_img = p.tiles_h * p.tiles_w;
  const int chalf = wave & 1, ct = NCO == 2 ? wave >> 1 : 0, ks0 = NCO == 2 ? 0 : (wave >> 1) * KSW;
  const bool bn = p.scale != nullptr;

  // staging pieces: 4 channels (16 B fp32) of one pixel; thread-constant channel group c4 (256 % 8 == 0): half c4 >> 2,
  // columns 4 (c4 & 3) .. + 3
  constexpr int YQ = TPX * 8 * NCO, YIT = YQ / 256;
  constexpr int XQ = PROWS * 8, XIT = (XQ + 255) / 256;
  static_assert(YQ % 256 == 0, "whole dY staging passes");
  const int c4 = tid & 7, chal = c4 >> 2, ccol = (c4 & 3) * 4;
  f32x4 sc = {1.f, 1.f, 1.f, 1.f}, sh = {0.f, 0.f, 0.f, 0.f};
  if (bn) {
    sc = *reinterpret_cast<const f32x4*>(p.scale + ci0 + c4 * 4);
    sh = *reinterpret_cast<const f32x4*>(p.shift + ci0 + c4 * 4);
  }
  // loop-invariant piece geometry: dY piece it -> (co tile, frame, row, column) of the tile, packed (the co tile is the
  // slowest index); input piece -> (frame, patch row, patch column)
  int ygeo[YIT], xgeo[XIT];
#pragma unroll
  for (int it = 0; it < YIT; ++it) {
    const int q = tid + it * 256, cg = q / (TPX * 8), m = (q % (TPX * 8)) >> 3;
    const int mi = m / (TH * TW), mr = m % (TH * TW);
    ygeo[it] = (cg << 24) | (mi << 16) | ((mr / TW) << 8) | (mr % TW);
  }
#pragma unroll
  for (int it = 0; it < XIT; ++it) {
    const int q = tid + it * 256, row = q >> 3;
    const int mi = row / (PH * PW), rr = row % (PH * PW), ry = rr / PW, rx = rr % PW;
    xgeo[it] = q < XQ ? (mi << 16) | (ry << 8) | rx : -1;
  }

  f32x4w acc[9][2];
#pragma unroll
  for (int t = 0; t < 9; ++t)
#pragma unroll
    for (int u = 0; u < 2; ++u) acc[t][u] = f32x4w{0.f, 0.f, 0.f, 0.f};

  // the next tile's pieces are loaded into registers while this tile's MFMAs run.  Buffer loads with 32-bit offsets
  // (the host keeps every tensor below 2^31 bytes): a piece outside the frames takes an offset past the buffer's end
  // and loads zeros, so every tile issues the same loads with no branches and the counted waits never drain the
  // prefetch; xmask keeps which input pieces are real (BN + ReLU apply to those only)
  constexpr int OOB = 0x7ffffff0;
  const __amdgpu_buffer_rsrc_t ry = __builtin_amdgcn_make_buffer_rsrc((void*)p.dY, (short)0, p.dy_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t rx = __builtin_amdgcn_make_buffer_rsrc((void*)p.src, (short)0, p.x_bytes, 0x00020000);
  f32x4 yv[YIT], xv[XIT];
  int xmask = 0;
  auto fetch = [&](int tile) {
    const int img0 = (tile / tiles_per_img) * NI, tr = tile % tiles_per_img;
    const int y0 = (tr / p.tiles_w) * TH, x0 = (tr % p.tiles_w) * TW;
    const int iy0 = S * y0 - 1, ix0 = S * x0 - 1;
    const int ybase = (((img0 * p.OH + y0) * p.OW + x0) * p.Co + co0 + c4 * 4) * 4;
    const int xbase = (((img0 * p.IH + iy0) * p.IW + ix0) * p.Ci + ci0 + c4 * 4) * 4;
#pragma unroll
    for (int it = 0; it < YIT; ++it) {
      const int g = ygeo[it], cg = g >> 24, mi = (g >> 16) & 255, py = (g >> 8) & 255, px = g & 255;
      const int ok = (img0 + mi < p.NF) & (y0 + py < p.OH) & (x0 + px < p.OW);
      const int off = ybase + ((((mi * p.OH + py) * p.OW + px) * p.Co + cg * 32) << 2);
      yv[it] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(ry, ok ? off : OOB, 0, 0));
    }
    xmask = 0;
#pragma unroll
    for (int it = 0; it < XIT; ++it) {
      const int g = xgeo[it], mi = (g >> 16) & 255, ry_ = (g >> 8) & 255, rx_ = g & 255;
      const int ok = (g >= 0) & (img0 + mi < p.NF) & ((unsigned)(iy0 + ry_) < (unsigned)p.IH) &
                     ((unsigned)(ix0 + rx_) < (unsigned)p.IW);
      const int off = xbase + ((((mi * p.IH + ry_) * p.IW + rx_) * p.Ci) << 2);
      xv[it] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rx, ok ? off : OOB, 0, 0));
      xmask |= ok << it;
    }
  };
  fetch(blockIdx.z);  // (the launch keeps gridDim.z <= ntiles)
  for (int tile = blockIdx.z; tile < p.ntiles; tile += gridDim.z) {
    int ltid = tid;  // (laundered: the stash addresses are recomputed per tile rather than held in registers)
    asm volatile("" : "+v"(ltid));
    lds_bar();  // the previous tile's fragment reads are done
#pragma unroll
    for (int it = 0; it < YIT; ++it) {
      const int q = ltid + it * 256, cg = q / (TPX * 8), m = (q % (TPX * 8)) >> 3;
      bfv4w a, b, c;
      f32x4 dy = yv[it];
      split4(dy, a, b, c);
      __bf16* d = ys + (cg * 2 + chal) * 3 * YH + m * 16 + ccol;
      *reinterpret_cast<bfv4w*>(d) = a;
      *reinterpret_cast<bfv4w*>(d + YH) = b;
      *reinterpret_cast<bfv4w*>(d + 2 * YH) = c;
    }
#pragma unroll
    for (int it = 0; it < XIT; ++it) {
      const int g = xgeo[it];
      const int mi = (g >> 16) & 255, ry_ = (g >> 8) & 255, rx_ = g & 255;
      const int col = S == 1 ? rx_ : ((rx_ & 1) ? PWE + (rx_ >> 1) : (rx_ >> 1));  // stride 2: [even | odd] columns
      f32x4 v = xv[it];
      if (bn) {  // zero padding stays zero (the reference pads relu(bn(y)) with zeros)
        const bool ok = (xmask >> it) & 1;
#pragma unroll
        for (int e = 0; e < 4; ++e) {  // (selects, no branches; NaN propagates like torch's relu)
          const float r = fmaf(v[e], sc[e], sh[e]);
          v[e] = (r <= 0.f || !ok) ? 0.f : r;
        }
      }
      bfv4w a, b, c;
      split4(v, a, b, c);
      // (the pieces past the patch, last pass only, land in the junk row behind the image)
      const int row = (it + 1) * 256 <= XQ || g >= 0 ? (mi * PH + ry_) * PW + col : PROWS;
      __bf16* d = xs + chal * 3 * XH + row * 16 + ccol;
      *reinterpret_cast<bfv4w*>(d) = a;
      *reinterpret_cast<bfv4w*>(d + XH) = b;
      *reinterpret_cast<bfv4w*>(d + 2 * XH) = c;
    }
    lds_bar();
    fetch(min(tile + (int)gridDim.z, p.ntiles - 1));
    // this lane's first pixel of a K step: group grp's block 16 (grp >> 1) + 4 (grp & 1), row q4 of the read
    // (laundered per tile: the fragment bases are recomputed in the loop, not hoisted into registers)
    int lm = 16 * (grp >> 1) + 4 * (grp & 1) + q4;
    asm volatile("" : "+v"(lm));
#pragma unroll
    for (int k = 0; k < KSW; ++k) {
      const int m = (ks0 + k) * 32 + lm;  // read 0; read 1: m + 8
      auto prow = [&](int mm) {            // patch LDS row of tap (0, 0) for tile pixel mm
        const int mi = mm / (TH * TW), mr = mm % (TH * TW);
        return (mi * PH + S * (mr / TW)) * PW + mr % TW;
      };
      const __bf16* ab = ys + ct * 6 * YH + m * 16 + 4 * p4;
      const __bf16* xb0 = xs + chalf * 3 * XH + prow(m) * 16 + 4 * p4;
      const __bf16* xb1 = xs + chalf * 3 * XH + prow(m + 8) * 16 + 4 * p4;
      bfv8w a[2][3];
#pragma unroll
      for (int u = 0; u < 2; ++u)
#pragma unroll
        for (int q = 0; q < 3; ++q) {
          const __bf16* base = ab + (u * 3 + q) * YH;
          a[u][q] = trf(base, base + 8 * 16);
        }
      auto tap_off = [&](int t) {
        const int kh = t / 3, kw = t % 3;
        const int cs = S == 1 ? kw : ((kw & 1) ? PWE + (kw >> 1) : (kw >> 1));
        return (kh * PW + cs) * 16;
      };
      // PFT: tap t + 1's input fragments are read before tap t's MFMAs (one tap of register double-buffering), so a
      // tap's 12 MFMAs do not wait for its own LDS reads
      bfv8w bn[3];
      if constexpr (PFT) {
#pragma unroll
        for (int q = 0; q < 3; ++q) bn[q] = trf(xb0 + q * XH, xb1 + q * XH);
      }
#pragma unroll
      for (int t = 0; t < 9; ++t) {
        const int to = tap_off(t);
        bfv8w b[3];
        if constexpr (PFT) {
#pragma unroll
          for (int q = 0; q < 3; ++q) b[q] = bn[q];
          if (t + 1 < 9) {
            const int tn = tap_off(t + 1);
#pragma unroll
            for (int q = 0; q < 3; ++q) bn[q] = trf(xb0 + q * XH + tn, xb1 + q * XH + tn);
          }
        } else {
#pragma unroll
          for (int q = 0; q < 3; ++q) b[q] = trf(xb0 + q * XH + to, xb1 + q * XH + to);
        }
        // the six products that reach fp32 resolution, smallest first (a: dY planes hi/mid/lo, b: input planes)
#pragma unroll
        for (int u = 0; u < 2; ++u) {
          f32x4w c = acc[t][u];
          c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[u][2], b[0], c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[u][1], b[1], c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[u][0], b[2], c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[u][1], b[0], c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[u][0], b[1], c, 0, 0, 0);
          acc[t][u] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[u][0], b[0], c, 0, 0, 0);
        }
        __builtin_amdgcn_sched_barrier(0);
      }
    }
  }

  // C of a 16x16 tile: lane l, register r -> row (co) 4 (l >> 4) + r, column (ci) l & 15
  float* out = p.slab + (int64_t)blockIdx.z * p.Co * 9 * p.Ci;
  const int cob = co0 + ct * 32 + 4 * grp, cic = ci0 + 16 * chalf + (lane & 15);
  if constexpr (NCO == 1) {  // K halves: waves 2, 3 hand theirs to waves 0, 1 (fixed order)
    float* red = reinterpret_cast<float*>(sm);  // [2 waves][72][64]
    __syncthreads();
    if (wave >= 2) {
#pragma unroll
      for (int t = 0; t < 9; ++t)
#pragma unroll
        for (int u = 0; u < 2; ++u)
#pragma unroll
          for (int r = 0; r < 4; ++r) red[((chalf * 9 + t) * 8 + u * 4 + r) * 64 + lane] = acc[t][u][r];
    }
    __syncthreads();
    if (wave >= 2) return;
#pragma unroll
    for (int t = 0; t < 9; ++t)
#pragma unroll
      for (int u = 0; u < 2; ++u)
#pragma unroll
        for (int r = 0; r < 4; ++r) acc[t][u][r] += red[((chalf * 9 + t) * 8 + u * 4 + r) * 64 + lane];
  }
#pragma unroll
  for (int t = 0; t < 9; ++t)
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
      for (int r = 0; r < 4; ++r) out[(int64_t)(cob + 16 * u + r) * 9 * p.Ci + t * p.Ci + cic] = acc[t][u][r];
}

int g_wgrad_tr = 1;           // knob "conv_wgrad_tr": fp32 weight gradients on x3_wgrad_tr_kernel
int g_wgrad_tr_blocks = 384;  // knob "conv_wgrad_tr_blocks": its target grid (1.5 blocks per CU: they share the CUs with the input gradients)

bool x3_wgrad_tr_supported(const Conv3Layer& L) {
  const int64_t lim = (int64_t)1 << 31;
  return g_wgrad_tr && g_conv_split && !g_conv_bf16 && !g_act_bf16 && (L.stride == 1 || L.stride == 2) &&
         L.Ci % 32 == 0 && L.Co % 32 == 0 && (L.stride == 1 || (L.IH >= 2 * L.OH - 1 && L.IW >= 2 * L.OW - 1)) &&
         (int64_t)L.NF * L.OH * L.OW * L.Co * 4 < lim - 64 && (int64_t)L.NF * L.IH * L.IW * L.Ci * 4 < lim - 64 &&
         L.OH < 256 && L.OW < 256;
}

int g_wgrad_tr_pft = 0;  // knob "conv_wgrad_tr_pft": the next tap's input fragments read before this tap's MFMAs (off:
                         // config-2 step 1.696 ms off vs 1.72-1.74 on, profiles/r05_prefetch_ab.json)

template <int S, int NI, int TH, int TW, int NCO>
static int trw_launch(TrwArgs a, int target_blocks, int64_t partial_cap, hipStream_t st, int* nsplit) {
  a.tiles_h = (int)cdiv(a.OH, TH);
  a.tiles_w = (int)cdiv(a.OW, TW);
  a.ntiles = (int)(cdiv(a.NF, NI) * a.tiles_h * a.tiles_w);
  const int pairs = (a.Co / (32 * NCO)) * (a.Ci / 32);
  int64_t z = std::max<int64_t>(1, std::min<int64_t>(cdiv(target_blocks, pairs), a.ntiles));
  z = std::min<int64_t>(z, std::max<int64_t>(1, partial_cap / ((int64_t)a.Co * 9 * a.Ci)));
  // (stride 2: the second fragment set does not fit beside the parity-split images' registers -- it spills)
  bool launched = false;
  if constexpr (S == 1) {
    if (g_wgrad_tr_pft) {
      VAD_KLAUNCH((x3_wgrad_tr_kernel<S, NI, TH, TW, NCO, true>), dim3(a.Co / (32 * NCO), a.Ci / 32, (unsigned)z),
                  dim3(256), 0, st, a);
      launched = true;
    }
  }
  if (!launched)
    VAD_KLAUNCH((x3_wgrad_tr_kernel<S, NI, TH, TW, NCO, false>), dim3(a.Co / (32 * NCO), a.Ci / 32, (unsigned)z),
                dim3(256), 0, st, a);
  VAD_LAUNCH_CHECK();
  *nsplit = (int)z;
  return 0;
}

int x3_wgrad_tr(const Conv3Layer& L, const float* dY, const float* src, const float* src_stats, float* slab,
                int* nsplit, int64_t partial_cap, int target_blocks, hipStream_t st) {
  VAD_CHECK(x3_wgrad_tr_supported(L), "x3_wgrad_tr: unsupported layer");
  VAD_CHECK(partial_cap >= (int64_t)L.Co * 9 * L.Ci, "x3_wgrad_tr: slab capacity below one split");
  TrwArgs a{};
  a.dY = dY;
  a.src = src;
  a.scale = src_stats ? src_stats + 2 * L.Ci : nullptr;
  a.shift = src_stats ? src_stats + 3 * L.Ci : nullptr;
  a.slab = slab;
  a.NF = L.NF; a.IH = L.IH; a.IW = L.IW; a.Ci = L.Ci; a.OH = L.OH; a.OW = L.OW; a.Co = L.Co;
  a.dy_bytes = (int)((int64_t)L.NF * L.OH * L.OW * L.Co * 4);
  a.x_bytes = (int)((int64_t)L.NF * L.IH * L.IW * L.Ci * 4);
  const int tb = target_blocks > 0 ? target_blocks : g_wgrad_tr_blocks;
  // tiles of 64 pixels (both co tiles of a 64-channel slice share the staged patch) or, for 32-channel layers, 128
  // pixels; at most ~80 KB of LDS so that 2 blocks fit a CU
  const bool c64 = L.Co % 64 == 0;
  if (L.stride == 2) {
    if (L.OW <= 8) return c64 ? trw_launch<2, 1, 8, 8, 2>(a, tb, partial_cap, st, nsplit)
                              : trw_launch<2, 1, 8, 8, 1>(a, tb, partial_cap, st, nsplit);
    return c64 ? trw_launch<2, 1, 4, 16, 2>(a, tb, partial_cap, st, nsplit)
               : trw_launch<2, 1, 4, 16, 1>(a, tb, partial_cap, st, nsplit);
  }
  if (!c64) return trw_launch<1, 1, 8, 16, 1>(a, tb, partial_cap, st, nsplit);
  if (L.OW <= 8 && L.OH <= 8) return trw_launch<1, 1, 8, 8, 2>(a, tb, partial_cap, st, nsplit);
  return trw_launch<1, 1, 4, 16, 2>(a, tb, partial_cap, st, nsplit);
}

}  // namespace vad
