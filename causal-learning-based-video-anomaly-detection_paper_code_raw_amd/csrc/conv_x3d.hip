// Weight gradient of the backbone's 3x3 convs (causal_anomaly_detection.py:128-139, the nn.Conv2d of _make_layer;
// its grad in the reference's loss.backward(), cad:688) on PRE-SPLIT operand planes staged by LDS-DMA:
//   dW[co][tap][ci] = sum_p dY[p][co] * relu(bn(x))[p + off(tap)][ci]   (zero padding, stride 1 or 2).
//
// Both operands arrive in HBM as three bf16 planes (hi + mid + lo: planes_split below, conv_x3.hip's split numerics)
// laid out [plane][pixel][channels].  A block stages a tile's dY rows and its input patch with global_load_lds_dwordx4
// only -- no VGPR staging, no BN / split VALU in the kernel -- into the same LDS images as x3_wgrad_tr_kernel
// (conv_x3w.hip: per (16-channel half, plane) an image of 32-B pixel rows, read with ds_read_b64_tr_b16), so the
// fragment reads and the six products per K step are that kernel's.  Padding pieces (halo outside the frame, pixels
// past a ragged tile, patch rows past the patch) are DMA'd from a zero page, so no fix-up pass follows the copies.
//
// Pipeline: NB LDS buffers, the copies of tile i + NB - 1 issued right after the one barrier of tile i, so they land
// while tile i (and i + 1) multiply; a counted s_waitcnt vmcnt before the raw barrier retires exactly the copies of the
// tile about to be read (every wave issues the same number of copies per tile).  One 512-thread block per CU (8 waves,
// 2 per SIMD): wave w owns 16 input channels (w & 1), a co tile of 32 (NCO = 2: (w >> 1) & 1) or a K-step parity
// (NCO = 1, combined in a fixed order at the end), and a tap group (w >> 2: taps 0-4 | 5-8, so the two waves sharing a
// SIMD carry 9 taps between them).  Block -> (co, ci) tile pair and K range: the blocks of one K range (which stage the
// same dY and patch bytes) are numbered consecutively inside one XCD's share of the grid (blocks b, b + 8, ... share an
// XCD under round-robin dispatch: speed only), so the XCD's L2 serves the re-reads.  Each block's sum lands in split-K
// slab z ([Z][Co][9 Ci], conv3_wgrad_reduce).
#include <type_traits>

#include "backbone.h"

namespace vad {

namespace {

typedef __bf16 bfv8d __attribute__((ext_vector_type(8)));
typedef __bf16 bfv4d __attribute__((ext_vector_type(4)));
typedef short s16x4d __attribute__((ext_vector_type(4)));

__device__ __forceinline__ bfv8d trd(const __bf16* a0, const __bf16* a1) {
  typedef __attribute__((address_space(3))) s16x4d lds_s16x4;
  const s16x4d u = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(a0));
  const s16x4d v = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(a1));
  const bfv4d x = __builtin_bit_cast(bfv4d, u), y = __builtin_bit_cast(bfv4d, v);
  return bfv8d{x[0], x[1], x[2], x[3], y[0], y[1], y[2], y[3]};
}

// one LDS-DMA copy (global_load_lds_dwordx4: 16 B per lane from its own address to lds + 16 lane), in inline asm so
// the compiler's wait insertion does not see it: it would otherwise wait for every copy in flight (vmcnt(0)) before
// the next LDS read, i.e. drain the next tiles' copies before this tile's MFMAs.  The kernel retires the copies
// itself with counted waits before its barriers.
__device__ __forceinline__ void dma16(const void* g, const __bf16* lds) {
  // (wave-uniform by construction; readfirstlane tells the compiler, which keeps it in an SGPR for M0)
  const uint32_t l = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)(const __attribute__((address_space(3))) __bf16*)lds);
  asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(g), "s"(l) : "memory", "m0");
}

}  // namespace

// 16-B aligned zeros: the source of every padding piece of the LDS-DMA staging
__device__ __attribute__((aligned(256))) __bf16 g_zero_page[128] = {};

// ---------------------------------------------------------------------------------------------------------------
// fp32 [M][C] -> bf16 planes [3][M][C] (hi, mid, lo; the split of conv_x3.hip / conv_x3w.hip, bit for bit), with the
// producer's BN + ReLU applied first when scale is given (zero padding is the consumer's zero page)
__global__ __launch_bounds__(256) void planes_split_kernel(const float* __restrict__ src, const float* __restrict__ scale,
                                                           const float* __restrict__ shift, int64_t n8, int C,
                                                           int64_t ps, __bf16* __restrict__ dst) {
  const int c = (threadIdx.x % (C / 8)) * 8;  // (the grid stride is a multiple of C / 8: a fixed channel group)
  float sc[8], sh[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    sc[e] = scale ? scale[c + e] : 1.f;
    sh[e] = scale ? shift[c + e] : 0.f;
  }
  for (int64_t i = blockIdx.x * 256ll + threadIdx.x; i < n8; i += (int64_t)gridDim.x * 256) {
    const f32x4 v0 = *reinterpret_cast<const f32x4*>(src + i * 8), v1 = *reinterpret_cast<const f32x4*>(src + i * 8 + 4);
    bfv8d hi, mid, lo;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      float v = e < 4 ? v0[e] : v1[e - 4];
      if (scale) {  // (NaN propagates like torch's relu)
        const float r = fmaf(v, sc[e], sh[e]);
        v = r <= 0.f ? 0.f : r;
      }
      const __bf16 h = (__bf16)v;
      const float r = v - (float)h;
      const __bf16 m = (__bf16)r;
      hi[e] = h;
      mid[e] = m;
      lo[e] = (__bf16)(r - (float)m);
    }
    *reinterpret_cast<bfv8d*>(dst + i * 8) = hi;
    *reinterpret_cast<bfv8d*>(dst + ps + i * 8) = mid;
    *reinterpret_cast<bfv8d*>(dst + 2 * ps + i * 8) = lo;
  }
}

int planes_split(const float* src, const float* stats, int64_t M, int C, __bf16* dst, hipStream_t st) {
  VAD_CHECK(C % 8 == 0 && C >= 8 && C <= 2048 && 256 % (C / 8) == 0, "planes_split: C must be 8 * a power of two");
  const int64_t n8 = M * C / 8;
  const int grid = (int)std::max<int64_t>(1, std::min<int64_t>(cdiv(n8, 256 * 4), 2048));
  hipLaunchKernelGGL(planes_split_kernel, dim3(grid), dim3(256), 0, st, src, stats ? stats + 2 * C : nullptr,
                     stats ? stats + 3 * C : nullptr, n8, C, M * C, dst);
  VAD_LAUNCH_CHECK();
  return 0;
}

// ---------------------------------------------------------------------------------------------------------------
struct DwArgs {
  const __bf16* dy;  // planes [3][NF OH OW][Co]
  const __bf16* x;   // planes [3][NF IH IW][Ci] of relu(bn(x)) (the layer's input as its forward read it)
  float* slab;       // [Z][Co][9 Ci]
  int dy_ps, x_ps;   // plane strides in elements (3 planes < 2^31 elements)
  int NF, IH, IW, Ci, OH, OW, Co;
  int tiles_h, tiles_w, ntiles;
  int P, Z, nco;  // (co tile, ci tile) pairs, K splits, co tiles
};

template <int S, int TH, int TW, int NCO, int NB>
__global__ __launch_bounds__(512, 2) void x3_wgrad_dma_kernel(const DwArgs p) {
  constexpr int TPX = TH * TW, KS = TPX / 32;
  static_assert(TPX % 32 == 0 && TW % 8 == 0 && (NCO == 2 || KS % 2 == 0), "whole K steps (NCO = 1: pairs of them)");
  static_assert(NB == 2 || NB == 3, "two or three LDS buffers");
  constexpr int PH = (TH - 1) * S + 3, PW = (TW - 1) * S + 3, PWE = (PW + 1) / 2, PROWS = PH * PW;
  constexpr int XR = (PROWS + 31) / 32 * 32;  // patch rows, whole DMA instructions
  constexpr int YI = TPX * 16, XI = XR * 16;  // one image: rows x 16 bf16 (32-B rows)
  constexpr int NYI = NCO * 6, NXI = 6;       // images per buffer: dY [co tile][co half][plane], patch [ci half][plane]
  constexpr int BUF = NYI * YI + NXI * XI;
  constexpr int NY = NYI * (TPX / 32), NDMA = NY + NXI * (XR / 32), DW = (NDMA + 7) / 8;
  static_assert(DW >= 2 && NB * BUF * 2 <= 163840, "LDS budget");
  __shared__ __attribute__((aligned(1024))) __bf16 sm[NB * BUF];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int chalf = wave & 1, tg = wave >> 2;
  const int ct = NCO == 2 ? (wave >> 1) & 1 : 0, kq = NCO == 2 ? 0 : (wave >> 1) & 1;
  const int grp = lane >> 4, q4 = (lane & 15) >> 2, p4 = lane & 3;  // transposed-read roles
  const int nb = gridDim.x, b = blockIdx.x;
  const int lin = nb % 8 == 0 ? (b % 8) * (nb / 8) + b / 8 : b;
  const int pair = lin % p.P, z = lin / p.P;
  const int co0 = (pair % p.nco) * 32 * NCO, ci0 = (pair / p.nco) * 32;
  const int tb = (int)((int64_t)z * p.ntiles / p.Z), te = (int)((int64_t)(z + 1) * p.ntiles / p.Z);
  const int count = te - tb;
  const int tiles_per_img = p.tiles_h * p.tiles_w;
  const __bf16* const zp = g_zero_page;

  // copy u of this wave = DMA instruction i = wave + 8u (past the last: its own previous one again, identical bytes):
  // its LDS offset (wave-uniform), this lane's piece geometry (pixel / patch row packed, -1: a padding row) and its
  // channel offset (plane stride included)
  int dsto[DW], geo[DW], cho[DW];
  bool isy[DW];
#pragma unroll
  for (int u = 0; u < DW; ++u) {
    int i = wave + 8 * u;
    if (i >= NDMA) i -= 8;
    const int r = lane >> 1, hp = (lane & 1) * 8;
    if (i < NY) {
      const int img = i / (TPX / 32), rg = i % (TPX / 32);
      const int plane = img % 3, uh = (img / 3) % 2, tct = img / 6;
      const int m = rg * 32 + r;
      isy[u] = true;
      dsto[u] = img * YI + rg * 32 * 16;
      geo[u] = ((m / TW) << 8) | (m % TW);
      cho[u] = plane * p.dy_ps + co0 + tct * 32 + uh * 16 + hp;
    } else {
      const int j = i - NY, img = j / (XR / 32), rg = j % (XR / 32);
      const int plane = img % 3, ch = img / 3;
      const int row = rg * 32 + r, ry = row / PW, scol = row % PW;
      const int rx = S == 1 ? scol : (scol < PWE ? 2 * scol : 2 * (scol - PWE) + 1);
      isy[u] = false;
      dsto[u] = NYI * YI + img * XI + rg * 32 * 16;
      geo[u] = row < PROWS ? (ry << 8) | rx : -1;
      cho[u] = plane * p.x_ps + ci0 + ch * 16 + hp;
    }
  }
  auto issue = [&](int tile, int buf) {
    const int img0 = tile / tiles_per_img, tr = tile % tiles_per_img;
    const int y0 = (tr / p.tiles_w) * TH, x0 = (tr % p.tiles_w) * TW;
    const int iy0 = S * y0 - 1, ix0 = S * x0 - 1;
#pragma unroll
    for (int u = 0; u < DW; ++u) {
      const int g = geo[u], gy = (g >> 8) & 255, gx = g & 255;
      const __bf16* gp;
      if (isy[u]) {  // (wave-uniform)
        const int oy = y0 + gy, ox = x0 + gx;
        const bool ok = oy < p.OH && ox < p.OW;
        gp = ok ? p.dy + (((img0 * p.OH + oy) * p.OW + ox) * p.Co + cho[u]) : zp;
      } else {
        const int iy = iy0 + gy, ix = ix0 + gx;
        const bool ok = g >= 0 && (unsigned)iy < (unsigned)p.IH && (unsigned)ix < (unsigned)p.IW;
        gp = ok ? p.x + (((img0 * p.IH + iy) * p.IW + ix) * p.Ci + cho[u]) : zp;
      }
      dma16(gp, sm + buf * BUF + dsto[u]);
    }
  };

  f32x4 acc[5][2];
#pragma unroll
  for (int t = 0; t < 5; ++t)
#pragma unroll
    for (int v = 0; v < 2; ++v) acc[t][v] = f32x4{0.f, 0.f, 0.f, 0.f};

  // taps [T0, T0 + NT) of this wave over the K steps of one staged tile
  auto compute = [&](auto t0c, auto ntc, int buf) {
    constexpr int T0 = decltype(t0c)::value, NT = decltype(ntc)::value;
    const __bf16* const yb = sm + buf * BUF;
    const __bf16* const xb = yb + NYI * YI;
    // this lane's first pixel of a K step: group grp's block 16 (grp >> 1) + 4 (grp & 1), row q4 of the read
    const int lm = 16 * (grp >> 1) + 4 * (grp & 1) + q4;
#pragma unroll 1
    for (int kk = 0; kk < (NCO == 2 ? KS : KS / 2); ++kk) {
      const int k = NCO == 2 ? kk : 2 * kk + kq;
      const int m = k * 32 + lm;  // read 0; read 1: m + 8
      auto prow = [&](int mm) { return S * (mm / TW) * PW + mm % TW; };  // patch row of tap (0, 0)
      const __bf16* ab = yb + ct * 6 * YI + m * 16 + 4 * p4;
      const __bf16* xb0 = xb + chalf * 3 * XI + prow(m) * 16 + 4 * p4;
      const __bf16* xb1 = xb + chalf * 3 * XI + prow(m + 8) * 16 + 4 * p4;
      bfv8d a[2][3];
#pragma unroll
      for (int v = 0; v < 2; ++v)
#pragma unroll
        for (int q = 0; q < 3; ++q) {
          const __bf16* base = ab + (v * 3 + q) * YI;
          a[v][q] = trd(base, base + 8 * 16);
        }
#pragma unroll
      for (int i = 0; i < NT; ++i) {
        const int t = T0 + i, kh = t / 3, kw = t % 3;
        const int cs = S == 1 ? kw : ((kw & 1) ? PWE + (kw >> 1) : (kw >> 1));
        const int to = (kh * PW + cs) * 16;
        bfv8d bq[3];
#pragma unroll
        for (int q = 0; q < 3; ++q) bq[q] = trd(xb0 + q * XI + to, xb1 + q * XI + to);
        // the six products that reach fp32 resolution, smallest first (a: dY planes hi/mid/lo, b: input planes)
#pragma unroll
        for (int v = 0; v < 2; ++v) {
          f32x4 c = acc[i][v];
          c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[v][2], bq[0], c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[v][1], bq[1], c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[v][0], bq[2], c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[v][1], bq[0], c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[v][0], bq[1], c, 0, 0, 0);
          acc[i][v] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[v][0], bq[0], c, 0, 0, 0);
        }
      }
    }
  };

  // prologue: tiles 0 .. NB - 2 in flight
#pragma unroll
  for (int s = 0; s < NB - 1; ++s)
    if (s < count) issue(tb + s, s);
  for (int it = 0; it < count; ++it) {
    // this wave's copies of tile `it` have landed (those of tile it + 1 may stay in flight), then every wave's have and
    // every wave is done reading the buffer the next issue overwrites
    if (NB == 3 && it + 1 < count) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(DW) : "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    if (it + NB - 1 < count) issue(tb + it + NB - 1, (it + NB - 1) % NB);
    const int buf = it % NB;
    if (tg == 0) compute(std::integral_constant<int, 0>{}, std::integral_constant<int, 5>{}, buf);
    else compute(std::integral_constant<int, 5>{}, std::integral_constant<int, 4>{}, buf);
  }

  // C of a 16x16 tile: lane l, register r -> row (co) 4 (l >> 4) + r, column (ci) l & 15
  float* out = p.slab + (int64_t)z * p.Co * 9 * p.Ci;
  const int cob = co0 + ct * 32 + 4 * grp, cic = ci0 + 16 * chalf + (lane & 15);
  const int T0 = tg ? 5 : 0, NT = tg ? 4 : 5;
  if constexpr (NCO == 1) {  // K parities: waves 2, 3, 6, 7 hand theirs to waves 0, 1, 4, 5 (fixed order)
    float* red = reinterpret_cast<float*>(sm);  // [chalf][tg][5 taps][2][4][64]
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    const int slot = (chalf * 2 + tg) * 40;
    if (kq) {
#pragma unroll
      for (int t = 0; t < 5; ++t)
#pragma unroll
        for (int v = 0; v < 2; ++v)
#pragma unroll
          for (int r = 0; r < 4; ++r) red[(slot + (t * 2 + v) * 4 + r) * 64 + lane] = acc[t][v][r];
    }
    __syncthreads();
    if (kq) return;
#pragma unroll
    for (int t = 0; t < 5; ++t)
#pragma unroll
      for (int v = 0; v < 2; ++v)
#pragma unroll
        for (int r = 0; r < 4; ++r) acc[t][v][r] += red[(slot + (t * 2 + v) * 4 + r) * 64 + lane];
  }
#pragma unroll
  for (int i = 0; i < 5; ++i) {
    if (i >= NT) break;
#pragma unroll
    for (int v = 0; v < 2; ++v)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        out[(int64_t)(cob + 16 * v + r) * 9 * p.Ci + (T0 + i) * p.Ci + cic] = acc[i][v][r];
  }
}

int g_wgrad_dma = 0;           // knob "conv_wgrad_dma": fp32 weight gradients on pre-split planes (x3_wgrad_dma_kernel)
int g_wgrad_dma_blocks = 256;  // knob "conv_wgrad_dma_blocks": target grid (one 512-thread block per CU)
int g_wgrad_dma_nb = 3;        // knob "conv_wgrad_dma_nb": LDS buffers (2 | 3)

bool x3_wgrad_dma_supported(const Conv3Layer& L) {
  const int64_t lim = ((int64_t)1 << 31) / 3 - 64;
  return g_wgrad_dma && !g_conv_bf16 && !g_act_bf16 && (L.stride == 1 || L.stride == 2) && L.Ci % 32 == 0 &&
         L.Co % 32 == 0 && (L.stride == 1 || L.Co % 64 == 0) &&
         (L.stride == 1 || (L.IH >= 2 * L.OH - 1 && L.IW >= 2 * L.OW - 1)) &&
         (int64_t)L.NF * L.OH * L.OW * L.Co < lim && (int64_t)L.NF * L.IH * L.IW * L.Ci < lim && L.OH < 256 &&
         L.OW < 256;
}

template <int S, int TH, int TW, int NCO>
static int dw_launch(DwArgs a, int target_blocks, int64_t partial_cap, hipStream_t st, int* nsplit) {
  a.tiles_h = (int)cdiv(a.OH, TH);
  a.tiles_w = (int)cdiv(a.OW, TW);
  a.ntiles = a.NF * a.tiles_h * a.tiles_w;
  a.nco = a.Co / (32 * NCO);
  a.P = a.nco * (a.Ci / 32);
  int64_t z = std::max<int64_t>(1, std::min<int64_t>(cdiv(target_blocks, a.P), a.ntiles));
  z = std::min<int64_t>(z, std::max<int64_t>(1, partial_cap / ((int64_t)a.Co * 9 * a.Ci)));
  a.Z = (int)z;
  const dim3 grid((unsigned)(a.P * z));
  if (g_wgrad_dma_nb == 2) VAD_KLAUNCH((x3_wgrad_dma_kernel<S, TH, TW, NCO, 2>), grid, dim3(512), 0, st, a);
  else VAD_KLAUNCH((x3_wgrad_dma_kernel<S, TH, TW, NCO, 3>), grid, dim3(512), 0, st, a);
  VAD_LAUNCH_CHECK();
  *nsplit = (int)z;
  return 0;
}

int x3_wgrad_dma(const Conv3Layer& L, const __bf16* dy_planes, const __bf16* x_planes, float* slab, int* nsplit,
                 int64_t partial_cap, int target_blocks, hipStream_t st) {
  VAD_CHECK(x3_wgrad_dma_supported(L), "x3_wgrad_dma: unsupported layer");
  VAD_CHECK(partial_cap >= (int64_t)L.Co * 9 * L.Ci, "x3_wgrad_dma: slab capacity below one split");
  DwArgs a{};
  a.dy = dy_planes;
  a.x = x_planes;
  a.slab = slab;
  a.dy_ps = (int)((int64_t)L.NF * L.OH * L.OW * L.Co);
  a.x_ps = (int)((int64_t)L.NF * L.IH * L.IW * L.Ci);
  a.NF = L.NF; a.IH = L.IH; a.IW = L.IW; a.Ci = L.Ci; a.OH = L.OH; a.OW = L.OW; a.Co = L.Co;
  const int tb = target_blocks > 0 ? target_blocks : g_wgrad_dma_blocks;
  if (L.stride == 2) return dw_launch<2, 4, 8, 2>(a, tb, partial_cap, st, nsplit);
  if (L.Co % 64 != 0) return dw_launch<1, 4, 16, 1>(a, tb, partial_cap, st, nsplit);
  if (L.OW <= 8) return dw_launch<1, 8, 8, 2>(a, tb, partial_cap, st, nsplit);
  return dw_launch<1, 4, 16, 2>(a, tb, partial_cap, st, nsplit);
}

}  // namespace vad
