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
typedef __bf16 bf16x8d __attribute__((ext_vector_type(8)));
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

// ---------------------------------------------------------------------------------------------------------------
// Stride-2 input gradient (the transpose of cad:128-136's stride-2 nn.Conv2d) on pre-split dY planes and the pre-split
// Wd image, staged by LDS-DMA.  The arithmetic is conv3x3_dgrad_s2x3_kernel's (conv_x3.hip): the four parity classes
// (ph, pw) of a 16x16 dX tile read one 9x9 dY patch, class (ph, pw) taking the kernel rows kh with ph + 1 - kh even at
// dY row offset (ph + 1 - kh) / 2 (likewise columns), six products per K step in the same order over the same 16-channel
// chunks -- so the result is that kernel's, bit for bit.  What changes is the staging: a 512-thread block owns TWO
// class tiles (waves 0-3 and 4-7) that share the staged weight slice, the copies are DMA'd into NB LDS buffers (no
// VGPR staging, no split), and a block walks a contiguous run of tile pairs x channel chunks as one pipelined stage
// sequence (the copies of stage s + NB - 1 issued right after the barrier of stage s).
struct DgS2Args {
  const __bf16* dy;  // planes [3][NF DH DW][C] (dY of the conv: C = its Co)
  const __bf16* w3;  // pre-split Wd [N][9][C / 16][3][16] (N = the conv's Ci)
  float* out;        // dX [NF][OH][OW][N]
  float* partials;   // fused BN-backward reduce of the layer below: column-major [2N][gridDim.x] (nullable)
  const float* bny;  //   its raw output y [NF][OH][OW][N]
  const float* bnst; //   its BN state (mean | invstd | scale | shift)
  int dy_ps;
  int NF, DH, DW, C, OH, OW, N;
  int tiles_h, tiles_w, ntiles, npairs, ppb;
};

template <int NB>
__global__ __launch_bounds__(512, 2) void dgrad_s2_dma_kernel(const DgS2Args p) {
  constexpr int PC = 16, NC = 32, RP = 3 * PC + 8, WP = 9 * 3 * PC + 8;  // odd 16-B row pitches (7 and 55 chunks)
  constexpr int PCH = 81 * RP / 8, WCH = NC * WP / 8;                     // 16-B chunks: one patch, the weight slice
  constexpr int NCHK = 2 * PCH + WCH, NI = (NCHK + 63) / 64, DW = (NI + 7) / 8, BUF = NI * 64 * 8;
  static_assert(NB * BUF * 2 <= 163840 && DW >= 2, "LDS budget");
  __shared__ __attribute__((aligned(1024))) __bf16 sm[NB * BUF];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int h = lane >> 5, j = lane & 31;
  const int n0 = blockIdx.y * NC;
  const int nch = p.C / PC;
  const int pb = blockIdx.x * p.ppb, pe = min(p.npairs, pb + p.ppb);
  const int stages = (pe - pb) * nch;
  const int tiles_per_img = p.tiles_h * p.tiles_w;
  const __bf16* const zp = g_zero_page;

  // copy u of this wave = DMA instruction i = wave + 8u (past the last: its own previous one again); this lane's
  // chunk c = 64 i + lane: kind 0 / 1 patch of tile A / B (geo = dY row, column in the patch), 2 weights, 3 padding
  int kind[DW], geo[DW], so[DW];
#pragma unroll
  for (int u = 0; u < DW; ++u) {
    int i = wave + 8 * u;
    if (i >= NI) i -= 8;
    const int c = 64 * i + lane;
    if (c < 2 * PCH) {
      const int cc = c % PCH, row = cc / 7, k = cc % 7;
      kind[u] = k < 6 ? c / PCH : 3;
      geo[u] = ((row / 9) << 8) | (row % 9);
      so[u] = (k >> 1) * p.dy_ps + (k & 1) * 8;
    } else if (c < NCHK) {
      const int cc = c - 2 * PCH, n = cc / 55, k = cc % 55;
      kind[u] = (k < 54 && n0 + n < p.N) ? 2 : 3;
      geo[u] = 0;
      so[u] = ((n0 + n) * 9 + k / 6) * (p.C / 16) * 48 + ((k % 6) >> 1) * 16 + (k & 1) * 8;
    } else {
      kind[u] = 3;
      geo[u] = 0;
      so[u] = 0;
    }
  }
  auto tile_at = [&](int t, int& img, int& i0, int& j0) {  // class-grid origin = dY patch origin
    img = t / tiles_per_img;
    const int tr = t % tiles_per_img;
    i0 = (tr / p.tiles_w) * 8;
    j0 = (tr % p.tiles_w) * 8;
  };
  auto issue = [&](int s, int buf) {
    const int pair = pb + s / nch, c0 = (s % nch) * PC;
    int imgA, i0A, j0A, imgB, i0B, j0B;
    tile_at(2 * pair, imgA, i0A, j0A);
    tile_at(2 * pair + 1, imgB, i0B, j0B);
    const bool okB = 2 * pair + 1 < p.ntiles;
#pragma unroll
    for (int u = 0; u < DW; ++u) {
      const int k = kind[u], gy = geo[u] >> 8, gx = geo[u] & 255;
      const __bf16* gp = zp;
      if (k == 2) {
        gp = p.w3 + so[u] + (c0 / 16) * 48;
      } else if (k < 2) {
        const int img = k ? imgB : imgA, y = (k ? i0B : i0A) + gy, x = (k ? j0B : j0A) + gx;
        if ((k == 0 || okB) && y < p.DH && x < p.DW) gp = p.dy + so[u] + ((img * p.DH + y) * p.DW + x) * p.C + c0;
      }
      dma16(gp, sm + buf * BUF + (wave + 8 * u - (wave + 8 * u >= NI ? 8 : 0)) * 512);
    }
  };

  // this wave: tile (wave >> 2), class-tile rows 4 g .. 4 g + 3, classes (1,1)+(0,0) or (0,1)+(1,0)
  const int tsel = wave >> 2, g = wave & 1, csel = (wave >> 1) & 1;
  const int arow = (4 * g + j / 8) * 9 + j % 8;
  f32x16 acc0, acc1;
  float s1 = 0.f, s2 = 0.f;
  const bool bnb = p.bny != nullptr;
  float bmean = 0.f, binv = 0.f, bsc = 0.f, bsh = 0.f;
  if (bnb) {
    const int col = min(n0 + j, p.N - 1);
    bmean = p.bnst[col];
    binv = p.bnst[p.N + col];
    bsc = p.bnst[2 * p.N + col];
    bsh = p.bnst[3 * p.N + col];
  }
  auto cls = [&](f32x16& acc, const __bf16* abase, const __bf16* bbase, int cph, int cpw) {
#pragma unroll
    for (int a = 0; a < 2; ++a) {
      if (a == 1 && !cph) break;
      const int kh = cph ? (a == 0 ? 0 : 2) : 1, dh = (cph && a == 0) ? 1 : 0;
#pragma unroll
      for (int b = 0; b < 2; ++b) {
        if (b == 1 && !cpw) break;
        const int kw = cpw ? (b == 0 ? 0 : 2) : 1, dw = (cpw && b == 0) ? 1 : 0;
        const __bf16* ap = abase + (dh * 9 + dw) * RP;
        const __bf16* bp = bbase + (kh * 3 + kw) * 3 * PC;
        bf16x8d av[3], bv[3];
#pragma unroll
        for (int q = 0; q < 3; ++q) {
          av[q] = *reinterpret_cast<const bf16x8d*>(ap + q * PC);
          bv[q] = *reinterpret_cast<const bf16x8d*>(bp + q * PC);
        }
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av[2], bv[0], acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av[1], bv[1], acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av[0], bv[2], acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av[1], bv[0], acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av[0], bv[1], acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av[0], bv[0], acc, 0, 0, 0);
      }
    }
  };

#pragma unroll
  for (int s = 0; s < NB - 1; ++s)
    if (s < stages) issue(s, s);
  for (int s = 0; s < stages; ++s) {
    if (NB == 3 && s + 1 < stages) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(DW) : "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    if (s + NB - 1 < stages) issue(s + NB - 1, (s + NB - 1) % NB);
    const int c = s % nch, pair = pb + s / nch;
    if (c == 0) {
#pragma unroll
      for (int r = 0; r < 16; ++r) acc0[r] = acc1[r] = 0.f;
    }
    const __bf16* const bb = sm + (s % NB) * BUF;
    const __bf16* abase = bb + tsel * 81 * RP + arow * RP + 8 * h;
    const __bf16* bbase = bb + 2 * 81 * RP + j * WP + 8 * h;
    if (csel == 0) {
      cls(acc0, abase, bbase, 1, 1);
      cls(acc1, abase, bbase, 0, 0);
    } else {
      cls(acc0, abase, bbase, 0, 1);
      cls(acc1, abase, bbase, 1, 0);
    }
    if (c == nch - 1) {  // this tile's dX (two parity classes) and the fused BN-backward sums
      const int t = 2 * pair + tsel;
      if (t < p.ntiles) {
        int img, i0, j0;
        tile_at(t, img, i0, j0);
        const int col = n0 + j;
#pragma unroll
        for (int q = 0; q < 2; ++q) {
          const int ph = q ? (csel ? 1 : 0) : (csel ? 0 : 1), pw = q ? 0 : 1;
          float yb[16];
          if (bnb) {
#pragma unroll
            for (int r = 0; r < 16; ++r) {
              const int pm = (r & 3) + 8 * (r >> 2) + 4 * h;
              const int yy = 2 * (i0 + 4 * g + pm / 8) + ph, xx = 2 * (j0 + pm % 8) + pw;
              const bool ok = yy < p.OH && xx < p.OW;
              yb[r] = p.bny[(ok ? ((int64_t)(img * p.OH + yy) * p.OW + xx) * p.N : 0) + min(col, p.N - 1)];
            }
          }
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int pm = (r & 3) + 8 * (r >> 2) + 4 * h;
            const int yy = 2 * (i0 + 4 * g + pm / 8) + ph, xx = 2 * (j0 + pm % 8) + pw;
            if (col >= p.N || yy >= p.OH || xx >= p.OW) continue;
            const float v = q ? acc1[r] : acc0[r];
            p.out[((int64_t)(img * p.OH + yy) * p.OW + xx) * p.N + col] = v;
            if (bnb) {
              const float dz = fmaf(yb[r], bsc, bsh) > 0.f ? v : 0.f;
              s1 += dz;
              s2 = fmaf(dz, (yb[r] - bmean) * binv, s2);
            }
          }
        }
      }
    }
  }
  if (bnb && p.partials) {  // per-block sums, fixed order: lane halves, then the 8 waves
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
    float* red = reinterpret_cast<float*>(sm);  // [8 waves][2][NC]
    const float a1 = s1 + __shfl_xor(s1, 32, 64), a2 = s2 + __shfl_xor(s2, 32, 64);
    if (lane < 32) {
      red[(wave * 2 + 0) * NC + lane] = a1;
      red[(wave * 2 + 1) * NC + lane] = a2;
    }
    __syncthreads();
    if (tid < 2 * NC) {
      const int which = tid / NC, c = tid % NC;
      float v = 0.f;
#pragma unroll
      for (int w = 0; w < 8; ++w) v += red[(2 * w + which) * NC + c];
      if (n0 + c < p.N) p.partials[(int64_t)(which * p.N + n0 + c) * gridDim.x + blockIdx.x] = v;
    }
  }
}

int g_dgrad_s2_dma = 0;  // knob "conv_dgrad_s2_dma": stride-2 input gradients on dY planes + the Wd planes by LDS-DMA
int g_dgrad_s2_dma_nb = 3;       // knob "conv_dgrad_s2_dma_nb": LDS buffers (2 | 3)
int g_dgrad_s2_dma_blocks = 256;  // knob "conv_dgrad_s2_dma_blocks": target grid

bool dgrad_s2_dma_supported(const Conv3Layer& L) {
  const int64_t lim = ((int64_t)1 << 31) / 3 - 64;
  return g_dgrad_s2_dma && !g_conv_bf16 && !g_act_bf16 && L.stride == 2 && L.Co % 16 == 0 && L.Ci % 32 == 0 &&
         L.OH == (L.IH - 1) / 2 + 1 && L.OW == (L.IW - 1) / 2 + 1 && (int64_t)L.NF * L.OH * L.OW * L.Co < lim &&
         (int64_t)L.NF * L.IH * L.IW * L.Ci < lim;
}

int dgrad_s2_dma(const Conv3Layer& L, const __bf16* dy_planes, const __bf16* w3, float* dX, hipStream_t st,
                 const BnBwdFuse* f) {
  VAD_CHECK(dgrad_s2_dma_supported(L) && w3 != nullptr, "dgrad_s2_dma: unsupported layer or no pre-split Wd image");
  DgS2Args a{};
  a.dy = dy_planes;
  a.w3 = w3;
  a.out = dX;
  a.dy_ps = (int)((int64_t)L.NF * L.OH * L.OW * L.Co);
  a.NF = L.NF; a.DH = L.OH; a.DW = L.OW; a.C = L.Co; a.OH = L.IH; a.OW = L.IW; a.N = L.Ci;
  a.tiles_h = (int)cdiv((L.IH + 1) / 2, 8);
  a.tiles_w = (int)cdiv((L.IW + 1) / 2, 8);
  a.ntiles = L.NF * a.tiles_h * a.tiles_w;
  a.npairs = (int)cdiv(a.ntiles, 2);
  const int nct = L.Ci / 32;
  a.ppb = (int)std::max<int64_t>(1, cdiv((int64_t)a.npairs * nct, g_dgrad_s2_dma_blocks));
  const int gx = (int)cdiv(a.npairs, a.ppb);
  if (f && f->cap < 2ll * L.Ci * gx) f = nullptr;  // (partial buffer too small: the caller runs the separate pass)
  if (f) {
    a.bny = f->y;
    a.bnst = f->stats;
    a.partials = f->parts;
    *f->nparts = gx;
  }
  const dim3 grid((unsigned)gx, (unsigned)nct);
  if (g_dgrad_s2_dma_nb == 2) VAD_KLAUNCH((dgrad_s2_dma_kernel<2>), grid, dim3(512), 0, st, a);
  else VAD_KLAUNCH((dgrad_s2_dma_kernel<3>), grid, dim3(512), 0, st, a);
  VAD_LAUNCH_CHECK();
  return 0;
}

// ---------------------------------------------------------------------------------------------------------------
// Stride-1 input gradient (the transpose of cad:128-139's stride-1 nn.Conv2d): dX[p][n] = sum_{tap, c} dY[p + off(tap)]
// [c] Wd[n][8 - tap][c], on pre-split dY planes and the pre-split Wd image staged by LDS-DMA, with the BN-backward
// reduce of the layer below fused into the epilogue (conv3x3_x3_kernel<FWD = false>'s arithmetic: 32 x 32 x 16 bf16
// MFMA, the six products per K step in the same order over the same 16-channel chunks, so its result bit for bit).
// A 512-thread block owns a run of 256-pixel tiles (NI images of TH x TW) x 32 output channels; each (tile, chunk)
// item's patch (TH + 2) x (TW + 2) x 16 channels x 3 planes and weight slice 32 x 9 taps x 16 x 3 planes are DMA'd
// into one of NB LDS buffers (rows padded to an odd number of 16-B units: conflict-free b128 fragment reads), the
// copies of item k + NB - 1 issued after the barrier of item k.
struct DgS1Args {
  const __bf16* dy;  // planes [3][NF H W][C]
  const __bf16* w3;  // pre-split Wd [N][9][C / 16][3][16]
  float* out;        // dX [NF][H][W][N]
  float* partials;   // fused BN-backward reduce: column-major [2N][gridDim.x] (nullable)
  const float* bny;  //   y of the layer below [NF][H][W][N]
  const float* bnst;
  int dy_ps;
  int NF, H, W, C, N;
  int tiles_h, tiles_w, ntiles, tpb;
};

template <int NI, int TH, int TW>
__device__ __forceinline__ void s1_tile_pixel(int m, int& mi, int& py, int& px) {
  if constexpr (TH == 8 && TW == 8 && NI == 4) {  // (conv3x3_x3_kernel's 8x8 map: 16-lane read phases 4 rows apart)
    const int w = m >> 5, g = (m >> 3) & 3;
    mi = w >> 1;
    py = 2 * (w & 1) + 4 * (g & 1) + (g >> 1);
    px = m & 7;
  } else {
    mi = m / (TH * TW);
    const int mr = m % (TH * TW);
    py = mr / TW;
    px = mr % TW;
  }
}

template <int NI, int TH, int TW, int NB>
__global__ __launch_bounds__(512, 2) void dgrad_s1_dma_kernel(const DgS1Args p) {
  static_assert(NI * TH * TW == 256, "a wave owns 32 pixels");
  constexpr int PC = 16, NC = 32, RP = 3 * PC + 8, WP = 9 * 3 * PC + 8;  // 7 and 55 chunks per row
  constexpr int PH = TH + 2, PW = TW + 2, PROWS = NI * PH * PW;
  constexpr int PCH = PROWS * RP / 8, WCH = NC * WP / 8, NCHK = PCH + WCH;
  constexpr int NI_ = (NCHK + 63) / 64, DW = (NI_ + 7) / 8, BUF = NI_ * 64 * 8;
  static_assert(NB * BUF * 2 <= 163840 && DW >= 2, "LDS budget");
  __shared__ __attribute__((aligned(1024))) __bf16 sm[NB * BUF];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int h = lane >> 5, j = lane & 31;
  const int n0 = blockIdx.y * NC;
  const int nch = p.C / PC;
  const int t0 = blockIdx.x * p.tpb, t1 = min(p.ntiles, t0 + p.tpb);
  const int items = (t1 - t0) * nch;
  const int tiles_per_img = p.tiles_h * p.tiles_w;
  const __bf16* const zp = g_zero_page;

  int kind[DW], geo[DW], so[DW];  // kind 0 patch, 1 weights, 2 padding
#pragma unroll
  for (int u = 0; u < DW; ++u) {
    int i = wave + 8 * u;
    if (i >= NI_) i -= 8;
    const int c = 64 * i + lane;
    if (c < PCH) {
      const int row = c / 7, k = c % 7;
      const int im = row / (PH * PW), rr = row % (PH * PW);
      kind[u] = k < 6 ? 0 : 2;
      geo[u] = (im << 16) | ((rr / PW) << 8) | (rr % PW);
      so[u] = (k >> 1) * p.dy_ps + (k & 1) * 8;
    } else if (c < NCHK) {
      const int cc = c - PCH, n = cc / 55, k = cc % 55;
      kind[u] = (k < 54 && n0 + n < p.N) ? 1 : 2;
      geo[u] = 0;
      so[u] = ((n0 + n) * 9 + 8 - k / 6) * (p.C / 16) * 48 + ((k % 6) >> 1) * 16 + (k & 1) * 8;
    } else {
      kind[u] = 2;
      geo[u] = 0;
      so[u] = 0;
    }
  }
  auto origin = [&](int tile, int& img0, int& oy0, int& ox0) {
    img0 = (tile / tiles_per_img) * NI;
    const int tr = tile % tiles_per_img;
    oy0 = (tr / p.tiles_w) * TH;
    ox0 = (tr % p.tiles_w) * TW;
  };
  auto issue = [&](int it, int buf) {
    const int tile = t0 + it / nch, c0 = (it % nch) * PC;
    int img0, oy0, ox0;
    origin(tile, img0, oy0, ox0);
#pragma unroll
    for (int u = 0; u < DW; ++u) {
      const int k = kind[u], g = geo[u];
      const __bf16* gp = zp;
      if (k == 1) {
        gp = p.w3 + so[u] + (c0 / 16) * 48;
      } else if (k == 0) {
        const int img = img0 + (g >> 16), y = oy0 - 1 + ((g >> 8) & 255), x = ox0 - 1 + (g & 255);
        if (img < p.NF && (unsigned)y < (unsigned)p.H && (unsigned)x < (unsigned)p.W)
          gp = p.dy + so[u] + ((img * p.H + y) * p.W + x) * p.C + c0;
      }
      dma16(gp, sm + buf * BUF + (wave + 8 * u - (wave + 8 * u >= NI_ ? 8 : 0)) * 512);
    }
  };

  int mi, py, px;
  s1_tile_pixel<NI, TH, TW>(wave * 32 + j, mi, py, px);
  const int arow0 = (mi * PH + py) * PW + px;
  f32x16 acc;
  float s1 = 0.f, s2 = 0.f;
  const bool bnb = p.bny != nullptr;
  const int col = n0 + j;
  float bmean = 0.f, binv = 0.f, bsc = 0.f, bsh = 0.f;
  if (bnb) {
    const int cc = min(col, p.N - 1);
    bmean = p.bnst[cc];
    binv = p.bnst[p.N + cc];
    bsc = p.bnst[2 * p.N + cc];
    bsh = p.bnst[3 * p.N + cc];
  }
#pragma unroll
  for (int s = 0; s < NB - 1; ++s)
    if (s < items) issue(s, s);
  for (int it = 0; it < items; ++it) {
    if (NB == 3 && it + 1 < items) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(DW) : "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    if (it + NB - 1 < items) issue(it + NB - 1, (it + NB - 1) % NB);
    const int ch = it % nch;
    if (ch == 0) {
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[r] = 0.f;
    }
    const __bf16* const bb = sm + (it % NB) * BUF;
    const __bf16* const wl = bb + PROWS * RP;
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      const int kh = t / 3, kw = t % 3;
      const __bf16* ap = bb + (arow0 + kh * PW + kw) * RP + 8 * h;
      const __bf16* bp = wl + j * WP + t * 3 * PC + 8 * h;
      bf16x8d a[3], b[3];
#pragma unroll
      for (int q = 0; q < 3; ++q) {
        a[q] = *reinterpret_cast<const bf16x8d*>(ap + q * PC);
        b[q] = *reinterpret_cast<const bf16x8d*>(bp + q * PC);
      }
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[2], b[0], acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[1], b[1], acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], b[2], acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[1], b[0], acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], b[1], acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], b[0], acc, 0, 0, 0);
    }
    if (ch == nch - 1) {
      int img0, oy0, ox0;
      origin(t0 + it / nch, img0, oy0, ox0);
      float yb[16];
      if (bnb) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          int qi, qy, qx;
          s1_tile_pixel<NI, TH, TW>(wave * 32 + (r & 3) + 8 * (r >> 2) + 4 * h, qi, qy, qx);
          const int oy = oy0 + qy, ox = ox0 + qx, img = img0 + qi;
          const bool ok = img < p.NF && oy < p.H && ox < p.W;
          yb[r] = p.bny[(ok ? ((int64_t)(img * p.H + oy) * p.W + ox) * p.N : 0) + min(col, p.N - 1)];
        }
      }
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        int qi, qy, qx;
        s1_tile_pixel<NI, TH, TW>(wave * 32 + (r & 3) + 8 * (r >> 2) + 4 * h, qi, qy, qx);
        const int oy = oy0 + qy, ox = ox0 + qx, img = img0 + qi;
        if (img >= p.NF || oy >= p.H || ox >= p.W || col >= p.N) continue;
        const float v = acc[r];
        p.out[((int64_t)(img * p.H + oy) * p.W + ox) * p.N + col] = v;
        if (bnb) {
          const float dz = fmaf(yb[r], bsc, bsh) > 0.f ? v : 0.f;
          s1 += dz;
          s2 = fmaf(dz, (yb[r] - bmean) * binv, s2);
        }
      }
    }
  }
  if (bnb && p.partials) {  // per-block sums, fixed order: lane halves, then the 8 waves
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
    float* red = reinterpret_cast<float*>(sm);  // [8 waves][2][NC]
    const float a1 = s1 + __shfl_xor(s1, 32, 64), a2 = s2 + __shfl_xor(s2, 32, 64);
    if (lane < 32) {
      red[(wave * 2 + 0) * NC + lane] = a1;
      red[(wave * 2 + 1) * NC + lane] = a2;
    }
    __syncthreads();
    if (tid < 2 * NC) {
      const int which = tid / NC, c = tid % NC;
      float v = 0.f;
#pragma unroll
      for (int w = 0; w < 8; ++w) v += red[(2 * w + which) * NC + c];
      if (n0 + c < p.N) p.partials[(int64_t)(which * p.N + n0 + c) * gridDim.x + blockIdx.x] = v;
    }
  }
}

int g_dgrad_s1_dma = 0;           // knob "conv_dgrad_s1_dma": stride-1 input gradients on dY planes by LDS-DMA
int g_dgrad_s1_dma_blocks = 256;  // knob "conv_dgrad_s1_dma_blocks": target grid

bool dgrad_s1_dma_supported(const Conv3Layer& L) {
  const int64_t lim = ((int64_t)1 << 31) / 3 - 64;
  return g_dgrad_s1_dma && !g_conv_bf16 && !g_act_bf16 && L.stride == 1 && L.Co % 16 == 0 && L.Ci % 32 == 0 &&
         L.OH == L.IH && L.OW == L.IW && (int64_t)L.NF * L.OH * L.OW * L.Co < lim &&
         (int64_t)L.NF * L.IH * L.IW * L.Ci < lim;
}

template <int NI, int TH, int TW>
static int ds1_launch(DgS1Args a, const BnBwdFuse* f, hipStream_t st) {
  a.tiles_h = (int)cdiv(a.H, TH);
  a.tiles_w = (int)cdiv(a.W, TW);
  a.ntiles = (int)cdiv(a.NF, NI) * a.tiles_h * a.tiles_w;
  const int nct = a.N / 32;
  a.tpb = (int)std::max<int64_t>(1, cdiv((int64_t)a.ntiles * nct, g_dgrad_s1_dma_blocks));
  const int gx = (int)cdiv(a.ntiles, a.tpb);
  if (f && f->cap < 2ll * a.N * gx) f = nullptr;
  if (f) {
    a.bny = f->y;
    a.bnst = f->stats;
    a.partials = f->parts;
    *f->nparts = gx;
  }
  const dim3 grid((unsigned)gx, (unsigned)nct);
  VAD_KLAUNCH((dgrad_s1_dma_kernel<NI, TH, TW, 2>), grid, dim3(512), 0, st, a);  // (3 buffers exceed the LDS)
  VAD_LAUNCH_CHECK();
  return 0;
}

int dgrad_s1_dma(const Conv3Layer& L, const __bf16* dy_planes, const __bf16* w3, float* dX, hipStream_t st,
                 const BnBwdFuse* f) {
  VAD_CHECK(dgrad_s1_dma_supported(L) && w3 != nullptr, "dgrad_s1_dma: unsupported layer or no pre-split Wd image");
  DgS1Args a{};
  a.dy = dy_planes;
  a.w3 = w3;
  a.out = dX;
  a.dy_ps = (int)((int64_t)L.NF * L.OH * L.OW * L.Co);
  a.NF = L.NF; a.H = L.IH; a.W = L.IW; a.C = L.Co; a.N = L.Ci;
  if (L.IW <= 8 && L.IH <= 8) return ds1_launch<4, 8, 8>(a, f, st);
  if (L.IW <= 16) return ds1_launch<1, 16, 16>(a, f, st);
  return ds1_launch<1, 8, 32>(a, f, st);
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
