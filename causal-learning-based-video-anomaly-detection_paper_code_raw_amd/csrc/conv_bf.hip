// Native bf16 3x3 convolutions: the forward and the stride-1 input gradient of the backbone's conv layers
// (causal_anomaly_detection.py:128-139, 148-151) for BASELINE config 4 (T = 32, 256x256, bf16 compute).
//
// Config 4 is HBM-bound (~76 FLOP/B against the bf16 ridge of ~315), so these kernels are built around
// bytes in flight, not around the matrix cores: bf16 NHWC activations and bf16 weight images (written by the weight
// prep beside the fp32 images), every staging load 16 B per lane, reduction chunks of 16-64 input channels so one
// (tile, chunk) item moves 20-50 KB, blocks small enough (<= 64 KB of LDS, 4 waves) that 2-3 share a CU, and the
// next item's loads issued before the current item's MFMAs (a register prefetch one item deep).  The epilogue
// goes through LDS: the 32x32 accumulator tiles (column = output channel on the lane) are written out as bf16
// [pixel][channel] rows, read back 16 B (8 channels of one pixel) per lane and stored with 16-B global stores; the
// per-block BN sums of the forward (sum y, sum y^2 of the stored bf16 values) and the fused BN-backward reduce of
// the input gradient (sum dZ, sum dZ * xhat of the layer below, reading its y 16 B per lane at the written pixel)
// are taken in that transposed domain, fixed order, column-major [2N][blocks] like the split kernels' partials.
//
// GEMM view: M = output pixels of a TH x TW tile (NI images of it), N = 32 * NCT output channels, K = 9 taps x CB
// input channels per item.  Wave w owns pixels [32 MF w, 32 MF (w + 1)) of the tile against all N channels.  LDS:
//   patch [NI * PH * PW rows][CB + 8]  (the tile's input patch incl. halo; BN + ReLU on load; stride 2 stores the
//                                        columns parity-split, [even | odd], so 16 consecutive output pixels read
//                                        16 consecutive rows for every tap)
//   wl    [32 NCT rows][9 CB + 8]      (the weight slice, rows = output channels)
// Both row pitches are odd multiples of 16 B: the b128 fragment reads of a 16-lane phase hit distinct bank quads.
#include <algorithm>

#include "backbone.h"

namespace vad {

typedef __bf16 bfv8 __attribute__((ext_vector_type(8)));
typedef unsigned u32v4 __attribute__((ext_vector_type(4)));

struct BfcArgs {
  const __bf16* src;   // NHWC [NF][IH][IW][C]
  const float* scale;  // forward: BN + ReLU of the producer applied on load (nullable)
  const float* shift;
  const __bf16* w;     // [N][9][C] bf16 (forward: the Wf image; input gradient: the Wd image, taps flipped here)
  const float* bias;   // forward only (nullable)
  __bf16* out;         // NHWC [NF][OH][OW][N]
  float* partials;     // column-major [2N][gridDim.x] per-block sums (nullable)
  const __bf16* bny;   // input gradient: raw output y of the layer whose dA this is (fused BN-backward reduce)
  const float* bnst;   // its BN state (mean | invstd | scale | shift)
  int NF, IH, IW, C, OH, OW, N;
  int tiles_h, tiles_w, ntiles, tpb;
};

// workgroup barrier for LDS hand-offs only: __syncthreads() also waits for every outstanding global load
// (s_waitcnt vmcnt(0)), which would drain the next item's prefetch at each barrier; the register uses of those loads get
// their own counted waits from the compiler.  (asm with a memory clobber: no LDS access moves across it.)
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

__device__ __forceinline__ void bf8_to_f32(u32v4 r, float (&v)[8]) {
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    v[2 * e] = __uint_as_float(r[e] << 16);
    v[2 * e + 1] = __uint_as_float(r[e] & 0xffff0000u);
  }
}

__device__ __forceinline__ u32v4 f32_to_bf8(const float (&v)[8]) {
  bfv8 b;
#pragma unroll
  for (int e = 0; e < 8; ++e) b[e] = (__bf16)v[e];
  return __builtin_bit_cast(u32v4, b);
}

// Per-block constants live in LDS (staged once): global loads issued inside the item loop would be younger than the
// prefetch and their waits (s_waitcnt vmcnt counts in issue order) would drain it.  The MFMA loop keeps the next K
// step's fragments in flight (one step of register double-buffering), so no MFMA waits on its own LDS reads.
template <int S, int NI, int TH, int TW, int CB, int NCT, bool FWD, bool WRES>
__global__ __launch_bounds__(256, 2) void bfc_conv_kernel(const BfcArgs p) {
  constexpr int NW = 4, NTHR = 256;
  constexpr int TPX = NI * TH * TW, MF = TPX / (32 * NW);
  static_assert(MF >= 1 && MF * 32 * NW == TPX, "a wave owns 32 MF output pixels");
  static_assert(FWD || S == 1, "stride-2 input gradients: bfc_dgrad_s2_kernel");
  static_assert(CB % 16 == 0 && CB <= 64, "16-deep K steps");
  constexpr int NC = 32 * NCT, G8 = CB / 8, NG = NC / 8, KK = CB / 16, NSTEP = 9 * KK;
  constexpr int PH = (TH - 1) * S + 3, PW = (TW - 1) * S + 3, PWE = (PW + 1) / 2, PROWS = NI * PH * PW;
  constexpr int RP = CB + 8, WP = 9 * CB + 8, EP = NC + 8;
  static_assert(((RP / 8) & 1) && ((WP / 8) & 1) && ((EP / 8) & 1), "odd 16-B row pitches");
  constexpr int PE = PROWS * RP > TPX * EP ? PROWS * RP : TPX * EP;
  constexpr int CMAX = 256, CST = FWD ? 2 * CMAX + NC : 4 * NC;  // constants (floats)
  static_assert(NTHR % G8 == 0 && NTHR % NG == 0, "a thread keeps its channel group");
  __shared__ __attribute__((aligned(16))) __bf16 sm[PE + NC * WP + 2 * CST];
  __bf16* const patch = sm;
  __bf16* const wl = sm + PE;
  float* const cst = reinterpret_cast<float*>(sm + PE + NC * WP);
  // forward: [scale | shift] of every input channel, then the bias of the block's NC outputs;
  // input gradient: [mean | invstd | scale | shift] of the block's NC outputs (the layer below's BN)
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int h = lane >> 5, j = lane & 31;
  const int tiles_per_img = p.tiles_h * p.tiles_w;
  const int n0 = blockIdx.y * NC;
  const int t0 = blockIdx.x * p.tpb, t1 = min(p.ntiles, t0 + p.tpb);
  const int nch = p.C / CB;
  const int nitems = (t1 - t0) * nch;
  const bool bn = FWD && p.scale != nullptr;
  const bool bnb = !FWD && p.bny != nullptr;
  if constexpr (FWD) {
    for (int c = tid; c < p.C; c += NTHR) {
      cst[c] = bn ? p.scale[c] : 1.f;
      cst[CMAX + c] = bn ? p.shift[c] : 0.f;
    }
    for (int c = tid; c < NC; c += NTHR) cst[2 * CMAX + c] = p.bias ? p.bias[min(n0 + c, p.N - 1)] : 0.f;
  } else {
    if (bnb)
      for (int q = tid; q < 4 * NC; q += NTHR) cst[q] = p.bnst[(q / NC) * p.N + min(n0 + q % NC, p.N - 1)];
  }
  __syncthreads();

  // this lane's A rows (MFMA row j of each of its MF pixel groups): patch row of tap (0, 0)
  int arow[MF];
#pragma unroll
  for (int mf = 0; mf < MF; ++mf) {
    const int m = (wave * MF + mf) * 32 + j;
    const int mi = m / (TH * TW), mr = m % (TH * TW);
    arow[mf] = (mi * PH + (mr / TW) * S) * PW + mr % TW;  // (stride 2: stored column of input column 2 px is px)
  }

  constexpr int PQ = PROWS * G8, PIT = (PQ + NTHR - 1) / NTHR;
  constexpr int WQ = NC * 9 * G8, WIT = (WQ + NTHR - 1) / NTHR;
  const int g8 = tid % G8;
  u32v4 pv[PIT], wv[WIT];
  bool pok[PIT];
  static_assert(PIT >= 1 && WIT >= 1, "staging passes");
  // piece geometry, loop-invariant (32-bit offsets: the host checks every tensor < 2^31 elements): patch piece it =
  // (frame im, patch row ry, patch column rx) packed, its NHWC offset from the tile's patch origin, its LDS offset
  int pgeo[PIT], pgo[PIT], plo[PIT];
#pragma unroll
  for (int it = 0; it < PIT; ++it) {
    const int q = tid + it * NTHR, row = min(q / G8, PROWS - 1);
    const int im = row / (PH * PW), rr = row % (PH * PW), ry = rr / PW, rx = rr % PW;
    const int col = S == 1 ? rx : ((rx & 1) ? PWE + (rx >> 1) : (rx >> 1));
    pgeo[it] = q < PQ ? (im << 16) | (ry << 8) | rx : -1;
    pgo[it] = ((im * p.IH + ry) * p.IW + rx) * p.C + g8 * 8;
    plo[it] = ((im * PH + ry) * PW + col) * RP + g8 * 8;
  }
  int wgo[WIT], wlo[WIT];  // weight pieces: offset in the image (from row n0, chunk 0) and in LDS
#pragma unroll
  for (int it = 0; it < WIT; ++it) {
    const int q = min(tid + it * NTHR, WQ - 1);
    const int n = q / (9 * G8), t = (q / G8) % 9;
    wgo[it] = (n * 9 + (FWD ? t : 8 - t)) * p.C + g8 * 8;
    wlo[it] = tid + it * NTHR < WQ ? n * WP + t * CB + g8 * 8 : -1;
  }
  auto origin = [&](int tile, int& img0, int& oy0, int& ox0) {
    img0 = (tile / tiles_per_img) * NI;
    const int tr = tile % tiles_per_img;
    oy0 = (tr / p.tiles_w) * TH;
    ox0 = (tr % p.tiles_w) * TW;
  };
  // loads from clamped addresses (no masked-load branches): out-of-range pieces are zeroed when stashed.  Every item
  // issues the same loads (WRES: the resident weight slice is loaded once, before the loop), so the compiler's counted
  // waits (vmcnt) stay exact and never drain the prefetch
  const __bf16* const wsrc = p.w + (int64_t)n0 * 9 * p.C;
  auto fetch_w = [&](int ch) {
#pragma unroll
    for (int it = 0; it < WIT; ++it) wv[it] = *reinterpret_cast<const u32v4*>(wsrc + wgo[it] + ch * CB);
  };
  auto fetch = [&](int tile, int ch) {
    int img0, oy0, ox0;
    origin(tile, img0, oy0, ox0);
    const int iy0 = oy0 * S - 1, ix0 = ox0 * S - 1;
    // (block-uniform) the whole patch inside the frames: only the padding pieces past PQ are masked
    const bool inner = iy0 >= 0 && ix0 >= 0 && iy0 + PH <= p.IH && ix0 + PW <= p.IW && img0 + NI <= p.NF;
    const int base = ((img0 * p.IH + iy0) * p.IW + ix0) * p.C + ch * CB;
#pragma unroll
    for (int it = 0; it < PIT; ++it) {
      const int g = pgeo[it], im = g >> 16, ry = (g >> 8) & 255, rx = g & 255;
      pok[it] = g >= 0 && (inner || (img0 + im < p.NF && (unsigned)(iy0 + ry) < (unsigned)p.IH &&
                                     (unsigned)(ix0 + rx) < (unsigned)p.IW));
      pv[it] = *reinterpret_cast<const u32v4*>(p.src + (pok[it] ? base + pgo[it] : 0));
    }
    if constexpr (!WRES) fetch_w(ch);
  };
  auto stash_w = [&]() {
#pragma unroll
    for (int it = 0; it < WIT; ++it)
      if (wlo[it] >= 0) *reinterpret_cast<u32v4*>(wl + wlo[it]) = wv[it];
  };
  auto stash = [&](int ch) {
    float sc[8], sh[8];
    if (bn) {  // BN scale / shift of this thread's 8 input channels
      const int c = ch * CB + g8 * 8;
#pragma unroll
      for (int e = 0; e < 8; e += 4) {
        const f32x4 a4 = *reinterpret_cast<const f32x4*>(cst + c + e);
        const f32x4 b4 = *reinterpret_cast<const f32x4*>(cst + CMAX + c + e);
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          sc[e + u] = a4[u];
          sh[e + u] = b4[u];
        }
      }
    }
#pragma unroll
    for (int it = 0; it < PIT; ++it) {
      if (pgeo[it] >= 0) {
        const bool ok = pok[it];
        u32v4 v = ok ? pv[it] : u32v4{0u, 0u, 0u, 0u};
        if (bn) {  // zero padding stays zero: the reference pads relu(bn(y)) with zeros (selects, no branch; NaN
                   // propagates like torch's relu)
          float f[8];
          bf8_to_f32(pv[it], f);
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            const float r = fmaf(f[e], sc[e], sh[e]);
            f[e] = (r <= 0.f || !ok) ? 0.f : r;
          }
          v = f32_to_bf8(f);
        }
        *reinterpret_cast<u32v4*>(patch + plo[it]) = v;
      }
    }
    if constexpr (!WRES) stash_w();
  };
  // fragments of K step s (tap s / KK, 16-channel slice s % KK)
  auto frags = [&](int s, bfv8 (&a)[MF], bfv8 (&b)[NCT]) {
    const int t = s / KK, kk = s % KK, kh = t / 3, kw = t % 3;
    const int co = S == 1 ? kw : ((kw & 1) ? PWE + (kw >> 1) : (kw >> 1));
#pragma unroll
    for (int nt = 0; nt < NCT; ++nt)
      b[nt] = *reinterpret_cast<const bfv8*>(wl + (nt * 32 + j) * WP + t * CB + kk * 16 + 8 * h);
#pragma unroll
    for (int mf = 0; mf < MF; ++mf)
      a[mf] = *reinterpret_cast<const bfv8*>(patch + (arow[mf] + kh * PW + co) * RP + kk * 16 + 8 * h);
  };

  // epilogue: this thread's 8 output channels (group cg) and their block sums; piece i = pixel m of the tile, packed
  // (frame, row, column) and its NHWC offset from the tile's output origin
  const int cg = tid % NG;
  constexpr int EQ = TPX * NG, EIT = (EQ + NTHR - 1) / NTHR;
  int egeo[EIT], ego[EIT];
#pragma unroll
  for (int i = 0; i < EIT; ++i) {
    const int q = tid + i * NTHR, m = min(q / NG, TPX - 1);
    const int mi = m / (TH * TW), mr = m % (TH * TW), py = mr / TW, px = mr % TW;
    egeo[i] = q < EQ ? (mi << 16) | (py << 8) | px : -1;
    ego[i] = ((mi * p.OH + py) * p.OW + px) * p.N + cg * 8;
  }
  float s1[8], s2[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) s1[e] = s2[e] = 0.f;
  u32v4 yv[FWD ? 1 : EIT];  // (input gradient: the layer below's y at the written pixels, loaded before the prefetch)
  (void)yv;

  f32x16 acc[MF][NCT];
  if (nitems <= 0) return;  // (block-uniform, before any barrier of the loop)
  if constexpr (WRES) {  // one reduction chunk: the weight slice is staged once and stays resident
    fetch_w(0);
    stash_w();
  }
  fetch(t0, 0);
  for (int item = 0; item < nitems; ++item) {
    const int tile = t0 + item / nch, ch = item % nch;
    lds_barrier();  // the previous item's fragment reads and epilogue reads are done
    stash(ch);
    lds_barrier();
    int img0, oy0, ox0;
    origin(tile, img0, oy0, ox0);
    const bool oinner = oy0 + TH <= p.OH && ox0 + TW <= p.OW && img0 + NI <= p.NF;
    const int obase = ((img0 * p.OH + oy0) * p.OW + ox0) * p.N + n0;
    auto piece = [&](int i, int& m, int& oi) {  // epilogue piece i of this thread: pixel m, NHWC offset (or -1)
      const int g = egeo[i], mi = g >> 16, py = (g >> 8) & 255, px = g & 255;
      m = (mi * TH + py) * TW + px;
      const bool ok = g >= 0 && (oinner || (img0 + mi < p.NF && oy0 + py < p.OH && ox0 + px < p.OW));
      oi = ok ? obase + ego[i] : -1;
    };
    if constexpr (!FWD) {
      if (bnb && ch == nch - 1) {
#pragma unroll
        for (int i = 0; i < EIT; ++i) {
          int m, oi;
          piece(i, m, oi);
          yv[i] = *reinterpret_cast<const u32v4*>(p.bny + (oi < 0 ? 0 : oi));
        }
      }
    }
    {  // (unconditional: the last item re-loads its own data)
      const int nx = min(item + 1, nitems - 1);
      fetch(t0 + nx / nch, nx % nch);
    }
    if (ch == 0) {
#pragma unroll
      for (int mf = 0; mf < MF; ++mf)
#pragma unroll
        for (int nt = 0; nt < NCT; ++nt)
#pragma unroll
          for (int r = 0; r < 16; ++r) acc[mf][nt][r] = 0.f;
    }
    {
      bfv8 a0[MF], b0[NCT], a1[MF], b1[NCT];
      frags(0, a0, b0);
#pragma unroll
      for (int s = 0; s < NSTEP; ++s) {
        bfv8(&ac)[MF] = (s & 1) ? a1 : a0;
        bfv8(&bc)[NCT] = (s & 1) ? b1 : b0;
        if (s + 1 < NSTEP) frags(s + 1, (s & 1) ? a0 : a1, (s & 1) ? b0 : b1);
        // (the compiler otherwise sinks those reads to their MFMAs; not where the pinned fragments would spill)
        if constexpr (!(NCT == 2 && CB == 32 && !WRES)) __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int mf = 0; mf < MF; ++mf)
#pragma unroll
          for (int nt = 0; nt < NCT; ++nt)
            acc[mf][nt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ac[mf], bc[nt], acc[mf][nt], 0, 0, 0);
      }
    }
    if (ch == nch - 1) {
      // accumulators -> bf16 [pixel][channel] rows in the patch region, then 16-B pieces to global
      lds_barrier();  // every wave is done reading the patch
      __bf16* epi = patch;
#pragma unroll
      for (int nt = 0; nt < NCT; ++nt) {
        const float bj = FWD ? cst[2 * CMAX + nt * 32 + j] : 0.f;
#pragma unroll
        for (int mf = 0; mf < MF; ++mf)
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int m = (wave * MF + mf) * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
            epi[m * EP + nt * 32 + j] = (__bf16)(acc[mf][nt][r] + bj);
          }
      }
      lds_barrier();
      // the layer below's BN state for this thread's 8 channels (input gradient with the fused reduce): the dZ mask
      // test fma(y, scale, shift) > 0 and xhat = (y - mean) * invstd
      float bmean[8], binv[8], bsc[8], bsh[8];
      if (bnb) {
#pragma unroll
        for (int e = 0; e < 8; e += 4) {
          const f32x4 m4 = *reinterpret_cast<const f32x4*>(cst + cg * 8 + e);
          const f32x4 i4 = *reinterpret_cast<const f32x4*>(cst + NC + cg * 8 + e);
          const f32x4 a4 = *reinterpret_cast<const f32x4*>(cst + 2 * NC + cg * 8 + e);
          const f32x4 b4 = *reinterpret_cast<const f32x4*>(cst + 3 * NC + cg * 8 + e);
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            bmean[e + u] = m4[u];
            binv[e + u] = i4[u];
            bsc[e + u] = a4[u];
            bsh[e + u] = b4[u];
          }
        }
      }
#pragma unroll
      for (int i = 0; i < EIT; ++i) {
        int m, oi;
        piece(i, m, oi);
        const u32v4 ev = *reinterpret_cast<const u32v4*>(epi + m * EP + cg * 8);
        if (oi < 0) continue;
        *reinterpret_cast<u32v4*>(p.out + oi) = ev;
        float f[8];
        bf8_to_f32(ev, f);
        if constexpr (FWD) {
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            s1[e] += f[e];
            s2[e] = fmaf(f[e], f[e], s2[e]);
          }
        } else if (bnb) {
          float yy[8];
          bf8_to_f32(yv[i], yy);
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            const float dz = fmaf(yy[e], bsc[e], bsh[e]) > 0.f ? f[e] : 0.f;
            s1[e] += dz;
            s2[e] = fmaf(dz, (yy[e] - bmean[e]) * binv[e], s2[e]);
          }
        }
      }
    }
  }
  if ((FWD || bnb) && p.partials) {
    // lanes of one channel group: butterfly over the lane bits above the group bits, then the 4 waves in order
#pragma unroll
    for (int o = NG; o < 64; o <<= 1)
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        s1[e] += __shfl_xor(s1[e], o, 64);
        s2[e] += __shfl_xor(s2[e], o, 64);
      }
    __syncthreads();
    float* red = reinterpret_cast<float*>(sm);  // [4 waves][2][NC]
    if (lane < NG) {
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        red[(wave * 2 + 0) * NC + lane * 8 + e] = s1[e];
        red[(wave * 2 + 1) * NC + lane * 8 + e] = s2[e];
      }
    }
    __syncthreads();
    for (int q = tid; q < 2 * NC; q += NTHR) {
      const int which = q / NC, c = q % NC;
      const float v = (red[(0 + which) * NC + c] + red[(2 + which) * NC + c]) +
                      (red[(4 + which) * NC + c] + red[(6 + which) * NC + c]);
      if (n0 + c < p.N) p.partials[(int64_t)(which * p.N + n0 + c) * gridDim.x + blockIdx.x] = v;
    }
  }
}

// ---------------------------------------------------------------------------------------------------------------
// Weight gradient dW[co][tap][ci] = sum_p dY[p][co] * relu(bn(x))[p + off(tap)][ci] (zero padding).
// GEMM view per tap: M = 32 output channels (A = dY^T), N = 32 input channels (B = the shifted input), K = output
// pixels.  Both operands need 8 consecutive pixels of one channel per lane, i.e. the transpose of the NHWC rows the
// loads deliver: the LDS images keep the NHWC order -- [pixel][32 channels], 64-B rows -- and the fragments are read
// with ds_read_b64_tr_b16 (gfx950's transposing LDS read: per 16-lane group, 4 rows x 16 columns delivered column-
// major), two per fragment.  So the staging is a plain 16-B copy (dY) or a 16-B BN + ReLU pass (x), no register
// transposition, and the 4 rows of a group are 4 consecutive pixels of one tile row: consecutive LDS rows (stride 2:
// the patch columns are stored parity-split, [even | odd]), i.e. 256 contiguous bytes per 32-lane half -- conflict-
// free.  K step = 16 consecutive tile pixels (TW % 8 == 0: the 8 of a lane half lie in one tile row).  A block owns
// 32 NCO output channels x 32 input channels and a strided set of tiles; with NCO = 2 waves 0-1 take co tile 0 and
// waves 2-3 co tile 1, each pair splitting the K steps; the waves of a co tile are summed in a fixed order and the
// block's sum lands in split-K slab blockIdx.z ([S][Co][9 Ci], conv3_wgrad_reduce).  No register prefetch: the
// co-resident block (2 per CU) overlaps its loads with this block's MFMAs.
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bfv4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ bfv8 tr_frag(const __bf16* a0, const __bf16* a1) {
  typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
  const s16x4 u = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(a0));
  const s16x4 v = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(a1));
  const bfv4 x = __builtin_bit_cast(bfv4, u), y = __builtin_bit_cast(bfv4, v);
  return bfv8{x[0], x[1], x[2], x[3], y[0], y[1], y[2], y[3]};
}

struct BfwArgs {
  const __bf16* dY;    // [NF][OH][OW][Co]
  const __bf16* src;   // [NF][IH][IW][Ci]
  const float* scale;  // BN + ReLU on load (nullable)
  const float* shift;
  float* slab;         // [S][Co][9 Ci]
  int NF, IH, IW, Ci, OH, OW, Co;
  int tiles_h, tiles_w, ntiles;
};

template <int S, int NI, int TH, int TW, int NCO>
__global__ __launch_bounds__(256, 2) void bfc_wgrad_kernel(const BfwArgs p) {
  constexpr int TPX = NI * TH * TW, KS = TPX / 16, WPC = 4 / NCO, KSW = KS / WPC;
  static_assert(TW % 8 == 0 && KS % WPC == 0 && (NCO == 1 || NCO == 2), "whole K steps per wave");
  constexpr int PH = (TH - 1) * S + 3, PW = (TW - 1) * S + 3, PWE = (PW + 1) / 2, PROWS = NI * PH * PW;
  constexpr int YIMG = TPX * 32 + 32;  // one co tile's dY image (+ 64 B)
  constexpr int XROWS = (PROWS + 15) / 16 * 16;  // patch rows, whole DMA instructions
  __shared__ __attribute__((aligned(16))) __bf16 sm[NCO * YIMG + XROWS * 32];
  __bf16* const ys = sm;
  __bf16* const xs = sm + NCO * YIMG;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int h = lane >> 5, j = lane & 31;
  const int q4 = (lane & 15) >> 2, p4 = lane & 3, g16 = (lane >> 4) & 1;  // transposed-read address roles
  const int co0 = blockIdx.x * 32 * NCO, ci0 = blockIdx.y * 32;
  const int tiles_per_img = p.tiles_h * p.tiles_w;
  const int ct = wave / WPC, ks0 = (wave % WPC) * KSW;  // this wave's co tile and first K step

  // Staging is all LDS-DMA (global_load_lds_dwordx4: no staging registers beside the 144 accumulator VGPRs): one
  // wave-instruction = 16 rows x 64 B, lane-linear in LDS, each lane's source row chosen by its position (dY:
  // pixels of one co tile's image; patch: stored rows, i.e. the parity-split column order for stride 2).  Then one
  // in-place pass over the patch applies BN + ReLU (and zeroes the halo outside the frame), and zeroes the dY rows of
  // pixels outside the map on ragged tiles.
  constexpr int YI = TPX * NCO / 16;                      // dY wave-instructions per tile
  constexpr int XI = (PROWS + 15) / 16;                   // patch wave-instructions per tile
  static_assert(YI % 4 == 0, "whole dY instructions per wave");
  const bool bn = p.scale != nullptr;
  const int g4 = tid & 3;  // fix-up pass: this thread's 8-channel group
  float sc[8], sh[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    sc[e] = bn ? p.scale[ci0 + g4 * 8 + e] : 1.f;
    sh[e] = bn ? p.shift[ci0 + g4 * 8 + e] : 0.f;
  }

  f32x16 acc[9];
#pragma unroll
  for (int t = 0; t < 9; ++t)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[t][r] = 0.f;

  // loop-invariant piece geometry, 32-bit offsets from the tile's origin (the host keeps every tensor below 2^31
  // elements): dY DMA piece u (pixel packed (frame, row, column)), patch DMA piece k (stored row -> (frame, patch row,
  // input column)), fix-up piece it
  constexpr int XIW = (XI + 3) / 4, FQ = (PROWS * 4 + 255) / 256;
  int ygeo[YI / 4], xgeo[XIW], fgeo[FQ];
#pragma unroll
  for (int u = 0; u < YI / 4; ++u) {
    const int i = wave + 4 * u, f = i / (TPX / 16), pb = i % (TPX / 16);
    const int m = pb * 16 + (lane >> 2);
    const int mi = m / (TH * TW), mr = m % (TH * TW), py = mr / TW, px = mr % TW;
    ygeo[u] = (f << 24) | (mi << 16) | (py << 8) | px;
  }
  auto patch_geo = [&](int row) {
    const int mi = row / (PH * PW), rr = row % (PH * PW), col = rr % PW;
    const int rx = S == 1 ? col : (col < PWE ? 2 * col : 2 * (col - PWE) + 1);
    return (mi << 16) | ((rr / PW) << 8) | rx;
  };
#pragma unroll
  for (int k = 0; k < XIW; ++k) {
    const int g = patch_geo(min((wave + 4 * k) * 16 + (lane >> 2), PROWS - 1));  // stored row
    xgeo[k] = g;
  }
#pragma unroll
  for (int it = 0; it < FQ; ++it) {
    const int q = tid + it * 256;
    fgeo[it] = q < PROWS * 4 ? patch_geo(q >> 2) : -1;
  }

  for (int tile = blockIdx.z; tile < p.ntiles; tile += gridDim.z) {
    const int img0 = (tile / tiles_per_img) * NI, tr = tile % tiles_per_img;
    const int y0 = (tr / p.tiles_w) * TH, x0 = (tr % p.tiles_w) * TW;
    const bool ragged = img0 + NI > p.NF || y0 + TH > p.OH || x0 + TW > p.OW;
    const int iy0 = S * y0 - 1, ix0 = S * x0 - 1;
    // (block-uniform) the whole patch inside the frames
    const bool xin = iy0 >= 0 && ix0 >= 0 && iy0 + PH <= p.IH && ix0 + PW <= p.IW && img0 + NI <= p.NF;
    const int ybase = ((img0 * p.OH + y0) * p.OW + x0) * p.Co + co0;
    const int xbase = ((img0 * p.IH + iy0) * p.IW + ix0) * p.Ci + ci0;
    auto xok = [&](int g) {
      return xin || (img0 + (g >> 16) < p.NF && (unsigned)(iy0 + ((g >> 8) & 255)) < (unsigned)p.IH &&
                     (unsigned)(ix0 + (g & 255)) < (unsigned)p.IW);
    };
    lds_barrier();  // the previous tile's fragment reads are done
#pragma unroll
    for (int u = 0; u < YI / 4; ++u) {
      const int i = wave + 4 * u, f = i / (TPX / 16), pb = i % (TPX / 16);
      const int g = ygeo[u], mi = (g >> 16) & 255, py = (g >> 8) & 255, px = g & 255;
      // (pixels outside the map: any in-range row, zeroed by the ragged pass below)
      const bool ok = !ragged || (img0 + mi < p.NF && y0 + py < p.OH && x0 + px < p.OW);
      const int off = ((mi * p.OH + py) * p.OW + px) * p.Co + (g >> 24) * 32 + (lane & 3) * 8;
      const __bf16* gp = p.dY + (ok ? ybase + off : 0);
      __builtin_amdgcn_global_load_lds((__attribute__((address_space(1))) void*)gp,
                                       (__attribute__((address_space(3))) void*)(ys + f * YIMG + pb * 16 * 32), 16, 0, 0);
    }
#pragma unroll
    for (int k = 0; k < XIW; ++k) {
      const int i = wave + 4 * k;
      if (i < XI) {  // (wave-uniform)
        const int g = xgeo[k];
        const int off = (((g >> 16) * p.IH + ((g >> 8) & 255)) * p.IW + (g & 255)) * p.Ci + (lane & 3) * 8;
        const __bf16* gp = p.src + (xok(g) ? xbase + off : 0);
        __builtin_amdgcn_global_load_lds((__attribute__((address_space(1))) void*)gp,
                                         (__attribute__((address_space(3))) void*)(xs + i * 16 * 32), 16, 0, 0);
      }
    }
    __syncthreads();  // (vmcnt(0) first: every wave's DMA has landed)
#pragma unroll
    for (int it = 0; it < FQ; ++it) {
      const int g = fgeo[it];
      if (g < 0) continue;
      const int row = (tid + it * 256) >> 2;
      u32v4* d = reinterpret_cast<u32v4*>(xs + row * 32 + g4 * 8);
      if (!xok(g)) {
        *d = u32v4{0u, 0u, 0u, 0u};  // zero padding stays zero (the reference pads relu(bn(y)) with zeros)
      } else if (bn) {
        float f[8];
        bf8_to_f32(*d, f);
#pragma unroll
        for (int e = 0; e < 8; ++e) {  // (NaN propagates like torch's relu)
          const float r = fmaf(f[e], sc[e], sh[e]);
          f[e] = r <= 0.f ? 0.f : r;
        }
        *d = f32_to_bf8(f);
      }
    }
    if (ragged) {  // (block-uniform) dY rows of pixels outside the map
      for (int q = tid; q < TPX * 4 * NCO; q += 256) {
        const int m = q / (4 * NCO), pc = q % (4 * NCO);
        const int mi = m / (TH * TW), mr = m % (TH * TW);
        if (img0 + mi >= p.NF || y0 + mr / TW >= p.OH || x0 + mr % TW >= p.OW)
          *reinterpret_cast<u32v4*>(ys + (pc >> 2) * YIMG + m * 32 + (pc & 3) * 8) = u32v4{0u, 0u, 0u, 0u};
      }
    }
    lds_barrier();
#pragma unroll 1
    for (int k = 0; k < KSW; ++k) {
      // rows of this lane's transposed reads: tile pixels 16 (ks0 + k) + 8h + 4u + q4, u = 0, 1
      const int m0 = (ks0 + k) * 16 + 8 * h + q4;
      const int mi = m0 / (TH * TW), mr = m0 % (TH * TW), oy = mr / TW, ox = mr % TW;
      const __bf16* ya = ys + ct * YIMG + m0 * 32 + 16 * g16 + 4 * p4;
      const bfv8 a = tr_frag(ya, ya + 4 * 32);
      const int prow = (mi * PH + S * oy) * PW;
      auto bfrag = [&](int t) {
        const int kh = t / 3, kw = t % 3;
        const int col = S == 1 ? ox + kw : ((kw & 1) ? PWE + ox + (kw >> 1) : ox + (kw >> 1));
        const __bf16* xb = xs + (prow + kh * PW + col) * 32 + 16 * g16 + 4 * p4;
        return tr_frag(xb, xb + 4 * 32);
      };
      // tap t + 1's fragment is read before tap t's MFMA (left to itself the compiler waits on each tap's own two
      // transposed reads right before its MFMA: MFMA busy 0.12)
      // (two taps ahead where the registers allow: the 144 accumulators leave 8-16 VGPRs)
      constexpr int PD = (S == 1 && NCO == 1) ? 2 : 1;
      bfv8 bq[PD + 1];
#pragma unroll
      for (int t = 0; t < PD; ++t) bq[t] = bfrag(t);
#pragma unroll
      for (int t = 0; t < 9; ++t) {
        if (t + PD < 9) bq[(t + PD) % (PD + 1)] = bfrag(t + PD);
        __builtin_amdgcn_sched_barrier(0);
        acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, bq[t % (PD + 1)], acc[t], 0, 0, 0);
      }
    }
  }

  // the WPC waves of a co tile, fixed order ((0 + 1) + (2 + 3) for NCO = 1; 0 + 1 per tile for NCO = 2), 3 taps at a time
  float* out = p.slab + (int64_t)blockIdx.z * p.Co * 9 * p.Ci;
  float* red = reinterpret_cast<float*>(sm);  // [2 waves][3 taps][16][64]
  const int cob = co0 + ct * 32;
#pragma unroll
  for (int tc = 0; tc < 3; ++tc) {
    if constexpr (NCO == 1) {
      __syncthreads();
      if (wave & 1) {
#pragma unroll
        for (int u = 0; u < 3; ++u)
#pragma unroll
          for (int r = 0; r < 16; ++r) red[(((wave >> 1) * 3 + u) * 16 + r) * 64 + lane] = acc[tc * 3 + u][r];
      }
      __syncthreads();
      if (!(wave & 1)) {
#pragma unroll
        for (int u = 0; u < 3; ++u)
#pragma unroll
          for (int r = 0; r < 16; ++r) acc[tc * 3 + u][r] += red[(((wave >> 1) * 3 + u) * 16 + r) * 64 + lane];
      }
      __syncthreads();
      if (wave == 2) {
#pragma unroll
        for (int u = 0; u < 3; ++u)
#pragma unroll
          for (int r = 0; r < 16; ++r) red[(u * 16 + r) * 64 + lane] = acc[tc * 3 + u][r];
      }
      __syncthreads();
      if (wave == 0) {
#pragma unroll
        for (int u = 0; u < 3; ++u)
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int co = cob + (r & 3) + 8 * (r >> 2) + 4 * h, t = tc * 3 + u;
            out[(int64_t)co * 9 * p.Ci + t * p.Ci + ci0 + j] = acc[t][r] + red[(u * 16 + r) * 64 + lane];
          }
      }
    } else {
      __syncthreads();
      if (wave & 1) {
#pragma unroll
        for (int u = 0; u < 3; ++u)
#pragma unroll
          for (int r = 0; r < 16; ++r) red[(((wave >> 1) * 3 + u) * 16 + r) * 64 + lane] = acc[tc * 3 + u][r];
      }
      __syncthreads();
      if (!(wave & 1)) {
#pragma unroll
        for (int u = 0; u < 3; ++u)
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int co = cob + (r & 3) + 8 * (r >> 2) + 4 * h, t = tc * 3 + u;
            out[(int64_t)co * 9 * p.Ci + t * p.Ci + ci0 + j] =
                acc[t][r] + red[(((wave >> 1) * 3 + u) * 16 + r) * 64 + lane];
          }
      }
    }
  }
}

// ---------------------------------------------------------------------------------------------------------------
// Stride-2 input gradient: dX[y][x] = sum over the taps with (y + 1 - kh) and (x + 1 - kw) even of
// dY[(y + 1 - kh) / 2][(x + 1 - kw) / 2] W[kh][kw].  The four parity classes (ph, pw) of dX are small convolutions
// of dY with 1x1, 1x2, 2x1 and 2x2 taps (ph = 0: kh = 1 at dY row yc; ph = 1: kh = 0 at row yc + 1, kh = 2 at row
// yc) -- 9 taps in all, like one stride-1 tile.  A block owns an 8 x 16 tile of the class grid and all four classes:
// the classes share one staged 9 x 17 dY patch and the 9-tap weight slice, wave w takes class-grid rows 2w, 2w + 1
// (32 class pixels) of every class (four accumulators).  The epilogue writes the four classes' rows to LDS and
// stores 16-B pieces at dX rows (2 yc + ph, 2 xc + pw), with the fused BN-backward reduce as in bfc_conv_kernel.
// the 9 (class, tap) pairs in class order: class c = 2 ph + pw, kh = ph ? {0, 2} : {1}, kw = pw ? {0, 2} : {1}
__device__ __forceinline__ void s2_pair(int i, int& c, int& kh, int& kw) {
  c = i == 0 ? 0 : (i <= 2 ? 1 : (i <= 4 ? 2 : 3));
  const int q = i == 0 ? 0 : (i <= 2 ? i - 1 : (i <= 4 ? i - 3 : i - 5));
  const int ph = c >> 1, pw = c & 1;
  kh = ph ? 2 * (pw ? q >> 1 : q) : 1;
  kw = pw ? 2 * (ph ? q & 1 : q) : 1;
}

template <int CB, bool WRES, int NI>
__global__ __launch_bounds__(256, 2) void bfc_dgrad_s2_kernel(const BfcArgs p) {
  // NI = 1: one frame's 8 x 16 class tile; NI = 2: 8 x 8 class tiles of two frames (class grids 8 wide or less)
  constexpr int NTHR = 256, TH = 8, TW = 16 / NI, TPX = NI * TH * TW, NC = 32, G8 = CB / 8, NG = NC / 8, KK = CB / 16;
  constexpr int PH = TH + 1, PW = TW + 1, PFR = PH * PW, PROWS = NI * PFR;
  constexpr int RP = CB + 8, WP = 9 * CB + 8, EP = NC + 8;
  static_assert(((RP / 8) & 1) && ((WP / 8) & 1) && ((EP / 8) & 1), "odd 16-B row pitches");
  constexpr int PE = PROWS * RP > 4 * TPX * EP ? PROWS * RP : 4 * TPX * EP;
  __shared__ __attribute__((aligned(16))) __bf16 sm[PE + NC * WP + 2 * 4 * NC];
  __bf16* const patch = sm;
  __bf16* const wl = sm + PE;
  float* const cst = reinterpret_cast<float*>(sm + PE + NC * WP);  // [mean | invstd | scale | shift] of the block's NC
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int h = lane >> 5, j = lane & 31;
  const int tiles_per_img = p.tiles_h * p.tiles_w;
  const int n0 = blockIdx.y * NC;
  const int t0 = blockIdx.x * p.tpb, t1 = min(p.ntiles, t0 + p.tpb);
  const int nch = p.C / CB;
  const int nitems = (t1 - t0) * nch;
  const bool bnb = p.bny != nullptr;
  if (bnb)
    for (int q = tid; q < 4 * NC; q += NTHR) cst[q] = p.bnst[(q / NC) * p.N + min(n0 + q % NC, p.N - 1)];
  __syncthreads();
  if (nitems <= 0) return;
  // this lane's class pixel (row j of the wave's 32): patch row of offset (0, 0)
  const int am = wave * 32 + j;
  const int arow = (am / (TH * TW)) * PFR + ((am % (TH * TW)) / TW) * PW + am % TW;

  constexpr int PQ = PROWS * G8, PIT = (PQ + NTHR - 1) / NTHR;
  constexpr int WQ = NC * 9 * G8, WIT = (WQ + NTHR - 1) / NTHR;
  const int g8 = tid % G8;
  u32v4 pv[PIT], wv[WIT];
  bool pok[PIT];
  auto origin = [&](int tile, int& img, int& yc0, int& xc0) {  // (img: the tile's first frame)
    img = (tile / tiles_per_img) * NI;
    const int tr = tile % tiles_per_img;
    yc0 = (tr / p.tiles_w) * TH;
    xc0 = (tr % p.tiles_w) * TW;
  };
  auto fetch_w = [&](int ch) {
    const int c0 = ch * CB + g8 * 8;
#pragma unroll
    for (int it = 0; it < WIT; ++it) {
      const int q = min(tid + it * NTHR, WQ - 1);
      const int n = q / (9 * G8), t = (q / G8) % 9;
      wv[it] = *reinterpret_cast<const u32v4*>(p.w + ((int64_t)(n0 + n) * 9 + t) * p.C + c0);
    }
  };
  auto stash_w = [&]() {
#pragma unroll
    for (int it = 0; it < WIT; ++it) {
      const int q = tid + it * NTHR;
      if (q < WQ) *reinterpret_cast<u32v4*>(wl + (q / (9 * G8)) * WP + ((q / G8) % 9) * CB + g8 * 8) = wv[it];
    }
  };
  auto fetch = [&](int tile, int ch) {
    int img, yc0, xc0;
    origin(tile, img, yc0, xc0);
    const int c0 = ch * CB + g8 * 8;
#pragma unroll
    for (int it = 0; it < PIT; ++it) {
      const int q = tid + it * NTHR;
      const int row = min(q / G8, PROWS - 1), fr = row / PFR, rr = row % PFR;
      const int iy = yc0 + rr / PW, ix = xc0 + rr % PW;
      pok[it] = q < PQ && iy < p.IH && ix < p.IW && img + fr < p.NF;
      pv[it] = *reinterpret_cast<const u32v4*>(
          p.src + (pok[it] ? (((int64_t)(img + fr) * p.IH + iy) * p.IW + ix) * p.C : 0) + c0);
    }
    if constexpr (!WRES) fetch_w(ch);
  };
  auto stash = [&]() {
#pragma unroll
    for (int it = 0; it < PIT; ++it) {
      const int q = tid + it * NTHR;
      if (q < PQ)
        *reinterpret_cast<u32v4*>(patch + (q / G8) * RP + g8 * 8) = pok[it] ? pv[it] : u32v4{0u, 0u, 0u, 0u};
    }
    if constexpr (!WRES) stash_w();
  };
  // fragments of K step s: (class, tap) pair s / KK, 16-channel slice s % KK
  auto frags = [&](int s, bfv8& a, bfv8& b) {
    int c, kh, kw;
    s2_pair(s / KK, c, kh, kw);
    const int kk = s % KK;
    const int dr = (c >> 1) ? (kh == 0 ? 1 : 0) : 0, dc = (c & 1) ? (kw == 0 ? 1 : 0) : 0;
    b = *reinterpret_cast<const bfv8*>(wl + j * WP + (kh * 3 + kw) * CB + kk * 16 + 8 * h);
    a = *reinterpret_cast<const bfv8*>(patch + (arow + dr * PW + dc) * RP + kk * 16 + 8 * h);
  };

  const int cg = tid % NG;
  constexpr int EQ = 4 * TPX * NG, EIT = EQ / NTHR;
  static_assert(EQ % NTHR == 0, "whole epilogue passes");
  float s1[8], s2[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) s1[e] = s2[e] = 0.f;
  u32v4 yv[EIT];
  f32x16 acc[4];
  if constexpr (WRES) {
    fetch_w(0);
    stash_w();
  }
  fetch(t0, 0);
  for (int item = 0; item < nitems; ++item) {
    const int tile = t0 + item / nch, ch = item % nch;
    lds_barrier();
    stash();
    lds_barrier();
    int img, yc0, xc0;
    origin(tile, img, yc0, xc0);
    auto piece = [&](int i, int& cm, int64_t& oi) {  // epilogue piece i: class pixel row cm, NHWC offset (or -1)
      const int q = tid + i * NTHR;
      cm = q / NG;
      const int c = cm / TPX, m = cm % TPX, fr = m / (TH * TW), mm = m % (TH * TW);
      const int yy = 2 * (yc0 + mm / TW) + (c >> 1), xx = 2 * (xc0 + mm % TW) + (c & 1);
      oi = (yy < p.OH && xx < p.OW && img + fr < p.NF)
               ? (((int64_t)(img + fr) * p.OH + yy) * p.OW + xx) * p.N + n0 + cg * 8 : -1;
    };
    if (bnb && ch == nch - 1) {  // the layer below's y at the pixels this item writes (issued before the prefetch)
#pragma unroll
      for (int i = 0; i < EIT; ++i) {
        int cm;
        int64_t oi;
        piece(i, cm, oi);
        yv[i] = *reinterpret_cast<const u32v4*>(p.bny + (oi < 0 ? 0 : oi));
      }
    }
    {
      const int nx = min(item + 1, nitems - 1);
      fetch(t0 + nx / nch, nx % nch);
    }
    if (ch == 0) {
#pragma unroll
      for (int c = 0; c < 4; ++c)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[c][r] = 0.f;
    }
    {
      bfv8 a0, b0, a1, b1;
      frags(0, a0, b0);
#pragma unroll
      for (int s = 0; s < 9 * KK; ++s) {
        if (s + 1 < 9 * KK) frags(s + 1, (s & 1) ? a0 : a1, (s & 1) ? b0 : b1);
        int c, kh, kw;
        s2_pair(s / KK, c, kh, kw);
        acc[c] = __builtin_amdgcn_mfma_f32_32x32x16_bf16((s & 1) ? a1 : a0, (s & 1) ? b1 : b0, acc[c], 0, 0, 0);
      }
    }
    if (ch == nch - 1) {
      lds_barrier();  // every wave is done reading the patch
      __bf16* epi = patch;  // [class][pixel][channel]
#pragma unroll
      for (int c = 0; c < 4; ++c)
#pragma unroll
        for (int r = 0; r < 16; ++r)
          epi[(c * TPX + wave * 32 + (r & 3) + 8 * (r >> 2) + 4 * h) * EP + j] = (__bf16)acc[c][r];
      lds_barrier();
      float bmean[8], binv[8], bsc[8], bsh[8];
      if (bnb) {
#pragma unroll
        for (int e = 0; e < 8; e += 4) {
          const f32x4 m4 = *reinterpret_cast<const f32x4*>(cst + cg * 8 + e);
          const f32x4 i4 = *reinterpret_cast<const f32x4*>(cst + NC + cg * 8 + e);
          const f32x4 a4 = *reinterpret_cast<const f32x4*>(cst + 2 * NC + cg * 8 + e);
          const f32x4 b4 = *reinterpret_cast<const f32x4*>(cst + 3 * NC + cg * 8 + e);
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            bmean[e + u] = m4[u];
            binv[e + u] = i4[u];
            bsc[e + u] = a4[u];
            bsh[e + u] = b4[u];
          }
        }
      }
#pragma unroll
      for (int i = 0; i < EIT; ++i) {
        int cm;
        int64_t oi;
        piece(i, cm, oi);
        const u32v4 ev = *reinterpret_cast<const u32v4*>(epi + cm * EP + cg * 8);
        if (oi < 0) continue;
        *reinterpret_cast<u32v4*>(p.out + oi) = ev;
        if (bnb) {
          float f[8], yy[8];
          bf8_to_f32(ev, f);
          bf8_to_f32(yv[i], yy);
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            const float dz = fmaf(yy[e], bsc[e], bsh[e]) > 0.f ? f[e] : 0.f;
            s1[e] += dz;
            s2[e] = fmaf(dz, (yy[e] - bmean[e]) * binv[e], s2[e]);
          }
        }
      }
    }
  }
  if (bnb && p.partials) {
#pragma unroll
    for (int o = NG; o < 64; o <<= 1)
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        s1[e] += __shfl_xor(s1[e], o, 64);
        s2[e] += __shfl_xor(s2[e], o, 64);
      }
    __syncthreads();
    float* red = reinterpret_cast<float*>(sm);  // [4 waves][2][NC]
    if (lane < NG) {
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        red[(wave * 2 + 0) * NC + lane * 8 + e] = s1[e];
        red[(wave * 2 + 1) * NC + lane * 8 + e] = s2[e];
      }
    }
    __syncthreads();
    for (int q = tid; q < 2 * NC; q += NTHR) {
      const int which = q / NC, c = q % NC;
      const float v = (red[(0 + which) * NC + c] + red[(2 + which) * NC + c]) +
                      (red[(4 + which) * NC + c] + red[(6 + which) * NC + c]);
      p.partials[(int64_t)(which * p.N + n0 + c) * gridDim.x + blockIdx.x] = v;
    }
  }
}

// ---------------------------------------------------------------------------------------------------------------
// host side
int g_bfc = 1;             // knob "conv_bfc": config-4 forwards / stride-1 input gradients on these kernels
int g_bfc_blocks = 512;    // knob "conv_bfc_blocks": target grid (persistent blocks over the tiles)
int g_bfc_s2_ni2 = 1;      // knob "conv_bfc_s2_ni2": stride-2 input gradients of class grids <= 8 wide on 2-frame tiles

bool bfc_supported(const Conv3Layer& L, bool fwd) {
  if (!g_bfc || !g_conv_bf16 || !g_act_bf16) return false;
  if (L.stride != 1 && L.stride != 2) return false;
  if (!fwd && L.stride == 2)  // the parity-class kernel: dX exactly 2x the dY grid (padding 1)
    return L.Co % 16 == 0 && L.Ci % 32 == 0 && L.OH == (L.IH - 1) / 2 + 1 && L.OW == (L.IW - 1) / 2 + 1;
  const int C = fwd ? L.Ci : L.Co, N = fwd ? L.Co : L.Ci;
  return C % 16 == 0 && N % 32 == 0;
}

template <int S, int NI, int TH, int TW, int CB, int NCT, bool FWD>
static int bfc_launch(BfcArgs a, int64_t max_blocks, hipStream_t st, int* nparts) {
  VAD_CHECK(a.C % CB == 0 && a.N % (32 * NCT) == 0, "bfc_conv: channel counts");
  VAD_CHECK((int64_t)a.NF * a.IH * a.IW * a.C < (1ll << 31) && (int64_t)a.NF * a.OH * a.OW * a.N < (1ll << 31),
            "bfc_conv: tensors of 2^31 elements or more (32-bit offsets)");
  a.tiles_h = (int)cdiv(a.OH, TH);
  a.tiles_w = (int)cdiv(a.OW, TW);
  a.ntiles = (int)(cdiv(a.NF, NI) * a.tiles_h * a.tiles_w);
  const int ny = a.N / (32 * NCT);
  const int64_t target = std::max<int64_t>(1, std::min<int64_t>(max_blocks, cdiv(g_bfc_blocks, ny)));
  a.tpb = (int)cdiv(a.ntiles, target);
  const int gx = (int)cdiv(a.ntiles, a.tpb);
  if (a.C == CB) VAD_KLAUNCH((bfc_conv_kernel<S, NI, TH, TW, CB, NCT, FWD, true>), dim3(gx, ny), dim3(256), 0, st, a);
  else VAD_KLAUNCH((bfc_conv_kernel<S, NI, TH, TW, CB, NCT, FWD, false>), dim3(gx, ny), dim3(256), 0, st, a);
  VAD_LAUNCH_CHECK();
  if (nparts) *nparts = gx;
  return 0;
}

// geometry per layer shape: stride 1 on 16x16 tiles (4 frames of 8x8 for 8-wide maps), stride 2 on 8x16 output
// tiles (two 8x8 frames) with 16-channel chunks; 64 output channels per block where N allows it
template <bool FWD>
static int bfc_dispatch(const BfcArgs& a, int stride, int64_t max_blocks, hipStream_t st, int* nparts) {
  if constexpr (FWD) {
    const bool n64 = a.N % 64 == 0;
    if (stride == 2) {
      if (a.OW <= 8)
        return n64 ? bfc_launch<2, 2, 8, 8, 16, 2, FWD>(a, max_blocks, st, nparts)
                   : bfc_launch<2, 2, 8, 8, 16, 1, FWD>(a, max_blocks, st, nparts);
      return n64 ? bfc_launch<2, 1, 8, 16, 16, 2, FWD>(a, max_blocks, st, nparts)
                 : bfc_launch<2, 1, 8, 16, 16, 1, FWD>(a, max_blocks, st, nparts);
    }
    if (a.OW <= 8 && a.OH <= 8) {
      if (a.C % 32 == 0)
        return n64 ? bfc_launch<1, 4, 8, 8, 32, 2, FWD>(a, max_blocks, st, nparts)
                   : bfc_launch<1, 4, 8, 8, 32, 1, FWD>(a, max_blocks, st, nparts);
      return bfc_launch<1, 4, 8, 8, 16, 1, FWD>(a, max_blocks, st, nparts);
    }
    if (a.C % 32 == 0)
      return (n64 && a.C > 32) ? bfc_launch<1, 1, 16, 16, 32, 2, FWD>(a, max_blocks, st, nparts)
                               : bfc_launch<1, 1, 16, 16, 32, 1, FWD>(a, max_blocks, st, nparts);
    return bfc_launch<1, 1, 16, 16, 16, 1, FWD>(a, max_blocks, st, nparts);
  } else {
    // input gradients: 32 channels per block (the fused BN-backward reduce's state leaves no registers for 64)
    if (a.OW <= 8 && a.OH <= 8)
      return a.C % 32 == 0 ? bfc_launch<1, 4, 8, 8, 32, 1, FWD>(a, max_blocks, st, nparts)
                           : bfc_launch<1, 4, 8, 8, 16, 1, FWD>(a, max_blocks, st, nparts);
    return a.C % 32 == 0 ? bfc_launch<1, 1, 16, 16, 32, 1, FWD>(a, max_blocks, st, nparts)
                         : bfc_launch<1, 1, 16, 16, 16, 1, FWD>(a, max_blocks, st, nparts);
  }
}

int bfc_fwd(const Conv3Layer& L, const __bf16* src, const float* src_stats, const __bf16* wfb, const float* bias,
            __bf16* y, float* partials, int64_t partial_cap, int* nparts, hipStream_t st) {
  VAD_CHECK(bfc_supported(L, true), "bfc_fwd: unsupported layer");
  BfcArgs a{};
  a.src = src;
  a.scale = src_stats ? src_stats + 2 * L.Ci : nullptr;
  a.shift = src_stats ? src_stats + 3 * L.Ci : nullptr;
  a.w = wfb;
  a.bias = bias;
  a.out = y;
  a.partials = partials;
  a.NF = L.NF; a.IH = L.IH; a.IW = L.IW; a.C = L.Ci; a.OH = L.OH; a.OW = L.OW; a.N = L.Co;
  // (the BN partial buffer holds [2 Co][blocks])
  const int64_t mb = partials ? std::max<int64_t>(1, partial_cap / (2ll * L.Co)) : (1 << 20);
  return bfc_dispatch<true>(a, L.stride, mb, st, nparts);
}

int bfc_dgrad(const Conv3Layer& L, const __bf16* dY, const __bf16* wdb, __bf16* dX, hipStream_t st,
              const BnBwdFuse* f) {
  VAD_CHECK(bfc_supported(L, false), "bfc_dgrad: unsupported layer");
  BfcArgs a{};
  a.src = dY;
  a.w = wdb;
  a.out = dX;
  a.NF = L.NF; a.IH = L.OH; a.IW = L.OW; a.C = L.Co; a.OH = L.IH; a.OW = L.IW; a.N = L.Ci;
  int64_t mb = 1 << 20;
  if (f) {
    a.bny = reinterpret_cast<const __bf16*>(f->y);
    a.bnst = f->stats;
    a.partials = f->parts;
    mb = std::max<int64_t>(1, f->cap / (2ll * L.Ci));
  }
  if (L.stride == 2) {
    // class grids 8 wide or less (the 8 x 8 dY maps of config 4's last stride-2 layer): two frames' 8 x 8 tiles per
    // block tile instead of a half-empty 8 x 16 one
    const int ni = (L.IW + 1) / 2 <= 8 && g_bfc_s2_ni2 ? 2 : 1;
    const int TH = 8, TW = 16 / ni;
    a.tiles_h = (int)cdiv((L.IH + 1) / 2, TH);
    a.tiles_w = (int)cdiv((L.IW + 1) / 2, TW);
    a.ntiles = (int)cdiv(L.NF, ni) * a.tiles_h * a.tiles_w;
    const int ny = L.Ci / 32;
    const int64_t target = std::max<int64_t>(1, std::min<int64_t>(mb, cdiv(g_bfc_blocks, ny)));
    a.tpb = (int)cdiv(a.ntiles, target);
    const int gx = (int)cdiv(a.ntiles, a.tpb);
    if (ni == 2) {
      if (L.Co == 32) VAD_KLAUNCH((bfc_dgrad_s2_kernel<32, true, 2>), dim3(gx, ny), dim3(256), 0, st, a);
      else if (L.Co % 32 == 0) VAD_KLAUNCH((bfc_dgrad_s2_kernel<32, false, 2>), dim3(gx, ny), dim3(256), 0, st, a);
      else VAD_KLAUNCH((bfc_dgrad_s2_kernel<16, false, 2>), dim3(gx, ny), dim3(256), 0, st, a);
    } else if (L.Co == 32) VAD_KLAUNCH((bfc_dgrad_s2_kernel<32, true, 1>), dim3(gx, ny), dim3(256), 0, st, a);
    else if (L.Co % 32 == 0) VAD_KLAUNCH((bfc_dgrad_s2_kernel<32, false, 1>), dim3(gx, ny), dim3(256), 0, st, a);
    else VAD_KLAUNCH((bfc_dgrad_s2_kernel<16, false, 1>), dim3(gx, ny), dim3(256), 0, st, a);
    VAD_LAUNCH_CHECK();
    if (f) *f->nparts = gx;
    return 0;
  }
  return bfc_dispatch<false>(a, 1, mb, st, f ? f->nparts : nullptr);
}

bool bfc_wgrad_supported(const Conv3Layer& L) {
  return g_bfc && g_conv_bf16 && g_act_bf16 && (L.stride == 1 || L.stride == 2) && L.Ci % 32 == 0 && L.Co % 32 == 0;
}

template <int S, int NI, int TH, int TW, int NCO>
static int bfw_launch(BfwArgs a, int target_blocks, int64_t partial_cap, hipStream_t st, int* nsplit) {
  a.tiles_h = (int)cdiv(a.OH, TH);
  a.tiles_w = (int)cdiv(a.OW, TW);
  a.ntiles = (int)(cdiv(a.NF, NI) * a.tiles_h * a.tiles_w);
  const int pairs = (a.Co / (32 * NCO)) * (a.Ci / 32);
  int64_t z = std::max<int64_t>(1, std::min<int64_t>(cdiv(target_blocks, pairs), a.ntiles));
  z = std::min<int64_t>(z, std::max<int64_t>(1, partial_cap / ((int64_t)a.Co * 9 * a.Ci)));
  VAD_KLAUNCH((bfc_wgrad_kernel<S, NI, TH, TW, NCO>), dim3(a.Co / (32 * NCO), a.Ci / 32, (unsigned)z), dim3(256), 0,
              st, a);
  VAD_LAUNCH_CHECK();
  *nsplit = (int)z;
  return 0;
}

int g_bfw_blocks = 384;  // knob "conv_bfw_blocks": target grid of the bf16 weight gradients (sweep: 384 best)

int bfc_wgrad(const Conv3Layer& L, const __bf16* dY, const __bf16* src, const float* src_stats, float* slab,
              int* nsplit, int64_t partial_cap, hipStream_t st) {
  VAD_CHECK(bfc_wgrad_supported(L), "bfc_wgrad: unsupported layer");
  VAD_CHECK(partial_cap >= (int64_t)L.Co * 9 * L.Ci, "bfc_wgrad: slab capacity below one split");
  VAD_CHECK((int64_t)L.NF * L.IH * L.IW * L.Ci < ((int64_t)1 << 31) && (int64_t)L.NF * L.OH * L.OW * L.Co < ((int64_t)1 << 31),
            "bfc_wgrad: 32-bit staging offsets");
  BfwArgs a{};
  a.dY = dY;
  a.src = src;
  a.scale = src_stats ? src_stats + 2 * L.Ci : nullptr;
  a.shift = src_stats ? src_stats + 3 * L.Ci : nullptr;
  a.slab = slab;
  a.NF = L.NF; a.IH = L.IH; a.IW = L.IW; a.Ci = L.Ci; a.OH = L.OH; a.OW = L.OW; a.Co = L.Co;
  const int tb = g_bfw_blocks;
  const bool c64 = L.Co % 64 == 0;
  if (L.stride == 2) {
    VAD_CHECK(L.IH >= 2 * L.OH - 1 && L.IW >= 2 * L.OW - 1, "bfc_wgrad: stride-2 geometry");
    if (L.OW <= 8) return c64 ? bfw_launch<2, 2, 8, 8, 2>(a, tb, partial_cap, st, nsplit)
                              : bfw_launch<2, 2, 8, 8, 1>(a, tb, partial_cap, st, nsplit);
    if (L.OW <= 16) return c64 ? bfw_launch<2, 1, 8, 16, 2>(a, tb, partial_cap, st, nsplit)
                               : bfw_launch<2, 1, 8, 16, 1>(a, tb, partial_cap, st, nsplit);
    return c64 ? bfw_launch<2, 1, 4, 32, 2>(a, tb, partial_cap, st, nsplit)
               : bfw_launch<2, 1, 4, 32, 1>(a, tb, partial_cap, st, nsplit);
  }
  if (L.OW <= 8 && L.OH <= 8) return c64 ? bfw_launch<1, 4, 8, 8, 2>(a, tb, partial_cap, st, nsplit)
                                         : bfw_launch<1, 4, 8, 8, 1>(a, tb, partial_cap, st, nsplit);
  return c64 ? bfw_launch<1, 1, 16, 16, 2>(a, tb, partial_cap, st, nsplit)
             : bfw_launch<1, 1, 16, 16, 1>(a, tb, partial_cap, st, nsplit);
}

}  // namespace vad
