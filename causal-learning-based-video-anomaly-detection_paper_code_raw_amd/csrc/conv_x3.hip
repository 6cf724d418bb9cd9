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
#include "conv3d.h"

namespace vad {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

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
  int parts_cm;  // forward: BN partial sums column-major [2N][gridDim.x] (coalesced finalize reads)
  int D;         // KD == 3 (Conv3d k3 p1 s1): depth of the NDHWC volumes; image index = n * D + d
  // input gradients (nullable): the BN-backward reduce of the layer whose activation this dX is, fused into the
  // epilogue -- bny = that layer's raw output y (same layout as out), bnst = its BN state (mean | invstd | scale |
  // shift); per-block sums of dZ = dX [scale*y + shift > 0] and dZ * xhat go to partials, column-major [2N][gridDim.x]
  const void* bny;
  const float* bnst;
  const __bf16* w3;  // stride-2 input gradient: pre-split Wd planes [N][9][C / 16][3][16] (nullable)
};

// epilogue half of the fused BN-backward reduce (bn_bwd_reduce_kernel's arithmetic on the value just computed; with
// bf16 storage on the value as stored)
struct BnBwdLane {
  float mean, inv, sc, sh;
  __device__ __forceinline__ void load(const float* st, int C, int c) {
    mean = st[c];
    inv = st[C + c];
    sc = st[2 * C + c];
    sh = st[3 * C + c];
  }
  template <bool AB>
  __device__ __forceinline__ static float ld(const void* bny, int64_t idx) {
    return act_ld(reinterpret_cast<const act_t<AB>*>(bny) + idx);
  }
  // (the y values are loaded for the whole epilogue first: one wait instead of a round trip per pixel)
  template <bool AB>
  __device__ __forceinline__ void add(float yy, float v, float& s1, float& s2, bool in = true) const {
    const float a = AB ? (float)(__bf16)v : v;
    const float dz = (in && fmaf(yy, sc, sh) > 0.f) ? a : 0.f;  // (in = false: adds exact zeros)
    s1 += dz;
    s2 = fmaf(dz, (yy - mean) * inv, s2);
  }
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

// stores 8 fp32 values as NP bf16 planes (hi[, mid, lo]) at d, d + pitch, d + 2 pitch
template <int NP>
__device__ __forceinline__ void put_planes(__bf16* d, int pitch, const float* v, bool hi_only) {
  bf16x8 hi, mid, lo;
  if (NP == 1 || hi_only) {
#pragma unroll
    for (int e = 0; e < 8; ++e) hi[e] = mid[e] = lo[e] = (__bf16)v[e];
  } else {
    split3(v, hi, mid, lo);
  }
  *reinterpret_cast<bf16x8*>(d) = hi;
  if constexpr (NP == 3) {
    *reinterpret_cast<bf16x8*>(d + pitch) = mid;
    *reinterpret_cast<bf16x8*>(d + 2 * pitch) = lo;
  }
}

// Output pixel m (0 .. NI*TH*TW) of a tile -> (image, row, column).  Row-major in general; 8x8 tiles (NI = NW/2
// images of one 8x8 block each) map the four 8-pixel groups g of a wave's 32 MFMA rows to rows r + {0, 4, 1, 5}
// (r = 2 (wave & 1)) of image wave / 2, so the 16 lanes of every ds_read_b128 phase (groups 0,1 or 2,3) read patch
// pixels four patch rows apart: 4 * PW * S pixels, == 8 (mod 16) for PW = 10 (S = 1) and 2 * 17 (S = 2), i.e. the
// second 8 lanes land on the other half of the 16 bank quads (row-major: PW = 10 put pixels 16, 17 on the quads of
// pixels 0, 1 -- SQ_LDS_BANK_CONFLICT 0.48 of the LDS cycles on the 8x8 layers)
template <int S, int NI, int TH, int TW, int NW>
__device__ __forceinline__ void tile_pixel(int m, int& mi, int& py, int& px) {
  if constexpr (TH == 8 && TW == 8 && 2 * NI == NW) {
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

// WCH > 1: the block keeps the split weights of all WCH reduction chunks resident in LDS (staged during its first
// tile, p.C == WCH * PC) instead of restaging the chunk's slice for every (tile, chunk) item -- the weight split is
// most of the staging VALU of the 32-channel layers
// NW = 8: 512-thread blocks over 256-pixel tiles (one block per CU): the weight slice staged per item serves twice
// the pixels (the weight staging per MFMA halves) and the halo share of the patch drops
// AB: bf16 activation storage (p.src / p.out hold bf16; only with NP == 1)
// KD = 3: Conv3d 3x3x3, stride 1, padding 1 on NDHWC volumes (images = depth slices, p.D per clip): the three depth taps
// kd are further reduction chunks -- chunk (kd, c0) stages depth slice d + kd - 1 (zero outside the clip) and the
// weight image kd of p.w [KD][N][9][C]; forward only
template <int S, int NI, int TH, int TW, int NT, int PC, bool FWD, int NP, int WCH = 1, int NW = 4, bool AB = false,
          int KD = 1>
__global__ __launch_bounds__(64 * NW, 8 / NW) void conv3x3_x3_kernel(const X3Args p) {
  static_assert(KD == 1 || (KD == 3 && FWD && S == 1 && WCH == 1), "depth taps: stride-1 forwards");
  static_assert(NP == 3 || NP == 1, "three split planes (fp32 numerics) or one (bf16 operands)");
  static_assert(!AB || NP == 1, "bf16 storage with bf16 operands only");
  using TA = act_t<AB>;
  const TA* src = reinterpret_cast<const TA*>(p.src);
  TA* out = reinterpret_cast<TA*>(p.out);
  static_assert(NW == 4 || NW == 8, "4 or 8 waves");
  static_assert(NI * TH * TW == 32 * NW, "a wave owns 32 output pixels");
  constexpr int NTHR = 64 * NW;
  static_assert(FWD || S == 1, "stride-2 input gradients use conv3x3_dgrad_s2_kernel");
  static_assert(PC % 16 == 0, "16-deep K steps");
  constexpr int NC = 32 * NT, G8 = PC / 8;
  constexpr int PH = (TH - 1) * S + 3, PW = (TW - 1) * S + 3, PROWS = NI * PH * PW, PWE = (PW + 1) / 2;
  constexpr int RP = NP * PC + 8;      // patch row: NP planes x PC + 16 B pad (odd number of 16-B units)
  constexpr int WCS = 9 * NP * PC;      // one chunk's weight row segment: 9 taps x NP planes x PC
  constexpr int WP = WCH * WCS + 8;     // weight row: WCH segments + pad
  static_assert(((RP * 2 / 16) & 1) && ((WP * 2 / 16) & 1), "odd 16-B row pitch");
  __shared__ __attribute__((aligned(16))) __bf16 sm[PROWS * RP + NC * WP];
  __bf16* patch = sm;
  __bf16* wl = sm + PROWS * RP;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int h = lane >> 5, j = lane & 31;
  const int tiles_per_img = p.tiles_h * p.tiles_w;
  const int n0 = blockIdx.y * NC;
  const int t0 = blockIdx.x * p.tpb, t1 = min(p.ntiles, t0 + p.tpb);
  const int nchc = p.C / PC, nch = KD * nchc;  // reduction chunks: (depth tap, channel chunk)

  // this lane's A pixel (MFMA row lane & 31) inside the tile
  int mi, py, px;
  tile_pixel<S, NI, TH, TW, NW>(wave * 32 + j, mi, py, px);
  const int arow0 = (mi * PH + py * S) * PW;
  const __bf16* bbase = wl + j * WP + 8 * h;

  // staging: thread tid always handles the channel group g8 = tid % G8 (NTHR % G8 == 0)
  constexpr int PQ = PROWS * G8, PIT = (PQ + NTHR - 1) / NTHR;
  constexpr int WQ = NC * 9 * G8, WIT = (WQ + NTHR - 1) / NTHR;
  const int g8 = tid % G8;  // weight staging: channel group of item q = q % G8
  // patch staging: item q -> (row, channel group) with the group above the 16 low bits, so a 16-lane ds_write_b128
  // phase covers 16 consecutive patch rows of one group -- distinct bank quads at the odd 16-B row pitch (q / G8,
  // q % G8 put 8 rows x 2 groups in a phase: two lanes on one quad in every phase)
  const int g8p = G8 == 2 ? (tid >> 4) & 1 : g8;
  auto prow = [](int q) { return G8 == 2 ? ((q >> 5) << 4) + (q & 15) : q / G8; };
  act_raw4<AB> pv[PIT][2];
  f32x4 wv[WIT][2];
  // prefetch loads are unconditional (out-of-range lanes read a valid dummy address) and the zero padding is applied
  // at stash time from these bits, so no masked-load branch makes the compiler wait for the loads before the MFMAs
  bool pok[PIT], wok[WIT];
  // loop-invariant piece geometry, 32-bit offsets (the host keeps every tensor below 2^31 elements): patch piece it =
  // (image, patch row, input column) packed (-1: past the patch), its NHWC offset from the tile's patch origin and its
  // LDS offset; weight piece it = its offset from row n0 of chunk 0 (-1: past the slice or the last channel)
  int pgeo[PIT], pgo[PIT], plo[PIT], wgo[WIT], wlo[WIT];
#pragma unroll
  for (int it = 0; it < PIT; ++it) {
    const int q = tid + it * NTHR;
    const int row = prow(q), r = min(row, PROWS - 1);
    const int im = r / (PH * PW), rr = r % (PH * PW), ry = rr / PW, scol = rr % PW;
    // (stride 2: staging items run in the stored, parity-split column order, see stash)
    const int rx = S == 1 ? scol : (scol < PWE ? 2 * scol : 2 * (scol - PWE) + 1);
    pgeo[it] = row < PROWS ? (im << 16) | (ry << 8) | rx : -1;
    pgo[it] = ((im * p.IH + ry) * p.IW + rx) * p.C + g8p * 8;
    plo[it] = ((im * PH + ry) * PW + scol) * RP + g8p * 8;
  }
#pragma unroll
  for (int it = 0; it < WIT; ++it) {
    const int q = min(tid + it * NTHR, WQ - 1);
    const int n = q / (9 * G8), t = (q / G8) % 9;
    wgo[it] = (tid + it * NTHR < WQ && n0 + n < p.N) ? (n * 9 + (FWD ? t : 8 - t)) * p.C + g8 * 8 : -1;
    wlo[it] = tid + it * NTHR < WQ ? n * WP + t * NP * PC + g8 * 8 : -1;
  }
  auto origin = [&](int tile, int& img0, int& oy0, int& ox0) {
    img0 = (tile / tiles_per_img) * NI;
    const int tr = tile % tiles_per_img;
    oy0 = (tr / p.tiles_w) * TH;
    ox0 = (tr % p.tiles_w) * TW;
  };
  auto fetch = [&](int tile, int ch, bool weights) {
    int img0, oy0, ox0;
    origin(tile, img0, oy0, ox0);
    const int kd = ch / nchc, c0 = (ch - kd * nchc) * PC;
    const int iy0 = oy0 * S - 1, ix0 = ox0 * S - 1;
    if constexpr (KD == 1) {
      // (block-uniform) the whole patch inside the frames: only the pieces past the patch are masked
      const bool inner = iy0 >= 0 && ix0 >= 0 && iy0 + PH <= p.IH && ix0 + PW <= p.IW && img0 + NI <= p.NF;
      const int base = ((img0 * p.IH + iy0) * p.IW + ix0) * p.C + c0;
#pragma unroll
      for (int it = 0; it < PIT; ++it) {
        const int g = pgeo[it], im = (g >> 16) & 255, ry = (g >> 8) & 255, rx = g & 255;
        pok[it] = g >= 0 && (inner || (img0 + im < p.NF && (unsigned)(iy0 + ry) < (unsigned)p.IH &&
                                       (unsigned)(ix0 + rx) < (unsigned)p.IW));
        const TA* s = src + (pok[it] ? base + pgo[it] : 0);
        pv[it][0] = act_ld4(s);
        pv[it][1] = act_ld4(s + 4);
      }
    } else {
#pragma unroll
      for (int it = 0; it < PIT; ++it) {
        const int g = pgeo[it], im = (g >> 16) & 255, ry = (g >> 8) & 255, rx = g & 255;
        const int iy = iy0 + ry, ix = ix0 + rx;
        // depth slice d + kd - 1 of the same clip
        const int img = img0 + im + kd - 1, d = (img0 + im) % p.D + kd - 1;
        pok[it] = g >= 0 && d >= 0 && d < p.D && img0 + im < p.NF && iy >= 0 && iy < p.IH && ix >= 0 && ix < p.IW;
        const TA* s = src + c0 + g8p * 8 + (pok[it] ? (((int64_t)img * p.IH + iy) * p.IW + ix) * p.C : (int64_t)0);
        pv[it][0] = act_ld4(s);
        pv[it][1] = act_ld4(s + 4);
      }
    }
    if (weights) {
      const float* wsrc = p.w + ((int64_t)kd * p.N + n0) * 9 * p.C + c0;
#pragma unroll
      for (int it = 0; it < WIT; ++it) {
        wok[it] = wgo[it] >= 0;
        const float* s = wok[it] ? wsrc + wgo[it] : p.w;
        wv[it][0] = *reinterpret_cast<const f32x4*>(s);
        wv[it][1] = *reinterpret_cast<const f32x4*>(s + 4);
      }
    }
  };
  auto stash = [&](int tile, int ch, bool weights) {
    const int c0 = (ch % nchc) * PC;
    // (BN constants loaded and used unconditionally -- from a dummy address when there is no BN -- so no load is
    // left pending on a branch the waitcnt analysis would have to assume, which made it drain the prefetch loads
    // before the first MFMA)
    const bool bn = FWD && p.scale;
    f32x4 sc[2], sh[2];
    if constexpr (FWD) {
      const float* scp = bn ? p.scale : p.w;
      const float* shp = bn ? p.shift : p.w;
      sc[0] = *reinterpret_cast<const f32x4*>(scp + c0 + g8p * 8);
      sc[1] = *reinterpret_cast<const f32x4*>(scp + c0 + g8p * 8 + 4);
      sh[0] = *reinterpret_cast<const f32x4*>(shp + c0 + g8p * 8);
      sh[1] = *reinterpret_cast<const f32x4*>(shp + c0 + g8p * 8 + 4);
    }
#pragma unroll
    for (int it = 0; it < PIT; ++it) {
      if (pgeo[it] >= 0) {
        float v[8];
        const f32x4 v0 = act_f4(pv[it][0]), v1 = act_f4(pv[it][1]);
        const bool ok = pok[it];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          v[e] = ok ? v0[e] : 0.f;
          v[4 + e] = ok ? v1[e] : 0.f;
        }
        if constexpr (FWD) {
          if (bn) {  // zero padding stays zero (padded taps read 0 in the reference's zero-padded relu(bn(y)));
                     // selects, no branches; NaN propagates like torch's relu
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              const float a0 = fmaf(v0[e], sc[0][e], sh[0][e]), a1 = fmaf(v1[e], sc[1][e], sh[1][e]);
              v[e] = (a0 <= 0.f || !ok) ? 0.f : a0;
              v[4 + e] = (a1 <= 0.f || !ok) ? 0.f : a1;
            }
          }
        }
        // stride 2: item rr % PW is already the stored column ([even input columns | odd ones]), so the 8 rows a
        // 16-lane ds_write_b128 phase covers are consecutive patch rows -- distinct bank quads at the odd 16-B pitch
        // (raw column order alternated between the two halves: SQ_LDS_BANK_CONFLICT 0.43-0.52 of the LDS cycles)
        put_planes<NP>(patch + plo[it], PC, v, false);
      }
    }
    if (weights) {
#pragma unroll
      for (int it = 0; it < WIT; ++it) {
        if (wlo[it] >= 0) {
          float v[8];
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            v[e] = wok[it] ? wv[it][0][e] : 0.f;
            v[4 + e] = wok[it] ? wv[it][1][e] : 0.f;
          }
          put_planes<NP>(wl + wlo[it] + (WCH > 1 ? (c0 / PC) * WCS : 0), PC, v, false);
        }
      }
    }
    // every load the stash consumed is complete here (vmcnt(0); the next prefetch is issued after the barrier),
    // so the waitcnt analysis does not carry them, pending on some branch, into the MFMA loop and drain the
    // prefetch there
    __builtin_amdgcn_s_waitcnt(0x0F70);
  };

  float bj[NT], s1[NT], s2[NT];
  BnBwdLane bl[NT];
  const bool bnb = !FWD && p.bny;
#pragma unroll
  for (int nt = 0; nt < NT; ++nt) {
    const int col = n0 + nt * 32 + j;
    bj[nt] = (FWD && col < p.N) ? p.bias[col] : 0.f;
    s1[nt] = s2[nt] = 0.f;
    if (bnb) bl[nt].load(p.bnst, p.N, min(col, p.N - 1));
  }
  f32x16 acc[NT];
  const int nitems = (t1 - t0) * nch;
  if (nitems > 0) fetch(t0, 0, true);
  for (int item = 0; item < nitems; ++item) {
    const int tile = t0 + item / nch, ch = item % nch;
    const bool wnow = WCH > 1 ? item < nch : (nch > 1 || item == 0);
    const int wseg = WCH > 1 ? ch * WCS : 0;
    __syncthreads();  // the previous item's fragment reads are done
    stash(tile, ch, wnow);
    __syncthreads();
    if (item + 1 < nitems) {
      const int nx = item + 1;
      fetch(t0 + nx / nch, nx % nch, WCH > 1 ? nx < nch : nch > 1);
    }
    if (ch == 0) {
#pragma unroll
      for (int nt = 0; nt < NT; ++nt)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[nt][r] = 0.f;
    }
    // K steps s = (tap t, 16-channel slice kk); the fragments of step s + 1 are read before step s's MFMAs (one step
    // of register double-buffering: left to itself the compiler reads each fragment right before its MFMA and the
    // single accumulation chain waits on every LDS read)
    auto frag = [&](int sidx, bf16x8 (&a)[NP], bf16x8 (&b)[NT][NP]) {
      const int t = sidx / (PC / 16), kk = sidx % (PC / 16);
      const int kh = t / 3, kw = t % 3;
      const int col = S == 1 ? px + kw : ((kw & 1) ? PWE + px + (kw >> 1) : px + (kw >> 1));
      const __bf16* ap = patch + (arow0 + kh * PW + col) * RP + 8 * h;
#pragma unroll
      for (int q = 0; q < NP; ++q) a[q] = *reinterpret_cast<const bf16x8*>(ap + q * PC + kk * 16);
#pragma unroll
      for (int nt = 0; nt < NT; ++nt)
#pragma unroll
        for (int q = 0; q < NP; ++q)
          b[nt][q] = *reinterpret_cast<const bf16x8*>(bbase + nt * 32 * WP + wseg + (t * NP + q) * PC + kk * 16);
    };
    // (not for 4-wave blocks with two channel tiles: the second fragment set would cost them their second block per CU)
    constexpr int NSTEP = 9 * (PC / 16);
    constexpr bool PF = NT == 1 || NW == 8;
    bf16x8 fa[2][NP], fb[2][NT][NP];
    if constexpr (PF) frag(0, fa[0], fb[0]);
#pragma unroll
    for (int sidx = 0; sidx < NSTEP; ++sidx) {
      const int cur = PF ? sidx & 1 : 0;
      if constexpr (PF) {
        if (sidx + 1 < NSTEP) frag(sidx + 1, fa[cur ^ 1], fb[cur ^ 1]);
        __builtin_amdgcn_sched_barrier(0);  // (keeps those reads ahead of this step's MFMAs)
      } else {
        frag(sidx, fa[0], fb[0]);
      }
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) {
        if constexpr (NP == 3) acc[nt] = mfma_x3(fa[cur], fb[cur][nt], acc[nt]);
        else acc[nt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[cur][0], fb[cur][nt][0], acc[nt], 0, 0, 0);
      }
    }
    if (ch == nch - 1) {
      // row = pixel (r&3) + 8(r>>2) + 4h of the wave's 32, column = channel n0 + 32 nt + j
      int img0, oy0, ox0;
      origin(tile, img0, oy0, ox0);
      float yb[16][NT];
      if (bnb) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          int qi, qy, qx;
          tile_pixel<S, NI, TH, TW, NW>(wave * 32 + (r & 3) + 8 * (r >> 2) + 4 * h, qi, qy, qx);
          const int oy = oy0 + qy, ox = ox0 + qx, img = img0 + qi;
          const bool ok = img < p.NF && oy < p.OH && ox < p.OW;
          const int64_t base = ok ? (((int64_t)img * p.OH + oy) * p.OW + ox) * p.N : 0;
#pragma unroll
          for (int nt = 0; nt < NT; ++nt) yb[r][nt] = BnBwdLane::ld<AB>(p.bny, base + min(n0 + nt * 32 + j, p.N - 1));
        }
      }
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        int qi, qy, qx;
        tile_pixel<S, NI, TH, TW, NW>(wave * 32 + (r & 3) + 8 * (r >> 2) + 4 * h, qi, qy, qx);
        const int oy = oy0 + qy, ox = ox0 + qx, img = img0 + qi;
        if (img < p.NF && oy < p.OH && ox < p.OW) {
          TA* o = out + (((int64_t)img * p.OH + oy) * p.OW + ox) * p.N + n0 + j;
#pragma unroll
          for (int nt = 0; nt < NT; ++nt) {
            if (n0 + nt * 32 + j < p.N) {
              const float v = acc[nt][r] + bj[nt];
              act_st(o + nt * 32, v);
              if (FWD) {
                s1[nt] += v;
                s2[nt] = fmaf(v, v, s2[nt]);
              } else if (bnb) {
                bl[nt].template add<AB>(yb[r][nt], v, s1[nt], s2[nt]);
              }
            }
          }
        }
      }
    }
  }
  if ((FWD || bnb) && p.partials) {
    __syncthreads();
    float* red = reinterpret_cast<float*>(sm);  // [NW waves][2][NC]
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
    for (int q = tid; q < 2 * NC; q += NTHR) {
      const int which = q / NC, c = q % NC;
      float v = 0.f;
#pragma unroll
      for (int w = 0; w < NW; ++w) v += red[(2 * w + which) * NC + c];  // fixed order
      float* dst = p.parts_cm ? p.partials + (int64_t)(which * p.N + n0 + c) * gridDim.x + blockIdx.x
                              : p.partials + (int64_t)blockIdx.x * 2 * p.N + which * p.N + n0 + c;
      if (n0 + c < p.N) *dst = v;
    }
  }
}

// Software-pipelined stride-1 variant (knob "conv_split_pipe"): 32 output channels per block, two LDS patch images
// (and two weight-slice images when the slice is restaged per item), ONE barrier per item.  While the waves multiply
// item k out of image k & 1, they stage item k+1 -- loaded into registers one item earlier -- into the other image,
// the staging pieces (BN+ReLU on load, the three-way split, the LDS stores) placed between the taps' MFMAs so the
// VALU work issues in the matrix cores' shadow instead of in a phase of its own; item k+2's global loads are issued at
// the top of item k (two register sets, the item loop unrolled by two so both stay in registers).  The BN scale /
// shift of every input channel sits in LDS (staged once).  WCH > 1: the whole split weight image is resident, staged
// before the loop.  Same numerics as conv3x3_x3_kernel (the same products per K step in the same fp32 accumulation
// order per output: identical y; the BN partial sums follow this kernel's own block decomposition).
template <int NI, int TH, int TW, int PC, bool FWD, int NP, int WCH, int NW, bool AB = false>
__global__ __launch_bounds__(64 * NW, 1) void conv3x3_x3p_kernel(const X3Args p) {
  static_assert(NP == 3 || NP == 1, "three split planes (fp32 numerics) or one (bf16 operands)");
  static_assert(!AB || NP == 1, "bf16 storage with bf16 operands only");
  using TA = act_t<AB>;
  const TA* src = reinterpret_cast<const TA*>(p.src);
  TA* out = reinterpret_cast<TA*>(p.out);
  static_assert(NI * TH * TW == 32 * NW, "a wave owns 32 output pixels");
  constexpr int S = 1, NTHR = 64 * NW, NC = 32, G8 = PC / 8;
  constexpr int PH = TH + 2, PW = TW + 2, PROWS = NI * PH * PW;
  constexpr int RP = NP * PC + 8, WCS = 9 * NP * PC, WP = WCH * WCS + 8;
  static_assert(((RP * 2 / 16) & 1) && ((WP * 2 / 16) & 1), "odd 16-B row pitch");
  constexpr int WB = WCH > 1 ? 1 : 2;  // weight images: resident, or double-buffered per-item slices
  constexpr int PSZ = PROWS * RP, WSZ = NC * WP, CMAX = 256;
  __shared__ __attribute__((aligned(16))) __bf16 sm[2 * PSZ + WB * WSZ];
  __shared__ __attribute__((aligned(16))) float bnl[2 * CMAX];  // [scale | shift] of every input channel
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int h = lane >> 5, j = lane & 31;
  const int tiles_per_img = p.tiles_h * p.tiles_w;
  const int n0 = blockIdx.y * NC;
  const int t0 = blockIdx.x * p.tpb, t1 = min(p.ntiles, t0 + p.tpb);
  const int nch = p.C / PC;
  const int nitems = (t1 - t0) * nch;
  if (nitems <= 0) return;  // (block-uniform)
  constexpr bool wper = WCH == 1;  // weight slice restaged for every item (the launcher routes nch == 1 elsewhere)
  const bool bn = FWD && p.scale;

  int mi, py, px;
  tile_pixel<S, NI, TH, TW, NW>(wave * 32 + j, mi, py, px);
  const int arow0 = (mi * PH + py) * PW + px;

  constexpr int PQ = PROWS * G8, PIT = (PQ + NTHR - 1) / NTHR;
  constexpr int WQ = NC * 9 * G8, WIT = (WQ + NTHR - 1) / NTHR;
  const int g8 = tid % G8;  // weight staging
  // patch staging: 16 consecutive rows of one channel group per 16-lane write phase (see conv3x3_x3_kernel)
  const int g8p = G8 == 2 ? (tid >> 4) & 1 : g8;
  auto prow = [](int q) { return G8 == 2 ? ((q >> 5) << 4) + (q & 15) : q / G8; };
  struct Regs {
    act_raw4<AB> pv[PIT][2];
    bool pok[PIT];
    f32x4 wv[WIT][2];
    bool wok[WIT];
  };
  Regs R0, R1;
  auto origin = [&](int tile, int& img0, int& oy0, int& ox0) {
    img0 = (tile / tiles_per_img) * NI;
    const int tr = tile % tiles_per_img;
    oy0 = (tr / p.tiles_w) * TH;
    ox0 = (tr % p.tiles_w) * TW;
  };
  auto fetch_w = [&](Regs& R, int ch) {
#pragma unroll
    for (int it = 0; it < WIT; ++it) {
      // (threads past the slice redo its last item: same loads, same LDS bytes -- no divergent branch in the stash)
      const int q = min(tid + it * NTHR, WQ - 1);
      const int n = q / (9 * G8), t = (q / G8) % 9;
      R.wok[it] = n0 + n < p.N;
      const float* s = p.w + ch * PC + g8 * 8 + (R.wok[it] ? ((int64_t)(n0 + n) * 9 + (FWD ? t : 8 - t)) * p.C : (int64_t)0);
      R.wv[it][0] = *reinterpret_cast<const f32x4*>(s);
      R.wv[it][1] = *reinterpret_cast<const f32x4*>(s + 4);
    }
  };
  // loop-invariant piece geometry, 32-bit offsets from the tile's patch origin (the host keeps the input below 2^31
  // elements): patch piece it = (image, patch row, patch column) packed
  int pgeo[PIT], pgo[PIT];
#pragma unroll
  for (int it = 0; it < PIT; ++it) {
    const int row = min(prow(tid + it * NTHR), PROWS - 1);  // (past the patch: the last row again, see fetch_w)
    const int im = row / (PH * PW), rr = row % (PH * PW), ry = rr / PW, rx = rr % PW;
    pgeo[it] = (im << 16) | (ry << 8) | rx;
    pgo[it] = ((im * p.IH + ry) * p.IW + rx) * p.C + g8p * 8;
  }
  auto fetch = [&](Regs& R, int item) {
    const int tile = t0 + item / nch, ch = item % nch;
    int img0, oy0, ox0;
    origin(tile, img0, oy0, ox0);
    const int iy0 = oy0 - 1, ix0 = ox0 - 1;
    // (block-uniform) the whole patch inside the frames
    const bool inner = iy0 >= 0 && ix0 >= 0 && iy0 + PH <= p.IH && ix0 + PW <= p.IW && img0 + NI <= p.NF;
    const int base = ((img0 * p.IH + iy0) * p.IW + ix0) * p.C + ch * PC;
#pragma unroll
    for (int it = 0; it < PIT; ++it) {
      const int g = pgeo[it], im = g >> 16, ry = (g >> 8) & 255, rx = g & 255;
      R.pok[it] = inner || (img0 + im < p.NF && (unsigned)(iy0 + ry) < (unsigned)p.IH &&
                            (unsigned)(ix0 + rx) < (unsigned)p.IW);
      const TA* s = src + (R.pok[it] ? base + pgo[it] : 0);
      R.pv[it][0] = act_ld4(s);
      R.pv[it][1] = act_ld4(s + 4);
    }
    if (wper) fetch_w(R, ch);
  };
  // staging pieces: patch piece `it` of item -> image b; weight piece `it` -> weight image b (segment seg)
  auto stash_p = [&](const Regs& R, int it, int item, __bf16* pimg) {
    {
      const int row = min(prow(tid + it * NTHR), PROWS - 1);
      const int c0 = (item % nch) * PC + g8p * 8;
      float v[8];
      const f32x4 v0 = act_f4(R.pv[it][0]), v1 = act_f4(R.pv[it][1]);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        v[e] = R.pok[it] ? v0[e] : 0.f;
        v[4 + e] = R.pok[it] ? v1[e] : 0.f;
      }
      if constexpr (FWD) {
        // zero padding stays zero: padded taps read 0 in the reference's zero-padded relu(bn(y)) (selects, no branch;
        // NaN propagates like torch's relu)
        if (bn) {
          const bool ok = R.pok[it];
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            const float a = fmaf(e < 4 ? v0[e] : v1[e - 4], bnl[c0 + e], bnl[CMAX + c0 + e]);
            v[e] = (a <= 0.f || !ok) ? 0.f : a;
          }
        }
      }
      put_planes<NP>(pimg + row * RP + g8p * 8, PC, v, false);
    }
  };
  auto stash_w = [&](const Regs& R, int it, __bf16* wimg, int seg) {
    const int q = min(tid + it * NTHR, WQ - 1);
    {
      const int n = q / (9 * G8), t = (q / G8) % 9;
      float v[8];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        v[e] = R.wok[it] ? R.wv[it][0][e] : 0.f;
        v[4 + e] = R.wok[it] ? R.wv[it][1][e] : 0.f;
      }
      put_planes<NP>(wimg + n * WP + seg * WCS + t * NP * PC + g8 * 8, PC, v, false);
    }
  };
  __bf16* const pimg0 = sm;
  __bf16* const pimg1 = sm + PSZ;
  __bf16* const wimg0 = sm + 2 * PSZ;
  __bf16* const wimg1 = sm + 2 * PSZ + (WB - 1) * WSZ;

  // prologue: BN constants of every input channel, resident weights, item 0 staged, item 1 in flight
  if (bn)
    for (int c = tid; c < p.C; c += NTHR) {
      bnl[c] = p.scale[c];
      bnl[CMAX + c] = p.shift[c];
    }
  if (!wper) {
    for (int c = 0; c < (WCH > 1 ? WCH : 1); ++c) {
      fetch_w(R0, c);
#pragma unroll
      for (int it = 0; it < WIT; ++it) stash_w(R0, it, wimg0, WCH > 1 ? c : 0);
    }
  }
  fetch(R0, 0);
  __syncthreads();  // bnl
#pragma unroll
  for (int it = 0; it < PIT; ++it) stash_p(R0, it, 0, pimg0);
  if (wper) {
#pragma unroll
    for (int it = 0; it < WIT; ++it) stash_w(R0, it, wimg0, 0);
  }
  fetch(R1, min(1, nitems - 1));
  __syncthreads();

  float bj = 0.f, s1 = 0.f, s2 = 0.f;
  if (FWD && n0 + j < p.N) bj = p.bias[n0 + j];
  BnBwdLane bl;
  const bool bnb = !FWD && p.bny;
  if (bnb) bl.load(p.bnst, p.N, min(n0 + j, p.N - 1));
  f32x16 acc;

  auto step = [&](auto curc, int k) {
    constexpr int cur = decltype(curc)::value;
    Regs& Rn = cur ? R0 : R1;  // item k+1, loaded one item ago
    Regs& Rf = cur ? R1 : R0;  // item k was staged out of it: item k+2's loads go here
    __bf16* const pc = cur ? pimg1 : pimg0;
    __bf16* const pn = cur ? pimg0 : pimg1;
    __bf16* const wc = (WB == 2 && cur) ? wimg1 : wimg0;
    __bf16* const wn = (WB == 2 && !cur) ? wimg1 : wimg0;
    // unconditional (item indices clamped): the staging of a nonexistent next item rewrites the idle image with
    // copies of the last one, so no branch splits the tap loop and the staging can interleave with the MFMAs
    fetch(Rf, min(k + 2, nitems - 1));
    const int ch = k % nch;
    const int wseg = WCH > 1 ? ch * WCS : 0;
    if (ch == 0) {
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[r] = 0.f;
    }
    const __bf16* bbase = wc + j * WP + 8 * h + wseg;
    // K steps s = (tap, 16-channel slice); step s + 1's fragments are read before step s's MFMAs (as conv3x3_x3_kernel)
    auto frag = [&](int sidx, bf16x8 (&a)[NP], bf16x8 (&b)[NP]) {
      const int t = sidx / (PC / 16), kk = sidx % (PC / 16), kh = t / 3, kw = t % 3;
      const __bf16* ap = pc + (arow0 + kh * PW + kw) * RP + 8 * h;
#pragma unroll
      for (int q = 0; q < NP; ++q) a[q] = *reinterpret_cast<const bf16x8*>(ap + q * PC + kk * 16);
#pragma unroll
      for (int q = 0; q < NP; ++q) b[q] = *reinterpret_cast<const bf16x8*>(bbase + (t * NP + q) * PC + kk * 16);
    };
    bf16x8 fa[2][NP], fb[2][NP];
    frag(0, fa[0], fb[0]);
#pragma unroll
    for (int t = 0; t < 9; ++t) {
#pragma unroll
      for (int kk = 0; kk < PC / 16; ++kk) {
        const int sidx = t * (PC / 16) + kk, cur = sidx & 1;
        if (sidx + 1 < 9 * (PC / 16)) frag(sidx + 1, fa[cur ^ 1], fb[cur ^ 1]);
        __builtin_amdgcn_sched_barrier(0);  // (keeps those reads ahead of this step's MFMAs)
        if constexpr (NP == 3) acc = mfma_x3(fa[cur], fb[cur], acc);
        else acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[cur][0], fb[cur][0], acc, 0, 0, 0);
      }
      // the next item's staging, spread over the taps: patch pieces after taps 0, 4 (, 8), weight pieces after 2, 6
      if ((t & 3) == 0 && t / 4 < PIT) stash_p(Rn, t / 4, min(k + 1, nitems - 1), pn);
      if constexpr (wper)
        if ((t & 3) == 2 && t / 4 < WIT) stash_w(Rn, t / 4, wn, 0);
    }
    // pieces beyond the tap slots (PIT > 3 or WIT > 2)
#pragma unroll
    for (int it = 3; it < PIT; ++it) stash_p(Rn, it, min(k + 1, nitems - 1), pn);
    if constexpr (wper) {
#pragma unroll
      for (int it = 2; it < WIT; ++it) stash_w(Rn, it, wn, 0);
    }
    if (ch == nch - 1) {
      int img0, oy0, ox0;
      origin(t0 + k / nch, img0, oy0, ox0);
      float yb[16];
      if (bnb) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          int qi, qy, qx;
          tile_pixel<S, NI, TH, TW, NW>(wave * 32 + (r & 3) + 8 * (r >> 2) + 4 * h, qi, qy, qx);
          const int oy = oy0 + qy, ox = ox0 + qx, img = img0 + qi;
          const bool ok = img < p.NF && oy < p.OH && ox < p.OW;
          yb[r] = BnBwdLane::ld<AB>(p.bny, (ok ? (((int64_t)img * p.OH + oy) * p.OW + ox) * p.N : 0) + min(n0 + j, p.N - 1));
        }
      }
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        int qi, qy, qx;
        tile_pixel<S, NI, TH, TW, NW>(wave * 32 + (r & 3) + 8 * (r >> 2) + 4 * h, qi, qy, qx);
        const int oy = oy0 + qy, ox = ox0 + qx, img = img0 + qi;
        if (img < p.NF && oy < p.OH && ox < p.OW && n0 + j < p.N) {
          const float v = acc[r] + bj;
          const int64_t oi = (((int64_t)img * p.OH + oy) * p.OW + ox) * p.N + n0 + j;
          act_st(out + oi, v);
          if (FWD) {
            s1 += v;
            s2 = fmaf(v, v, s2);
          } else if (bnb) {
            bl.template add<AB>(yb[r], v, s1, s2);
          }
        }
      }
    }
    __syncthreads();  // image cur read, image cur^1 written: the next item multiplies out of it
  };
  for (int k = 0; k < nitems; k += 2) {
    step(std::integral_constant<int, 0>{}, k);
    if (k + 1 < nitems) step(std::integral_constant<int, 1>{}, k + 1);
  }
  if ((FWD || bnb) && p.partials) {
    float* red = reinterpret_cast<float*>(sm);  // [NW waves][2][32]
    const float a1 = s1 + __shfl_xor(s1, 32, 64);
    const float a2 = s2 + __shfl_xor(s2, 32, 64);
    if (lane < 32) {
      red[(wave * 2 + 0) * NC + lane] = a1;
      red[(wave * 2 + 1) * NC + lane] = a2;
    }
    __syncthreads();
    for (int q = tid; q < 2 * NC; q += NTHR) {
      const int which = q / NC, c = q % NC;
      float v = 0.f;
#pragma unroll
      for (int w = 0; w < NW; ++w) v += red[(2 * w + which) * NC + c];  // fixed order
      float* dst = p.parts_cm ? p.partials + (int64_t)(which * p.N + n0 + c) * gridDim.x + blockIdx.x
                              : p.partials + (int64_t)blockIdx.x * 2 * p.N + which * p.N + n0 + c;
      if (n0 + c < p.N) *dst = v;
    }
  }
}

int g_x3_dgrad_blocks = 512;  // knob "conv_dgrad_blocks"

template <int S, int NI, int TH, int TW, int NT, int PC, bool FWD, int NP, int WCH = 1, int NW = 4>
static int launch_np(X3Args a, int max_blocks, hipStream_t st, int* nparts) {
  VAD_CHECK(!g_act_bf16 || NP == 1, "conv3x3_x3: bf16 activations need the bf16-operand kernels (conv_bf16)");
  VAD_CHECK(WCH == 1 || a.C == WCH * PC, "conv3x3_x3: resident weights need C == WCH * PC");
  VAD_CHECK((int64_t)a.NF * a.IH * a.IW * a.C < ((int64_t)1 << 31) && (int64_t)a.N * 9 * a.C < ((int64_t)1 << 31),
            "conv3x3_x3: 32-bit staging offsets (input and weight images below 2^31 elements)");
  a.tiles_h = (int)cdiv(a.OH, TH);
  a.tiles_w = (int)cdiv(a.OW, TW);
  a.ntiles = (int)(cdiv(a.NF, NI) * a.tiles_h * a.tiles_w);
  const int ny = (int)cdiv(a.N, 32 * NT);
  // 2 resident blocks per CU over 256 CUs (input gradients: knob "conv_dgrad_blocks", they share the GPU with the
  // weight gradients)
  const int target = std::max(1, std::min(max_blocks, (FWD ? 512 : g_x3_dgrad_blocks) * 4 / NW / ny));
  a.tpb = (int)cdiv(a.ntiles, target);
  const int gx = (int)cdiv(a.ntiles, a.tpb);
  if constexpr (NP == 1) {
    if (g_act_bf16)
      VAD_KLAUNCH((conv3x3_x3_kernel<S, NI, TH, TW, NT, PC, FWD, NP, WCH, NW, true>), dim3(gx, ny), dim3(64 * NW), 0,
                  st, a);
    else
      VAD_KLAUNCH((conv3x3_x3_kernel<S, NI, TH, TW, NT, PC, FWD, NP, WCH, NW>), dim3(gx, ny), dim3(64 * NW), 0, st, a);
  } else {
    VAD_KLAUNCH((conv3x3_x3_kernel<S, NI, TH, TW, NT, PC, FWD, NP, WCH, NW>), dim3(gx, ny), dim3(64 * NW), 0, st, a);
  }
  VAD_LAUNCH_CHECK();
  if (nparts) *nparts = gx;
  return 0;
}

int g_conv_split = 1;  // tuning knob "conv_split": 1 = split-bf16 patch kernels where supported, 0 = f32 MFMA
thread_local int g_conv_bf16 = 0;  // bf16-operand convs (one plane, one product; set per plan, see ConvPrecision)
thread_local int g_act_bf16 = 0;   // bf16 activation storage (set per plan, see ActStorage)
int g_x3_nt = 0;       // tuning knob "conv_split_nt": 0 = auto, 1 / 2 = force 32 / 64 output channels per block


int g_x3_wres = 1;  // knob "conv_split_wres": 32-channel stride-1 layers keep all split weights resident in LDS

template <int S, int NI, int TH, int TW, int NT, int PC, bool FWD, int NW = 4>
static int launch_x3(X3Args a, int max_blocks, hipStream_t st, int* nparts) {
  if constexpr (S == 1 && NT == 1) {
    if (g_x3_wres && a.C == 2 * PC) {
      if (g_conv_bf16) return launch_np<S, NI, TH, TW, NT, PC, FWD, 1, 2, NW>(a, max_blocks, st, nparts);
      return launch_np<S, NI, TH, TW, NT, PC, FWD, 3, 2, NW>(a, max_blocks, st, nparts);
    }
  }
  if (g_conv_bf16) return launch_np<S, NI, TH, TW, NT, PC, FWD, 1, 1, NW>(a, max_blocks, st, nparts);
  return launch_np<S, NI, TH, TW, NT, PC, FWD, 3, 1, NW>(a, max_blocks, st, nparts);
}

// knob "conv_split_pipe": stride-1 layers on the software-pipelined kernel (conv3x3_x3p_kernel); bit 0 forwards, bit 1
// input gradients (these share the CUs with the weight gradients, which a 132 KB block leaves no LDS for)
int g_x3_pipe = 1;

template <int NI, int TH, int TW, bool FWD, int NP, int WCH>
static int launch_pipe(X3Args a, int max_blocks, hipStream_t st, int* nparts) {
  constexpr int PC = 16, NW = 8;
  VAD_CHECK(!g_act_bf16 || NP == 1, "conv3x3_x3p: bf16 activations need the bf16-operand kernels (conv_bf16)");
  VAD_CHECK(a.C % PC == 0 && a.C <= 256 && (WCH == 1 ? a.C > PC : a.C == WCH * PC), "conv3x3_x3p: channel count");
  VAD_CHECK((int64_t)a.NF * a.IH * a.IW * a.C < ((int64_t)1 << 31), "conv3x3_x3p: 32-bit staging offsets");
  a.tiles_h = (int)cdiv(a.OH, TH);
  a.tiles_w = (int)cdiv(a.OW, TW);
  a.ntiles = (int)(cdiv(a.NF, NI) * a.tiles_h * a.tiles_w);
  const int ny = (int)cdiv(a.N, 32);
  // one 512-thread block per CU (two patch images + weights: 98-132 KB of LDS)
  const int target = std::max(1, std::min(max_blocks, (FWD ? 256 : g_x3_dgrad_blocks / 2) / ny));
  a.tpb = (int)cdiv(a.ntiles, target);
  const int gx = (int)cdiv(a.ntiles, a.tpb);
  if (NP == 1 && g_act_bf16)
    VAD_KLAUNCH((conv3x3_x3p_kernel<NI, TH, TW, PC, FWD, NP, WCH, NW, NP == 1>), dim3(gx, ny), dim3(64 * NW), 0, st, a);
  else
    VAD_KLAUNCH((conv3x3_x3p_kernel<NI, TH, TW, PC, FWD, NP, WCH, NW>), dim3(gx, ny), dim3(64 * NW), 0, st, a);
  VAD_LAUNCH_CHECK();
  if (nparts) *nparts = gx;
  return 0;
}

template <int NI, int TH, int TW, bool FWD>
static int dispatch_pipe_np(const X3Args& a, int max_blocks, hipStream_t st, int* nparts) {
  const bool wres = g_x3_wres && a.C == 32;
  if (g_conv_bf16)
    return wres ? launch_pipe<NI, TH, TW, FWD, 1, 2>(a, max_blocks, st, nparts)
                : launch_pipe<NI, TH, TW, FWD, 1, 1>(a, max_blocks, st, nparts);
  return wres ? launch_pipe<NI, TH, TW, FWD, 3, 2>(a, max_blocks, st, nparts)
              : launch_pipe<NI, TH, TW, FWD, 3, 1>(a, max_blocks, st, nparts);
}

template <bool FWD>
static int dispatch_pipe(const X3Args& a, int max_blocks, hipStream_t st, int* nparts) {
  if (a.OH <= 8 && a.OW <= 8) return dispatch_pipe_np<4, 8, 8, FWD>(a, max_blocks, st, nparts);
  if (a.OW <= 16) return dispatch_pipe_np<2, 8, 16, FWD>(a, max_blocks, st, nparts);
  return dispatch_pipe_np<1, 8, 32, FWD>(a, max_blocks, st, nparts);
}

int g_x3_big = 1;  // knob "conv_split_big": stride-1 layers on 256-pixel tiles, 512-thread blocks (NW = 8)
int g_x3_s2big = 1;  // knob "conv_split_s2big": fp32 stride-2 forwards on 256-pixel tiles, 8 waves, 32 channels


template <int S, bool FWD, int NT>
static int dispatch_x3_nt(const X3Args& a, int max_blocks, hipStream_t st, int* nparts) {
  const int OH = a.OH, OW = a.OW;
  if constexpr (S == 1) {
    if (g_x3_big) {
      if (OH <= 8 && OW <= 8) return launch_x3<S, 4, 8, 8, NT, 16, FWD, 8>(a, max_blocks, st, nparts);
      if (OW <= 16) return launch_x3<S, 2, 8, 16, NT, 16, FWD, 8>(a, max_blocks, st, nparts);
      return launch_x3<S, 1, 8, 32, NT, 16, FWD, 8>(a, max_blocks, st, nparts);
    }
  }
  if (OH <= 8 && OW <= 8) return launch_x3<S, 2, 8, 8, NT, 16, FWD>(a, max_blocks, st, nparts);
  if (OW <= 16) return launch_x3<S, 1, 8, 16, NT, 16, FWD>(a, max_blocks, st, nparts);
  return launch_x3<S, 1, 4, 32, NT, 16, FWD>(a, max_blocks, st, nparts);
}

template <int S, bool FWD>
static int dispatch_x3(const X3Args& a, int max_blocks, hipStream_t st, int* nparts) {
  if constexpr (S == 2) {
    // fp32 numerics (three split planes): a 128-pixel stride-2 tile needs a 4.5x larger patch than its output, so the
    // 4-wave block's LDS (patch + 64-channel weight slice, 121 KB) allows one block -- one wave per SIMD -- per CU.
    // 256-pixel tiles of 8 waves over 32 output channels fit 152-158 KB: two waves per SIMD
    if (g_x3_s2big && !g_conv_bf16) {
      if (a.OH <= 8 && a.OW <= 8) return launch_x3<2, 4, 8, 8, 1, 16, FWD, 8>(a, max_blocks, st, nparts);
      if (a.OW <= 16) return launch_x3<2, 2, 8, 16, 1, 16, FWD, 8>(a, max_blocks, st, nparts);
      return launch_x3<2, 1, 8, 32, 1, 16, FWD, 8>(a, max_blocks, st, nparts);
    }
  }
  int nt = g_x3_nt;
  if (nt == 0) {
    // 64 channels per block halves the fragment reads per MFMA; keep 32 when that would leave the chip underfull
    const int64_t tiles = conv3_patch_blocks(a.NF, a.OH, a.OW);
    // (stride 2: the 4x larger input patch per tile makes sharing it over 64 channels pay even on a small grid)
    nt = (a.N % 64 == 0 && (S == 2 || tiles * (a.N / 64) >= 512)) ? 2 : 1;
  }
  if constexpr (S == 1) {
    // 32-channel blocks: the pipelined kernel (measured: L0/L1 -1..-3 us, L7 -5 us; on the layers that take 64
    // channels per block it would lose the patch sharing, +10 us each: profiles/r03_pipe_ab.json)
    if ((g_x3_pipe & (FWD ? 1 : 2)) && nt == 1 && a.C <= 256 && a.C > 16 && g_x3_big && !g_conv_bf16)
      return dispatch_pipe<FWD>(a, max_blocks, st, nparts);
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
                 float* y, float* partials, int* nparts, hipStream_t st, int* parts_cm) {
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
  a.parts_cm = parts_cm ? 1 : 0;  // column-major partials when the caller reads them so
  if (parts_cm) *parts_cm = a.parts_cm;
  // BN partial rows are bounded by conv3_patch_blocks (the caller's partial buffer)
  const int max_blocks = (int)std::min<int64_t>(conv3_patch_blocks(L.NF, L.OH, L.OW), 1 << 20);
  return L.stride == 1 ? dispatch_x3<1, true>(a, max_blocks, st, nparts) : dispatch_x3<2, true>(a, max_blocks, st, nparts);
}

// Conv3d 3x3x3 / stride 1 / padding 1 forward (+ bias, no BN sums) on NDHWC volumes: the KD = 3 instantiation of
// conv3x3_x3_kernel on 256-pixel tiles of 8 waves (three split planes: fp32-class numerics)
template <int NI, int TH, int TW, int NT>
static int launch_x3_3d(X3Args a, hipStream_t st) {
  a.tiles_h = (int)cdiv(a.OH, TH);
  a.tiles_w = (int)cdiv(a.OW, TW);
  a.ntiles = (int)(cdiv(a.NF, NI) * a.tiles_h * a.tiles_w);
  const int ny = (int)cdiv(a.N, 32 * NT);
  const int target = std::max(1, 512 * 4 / 8 / ny);
  a.tpb = (int)cdiv(a.ntiles, target);
  const int gx = (int)cdiv(a.ntiles, a.tpb);
  VAD_KLAUNCH((conv3x3_x3_kernel<1, NI, TH, TW, NT, 16, true, 3, 1, 8, false, 3>), dim3(gx, ny), dim3(512), 0, st, a);
  VAD_LAUNCH_CHECK();
  return 0;
}

int conv3d_x3_fwd(int B, int D, int H, int W, int C, int N, const float* src, const float* w3, const float* bias,
                  float* out, hipStream_t st) {
  VAD_CHECK(C % 16 == 0 && N % 32 == 0 && D >= 1, "conv3d_x3_fwd: C % 16 and N % 32");
  VAD_CHECK(!g_act_bf16, "conv3d_x3_fwd: fp32 activations");
  X3Args a{};
  a.src = src;
  a.w = w3;
  a.bias = bias;
  a.out = out;
  a.NF = B * D; a.D = D; a.IH = H; a.IW = W; a.C = C; a.OH = H; a.OW = W; a.N = N;
  const bool nt2 = N % 64 == 0;
  if (H <= 8 && W <= 8) return nt2 ? launch_x3_3d<4, 8, 8, 2>(a, st) : launch_x3_3d<4, 8, 8, 1>(a, st);
  if (W <= 16) return nt2 ? launch_x3_3d<2, 8, 16, 2>(a, st) : launch_x3_3d<2, 8, 16, 1>(a, st);
  return nt2 ? launch_x3_3d<1, 8, 32, 2>(a, st) : launch_x3_3d<1, 8, 32, 1>(a, st);
}

int conv3_x3_dgrad(const Conv3Layer& L, const float* dY, const float* wd, float* dX, hipStream_t st,
                   const BnBwdFuse* f) {
  VAD_CHECK(conv3_x3_supported(L, false), "conv3_x3_dgrad: unsupported layer");
  X3Args a{};
  a.src = dY;
  a.w = wd;
  a.out = dX;
  a.NF = L.NF; a.IH = L.OH; a.IW = L.OW; a.C = L.Co; a.OH = L.IH; a.OW = L.IW; a.N = L.Ci;
  if (f) {
    // (grid bounded by the partial buffer: [2 Ci][blocks])
    const int mb = (int)std::min<int64_t>(512, f->cap / (2ll * L.Ci));
    if (mb >= 64) {
      a.bny = f->y;
      a.bnst = f->stats;
      a.partials = f->parts;
      a.parts_cm = 1;
      return dispatch_x3<1, false>(a, mb, st, f->nparts);
    }
  }
  return dispatch_x3<1, false>(a, 1 << 20, st, nullptr);
}

// =====================================================================================================
// Stride-2 input gradient on the split-bf16 MFMA (the parity-class scheme of conv_patch.hip's f32 kernel): the four
// parity classes (ph, pw) of a 16x16 dX tile read one 9x9 dY patch -- class (ph, pw) uses the kernel rows kh with
// ph + 1 - kh even at dY row offset (ph + 1 - kh) / 2, likewise columns -- so one staged patch and one staged
// 9-tap weight slice serve 1 + 2 + 2 + 4 taps.  Wave w takes the class-tile half w & 1 (4 x 8 class pixels) of two
// classes, (1,1)+(0,0) for waves 0-1 and (0,1)+(1,0) for waves 2-3 (5 / 4 taps), for 32*NT input channels.
// p.src = dY [NF][IH][IW][C = Co], p.w = Wd [N = Ci][9][C], p.out = dX [NF][OH][OW][N].
//
// LDS geometry (SQ_LDS_BANK_CONFLICT was 0.27 of the LDS cycles with 9-pixel patch rows): patch row py is stored at
// LDS row 12 py (12 pixel slots per patch row, 3 unused) and MFMA row m of a wave takes class pixel S2_PERM[m], which
// puts rows 0 and 2 of its 4 x 8 half on the lanes of one ds_read_b128 group ({0-3, 12-15, 20-27}) and rows 1 and 3
// on the other: the 16 lanes of a group then address 16 distinct 16-B slots of the 64 banks (LDS row index mod 16 is
// a bijection for both groups and the 7-slot row pitch is odd), for every tap's uniform (dh, dw) shift.  Staging:
// every global load goes through a buffer resource at a 32-bit offset computed once per thread (per chunk only + c0),
// out-of-range pieces at an offset past the buffer's end (zeros, no selects); the patch pieces are assigned so the 8
// lanes of a ds_write_b128 group store 8 consecutive patch pixels of one channel half.
// =====================================================================================================
__constant__ constexpr int S2_PERM[32] = {0,  1,  2,  3,  8,  9,  10, 11, 12, 13, 14, 15, 4,  5,  6,  7,
                                          24, 25, 26, 27, 16, 17, 18, 19, 20, 21, 22, 23, 28, 29, 30, 31};
constexpr int S2_PR = 12;    // LDS pixel slots per patch row
constexpr int S2_DUMMY = 9;  // patch row 0's pixel slot 9: never read, the target of the staging's empty slots

template <int NT, int PC, int NP, int CPH, int CPW>
__device__ __forceinline__ void dgrad_s2x3_class(f32x16 (&acc)[NT], const __bf16* abase, const __bf16* bbase,
                                                 int WP) {
#pragma unroll
  for (int a = 0; a < (CPH ? 2 : 1); ++a) {
    const int kh = CPH ? (a == 0 ? 0 : 2) : 1, dh = (CPH && a == 0) ? 1 : 0;
#pragma unroll
    for (int b = 0; b < (CPW ? 2 : 1); ++b) {
      const int kw = CPW ? (b == 0 ? 0 : 2) : 1, dw = (CPW && b == 0) ? 1 : 0;
      const __bf16* ap = abase + (dh * S2_PR + dw) * (NP * PC + 8);
      const __bf16* bp = bbase + (kh * 3 + kw) * NP * PC;
#pragma unroll
      for (int kk = 0; kk < PC / 16; ++kk) {
        bf16x8 av[NP];
#pragma unroll
        for (int q = 0; q < NP; ++q) av[q] = *reinterpret_cast<const bf16x8*>(ap + q * PC + kk * 16);
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) {
          bf16x8 bv[NP];
#pragma unroll
          for (int q = 0; q < NP; ++q)
            bv[q] = *reinterpret_cast<const bf16x8*>(bp + nt * 32 * WP + q * PC + kk * 16);
          if constexpr (NP == 3) acc[nt] = mfma_x3(av, bv, acc[nt]);
          else acc[nt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av[0], bv[0], acc[nt], 0, 0, 0);
        }
      }
    }
  }
}

constexpr int S2_OOB = 0x7ffffff0;  // a byte offset past every buffer's end: the load returns zeros
__device__ __forceinline__ __amdgpu_buffer_rsrc_t s2_rsrc(const void* p, int64_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0,
                                           (int)(bytes < (int64_t)S2_OOB ? bytes : (int64_t)S2_OOB), 0x00020000);
}
__device__ __forceinline__ int s2_add(int off, int add) { return off == S2_OOB ? S2_OOB : off + add; }

// W3: the weight slices come pre-split (p.w3, PC == 16, NP == 3): plain 16-B copies instead of the fp32 load + split
template <int NT, int PC, int NP, bool AB = false, bool W3 = false>
__global__ __launch_bounds__(256, 2) void conv3x3_dgrad_s2x3_kernel(const X3Args p) {
  static_assert(!W3 || (NP == 3 && PC == 16), "pre-split weights: 3 planes of 16-channel slices");
  static_assert(PC == 16, "16-channel chunks (two 8-channel halves per patch pixel)");
  static_assert(!AB || NP == 1, "bf16 storage with bf16 operands only");
  using TA = act_t<AB>;
  TA* out = reinterpret_cast<TA*>(p.out);
  constexpr int NC = 32 * NT, PROWS = 9 * S2_PR;
  constexpr int RP = NP * PC + 8, WP = 9 * NP * PC + 8;
  static_assert(((RP * 2 / 16) & 1) && ((WP * 2 / 16) & 1), "odd 16-B row pitch");
  __shared__ __attribute__((aligned(16))) __bf16 sm[PROWS * RP + NC * WP];
  __bf16* patch = sm;
  __bf16* wl = sm + PROWS * RP;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int h = lane >> 5, j = lane & 31;
  const int tiles_per_img = p.tiles_h * p.tiles_w;
  const int img = blockIdx.x / tiles_per_img, trem = blockIdx.x % tiles_per_img;
  const int i0 = (trem / p.tiles_w) * 8, j0 = (trem % p.tiles_w) * 8;  // class-grid origin = dY patch origin
  const int n0 = blockIdx.y * NC;
  const int g = wave & 1;  // class-tile rows 4g .. 4g+3
  const int pj = S2_PERM[j];
  const __bf16* abase = patch + ((4 * g + pj / 8) * S2_PR + pj % 8) * RP + 8 * h;
  const __bf16* bbase = wl + j * WP + 8 * h;
  const int nch = p.C / PC;

  // ---- per-thread staging geometry, computed once (a chunk adds its channel offset to the global offsets)
  // patch pieces: q -> pixel (q / 16) * 8 + q % 8 of the 81, channel half (q / 8) & 1 (176 slots for 162 pieces)
  constexpr int PIT = 1;
  constexpr int WQ = NC * 9 * 2, W3Q = NC * 9 * 6;  // fp32 weights: 8-channel halves; W3: 16-B pieces, 6 per row
  constexpr int WN = ((W3 ? W3Q : WQ) + 255) / 256;
  const __amdgpu_buffer_rsrc_t src_rs = s2_rsrc(p.src, (int64_t)p.NF * p.IH * p.IW * p.C * (int64_t)sizeof(TA));
  const __amdgpu_buffer_rsrc_t w_rs =
      W3 ? s2_rsrc(p.w3, (int64_t)p.N * 9 * p.C * 3 * 2) : s2_rsrc(p.w, (int64_t)p.N * 9 * p.C * 4);
  // global byte offset (S2_OOB: a zero piece) / LDS element offset (slots past the pieces store into S2_DUMMY, an
  // unused pixel slot of patch row 0: no branches in the staging)
  int poff[PIT], plds[PIT];
#pragma unroll
  for (int it = 0; it < PIT; ++it) {
    const int q = tid + it * 256;
    const int row = (q >> 4) * 8 + (q & 7), half = (q >> 3) & 1;
    const int y = i0 + row / 9, x = j0 + row % 9;
    const bool ok = row < 81 && y < p.IH && x < p.IW;
    poff[it] = ok ? (((img * p.IH + y) * p.IW + x) * p.C + half * 8) * (int)sizeof(TA) : S2_OOB;
    plds[it] = row < 81 ? ((row / 9) * S2_PR + row % 9) * RP + half * 8 : S2_DUMMY * RP;
  }
  int woff[WN], wlds[WN];
#pragma unroll
  for (int it = 0; it < WN; ++it) {
    const int q = tid + it * 256;
    if constexpr (W3) {
      const int n = q / 54, t = (q / 6) % 9, jj = q % 6;
      woff[it] = (q < W3Q && n0 + n < p.N) ? (((n0 + n) * 9 + t) * (p.C / 16) * 48 + jj * 8) * 2 : S2_OOB;
      wlds[it] = q < W3Q ? PROWS * RP + n * WP + t * NP * PC + jj * 8 : S2_DUMMY * RP;
    } else {
      const int n = q / 18, t = (q / 2) % 9, half = q % 2;
      woff[it] = (q < WQ && n0 + n < p.N) ? (((n0 + n) * 9 + t) * p.C + half * 8) * 4 : S2_OOB;
      wlds[it] = q < WQ ? PROWS * RP + n * WP + t * NP * PC + half * 8 : S2_DUMMY * RP;
    }
  }

  u32x4 pv[PIT][AB ? 1 : 2];
  u32x4 wv[WN][W3 ? 1 : 2];
  auto fetch = [&](int c0) {
#pragma unroll
    for (int it = 0; it < PIT; ++it) {
      const int o = s2_add(poff[it], c0 * (int)sizeof(TA));
      pv[it][0] = __builtin_amdgcn_raw_buffer_load_b128(src_rs, o, 0, 0);
      if constexpr (!AB) pv[it][1] = __builtin_amdgcn_raw_buffer_load_b128(src_rs, s2_add(o, 16), 0, 0);
    }
#pragma unroll
    for (int it = 0; it < WN; ++it) {
      if constexpr (W3) {
        wv[it][0] = __builtin_amdgcn_raw_buffer_load_b128(w_rs, s2_add(woff[it], c0 * 6), 0, 0);  // (c0 / 16 x 96 B)
      } else {
        const int o = s2_add(woff[it], c0 * 4);
        wv[it][0] = __builtin_amdgcn_raw_buffer_load_b128(w_rs, o, 0, 0);
        wv[it][1] = __builtin_amdgcn_raw_buffer_load_b128(w_rs, s2_add(o, 16), 0, 0);
      }
    }
  };
  auto stash = [&]() {
#pragma unroll
    for (int it = 0; it < PIT; ++it) {
      float v[8];
      if constexpr (AB) {
        const bf16x8 b = __builtin_bit_cast(bf16x8, pv[it][0]);
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = (float)b[e];
      } else {
        const f32x4 v0 = __builtin_bit_cast(f32x4, pv[it][0]), v1 = __builtin_bit_cast(f32x4, pv[it][1]);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          v[e] = v0[e];
          v[4 + e] = v1[e];
        }
      }
      put_planes<NP>(sm + plds[it], PC, v, false);
    }
#pragma unroll
    for (int it = 0; it < WN; ++it) {
      if constexpr (W3) {
        *reinterpret_cast<u32x4*>(sm + wlds[it]) = wv[it][0];
      } else {
        float v[8];
        const f32x4 v0 = __builtin_bit_cast(f32x4, wv[it][0]), v1 = __builtin_bit_cast(f32x4, wv[it][1]);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          v[e] = v0[e];
          v[4 + e] = v1[e];
        }
        put_planes<NP>(sm + wlds[it], PC, v, false);
      }
    }
    __builtin_amdgcn_s_waitcnt(0x0F70);  // (see conv3x3_x3_kernel's stash)
  };

  f32x16 acc0[NT], acc1[NT];
#pragma unroll
  for (int nt = 0; nt < NT; ++nt)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc0[nt][r] = acc1[nt][r] = 0.f;
  fetch(0);
  for (int ch = 0; ch < nch; ++ch) {
    __syncthreads();  // the previous chunk's fragment reads are done
    stash();
    __syncthreads();
    if (ch + 1 < nch) fetch((ch + 1) * PC);
    if (wave < 2) {
      dgrad_s2x3_class<NT, PC, NP, 1, 1>(acc0, abase, bbase, WP);
      dgrad_s2x3_class<NT, PC, NP, 0, 0>(acc1, abase, bbase, WP);
    } else {
      dgrad_s2x3_class<NT, PC, NP, 0, 1>(acc0, abase, bbase, WP);
      dgrad_s2x3_class<NT, PC, NP, 1, 0>(acc1, abase, bbase, WP);
    }
  }
  const int ph0 = wave < 2 ? 1 : 0, pw0 = 1;  // acc0 class: (1,1) or (0,1)
  const int ph1 = wave < 2 ? 0 : 1, pw1 = 0;  // acc1 class: (0,0) or (1,0)
  float s1[NT], s2[NT];
  BnBwdLane bl[NT];
  const bool bnb = p.bny != nullptr;
#pragma unroll
  for (int nt = 0; nt < NT; ++nt) {
    s1[nt] = s2[nt] = 0.f;
    if (bnb) bl[nt].load(p.bnst, p.N, min(n0 + nt * 32 + j, p.N - 1));
  }
  // Two passes, one per parity class.  Branch-free: every store / y load goes through a buffer resource, a pixel
  // outside dX at an offset past the buffer's end (the store is dropped, the load reads 0 and the BN sums mask it).
  // MFMA row m of lane half h is class pixel (cy, cx) = S2_PERM[m] (compile-time per r and h: one select each), at
  // element offset base + cy * 2 OW N + cx * 2 N (32-bit: the host checks dX is below 2 GB).
  const __amdgpu_buffer_rsrc_t out_rs = s2_rsrc(p.out, (int64_t)p.NF * p.OH * p.OW * p.N * (int64_t)sizeof(TA));
  const __amdgpu_buffer_rsrc_t y_rs = s2_rsrc(p.bny, bnb ? (int64_t)p.NF * p.OH * p.OW * p.N * (int64_t)sizeof(TA) : 0);
  const int N2 = 2 * p.N, OWN2 = 2 * p.OW * p.N;
#pragma unroll
  for (int cls = 0; cls < 2; ++cls) {
    const int ph = cls ? ph1 : ph0, pw = cls ? pw1 : pw0;
    const int y0 = 2 * (i0 + 4 * g) + ph, x0 = 2 * j0 + pw;
    const int ylim = p.OH - y0, xlim = p.OW - x0;  // class pixel (cy, cx) lies in dX iff 2 cy < ylim, 2 cx < xlim
    const int base = ((img * p.OH + y0) * p.OW + x0) * p.N + n0 + j;
    int off[16][NT];
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int m0 = (r & 3) + 8 * (r >> 2);  // C row of lane half 0 (half 1: m0 + 4)
      const int cy = h ? S2_PERM[m0 + 4] / 8 : S2_PERM[m0] / 8, cx = h ? S2_PERM[m0 + 4] % 8 : S2_PERM[m0] % 8;
      const bool ok = 2 * cy < ylim && 2 * cx < xlim;
      const int o = base + cy * OWN2 + cx * N2;
#pragma unroll
      for (int nt = 0; nt < NT; ++nt)
        off[r][nt] = (ok && n0 + nt * 32 + j < p.N) ? (o + nt * 32) * (int)sizeof(TA) : S2_OOB;
    }
    float yb[16][NT];
    if (bnb) {
#pragma unroll
      for (int r = 0; r < 16; ++r)
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) {
          if constexpr (AB)
            yb[r][nt] = (float)__builtin_bit_cast(__bf16, __builtin_amdgcn_raw_buffer_load_b16(y_rs, off[r][nt], 0, 0));
          else
            yb[r][nt] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(y_rs, off[r][nt], 0, 0));
        }
    }
#pragma unroll
    for (int r = 0; r < 16; ++r) {
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) {
        const float v = cls ? acc1[nt][r] : acc0[nt][r];
        if constexpr (AB)
          __builtin_amdgcn_raw_buffer_store_b16(__builtin_bit_cast(unsigned short, (__bf16)v), out_rs, off[r][nt], 0, 0);
        else
          __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, v), out_rs, off[r][nt], 0, 0);
        if (bnb) bl[nt].template add<AB>(yb[r][nt], v, s1[nt], s2[nt], off[r][nt] != S2_OOB);
      }
    }
  }
  if (bnb && p.partials) {  // per-block sums, fixed order: lane halves, then the 4 waves
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
      const float v = (red[(0 + which) * NC + c] + red[(2 + which) * NC + c]) +
                      (red[(4 + which) * NC + c] + red[(6 + which) * NC + c]);
      if (n0 + c < p.N) p.partials[(int64_t)(which * p.N + n0 + c) * gridDim.x + blockIdx.x] = v;
    }
  }
}

int g_dgrad_s2_x3 = 1;  // tuning knob "conv_dgrad_s2_x3": stride-2 input gradients on the split-bf16 kernel

bool conv3_x3_dgrad_s2_supported(const Conv3Layer& L) {
  return g_conv_split && g_dgrad_s2_x3 && L.stride == 2 && L.Co % 16 == 0 && L.Ci % 32 == 0 &&
         L.OH == (L.IH - 1) / 2 + 1 && L.OW == (L.IW - 1) / 2 + 1;
}

int g_dgrad_s2_w3 = 1;
int g_dgrad_s2_nt = 1;  // knob "conv_dgrad_s2_nt": 1 = 32 input channels per block (default: config-2 layer 4 92 -> 75 us, profiles/r04_s2_nt_ab.json), 0 = 64 where the grid allows

bool conv3_dgrad_w3_wanted(const Conv3Layer& L) {
  return g_dgrad_s2_w3 && !g_conv_bf16 && conv3_x3_dgrad_s2_supported(L);
}

int conv3_x3_dgrad_s2(const Conv3Layer& L, const float* dY, const float* wd, float* dX, hipStream_t st,
                      const BnBwdFuse* f, const __bf16* w3) {
  VAD_CHECK(conv3_x3_dgrad_s2_supported(L), "conv3_x3_dgrad_s2: unsupported layer");
  VAD_CHECK((int64_t)L.NF * L.IH * L.IW * L.Ci * 4 < 0x7ffffff0ll && (int64_t)L.NF * L.OH * L.OW * L.Co * 4 < 0x7ffffff0ll &&
                (int64_t)L.Ci * 9 * L.Co * 6 < 0x7ffffff0ll,
            "conv3_x3_dgrad_s2: 32-bit offsets (dX, dY and the weight image below 2 GB)");
  X3Args a{};
  a.src = dY;
  a.w = wd;
  a.out = dX;
  const int tiles0 = L.NF * (int)cdiv((L.IH + 1) / 2, 8) * (int)cdiv((L.IW + 1) / 2, 8);
  if (f && f->cap < 2ll * L.Ci * tiles0) f = nullptr;  // (partial buffer too small: the caller runs the separate pass)
  if (f) {
    a.bny = f->y;
    a.bnst = f->stats;
    a.partials = f->parts;
  }
  a.NF = L.NF; a.IH = L.OH; a.IW = L.OW; a.C = L.Co; a.OH = L.IH; a.OW = L.IW; a.N = L.Ci;
  a.tiles_h = (int)cdiv((L.IH + 1) / 2, 8);
  a.tiles_w = (int)cdiv((L.IW + 1) / 2, 8);
  const int tiles = L.NF * a.tiles_h * a.tiles_w;
  // 64 input channels per block where that still gives >= 2 blocks per CU, else 32
  const bool nt2 = g_dgrad_s2_nt != 1 && L.Ci % 64 == 0 && (int64_t)tiles * (L.Ci / 64) >= 512;
  dim3 grid((unsigned)tiles, (unsigned)(L.Ci / (nt2 ? 64 : 32)));
  VAD_CHECK(!g_act_bf16 || g_conv_bf16, "conv3_x3_dgrad_s2: bf16 activations need conv_bf16");
  if (f) *f->nparts = tiles;
  if (g_conv_bf16 && g_act_bf16) {
    if (nt2) VAD_KLAUNCH((conv3x3_dgrad_s2x3_kernel<2, 16, 1, true>), grid, dim3(256), 0, st, a);
    else VAD_KLAUNCH((conv3x3_dgrad_s2x3_kernel<1, 16, 1, true>), grid, dim3(256), 0, st, a);
  } else if (g_conv_bf16) {
    if (nt2) VAD_KLAUNCH((conv3x3_dgrad_s2x3_kernel<2, 16, 1>), grid, dim3(256), 0, st, a);
    else VAD_KLAUNCH((conv3x3_dgrad_s2x3_kernel<1, 16, 1>), grid, dim3(256), 0, st, a);
  } else if (w3) {
    a.w3 = w3;
    if (nt2) VAD_KLAUNCH((conv3x3_dgrad_s2x3_kernel<2, 16, 3, false, true>), grid, dim3(256), 0, st, a);
    else VAD_KLAUNCH((conv3x3_dgrad_s2x3_kernel<1, 16, 3, false, true>), grid, dim3(256), 0, st, a);
  } else {
    if (nt2) VAD_KLAUNCH((conv3x3_dgrad_s2x3_kernel<2, 16, 3>), grid, dim3(256), 0, st, a);
    else VAD_KLAUNCH((conv3x3_dgrad_s2x3_kernel<1, 16, 3>), grid, dim3(256), 0, st, a);
  }
  VAD_LAUNCH_CHECK();
  return 0;
}

// =====================================================================================================
// Stride-1 weight gradient on the split-bf16 MFMA: dW[co][t][ci] = sum_p dY[p][co] * relu(bn(x))[p + off_t][ci].
// GEMM view per tap: M = 32 co (A = dY^T), N = 32 ci (B = shifted input), K = output pixels.  A K step is 16
// consecutive tile pixels; lane half h holds 8 of them, which lie in one tile row (TW % 8 == 0).  LDS holds
//   Ys[co][plane][pixel]           (the dY tile, 3 bf16 planes, pixels contiguous)
//   Xs[ci][plane][patch row][col]  (input patch incl. halo, BN+ReLU on load, cols padded to TW + 8)
// so the A fragment is one b128 read per plane and, per kernel row kh, two aligned b128 reads per plane give
// columns ox..ox+15 from which the kw = 0 / 2 fragments are dword-aligned subsets and kw = 1 is assembled with
// v_alignbyte (a 2-byte shift): no unaligned LDS access.  Every wave owns KS K steps of each tile and all 9 tap
// accumulators; the 4 waves are combined in a fixed order at the end ((0+2) + (1+3)), and the block's sum lands
// in slab blockIdx.z of the [S][co][t*Ci + ci] split-K layout that conv3_wgrad_reduce consumes.
// =====================================================================================================

struct WgX3Args {
  const float* dY;     // [NF][OH][OW][Co]
  const float* src;    // [NF][IH][IW][Ci]
  const float* scale;  // BN+ReLU on load, nullable
  const float* shift;
  float* slab;         // [S][Co][9*Ci]
  int NF, IH, IW, Ci, OH, OW, Co;
  int tiles_h, tiles_w, ntiles;
};

// LDS row pitch (elements, a multiple of 8) with an odd number of 16-B units: the 16 lanes of a b128 read phase
// hit distinct bank quads
constexpr int odd16_pitch(int n) { return ((n / 8) & 1) ? n : n + 8; }
// Staging item t -> (4-channel group, 4-pixel chunk) of the weight-gradient kernels: a 16-lane ds_write_b64 group covers
// 8 consecutive chunks (64 contiguous bytes) of 2 channel rows 4 rows apart, which the odd 16-B pitch puts 16 banks
// apart -- all 32 banks, conflict-free (the previous t & 7 -> channel group mapping stored 8 rows at one column: 4-way,
// SQ_LDS_BANK_CONFLICT 0.6 of the LDS cycles; tools/lds_conflicts.py).  ngroups channel groups; chunks of 8 x ngroups
// items; the group depends on bits 3.. of t only, so a thread keeps its group across 256-item passes when
// 16 % (ngroups / 2) == 0.
// With bf16 activation storage (AB; config 4, HBM-bound) the staging loads are 8 B per lane and this mapping would read
// each 128-B line in two halves from two wave-instructions (measured +43 us/step at config 4): AB keeps the
// channel-fastest mapping (group = t % ngroups, chunk = t / ngroups), whose single bf16 plane costs few stores.
template <bool AB>
__device__ __forceinline__ int stage_group(int t, int ngroups) {
  return AB ? t % ngroups : ((t >> 3) & 1) + 2 * ((t >> 4) % (ngroups / 2));
}
template <bool AB>
__device__ __forceinline__ int stage_chunk(int t, int ngroups) {
  return AB ? t / ngroups : (t & 7) + 8 * (t / (8 * ngroups));
}

__device__ __forceinline__ void wgrad_combine_store(f32x16 (&acc)[9], __bf16* sm, float* out, int co0, int ci0,
                                                    int Ci);

template <int NI, int TH, int TW, bool PF, int NP, bool AB = false>
__global__ __launch_bounds__(256, 2) void conv3x3_wgrad_x3_kernel(const WgX3Args p) {
  static_assert(!AB || NP == 1, "bf16 storage with bf16 operands only");
  using TA = act_t<AB>;
  using R4 = act_raw4<AB>;
  const TA* dYp = reinterpret_cast<const TA*>(p.dY);
  const TA* srcp = reinterpret_cast<const TA*>(p.src);
  constexpr int TPX = NI * TH * TW, KS = TPX / 64;
  static_assert(TPX % 64 == 0 && TW % 8 == 0, "whole 16-pixel K steps per wave, 8-pixel row runs");
  constexpr int PH = TH + 2, PW = TW + 2, PWP = TW + 8, NCG = PWP / 4;
  constexpr int PLANE = NI * PH * PWP, CIP = odd16_pitch(NP * PLANE), DYP = odd16_pitch(NP * TPX);
  constexpr int XE = 32 * CIP, YE = 32 * DYP, RE = 2 * 3 * 16 * 64 * 2;  // RE: the combine buffer (floats x2)
  __shared__ __attribute__((aligned(16))) __bf16 sm[(XE + YE) > RE ? (XE + YE) : RE];
  __bf16* xs = sm;
  __bf16* ys = sm + XE;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int h = lane >> 5, j = lane & 31;
  const int co0 = blockIdx.x * 32, ci0 = blockIdx.y * 32;
  const int tiles_per_img = p.tiles_h * p.tiles_w;
  const int c4 = stage_group<AB>(tid, 8);  // staging: this thread's 4-channel group

  constexpr int XCH = NI * PH * NCG, XQ = (XCH + 7) / 8 * 64, XIT = (XQ + 255) / 256;  // patch: row x 4-column chunks
  constexpr int YCH = TPX / 4, YQ = (YCH + 7) / 8 * 64, YIT = (YQ + 255) / 256;         // dY: 4-pixel chunks
  R4 xv[XIT][4], yv[YIT][4];
  auto origin = [&](int tile, int& i0, int& y0, int& x0) {
    i0 = (tile / tiles_per_img) * NI;
    const int tr = tile % tiles_per_img;
    y0 = (tr / p.tiles_w) * TH;
    x0 = (tr % p.tiles_w) * TW;
  };
  auto fetch = [&](int tile) {
    int i0, y0, x0;
    origin(tile, i0, y0, x0);
#pragma unroll
    for (int it = 0; it < YIT; ++it) {
      const int yk = stage_chunk<AB>(tid + it * 256, 8), lin = yk * 4;
      const int mi = lin / (TH * TW), mr = lin % (TH * TW);
      const int oy = y0 + mr / TW, ox = x0 + mr % TW, img = i0 + mi;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        yv[it][e] = R4{};
        if (yk < YCH && img < p.NF && oy < p.OH && ox + e < p.OW)
          yv[it][e] = act_ld4(dYp + (((int64_t)img * p.OH + oy) * p.OW + ox + e) * p.Co + co0 + c4 * 4);
      }
    }
#pragma unroll
    for (int it = 0; it < XIT; ++it) {
      const int g = stage_chunk<AB>(tid + it * 256, 8);
      const int row = g / NCG, cg = g % NCG;
      const int mi = row / PH, iy = y0 - 1 + row % PH, img = i0 + mi;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int px = cg * 4 + e, ix = x0 - 1 + px;
        xv[it][e] = R4{};
        if (g < XCH && px < PW && img < p.NF && iy >= 0 && iy < p.IH && ix >= 0 && ix < p.IW)
          xv[it][e] = act_ld4(srcp + (((int64_t)img * p.IH + iy) * p.IW + ix) * p.Ci + ci0 + c4 * 4);
      }
    }
  };
  f32x4 sc = {1.f, 1.f, 1.f, 1.f}, sh = {0.f, 0.f, 0.f, 0.f};
  if (p.scale) {
    sc = *reinterpret_cast<const f32x4*>(p.scale + ci0 + c4 * 4);
    sh = *reinterpret_cast<const f32x4*>(p.shift + ci0 + c4 * 4);
  }
  // 4 channels x 4 consecutive pixels -> per channel and plane one 8-B LDS store
  auto put4 = [&](__bf16* dst, int pitch, int plane_stride, const f32x4* v) {
#pragma unroll
    for (int cc = 0; cc < 4; ++cc) {
      typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
      bf16x4 hi, mid, lo;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float x = v[e][cc];
        const __bf16 a = (__bf16)x;
        if (NP == 1) {
          hi[e] = mid[e] = lo[e] = a;
          continue;
        }
        const float r = x - (float)a;
        const __bf16 b = (__bf16)r;
        hi[e] = a;
        mid[e] = b;
        lo[e] = (__bf16)(r - (float)b);
      }
      __bf16* d = dst + (c4 * 4 + cc) * pitch;
      *reinterpret_cast<bf16x4*>(d) = hi;
      if constexpr (NP == 3) {
        *reinterpret_cast<bf16x4*>(d + plane_stride) = mid;
        *reinterpret_cast<bf16x4*>(d + 2 * plane_stride) = lo;
      }
    }
  };
  auto stash = [&](int tile) {
    int i0, y0, x0;
    origin(tile, i0, y0, x0);
#pragma unroll
    for (int it = 0; it < YIT; ++it) {
      const int yk = stage_chunk<AB>(tid + it * 256, 8);
      if (yk < YCH) {
        const f32x4 v[4] = {act_f4(yv[it][0]), act_f4(yv[it][1]), act_f4(yv[it][2]), act_f4(yv[it][3])};
        put4(ys + yk * 4, DYP, TPX, v);
      }
    }
#pragma unroll
    for (int it = 0; it < XIT; ++it) {
      const int g = stage_chunk<AB>(tid + it * 256, 8);
      if (g < XCH) {
        const int row = g / NCG, cg = g % NCG;
        const int mi = row / PH, iy = y0 - 1 + row % PH;
        f32x4 v[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          v[e] = act_f4(xv[it][e]);
          const int ix = x0 - 1 + cg * 4 + e;
          // zero padding stays zero: padded taps read 0 in the reference's zero-padded relu(bn(y))
          if (p.scale && i0 + mi < p.NF && iy >= 0 && iy < p.IH && ix >= 0 && ix < p.IW && cg * 4 + e < PW) {
#pragma unroll
            for (int cc = 0; cc < 4; ++cc) v[e][cc] = relu_nan(fmaf(v[e][cc], sc[cc], sh[cc]));
          }
        }
        put4(xs + row * PWP + cg * 4, CIP, PLANE, v);
      }
    }
  };

  f32x16 acc[9];
#pragma unroll
  for (int t = 0; t < 9; ++t)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[t][r] = 0.f;

  int tile = blockIdx.z;
  if (PF && tile < p.ntiles) fetch(tile);
  for (; tile < p.ntiles; tile += gridDim.z) {
    if (!PF) fetch(tile);  // (no register prefetch: the co-resident block hides the load latency)
    __syncthreads();  // the previous tile's fragment reads are done
    stash(tile);
    __syncthreads();
    if (PF && tile + (int)gridDim.z < p.ntiles) fetch(tile + gridDim.z);
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      const int lin = (wave * KS + ks) * 16 + 8 * h;
      const int mi = lin / (TH * TW), mr = lin % (TH * TW);
      const int oy = mr / TW, ox = mr % TW;
      bf16x8 a[NP];
#pragma unroll
      for (int q = 0; q < NP; ++q) a[q] = *reinterpret_cast<const bf16x8*>(ys + j * DYP + q * TPX + lin);
#pragma unroll
      for (int kh = 0; kh < 3; ++kh) {
        const __bf16* xb = xs + j * CIP + (mi * PH + oy + kh) * PWP + ox;
        // B planes smallest first: lo (x a.hi), mid (x a.mid, a.hi), hi (x a.lo, a.mid, a.hi)
#pragma unroll
        for (int q = NP - 1; q >= 0; --q) {
          const u32x4 d0 = *reinterpret_cast<const u32x4*>(xb + q * PLANE);
          const u32x4 d1 = *reinterpret_cast<const u32x4*>(xb + q * PLANE + 8);
          const u32x4 s1 = {__builtin_amdgcn_alignbyte(d0[1], d0[0], 2), __builtin_amdgcn_alignbyte(d0[2], d0[1], 2),
                            __builtin_amdgcn_alignbyte(d0[3], d0[2], 2), __builtin_amdgcn_alignbyte(d1[0], d0[3], 2)};
          const u32x4 s2 = {d0[1], d0[2], d0[3], d1[0]};
          const bf16x8 b0 = __builtin_bit_cast(bf16x8, d0);
          const bf16x8 b1 = __builtin_bit_cast(bf16x8, s1);
          const bf16x8 b2 = __builtin_bit_cast(bf16x8, s2);
#pragma unroll
          for (int qa = NP - 1 - q; qa >= 0; --qa) {
            acc[kh * 3 + 0] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[qa], b0, acc[kh * 3 + 0], 0, 0, 0);
            acc[kh * 3 + 1] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[qa], b1, acc[kh * 3 + 1], 0, 0, 0);
            acc[kh * 3 + 2] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[qa], b2, acc[kh * 3 + 2], 0, 0, 0);
          }
        }
      }
    }
  }

  wgrad_combine_store(acc, sm, p.slab + (int64_t)blockIdx.z * p.Co * 9 * p.Ci, co0, ci0, p.Ci);
}

// fixed-order combine of the 4 waves' tap accumulators, 3 taps at a time: (2,3) -> (0,1), then 1 -> 0; wave 0
// writes the block's [32 co][9 taps][32 ci] sum into its slab (LDS: 2*3*16*64 floats)
__device__ __forceinline__ void wgrad_combine_store(f32x16 (&acc)[9], __bf16* sm, float* out, int co0, int ci0,
                                                    int Ci) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int h = lane >> 5, j = lane & 31;
  float* red = reinterpret_cast<float*>(sm);
#pragma unroll
  for (int tc = 0; tc < 3; ++tc) {
    __syncthreads();
    if (wave >= 2) {
#pragma unroll
      for (int u = 0; u < 3; ++u)
#pragma unroll
        for (int r = 0; r < 16; ++r) red[(((wave - 2) * 3 + u) * 16 + r) * 64 + lane] = acc[tc * 3 + u][r];
    }
    __syncthreads();
    if (wave < 2) {
#pragma unroll
      for (int u = 0; u < 3; ++u)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[tc * 3 + u][r] += red[((wave * 3 + u) * 16 + r) * 64 + lane];
    }
    __syncthreads();
    if (wave == 1) {
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
          const int co = co0 + (r & 3) + 8 * (r >> 2) + 4 * h, t = tc * 3 + u;
          out[(int64_t)co * 9 * Ci + t * Ci + ci0 + j] = acc[t][r] + red[(u * 16 + r) * 64 + lane];
        }
    }
  }
}

// Multi-co-tile weight gradient (same GEMM view: M = co, N = ci, K = output pixels) for the layers whose staged
// patch is large against the tile's MFMA work: stride 2 (the patch is ~4x the tile's pixel count) and 8x8 frames
// (the halo is 56% of the tile).  The block amortises one patch over 32*NT output channels (NT = 2 or 4) of a
// TPX-pixel tile: wave w owns co tile w % NT and KSW = TPX/16*NT/4 consecutive K steps; the 4/NT waves of a co tile
// are summed in a fixed order at the end (none for NT = 4).
// Stride 1: patch rows of TW+8 columns, the kw shifts are a 2-byte v_alignbyte (kw = 1) and a dword shift (kw = 2)
// of two aligned reads.  Stride 2: output pixel ox reads input columns 2ox-1+kw, so each patch row (2TH+1 rows x
// 2TW+1 columns incl. halo) is stored parity-split as [E: even patch columns, TW+8 slots][O: odd ones, TW slots];
// the 8 consecutive output pixels of a lane half need E[ox..ox+7] (kw = 0), O[ox..ox+7] (kw = 1) and E[ox+1..ox+8]
// (kw = 2, the 2-byte shift): every fragment is an aligned b128 read per plane, no strided LDS access.
template <int S, int TH, int TW, int NT, int NP, bool AB = false>
__global__ __launch_bounds__(256, 2) void conv3x3_wgrad_x3nt_kernel(const WgX3Args p) {
  static_assert(!AB || NP == 1, "bf16 storage with bf16 operands only");
  using TA = act_t<AB>;
  using R4 = act_raw4<AB>;
  const TA* dYp = reinterpret_cast<const TA*>(p.dY);
  const TA* srcp = reinterpret_cast<const TA*>(p.src);
  constexpr int TPX = TH * TW, NC = 32 * NT, KT = TPX / 16, KSW = KT * NT / 4;
  static_assert((TPX == 32 || TPX == 64) && TW % 8 == 0 && (NT == 2 || NT == 4) && (S == 1 || S == 2),
                "whole K steps per wave, 8-pixel row runs");
  constexpr int PH = S * (TH - 1) + 3, PW = S * (TW - 1) + 3, EW = TW + 8, PWP = S == 1 ? TW + 8 : EW + TW;
  constexpr int NCG = PWP / 4;
  constexpr int PLANE = PH * PWP, CIP = odd16_pitch(NP * PLANE), DYP = odd16_pitch(NP * TPX);
  constexpr int XE = 32 * CIP, YE = NC * DYP, RE = 2 * 3 * 16 * 64 * 2;
  __shared__ __attribute__((aligned(16))) __bf16 sm[(XE + YE) > RE ? (XE + YE) : RE];
  __bf16* xs = sm;
  __bf16* ys = sm + XE;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int h = lane >> 5, j = lane & 31;
  const int co0 = blockIdx.x * NC, ci0 = blockIdx.y * 32;
  const int c4 = stage_group<AB>(tid, 8);  // patch staging: this thread's 4-channel group of the 32 ci
  // dY staging: 4 pixels x 4 co per item (stage_group / stage_chunk over YG co groups)
  constexpr int YG = NC / 4, YCH = TPX / 4, YQ = (YCH + 7) / 8 * 8 * YG, YIT = (YQ + 255) / 256;
  static_assert(YG % 2 == 0 && 16 % (YG / 2) == 0 && (YQ <= 256 || YQ % 256 == 0), "whole dY staging passes");
  const int yc = stage_group<AB>(tid, YG);

  constexpr int XCH = PH * NCG, XQ = (XCH + 7) / 8 * 64, XIT = (XQ + 255) / 256;
  static_assert(XIT <= 2, "patch staged in one register pass");
  R4 xv[XIT][4], yv[YIT][4];
  // patch column (0 = input column S*x0 - 1) held by LDS column c of a row
  auto pcol = [](int c) { return S == 1 ? c : (c < EW ? 2 * c : 2 * (c - EW) + 1); };
  auto origin = [&](int tile, int& img, int& y0, int& x0) {
    const int tpi = p.tiles_h * p.tiles_w, tr = tile % tpi;
    img = tile / tpi;
    y0 = (tr / p.tiles_w) * TH;
    x0 = (tr % p.tiles_w) * TW;
  };
  auto fetch = [&](int tile) {
    int img, y0, x0;
    origin(tile, img, y0, x0);
#pragma unroll
    for (int it = 0; it < YIT; ++it) {
      const int yk = stage_chunk<AB>(tid + it * 256, YG), yp = yk * 4, oy = y0 + yp / TW, ox = x0 + yp % TW;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        yv[it][e] = R4{};
        if (yk < YCH && tid + it * 256 < YQ && oy < p.OH && ox + e < p.OW)
          yv[it][e] = act_ld4(dYp + (((int64_t)img * p.OH + oy) * p.OW + ox + e) * p.Co + co0 + yc * 4);
      }
    }
#pragma unroll
    for (int it = 0; it < XIT; ++it) {
      const int g = stage_chunk<AB>(tid + it * 256, 8);
      const int row = g / NCG, cg = g % NCG, iy = S * y0 - 1 + row;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int pc = pcol(cg * 4 + e), ix = S * x0 - 1 + pc;
        xv[it][e] = R4{};
        if (g < XCH && pc < PW && iy >= 0 && iy < p.IH && ix >= 0 && ix < p.IW)
          xv[it][e] = act_ld4(srcp + (((int64_t)img * p.IH + iy) * p.IW + ix) * p.Ci + ci0 + c4 * 4);
      }
    }
  };
  f32x4 sc = {1.f, 1.f, 1.f, 1.f}, sh = {0.f, 0.f, 0.f, 0.f};
  if (p.scale) {
    sc = *reinterpret_cast<const f32x4*>(p.scale + ci0 + c4 * 4);
    sh = *reinterpret_cast<const f32x4*>(p.shift + ci0 + c4 * 4);
  }
  // 4 channels (rows ch0..ch0+3 of pitch `pitch`) x 4 consecutive columns -> per channel and plane one 8-B store
  auto put4 = [&](__bf16* dst, int pitch, int plane_stride, const f32x4* v) {
#pragma unroll
    for (int cc = 0; cc < 4; ++cc) {
      typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
      bf16x4 hi, mid, lo;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float x = v[e][cc];
        const __bf16 a = (__bf16)x;
        if (NP == 1) {
          hi[e] = mid[e] = lo[e] = a;
          continue;
        }
        const float r = x - (float)a;
        const __bf16 b = (__bf16)r;
        hi[e] = a;
        mid[e] = b;
        lo[e] = (__bf16)(r - (float)b);
      }
      __bf16* d = dst + cc * pitch;
      *reinterpret_cast<bf16x4*>(d) = hi;
      if constexpr (NP == 3) {
        *reinterpret_cast<bf16x4*>(d + plane_stride) = mid;
        *reinterpret_cast<bf16x4*>(d + 2 * plane_stride) = lo;
      }
    }
  };
  auto stash = [&](int tile) {
    int img, y0, x0;
    origin(tile, img, y0, x0);
#pragma unroll
    for (int it = 0; it < YIT; ++it)
      if (stage_chunk<AB>(tid + it * 256, YG) < YCH && tid + it * 256 < YQ) {
        const f32x4 v[4] = {act_f4(yv[it][0]), act_f4(yv[it][1]), act_f4(yv[it][2]), act_f4(yv[it][3])};
        put4(ys + yc * 4 * DYP + stage_chunk<AB>(tid + it * 256, YG) * 4, DYP, TPX, v);
      }
#pragma unroll
    for (int it = 0; it < XIT; ++it) {
      const int g = stage_chunk<AB>(tid + it * 256, 8);
      if (g < XCH) {
        const int row = g / NCG, cg = g % NCG, iy = S * y0 - 1 + row;
        f32x4 v[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          v[e] = act_f4(xv[it][e]);
          const int pc = pcol(cg * 4 + e), ix = S * x0 - 1 + pc;
          // zero padding stays zero (the reference pads relu(bn(y)) with zeros)
          if (p.scale && iy >= 0 && iy < p.IH && ix >= 0 && ix < p.IW && pc < PW) {
#pragma unroll
            for (int cc = 0; cc < 4; ++cc) v[e][cc] = relu_nan(fmaf(v[e][cc], sc[cc], sh[cc]));
          }
        }
        put4(xs + c4 * 4 * CIP + row * PWP + cg * 4, CIP, PLANE, v);
      }
    }
  };

  f32x16 acc[9];
#pragma unroll
  for (int t = 0; t < 9; ++t)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[t][r] = 0.f;

  const int ct = wave % NT, ks0 = (wave / NT) * KSW;  // this wave's co tile and first K step
  for (int tile = blockIdx.z; tile < p.ntiles; tile += gridDim.z) {
    fetch(tile);
    __syncthreads();  // the previous tile's fragment reads are done
    stash(tile);
    __syncthreads();
#pragma unroll
    for (int k = 0; k < KSW; ++k) {
      const int lin = (ks0 + k) * 16 + 8 * h, oyr = lin / TW, oxr = lin % TW;
      bf16x8 a[NP];
#pragma unroll
      for (int q = 0; q < NP; ++q) a[q] = *reinterpret_cast<const bf16x8*>(ys + (ct * 32 + j) * DYP + q * TPX + lin);
#pragma unroll
      for (int kh = 0; kh < 3; ++kh) {
        const __bf16* xb = xs + j * CIP + (S * oyr + kh) * PWP + oxr;
#pragma unroll
        for (int q = NP - 1; q >= 0; --q) {
          const u32x4 d0 = *reinterpret_cast<const u32x4*>(xb + q * PLANE);
          const u32x4 d1 = *reinterpret_cast<const u32x4*>(xb + q * PLANE + 8);
          const u32x4 s1 = {__builtin_amdgcn_alignbyte(d0[1], d0[0], 2), __builtin_amdgcn_alignbyte(d0[2], d0[1], 2),
                            __builtin_amdgcn_alignbyte(d0[3], d0[2], 2), __builtin_amdgcn_alignbyte(d1[0], d0[3], 2)};
          bf16x8 b0 = __builtin_bit_cast(bf16x8, d0), b1, b2;
          if constexpr (S == 1) {
            const u32x4 s2 = {d0[1], d0[2], d0[3], d1[0]};
            b1 = __builtin_bit_cast(bf16x8, s1);
            b2 = __builtin_bit_cast(bf16x8, s2);
          } else {
            b1 = __builtin_bit_cast(bf16x8, *reinterpret_cast<const u32x4*>(xb + q * PLANE + EW));
            b2 = __builtin_bit_cast(bf16x8, s1);
          }
#pragma unroll
          for (int qa = NP - 1 - q; qa >= 0; --qa) {
            acc[kh * 3 + 0] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[qa], b0, acc[kh * 3 + 0], 0, 0, 0);
            acc[kh * 3 + 1] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[qa], b1, acc[kh * 3 + 1], 0, 0, 0);
            acc[kh * 3 + 2] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[qa], b2, acc[kh * 3 + 2], 0, 0, 0);
          }
        }
      }
    }
  }

  float* out = p.slab + (int64_t)blockIdx.z * p.Co * 9 * p.Ci;
  const int cob = co0 + ct * 32;
  if constexpr (NT == 2) {
    // waves w and w + 2 hold the two K steps of co tile w: (w) + (w + 2), 3 taps at a time
    float* red = reinterpret_cast<float*>(sm);
#pragma unroll
    for (int tc = 0; tc < 3; ++tc) {
      __syncthreads();
      if (wave >= 2) {
#pragma unroll
        for (int u = 0; u < 3; ++u)
#pragma unroll
          for (int r = 0; r < 16; ++r) red[(((wave - 2) * 3 + u) * 16 + r) * 64 + lane] = acc[tc * 3 + u][r];
      }
      __syncthreads();
      if (wave < 2) {
#pragma unroll
        for (int u = 0; u < 3; ++u)
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int co = cob + (r & 3) + 8 * (r >> 2) + 4 * h, t = tc * 3 + u;
            out[(int64_t)co * 9 * p.Ci + t * p.Ci + ci0 + j] = acc[t][r] + red[((wave * 3 + u) * 16 + r) * 64 + lane];
          }
      }
    }
  } else {
#pragma unroll
    for (int t = 0; t < 9; ++t)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int co = cob + (r & 3) + 8 * (r >> 2) + 4 * h;
        out[(int64_t)co * 9 * p.Ci + t * p.Ci + ci0 + j] = acc[t][r];
      }
  }
}

template <int NI, int TH, int TW, bool PF = false>
static int launch_wgrad_x3(WgX3Args a, int target_blocks, int64_t partial_cap, hipStream_t st, int* nsplit) {
  a.tiles_h = (int)cdiv(a.OH, TH);
  a.tiles_w = (int)cdiv(a.OW, TW);
  a.ntiles = (int)(cdiv(a.NF, NI) * a.tiles_h * a.tiles_w);
  const int pairs = (a.Co / 32) * (a.Ci / 32);
  int64_t z = std::max<int64_t>(1, std::min<int64_t>(cdiv(target_blocks, pairs), a.ntiles));
  z = std::min<int64_t>(z, std::max<int64_t>(1, partial_cap / ((int64_t)a.Co * 9 * a.Ci)));
  dim3 grid((unsigned)(a.Co / 32), (unsigned)(a.Ci / 32), (unsigned)z);
  VAD_CHECK(!g_act_bf16 || g_conv_bf16, "conv3_wgrad_x3: bf16 activations need conv_bf16");
  if (g_conv_bf16 && g_act_bf16) VAD_KLAUNCH((conv3x3_wgrad_x3_kernel<NI, TH, TW, PF, 1, true>), grid, dim3(256), 0, st, a);
  else if (g_conv_bf16) VAD_KLAUNCH((conv3x3_wgrad_x3_kernel<NI, TH, TW, PF, 1>), grid, dim3(256), 0, st, a);
  else VAD_KLAUNCH((conv3x3_wgrad_x3_kernel<NI, TH, TW, PF, 3>), grid, dim3(256), 0, st, a);
  VAD_LAUNCH_CHECK();
  *nsplit = (int)z;
  return 0;
}

template <int S, int TH, int TW, int NT>
static int launch_wgrad_x3nt(WgX3Args a, int target_blocks, int64_t partial_cap, hipStream_t st, int* nsplit) {
  a.tiles_h = (int)cdiv(a.OH, TH);
  a.tiles_w = (int)cdiv(a.OW, TW);
  a.ntiles = (int)((int64_t)a.NF * a.tiles_h * a.tiles_w);
  const int pairs = (a.Co / (32 * NT)) * (a.Ci / 32);
  int64_t z = std::max<int64_t>(1, std::min<int64_t>(cdiv(target_blocks, pairs), a.ntiles));
  z = std::min<int64_t>(z, std::max<int64_t>(1, partial_cap / ((int64_t)a.Co * 9 * a.Ci)));
  dim3 grid((unsigned)(a.Co / (32 * NT)), (unsigned)(a.Ci / 32), (unsigned)z);
  VAD_CHECK(!g_act_bf16 || g_conv_bf16, "conv3_wgrad_x3: bf16 activations need conv_bf16");
  if (g_conv_bf16 && g_act_bf16) VAD_KLAUNCH((conv3x3_wgrad_x3nt_kernel<S, TH, TW, NT, 1, true>), grid, dim3(256), 0, st, a);
  else if (g_conv_bf16) VAD_KLAUNCH((conv3x3_wgrad_x3nt_kernel<S, TH, TW, NT, 1>), grid, dim3(256), 0, st, a);
  else VAD_KLAUNCH((conv3x3_wgrad_x3nt_kernel<S, TH, TW, NT, 3>), grid, dim3(256), 0, st, a);
  VAD_LAUNCH_CHECK();
  *nsplit = (int)z;
  return 0;
}

template <int S, int TH, int TW>
static int launch_wgrad_x3nt_co(WgX3Args a, int nt, int target_blocks, int64_t partial_cap, hipStream_t st,
                                int* nsplit) {
  if (nt == 4 && a.Co % 128 == 0) return launch_wgrad_x3nt<S, TH, TW, 4>(a, target_blocks, partial_cap, st, nsplit);
  return launch_wgrad_x3nt<S, TH, TW, 2>(a, target_blocks, partial_cap, st, nsplit);
}

int g_wgrad_split = 1;     // tuning knob "conv_wgrad_split": stride-1 weight gradients on the split-bf16 kernel
int g_wgrad_split_s2 = 1;  // tuning knob "conv_wgrad_split_s2": stride-2 weight gradients on the split-bf16 kernel
int g_wgrad_s2_blocks = 384;  // tuning knob "conv_wgrad_s2_blocks": their target grid size (sweep: profiles/r02_wgrad_grid_sweep.json)
int g_wgrad_s1_nt = 2;  // tuning knob "conv_wgrad_s1_nt": stride-1 frames <= 16 wide on the multi-co-tile kernel (2|4)
int g_wgrad_s1_nt_wide = 0;  // knob "conv_wgrad_s1_nt_wide": wider stride-1 frames too (2x32 tiles)
int g_wgrad_s1_nt_blocks = 384;  // knob "conv_wgrad_s1_nt_blocks"

bool conv3_wgrad_x3_supported(const Conv3Layer& L) {
  if (!g_conv_split || L.Ci % 32 != 0 || L.Co % 32 != 0) return false;
  if (L.stride == 2) return g_wgrad_split_s2 != 0 && L.Co % 64 == 0;
  // (8x8 frames: 64-pixel tiles carry too little MFMA work per staged patch; the f32 patch kernel is faster there)
  return L.stride == 1 && g_wgrad_split &&
         (L.OH > 8 || L.OW > 8 || g_wgrad_split == 2 || g_conv_bf16 || (g_wgrad_s1_nt && L.Co % 64 == 0));
}

int conv3_wgrad_x3(const Conv3Layer& L, const float* dY, const float* src, const float* src_stats, float* slab,
                   int* nsplit, int64_t partial_cap, int target_blocks, hipStream_t st) {
  VAD_CHECK(conv3_wgrad_x3_supported(L), "conv3_wgrad_x3: Ci and Co multiples of 32");
  VAD_CHECK(partial_cap >= (int64_t)L.Co * 9 * L.Ci, "conv3_wgrad_x3: slab capacity below one split");
  WgX3Args a{};
  a.dY = dY;
  a.src = src;
  a.scale = src_stats ? src_stats + 2 * L.Ci : nullptr;
  a.shift = src_stats ? src_stats + 3 * L.Ci : nullptr;
  a.slab = slab;
  a.NF = L.NF; a.IH = L.IH; a.IW = L.IW; a.Ci = L.Ci; a.OH = L.OH; a.OW = L.OW; a.Co = L.Co;
  if (L.stride == 2) {
    VAD_CHECK(L.IH >= 2 * L.OH - 1 && L.IW >= 2 * L.OW - 1, "conv3_wgrad_x3: stride-2 geometry");
    target_blocks = g_wgrad_s2_blocks;
    if (L.OW > 16) return launch_wgrad_x3nt_co<2, 1, 32>(a, 4, target_blocks, partial_cap, st, nsplit);
    if (L.OW > 8) return launch_wgrad_x3nt_co<2, 2, 16>(a, 4, target_blocks, partial_cap, st, nsplit);
    return launch_wgrad_x3nt_co<2, 4, 8>(a, 4, target_blocks, partial_cap, st, nsplit);
  }
  if (g_wgrad_s1_nt && L.Co % 64 == 0 && (L.OW <= 16 || g_wgrad_s1_nt_wide)) {
    if (L.OW > 16) return launch_wgrad_x3nt_co<1, 2, 32>(a, g_wgrad_s1_nt, g_wgrad_s1_nt_blocks, partial_cap, st, nsplit);
    if (L.OW <= 8 && L.OH <= 8)
      return launch_wgrad_x3nt_co<1, 8, 8>(a, g_wgrad_s1_nt, g_wgrad_s1_nt_blocks, partial_cap, st, nsplit);
    return launch_wgrad_x3nt_co<1, 4, 16>(a, g_wgrad_s1_nt, g_wgrad_s1_nt_blocks, partial_cap, st, nsplit);
  }
  if (L.OH <= 8 && L.OW <= 8) return launch_wgrad_x3<1, 8, 8>(a, target_blocks, partial_cap, st, nsplit);
  if (L.OW <= 16) return launch_wgrad_x3<1, 8, 16>(a, target_blocks, partial_cap, st, nsplit);
  return launch_wgrad_x3<1, 4, 32>(a, target_blocks, partial_cap, st, nsplit);
}

}  // namespace vad
