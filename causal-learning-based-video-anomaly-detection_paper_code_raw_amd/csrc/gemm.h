// Generic f32 MFMA GEMM for gfx950:  C[m][n] = sum_k A(m,k) * B(n,k)   (exact f32, v_mfma_f32_32x32x2_f32)
//
// Block = 256 threads = 4 waves arranged WM x WN; each wave owns TM x TN 32x32 accumulator tiles.
// K is walked in BK=32 slices, register-prefetched one slice ahead into a double-buffered LDS tile.
//
// Every operand comes from a Loader policy that fills one of two LDS images:
//   * K-contiguous (KC): lds[row][k], rows padded to 36 floats.  A lane reads 4 consecutive k with one
//     ds_read_b128 and feeds 4 MFMAs; the k order inside an 8-wide sub-step is permuted so that lane
//     half h supplies k = 8*kk + 4*h + s at MFMA s (both operands use the same map, so the sum is exact).
//     The +4 float pad makes the 16-lane ds_read_b128 groups conflict-free (slot = 9*row mod 16).
//   * K-major (KM): lds[k][row] (row contiguous); a lane reads one float (ds_read_b32) per MFMA.
// Loaders: dense row-major KC/KM matrices, the NHWC conv patch gather (implicit GEMM with a tap table and
// optional BN+ReLU applied on load), and the K-major patch gather used by the conv weight gradient.
#pragma once
#include <type_traits>

#include "common.h"

namespace vad {

constexpr int BK = 32;
constexpr int KC_STRIDE = BK + 4;

template <int WM_, int WN_, int TM_, int TN_>
struct TileCfg {
  static constexpr int WM = WM_, WN = WN_, TM = TM_, TN = TN_;
  static constexpr int BM = WM * TM * 32;
  static constexpr int BN = WN * TN * 32;
  static_assert(WM * WN == 4, "block is 4 waves");
};

template <bool KC, int R>
struct LdsSize {
  static constexpr int floats = KC ? R * KC_STRIDE : BK * R;
};

// ------------------------------------------------------------------ fragment reads
template <int R>
__device__ inline void frag_kc(const float* __restrict__ lds, int row, int kbase, float (&v)[4]) {
  const f32x4 t = *reinterpret_cast<const f32x4*>(lds + row * KC_STRIDE + kbase);
  v[0] = t[0]; v[1] = t[1]; v[2] = t[2]; v[3] = t[3];
}
template <int R>
__device__ inline void frag_km(const float* __restrict__ lds, int row, int kbase, float (&v)[4]) {
#pragma unroll
  for (int s = 0; s < 4; ++s) v[s] = lds[(kbase + s) * R + row];
}

// ------------------------------------------------------------------ gather helpers
// The conv gathers load through buffer resources with 32-bit offsets (the host checks every gathered tensor is below
// 2^31 bytes, gather_fits): an element outside the source image takes an offset past the buffer's end and loads
// zeros, so a K slice issues the same loads on every lane with no branches (the counted waits never drain the
// prefetch) and no 64-bit address arithmetic.
constexpr int GATHER_OOB = 0x7ffffff0;
inline bool gather_fits(int64_t numel) { return numel >= 0 && numel * 4 < 0x7ffffff0ll; }
__device__ inline __amdgpu_buffer_rsrc_t gather_rsrc(const float* p, int64_t numel) {
  return __builtin_amdgcn_make_buffer_rsrc((void*)p, (short)0, (int)(numel * 4 < 0x7ffffff0ll ? numel * 4 : 0x7ffffff0ll),
                                           0x00020000);
}
__device__ inline f32x4 gather_load(__amdgpu_buffer_rsrc_t r, bool ok, int elem) {
  return __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(r, ok ? elem * 4 : GATHER_OOB, 0, 0));
}
// loaders that keep a per-block table in LDS declare TAB (ints); gemm_kernel allocates it and passes it to init
template <class L, class = void>
struct LoaderTab {
  static constexpr int n = 0;
};
template <class L>
struct LoaderTab<L, std::void_t<decltype(L::TAB)>> {
  static constexpr int n = L::TAB;
};

// ------------------------------------------------------------------ dense loaders
// Row-major matrix X[rows][ld] read as operand rows=r, k=c (K-contiguous).  Below 2^31 bytes the loads go through a
// buffer resource (out-of-range elements at an offset past its end: zeros, no branches), one 16-B load per float4 when
// ld and kdim are multiples of 4, else four 4-B loads; larger matrices take plain guarded loads.
template <int R>
struct DenseKC {
  static constexpr bool KC = true;
  static constexpr int NL = R / 32;  // float4 per thread per tile
  struct Params { const float* p; int64_t ld; int rows; int kdim; };
  const float* base; int64_t ld; int rows, kdim; int r0;
  bool buf, vec;
  __amdgpu_buffer_rsrc_t rs;
  f32x4 reg[NL];
  __device__ void init(const Params& P, int r0_, int tid_) {
    base = P.p; ld = P.ld; rows = P.rows; kdim = P.kdim; r0 = r0_;
    const int64_t numel = (int64_t)rows * ld;
    buf = numel * 4 < 0x7ffffff0ll;
    vec = ((ld | kdim) & 3) == 0;
    rs = gather_rsrc(base, numel);
  }
  __device__ void load(int k0) {
    const int tid = threadIdx.x;
#pragma unroll
    for (int j = 0; j < NL; ++j) {
      const int row = tid / 8 + 32 * j, kq = tid % 8;
      const int r = r0 + row, k = k0 + kq * 4;
      if (buf && vec) {
        reg[j] = gather_load(rs, r < rows && k < kdim, r * (int)ld + k);
      } else if (buf) {
#pragma unroll
        for (int e = 0; e < 4; ++e)
          reg[j][e] = __builtin_bit_cast(
              float, __builtin_amdgcn_raw_buffer_load_b32(rs, (r < rows && k + e < kdim) ? (r * (int)ld + k + e) * 4
                                                                                        : GATHER_OOB, 0, 0));
      } else {
        f32x4 v = {0.f, 0.f, 0.f, 0.f};
        if (r < rows && k < kdim) {
          const float* src = base + (int64_t)r * ld + k;
          if (k + 3 < kdim && ((ld & 3) == 0)) v = *reinterpret_cast<const f32x4*>(src);
          else {
#pragma unroll
            for (int e = 0; e < 4; ++e) v[e] = (k + e < kdim) ? src[e] : 0.f;
          }
        }
        reg[j] = v;
      }
    }
  }
  __device__ void store(float* lds) const {
    const int tid = threadIdx.x;
#pragma unroll
    for (int j = 0; j < NL; ++j) {
      const int row = tid / 8 + 32 * j, kq = tid % 8;
      *reinterpret_cast<f32x4*>(lds + row * KC_STRIDE + kq * 4) = reg[j];
    }
  }
};

// Row-major matrix X[kdim][ld] read as operand k=row of X, r=column of X (K-major), below 2^31 bytes (host:
// gather_fits).  Loads go through a buffer resource with out-of-range elements at an offset past its end (zeros, no
// branches): one 16-B load per float4 when ld and rows are multiples of 4, else four 4-B loads.  Optional virtual
// "ones" column at r == ones_col (used to fold bias grads into weight-grad GEMMs), set at store time so the prefetch
// is never waited for at load time.
template <int R>
struct DenseKM {
  static constexpr bool KC = false;
  static constexpr int NL = R / 32;
  struct Params { const float* p; int64_t ld; int rows; int kdim; int ones_col; };
  int ld, rows, kdim, ones_col, r0, tid, k0s;
  bool vec;
  __amdgpu_buffer_rsrc_t rs;
  f32x4 reg[NL];
  __device__ void init(const Params& P, int r0_, int tid_) {
    ld = (int)P.ld; rows = P.rows; kdim = P.kdim; ones_col = P.ones_col; r0 = r0_; tid = tid_;
    vec = ((ld | rows) & 3) == 0;
    rs = gather_rsrc(P.p, (int64_t)kdim * P.ld);
  }
  __device__ void load(int k0) {
    k0s = k0;
#pragma unroll
    for (int j = 0; j < NL; ++j) {
      const int q = tid + 256 * j;
      const int kr = q / (R / 4), rq = q % (R / 4);
      const int k = k0 + kr, r = r0 + rq * 4;
      if (vec) {
        reg[j] = gather_load(rs, k < kdim && r < rows, k * ld + r);
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e)
          reg[j][e] = __builtin_bit_cast(
              float, __builtin_amdgcn_raw_buffer_load_b32(rs, (k < kdim && r + e < rows) ? (k * ld + r + e) * 4
                                                                                          : GATHER_OOB, 0, 0));
      }
    }
  }
  __device__ void store(float* lds) const {
#pragma unroll
    for (int j = 0; j < NL; ++j) {
      const int q = tid + 256 * j;
      const int kr = q / (R / 4), rq = q % (R / 4);
      const int k = k0s + kr, r = r0 + rq * 4;
      f32x4 v = reg[j];
#pragma unroll
      for (int e = 0; e < 4; ++e)
        if (k < kdim && r + e == ones_col) v[e] = 1.f;
      *reinterpret_cast<f32x4*>(lds + kr * R + rq * 4) = v;
    }
  }
};

// ------------------------------------------------------------------ conv gathers
// Tap table: for tap t, src pixel = (a*sa + dh[t], b*sb + dw[t]) where (a,b) is the GEMM row's position in
// its destination grid.  Covers forward conv (dh = kh - pad), stride-1 transposed conv (dh = pad - kh) and
// each stride-2 parity class of the transposed conv.
struct TapTable {
  int ntaps;
  int8_t dh[16], dw[16];  // (16: the 4x4 convs of cad1's autoencoder)
};

struct ConvGeom {
  int imgs;          // frames
  int GA, GB;        // destination grid (rows of the GEMM = imgs*GA*GB)
  int sa, sb;        // src step per grid step
  int SH, SW, C;     // src spatial dims / channels (C % 32 == 0)
};

// A operand of forward / data-grad conv: row m = (img, a, b), k = tap*C + c; value = act(src[img][sh][sw][c]).
// C % 32 == 0, so a K slice lies in one tap (uniform: its offsets are scalar).
template <int R>
struct ConvGatherKC {
  static constexpr bool KC = true;
  static constexpr int NL = R / 32;
  struct Params {
    const float* src; ConvGeom g; TapTable taps;
    const float* scale; const float* shift;  // BN+ReLU applied on load when scale != nullptr
  };
  const Params* P;
  __amdgpu_buffer_rsrc_t rs;
  int cq;
  int rowoff[NL];        // element offset of the row's pixel (a*sa, b*sb) in its image
  int ya[NL], xb[NL];    // a*sa, b*sb  (ya < 0 marks an out-of-range row)
  f32x4 reg[NL];
  __device__ void init(const Params& Pp, int r0, int tid) {
    P = &Pp;
    cq = (tid % 8) * 4;
    const ConvGeom& g = Pp.g;
    rs = gather_rsrc(Pp.src, (int64_t)g.imgs * g.SH * g.SW * g.C);
    const int M = g.imgs * g.GA * g.GB;
#pragma unroll
    for (int j = 0; j < NL; ++j) {
      const int m = r0 + tid / 8 + 32 * j;
      if (m < M) {
        const int img = m / (g.GA * g.GB);
        const int rem = m - img * g.GA * g.GB;
        const int a = rem / g.GB, b = rem - a * g.GB;
        ya[j] = a * g.sa;
        xb[j] = b * g.sb;
        rowoff[j] = ((img * g.SH + ya[j]) * g.SW + xb[j]) * g.C;
      } else {
        rowoff[j] = 0; ya[j] = -100000; xb[j] = 0;
      }
    }
  }
  __device__ void load(int k0) {
    const ConvGeom& g = P->g;
    const int C = g.C;
    const int tap = k0 / C;
    const int c = k0 - tap * C + cq;
    const int dh = P->taps.dh[tap], dw = P->taps.dw[tap];
    const int toff = (dh * g.SW + dw) * C + c;
    f32x4 sc = {1.f, 1.f, 1.f, 1.f}, sh = {0.f, 0.f, 0.f, 0.f};
    const bool bn = P->scale != nullptr;
    if (bn) {
      sc = *reinterpret_cast<const f32x4*>(P->scale + c);
      sh = *reinterpret_cast<const f32x4*>(P->shift + c);
    }
#pragma unroll
    for (int j = 0; j < NL; ++j) {
      const bool ok = (unsigned)(ya[j] + dh) < (unsigned)g.SH && (unsigned)(xb[j] + dw) < (unsigned)g.SW;
      f32x4 v = gather_load(rs, ok, rowoff[j] + toff);
      if (bn) {
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = ok ? fmaxf(fmaf(v[e], sc[e], sh[e]), 0.f) : 0.f;
      }
      reg[j] = v;
    }
  }
  __device__ void store(float* lds) const {
    const int tid = threadIdx.x;
#pragma unroll
    for (int j = 0; j < NL; ++j) {
      const int row = tid / 8 + 32 * j, kq = tid % 8;
      *reinterpret_cast<f32x4*>(lds + row * KC_STRIDE + kq * 4) = reg[j];
    }
  }
};

// B operand of the conv weight gradient (K-major over output pixels):
//   k = output pixel p = (img, oh, ow) of the forward conv, r = tap*C + c,
//   value = act(src[img][oh*s - pad + kh][ow*s - pad + kw][c]).
// A thread's rows r (hence tap, c) are fixed and its pixels advance by BK per K slice: both are decomposed once
// (init / the first load of a split) and the pixel coordinates then stepped, not divided, per slice.
template <int R>
struct ConvPatchKM {
  static constexpr bool KC = false;
  static constexpr int NL = R / 32;
  struct Params {
    const float* src; int imgs, OH, OW, stride, pad, SH, SW, C, KW, rows;  // rows = taps*C
    const float* scale; const float* shift;
  };
  const Params* P;
  __amdgpu_buffer_rsrc_t rs;
  int nextk;
  int kh[NL], kw[NL], cc[NL];  // tap rows / columns (minus pad) and channel of the thread's r (kh < -64: r out of range)
  int img[NL], oh[NL], ow[NL];  // the pixel of the thread's next load
  f32x4 reg[NL];
  __device__ void init(const Params& Pp, int r0, int tid) {
    P = &Pp; nextk = -1;
    rs = gather_rsrc(Pp.src, (int64_t)Pp.imgs * Pp.SH * Pp.SW * Pp.C);
#pragma unroll
    for (int j = 0; j < NL; ++j) {
      const int q = tid + 256 * j;
      const int r = r0 + (q % (R / 4)) * 4;
      if (r < Pp.rows) {
        const int tap = r / Pp.C;
        cc[j] = r - tap * Pp.C;
        kh[j] = tap / Pp.KW - Pp.pad;
        kw[j] = tap - (tap / Pp.KW) * Pp.KW - Pp.pad;
      } else {
        cc[j] = 0; kh[j] = -100000; kw[j] = 0;
      }
    }
  }
  __device__ void load(int k0) {
    const Params& q = *P;
    const int tid = threadIdx.x;
#pragma unroll
    for (int j = 0; j < NL; ++j) {
      const int kr = (tid + 256 * j) / (R / 4);
      if (k0 != nextk) {  // (first slice of this split: full decomposition)
        const int p = k0 + kr;
        img[j] = p / (q.OH * q.OW);
        const int rem = p - img[j] * q.OH * q.OW;
        oh[j] = rem / q.OW;
        ow[j] = rem - oh[j] * q.OW;
      } else {  // the previous slice's pixel + BK, as a mixed-radix add of (BK / (OH OW), BK / OW % OH, BK % OW)
        const int sw = BK % q.OW, sh = (BK / q.OW) % q.OH, si = BK / (q.OH * q.OW);
        ow[j] += sw;
        const bool cw = ow[j] >= q.OW;
        ow[j] -= cw ? q.OW : 0;
        oh[j] += sh + cw;
        const bool ch = oh[j] >= q.OH;
        oh[j] -= ch ? q.OH : 0;
        img[j] += si + ch;
      }
      const int y = oh[j] * q.stride + kh[j], x = ow[j] * q.stride + kw[j];
      const bool ok = img[j] < q.imgs && (unsigned)y < (unsigned)q.SH && (unsigned)x < (unsigned)q.SW;
      f32x4 v = gather_load(rs, ok, ((img[j] * q.SH + y) * q.SW + x) * q.C + cc[j]);
      if (q.scale) {
        const f32x4 sc = *reinterpret_cast<const f32x4*>(q.scale + cc[j]);
        const f32x4 sh = *reinterpret_cast<const f32x4*>(q.shift + cc[j]);
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = ok ? fmaxf(fmaf(v[e], sc[e], sh[e]), 0.f) : 0.f;
      }
      reg[j] = v;
    }
    nextk = k0 + BK;
  }
  __device__ void store(float* lds) const {
    const int tid = threadIdx.x;
#pragma unroll
    for (int j = 0; j < NL; ++j) {
      const int q = tid + 256 * j;
      const int kr = q / (R / 4), rq = q % (R / 4);
      *reinterpret_cast<f32x4*>(lds + kr * R + rq * 4) = reg[j];
    }
  }
};

// 3-D variants (a2's strided Conv3d, avenue_training_script2.py:19-21): row m = (img, a, b, c) of a GD x GA x GB grid,
// k = tap * C + ch over up to 27 (dd, dh, dw) taps; C % 4 == 0 (each thread's 4 channels lie in one tap), K need not be
// a multiple of BK (k >= taps * C loads zero).
struct TapTable3 {
  int ntaps;
  int8_t dd[27], dh[27], dw[27];
};
struct ConvGeom3 {
  int imgs;
  int GD, GA, GB;  // destination grid
  int sd, sa, sb;  // source step per grid step
  int SD, SH, SW, C;
};

// Per-thread tap walk of the 3-D gathers: a thread's k = k0 + cq advances by BK per slice, its (tap, channel) is
// decomposed at the first slice of a split and then stepped; the taps' (dd, dh, dw, element offset) sit in an LDS
// table (one ds_read_b128 per slice instead of three dependent table loads), entries past the tap count out of range.
constexpr int G3_TAB = 40;  // taps (27 + the tail of a K padded to BK with C >= 4)
__device__ inline void gather3_fill(int* tab, const TapTable3& t, int SH, int SW, int C, int tid) {
  if (tid < G3_TAB) {
    int4 e = {-100000, 0, 0, 0};
    if (tid < t.ntaps) e = {t.dd[tid], t.dh[tid], t.dw[tid], ((t.dd[tid] * SH + t.dh[tid]) * SW + t.dw[tid]) * C};
    reinterpret_cast<int4*>(tab)[tid] = e;
  }
}
struct Gather3Walk {
  int tap, c, nextk;
  __device__ void step(int k0, int cq, int C) {
    if (k0 != nextk) {
      const int k = k0 + cq;
      tap = k / C;
      c = k - tap * C;
    } else {
      c += BK;
      while (c >= C) {
        c -= C;
        ++tap;
      }
    }
    nextk = k0 + BK;
  }
};

template <int R>
struct ConvGather3KC {
  static constexpr bool KC = true;
  static constexpr int NL = R / 32;
  static constexpr int TAB = 4 * G3_TAB;
  struct Params {
    const float* src; ConvGeom3 g; TapTable3 taps;
  };
  const Params* P;
  const int* tab;
  __amdgpu_buffer_rsrc_t rs;
  int cq;
  Gather3Walk w;
  int rowoff[NL];             // element offset of the row's voxel (a * sd, b * sa, c * sb)
  int zd[NL], ya[NL], xb[NL];  // a * sd, b * sa, c * sb (zd < 0: an out-of-range row)
  f32x4 reg[NL];
  __device__ void init(const Params& Pp, int r0, int tid, int* tab_) {
    P = &Pp; tab = tab_; cq = (tid % 8) * 4; w.nextk = -1;
    const ConvGeom3& g = Pp.g;
    rs = gather_rsrc(Pp.src, (int64_t)g.imgs * g.SD * g.SH * g.SW * g.C);
    gather3_fill(tab_, Pp.taps, g.SH, g.SW, g.C, tid);
    const int per = g.GD * g.GA * g.GB;
    const int M = g.imgs * per;
#pragma unroll
    for (int j = 0; j < NL; ++j) {
      const int m = r0 + tid / 8 + 32 * j;
      if (m < M) {
        const int img = m / per, rem = m - img * per;
        const int a = rem / (g.GA * g.GB), r2 = rem - a * g.GA * g.GB;
        const int b = r2 / g.GB, c = r2 - b * g.GB;
        zd[j] = a * g.sd;
        ya[j] = b * g.sa;
        xb[j] = c * g.sb;
        rowoff[j] = (((img * g.SD + zd[j]) * g.SH + ya[j]) * g.SW + xb[j]) * g.C;
      } else {
        rowoff[j] = 0; zd[j] = -100000; ya[j] = 0; xb[j] = 0;
      }
    }
  }
  __device__ void load(int k0) {
    const ConvGeom3& g = P->g;
    w.step(k0, cq, g.C);
    const int4 t = reinterpret_cast<const int4*>(tab)[min(w.tap, G3_TAB - 1)];
    const int toff = t.w + w.c;
#pragma unroll
    for (int j = 0; j < NL; ++j) {
      const bool ok = (unsigned)(zd[j] + t.x) < (unsigned)g.SD && (unsigned)(ya[j] + t.y) < (unsigned)g.SH &&
                      (unsigned)(xb[j] + t.z) < (unsigned)g.SW;
      reg[j] = gather_load(rs, ok, rowoff[j] + toff);
    }
  }
  __device__ void store(float* lds) const {
    const int tid = threadIdx.x;
#pragma unroll
    for (int j = 0; j < NL; ++j) {
      const int row = tid / 8 + 32 * j, kq = tid % 8;
      *reinterpret_cast<f32x4*>(lds + row * KC_STRIDE + kq * 4) = reg[j];
    }
  }
};

// The parity classes of a stride-2 3-D conv's input gradient as one batched GEMM (blockIdx.z = class; k_per_split < 0):
// class z gathers its own taps over its own grid (rows beyond the class's grid load zeros; taps beyond its count too).
struct Conv3ClsGeom {
  int imgs, SD, SH, SW, C;
  int GD[8], GA[8], GB[8];
  TapTable3 taps[8];
};
template <int R>
struct ConvGather3ClsKC {
  static constexpr bool KC = true;
  static constexpr int NL = R / 32;
  static constexpr int TAB = 4 * G3_TAB;
  struct Params {
    const float* src; Conv3ClsGeom g;
  };
  const Params* P;
  const int* tab;
  __amdgpu_buffer_rsrc_t rs;
  int cq;
  Gather3Walk w;
  int rowoff[NL];
  int zd[NL], ya[NL], xb[NL];
  f32x4 reg[NL];
  __device__ void init(const Params& Pp, int r0, int tid, int* tab_) {
    P = &Pp; tab = tab_; cq = (tid % 8) * 4; w.nextk = -1;
    const Conv3ClsGeom& g = Pp.g;
    const int z = blockIdx.z;
    rs = gather_rsrc(Pp.src, (int64_t)g.imgs * g.SD * g.SH * g.SW * g.C);
    gather3_fill(tab_, g.taps[z], g.SH, g.SW, g.C, tid);
    const int GA = g.GA[z], GB = g.GB[z], per = g.GD[z] * GA * GB, M = g.imgs * per;
#pragma unroll
    for (int j = 0; j < NL; ++j) {
      const int m = r0 + tid / 8 + 32 * j;
      if (m < M) {
        const int img = m / per, rem = m - img * per;
        const int a = rem / (GA * GB), r2 = rem - a * GA * GB;
        const int b = r2 / GB, c = r2 - b * GB;
        zd[j] = a; ya[j] = b; xb[j] = c;
        rowoff[j] = (((img * g.SD + a) * g.SH + b) * g.SW + c) * g.C;
      } else {
        rowoff[j] = 0; zd[j] = -100000; ya[j] = 0; xb[j] = 0;
      }
    }
  }
  // the class's real K extent (its own taps x C; the batched launch's K is the largest class's): the K loop of a
  // block stops there instead of multiplying the zero-padded taps
  static __device__ int batch_kend(const Params& Pp) { return Pp.g.taps[blockIdx.z].ntaps * Pp.g.C; }
  __device__ void load(int k0) {
    const Conv3ClsGeom& g = P->g;
    w.step(k0, cq, g.C);
    const int4 t = reinterpret_cast<const int4*>(tab)[min(w.tap, G3_TAB - 1)];
    const int toff = t.w + w.c;
#pragma unroll
    for (int j = 0; j < NL; ++j) {
      const bool ok = (unsigned)(zd[j] + t.x) < (unsigned)g.SD && (unsigned)(ya[j] + t.y) < (unsigned)g.SH &&
                      (unsigned)(xb[j] + t.z) < (unsigned)g.SW;
      reg[j] = gather_load(rs, ok, rowoff[j] + toff);
    }
  }
  __device__ void store(float* lds) const {
    const int tid = threadIdx.x;
#pragma unroll
    for (int j = 0; j < NL; ++j) {
      const int row = tid / 8 + 32 * j, kq = tid % 8;
      *reinterpret_cast<f32x4*>(lds + row * KC_STRIDE + kq * 4) = reg[j];
    }
  }
};

// Row-major matrices X_z[rows][kdim_z] at p + off[z] (blockIdx.z = batch), read K-contiguous (as DenseKC; kdim_z % 4
// == 0, each below 2^31 bytes: buffer loads)
template <int R>
struct DenseKCz {
  static constexpr bool KC = true;
  static constexpr int NL = R / 32;
  struct Params { const float* p; int64_t off[8]; int kdim[8]; int rows; };
  int kdim, rows, r0;
  __amdgpu_buffer_rsrc_t rs;
  f32x4 reg[NL];
  __device__ void init(const Params& P, int r0_, int tid_) {
    kdim = P.kdim[blockIdx.z]; rows = P.rows; r0 = r0_;
    rs = gather_rsrc(P.p + P.off[blockIdx.z], (int64_t)rows * kdim);
  }
  __device__ void load(int k0) {
    const int tid = threadIdx.x;
#pragma unroll
    for (int j = 0; j < NL; ++j) {
      const int row = tid / 8 + 32 * j, kq = tid % 8;
      const int r = r0 + row, k = k0 + kq * 4;
      reg[j] = gather_load(rs, r < rows && k < kdim, r * kdim + k);
    }
  }
  __device__ void store(float* lds) const {
    const int tid = threadIdx.x;
#pragma unroll
    for (int j = 0; j < NL; ++j) {
      const int row = tid / 8 + 32 * j, kq = tid % 8;
      *reinterpret_cast<f32x4*>(lds + row * KC_STRIDE + kq * 4) = reg[j];
    }
  }
};

// B operand of the 3-D conv weight gradient (K-major over output voxels): k = output voxel p = (img, od, oh, ow),
// r = tap * C + c (27 taps kd, kh, kw), value = src[od * s - pad + kd][oh * s - pad + kh][ow * s - pad + kw][c]; the
// voxel coordinates are stepped by BK per slice as in ConvPatchKM
template <int R>
struct ConvPatch3KM {
  static constexpr bool KC = false;
  static constexpr int NL = R / 32;
  struct Params {
    const float* src; int imgs, OD, OH, OW, sd, sh, sw, pad, SD, SH, SW, C, rows;  // rows = 27 * C
    int ones;  // 1: column `rows` is 1 for every pixel (the conv bias gradient as one more GEMM column)
  };
  const Params* P;
  __amdgpu_buffer_rsrc_t rs;
  int r0, tid, nextk;
  int kd[NL], kh[NL], kw[NL], cc[NL];  // kd < 0: r out of range
  int img[NL], od[NL], oh[NL], ow[NL];
  f32x4 reg[NL];
  __device__ void init(const Params& Pp, int r0_, int tid_) {
    P = &Pp; r0 = r0_; tid = tid_; nextk = -1;
    rs = gather_rsrc(Pp.src, (int64_t)Pp.imgs * Pp.SD * Pp.SH * Pp.SW * Pp.C);
#pragma unroll
    for (int j = 0; j < NL; ++j) {
      const int r = r0 + ((tid + 256 * j) % (R / 4)) * 4;
      if (r < Pp.rows) {
        const int tap = r / Pp.C;
        cc[j] = r - tap * Pp.C;
        kd[j] = tap / 9;
        kh[j] = (tap / 3) % 3;
        kw[j] = tap % 3;
      } else {  // (kd = -2: the ones column, r == rows)
        cc[j] = 0; kd[j] = (Pp.ones && r == Pp.rows) ? -2 : -1; kh[j] = 0; kw[j] = 0;
      }
    }
  }
  __device__ void load(int k0) {
    const Params& q = *P;
#pragma unroll
    for (int j = 0; j < NL; ++j) {
      const int kr = (tid + 256 * j) / (R / 4);
      if (k0 != nextk) {
        const int p = k0 + kr, per = q.OD * q.OH * q.OW;
        img[j] = p / per;
        const int rem = p - img[j] * per;
        od[j] = rem / (q.OH * q.OW);
        const int r2 = rem - od[j] * q.OH * q.OW;
        oh[j] = r2 / q.OW;
        ow[j] = r2 - oh[j] * q.OW;
      } else {  // + BK as a mixed-radix add over (img, od, oh, ow)
        const int sw = BK % q.OW, sh = (BK / q.OW) % q.OH, sd = (BK / (q.OW * q.OH)) % q.OD,
                  si = BK / (q.OD * q.OH * q.OW);
        ow[j] += sw;
        const bool cw = ow[j] >= q.OW;
        ow[j] -= cw ? q.OW : 0;
        oh[j] += sh + cw;
        const bool ch = oh[j] >= q.OH;
        oh[j] -= ch ? q.OH : 0;
        od[j] += sd + ch;
        const bool cd = od[j] >= q.OD;
        od[j] -= cd ? q.OD : 0;
        img[j] += si + cd;
      }
      const int z = od[j] * q.sd - q.pad + kd[j], y = oh[j] * q.sh - q.pad + kh[j], x = ow[j] * q.sw - q.pad + kw[j];
      const bool ok = img[j] < q.imgs && kd[j] >= 0 && (unsigned)z < (unsigned)q.SD && (unsigned)y < (unsigned)q.SH &&
                      (unsigned)x < (unsigned)q.SW;
      const f32x4 v = gather_load(rs, ok, (((img[j] * q.SD + z) * q.SH + y) * q.SW + x) * q.C + cc[j]);
      const float one = (kd[j] == -2 && img[j] < q.imgs) ? 1.f : 0.f;
      reg[j] = kd[j] == -2 ? f32x4{one, 0.f, 0.f, 0.f} : v;
    }
    nextk = k0 + BK;
  }
  __device__ void store(float* lds) const {
#pragma unroll
    for (int j = 0; j < NL; ++j) {
      const int qq = tid + 256 * j;
      const int kr = qq / (R / 4), rq = qq % (R / 4);
      *reinterpret_cast<f32x4*>(lds + kr * R + rq * 4) = reg[j];
    }
  }
};

// loaders of a batched launch (k_per_split < 0) may bound each batch's K: static batch_kend(params) (detection idiom)
template <class L, class = void>
struct HasBatchK : std::false_type {};
template <class L>
struct HasBatchK<L, std::void_t<decltype(L::batch_kend(std::declval<const typename L::Params&>()))>> : std::true_type {};

// ------------------------------------------------------------------ the kernel body
// Epi::apply(params, acc, m0, n0, wm, wn, lane, lds_scratch) writes the block's results.
template <class Cfg, class LA, class LB, class Epi>
__global__ __launch_bounds__(256) void gemm_kernel(const typename LA::Params pa, const typename LB::Params pb,
                                                   const typename Epi::Params pe, int M, int N, int K,
                                                   int k_per_split, const int* skip_if_zero) {
  constexpr int BM = Cfg::BM, BN = Cfg::BN, TM = Cfg::TM, TN = Cfg::TN, WN = Cfg::WN;
  constexpr int A_FL = LdsSize<LA::KC, BM>::floats, B_FL = LdsSize<LB::KC, BN>::floats;
  constexpr int STAGE = A_FL + B_FL;
  constexpr int TOTAL = 2 * STAGE > Epi::SCRATCH ? 2 * STAGE : Epi::SCRATCH;
  __shared__ __attribute__((aligned(16))) float lds[TOTAL];
  constexpr int TA = LoaderTab<LA>::n, TB = LoaderTab<LB>::n;
  __shared__ __attribute__((aligned(16))) int tabs[TA + TB + 4];
  if (skip_if_zero != nullptr && *skip_if_zero == 0) return;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;
  const int m0 = blockIdx.x * BM, n0 = blockIdx.y * BN;
  // k_per_split < 0: blockIdx.z is a batch index the loaders / epilogue read themselves (the whole K per block)
  const int kbeg = k_per_split > 0 ? (int)blockIdx.z * k_per_split : 0;
  int kend = k_per_split > 0 ? min(K, kbeg + k_per_split) : K;
  if constexpr (HasBatchK<LA>::value)
    if (k_per_split < 0) kend = min(kend, (LA::batch_kend(pa) + BK - 1) / BK * BK);

  LA la;
  LB lb;
  if constexpr (TA > 0) la.init(pa, m0, tid, tabs);
  else la.init(pa, m0, tid);
  if constexpr (TB > 0) lb.init(pb, n0, tid, tabs + TA);
  else lb.init(pb, n0, tid);
  if constexpr (TA + TB > 0) __syncthreads();
  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  if (kbeg < kend) {
    la.load(kbeg);
    lb.load(kbeg);
    la.store(lds);
    lb.store(lds + A_FL);
    __syncthreads();
    int buf = 0;
    for (int k0 = kbeg; k0 < kend; k0 += BK) {
      const bool more = k0 + BK < kend;
      if (more) {
        la.load(k0 + BK);
        lb.load(k0 + BK);
      }
      const float* As = lds + buf * STAGE;
      const float* Bs = As + A_FL;
#pragma unroll
      for (int kk = 0; kk < BK / 8; ++kk) {
        const int kb = kk * 8 + 4 * (lane >> 5);
        float a[TM][4], b[TN][4];
#pragma unroll
        for (int i = 0; i < TM; ++i) {
          const int row = (wm * TM + i) * 32 + (lane & 31);
          if constexpr (LA::KC) frag_kc<BM>(As, row, kb, a[i]);
          else frag_km<BM>(As, row, kb, a[i]);
        }
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          const int row = (wn * TN + j) * 32 + (lane & 31);
          if constexpr (LB::KC) frag_kc<BN>(Bs, row, kb, b[j]);
          else frag_km<BN>(Bs, row, kb, b[j]);
        }
#pragma unroll
        for (int s = 0; s < 4; ++s)
#pragma unroll
          for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int j = 0; j < TN; ++j) acc[i][j] = mfma32(a[i][s], b[j][s], acc[i][j]);
      }
      if (more) {
        float* Ad = lds + (buf ^ 1) * STAGE;
        la.store(Ad);
        lb.store(Ad + A_FL);
      }
      __syncthreads();
      buf ^= 1;
    }
  }
  Epi::template apply<Cfg>(pe, acc, m0, n0, wm, wn, lane, M, N, lds);
}

// accumulator element -> (row, col) inside the block tile
template <class Cfg>
__device__ inline int acc_row(int wm, int i, int r, int lane) {
  return (wm * Cfg::TM + i) * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
}
template <class Cfg>
__device__ inline int acc_col(int wn, int j, int lane) {
  return (wn * Cfg::TN + j) * 32 + (lane & 31);
}

}  // namespace vad
