// Causal head of CausalAnomalyDetector (cad:194-502) — the stages the reference runs as Python loops over clips,
// frames, detections and trajectories — as five kernels:
//   rows_fwd  (one block per frame)  : box decode + range filter + fallback (cad:198-228), ReID MLP on the real
//                                      boxes, zero-padded trajectory rows x = [box, reid] (cad:248-274) and the GRU
//                                      input projection W_ih x + b_ih for all 5 rows of the frame;
//   seq_fwd   (one block per clip)   : the GRU recurrence over T for all trajectories at once (W_hh in LDS), encoder,
//                                      VAE + KL, pairwise edge MLP, (A z^T)^T dynamics, three scorers (cad:287-502);
//   seq_bwd   (one block per clip)   : reverse of seq_fwd incl. BPTT; small-layer weight grads into a per-clip slab;
//   rows_bwd  (one block per frame)  : d x = W_ih^T d gates, ReID backward, d box -> d detector logits;
//   rows_wgrad (output-parallel)     : GRU and ReID weight/bias grads as fixed-order reductions over all B*T*5 rows.
// Trajectory row r = (b*T + t)*5 + j (j = compacted detection index in frame t = trajectory index n).
// Deterministic: no atomics; per-clip slabs are reduced in clip order.
#include "head.h"
#include "mlp.h"

namespace vad {

constexpr int HT = 512;  // threads of the per-clip sequential kernels
constexpr int G3 = 3 * GH;
constexpr int WHH_LD = GH + 4;  // padded LDS row of W_hh (conflict-free ds_read_b128 over rows)

// ------------------------------------------------------------------ per-row arrays (global, all clips)
struct RowLayout {
  int64_t R;
  int64_t box, x, rh1, rh2, gi, r, z, n, ghn, hp, dgi, dgh, dp4, dp2, dp0, total;
  __host__ __device__ explicit RowLayout(int64_t R_) : R(R_) {
    int64_t o = 0;
    auto take = [&](int64_t w) { int64_t r_ = o; o += (R * w + 63) & ~63ll; return r_; };
    box = take(4); x = take(GIN); rh1 = take(32); rh2 = take(64); gi = take(G3);
    r = take(GH); z = take(GH); n = take(GH); ghn = take(GH); hp = take(GH);
    dgi = take(G3); dgh = take(G3); dp4 = take(64); dp2 = take(64); dp0 = take(32);
    total = o;
  }
};

int64_t head_rows_floats(int B, int T) { return RowLayout((int64_t)B * T * NMAX).total; }

// ------------------------------------------------------------------ per-clip small workspace
struct HL {
  int64_t hT = 0, enc = 0, ce1 = 0, ce2 = 0, mu = 0, lv = 0, zz = 0, node = 0, e = 0, A = 0, s = 0, d1 = 0, d2 = 0,
          pred = 0, cur = 0, prd = 0, cin = 0, cs1 = 0, cs2 = 0, cs = 0, ms1 = 0, ms2 = 0, ms = 0, ts1 = 0, ts2 = 0,
          ts = 0, dh = 0, dhn = 0, scratch = 0, dz = 0, dnode = 0, dA = 0, dpred = 0, ds = 0, total = 0;
  __host__ __device__ constexpr HL() {
    int64_t o = 0;
    auto take = [&](int64_t n_) { int64_t r_ = o; o += (n_ + 3) & ~3ll; return r_; };
    hT = take(NMAX * GH); enc = take(NMAX * 32); ce1 = take(NMAX * 32); ce2 = take(NMAX * 32);
    mu = take(NMAX * NF_); lv = take(NMAX * NF_); zz = take(NMAX * NF_); node = take(NMAX * 32);
    e = take(NMAX * NMAX * 32); A = take(36); s = take(NMAX * NF_); d1 = take(NMAX * 32); d2 = take(NMAX * 32);
    pred = take(NMAX * NF_); cur = take(8); prd = take(8); cin = take(20); cs1 = take(64); cs2 = take(32);
    cs = take(4); ms1 = take(32); ms2 = take(16); ms = take(4); ts1 = take(32); ts2 = take(16); ts = take(4);
    dh = take(NMAX * GH); dhn = take(NMAX * GH); scratch = take(1024); dz = take(NMAX * NF_);
    dnode = take(NMAX * 32); dA = take(36); dpred = take(NMAX * NF_); ds = take(NMAX * NF_);
    total = o;
  }
};

// the per-clip workspace lives in LDS inside the two sequence kernels; [0, dh) is handed from forward to backward
// through global memory
constexpr int HL_TOTAL = (int)HL().total;
constexpr int HL_HANDOFF = (int)HL().dh;
static_assert(HL_TOTAL % 4 == 0 && HL_HANDOFF % 4 == 0, "float4 copies");
// LDS image of the head's small-MLP weights (slots H_ENC_W .. H_NUM-1, packed at HeadArgs::lw_off); it shares its
// LDS with W_hh, which the recurrences need before (forward) or after (backward) the MLP phases
constexpr int HF_BIG = HW_LDS > G3 * WHH_LD ? HW_LDS : G3 * WHH_LD;

int head_pack_weights(HeadArgs& a, const int64_t* numel) {
  const int64_t len = a.off[H_NUM - 1] + numel[H_NUM - 1] - a.off[H_ENC_W];
  a.lw_len = (int)((len + 3) & ~3ll);
  for (int i = H_ENC_W; i < H_NUM; ++i)
    if (a.off[i] % 4) return 1;
  return a.lw_len <= HW_LDS ? 0 : 1;
}

int64_t head_ws_floats(int T) {
  (void)T;
  return HL().total;
}
int64_t head_iws_ints(int T) { return (int64_t)T * (1 + NMAX) + 8; }

// ------------------------------------------------------------------ block-wide small dense layers
// Every layer here is tiny (R <= 5 rows, I, O <= 64) and sits on the head's serial chain, so latency rules: an
// output's dot product is split over a quad of lanes (k = lane&3, +4, ...) and summed with two DPP quad
// permutations, so one pass costs ~I/4 dependent LDS-fed FMAs instead of I. The weight chunk a quad starts at
// is rotated by its output index, spreading the quads of a wave over the LDS banks.
__device__ inline float quad_sum(float s) {
  s += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, s), 0xB1, 0xF, 0xF, false));
  s += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, s), 0x4E, 0xF, 0xF, false));
  return s;
}

// sum_k a[k * sa] b[k * sb] over k < K, split over the quad (lane q = threadIdx.x & 3), chunk start rotated by rot
__device__ inline float quad_dot(const float* a, int sa, const float* b, int sb, int K, int q, int rot) {
  const int nch = (K + 3) >> 2;
  int c = rot % nch;
  float s = 0.f;
  for (int j = 0; j < nch; ++j) {
    const int k = 4 * c + q;
    if (k < K) s = fmaf(a[k * sa], b[k * sb], s);
    c = c + 1 == nch ? 0 : c + 1;
  }
  return quad_sum(s);
}

// out[r][o] = act(b[o] + sum_i W[o][i] in[r][i]) for r < R, o < O (W row-major [O][I])
struct LinF {
  const float* in; int ldi, R, I;
  const float* W; const float* b; int O;
  float* out; int ldo; bool relu;
};

// NL independent layers in one pass (one barrier): layer l's outputs go to the quads following layer l-1's
template <int NL>
__device__ void lin_fwd_n(const LinF (&L)[NL]) {
  const int q = threadIdx.x & 3, nq = blockDim.x >> 2, me = threadIdx.x >> 2;
  int off = 0;
#pragma unroll
  for (int l = 0; l < NL; ++l) {
    const LinF& f = L[l];
    const int n = f.R * f.O;
    int idx = me - off;
    if (idx < 0) idx += nq;
    for (; idx < n; idx += nq) {
      const int r = idx / f.O, o = idx - r * f.O;
      float s = quad_dot(f.W + o * f.I, 1, f.in + r * f.ldi, 1, f.I, q, o);
      if (q == 0) {
        if (f.b) s += f.b[o];
        f.out[r * f.ldo + o] = f.relu ? fmaxf(s, 0.f) : s;
      }
    }
    off = (off + n) % nq;
  }
  __syncthreads();
}

__device__ void lin_fwd(const float* in, int ldi, int R, int I, const float* W, const float* b, int O, float* out,
                        int ldo, bool relu) {
  const LinF L[1] = {{in, ldi, R, I, W, b, O, out, ldo, relu}};
  lin_fwd_n(L);
}

// backward of one LinF-shaped layer given dpre = d(pre-activation) [R][O]:
//   dW[o][i] = sum_r dpre[r][o] in[r][i];  db[o] = sum_r dpre[r][o];
//   din[r][i] (= | +=) sum_o W[o][i] dpre[r][o], then optionally gated by the producer's ReLU: din = gate > 0 ?
//   din * gscale : 0 (fuses the relu_gate pass of the layer below)
struct LinB {
  const float* dpre; int ldd;
  const float* in; int ldi, R, I;
  const float* W; int O;
  float* dW; float* db;
  float* din; int lddin; bool acc;
  const float* gate; int ldg; float gscale;
};

template <int NL>
__device__ void lin_bwd_n(const LinB (&L)[NL]) {
  const int tid = threadIdx.x, q = tid & 3, nq = blockDim.x >> 2, me = tid >> 2;
  // weight / bias grads: R <= 5 terms each, one thread per element
#pragma unroll
  for (int l = 0; l < NL; ++l) {
    const LinB& f = L[l];
    for (int idx = tid; idx < f.O * f.I; idx += blockDim.x) {
      const int o = idx / f.I, i = idx - o * f.I;
      float s = 0.f;
      for (int r = 0; r < f.R; ++r) s = fmaf(f.dpre[r * f.ldd + o], f.in[r * f.ldi + i], s);
      f.dW[idx] = s;  // every head slot is produced by exactly one layer call
    }
    if (f.db) {
      for (int o = tid; o < f.O; o += blockDim.x) {
        float s = 0.f;
        for (int r = 0; r < f.R; ++r) s += f.dpre[r * f.ldd + o];
        f.db[o] = s;
      }
    }
  }
  // input grads: O-long dots, quad-split
  int off = 0;
#pragma unroll
  for (int l = 0; l < NL; ++l) {
    const LinB& f = L[l];
    if (!f.din) continue;
    const int n = f.R * f.I;
    int idx = me - off;
    if (idx < 0) idx += nq;
    for (; idx < n; idx += nq) {
      const int r = idx / f.I, i = idx - r * f.I;
      const float s = quad_dot(f.W + i, f.I, f.dpre + r * f.ldd, 1, f.O, q, i);
      if (q == 0) {
        float* d = f.din + r * f.lddin + i;
        const float v = f.acc ? *d + s : s;
        *d = f.gate ? (f.gate[r * f.ldg + i] > 0.f ? v * f.gscale : 0.f) : v;
      }
    }
    off = (off + n) % nq;
  }
  __syncthreads();
}

__device__ void lin_bwd(const float* dpre, int ldd, const float* in, int ldi, int R, int I,
                        const float* __restrict__ W, int O, float* dW, float* db, float* din, int lddin, bool acc,
                        const float* gate = nullptr, int ldg = 0, float gscale = 1.f) {
  const LinB L[1] = {{dpre, ldd, in, ldi, R, I, W, O, dW, db, din, lddin, acc, gate, ldg, gscale}};
  lin_bwd_n(L);
}

#define PW(slot) (a.pbase + a.off[slot])
#define PL(slot) (sW + (a.off[slot] - a.off[H_ENC_W]))  // LDS weight image

// block-wide copy of n4 float4s (dst index remapped by map): every thread issues U loads before its LDS stores,
// so a copy costs one memory latency per U*blockDim float4s instead of one per blockDim. The loads are
// unconditional (clamped index): a predicated load makes the compiler wait for the previous one before issuing
// the next (its destination registers may still be pending), i.e. U serial round trips.
template <int U, typename Map>
__device__ void block_copy4(float* dst, const float* src, int n4, Map map) {
  if (n4 <= 0) return;
  for (int base = 0; base < n4; base += U * (int)blockDim.x) {
    f32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int i = base + u * (int)blockDim.x + (int)threadIdx.x;
      v[u] = reinterpret_cast<const f32x4*>(src)[min(i, n4 - 1)];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int i = base + u * (int)blockDim.x + (int)threadIdx.x;
      if (i < n4) reinterpret_cast<f32x4*>(dst)[map(i)] = v[u];
    }
  }
}
struct Ident {
  __device__ int operator()(int i) const { return i; }
};

__device__ void stage_head_weights(const HeadArgs& a, float* sW) {
  block_copy4<12>(sW, a.pbase + a.off[H_ENC_W], a.lw_len / 4, Ident{});
}

// ================================================================== forward
// One block per frame.  Every weight row a thread needs is loaded into its registers at the start, in one batch
// beside the box decode: threads 0-191 own the GRU input-projection row q = tid (17 float4), threads 192-255 the ReID
// rows u = tid - 192 (W0 row u < 32, W2 row u, W4 row u).  The dot products keep the reference order (bias first,
// then the inputs in order), so the rows are bitwise those of a per-output loop.
__global__ __launch_bounds__(256) void head_rows_fwd_kernel(HeadArgs a, const float* __restrict__ logits, HeadOut o) {
  static_assert(G3 == 192 && GIN == 68 && NMAX * 4 <= 64, "thread roles: 192 projection rows + 64 ReID rows");
  const int f = blockIdx.x;  // frame b*T + t
  const int b = f / a.T, t = f - b * a.T;
  const int tid = threadIdx.x;
  const RowLayout RL((int64_t)a.B * a.T * NMAX);
  float* rows = a.rows;
  int* iw = a.iws + (int64_t)b * a.iws_stride;
  __shared__ float sbox[NMAX][4];
  __shared__ int svalid[NMAX];
  __shared__ __attribute__((aligned(16))) float sx[NMAX][GIN];
  __shared__ __attribute__((aligned(16))) float sh1[NMAX][32];
  __shared__ __attribute__((aligned(16))) float sh2[NMAX][64];
  __shared__ int scnt;
  const bool proj = tid < G3;
  const int u = proj ? 0 : tid - G3;  // ReID output of threads 192-255
  // weight rows (unconditional loads from valid rows: see block_copy4)
  f32x4 wr[GIN / 4];  // projection row q = tid, or W4 row u (16 float4) + W2 row u (8 float4, in wr[16] / w2)
  f32x4 w2[8];
  f32x4 w0 = *reinterpret_cast<const f32x4*>(PW(H_REID0_W) + (u & 31) * 4);
  if (proj) {
#pragma unroll
    for (int k = 0; k < GIN / 4; ++k) wr[k] = *reinterpret_cast<const f32x4*>(PW(H_GRU_WIH) + tid * GIN + 4 * k);
  } else {
#pragma unroll
    for (int k = 0; k < 16; ++k) wr[k] = *reinterpret_cast<const f32x4*>(PW(H_REID4_W) + u * 64 + 4 * k);
#pragma unroll
    for (int k = 0; k < 8; ++k) w2[k] = *reinterpret_cast<const f32x4*>(PW(H_REID2_W) + u * 32 + 4 * k);
  }
  const float bq = proj ? PW(H_GRU_BIH)[tid] : PW(H_REID4_B)[u];
  const float b2 = PW(H_REID2_B)[u], b0 = PW(H_REID0_B)[u & 31];
  if (tid < NMAX) {
    const float* lg = logits + (int64_t)f * 20 + tid * 4;
    const float X = sigmoidf_(lg[0]) * 360.f, Y = sigmoidf_(lg[1]) * 240.f;
    const float Wd = sigmoidf_(lg[2]) * 80.f + 15.f, Hh = sigmoidf_(lg[3]) * 120.f + 25.f;
    sbox[tid][0] = X; sbox[tid][1] = Y; sbox[tid][2] = Wd; sbox[tid][3] = Hh;
    svalid[tid] = (X >= 10.f && X <= 350.f && Y >= 10.f && Y <= 230.f && Wd >= 10.f && Wd <= 100.f && Hh >= 20.f &&
                   Hh <= 150.f) ? 1 : 0;
  }
  __syncthreads();
  // compaction of the in-range boxes (order kept), fallback box when none (cad:225), zero rows after: box k lands at
  // the number of valid boxes before it (no per-thread array with a runtime index: that would live in scratch)
  __shared__ float cbox[NMAX][4];
  if (tid < NMAX) {
    int n = 0, pos = 0;
    for (int k = 0; k < NMAX; ++k) {
      n += svalid[k];
      if (k < tid) pos += svalid[k];
    }
    int* slot = iw + a.T + t * NMAX;
    if (svalid[tid]) {
      for (int q = 0; q < 4; ++q) cbox[pos][q] = sbox[tid][q];
      slot[pos] = tid;
    }
    if (tid >= n) {
      const bool fb = n == 0 && tid == 0;
      cbox[tid][0] = fb ? 180.f : 0.f;
      cbox[tid][1] = fb ? 120.f : 0.f;
      cbox[tid][2] = fb ? 30.f : 0.f;
      cbox[tid][3] = fb ? 60.f : 0.f;
      slot[tid] = fb ? -1 : -2;
    }
    if (tid == 0) {
      const int c = n > 0 ? n : 1;
      iw[t] = c;
      o.counts[f] = c;
      scnt = c;
    }
  }
  __syncthreads();
  const int cnt = scnt;
  const int64_t r0 = (int64_t)f * NMAX;
  if (tid < NMAX * 4) {
    const int j = tid / 4, q = tid % 4;
    rows[RL.box + (r0 + j) * 4 + q] = cbox[j][q];
    o.boxes[(int64_t)f * NMAX * 4 + tid] = cbox[j][q];
    sx[j][q] = j < cnt ? cbox[j][q] : 0.f;
  }
  // ReID MLP 4 -> 32 -> 64 -> 64 on real rows (zeros elsewhere)
  if (!proj && u < 32) {
#pragma unroll
    for (int j = 0; j < NMAX; ++j) {
      float v = 0.f;
      if (j < cnt) {
        v = b0;
        for (int q = 0; q < 4; ++q) v = fmaf(w0[q], cbox[j][q], v);
        v = fmaxf(v, 0.f);
      }
      sh1[j][u] = v;
      rows[RL.rh1 + (r0 + j) * 32 + u] = v;
    }
  }
  __syncthreads();
  if (!proj) {
#pragma unroll
    for (int j = 0; j < NMAX; ++j) {
      float v = 0.f;
      if (j < cnt) {
        v = b2;
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const f32x4 x = *reinterpret_cast<const f32x4*>(&sh1[j][4 * k]);
          for (int e = 0; e < 4; ++e) v = fmaf(w2[k][e], x[e], v);
        }
        v = fmaxf(v, 0.f);
      }
      sh2[j][u] = v;
      rows[RL.rh2 + (r0 + j) * 64 + u] = v;
    }
  }
  __syncthreads();
  if (!proj) {
#pragma unroll
    for (int j = 0; j < NMAX; ++j) {
      float v = 0.f;
      if (j < cnt) {
        v = bq;
#pragma unroll
        for (int k = 0; k < 16; ++k) {
          const f32x4 x = *reinterpret_cast<const f32x4*>(&sh2[j][4 * k]);
          for (int e = 0; e < 4; ++e) v = fmaf(wr[k][e], x[e], v);
        }
      }
      sx[j][4 + u] = v;
    }
  }
  __syncthreads();
  for (int idx = tid; idx < NMAX * GIN; idx += 256) rows[RL.x + r0 * GIN + idx] = (&sx[0][0])[idx];
  // GRU input projection W_ih x + b_ih for all 5 rows (padded rows see x = 0)
  if (proj) {
#pragma unroll
    for (int j = 0; j < NMAX; ++j) {
      float v = bq;
#pragma unroll
      for (int k = 0; k < GIN / 4; ++k) {
        const f32x4 x = *reinterpret_cast<const f32x4*>(&sx[j][4 * k]);
        for (int e = 0; e < 4; ++e) v = fmaf(wr[k][e], x[e], v);
      }
      rows[RL.gi + (r0 + j) * G3 + tid] = v;
    }
  }
}

__global__ __launch_bounds__(HT) void head_seq_fwd_kernel(HeadArgs a, HeadOut o) {
  const int b = blockIdx.x, T = a.T, tid = threadIdx.x;
  const HL L;
  const RowLayout RL((int64_t)a.B * T * NMAX);
  float* rows = a.rows;
  float* wg = a.ws + (int64_t)b * a.ws_stride;
  const int* iw = a.iws + (int64_t)b * a.iws_stride;
  const int* cnt = iw;
  const int* slot = iw + T;
  __shared__ __attribute__((aligned(16))) float big[HF_BIG];  // W_hh during the recurrence, then the MLP weights
  __shared__ __attribute__((aligned(16))) float sw[HL_TOTAL];
  __shared__ float hs[NMAX * GH];
  float* whh = big;
  float* sW = big;
  float* w = sw;
  __shared__ int s_N, s_any;
  __shared__ float s_red[4];
  const float* Whh = PW(H_GRU_WHH);
  // the n-gate rows of W_hh in LDS (the r / z rows live in registers, below)
  block_copy4<6>(whh, Whh + 2 * GH * GH, GH * GH / 4, [](int i) { return (i >> 4) * (WHH_LD / 4) + (i & 15); });
  for (int i = tid; i < NMAX * GH; i += HT) hs[i] = 0.f;
  if (tid == 0) {
    int N = 1, any = 0;
    for (int t = 0; t < T; ++t) {
      N = max(N, cnt[t]);
      if (slot[t * NMAX] >= 0) any = 1;
    }
    s_N = N;
    s_any = any;
  }
  __syncthreads();
  const int N = s_N;
  const float* bhh = PW(H_GRU_BHH);
  // GRU recurrence, gate order (r, z, n) (cad:284,298): one wave per trajectory slot, lane u owns hidden unit u
  // and computes exactly its three gate pre-activations from W_hh rows u, GH+u (held in its registers: 128 VGPRs,
  // read once) and 2GH+u (LDS), so a time step needs no block barrier -- only the wave's own LDS copy of h
  // (broadcast reads) is exchanged between steps.
  static_assert(NMAX * 64 <= HT && GH == 64, "one wave per trajectory, one lane per hidden unit");
  {
    const int nn = tid >> 6, u = tid & 63;
    if (nn < NMAX) {
      float h = 0.f;
      const bool live = nn < N;
      const float br = bhh[u], bz = bhh[GH + u], bn = bhh[2 * GH + u];
      // (W_hr[u][i], W_hz[u][i]) pairs: the r and z dot products advance together in packed FMAs (v_pk_fma_f32,
      // two fp32 FMAs per lane per instruction -- the step is VALU-bound, two of the five waves share a SIMD)
      f32x2 wrz[GH];
#pragma unroll
      for (int kk = 0; kk < GH / 4; ++kk) {
        const f32x4 r4 = *reinterpret_cast<const f32x4*>(Whh + u * GH + 4 * kk);
        const f32x4 z4 = *reinterpret_cast<const f32x4*>(Whh + (GH + u) * GH + 4 * kk);
#pragma unroll
        for (int j = 0; j < 4; ++j) wrz[4 * kk + j] = f32x2{r4[j], z4[j]};
      }
      const f32x4* wn = reinterpret_cast<const f32x4*>(whh + u * WHH_LD);
      const f32x4* hv = reinterpret_cast<const f32x4*>(hs + nn * GH);
      // the input projections are loaded TC steps at a time, one chunk ahead (double-buffered in registers): a
      // per-step prefetch would be waited for together with the previous step's stores (vmcnt counts both, and
      // with loads and stores both pending the compiler can only wait for zero). The first chunk is waited for
      // explicitly before the loop: left pending, its registers would be treated as pending at every step of
      // every chunk (loop-header merge), i.e. one full store round trip per step.
      constexpr int TC = 4;
      float gc[TC][3], gn[TC][3];
      auto load_gi = [&](int t0, float (&g)[TC][3]) {
#pragma unroll
        for (int k = 0; k < TC; ++k) {
          g[k][0] = g[k][1] = g[k][2] = 0.f;
          if (t0 + k < T) {
            const float* gi = rows + RL.gi + (((int64_t)b * T + t0 + k) * NMAX + nn) * G3;
            g[k][0] = gi[u]; g[k][1] = gi[GH + u]; g[k][2] = gi[2 * GH + u];
          }
        }
      };
      if (live) load_gi(0, gc);
      __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
      for (int t0 = 0; t0 < T; t0 += TC) {
        if (live && t0 + TC < T) load_gi(t0 + TC, gn);
#pragma unroll
        for (int k = 0; k < TC; ++k) {
          const int t = t0 + k;
          if (t >= T) break;
          const int64_t row = ((int64_t)b * T + t) * NMAX + nn;
          if (live) {
            f32x2 rz0 = {br, bz}, rz1 = {0.f, 0.f}, n0 = {bn, 0.f}, n1 = {0.f, 0.f};
#pragma unroll
            for (int kk = 0; kk < GH / 4; ++kk) {
              const f32x4 x = hv[kk], a2 = wn[kk];
              rz0 = __builtin_elementwise_fma(wrz[4 * kk], f32x2{x[0], x[0]}, rz0);
              rz1 = __builtin_elementwise_fma(wrz[4 * kk + 1], f32x2{x[1], x[1]}, rz1);
              rz0 = __builtin_elementwise_fma(wrz[4 * kk + 2], f32x2{x[2], x[2]}, rz0);
              rz1 = __builtin_elementwise_fma(wrz[4 * kk + 3], f32x2{x[3], x[3]}, rz1);
              n0 = __builtin_elementwise_fma(f32x2{a2[0], a2[1]}, f32x2{x[0], x[1]}, n0);
              n1 = __builtin_elementwise_fma(f32x2{a2[2], a2[3]}, f32x2{x[2], x[3]}, n1);
            }
            const f32x2 rz = rz0 + rz1, nn2 = n0 + n1;
            const float an = nn2[0] + nn2[1];
            const float r = gate_sigmoid(gc[k][0] + rz[0]);
            const float z = gate_sigmoid(gc[k][1] + rz[1]);
            const float nv = gate_tanh(gc[k][2] + r * an);
            rows[RL.r + row * GH + u] = r;
            rows[RL.z + row * GH + u] = z;
            rows[RL.n + row * GH + u] = nv;
            rows[RL.ghn + row * GH + u] = an;
            rows[RL.hp + row * GH + u] = h;
            h = (1.f - z) * nv + z * h;
            // every lane's reads of the old h are done (lockstep wave) before the new h is published
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            hs[nn * GH + u] = h;
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            __builtin_amdgcn_wave_barrier();
          } else {  // trajectory slots that do not exist in this clip
            rows[RL.r + row * GH + u] = 0.f;
            rows[RL.z + row * GH + u] = 0.f;
            rows[RL.n + row * GH + u] = 0.f;
            rows[RL.ghn + row * GH + u] = 0.f;
            rows[RL.hp + row * GH + u] = 0.f;
          }
        }
#pragma unroll
        for (int k = 0; k < TC; ++k) {
          gc[k][0] = gn[k][0]; gc[k][1] = gn[k][1]; gc[k][2] = gn[k][2];
        }
      }
    }
  }
  __syncthreads();  // W_hh is dead: its LDS now takes the MLP weight image
  stage_head_weights(a, sW);
  for (int i = tid; i < NMAX * GH; i += HT) w[L.hT + i] = hs[i];
  __syncthreads();
  // encoder + VAE (cad:299, 333-352)
  lin_fwd(w + L.hT, GH, N, GH, PL(H_ENC_W), PL(H_ENC_B), 32, w + L.enc, 32, false);
  lin_fwd(w + L.enc, 32, N, 32, PL(H_CE0_W), PL(H_CE0_B), 32, w + L.ce1, 32, true);
  lin_fwd(w + L.ce1, 32, N, 32, PL(H_CE2_W), PL(H_CE2_B), 32, w + L.ce2, 32, true);
  {
    const LinF V[2] = {{w + L.ce2, 32, N, 32, PL(H_MU_W), PL(H_MU_B), NF_, w + L.mu, NF_, false},
                       {w + L.ce2, 32, N, 32, PL(H_LV_W), PL(H_LV_B), NF_, w + L.lv, NF_, false}};
    lin_fwd_n(V);
  }
  if (tid < N * NF_) {
    const int nn = tid / NF_, f = tid - nn * NF_;
    const float eps = rng_normal(a.h1_eps, (uint64_t)(a.clip0 + b), (uint64_t)(nn * NF_ + f));
    w[L.zz + tid] = w[L.mu + tid] + eps * expf(0.5f * w[L.lv + tid]);
  }
  __syncthreads();
  if (tid < 64) {
    float s = 0.f;
    if (tid < N) {
      float k = 0.f;
      for (int f = 0; f < NF_; ++f) {
        const float mu = w[L.mu + tid * NF_ + f], lv = w[L.lv + tid * NF_ + f];
        k += 1.f + lv - mu * mu - expf(lv);
      }
      s = -0.5f * k;
    }
    s = wave_sum(s);
    if (tid == 0) s_red[0] = s / (float)N;
  }
  // structure learner (cad:371-398)
  lin_fwd(w + L.zz, NF_, N, NF_, PL(H_NODE_W), PL(H_NODE_B), 32, w + L.node, 32, false);
  const int m = min(N, NF_);
  {
    const float* W0 = PL(H_EDGE0_W);
    const float* b0 = PL(H_EDGE0_B);
    for (int idx = tid; idx < m * m * 32; idx += HT) {
      const int pr = idx / 32, u = idx - pr * 32;
      const int i = pr / m, j = pr - i * m;
      if (i == j) continue;
      float s = b0[u];
      const float* wr = W0 + u * 64;
      for (int k = 0; k < 32; ++k) {  // start column rotated by u: conflict-free LDS weight reads
        const int q = (k + u) & 31;
        s = fmaf(wr[q], w[L.node + i * 32 + q], s);
        s = fmaf(wr[32 + q], w[L.node + j * 32 + q], s);
      }
      w[L.e + (int64_t)(i * NMAX + j) * 32 + u] = fmaxf(s, 0.f);
    }
    __syncthreads();
    if (tid < 36) {
      const int i = tid / 6, j = tid - i * 6;
      float v = 0.f;
      if (i != j && i < m && j < m) {
        const float* W2 = PL(H_EDGE2_W);
        float s = PL(H_EDGE2_B)[0];
        for (int q = 0; q < 32; ++q) s = fmaf(W2[q], w[L.e + (int64_t)(i * NMAX + j) * 32 + q], s);
        v = sigmoidf_(s);
      }
      w[L.A + tid] = v;
    }
    __syncthreads();
  }
  // dynamics (cad:415-426): s[n][i] = sum_j A[i][j] z[n][j]
  if (tid < N * NF_) {
    const int nn = tid / NF_, i = tid - nn * NF_;
    float s = 0.f;
    for (int j = 0; j < NF_; ++j) s = fmaf(w[L.A + i * 6 + j], w[L.zz + nn * NF_ + j], s);
    w[L.s + tid] = s;
  }
  __syncthreads();
  lin_fwd(w + L.s, NF_, N, NF_, PL(H_DYN0_W), PL(H_DYN0_B), 32, w + L.d1, 32, true);
  lin_fwd(w + L.d1, 32, N, 32, PL(H_DYN2_W), PL(H_DYN2_B), 32, w + L.d2, 32, true);
  lin_fwd(w + L.d2, 32, N, 32, PL(H_DYN4_W), PL(H_DYN4_B), NF_, w + L.pred, NF_, false);
  // scorer (cad:463-502)
  float* cin = w + L.cin;
  if (tid < NF_) {
    float c = 0.f, p = 0.f;
    for (int nn = 0; nn < N; ++nn) {
      c += w[L.zz + nn * NF_ + tid];
      p += w[L.pred + nn * NF_ + tid];
    }
    c /= (float)N;
    p /= (float)N;
    w[L.cur + tid] = c;
    w[L.prd + tid] = p;
    cin[tid] = c;
    cin[6 + tid] = p;
    cin[12 + tid] = fabsf(c - p);
  }
  __syncthreads();
  // the three scorers are independent: one pass (and barrier) per depth
  {
    const LinF S0[3] = {{cin, 18, 1, 18, PL(H_CS0_W), PL(H_CS0_B), 64, w + L.cs1, 64, true},
                        {cin, 18, 1, 12, PL(H_MS0_W), PL(H_MS0_B), 32, w + L.ms1, 32, true},
                        {cin, 18, 1, 6, PL(H_TS0_W), PL(H_TS0_B), 32, w + L.ts1, 32, true}};
    lin_fwd_n(S0);
  }
  if (a.training && tid < 64) {
    const bool keep = rng_u24(a.h1_drop, (uint64_t)(a.clip0 + b), (uint64_t)tid) >= a.thr_drop;
    w[L.cs1 + tid] = keep ? w[L.cs1 + tid] * (1.0f / 0.8f) : 0.f;
  }
  __syncthreads();
  {
    const LinF S1[3] = {{w + L.cs1, 64, 1, 64, PL(H_CS3_W), PL(H_CS3_B), 32, w + L.cs2, 32, true},
                        {w + L.ms1, 32, 1, 32, PL(H_MS2_W), PL(H_MS2_B), 16, w + L.ms2, 16, true},
                        {w + L.ts1, 32, 1, 32, PL(H_TS2_W), PL(H_TS2_B), 16, w + L.ts2, 16, true}};
    lin_fwd_n(S1);
    const LinF S2[3] = {{w + L.cs2, 32, 1, 32, PL(H_CS5_W), PL(H_CS5_B), 1, w + L.cs, 1, false},
                        {w + L.ms2, 16, 1, 16, PL(H_MS4_W), PL(H_MS4_B), 1, w + L.ms, 1, false},
                        {w + L.ts2, 16, 1, 16, PL(H_TS4_W), PL(H_TS4_B), 1, w + L.ts, 1, false}};
    lin_fwd_n(S2);
  }
  if (tid == 0) {
    const float cs = sigmoidf_(w[L.cs]), ms = sigmoidf_(w[L.ms]), ts = sigmoidf_(w[L.ts]);
    w[L.cs + 1] = cs; w[L.ms + 1] = ms; w[L.ts + 1] = ts;
    o.causal[b] = 0.5f * cs + 0.3f * ms + 0.2f * ts;
    o.kl[b] = s_red[0];
    o.nmax[b] = N;
    o.clip_flags[b * 2 + 0] = s_any;
    o.clip_flags[b * 2 + 1] = m >= 2 ? 1 : 0;
  }
  for (int i = tid; i < NMAX * NF_; i += HT) o.z[(int64_t)b * NMAX * NF_ + i] = (i < N * NF_) ? w[L.zz + i] : 0.f;
  for (int i = tid; i < 36; i += HT) o.adj[(int64_t)b * 36 + i] = w[L.A + i];
  __syncthreads();
  // hand the activations to the backward kernel
  block_copy4<3>(wg, sw, HL_HANDOFF / 4, Ident{});
}

int head_rows_fwd(const HeadArgs& a, const float* det_logits, const HeadOut& o, hipStream_t st) {
  VAD_CHECK(a.T <= 4096, "head: T too large");
  VAD_KLAUNCH(head_rows_fwd_kernel, dim3(a.B * a.T), dim3(256), 0, st, a, det_logits, o);
  VAD_LAUNCH_CHECK();
  return 0;
}
int head_seq_fwd(const HeadArgs& a, const HeadOut& o, hipStream_t st) {
  VAD_KLAUNCH(head_seq_fwd_kernel, dim3(a.B), dim3(HT), 0, st, a, o);
  VAD_LAUNCH_CHECK();
  return 0;
}
int head_fwd(const HeadArgs& a, const float* det_logits, const HeadOut& o, hipStream_t st) {
  VAD_TRY(head_rows_fwd(a, det_logits, o, st));
  return head_seq_fwd(a, o, st);
}


// ================================================================== backward
#define GW(slot) (g + (a.off[slot] - a.head_begin))

__global__ __launch_bounds__(HT) void head_seq_bwd_kernel(HeadArgs a, HeadOut o, HeadUp up, float* slabs,
                                                          int64_t slab_len) {
  const int b = blockIdx.x, T = a.T, tid = threadIdx.x;
  const HL L;
  const RowLayout RL((int64_t)a.B * T * NMAX);
  float* rows = a.rows;
  const float* wg = a.ws + (int64_t)b * a.ws_stride;
  float* g = slabs + (int64_t)b * slab_len;
  __shared__ __attribute__((aligned(16))) float big[HF_BIG];  // MLP weight image, then W_hh [q][j] for BPTT
  __shared__ __attribute__((aligned(16))) float sw[HL_TOTAL];
  __shared__ __attribute__((aligned(16))) float dgh_s[NMAX * G3];
  float* sW = big;
  float* w = sw;
  stage_head_weights(a, sW);
  block_copy4<3>(sw, wg, HL_HANDOFF / 4, Ident{});
  // slots the layer calls below may not write (structure learner without edges, the sparsity weight) read as 0;
  // GRU / ReID slots are overwritten by head_rows_wgrad
  for (int64_t i = tid; i < slab_len / 4; i += HT) reinterpret_cast<f32x4*>(g)[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int N = o.nmax[b];
  const int m = min(N, NF_);
  const float dscore = up.d_causal[b];
  const float dkl = up.d_kl[b];
  float* cin = w + L.cin;
  float* d1 = w + L.scratch;  // 1024-float scratch
  float* dcin = w + L.scratch + 960;
  for (int i = tid; i < 18; i += HT) dcin[i] = 0.f;
  __syncthreads();
  // ---- scorer (cad:485-497)
  {
    const float cs = w[L.cs + 1], ms = w[L.ms + 1], ts = w[L.ts + 1];
    if (tid == 0) {
      d1[0] = 0.5f * dscore * cs * (1.f - cs);
      d1[1] = 0.3f * dscore * ms * (1.f - ms);
      d1[2] = 0.2f * dscore * ts * (1.f - ts);
    }
    __syncthreads();
    // the three scorers are independent: one pass per depth, the ReLU gates fused into the input grads; their
    // d cin parts land in separate rows and are summed in the reference's order (cs, ms, ts) below
    float* dcs2 = d1 + 8;
    float* dcs1 = d1 + 40;
    float* dms2 = d1 + 104;
    float* dms1 = d1 + 120;
    float* dts2 = d1 + 152;
    float* dts1 = d1 + 168;
    float* dcin3 = d1 + 200;  // [3][18]: d cin from cs / ms / ts
    const LinB S2[3] = {
        {d1 + 0, 1, w + L.cs2, 32, 1, 32, PL(H_CS5_W), 1, GW(H_CS5_W), GW(H_CS5_B), dcs2, 32, false, w + L.cs2, 32, 1.f},
        {d1 + 1, 1, w + L.ms2, 16, 1, 16, PL(H_MS4_W), 1, GW(H_MS4_W), GW(H_MS4_B), dms2, 16, false, w + L.ms2, 16, 1.f},
        {d1 + 2, 1, w + L.ts2, 16, 1, 16, PL(H_TS4_W), 1, GW(H_TS4_W), GW(H_TS4_B), dts2, 16, false, w + L.ts2, 16, 1.f}};
    lin_bwd_n(S2);
    const float sdrop = a.training ? 1.f / 0.8f : 1.f;
    const LinB S1[3] = {
        {dcs2, 32, w + L.cs1, 64, 1, 64, PL(H_CS3_W), 32, GW(H_CS3_W), GW(H_CS3_B), dcs1, 64, false, w + L.cs1, 64, sdrop},
        {dms2, 16, w + L.ms1, 32, 1, 32, PL(H_MS2_W), 16, GW(H_MS2_W), GW(H_MS2_B), dms1, 32, false, w + L.ms1, 32, 1.f},
        {dts2, 16, w + L.ts1, 32, 1, 32, PL(H_TS2_W), 16, GW(H_TS2_W), GW(H_TS2_B), dts1, 32, false, w + L.ts1, 32, 1.f}};
    lin_bwd_n(S1);
    const LinB S0[3] = {
        {dcs1, 64, cin, 18, 1, 18, PL(H_CS0_W), 64, GW(H_CS0_W), GW(H_CS0_B), dcin3, 18, false, nullptr, 0, 1.f},
        {dms1, 32, cin, 18, 1, 12, PL(H_MS0_W), 32, GW(H_MS0_W), GW(H_MS0_B), dcin3 + 18, 18, false, nullptr, 0, 1.f},
        {dts1, 32, cin, 18, 1, 6, PL(H_TS0_W), 32, GW(H_TS0_W), GW(H_TS0_B), dcin3 + 36, 18, false, nullptr, 0, 1.f}};
    lin_bwd_n(S0);
    if (tid < 18) dcin[tid] = (dcin3[tid] + (tid < 12 ? dcin3[18 + tid] : 0.f)) + (tid < 6 ? dcin3[36 + tid] : 0.f);
    __syncthreads();
  }
  float* dz = w + L.dz;
  float* dpred = w + L.dpred;
  if (tid < NMAX * NF_) {
    const int nn = tid / NF_, f = tid - nn * NF_;
    const float c = w[L.cur + f], p = w[L.prd + f];
    const float sg = c > p ? 1.f : (c < p ? -1.f : 0.f);  // d|c-p| (sign(0) = 0)
    const float dc = dcin[f] + dcin[12 + f] * sg;
    const float dp = dcin[6 + f] - dcin[12 + f] * sg;
    const bool live = nn < N;
    dz[tid] = live ? dc / (float)N + (up.d_z ? up.d_z[(int64_t)b * NMAX * NF_ + tid] : 0.f) : 0.f;
    dpred[tid] = live ? dp / (float)N : 0.f;
  }
  __syncthreads();
  // ---- dynamics
  float* ds = w + L.ds;
  {
    float* dd2 = d1;
    float* dd1 = d1 + NMAX * 32;
    lin_bwd(dpred, NF_, w + L.d2, 32, N, 32, PL(H_DYN4_W), NF_, GW(H_DYN4_W), GW(H_DYN4_B), dd2, 32, false,
            w + L.d2, 32);
    lin_bwd(dd2, 32, w + L.d1, 32, N, 32, PL(H_DYN2_W), 32, GW(H_DYN2_W), GW(H_DYN2_B), dd1, 32, false, w + L.d1, 32);
    lin_bwd(dd1, 32, w + L.s, NF_, N, NF_, PL(H_DYN0_W), 32, GW(H_DYN0_W), GW(H_DYN0_B), ds, NF_, false);
  }
  float* dA = w + L.dA;
  if (tid < 36) {
    const int i = tid / 6, j = tid - i * 6;
    float s = up.d_adj ? up.d_adj[(int64_t)b * 36 + tid] : 0.f;
    for (int nn = 0; nn < N; ++nn) s = fmaf(ds[nn * NF_ + i], w[L.zz + nn * NF_ + j], s);
    dA[tid] = (i == j) ? 0.f : s;
  }
  if (tid >= 64 && tid < 64 + N * NF_) {
    const int q = tid - 64, nn = q / NF_, j = q - nn * NF_;
    float s = 0.f;
    for (int i = 0; i < NF_; ++i) s = fmaf(w[L.A + i * 6 + j], ds[nn * NF_ + i], s);
    dz[q] += s;
  }
  __syncthreads();
  // ---- structure learner (only when edges exist)
  if (m >= 2) {
    float* dnode = w + L.dnode;
    for (int i = tid; i < NMAX * 32; i += HT) dnode[i] = 0.f;
    float* de = d1;  // [pairs][32]
    const float* W2 = PL(H_EDGE2_W);
    for (int idx = tid; idx < m * m * 32; idx += HT) {
      const int pr = idx / 32, u = idx - pr * 32;
      const int i = pr / m, j = pr - i * m;
      float v = 0.f;
      if (i != j) {
        const float Aij = w[L.A + i * 6 + j];
        const float da = dA[i * 6 + j] * Aij * (1.f - Aij);
        const float e = w[L.e + (int64_t)(i * NMAX + j) * 32 + u];
        v = e > 0.f ? da * W2[u] : 0.f;
      }
      de[idx] = v;
    }
    __syncthreads();
    if (tid < 33) {
      float s = 0.f;
      for (int i = 0; i < m; ++i)
        for (int j = 0; j < m; ++j) {
          if (i == j) continue;
          const float Aij = w[L.A + i * 6 + j];
          const float da = dA[i * 6 + j] * Aij * (1.f - Aij);
          s += tid < 32 ? da * w[L.e + (int64_t)(i * NMAX + j) * 32 + tid] : da;
        }
      if (tid < 32) GW(H_EDGE2_W)[tid] = s;
      else GW(H_EDGE2_B)[0] = s;
    }
    float* dW0 = GW(H_EDGE0_W);
    for (int idx = tid; idx < 32 * 64; idx += HT) {
      const int u = idx / 64, q = idx - u * 64;
      float s = 0.f;
      for (int i = 0; i < m; ++i)
        for (int j = 0; j < m; ++j) {
          if (i == j) continue;
          const float in = q < 32 ? w[L.node + i * 32 + q] : w[L.node + j * 32 + q - 32];
          s = fmaf(de[(i * m + j) * 32 + u], in, s);
        }
      dW0[idx] = s;
    }
    if (tid < 32) {
      float s = 0.f;
      for (int pr = 0; pr < m * m; ++pr) s += de[pr * 32 + tid];
      GW(H_EDGE0_B)[tid] = s;
    }
    const float* W0 = PL(H_EDGE0_W);
    for (int idx = tid; idx < m * 32; idx += HT) {
      const int k = idx / 32, q = idx - k * 32;
      float s = 0.f;
      for (int j = 0; j < m; ++j) {
        if (j == k) continue;
        for (int u = 0; u < 32; ++u) {
          s = fmaf(W0[u * 64 + q], de[(k * m + j) * 32 + u], s);       // k as source i
          s = fmaf(W0[u * 64 + 32 + q], de[(j * m + k) * 32 + u], s);  // k as target j
        }
      }
      dnode[idx] = s;
    }
    __syncthreads();
    lin_bwd(dnode, 32, w + L.zz, NF_, N, NF_, PL(H_NODE_W), 32, GW(H_NODE_W), GW(H_NODE_B), dz, NF_, true);
  }
  // ---- VAE + KL (cad:328-347)
  {
    float* dmu = d1;
    float* dlv = d1 + 32;
    if (tid < N * NF_) {
      const int nn = tid / NF_, f = tid - nn * NF_;
      const float eps = rng_normal(a.h1_eps, (uint64_t)(a.clip0 + b), (uint64_t)(nn * NF_ + f));
      const float mu = w[L.mu + tid], lv = w[L.lv + tid];
      const float dzz = dz[tid];
      const float kls = dkl / (float)N;
      dmu[tid] = dzz + kls * mu;
      dlv[tid] = dzz * eps * 0.5f * expf(0.5f * lv) + kls * 0.5f * (expf(lv) - 1.f);
    }
    __syncthreads();
    float* dce2 = d1 + 64;
    float* dce1 = d1 + 256;
    lin_bwd(dmu, NF_, w + L.ce2, 32, N, 32, PL(H_MU_W), NF_, GW(H_MU_W), GW(H_MU_B), dce2, 32, false);
    lin_bwd(dlv, NF_, w + L.ce2, 32, N, 32, PL(H_LV_W), NF_, GW(H_LV_W), GW(H_LV_B), dce2, 32, true, w + L.ce2, 32);
    lin_bwd(dce2, 32, w + L.ce1, 32, N, 32, PL(H_CE2_W), 32, GW(H_CE2_W), GW(H_CE2_B), dce1, 32, false, w + L.ce1, 32);
    float* denc = d1 + 448;
    lin_bwd(dce1, 32, w + L.enc, 32, N, 32, PL(H_CE0_W), 32, GW(H_CE0_W), GW(H_CE0_B), denc, 32, false);
    lin_bwd(denc, 32, w + L.hT, GH, N, GH, PL(H_ENC_W), 32, GW(H_ENC_W), GW(H_ENC_B), w + L.dh, GH, false);
  }
  // ---- GRU backward through time (dh'/dz = h - n, dh'/dn = 1 - z)
  {
    float* dh = w + L.dh;
    // one wave per trajectory slot, lane u owns hidden unit u: the 3 gate grads of unit u are computed in-lane,
    // published to the wave's LDS row, and dh_prev[u] = dh[u] z[u] + sum_q W_hh[q][u] dgh[q] reads them back --
    // no block barrier inside the time loop
    static_assert(NMAX * 64 <= HT && GH == 64, "one wave per trajectory, one lane per hidden unit");
    // column u of W_hh (W_hh[q][u], q < 3 GH) lives in lane u's registers: the recurrence reads only the
    // wave's 3 GH gate grads from LDS (broadcast b128), not 192 lane-distinct LDS words per step
    const float* Whh = PW(H_GRU_WHH);
    const int nn = tid >> 6, u = tid & 63;
    if (nn < NMAX) {
      const bool live = nn < N;
      f32x2 wc[G3 / 2];  // (W_hh[2p][u], W_hh[2p+1][u]): packed FMAs, two partial-sum chains (see the forward)
#pragma unroll
      for (int q = 0; q < G3 / 2; ++q) wc[q] = f32x2{Whh[2 * q * GH + u], Whh[(2 * q + 1) * GH + u]};
      float d = live ? dh[nn * GH + u] : 0.f;
      float* dgv = dgh_s + nn * G3;
      // the saved gates are loaded TC steps at a time, one chunk ahead (double-buffered in registers; see the
      // forward recurrence)
      constexpr int TC = 2;
      float sc_[TC][5], sn_[TC][5];  // r, z, n, h_prev, W_hn h_prev + b_hn of steps t0, t0-1, ...
      auto load_gates = [&](int t0, float (&g)[TC][5]) {
#pragma unroll
        for (int k = 0; k < TC; ++k) {
          g[k][0] = g[k][1] = g[k][2] = g[k][3] = g[k][4] = 0.f;
          if (t0 - k >= 0) {
            const int64_t row = ((int64_t)b * T + t0 - k) * NMAX + nn;
            g[k][0] = rows[RL.r + row * GH + u]; g[k][1] = rows[RL.z + row * GH + u];
            g[k][2] = rows[RL.n + row * GH + u]; g[k][3] = rows[RL.hp + row * GH + u];
            g[k][4] = rows[RL.ghn + row * GH + u];
          }
        }
      };
      if (live) load_gates(T - 1, sc_);
      __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): see the forward recurrence
      for (int t0 = T - 1; t0 >= 0; t0 -= TC) {
        if (live && t0 - TC >= 0) load_gates(t0 - TC, sn_);
#pragma unroll
        for (int k = 0; k < TC; ++k) {
          const int t = t0 - k;
          if (t < 0) break;
          const int64_t row = ((int64_t)b * T + t) * NMAX + nn;
          float* dgi = rows + RL.dgi + row * G3;
          float* dgh = rows + RL.dgh + row * G3;
          if (live) {
            const float r = sc_[k][0], z = sc_[k][1], nv = sc_[k][2], hp = sc_[k][3], ghn = sc_[k][4];
            const float dan = d * (1.f - z) * (1.f - nv * nv);
            const float daz = d * (hp - nv) * z * (1.f - z);
            const float dar = dan * ghn * r * (1.f - r);
            dgi[u] = dar; dgi[GH + u] = daz; dgi[2 * GH + u] = dan;
            dgh[u] = dar; dgh[GH + u] = daz; dgh[2 * GH + u] = dan * r;
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            dgv[u] = dar;
            dgv[GH + u] = daz;
            dgv[2 * GH + u] = dan * r;
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            f32x2 s0 = {d * z, 0.f}, s1 = {0.f, 0.f};
            const f32x4* dg4 = reinterpret_cast<const f32x4*>(dgv);
#pragma unroll
            for (int q4 = 0; q4 < G3 / 4; ++q4) {
              const f32x4 g = dg4[q4];
              s0 = __builtin_elementwise_fma(wc[2 * q4], f32x2{g[0], g[1]}, s0);
              s1 = __builtin_elementwise_fma(wc[2 * q4 + 1], f32x2{g[2], g[3]}, s1);
            }
            const f32x2 s2 = s0 + s1;
            d = s2[0] + s2[1];
          } else {
            dgi[u] = 0.f; dgi[GH + u] = 0.f; dgi[2 * GH + u] = 0.f;
            dgh[u] = 0.f; dgh[GH + u] = 0.f; dgh[2 * GH + u] = 0.f;
          }
        }
#pragma unroll
        for (int k = 0; k < TC; ++k)
#pragma unroll
          for (int e = 0; e < 5; ++e) sc_[k][e] = sn_[k][e];
      }
    }
  }
}

// per frame: d x = W_ih^T d gi for real rows, ReID backward, d box -> d detector logits
__global__ __launch_bounds__(256) void head_rows_bwd_kernel(HeadArgs a, const float* __restrict__ logits,
                                                            float* __restrict__ dlog,
                                                            const float* __restrict__ dboxes) {
  const int f = blockIdx.x;
  const int b = f / a.T, t = f - b * a.T;
  const int tid = threadIdx.x;
  const RowLayout RL((int64_t)a.B * a.T * NMAX);
  float* rows = a.rows;
  const int* iw = a.iws + (int64_t)b * a.iws_stride;
  const int cnt = iw[t];
  const int* slot = iw + a.T + t * NMAX;
  const int64_t r0 = (int64_t)f * NMAX;
  __shared__ float sdx[NMAX][GIN];
  __shared__ float sd2[NMAX][64];
  __shared__ float sd1[NMAX][32];
  const float* Wih = PW(H_GRU_WIH);
  for (int idx = tid; idx < NMAX * GIN; idx += 256) {
    const int j = idx / GIN, i = idx - j * GIN;
    float s = 0.f;
    if (j < cnt) {
      const float* dgi = rows + RL.dgi + (r0 + j) * G3;
      for (int q = 0; q < G3; ++q) s = fmaf(Wih[(int64_t)q * GIN + i], dgi[q], s);
    }
    sdx[j][i] = s;
  }
  __syncthreads();
  // reid layer 4 (no activation): d pre = d x[4:68]
  for (int idx = tid; idx < NMAX * 64; idx += 256) {
    const int j = idx / 64, u = idx - j * 64;
    rows[RL.dp4 + (r0 + j) * 64 + u] = sdx[j][4 + u];  // zero for padding rows
  }
  const float* W4 = PW(H_REID4_W);
  for (int idx = tid; idx < NMAX * 64; idx += 256) {
    const int j = idx / 64, k = idx - j * 64;
    float s = 0.f;
    if (j < cnt) {
      for (int u = 0; u < 64; ++u) s = fmaf(W4[u * 64 + k], sdx[j][4 + u], s);
      s = rows[RL.rh2 + (r0 + j) * 64 + k] > 0.f ? s : 0.f;
    }
    sd2[j][k] = s;
    rows[RL.dp2 + (r0 + j) * 64 + k] = s;
  }
  __syncthreads();
  const float* W2 = PW(H_REID2_W);
  for (int idx = tid; idx < NMAX * 32; idx += 256) {
    const int j = idx / 32, k = idx - j * 32;
    float s = 0.f;
    if (j < cnt) {
      for (int u = 0; u < 64; ++u) s = fmaf(W2[u * 32 + k], sd2[j][u], s);
      s = rows[RL.rh1 + (r0 + j) * 32 + k] > 0.f ? s : 0.f;
    }
    sd1[j][k] = s;
    rows[RL.dp0 + (r0 + j) * 32 + k] = s;
  }
  __syncthreads();
  const float* W0 = PW(H_REID0_W);
  if (tid < NMAX * 4) {
    const int j = tid / 4, c = tid % 4;
    if (j < cnt && slot[j] >= 0) {  // the fallback box is a constant: no grad
      float dv = sdx[j][c];
      for (int u = 0; u < 32; ++u) dv = fmaf(W0[u * 4 + c], sd1[j][u], dv);
      // a loss on the returned detections (the reference's boxes are slices of the rescaled detector output,
      // cad:201-222): its grad enters at the same compacted slot
      if (dboxes) dv += dboxes[(int64_t)f * NMAX * 4 + j * 4 + c];
      const int k = slot[j];
      const float sg = sigmoidf_(logits[(int64_t)f * 20 + k * 4 + c]);
      const float sc = c == 0 ? 360.f : (c == 1 ? 240.f : (c == 2 ? 80.f : 120.f));
      dlog[(int64_t)f * 20 + k * 4 + c] = dv * sc * sg * (1.f - sg);
    }
  }
}

int head_bwd(const HeadArgs& a, const float* det_logits, const HeadOut& o, const HeadUp& up, float* slabs,
             int64_t slab_len, float* d_det_logits, hipStream_t st) {
  VAD_HIP(hipMemsetAsync(d_det_logits, 0, sizeof(float) * (size_t)a.B * a.T * 20, st));
  hipLaunchKernelGGL(head_seq_bwd_kernel, dim3(a.B), dim3(HT), 0, st, a, o, up, slabs, slab_len);
  VAD_LAUNCH_CHECK();
  hipLaunchKernelGGL(head_rows_bwd_kernel, dim3(a.B * a.T), dim3(256), 0, st, a, det_logits, d_det_logits,
                     up.d_boxes);
  VAD_LAUNCH_CHECK();
  return 0;
}

__global__ void head_slab_reduce_kernel(const float* __restrict__ slabs, int B, int64_t len, float* __restrict__ g) {
  for (int64_t i = blockIdx.x * 256ll + threadIdx.x; i < len; i += (int64_t)gridDim.x * 256) {
    float s = 0.f;
    for (int b = 0; b < B; ++b) s += slabs[(int64_t)b * len + i];
    g[i] = s;
  }
}

int head_slab_reduce(const float* slabs, int B, int64_t slab_len, float* grad_head, hipStream_t st) {
  hipLaunchKernelGGL(head_slab_reduce_kernel, dim3((unsigned)std::min<int64_t>(cdiv(slab_len, 256), 512)), dim3(256),
                     0, st, slabs, B, slab_len, grad_head);
  VAD_LAUNCH_CHECK();
  return 0;
}

// GRU + ReID weight/bias grads over all R trajectory rows: five Linear-style (W, b) pairs, one rows_wgrad launch
int head_rows_wgrad(const HeadArgs& a, hipStream_t st) {
  const RowLayout RL((int64_t)a.B * a.T * NMAX);
  RowsWgradArgs w{};
  w.R = (int)RL.R;
  w.nseg = 5;
  auto seg = [&](int k, int ws, int bs, int64_t dA, int64_t dX, int O, int I) {
    w.seg[k] = RowsWgradSeg{a.grad + a.off[ws], a.grad + a.off[bs], a.rows + dA, a.rows + dX, O, I};
  };
  seg(0, H_GRU_WIH, H_GRU_BIH, RL.dgi, RL.x, G3, GIN);
  seg(1, H_GRU_WHH, H_GRU_BHH, RL.dgh, RL.hp, G3, GH);
  seg(2, H_REID4_W, H_REID4_B, RL.dp4, RL.rh2, 64, 64);
  seg(3, H_REID2_W, H_REID2_B, RL.dp2, RL.rh1, 64, 32);
  seg(4, H_REID0_W, H_REID0_B, RL.dp0, RL.box, 32, 4);
  return rows_wgrad(w, st);
}

// ================================================================== tail: softmax, blend, losses
// loss-mode upstream grads of clip b (cad:655-676 through the blend fin = 0.6 c + 0.4 p1 and the softmax)
__device__ inline void tail_loss_grads(const TailArgs& t, int b, float p0, float p1, float c, float fin) {
  const float fB = (float)t.B;
  const int y = (int)t.labels[b];
  const float yf = (float)y;
  float d_final = 0.3f * 2.f * (fin - yf) / fB;
  float d_c = 0.2f * 2.f * (c - yf) / fB;
  const float m2 = fmaxf(p0, p1);
  const float e0 = expf(p0 - m2), e1 = expf(p1 - m2);
  const float q0 = e0 / (e0 + e1), q1 = e1 / (e0 + e1);
  float dp0 = 0.4f * (q0 - (y == 0 ? 1.f : 0.f)) / fB;
  float dp1 = 0.4f * (q1 - (y == 1 ? 1.f : 0.f)) / fB;
  const float dk = isfinite(t.kl[b]) ? 0.1f / fB : 0.f;
  d_c += 0.6f * d_final;
  dp1 += 0.4f * d_final;
  const float dot = p0 * dp0 + p1 * dp1;  // through softmax: dl = p * (dp - <p, dp>)
  t.d_direct_logits[b * 2] = p0 * (dp0 - dot);
  t.d_direct_logits[b * 2 + 1] = p1 * (dp1 - dot);
  t.d_causal[b] = d_c;
  t.d_kl[b] = dk;
}

__global__ void cad_tail_fwd_kernel(TailArgs t) {
  const int B = t.B;
  if (t.nbt && (int)threadIdx.x < t.nbt_n) t.nbt[threadIdx.x] += 1;
  __shared__ float red[4][256];
  float cls = 0.f, an = 0.f, ca = 0.f, kl = 0.f;
  int fdet = 0, fst = 0;
  for (int b = threadIdx.x; b < B; b += 256) {
    const float l0 = t.direct_logits[b * 2], l1 = t.direct_logits[b * 2 + 1];
    const float mx = fmaxf(l0, l1);
    const float e0 = expf(l0 - mx), e1 = expf(l1 - mx);
    const float p0 = e0 / (e0 + e1), p1 = e1 / (e0 + e1);
    t.probs[b * 2] = p0;
    t.probs[b * 2 + 1] = p1;
    const float c = t.causal[b];
    const float fin = 0.6f * c + 0.4f * p1;
    t.final_scores[b] = fin;
    fdet |= t.clip_flags[b * 2];
    fst |= t.clip_flags[b * 2 + 1];
    if (t.labels) {
      const int y = (int)t.labels[b];
      const float yf = (float)y;
      // CrossEntropy over the softmax OUTPUT used as logits (cad:673)
      const float m2 = fmaxf(p0, p1);
      const float lse = m2 + logf(expf(p0 - m2) + expf(p1 - m2));
      cls += lse - (y == 0 ? p0 : p1);
      an += (fin - yf) * (fin - yf);
      ca += (c - yf) * (c - yf);
      const float k = t.kl[b];
      if (isfinite(k)) kl += k;
      if (t.fwd_bwd) tail_loss_grads(t, b, p0, p1, c, fin);
    }
  }
  red[0][threadIdx.x] = cls;
  red[1][threadIdx.x] = an;
  red[2][threadIdx.x] = ca;
  red[3][threadIdx.x] = kl;
  __shared__ int fl[2];
  if (threadIdx.x == 0) fl[0] = fl[1] = 0;
  __syncthreads();
  if (fdet) atomicOr(&fl[0], 1);
  if (fst) atomicOr(&fl[1], 1);
  for (int s = 128; s > 0; s >>= 1) {
    if (threadIdx.x < s)
      for (int q = 0; q < 4; ++q) red[q][threadIdx.x] += red[q][threadIdx.x + s];
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    t.flags[0] = fl[0];
    t.flags[1] = fl[1];
    if (t.det_gate) *t.det_gate = fl[0] ? 0ull : 1ull;
    if (t.flags_f) {
      t.flags_f[0] = (float)fl[0];
      t.flags_f[1] = (float)fl[1];
    }
    if (t.labels) {
      const float fB = (float)B;
      const float c = red[0][0] / fB, an2 = red[1][0] / fB, ca2 = red[2][0] / fB, k = red[3][0] / fB;
      t.losses[0] = c;
      t.losses[1] = an2;
      t.losses[2] = ca2;
      t.losses[3] = k;
      t.losses[4] = 0.4f * c + 0.3f * an2 + 0.2f * ca2 + 0.1f * k;
    }
  }
}

int cad_tail_fwd(const TailArgs& t, hipStream_t st) {
  VAD_KLAUNCH(cad_tail_fwd_kernel, dim3(1), dim3(256), 0, st, t);
  VAD_LAUNCH_CHECK();
  return 0;
}

// upstream grads: from the loss (labels) or from external autograd grads
__global__ void cad_tail_bwd_kernel(TailArgs t) {
  const int B = t.B;
  // re-arm the detector gate for this backward (a second backward on the same forward must wait for its own detector
  // input gradient again): 0 = wait, 1 = no detector gradient (no box in range)
  if (threadIdx.x == 0 && t.det_gate) *t.det_gate = t.flags[0] ? 0ull : 1ull;
  for (int b = threadIdx.x; b < B; b += 256) {
    const float p0 = t.probs[b * 2], p1 = t.probs[b * 2 + 1];
    const float c = t.causal[b], fin = t.final_scores[b];
    if (t.labels) {
      tail_loss_grads(t, b, p0, p1, c, fin);
      continue;
    }
    float d_final = t.ext_d_final ? t.ext_d_final[b] : 0.f;
    float d_c = t.ext_d_causal ? t.ext_d_causal[b] : 0.f;
    float dp0 = t.ext_d_probs ? t.ext_d_probs[b * 2] : 0.f;
    float dp1 = t.ext_d_probs ? t.ext_d_probs[b * 2 + 1] : 0.f;
    const float dk = t.ext_d_kl ? t.ext_d_kl[b] : 0.f;
    d_c += 0.6f * d_final;
    dp1 += 0.4f * d_final;
    const float dot = p0 * dp0 + p1 * dp1;  // through softmax: dl = p * (dp - <p, dp>)
    t.d_direct_logits[b * 2] = p0 * (dp0 - dot);
    t.d_direct_logits[b * 2 + 1] = p1 * (dp1 - dot);
    t.d_causal[b] = d_c;
    t.d_kl[b] = dk;
  }
}

int cad_tail_bwd(const TailArgs& t, hipStream_t st) {
  hipLaunchKernelGGL(cad_tail_bwd_kernel, dim3(1), dim3(256), 0, st, t);
  VAD_LAUNCH_CHECK();
  return 0;
}

}  // namespace vad
