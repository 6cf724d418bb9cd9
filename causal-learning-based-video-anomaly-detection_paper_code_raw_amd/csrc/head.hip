// Fused causal head: one 256-thread block per clip runs every per-clip stage of CausalAnomalyDetector that the
// reference executes as Python loops (cad:194-502): box decode + range filter + fallback, ReID MLP, zero-padded
// trajectory tensor, GRU(68->64) over T for all trajectories at once, latent encoder, VAE + KL, pairwise edge
// MLP -> 6x6 adjacency, (A z^T)^T dynamics MLP, three scorers and the 0.5/0.3/0.2 blend.  The backward kernel is
// the hand-derived reverse of the same graph (BPTT through the GRU) writing a per-clip gradient slab, reduced
// afterwards in a fixed clip order (deterministic, no atomics).
#include "head.h"

namespace vad {

// ------------------------------------------------------------------ per-clip workspace layout
struct HL {
  int T;
  int64_t boxes, x, rh1, rh2, gi, ghn, r, z, n, hp, hT, enc, ce1, ce2, mu, lv, zz, node, e, A, s, d1, d2, pred;
  int64_t cur, prd, cs1, cs2, cs, ms1, ms2, ms, ts1, ts2, ts;
  int64_t dgi, dgh, dx, dh, dtmp, dtmp2, dz, dnode, dA, dpred, ds, total;
  __host__ __device__ HL(int T_) : T(T_) {
    int64_t o = 0;
    auto take = [&](int64_t n_) { int64_t r_ = o; o += (n_ + 3) & ~3ll; return r_; };
    const int64_t TN = (int64_t)T * NMAX;
    boxes = take(TN * 4); x = take(TN * GIN); rh1 = take(TN * 32); rh2 = take(TN * 64);
    gi = take(TN * 3 * GH); ghn = take(TN * GH); r = take(TN * GH); z = take(TN * GH); n = take(TN * GH);
    hp = take(TN * GH); hT = take(NMAX * GH); enc = take(NMAX * 32); ce1 = take(NMAX * 32); ce2 = take(NMAX * 32);
    mu = take(NMAX * NF_); lv = take(NMAX * NF_); zz = take(NMAX * NF_); node = take(NMAX * 32);
    e = take(NMAX * NMAX * 32); A = take(36); s = take(NMAX * NF_); d1 = take(NMAX * 32); d2 = take(NMAX * 32);
    pred = take(NMAX * NF_); cur = take(8); prd = take(8); cs1 = take(64); cs2 = take(32); cs = take(4);
    ms1 = take(32); ms2 = take(16); ms = take(4); ts1 = take(32); ts2 = take(16); ts = take(4);
    dgi = take(TN * 3 * GH); dgh = take(TN * 3 * GH); dx = take(TN * GIN); dh = take(NMAX * GH);
    dtmp = take(TN * 64 > 1024 ? TN * 64 : 1024); dtmp2 = take(TN * 64 > 512 ? TN * 64 : 512); dz = take(NMAX * NF_); dnode = take(NMAX * 32); dA = take(36);
    dpred = take(NMAX * NF_); ds = take(NMAX * NF_);
    total = o;
  }
};

int64_t head_ws_floats(int T) { return HL(T).total; }
int64_t head_iws_ints(int T) { return (int64_t)T * (1 + NMAX) + 8; }

// ------------------------------------------------------------------ block-wide small dense layers
// out[r][o] = act(b[o] + sum_i W[o][i] * in[r][i])
__device__ void lin_fwd(const float* in, int ldi, int R, int I, const float* __restrict__ W,
                        const float* __restrict__ b, int O, float* out, int ldo, bool relu) {
  for (int idx = threadIdx.x; idx < R * O; idx += blockDim.x) {
    const int r = idx / O, o = idx - r * O;
    float s = b ? b[o] : 0.f;
    const float* w = W + (int64_t)o * I;
    const float* v = in + (int64_t)r * ldi;
    for (int i = 0; i < I; ++i) s = fmaf(w[i], v[i], s);
    out[(int64_t)r * ldo + o] = relu ? fmaxf(s, 0.f) : s;
  }
  __syncthreads();
}

// given dpre[r][o]: dW[o][i] += sum_r dpre[r][o] in[r][i]; db[o] += sum_r dpre[r][o];
// din[r][i] (=, or += when acc) = sum_o W[o][i] dpre[r][o]
__device__ void lin_bwd(const float* dpre, int ldd, const float* in, int ldi, int R, int I,
                        const float* __restrict__ W, int O, float* dW, float* db, float* din, int lddin, bool acc) {
  for (int idx = threadIdx.x; idx < O * I; idx += blockDim.x) {
    const int o = idx / I, i = idx - o * I;
    float s = 0.f;
    for (int r = 0; r < R; ++r) s = fmaf(dpre[(int64_t)r * ldd + o], in[(int64_t)r * ldi + i], s);
    dW[idx] += s;
  }
  if (db) {
    for (int o = threadIdx.x; o < O; o += blockDim.x) {
      float s = 0.f;
      for (int r = 0; r < R; ++r) s += dpre[(int64_t)r * ldd + o];
      db[o] += s;
    }
  }
  if (din) {
    for (int idx = threadIdx.x; idx < R * I; idx += blockDim.x) {
      const int r = idx / I, i = idx - r * I;
      float s = 0.f;
      for (int o = 0; o < O; ++o) s = fmaf(W[(int64_t)o * I + i], dpre[(int64_t)r * ldd + o], s);
      if (acc) din[(int64_t)r * lddin + i] += s;
      else din[(int64_t)r * lddin + i] = s;
    }
  }
  __syncthreads();
}

// relu gate in place: d[r][o] *= (out[r][o] > 0) * scale
__device__ void relu_gate(float* d, int ldd, const float* out, int ldo, int R, int O, float scale) {
  for (int idx = threadIdx.x; idx < R * O; idx += blockDim.x) {
    const int r = idx / O, o = idx - r * O;
    d[(int64_t)r * ldd + o] = out[(int64_t)r * ldo + o] > 0.f ? d[(int64_t)r * ldd + o] * scale : 0.f;
  }
  __syncthreads();
}

#define PW(slot) (a.pbase + a.off[slot])

// ------------------------------------------------------------------ forward
__global__ __launch_bounds__(256) void head_fwd_kernel(HeadArgs a, const float* __restrict__ logits, HeadOut o) {
  const int b = blockIdx.x, T = a.T, tid = threadIdx.x;
  const HL L(T);
  float* w = a.ws + (int64_t)b * a.ws_stride;
  int* iw = a.iws + (int64_t)b * a.iws_stride;
  int* cnt = iw;               // [T]
  int* slot = iw + T;          // [T][5] original detection index of compacted row j (-1: fallback)
  __shared__ int s_N, s_valid_any;
  __shared__ float s_red[8];

  // 1. box decode + range filter + fallback (cad:198-228)
  if (tid < T) {
    const int t = tid;
    const float* lg = logits + ((int64_t)b * T + t) * 20;
    float* bx = w + L.boxes + (int64_t)t * NMAX * 4;
    int c = 0;
    for (int k = 0; k < NMAX; ++k) {
      const float X = sigmoidf_(lg[k * 4 + 0]) * 360.f;
      const float Y = sigmoidf_(lg[k * 4 + 1]) * 240.f;
      const float Wd = sigmoidf_(lg[k * 4 + 2]) * 80.f + 15.f;
      const float Hh = sigmoidf_(lg[k * 4 + 3]) * 120.f + 25.f;
      if (X >= 10.f && X <= 350.f && Y >= 10.f && Y <= 230.f && Wd >= 10.f && Wd <= 100.f && Hh >= 20.f &&
          Hh <= 150.f) {
        bx[c * 4 + 0] = X; bx[c * 4 + 1] = Y; bx[c * 4 + 2] = Wd; bx[c * 4 + 3] = Hh;
        slot[t * NMAX + c] = k;
        ++c;
      }
    }
    if (c == 0) {
      bx[0] = 180.f; bx[1] = 120.f; bx[2] = 30.f; bx[3] = 60.f;
      slot[t * NMAX] = -1;
      c = 1;
    }
    for (int j = c; j < NMAX; ++j) {
      bx[j * 4 + 0] = bx[j * 4 + 1] = bx[j * 4 + 2] = bx[j * 4 + 3] = 0.f;
      slot[t * NMAX + j] = -2;
    }
    cnt[t] = c;
  }
  __syncthreads();
  if (tid == 0) {
    int N = 1, any = 0;
    for (int t = 0; t < T; ++t) {
      N = max(N, cnt[t]);
      if (slot[t * NMAX] >= 0) any = 1;
    }
    s_N = N;
    s_valid_any = any;
  }
  __syncthreads();
  const int N = s_N;
  // export detections
  for (int i = tid; i < T * NMAX * 4; i += 256) o.boxes[(int64_t)b * T * NMAX * 4 + i] = w[L.boxes + i];
  for (int t = tid; t < T; t += 256) o.counts[(int64_t)b * T + t] = cnt[t];

  // 2. ReID MLP on every real row; trajectory rows x[t][j] = [box, reid] or zeros (cad:248-274)
  //    rows are laid out [t][j] with j < NMAX; rows j >= cnt[t] are zero padding.
  const int TN = T * NMAX;
  lin_fwd(w + L.boxes, 4, TN, 4, PW(H_REID0_W), PW(H_REID0_B), 32, w + L.rh1, 32, true);
  lin_fwd(w + L.rh1, 32, TN, 32, PW(H_REID2_W), PW(H_REID2_B), 64, w + L.rh2, 64, true);
  lin_fwd(w + L.rh2, 64, TN, 64, PW(H_REID4_W), PW(H_REID4_B), 64, w + L.x + 4, GIN, false);
  for (int idx = tid; idx < TN * GIN; idx += 256) {
    const int row = idx / GIN, col = idx - row * GIN;
    const int t = row / NMAX, j = row - t * NMAX;
    float* xr = w + L.x + (int64_t)row * GIN;
    if (j >= cnt[t]) xr[col] = 0.f;
    else if (col < 4) xr[col] = w[L.boxes + (int64_t)row * 4 + col];
  }
  __syncthreads();

  // 3. GRU input projections for all steps, then the recurrence (cad:284,298; gate order r,z,n)
  lin_fwd(w + L.x, GIN, TN, GIN, PW(H_GRU_WIH), PW(H_GRU_BIH), 3 * GH, w + L.gi, 3 * GH, false);
  float* h = w + L.hT;  // running hidden state, final value = h_T
  for (int i = tid; i < NMAX * GH; i += 256) h[i] = 0.f;
  __syncthreads();
  const float* Whh = PW(H_GRU_WHH);
  const float* bhh = PW(H_GRU_BHH);
  float* ghs = w + L.dtmp;  // scratch [N][192]
  for (int t = 0; t < T; ++t) {
    for (int idx = tid; idx < N * 3 * GH; idx += 256) {
      const int nn = idx / (3 * GH), g = idx - nn * 3 * GH;
      float s = bhh[g];
      const float* wr = Whh + (int64_t)g * GH;
      const float* hv = h + nn * GH;
      for (int j = 0; j < GH; ++j) s = fmaf(wr[j], hv[j], s);
      ghs[idx] = s;
    }
    __syncthreads();
    for (int idx = tid; idx < N * GH; idx += 256) {
      const int nn = idx / GH, u = idx - nn * GH;
      const int64_t row = (int64_t)t * NMAX + nn;
      const float* gi = w + L.gi + row * 3 * GH;
      const float* gh = ghs + nn * 3 * GH;
      const float r = sigmoidf_(gi[u] + gh[u]);
      const float z = sigmoidf_(gi[GH + u] + gh[GH + u]);
      const float nv = tanhf(gi[2 * GH + u] + r * gh[2 * GH + u]);
      const float hprev = h[idx];
      w[L.r + row * GH + u] = r;
      w[L.z + row * GH + u] = z;
      w[L.n + row * GH + u] = nv;
      w[L.ghn + row * GH + u] = gh[2 * GH + u];
      w[L.hp + row * GH + u] = hprev;
      h[idx] = (1.f - z) * nv + z * hprev;
    }
    __syncthreads();
  }

  // 4. encoder + VAE (cad:299, 333-352)
  lin_fwd(h, GH, N, GH, PW(H_ENC_W), PW(H_ENC_B), 32, w + L.enc, 32, false);
  lin_fwd(w + L.enc, 32, N, 32, PW(H_CE0_W), PW(H_CE0_B), 32, w + L.ce1, 32, true);
  lin_fwd(w + L.ce1, 32, N, 32, PW(H_CE2_W), PW(H_CE2_B), 32, w + L.ce2, 32, true);
  lin_fwd(w + L.ce2, 32, N, 32, PW(H_MU_W), PW(H_MU_B), NF_, w + L.mu, NF_, false);
  lin_fwd(w + L.ce2, 32, N, 32, PW(H_LV_W), PW(H_LV_B), NF_, w + L.lv, NF_, false);
  if (tid < N * NF_) {
    const int nn = tid / NF_, f = tid - nn * NF_;
    const float eps = rng_normal(a.h1_eps, (uint64_t)(a.clip0 + b), (uint64_t)(nn * NF_ + f));
    const float mu = w[L.mu + tid], lv = w[L.lv + tid];
    w[L.zz + tid] = mu + eps * expf(0.5f * lv);
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
  // 5. structure learner (cad:371-398): node encoder + pairwise edge MLP for i != j < min(N,6)
  lin_fwd(w + L.zz, NF_, N, NF_, PW(H_NODE_W), PW(H_NODE_B), 32, w + L.node, 32, false);
  const int m = min(N, NF_);
  {
    const float* W0 = PW(H_EDGE0_W);
    const float* b0 = PW(H_EDGE0_B);
    for (int idx = tid; idx < m * m * 32; idx += 256) {
      const int pr = idx / 32, u = idx - pr * 32;
      const int i = pr / m, j = pr - i * m;
      if (i == j) continue;
      float s = b0[u];
      const float* wr = W0 + u * 64;
      const float* ni = w + L.node + i * 32;
      const float* nj = w + L.node + j * 32;
      for (int q = 0; q < 32; ++q) s = fmaf(wr[q], ni[q], s);
      for (int q = 0; q < 32; ++q) s = fmaf(wr[32 + q], nj[q], s);
      w[L.e + (int64_t)(i * NMAX + j) * 32 + u] = fmaxf(s, 0.f);
    }
    __syncthreads();
    if (tid < 36) {
      const int i = tid / 6, j = tid - i * 6;
      float v = 0.f;
      if (i != j && i < m && j < m) {
        const float* W2 = PW(H_EDGE2_W);
        float s = PW(H_EDGE2_B)[0];
        const float* ev = w + L.e + (int64_t)(i * NMAX + j) * 32;
        for (int q = 0; q < 32; ++q) s = fmaf(W2[q], ev[q], s);
        v = sigmoidf_(s);
      }
      w[L.A + tid] = v;
    }
    __syncthreads();
  }
  // 6. dynamics (cad:415-426): s[n][i] = sum_j A[i][j] z[n][j]
  if (tid < N * NF_) {
    const int nn = tid / NF_, i = tid - nn * NF_;
    float s = 0.f;
    for (int j = 0; j < NF_; ++j) s = fmaf(w[L.A + i * 6 + j], w[L.zz + nn * NF_ + j], s);
    w[L.s + tid] = s;
  }
  __syncthreads();
  lin_fwd(w + L.s, NF_, N, NF_, PW(H_DYN0_W), PW(H_DYN0_B), 32, w + L.d1, 32, true);
  lin_fwd(w + L.d1, 32, N, 32, PW(H_DYN2_W), PW(H_DYN2_B), 32, w + L.d2, 32, true);
  lin_fwd(w + L.d2, 32, N, 32, PW(H_DYN4_W), PW(H_DYN4_B), NF_, w + L.pred, NF_, false);
  // 7. scorer (cad:463-502)
  float* cin = w + L.dtmp2;  // [cur(6) prd(6) diff(6)]
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
  lin_fwd(cin, 18, 1, 18, PW(H_CS0_W), PW(H_CS0_B), 64, w + L.cs1, 64, true);
  if (a.training && tid < 64) {
    const bool keep = rng_u24(a.h1_drop, (uint64_t)(a.clip0 + b), (uint64_t)tid) >= a.thr_drop;
    w[L.cs1 + tid] = keep ? w[L.cs1 + tid] * (1.0f / 0.8f) : 0.f;
  }
  __syncthreads();
  lin_fwd(w + L.cs1, 64, 1, 64, PW(H_CS3_W), PW(H_CS3_B), 32, w + L.cs2, 32, true);
  lin_fwd(w + L.cs2, 32, 1, 32, PW(H_CS5_W), PW(H_CS5_B), 1, w + L.cs, 1, false);
  lin_fwd(cin, 18, 1, 12, PW(H_MS0_W), PW(H_MS0_B), 32, w + L.ms1, 32, true);
  lin_fwd(w + L.ms1, 32, 1, 32, PW(H_MS2_W), PW(H_MS2_B), 16, w + L.ms2, 16, true);
  lin_fwd(w + L.ms2, 16, 1, 16, PW(H_MS4_W), PW(H_MS4_B), 1, w + L.ms, 1, false);
  lin_fwd(cin, 18, 1, 6, PW(H_TS0_W), PW(H_TS0_B), 32, w + L.ts1, 32, true);
  lin_fwd(w + L.ts1, 32, 1, 32, PW(H_TS2_W), PW(H_TS2_B), 16, w + L.ts2, 16, true);
  lin_fwd(w + L.ts2, 16, 1, 16, PW(H_TS4_W), PW(H_TS4_B), 1, w + L.ts, 1, false);
  if (tid == 0) {
    const float cs = sigmoidf_(w[L.cs]), ms = sigmoidf_(w[L.ms]), ts = sigmoidf_(w[L.ts]);
    w[L.cs + 1] = cs; w[L.ms + 1] = ms; w[L.ts + 1] = ts;
    o.causal[b] = 0.5f * cs + 0.3f * ms + 0.2f * ts;
    o.kl[b] = s_red[0];
    o.nmax[b] = N;
    o.clip_flags[b * 2 + 0] = s_valid_any;
    o.clip_flags[b * 2 + 1] = m >= 2 ? 1 : 0;
  }
  for (int i = tid; i < NMAX * NF_; i += 256) o.z[(int64_t)b * NMAX * NF_ + i] = (i < N * NF_) ? w[L.zz + i] : 0.f;
  for (int i = tid; i < 36; i += 256) o.adj[(int64_t)b * 36 + i] = w[L.A + i];
}

int head_fwd(const HeadArgs& a, const float* det_logits, const HeadOut& o, hipStream_t st) {
  VAD_CHECK(a.T <= 256, "head: T must be <= 256");
  hipLaunchKernelGGL(head_fwd_kernel, dim3(a.B), dim3(256), 0, st, a, det_logits, o);
  VAD_LAUNCH_CHECK();
  return 0;
}

// ------------------------------------------------------------------ backward
#define GW(slot) (g + (a.off[slot] - a.head_begin))

__global__ __launch_bounds__(256) void head_bwd_kernel(HeadArgs a, const float* __restrict__ logits, HeadOut o,
                                                       HeadUp up, float* slabs, int64_t slab_len,
                                                       float* __restrict__ dlog) {
  const int b = blockIdx.x, T = a.T, tid = threadIdx.x;
  const HL L(T);
  float* w = a.ws + (int64_t)b * a.ws_stride;
  const int* iw = a.iws + (int64_t)b * a.iws_stride;
  const int* cnt = iw;
  const int* slot = iw + T;
  float* g = slabs + (int64_t)b * slab_len;
  for (int64_t i = tid; i < slab_len; i += 256) g[i] = 0.f;
  const int N = o.nmax[b];
  const int m = min(N, NF_);
  const float dscore = up.d_causal[b];
  const float dkl = up.d_kl[b];
  __syncthreads();

  // ---- scorer (cad:485-497)
  float* dcin = w + L.dtmp2 + 32;  // [18]
  float* cin = w + L.dtmp2;
  float* d1 = w + L.dtmp;          // scratch rows
  for (int i = tid; i < 18; i += 256) dcin[i] = 0.f;
  __syncthreads();
  {
    // causal scorer: sigmoid -> L5 <- relu L3 <- dropout relu L0
    const float cs = w[L.cs + 1], ms = w[L.ms + 1], ts = w[L.ts + 1];
    if (tid == 0) {
      d1[0] = 0.5f * dscore * cs * (1.f - cs);
      d1[1] = 0.3f * dscore * ms * (1.f - ms);
      d1[2] = 0.2f * dscore * ts * (1.f - ts);
    }
    __syncthreads();
    float* dcs2 = d1 + 8;   // [32]
    float* dcs1 = d1 + 40;  // [64]
    lin_bwd(d1 + 0, 1, w + L.cs2, 32, 1, 32, PW(H_CS5_W), 1, GW(H_CS5_W), GW(H_CS5_B), dcs2, 32, false);
    relu_gate(dcs2, 32, w + L.cs2, 32, 1, 32, 1.f);
    lin_bwd(dcs2, 32, w + L.cs1, 64, 1, 64, PW(H_CS3_W), 32, GW(H_CS3_W), GW(H_CS3_B), dcs1, 64, false);
    relu_gate(dcs1, 64, w + L.cs1, 64, 1, 64, a.training ? 1.f / 0.8f : 1.f);
    lin_bwd(dcs1, 64, cin, 18, 1, 18, PW(H_CS0_W), 64, GW(H_CS0_W), GW(H_CS0_B), dcin, 18, true);
    float* dms2 = d1 + 104;  // [16]
    float* dms1 = d1 + 120;  // [32]
    lin_bwd(d1 + 1, 1, w + L.ms2, 16, 1, 16, PW(H_MS4_W), 1, GW(H_MS4_W), GW(H_MS4_B), dms2, 16, false);
    relu_gate(dms2, 16, w + L.ms2, 16, 1, 16, 1.f);
    lin_bwd(dms2, 16, w + L.ms1, 32, 1, 32, PW(H_MS2_W), 16, GW(H_MS2_W), GW(H_MS2_B), dms1, 32, false);
    relu_gate(dms1, 32, w + L.ms1, 32, 1, 32, 1.f);
    lin_bwd(dms1, 32, cin, 18, 1, 12, PW(H_MS0_W), 32, GW(H_MS0_W), GW(H_MS0_B), dcin, 18, true);
    float* dts2 = d1 + 152;  // [16]
    float* dts1 = d1 + 168;  // [32]
    lin_bwd(d1 + 2, 1, w + L.ts2, 16, 1, 16, PW(H_TS4_W), 1, GW(H_TS4_W), GW(H_TS4_B), dts2, 16, false);
    relu_gate(dts2, 16, w + L.ts2, 16, 1, 16, 1.f);
    lin_bwd(dts2, 16, w + L.ts1, 32, 1, 32, PW(H_TS2_W), 16, GW(H_TS2_W), GW(H_TS2_B), dts1, 32, false);
    relu_gate(dts1, 32, w + L.ts1, 32, 1, 32, 1.f);
    lin_bwd(dts1, 32, cin, 18, 1, 6, PW(H_TS0_W), 32, GW(H_TS0_W), GW(H_TS0_B), dcin, 18, true);
  }
  // d cur / d prd including |cur - prd| (sign(0) = 0), then the means over N
  float* dz = w + L.dz;
  float* dpred = w + L.dpred;
  if (tid < NMAX * NF_) {
    const int nn = tid / NF_, f = tid - nn * NF_;
    const float c = w[L.cur + f], p = w[L.prd + f];
    const float sg = c > p ? 1.f : (c < p ? -1.f : 0.f);
    const float dc = dcin[f] + dcin[12 + f] * sg;
    const float dp = dcin[6 + f] - dcin[12 + f] * sg;
    const bool live = nn < N;
    dz[tid] = live ? dc / (float)N + (up.d_z ? up.d_z[(int64_t)b * NMAX * NF_ + tid] : 0.f) : 0.f;
    dpred[tid] = live ? dp / (float)N : 0.f;
  }
  __syncthreads();

  // ---- dynamics MLP backward -> d s
  float* ds = w + L.ds;
  {
    float* dd2 = d1;            // [N][32]
    float* dd1 = d1 + NMAX * 32;
    lin_bwd(dpred, NF_, w + L.d2, 32, N, 32, PW(H_DYN4_W), NF_, GW(H_DYN4_W), GW(H_DYN4_B), dd2, 32, false);
    relu_gate(dd2, 32, w + L.d2, 32, N, 32, 1.f);
    lin_bwd(dd2, 32, w + L.d1, 32, N, 32, PW(H_DYN2_W), 32, GW(H_DYN2_W), GW(H_DYN2_B), dd1, 32, false);
    relu_gate(dd1, 32, w + L.d1, 32, N, 32, 1.f);
    lin_bwd(dd1, 32, w + L.s, NF_, N, NF_, PW(H_DYN0_W), 32, GW(H_DYN0_W), GW(H_DYN0_B), ds, NF_, false);
  }
  // s = (A z^T)^T: dA[i][j] = sum_n ds[n][i] z[n][j] (+ external), dz[n][j] += sum_i A[i][j] ds[n][i]
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
  // ---- structure learner backward (only when edges exist)
  if (m >= 2) {
    float* dnode = w + L.dnode;
    for (int i = tid; i < NMAX * 32; i += 256) dnode[i] = 0.f;
    float* de = d1;  // [pairs][32] pre-activation grads
    float* dW2 = GW(H_EDGE2_W);
    __syncthreads();
    const float* W2 = PW(H_EDGE2_W);
    for (int idx = tid; idx < m * m * 32; idx += 256) {
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
    // edge2 weight/bias grads
    if (tid < 33) {
      float s = 0.f;
      for (int i = 0; i < m; ++i)
        for (int j = 0; j < m; ++j) {
          if (i == j) continue;
          const float Aij = w[L.A + i * 6 + j];
          const float da = dA[i * 6 + j] * Aij * (1.f - Aij);
          s += tid < 32 ? da * w[L.e + (int64_t)(i * NMAX + j) * 32 + tid] : da;
        }
      if (tid < 32) dW2[tid] += s;
      else GW(H_EDGE2_B)[0] += s;
    }
    // edge0: input [node_i, node_j] (64)
    float* dW0 = GW(H_EDGE0_W);
    for (int idx = tid; idx < 32 * 64; idx += 256) {
      const int u = idx / 64, q = idx - u * 64;
      float s = 0.f;
      for (int i = 0; i < m; ++i)
        for (int j = 0; j < m; ++j) {
          if (i == j) continue;
          const float in = q < 32 ? w[L.node + i * 32 + q] : w[L.node + j * 32 + q - 32];
          s = fmaf(de[(i * m + j) * 32 + u], in, s);
        }
      dW0[idx] += s;
    }
    if (tid < 32) {
      float s = 0.f;
      for (int pr = 0; pr < m * m; ++pr) s += de[pr * 32 + tid];
      GW(H_EDGE0_B)[tid] += s;
    }
    const float* W0 = PW(H_EDGE0_W);
    for (int idx = tid; idx < m * 32; idx += 256) {
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
    lin_bwd(dnode, 32, w + L.zz, NF_, N, NF_, PW(H_NODE_W), 32, GW(H_NODE_W), GW(H_NODE_B), dz, NF_, true);
  }
  // ---- VAE + KL backward (cad:328-347)
  {
    float* dmu = d1;
    float* dlv = d1 + NMAX * NF_;
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
    float* dce2 = d1 + 64;   // [N][32]
    float* dce1 = d1 + 256;  // [N][32]
    lin_bwd(dmu, NF_, w + L.ce2, 32, N, 32, PW(H_MU_W), NF_, GW(H_MU_W), GW(H_MU_B), dce2, 32, false);
    lin_bwd(dlv, NF_, w + L.ce2, 32, N, 32, PW(H_LV_W), NF_, GW(H_LV_W), GW(H_LV_B), dce2, 32, true);
    relu_gate(dce2, 32, w + L.ce2, 32, N, 32, 1.f);
    lin_bwd(dce2, 32, w + L.ce1, 32, N, 32, PW(H_CE2_W), 32, GW(H_CE2_W), GW(H_CE2_B), dce1, 32, false);
    relu_gate(dce1, 32, w + L.ce1, 32, N, 32, 1.f);
    float* denc = d1 + 448;  // [N][32]
    lin_bwd(dce1, 32, w + L.enc, 32, N, 32, PW(H_CE0_W), 32, GW(H_CE0_W), GW(H_CE0_B), denc, 32, false);
    // encoder: enc = We h_T + be
    lin_bwd(denc, 32, w + L.hT, GH, N, GH, PW(H_ENC_W), 32, GW(H_ENC_W), GW(H_ENC_B), w + L.dh, GH, false);
  }
  // ---- GRU backward through time
  {
    const float* Whh = PW(H_GRU_WHH);
    float* dh = w + L.dh;
    float* dhn = w + L.dtmp2 + 64;  // [N][64] next dh
    for (int t = T - 1; t >= 0; --t) {
      for (int idx = tid; idx < N * GH; idx += 256) {
        const int nn = idx / GH, u = idx - nn * GH;
        const int64_t row = (int64_t)t * NMAX + nn;
        const float r = w[L.r + row * GH + u], z = w[L.z + row * GH + u], nv = w[L.n + row * GH + u];
        const float hp = w[L.hp + row * GH + u], ghn = w[L.ghn + row * GH + u];
        const float d = dh[idx];
        const float dn = d * (1.f - z);
        const float dzg = d * (hp - nv);  // dh'/dz = h - n
        const float dan = dn * (1.f - nv * nv);
        const float dr = dan * ghn;
        const float daz = dzg * z * (1.f - z);
        const float dar = dr * r * (1.f - r);
        float* dgi = w + L.dgi + row * 3 * GH;
        float* dgh = w + L.dgh + row * 3 * GH;
        dgi[u] = dar; dgi[GH + u] = daz; dgi[2 * GH + u] = dan;
        dgh[u] = dar; dgh[GH + u] = daz; dgh[2 * GH + u] = dan * r;
        dhn[idx] = d * z;
      }
      __syncthreads();
      for (int idx = tid; idx < N * GH; idx += 256) {
        const int nn = idx / GH, j = idx - nn * GH;
        const float* dgh = w + L.dgh + ((int64_t)t * NMAX + nn) * 3 * GH;
        float s = dhn[idx];
        for (int q = 0; q < 3 * GH; ++q) s = fmaf(Whh[(int64_t)q * GH + j], dgh[q], s);
        dh[idx] = s;
      }
      __syncthreads();
    }
    // weight grads over all (t, n < N) rows; rows n >= N never ran
    float* dWih = GW(H_GRU_WIH);
    float* dWhh = GW(H_GRU_WHH);
    for (int idx = tid; idx < 3 * GH * GIN; idx += 256) {
      const int q = idx / GIN, i = idx - q * GIN;
      float s = 0.f;
      for (int t = 0; t < T; ++t)
        for (int nn = 0; nn < N; ++nn) {
          const int64_t row = (int64_t)t * NMAX + nn;
          s = fmaf(w[L.dgi + row * 3 * GH + q], w[L.x + row * GIN + i], s);
        }
      dWih[idx] += s;
    }
    for (int idx = tid; idx < 3 * GH * GH; idx += 256) {
      const int q = idx / GH, j = idx - q * GH;
      float s = 0.f;
      for (int t = 0; t < T; ++t)
        for (int nn = 0; nn < N; ++nn) {
          const int64_t row = (int64_t)t * NMAX + nn;
          s = fmaf(w[L.dgh + row * 3 * GH + q], w[L.hp + row * GH + j], s);
        }
      dWhh[idx] += s;
    }
    for (int q = tid; q < 3 * GH; q += 256) {
      float si = 0.f, sh = 0.f;
      for (int t = 0; t < T; ++t)
        for (int nn = 0; nn < N; ++nn) {
          const int64_t row = (int64_t)t * NMAX + nn;
          si += w[L.dgi + row * 3 * GH + q];
          sh += w[L.dgh + row * 3 * GH + q];
        }
      GW(H_GRU_BIH)[q] += si;
      GW(H_GRU_BHH)[q] += sh;
    }
    // d x for every real trajectory row (t, j < cnt[t])
    const float* Wih = PW(H_GRU_WIH);
    for (int idx = tid; idx < T * NMAX * GIN; idx += 256) {
      const int row = idx / GIN, i = idx - row * GIN;
      const int t = row / NMAX, j = row - t * NMAX;
      float s = 0.f;
      if (j < cnt[t]) {
        const float* dgi = w + L.dgi + (int64_t)row * 3 * GH;
        for (int q = 0; q < 3 * GH; ++q) s = fmaf(Wih[(int64_t)q * GIN + i], dgi[q], s);
      }
      w[L.dx + idx] = s;
    }
    __syncthreads();
  }
  // ---- ReID MLP backward over real rows (padding rows carry zero d x and zero inputs -> contribute 0)
  {
    const int TN = T * NMAX;
    float* dr2 = w + L.dtmp;  // [TN][64]
    float* dr1 = w + L.dtmp2; // [TN][32] (dtmp2 is free now)
    // layer 4 (no act): d pre = d x[:, 4:68] on real rows only
    for (int idx = tid; idx < TN * 64; idx += 256) {
      const int row = idx / 64, u = idx - row * 64;
      const int t = row / NMAX, j = row - t * NMAX;
      w[L.dgh + idx] = (j < cnt[t]) ? w[L.dx + (int64_t)row * GIN + 4 + u] : 0.f;  // reuse dgh as scratch
    }
    __syncthreads();
    lin_bwd(w + L.dgh, 64, w + L.rh2, 64, TN, 64, PW(H_REID4_W), 64, GW(H_REID4_W), GW(H_REID4_B), dr2, 64, false);
    relu_gate(dr2, 64, w + L.rh2, 64, TN, 64, 1.f);
    lin_bwd(dr2, 64, w + L.rh1, 32, TN, 32, PW(H_REID2_W), 64, GW(H_REID2_W), GW(H_REID2_B), dr1, 32, false);
    relu_gate(dr1, 32, w + L.rh1, 32, TN, 32, 1.f);
    // box grads: d box = d x[:, 0:4] + W0^T dr1, then into the detector logits for valid boxes
    float* dbox = w + L.dgi;  // [TN][4]
    lin_bwd(dr1, 32, w + L.boxes, 4, TN, 4, PW(H_REID0_W), 32, GW(H_REID0_W), GW(H_REID0_B), dbox, 4, false);
    for (int idx = tid; idx < TN * 4; idx += 256) {
      const int row = idx / 4, c = idx - row * 4;
      const int t = row / NMAX, j = row - t * NMAX;
      if (j >= cnt[t]) continue;
      const int k = slot[t * NMAX + j];
      if (k < 0) continue;  // fallback box is a constant
      const float dv = dbox[idx] + w[L.dx + (int64_t)row * GIN + c];
      const float lg = logits[((int64_t)b * T + t) * 20 + k * 4 + c];
      const float sg = sigmoidf_(lg);
      const float sc = c == 0 ? 360.f : (c == 1 ? 240.f : (c == 2 ? 80.f : 120.f));
      dlog[((int64_t)b * T + t) * 20 + k * 4 + c] = dv * sc * sg * (1.f - sg);
    }
  }
}

int head_bwd(const HeadArgs& a, const float* det_logits, const HeadOut& o, const HeadUp& up, float* slabs,
             int64_t slab_len, float* d_det_logits, hipStream_t st) {
  VAD_HIP(hipMemsetAsync(d_det_logits, 0, sizeof(float) * (size_t)a.B * a.T * 20, st));
  hipLaunchKernelGGL(head_bwd_kernel, dim3(a.B), dim3(256), 0, st, a, det_logits, o, up, slabs, slab_len,
                     d_det_logits);
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

// ------------------------------------------------------------------ tail: softmax, blend, losses
__global__ void cad_tail_fwd_kernel(TailArgs t) {
  const int B = t.B;
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
    if (t.flags_f) {
      t.flags_f[0] = (float)fl[0];
      t.flags_f[1] = (float)fl[1];
    }
    if (t.labels) {
      const float fB = (float)B;
      const float c = red[0][0] / fB, a = red[1][0] / fB, ca2 = red[2][0] / fB, k = red[3][0] / fB;
      t.losses[0] = c;
      t.losses[1] = a;
      t.losses[2] = ca2;
      t.losses[3] = k;
      t.losses[4] = 0.4f * c + 0.3f * a + 0.2f * ca2 + 0.1f * k;
    }
  }
}

int cad_tail_fwd(const TailArgs& t, hipStream_t st) {
  hipLaunchKernelGGL(cad_tail_fwd_kernel, dim3(1), dim3(256), 0, st, t);
  VAD_LAUNCH_CHECK();
  return 0;
}

// upstream grads: from the loss (labels) or from external autograd grads
__global__ void cad_tail_bwd_kernel(TailArgs t) {
  const int B = t.B;
  const float fB = (float)B;
  for (int b = threadIdx.x; b < B; b += 256) {
    const float p0 = t.probs[b * 2], p1 = t.probs[b * 2 + 1];
    const float c = t.causal[b], fin = t.final_scores[b];
    float d_final = 0.f, d_c = 0.f, dp0 = 0.f, dp1 = 0.f, dk = 0.f;
    if (t.labels) {
      const int y = (int)t.labels[b];
      const float yf = (float)y;
      d_final = 0.3f * 2.f * (fin - yf) / fB;
      d_c = 0.2f * 2.f * (c - yf) / fB;
      // d CE / d p = softmax(p) - onehot
      const float m2 = fmaxf(p0, p1);
      const float e0 = expf(p0 - m2), e1 = expf(p1 - m2);
      const float q0 = e0 / (e0 + e1), q1 = e1 / (e0 + e1);
      dp0 = 0.4f * (q0 - (y == 0 ? 1.f : 0.f)) / fB;
      dp1 = 0.4f * (q1 - (y == 1 ? 1.f : 0.f)) / fB;
      dk = isfinite(t.kl[b]) ? 0.1f / fB : 0.f;
    } else {
      d_final = t.ext_d_final ? t.ext_d_final[b] : 0.f;
      d_c = t.ext_d_causal ? t.ext_d_causal[b] : 0.f;
      dp0 = t.ext_d_probs ? t.ext_d_probs[b * 2] : 0.f;
      dp1 = t.ext_d_probs ? t.ext_d_probs[b * 2 + 1] : 0.f;
      dk = t.ext_d_kl ? t.ext_d_kl[b] : 0.f;
    }
    d_c += 0.6f * d_final;
    dp1 += 0.4f * d_final;
    // through softmax: dl = p * (dp - <p, dp>)
    const float dot = p0 * dp0 + p1 * dp1;
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
