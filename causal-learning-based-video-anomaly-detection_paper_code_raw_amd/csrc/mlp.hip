// The two 5-layer MLP chains of the model (detector_net cad:167-179 on every frame, direct_classifier
// cad:525-538 on the clip mean), fused so each chain costs a handful of launches instead of ~25:
//   forward   layer 0 (6144 -> 512) stays a split-K MFMA GEMM (its 12.6 MB weight needs the whole chip);
//             mlp_tail_fwd_kernel sums its partials (+bias, ReLU, dropout) and runs layers 1-4 for RB rows per
//             block with the activations in LDS (rows are independent through the chain).
//   backward  mlp_tail_bwd_kernel walks the gated input-gradient chain 4 -> 0 for RB rows per block;
//             rows_wgrad_kernel computes every layer-1..4 weight/bias gradient in one launch (f32 MFMA over the
//             rows, 32x32 tiles, bias as a ones column, fixed-order combine of the 4 waves).
// Dropout masks come from the keyed counter RNG (common.h), keyed by (stream, step, global row, column) exactly
// like the unfused EpiDense path.
#include "mlp.h"

namespace vad {

__device__ __forceinline__ float mlp_finish(const MlpLayer& L, int64_t grow, int col, float v) {
  v += L.b[col];
  if (L.relu) v = relu_nan(v);  // (NaN kept, as dense_finish)
  if (L.drop) v = (rng_u24(L.h1, (uint64_t)grow, (uint64_t)col) >= L.thr) ? v * L.dscale : 0.f;
  return v;
}

// layers 1-4 for RB rows; h0 (layer-0 output, finished by the split-K reduce) is read from global.  Thread t of a
// layer owns 4 consecutive outputs g = t % (N/4) over the K-slice p = t / (N/4): float4 loads of the transposed
// weight WT[k][4g..4g+3] (coalesced across g), 8 in flight; the K-slices are combined in a fixed order in LDS.
// NTH = 1024 (knob mlp_tail_wide) gives each layer 4x the K-slices of 256; measured no faster, so 256 is the default.
template <int RB, int NTH>
__global__ __launch_bounds__(NTH) void mlp_tail_fwd_kernel(const MlpTailArgs a) {
  __shared__ __attribute__((aligned(16))) float buf[2][RB][MLP_MAXW];
  __shared__ __attribute__((aligned(16))) float red[NTH * 4 * RB];
  const int tid = threadIdx.x;
  const int r0 = blockIdx.x * RB;
  {
    const int N = a.L[0].N;
    // (loads from clamped addresses, zeroed after: predicated loads would be issued one round trip apart)
    constexpr int PER = (RB * MLP_MAXW + NTH - 1) / NTH;
    float v[PER];
    if (a.parts) {
      // layer 0's split-K partials summed in split order (as dense_splitk_reduce_kernel), ZC splits per batch of loads
      // (32 loads in flight per thread)
      constexpr int ZC = PER >= 8 ? 4 : 32 / PER;
#pragma unroll
      for (int u = 0; u < PER; ++u) v[u] = 0.f;
      for (int z0 = 0; z0 < a.nsplit; z0 += ZC) {
        float pv[ZC][PER];
#pragma unroll
        for (int zz = 0; zz < ZC; ++zz)
#pragma unroll
          for (int u = 0; u < PER; ++u) {
            const int idx = min(tid + u * NTH, RB * N - 1), r = idx / N, n = idx % N;
            pv[zz][u] = a.parts[((int64_t)min(z0 + zz, a.nsplit - 1) * a.M + min(r0 + r, a.M - 1)) * N + n];
          }
#pragma unroll
        for (int zz = 0; zz < ZC; ++zz)
#pragma unroll
          for (int u = 0; u < PER; ++u)
            if (z0 + zz < a.nsplit) v[u] += pv[zz][u];
      }
#pragma unroll
      for (int u = 0; u < PER; ++u) {
        const int idx = tid + u * NTH, r = idx / N, n = idx % N;
        if (idx < RB * N && r0 + r < a.M) {
          v[u] = mlp_finish(a.L[0], a.row0 + r0 + r, n, v[u]);
          a.L[0].out[(int64_t)(r0 + r) * N + n] = v[u];
        }
      }
    } else {
#pragma unroll
      for (int u = 0; u < PER; ++u) {
        const int idx = min(tid + u * NTH, RB * N - 1), r = idx / N, n = idx % N;
        v[u] = a.L[0].out[(int64_t)min(r0 + r, a.M - 1) * N + n];
      }
    }
#pragma unroll
    for (int u = 0; u < PER; ++u) {
      const int idx = tid + u * NTH, r = idx / N, n = idx % N;
      if (idx < RB * N) buf[0][r][n] = r0 + r < a.M ? v[u] : 0.f;
    }
  }
  __syncthreads();
#pragma unroll 1
  for (int i = 1; i < 5; ++i) {
    const MlpLayer& L = a.L[i];
    const float(*in)[MLP_MAXW] = buf[(i - 1) & 1];
    float(*outb)[MLP_MAXW] = buf[i & 1];
    const int K = L.K, N = L.N, NG = N / 4;
    // K-slices of >= 8 inputs only (the combine below reads P partials per output: idle slices would cost reads)
    const int P = min(NTH / NG, max(1, K / 8));
    const int kper = ((K + P - 1) / P + 7) & ~7;
    const float* WT = a.WT[i];
    if (tid < NG * P) {
      const int g = tid % NG, p = tid / NG;
      const int k0 = p * kper, k1 = min(K, k0 + kper);
      f32x4 acc[RB];
#pragma unroll
      for (int r = 0; r < RB; ++r) acc[r] = f32x4{0.f, 0.f, 0.f, 0.f};
      for (int kb = k0; kb < k1; kb += 8) {  // K and kper are multiples of 8
        f32x4 wv[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) wv[u] = *reinterpret_cast<const f32x4*>(WT + (int64_t)(kb + u) * N + 4 * g);
#pragma unroll
        for (int u = 0; u < 8; ++u)
#pragma unroll
          for (int r = 0; r < RB; ++r) {
            const float x = in[r][kb + u];
            acc[r][0] = fmaf(wv[u][0], x, acc[r][0]);
            acc[r][1] = fmaf(wv[u][1], x, acc[r][1]);
            acc[r][2] = fmaf(wv[u][2], x, acc[r][2]);
            acc[r][3] = fmaf(wv[u][3], x, acc[r][3]);
          }
      }
#pragma unroll
      for (int r = 0; r < RB; ++r) *reinterpret_cast<f32x4*>(&red[(p * RB + r) * N + 4 * g]) = acc[r];
    }
    __syncthreads();
    for (int idx = tid; idx < RB * N; idx += NTH) {
      const int r = idx / N, n = idx % N, row = r0 + r;
      float sum = 0.f;
      for (int p = 0; p < P; ++p) sum += red[(p * RB + r) * N + n];
      float v = 0.f;
      if (row < a.M) {
        v = mlp_finish(L, a.row0 + row, n, sum);
        L.out[(int64_t)row * N + n] = v;
      }
      outb[r][n] = v;
    }
    __syncthreads();
  }
}

// WT[k][n] = W[n][k] for up to 8 matrices (the detector's layer-1..4 weights), once per step: 32x32 tiles through
// LDS so both the read of W rows and the write of WT rows are coalesced.
__global__ __launch_bounds__(256) void mlp_transpose_kernel(const MlpTransposeArgs a) {
  __shared__ float tile[32][33];
  int m = 0, t = blockIdx.x;
  for (; m < a.n; ++m) {
    const int nt = ((a.N[m] + 31) / 32) * ((a.K[m] + 31) / 32);
    if (t < nt) break;
    t -= nt;
  }
  if (m >= a.n) return;
  const int K = a.K[m], N = a.N[m], tk = (K + 31) / 32;
  const int n0 = (t / tk) * 32, k0 = (t % tk) * 32;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;  // 32 x 8
#pragma unroll
  for (int j = 0; j < 32; j += 8) {
    const int n = n0 + ty + j, k = k0 + tx;
    tile[ty + j][tx] = (n < N && k < K) ? a.W[m][(int64_t)n * K + k] : 0.f;
  }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < 32; j += 8) {
    const int k = k0 + ty + j, n = n0 + tx;
    if (k < K && n < N) a.WT[m][(int64_t)k * N + n] = tile[tx][ty + j];
  }
}

int mlp_transpose(const MlpTransposeArgs& a, hipStream_t st) {
  int blocks = 0;
  for (int m = 0; m < a.n; ++m) blocks += (int)(cdiv(a.N[m], 32) * cdiv(a.K[m], 32));
  hipLaunchKernelGGL(mlp_transpose_kernel, dim3(blocks), dim3(256), 0, st, a);
  VAD_LAUNCH_CHECK();
  return 0;
}

// d_{i-1}[r][k] = (sum_n d_i[r][n] W_i[n][k]) * (h_{i-1}[r][k] > 0 ? gscale_{i-1} : 0),  i = 4 .. 1
template <int RB>
__global__ __launch_bounds__(256) void mlp_tail_bwd_kernel(const MlpTailBwdArgs a) {
  if (a.skip && *a.skip == 0) return;
  __shared__ __attribute__((aligned(16))) float buf[2][RB][MLP_MAXW];
  const int tid = threadIdx.x;
  const int r0 = blockIdx.x * RB;
  {
    const int N = a.N[4], N4 = (N + 3) & ~3;  // zero-filled to the 4-wide n-batches below
    for (int idx = tid; idx < RB * N4; idx += 256) {
      const int r = idx / N4, n = idx % N4, row = r0 + r;
      buf[0][r][n] = (row < a.M && n < N) ? a.dout[(int64_t)row * N + n] : 0.f;
    }
  }
  __syncthreads();
#pragma unroll 1
  for (int i = 4; i >= 1; --i) {
    const float(*din)[MLP_MAXW] = buf[(4 - i) & 1];
    float(*dout)[MLP_MAXW] = buf[(5 - i) & 1];
    const float* W = a.W[i];
    const int K = a.K[i], N = a.N[i];
    const float* gate = a.h[i - 1];
    const float gs = a.gscale[i - 1];
    float* dst = a.d[i - 1];
    for (int k = tid; k < K; k += 256) {
      float acc[RB];
#pragma unroll
      for (int r = 0; r < RB; ++r) acc[r] = 0.f;
      for (int n0 = 0; n0 < N; n0 += 4) {  // 4 coalesced weight loads in flight per batch
        float wv[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) wv[u] = n0 + u < N ? W[(int64_t)(n0 + u) * K + k] : 0.f;
#pragma unroll
        for (int u = 0; u < 4; ++u)
#pragma unroll
          for (int r = 0; r < RB; ++r) acc[r] = fmaf(din[r][n0 + u], wv[u], acc[r]);
      }
#pragma unroll
      for (int r = 0; r < RB; ++r) {
        const int row = r0 + r;
        float v = 0.f;
        if (row < a.M) {
          v = gate[(int64_t)row * K + k] > 0.f ? acc[r] * gs : 0.f;
          dst[(int64_t)row * K + k] = v;
        }
        dout[r][k] = v;
      }
    }
    __syncthreads();
  }
}

// ------------------------------------------------------------------ generic row-reduction weight gradients
__global__ __launch_bounds__(256) void rows_wgrad_kernel(const RowsWgradArgs a) {
  if (a.skip && *a.skip == 0) return;
  int s = 0, t = blockIdx.x;
  for (; s < a.nseg; ++s) {
    const int n = ((a.seg[s].O + 31) / 32) * ((a.seg[s].I + 1 + 31) / 32);
    if (t < n) break;
    t -= n;
  }
  if (s >= a.nseg) return;
  const RowsWgradSeg sg = a.seg[s];
  const int ti = (sg.I + 1 + 31) / 32;
  const int o0 = (t / ti) * 32, i0 = (t % ti) * 32;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, h = lane >> 5, l = lane & 31;
  const int o = o0 + l, i = i0 + l;
  f32x16 acc;
#pragma unroll
  for (int r = 0; r < 16; ++r) acc[r] = 0.f;
  const int R = a.R;
  const int per = (R + 3) / 4;
  const int r0 = wave * per, r1 = min(R, r0 + per);
  // wave-uniform trip count; row rb + 2u + h, zero past the share.  8 row pairs per batch: every load of the batch is
  // issued before its MFMAs (one load pair per MFMA left each MFMA waiting on an L2 round trip: the 640-row GRU / ReID
  // segments took 65 us); the MFMAs run in the same row order as one pair at a time (bit-identical)
  for (int rb = r0; rb < r1; rb += 16) {
    float av[8], xv[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int r = rb + 2 * u + h;
      const bool ok = r < r1;
      av[u] = (ok && o < sg.O) ? sg.A[(int64_t)r * sg.O + o] : 0.f;
      xv[u] = !ok ? 0.f : (i < sg.I ? sg.X[(int64_t)r * sg.I + i] : (i == sg.I ? 1.f : 0.f));
    }
#pragma unroll
    for (int u = 0; u < 8; ++u)
      if (rb + 2 * u < r1) acc = mfma32(av[u], xv[u], acc);
  }
  __shared__ float red[4][16][64];
#pragma unroll
  for (int r = 0; r < 16; ++r) red[wave][r][lane] = acc[r];
  __syncthreads();
  if (wave == 0) {
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const float v = (red[0][r][lane] + red[1][r][lane]) + (red[2][r][lane] + red[3][r][lane]);
      const int oo = o0 + (r & 3) + 8 * (r >> 2) + 4 * h, ii = i0 + l;
      if (oo < sg.O) {
        if (ii < sg.I) sg.dW[(int64_t)oo * sg.I + ii] = v;
        else if (ii == sg.I && sg.db) sg.db[oo] = v;
      }
    }
  }
}

int rows_wgrad(const RowsWgradArgs& a, hipStream_t st) {
  VAD_CHECK(a.nseg >= 1 && a.nseg <= ROWS_WGRAD_MAXSEG, "rows_wgrad: bad segment count");
  int blocks = 0;
  for (int s = 0; s < a.nseg; ++s) blocks += (int)(cdiv(a.seg[s].O, 32) * cdiv(a.seg[s].I + 1, 32));
  hipLaunchKernelGGL(rows_wgrad_kernel, dim3(blocks), dim3(256), 0, st, a);
  VAD_LAUNCH_CHECK();
  return 0;
}

// ------------------------------------------------------------------ direct classifier: affine loss-mode backward
// dst = lane bit set in mask ? a : b, as one v_cndmask with a constant lane mask (written as inline asm: a plain select
// between two elements of the unrolled array is rewritten by the compiler into a dynamically indexed vector extract,
// i.e. a compare/select chain over the whole array)
__device__ __forceinline__ float lane_sel(float a, float b, unsigned long long mask) {
  float r;
  asm("v_cndmask_b32_e64 %0, %1, %2, %3" : "=v"(r) : "v"(b), "v"(a), "s"(mask));
  return r;
}
constexpr int ilog2(int v) { return v <= 1 ? 0 : 1 + ilog2(v / 2); }
// Sums V per-lane values over each aligned group of 2^LGP lanes at once (V a power of two <= 2^LGP): a reduce-scatter
// over lane bits 0 .. log2 V - 1 (the lane with bit s set keeps the upper half of the remaining values and sends the
// lower half), then a butterfly over the remaining group bits -- V - 1 + LGP - log2 V shuffles for V sums.  Lane l
// returns the group total of value rs_index<V>(l).
template <int V, int LGP>
__device__ __forceinline__ float group_rs(float (&v)[V]) {
  constexpr int LV = ilog2(V);
  static_assert((1 << LV) == V && LV <= LGP && LGP <= 6, "power-of-two values within the lane group");
  constexpr unsigned long long up_mask[6] = {0xAAAAAAAAAAAAAAAAull, 0xCCCCCCCCCCCCCCCCull, 0xF0F0F0F0F0F0F0F0ull,
                                             0xFF00FF00FF00FF00ull, 0xFFFF0000FFFF0000ull, 0xFFFFFFFF00000000ull};
#pragma unroll
  for (int s = 0; s < LV; ++s) {
    const int half = V >> (s + 1);
#pragma unroll
    for (int i = 0; i < half; ++i) {
      const float keep = lane_sel(v[i + half], v[i], up_mask[s]);
      const float send = lane_sel(v[i], v[i + half], up_mask[s]);
      v[i] = keep + __shfl_xor(send, 1 << s, 64);
    }
  }
  float x = v[0];
#pragma unroll
  for (int b = LV; b < LGP; ++b) x += __shfl_xor(x, 1 << b, 64);
  return x;
}
template <int V>
__device__ __forceinline__ int rs_index(int l) {
  int r = 0;
#pragma unroll
  for (int s = 0; (V >> (s + 1)) >= 1; ++s) r |= ((l >> s) & 1) * (V >> (s + 1));
  return r;
}

// out[r][o] = act(b[o] + sum_i W[o][i] in[r][i]) for RB rows (LDS in / out, rows >= B zero).  Thread (output group g
// of OG outputs, K-slice p of I / P inputs; p fastest, so a group's P lanes read consecutive chunks of the W rows):
// RB x OG partial dots, summed over the group's lanes by group_rs (one value per lane, no LDS combine)
template <int RB, int I, int O, int OG, int P, bool RELU>
__device__ __forceinline__ void dir_layer_fwd(const float* __restrict__ W, const float* __restrict__ bias,
                                              const float (*in)[I], float (*out)[O], float* gout, int B) {
  constexpr int KPER = I / P, NG = O / OG, V = RB * OG;
  static_assert(KPER % 4 == 0 && KPER * P == I && NG * OG == O && NG * P <= 1024 && V <= P && 64 % P == 0,
                "layer tiling");
  const int p = threadIdx.x % P, g = threadIdx.x / P;
  if (g >= NG) return;  // (whole lane groups)
  f32x4 w[OG][KPER / 4];
#pragma unroll
  for (int c = 0; c < OG; ++c)
#pragma unroll
    for (int kk = 0; kk < KPER / 4; ++kk)
      w[c][kk] = *reinterpret_cast<const f32x4*>(W + (int64_t)(g * OG + c) * I + p * KPER + 4 * kk);
  float v[V];
#pragma unroll
  for (int r = 0; r < RB; ++r) {
#pragma unroll
    for (int c = 0; c < OG; ++c) v[r * OG + c] = 0.f;
#pragma unroll
    for (int kk = 0; kk < KPER / 4; ++kk) {
      const f32x4 x = *reinterpret_cast<const f32x4*>(&in[r][p * KPER + 4 * kk]);
#pragma unroll
      for (int c = 0; c < OG; ++c)
        v[r * OG + c] = fmaf(w[c][kk][3], x[3], fmaf(w[c][kk][2], x[2], fmaf(w[c][kk][1], x[1],
                        fmaf(w[c][kk][0], x[0], v[r * OG + c]))));
    }
  }
  const float sum = group_rs<V, ilog2(P)>(v);
  if (p < V) {
    const int idx = rs_index<V>(p), r = idx / OG, o = g * OG + idx % OG;
    float y = sum + bias[o];
    if (RELU) y = relu_nan(y);
    if (r >= B) y = 0.f;
    out[r][o] = y;
    if (r < B && gout) gout[(int64_t)r * O + o] = y;
  }
}

// din[r][i] = (sum_o W[o][i] dout[r][o]) * (gate[r % B][i] > 0 ? gs : 0) for R2 stacked rows (rows >= 2B zero):
// thread (i, slice) accumulates its slice of o (coalesced W row reads, batches of up to 32 loads), the S slices are
// combined in a fixed order through red
// (LD > I: the block computes the columns [i0, i0 + I) of rows LD wide; W rows and gate rows are LD wide, din / gdin
// are written at their full-width positions)
template <int R2, int I, int O, int LD = I>
__device__ __forceinline__ void dir_layer_bwd(const float* __restrict__ W, const float (*dout)[O],
                                              const float (*gate)[LD], float gs, float (*din)[LD], float* gdin, int B,
                                              float* red, int i0 = 0) {
  constexpr int S = 1024 / I, OPS = (O + S - 1) / S, UB = OPS < 32 ? OPS : 32;
  const int i = threadIdx.x % I, sl = threadIdx.x / I;
  W += i0;
  const int o0 = sl * OPS;
  float acc[R2];
  if constexpr (OPS % 4 == 0 && S * OPS == O) {
    // packed: even / odd o in the two halves of a v_pk_fma_f32, dout read as float4 (4 o per LDS broadcast)
    f32x2 acc2[R2];
#pragma unroll
    for (int r = 0; r < R2; ++r) acc2[r] = f32x2{0.f, 0.f};
#pragma unroll
    for (int ob = 0; ob < OPS; ob += UB) {
      float w[UB];  // (unconditional loads, issued together)
#pragma unroll
      for (int u = 0; u < UB; ++u) w[u] = W[(int64_t)(o0 + ob + u) * LD + i];
      // row by row: the row's UB / 4 float4 reads are issued together, then its 2 x UB / 4 packed FMAs (the u-outer
      // order waited for each read before its two FMAs)
#pragma unroll
      for (int r = 0; r < R2; ++r) {
        f32x4 d[UB / 4];
#pragma unroll
        for (int q = 0; q < UB / 4; ++q) d[q] = *reinterpret_cast<const f32x4*>(&dout[r][o0 + ob + 4 * q]);
#pragma unroll
        for (int q = 0; q < UB / 4; ++q) {
          acc2[r] = __builtin_elementwise_fma(f32x2{w[4 * q], w[4 * q + 1]}, f32x2{d[q][0], d[q][1]}, acc2[r]);
          acc2[r] = __builtin_elementwise_fma(f32x2{w[4 * q + 2], w[4 * q + 3]}, f32x2{d[q][2], d[q][3]}, acc2[r]);
        }
      }
    }
#pragma unroll
    for (int r = 0; r < R2; ++r) acc[r] = acc2[r][0] + acc2[r][1];
  } else {
#pragma unroll
    for (int r = 0; r < R2; ++r) acc[r] = 0.f;
#pragma unroll
    for (int ob = 0; ob < OPS; ob += UB) {
      float w[UB];  // (clamped rows: unconditional loads, issued together)
#pragma unroll
      for (int u = 0; u < UB; ++u) w[u] = W[(int64_t)min(o0 + ob + u, O - 1) * LD + i];
#pragma unroll
      for (int u = 0; u < UB; ++u) {
        if (o0 + ob + u >= O) break;
#pragma unroll
        for (int r = 0; r < R2; ++r) acc[r] = fmaf(w[u], dout[r][o0 + ob + u], acc[r]);
      }
    }
  }
#pragma unroll
  for (int r = 0; r < R2; ++r) red[(sl * R2 + r) * I + i] = acc[r];
  __syncthreads();
  for (int q = threadIdx.x; q < R2 * I; q += 1024) {
    const int r = q / I, ii = q % I;
    float v = 0.f;
    for (int t = 0; t < S; ++t) v += red[(t * R2 + r) * I + ii];
    v = (r < 2 * B && gate[r % B][i0 + ii] > 0.f) ? v * gs : 0.f;
    if (din) din[r][i0 + ii] = v;
    if (r < 2 * B && gdin) gdin[(int64_t)r * LD + i0 + ii] = v;
  }
  __syncthreads();
}

template <int RB>
__global__ __launch_bounds__(1024) void dir_mid_kernel(const DirMidArgs a) {
  static_assert(RB * 256 == 2 * 1024, "layer-1 / layer-0 rows staged as two / four loads per thread");
  constexpr int R2 = 2 * RB;
  __shared__ __attribute__((aligned(16))) float in0[RB][512];  // layer 0 output: the layer-1 input gradient's gate
  __shared__ __attribute__((aligned(16))) float in1[RB][256];
  __shared__ __attribute__((aligned(16))) float dd1[R2][256];
  __shared__ __attribute__((aligned(16))) float a2[RB][128];
  __shared__ __attribute__((aligned(16))) float a3[RB][64];
  __shared__ __attribute__((aligned(16))) float lg[RB][2];
  __shared__ __attribute__((aligned(16))) float dl[R2][2];
  __shared__ __attribute__((aligned(16))) float dd3[R2][64];
  __shared__ __attribute__((aligned(16))) float dd2[R2][128];
  __shared__ __attribute__((aligned(16))) float red[4 * R2 * 256];  // (= 2 x R2 x 512: the layer-1 combine too)
  const int B = a.B, tid = threadIdx.x;
  // every block runs layers 2-4, the seed and the layer 4-2 input gradients (cheap, redundant); block k then takes the
  // layer-1 input-gradient columns [64k, 64k + 64).  Block 0 alone writes the shared outputs.
  const bool w0 = blockIdx.x == 0;
  {
    float v[2];  // RB * 256 = 2048 = 2 x 1024 (clamped loads, zeroed after)
#pragma unroll
    for (int u = 0; u < 2; ++u) v[u] = a.h1[min(tid + u * 1024, B * 256 - 1)];
    float v0[4];  // RB * 512 = 4 x 1024
#pragma unroll
    for (int u = 0; u < 4; ++u) v0[u] = a.h0[min(tid + u * 1024, B * 512 - 1)];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int q = tid + u * 1024;
      in1[q / 256][q % 256] = q / 256 < B ? v[u] : 0.f;
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int q = tid + u * 1024;
      in0[q / 512][q % 512] = q / 512 < B ? v0[u] : 0.f;
    }
  }
  __syncthreads();
  dir_layer_fwd<RB, 256, 128, 4, 32, true>(a.W2, a.b2, in1, a2, w0 ? a.h2 : nullptr, B);
  __syncthreads();
  dir_layer_fwd<RB, 128, 64, 2, 32, true>(a.W3, a.b3, a2, a3, w0 ? a.h3 : nullptr, B);
  __syncthreads();
  dir_layer_fwd<RB, 64, 2, 2, 16, false>(a.W4, a.b4, a3, lg, w0 ? a.logits : nullptr, B);
  __syncthreads();
  // seed rows: softmax, cross entropy on the probabilities (cad:673) and the c-free / c-linear parts of the anomaly
  // MSE through fin (cad:674), then the softmax backward -- the per-row arithmetic of cad_tail_bwd_kernel
  if (tid < R2) {
    float d0 = 0.f, d1 = 0.f;
    const int b = tid % RB;
    if (b < B && (tid < RB || tid - RB < B)) {
      const bool beta = tid >= RB;
      const float fB = (float)B;
      const float l0 = lg[b][0], l1 = lg[b][1];
      const float mx = fmaxf(l0, l1);
      const float e0 = expf(l0 - mx), e1 = expf(l1 - mx);
      const float p0 = e0 / (e0 + e1), p1 = e1 / (e0 + e1);
      const int y = (int)a.labels[b];
      const float yf = (float)y;
      float dp0, dp1;
      const float k = 0.4f * (0.3f * 2.f / fB);  // d fin / d p1 * d loss / d fin per unit (fin - y)
      if (!beta) {
        const float m2 = fmaxf(p0, p1);
        const float q0e = expf(p0 - m2), q1e = expf(p1 - m2);
        const float q0 = q0e / (q0e + q1e), q1 = q1e / (q0e + q1e);
        dp0 = 0.4f * (q0 - (y == 0 ? 1.f : 0.f)) / fB;
        dp1 = 0.4f * (q1 - (y == 1 ? 1.f : 0.f)) / fB + k * (0.4f * p1 - yf);
      } else {
        dp0 = 0.f;
        dp1 = k * 0.6f;
      }
      const float dot = p0 * dp0 + p1 * dp1;
      d0 = p0 * (dp0 - dot);
      d1 = p1 * (dp1 - dot);
    }
    // stacked row index: A rows 0 .. B-1, beta rows B .. 2B-1 (then zero rows)
    const int r = tid < RB ? tid : B + (tid - RB);
    if (tid < RB ? tid < B : tid - RB < B) {
      dl[r][0] = d0;
      dl[r][1] = d1;
      if (w0) {
        a.dl2[r * 2] = d0;
        a.dl2[r * 2 + 1] = d1;
      }
    }
  }
  if (tid >= R2 && tid < 2 * R2) {  // zero rows 2B .. R2-1
    const int r = tid - R2;
    if (r >= 2 * B) dl[r][0] = dl[r][1] = 0.f;
  }
  __syncthreads();
  dir_layer_bwd<R2, 64, 2>(a.W4, dl, a3, 1.f, dd3, w0 ? a.d3 : nullptr, B, red);
  dir_layer_bwd<R2, 128, 64>(a.W3, dd3, a2, 1.f, dd2, w0 ? a.d2 : nullptr, B, red);
  dir_layer_bwd<R2, 256, 128>(a.W2, dd2, in1, a.gs1, dd1, w0 ? a.d1 : nullptr, B, red);
  dir_layer_bwd<R2, 64, 256, 512>(a.W1, dd1, in0, a.gs0, nullptr, a.d0, B, red, 64 * (int)blockIdx.x);
}

int dir_mid(const DirMidArgs& a, hipStream_t st) {
  // (16 stacked rows: the slice-combine buffer of the layer-2 input gradient, 4 x 16 x 256 floats, fills 64 KB of LDS)
  VAD_CHECK(a.B >= 1 && a.B <= 8, "dir_mid: 1 <= B <= 8");
  VAD_KLAUNCH(dir_mid_kernel<8>, dim3(512 / 64), dim3(1024), 0, st, a);
  VAD_LAUNCH_CHECK();
  return 0;
}

__global__ __launch_bounds__(256) void dir_combine_kernel(const DirCombineArgs a) {
  int s = 0, q = blockIdx.x * 256 + threadIdx.x;
  for (; s < a.nseg; ++s) {
    const int n = a.B * a.width[s];
    if (q < n) break;
    q -= n;
  }
  if (s >= a.nseg) return;
  const int w = a.width[s], b = q / w, k = q % w;
  a.dst[s][q] = fmaf(a.c[b], a.src[s][(int64_t)(a.B + b) * w + k], a.src[s][q]);
}

int dir_combine(const DirCombineArgs& a, hipStream_t st) {
  VAD_CHECK(a.nseg >= 1 && a.nseg <= 6, "dir_combine: segments");
  int64_t n = 0;
  for (int s = 0; s < a.nseg; ++s) n += (int64_t)a.B * a.width[s];
  hipLaunchKernelGGL(dir_combine_kernel, dim3((unsigned)cdiv(n, 256)), dim3(256), 0, st, a);
  VAD_LAUNCH_CHECK();
  return 0;
}

static int mlp_rb(int M) { return M >= 64 ? 4 : 8; }

int g_mlp_tail_rb = 0;  // knob "mlp_tail_rb": rows per block of the detector's layers 1-4 (0: auto)
int g_mlp_tail_wide = 1;  // knob "mlp_tail_wide": 1024-thread blocks for the detector's layers 1-4 (4 x the K-slices
                          // and split-K loads in flight of 256 threads; profiles/r03_mlp_tail_sweep.txt)

int mlp_tail_fwd(const MlpTailArgs& a, hipStream_t st) {
  for (int i = 1; i < 5; ++i)
    VAD_CHECK(a.L[i].N <= MLP_MAXW && a.L[i].N % 4 == 0 && a.L[i].N / 4 <= 256 && a.L[i].K <= MLP_MAXW &&
                  a.L[i].K % 8 == 0 && a.WT[i],
              "mlp_tail_fwd: layer shape");
  const int rb = g_mlp_tail_rb ? g_mlp_tail_rb : mlp_rb(a.M);
  VAD_CHECK(rb == 2 || rb == 4 || rb == 8, "mlp_tail_fwd: rows per block 2, 4 or 8");
  if (rb == 2 && g_mlp_tail_wide)
    VAD_KLAUNCH((mlp_tail_fwd_kernel<2, 1024>), dim3((unsigned)cdiv(a.M, 2)), dim3(1024), 0, st, a);
  else if (rb == 2)
    VAD_KLAUNCH((mlp_tail_fwd_kernel<2, 256>), dim3((unsigned)cdiv(a.M, 2)), dim3(256), 0, st, a);
  else if (rb == 4 && g_mlp_tail_wide)
    VAD_KLAUNCH((mlp_tail_fwd_kernel<4, 1024>), dim3((unsigned)cdiv(a.M, 4)), dim3(1024), 0, st, a);
  else if (rb == 4)
    VAD_KLAUNCH((mlp_tail_fwd_kernel<4, 256>), dim3((unsigned)cdiv(a.M, 4)), dim3(256), 0, st, a);
  else
    VAD_KLAUNCH((mlp_tail_fwd_kernel<8, 256>), dim3((unsigned)cdiv(a.M, 8)), dim3(256), 0, st, a);
  VAD_LAUNCH_CHECK();
  return 0;
}

int mlp_tail_bwd(const MlpTailBwdArgs& a, hipStream_t st) {
  for (int i = 1; i < 5; ++i) VAD_CHECK(a.K[i] <= MLP_MAXW && a.N[i] <= MLP_MAXW, "mlp_tail_bwd: layer width");
  const int rb = mlp_rb(a.M);
  if (rb == 4)
    hipLaunchKernelGGL(mlp_tail_bwd_kernel<4>, dim3((unsigned)cdiv(a.M, 4)), dim3(256), 0, st, a);
  else
    hipLaunchKernelGGL(mlp_tail_bwd_kernel<8>, dim3((unsigned)cdiv(a.M, 8)), dim3(256), 0, st, a);
  VAD_LAUNCH_CHECK();
  return 0;
}

}  // namespace vad
