// Shared device/host helpers for libvadhip (gfx950 / CDNA4 only).
#pragma once
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string>

typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

namespace vad {

// ---------------------------------------------------------------- errors
void set_error(const std::string& msg);
const char* last_error();

#define VAD_HIP(expr)                                                                     \
  do {                                                                                    \
    hipError_t _e = (expr);                                                               \
    if (_e != hipSuccess) {                                                               \
      ::vad::set_error(std::string(#expr) + ": " + hipGetErrorString(_e) + " @" __FILE__ \
                       ":" + std::to_string(__LINE__));                                   \
      return 2;                                                                           \
    }                                                                                     \
  } while (0)

#define VAD_CHECK(cond, msg)                 \
  do {                                       \
    if (!(cond)) {                           \
      ::vad::set_error(std::string(msg));    \
      return 1;                              \
    }                                        \
  } while (0)

#define VAD_LAUNCH_CHECK() VAD_HIP(hipGetLastError())

// Kernel-timing hook for live roofline measurement: when armed, the next VAD_KLAUNCH (the conv kernels) is
// dispatched with hipExtLaunchKernel's start/stop events, which take their timestamps from the dispatch itself
// (no marker packets between kernels, unlike hipEventRecord around the launch).
struct KTimer {
  hipEvent_t a = nullptr, b = nullptr;
};
KTimer& ktimer();
#define VAD_KLAUNCH(kernel, grid, block, shm, st, ...)                                                       \
  do {                                                                                                     \
    ::vad::KTimer& _kt = ::vad::ktimer();                                                                   \
    if (_kt.a) {                                                                                           \
      hipExtLaunchKernelGGL(kernel, grid, block, shm, st, _kt.a, _kt.b, 0, __VA_ARGS__);                   \
      _kt.a = _kt.b = nullptr;                                                                             \
    } else {                                                                                               \
      hipLaunchKernelGGL(kernel, grid, block, shm, st, __VA_ARGS__);                                       \
    }                                                                                                      \
  } while (0)

#define VAD_TRY(expr)        \
  do {                       \
    int _rc = (expr);        \
    if (_rc != 0) return _rc; \
  } while (0)

static inline int64_t cdiv(int64_t a, int64_t b) { return (a + b - 1) / b; }

// ---------------------------------------------------------------- RNG
// Keyed counter hash; bit-exact twin of oracle/rng.py (see its docstring for the contract).
enum RngStream : uint32_t {
  S_INPUT = 1,
  S_DET_DROP1 = 2,
  S_DET_DROP2 = 3,
  S_EPS = 4,
  S_SCORER_DROP = 5,
  S_DIRECT_DROP1 = 6,
  S_DIRECT_DROP2 = 7,
  S_MC_DROP1 = 8,
  S_MC_DROP2 = 9,
  S_A2_DROP_FC = 10,
  S_A2_DROP_GRAPH = 11,
  S_A2_PSEUDO = 12,
  S_BBOX_DROP = 13,
};

__host__ __device__ inline uint64_t mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

// h1 depends only on (seed, stream, step): computed on the host once per launch.
__host__ __device__ inline uint64_t rng_h1(uint64_t seed, uint32_t stream, uint64_t step) {
  uint64_t h0 = mix64(seed + 0x9E3779B97F4A7C15ull * (uint64_t)(stream + 1));
  return mix64(h0 ^ step);
}

__host__ __device__ inline uint64_t rng_hash(uint64_t h1, uint64_t row, uint64_t col) {
  return mix64(h1 ^ ((row << 32) | col));
}

__host__ __device__ inline uint32_t rng_u24(uint64_t h1, uint64_t row, uint64_t col) {
  return (uint32_t)(rng_hash(h1, row, col) >> 40);
}

// dropout: keep iff u24 >= thr, thr = floor(p * 2^24)
static inline uint32_t drop_threshold(double p) { return (uint32_t)(p * 16777216.0); }

__device__ inline float rng_normal(uint64_t h1, uint64_t row, uint64_t idx) {
  double u1 = ((double)rng_u24(h1, row, 2 * idx) + 1.0) / 16777216.0;
  double u2 = (double)rng_u24(h1, row, 2 * idx + 1) / 16777216.0;
  return (float)(sqrt(-2.0 * log(u1)) * cos(6.283185307179586 * u2));
}

// ---------------------------------------------------------------- device math
__device__ inline float sigmoidf_(float x) { return 1.0f / (1.0f + expf(-x)); }
// gate nonlinearities of the GRU recurrences: hardware exp2 and reciprocal (v_exp_f32 / v_rcp_f32, ~1 ulp each)
// instead of the correctly rounded library forms (division: ~10 instructions) -- absolute error < 2e-7, both
// saturate cleanly (exp -> inf gives 0 / +-1)
__device__ inline float gate_sigmoid(float x) { return __builtin_amdgcn_rcpf(1.0f + __expf(-x)); }
__device__ inline float gate_tanh(float x) { return 1.0f - 2.0f * __builtin_amdgcn_rcpf(1.0f + __expf(2.0f * x)); }

// ---------------------------------------------------------------- activation storage
// Backbone activations (raw conv outputs, the pooled stem map) and their gradients are fp32, or bf16 in plans that
// run the convs on bf16 operands (config 4, CadPlan option conv_bf16): AB selects the element type. Loads keep the
// raw element vector (act_raw4) until the value is needed, so a prefetch is not waited for at the load.
typedef __bf16 bf16x4_t __attribute__((ext_vector_type(4)));
template <bool AB>
struct ActT {
  using T = float;
  using R4 = f32x4;
};
template <>
struct ActT<true> {
  using T = __bf16;
  using R4 = bf16x4_t;
};
template <bool AB>
using act_t = typename ActT<AB>::T;
template <bool AB>
using act_raw4 = typename ActT<AB>::R4;
__device__ inline f32x4 act_f4(f32x4 v) { return v; }
__device__ inline f32x4 act_f4(bf16x4_t v) { return f32x4{(float)v[0], (float)v[1], (float)v[2], (float)v[3]}; }
template <typename T>
__device__ inline typename ActT<sizeof(T) == 2>::R4 act_ld4(const T* p) {
  return *reinterpret_cast<const typename ActT<sizeof(T) == 2>::R4*>(p);
}
__device__ inline void act_st4(float* p, f32x4 v) { *reinterpret_cast<f32x4*>(p) = v; }
__device__ inline void act_st4(__bf16* p, f32x4 v) {
  *reinterpret_cast<bf16x4_t*>(p) = bf16x4_t{(__bf16)v[0], (__bf16)v[1], (__bf16)v[2], (__bf16)v[3]};
}
__device__ inline float act_ld(const float* p) { return *p; }
__device__ inline float act_ld(const __bf16* p) { return (float)*p; }
__device__ inline void act_st(float* p, float v) { *p = v; }
__device__ inline void act_st(__bf16* p, float v) { *p = (__bf16)v; }

__device__ inline float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__device__ inline double wave_sum(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// sums of a and b over a 256-thread block (wave butterflies, then the 4 wave sums in a fixed order), returned to every
// thread; one barrier (the finalize kernels: an 8-level LDS tree with a barrier per level cost ~2 us per launch)
__device__ inline void block_sum2_256(double& a, double& b) {
  __shared__ double red2[2][4];
  a = wave_sum(a);
  b = wave_sum(b);
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    red2[0][w] = a;
    red2[1][w] = b;
  }
  __syncthreads();
  a = (red2[0][0] + red2[0][1]) + (red2[0][2] + red2[0][3]);
  b = (red2[1][0] + red2[1][1]) + (red2[1][2] + red2[1][3]);
}

// f32-in / f32-acc MFMA 32x32x2: lane l supplies A[l&31][l>>5], B[l>>5][l&31];
// D row = (r&3) + 8*(r>>2) + 4*(l>>5), col = l&31.
// torch.relu semantics: NaN propagates (fmaxf(NaN, 0) would return 0 and hide a non-finite batch from the
// trainers' NaN checks, mc:281 / a2:230)
__device__ inline float relu_nan(float v) { return v > 0.f ? v : (v == v ? 0.f : v); }

// BatchNorm state per layer: [7C] floats (backbone.h: mean | invstd | scale | shift | k | mean(dZ) | mean(dZ xhat))
constexpr int BN_STATS_PER_C = 7;

__device__ inline f32x16 mfma32(float a, float b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}

}  // namespace vad
