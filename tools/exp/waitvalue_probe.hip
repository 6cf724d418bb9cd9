// Probe: hipStreamWaitValue64 / hipStreamWriteValue64 semantics on this device (signal memory and plain device
// memory), gate written by a kernel store or by another stream's WriteValue.  Each case prints and returns.
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s -> %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)
__global__ void set_gate(uint64_t* g, uint64_t v) { if (threadIdx.x == 0) *g = v; }
__global__ void spin_us(int us, int* out) {
  const long long t0 = wall_clock64();
  while (wall_clock64() - t0 < (long long)us * 100) {}
  if (threadIdx.x == 0) *out = 1;
}
__global__ void mark(int* out, int v) { if (threadIdx.x == 0) *out = v; }
static int run(const char* name, uint64_t* gate) {
  hipStream_t a, b;
  CK(hipStreamCreateWithFlags(&a, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&b, hipStreamNonBlocking));
  int* d; CK(hipMalloc(&d, 16)); CK(hipMemset(d, 0, 16));
  // case 1: gate set to 1 by a kernel on stream a, then a waits for == 1 (already satisfied)
  set_gate<<<1, 64, 0, a>>>(gate, 1);
  CK(hipStreamWaitValue64(a, gate, 1, hipStreamWaitValueEq, ~0ull));
  mark<<<1, 64, 0, a>>>(d, 7);
  auto t0 = std::chrono::steady_clock::now();
  CK(hipStreamSynchronize(a));
  double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  int h = 0; CK(hipMemcpy(&h, d, 4, hipMemcpyDeviceToHost));
  printf("%s case1 (pre-satisfied, kernel store): mark=%d %.3f ms\n", name, h, ms);
  // case 2: gate 0 (kernel store), a waits; b spins 2 ms then WriteValue 1
  set_gate<<<1, 64, 0, a>>>(gate, 0);
  CK(hipStreamSynchronize(a));
  CK(hipMemset(d, 0, 16));
  CK(hipStreamWaitValue64(a, gate, 1, hipStreamWaitValueEq, ~0ull));
  mark<<<1, 64, 0, a>>>(d, 9);
  spin_us<<<1, 64, 0, b>>>(2000, d + 1);
  CK(hipStreamWriteValue64(b, gate, 1, 0));
  t0 = std::chrono::steady_clock::now();
  CK(hipStreamSynchronize(a));
  ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  int hh[2]; CK(hipMemcpy(hh, d, 8, hipMemcpyDeviceToHost));
  printf("%s case2 (wait, other stream WriteValue after 2 ms spin): mark=%d spin_done=%d %.3f ms\n", name, hh[0], hh[1], ms);
  // case 3: repeated 200x pre-satisfied waits, time per wait
  t0 = std::chrono::steady_clock::now();
  for (int i = 0; i < 200; ++i) {
    set_gate<<<1, 64, 0, a>>>(gate, 1);
    CK(hipStreamWaitValue64(a, gate, 1, hipStreamWaitValueEq, ~0ull));
    mark<<<1, 64, 0, a>>>(d, i);
  }
  CK(hipStreamSynchronize(a));
  ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  printf("%s case3 200x (store, wait, kernel): %.3f ms total\n", name, ms);
  t0 = std::chrono::steady_clock::now();
  for (int i = 0; i < 200; ++i) { set_gate<<<1, 64, 0, a>>>(gate, 1); mark<<<1, 64, 0, a>>>(d, i); }
  CK(hipStreamSynchronize(a));
  ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  printf("%s case3 baseline 200x (store, kernel): %.3f ms total\n", name, ms);
  return 0;
}
int main(int argc, char** argv) {
  int attr = 0;
  CK(hipDeviceGetAttribute(&attr, hipDeviceAttributeCanUseStreamWaitValue, 0));
  printf("CanUseStreamWaitValue=%d\n", attr);
  const int which = argc > 1 ? atoi(argv[1]) : 0;
  uint64_t* g = nullptr;
  if (which == 0) { CK(hipExtMallocWithFlags((void**)&g, 8, hipMallocSignalMemory)); return run("signal", g); }
  CK(hipMalloc((void**)&g, 8));
  return run("device", g);
}
