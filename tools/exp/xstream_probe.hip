// Probe: latency from the end of a kernel on stream a to the start of a dependent kernel on stream b (GPU wall clock,
// 100 MHz), for: same stream; hipEventRecord / hipStreamWaitEvent (timing-disabled events, with and without the
// system fence); hipStreamWriteValue64 / hipStreamWaitValue64 on signal memory.  20 reps each, median in us.
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <vector>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s -> %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)
__global__ void stamp(unsigned long long* out, int idx, int spin) {
  if (threadIdx.x == 0) {
    const unsigned long long t0 = wall_clock64();
    out[2 * idx] = t0;
    while (wall_clock64() - t0 < (unsigned long long)spin) {}
    out[2 * idx + 1] = wall_clock64();
  }
}
static double med(std::vector<double> v) { std::sort(v.begin(), v.end()); return v[v.size() / 2]; }
int main() {
  hipStream_t a, b;
  CK(hipStreamCreateWithFlags(&a, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&b, hipStreamNonBlocking));
  unsigned long long* d; CK(hipMalloc(&d, 64 * 8));
  unsigned long long h[64];
  hipEvent_t e1, e2;
  CK(hipEventCreateWithFlags(&e1, hipEventDisableTiming));
  CK(hipEventCreateWithFlags(&e2, hipEventDisableTiming | hipEventDisableSystemFence));
  uint64_t* gate; CK(hipExtMallocWithFlags((void**)&gate, 8, hipMallocSignalMemory));
  const int spin = 2000;  // 20 us of work on a first, so b's dependency is queued long before it is satisfied
  const char* names[] = {"same stream", "event (sys fence)", "event (no sys fence)", "write/wait value (signal mem)",
                         "event, b waits with prior work"};
  for (int cse = 0; cse < 5; ++cse) {
    std::vector<double> gaps;
    for (int rep = 0; rep < 21; ++rep) {
      CK(hipMemset(gate, 0, 8));
      CK(hipDeviceSynchronize());
      if (cse == 0) {
        stamp<<<1, 64, 0, a>>>(d, 0, spin);
        stamp<<<1, 64, 0, a>>>(d, 1, 0);
      } else if (cse == 1 || cse == 2 || cse == 4) {
        hipEvent_t ev = cse == 2 ? e2 : e1;
        if (cse == 4) stamp<<<1, 64, 0, b>>>(d, 2, 100);
        stamp<<<1, 64, 0, a>>>(d, 0, spin);
        CK(hipEventRecord(ev, a));
        CK(hipStreamWaitEvent(b, ev, 0));
        stamp<<<1, 64, 0, b>>>(d, 1, 0);
      } else {
        CK(hipStreamWaitValue64(b, gate, 1, hipStreamWaitValueEq, ~0ull));
        stamp<<<1, 64, 0, b>>>(d, 1, 0);
        stamp<<<1, 64, 0, a>>>(d, 0, spin);
        CK(hipStreamWriteValue64(a, gate, 1, 0));
      }
      CK(hipDeviceSynchronize());
      CK(hipMemcpy(h, d, 8 * 8, hipMemcpyDeviceToHost));
      if (rep) gaps.push_back((double)((long long)h[2] - (long long)h[1]) / 100.0);
    }
    printf("%-34s end(a) -> start(b) median %.2f us (min %.2f max %.2f)\n", names[cse], med(gaps),
           *std::min_element(gaps.begin(), gaps.end()), *std::max_element(gaps.begin(), gaps.end()));
  }
  return 0;
}
