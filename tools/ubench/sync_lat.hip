// Host-observed completion latency of one small launch (the latency calls' tail:
// launch + wait for the verdicts).  Modes, 2000 calls each, median / min us:
//   sync   hipLaunchKernelGGL + hipStreamSynchronize
//   event  + hipEventRecord + hipEventSynchronize
//   poll   the kernel stores a sequence number into fine-grained host memory
//          (after __threadfence_system); the host spins on it, no HIP wait call
// argv[1] == "spin": hipSetDeviceFlags(hipDeviceScheduleSpin) before any HIP call.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -o sync_lat sync_lat.hip
#include <hip/hip_runtime.h>
#include <algorithm>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <vector>

__global__ void k_flag(uint32_t* flag, uint32_t seq) {
  if (threadIdx.x == 0) {
    __threadfence_system();
    __hip_atomic_store(flag + threadIdx.x, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

static double now_us() {
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main(int argc, char** argv) {
  const bool spin = argc > 1 && !strcmp(argv[1], "spin");
  if (spin && hipSetDeviceFlags(hipDeviceScheduleSpin) != hipSuccess) return 1;
  hipStream_t s;
  if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) return 1;
  uint32_t* hflag = nullptr;
  if (hipHostMalloc(reinterpret_cast<void**>(&hflag), 64, hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess)
    return 1;
  void* dflag = nullptr;
  if (hipHostGetDevicePointer(&dflag, hflag, 0) != hipSuccess) return 1;
  *hflag = 0;
  hipEvent_t ev;
  if (hipEventCreateWithFlags(&ev, hipEventDisableTiming) != hipSuccess) return 1;
  const int N = 2000;
  const char* names[3] = {"sync", "event", "poll"};
  printf("{\"schedule\": \"%s\", \"modes\": [", spin ? "spin" : "default");
  uint32_t seq = 1;
  for (int m = 0; m < 3; ++m) {
    std::vector<double> t;
    for (int i = 0; i < N + 50; ++i, ++seq) {
      const double t0 = now_us();
      hipLaunchKernelGGL(k_flag, dim3(1), dim3(64), 0, s, static_cast<uint32_t*>(dflag), seq);
      if (m == 0) {
        if (hipStreamSynchronize(s) != hipSuccess) return 2;
      } else if (m == 1) {
        if (hipEventRecord(ev, s) != hipSuccess || hipEventSynchronize(ev) != hipSuccess) return 2;
      } else {
        const double lim = t0 + 1e6;
        while (__atomic_load_n(hflag, __ATOMIC_ACQUIRE) != seq)
          if (now_us() > lim) return 3;
      }
      const double t1 = now_us();
      if (m == 2 && hipStreamSynchronize(s) != hipSuccess) return 2;   // drained outside the timed span
      if (i >= 50) t.push_back(t1 - t0);
    }
    std::sort(t.begin(), t.end());
    printf("%s{\"mode\": \"%s\", \"median_us\": %.2f, \"min_us\": %.2f, \"p90_us\": %.2f}", m ? ", " : "", names[m],
           t[t.size() / 2], t[0], t[t.size() * 9 / 10]);
  }
  printf("]}\n");
  return 0;
}
