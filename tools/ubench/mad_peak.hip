// Peak issue rate of v_mad_u64_u32 (and two reference ops) on one MI355X:
// independent accumulation chains, 1..8 waves per SIMD, ~50 ms launches, and
// the in-kernel clock (s_memtime / s_memrealtime x 100 MHz) the chip held.
// The curve kernel's roofline `peak` is the best lane-ops/s measured here.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -o mad_peak mad_peak.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define CHAINS 8
#define UNROLL 16

#define KERNEL(NAME, T, INIT, BODY)                                                                  \
  __global__ __launch_bounds__(256) void k_##NAME(uint64_t* clk, uint32_t* sink, uint32_t s, int iters) { \
    T acc[CHAINS];                                                                                   \
    uint32_t a = threadIdx.x * 2654435761u + s, b = a ^ 0x9e3779b9u;                                 \
    _Pragma("unroll") for (int c = 0; c < CHAINS; ++c) acc[c] = INIT;                                \
    const uint64_t t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();         \
    for (int it = 0; it < iters; ++it) {                                                             \
      _Pragma("unroll") for (int u = 0; u < UNROLL; ++u) {                                           \
        _Pragma("unroll") for (int c = 0; c < CHAINS; ++c) { BODY; }                                 \
      }                                                                                              \
    }                                                                                                \
    const uint64_t t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();         \
    uint32_t r = 0;                                                                                  \
    _Pragma("unroll") for (int c = 0; c < CHAINS; ++c) r ^= (uint32_t)acc[c];                        \
    sink[blockIdx.x * 256 + threadIdx.x] = r;                                                        \
    if (threadIdx.x == 0) {                                                                          \
      clk[2 * blockIdx.x] = t1 - t0;                                                                 \
      clk[2 * blockIdx.x + 1] = r1 - r0;                                                             \
    }                                                                                                \
  }

KERNEL(mad_u64_u32, uint64_t, (uint64_t)(a + c),
       { uint64_t cc; asm volatile("v_mad_u64_u32 %0, %1, %2, %3, %0" : "+v"(acc[c]), "=s"(cc) : "v"(a), "v"(b)); })
KERNEL(add_u32, uint32_t, a + c, { asm volatile("v_add_u32 %0, %0, %1" : "+v"(acc[c]) : "v"(b)); })
KERNEL(lshrrev_b64, uint64_t, (uint64_t)(a + c), { asm volatile("v_lshrrev_b64 %0, 3, %0" : "+v"(acc[c])); })
KERNEL(alignbit_b32, uint32_t, a + c, { asm volatile("v_alignbit_b32 %0, %0, %1, 7" : "+v"(acc[c]) : "v"(b)); })
KERNEL(bitop3_b32, uint32_t, a + c,
       { asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96" : "+v"(acc[c]) : "v"(a), "v"(b)); })
KERNEL(xor_b32, uint32_t, a + c, { asm volatile("v_xor_b32 %0, %0, %1" : "+v"(acc[c]) : "v"(b)); })
KERNEL(lshl_add_u64, uint64_t, (uint64_t)(a + c),
       { asm volatile("v_lshl_add_u64 %0, %0, 0, %1" : "+v"(acc[c]) : "v"((uint64_t)b)); })

typedef void (*kfn)(uint64_t*, uint32_t*, uint32_t, int);

int main() {
  struct { const char* name; kfn f; } ks[] = {
      {"v_mad_u64_u32", k_mad_u64_u32}, {"v_add_u32", k_add_u32}, {"v_lshrrev_b64", k_lshrrev_b64},
      {"v_alignbit_b32", k_alignbit_b32}, {"v_bitop3_b32", k_bitop3_b32}, {"v_xor_b32", k_xor_b32},
      {"v_lshl_add_u64", k_lshl_add_u64}};
  int cus = 256;
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, 0) == hipSuccess) cus = prop.multiProcessorCount;
  const int maxb = cus * 8;
  uint64_t* clk;
  uint32_t* sink;
  if (hipMalloc(&clk, maxb * 2 * sizeof(uint64_t)) != hipSuccess) return 1;
  if (hipMalloc(&sink, maxb * 256 * sizeof(uint32_t)) != hipSuccess) return 1;
  uint64_t* h = new uint64_t[maxb * 2];
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  printf("{\"cus\": %d, \"results\": [\n", cus);
  bool first = true;
  for (auto& k : ks) {
    for (int w : {1, 2, 3, 4, 6, 8}) {
      const int blocks = cus * w;
      // size for ~50 ms at ~3 cycles/insn/SIMD-wave-slot
      const int iters = 2400000 / (CHAINS * UNROLL) * 12 / w;
      hipLaunchKernelGGL(k.f, dim3(blocks), dim3(256), 0, 0, clk, sink, 1u, iters / 4);
      float best = 1e30f;
      double ghz = 0;
      for (int r = 0; r < 3; ++r) {
        if (hipEventRecord(e0) != hipSuccess) return 2;
        hipLaunchKernelGGL(k.f, dim3(blocks), dim3(256), 0, 0, clk, sink, (uint32_t)r + 2, iters);
        hipEventRecord(e1);
        if (hipEventSynchronize(e1) != hipSuccess) return 3;
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        if (ms < best) {
          best = ms;
          hipMemcpy(h, clk, blocks * 2 * sizeof(uint64_t), hipMemcpyDeviceToHost);
          double sc = 0, sr = 0;
          for (int b = 0; b < blocks; ++b) { sc += (double)h[2 * b]; sr += (double)h[2 * b + 1]; }
          ghz = sc / sr * 0.1;
        }
      }
      const double ops = (double)blocks * 256 * CHAINS * UNROLL * iters;
      const double rate = ops / (best * 1e-3);
      printf("%s  {\"insn\": \"%s\", \"waves_per_simd\": %d, \"ms\": %.3f, \"lane_ops_per_s\": %.4e, "
             "\"clock_ghz\": %.3f, \"lane_ops_per_clk_per_cu\": %.2f}",
             first ? "" : ",\n", k.name, w, best, rate, ghz, rate / (ghz * 1e9) / cus);
      first = false;
    }
  }
  printf("\n]}\n");
  return hipGetLastError() == hipSuccess ? 0 : 4;
}
