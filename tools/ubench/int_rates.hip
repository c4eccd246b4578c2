// Integer/VALU issue-rate microbenchmark for gfx950.
// Measures lane-ops/s for the instructions the Ed25519 field arithmetic and
// SHA-512 are built from; the v_mad_u64_u32 rate is the roofline peak P_mad
// used by bench.py.
// Build: hipcc --offload-arch=gfx950 -O3 -o int_rates int_rates.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define CHAINS 8
#define UNROLL 16
#define ITERS 512

#define KERNEL(NAME, T, INIT, BODY, FOLD)                                      \
  __global__ __launch_bounds__(256) void k_##NAME(uint32_t* out, uint32_t s) { \
    T acc[CHAINS];                                                             \
    uint32_t a = threadIdx.x * 2654435761u + s, b = a ^ 0x9e3779b9u;           \
    _Pragma("unroll") for (int c = 0; c < CHAINS; ++c) acc[c] = INIT;          \
    for (int it = 0; it < ITERS; ++it) {                                       \
      _Pragma("unroll") for (int u = 0; u < UNROLL; ++u) {                     \
        _Pragma("unroll") for (int c = 0; c < CHAINS; ++c) { BODY; }           \
      }                                                                        \
    }                                                                          \
    uint32_t r = 0;                                                            \
    _Pragma("unroll") for (int c = 0; c < CHAINS; ++c) r ^= FOLD;              \
    out[blockIdx.x * 256 + threadIdx.x] = r;                                   \
  }

KERNEL(mad_u64_u32, uint64_t, (uint64_t)(a + c),
       { uint64_t cc; asm volatile("v_mad_u64_u32 %0, %1, %2, %3, %0" : "+v"(acc[c]), "=s"(cc) : "v"(a), "v"(b)); },
       (uint32_t)acc[c] ^ (uint32_t)(acc[c] >> 32))
KERNEL(mul_lo_u32, uint32_t, a + c,
       { asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(acc[c]) : "v"(b)); }, acc[c])
KERNEL(mul_hi_u32, uint32_t, a + c,
       { asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(acc[c]) : "v"(b)); }, acc[c])
KERNEL(mul_u32_u24, uint32_t, a + c,
       { asm volatile("v_mul_u32_u24 %0, %0, %1" : "+v"(acc[c]) : "v"(b)); }, acc[c])
KERNEL(mul_hi_u32_u24, uint32_t, a + c,
       { asm volatile("v_mul_hi_u32_u24 %0, %0, %1" : "+v"(acc[c]) : "v"(b)); }, acc[c])
KERNEL(mad_u32_u24, uint32_t, a + c,
       { asm volatile("v_mad_u32_u24 %0, %1, %2, %0" : "+v"(acc[c]) : "v"(a), "v"(b)); }, acc[c])
KERNEL(add_u32, uint32_t, a + c,
       { asm volatile("v_add_u32 %0, %0, %1" : "+v"(acc[c]) : "v"(b)); }, acc[c])
KERNEL(add3_u32, uint32_t, a + c,
       { asm volatile("v_add3_u32 %0, %0, %1, %2" : "+v"(acc[c]) : "v"(a), "v"(b)); }, acc[c])
KERNEL(alignbit_b32, uint32_t, a + c,
       { asm volatile("v_alignbit_b32 %0, %0, %1, 7" : "+v"(acc[c]) : "v"(b)); }, acc[c])
KERNEL(xor_b32, uint32_t, a + c,
       { asm volatile("v_xor_b32 %0, %0, %1" : "+v"(acc[c]) : "v"(b)); }, acc[c])
KERNEL(add_co_u32, uint32_t, a + c,
       { uint64_t cc; asm volatile("v_add_co_u32 %0, %1, %0, %2" : "+v"(acc[c]), "=s"(cc) : "v"(b)); }, acc[c])
KERNEL(lshl_add_u64, uint64_t, (uint64_t)(a + c),
       { asm volatile("v_lshl_add_u64 %0, %0, 0, %1" : "+v"(acc[c]) : "v"((uint64_t)b)); },
       (uint32_t)acc[c] ^ (uint32_t)(acc[c] >> 32))
KERNEL(lshrrev_b64, uint64_t, (uint64_t)(a + c),
       { asm volatile("v_lshrrev_b64 %0, 3, %0" : "+v"(acc[c])); },
       (uint32_t)acc[c] ^ (uint32_t)(acc[c] >> 32))
KERNEL(fma_f64, double, (double)(a + c),
       { asm volatile("v_fma_f64 %0, %0, %1, %2" : "+v"(acc[c]) : "v"((double)b), "v"((double)a)); },
       (uint32_t)acc[c])
KERNEL(fma_f32, float, (float)(a + c),
       { asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(acc[c]) : "v"((float)b), "v"((float)a)); },
       (uint32_t)acc[c])
KERNEL(dot2_u32_u16, uint32_t, a + c,
       { asm volatile("v_dot2_u32_u16 %0, %1, %2, %0" : "+v"(acc[c]) : "v"(a), "v"(b)); }, acc[c])
KERNEL(bfi_b32, uint32_t, a + c,
       { asm volatile("v_bfi_b32 %0, %0, %1, %2" : "+v"(acc[c]) : "v"(a), "v"(b)); }, acc[c])
KERNEL(bitop3_b32, uint32_t, a + c,
       { asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96" : "+v"(acc[c]) : "v"(a), "v"(b)); }, acc[c])
KERNEL(lshrrev_b32, uint32_t, a + c,
       { asm volatile("v_lshrrev_b32 %0, 3, %0" : "+v"(acc[c])); }, acc[c])
KERNEL(perm_b32, uint32_t, a + c,
       { asm volatile("v_perm_b32 %0, %0, %1, %2" : "+v"(acc[c]) : "v"(a), "v"(0x00010203u)); }, acc[c])

typedef void (*kfn)(uint32_t*, uint32_t);

int main() {
  struct { const char* name; kfn f; } ks[] = {
    {"v_mad_u64_u32", k_mad_u64_u32}, {"v_mul_lo_u32", k_mul_lo_u32},
    {"v_mul_hi_u32", k_mul_hi_u32}, {"v_mul_u32_u24", k_mul_u32_u24},
    {"v_mul_hi_u32_u24", k_mul_hi_u32_u24}, {"v_mad_u32_u24", k_mad_u32_u24},
    {"v_add_u32", k_add_u32}, {"v_add3_u32", k_add3_u32},
    {"v_alignbit_b32", k_alignbit_b32}, {"v_xor_b32", k_xor_b32},
    {"v_add_co_u32", k_add_co_u32}, {"v_lshl_add_u64", k_lshl_add_u64},
    {"v_lshrrev_b64", k_lshrrev_b64}, {"v_fma_f64", k_fma_f64},
    {"v_fma_f32", k_fma_f32}, {"v_dot2_u32_u16", k_dot2_u32_u16},
    {"v_bfi_b32", k_bfi_b32}, {"v_bitop3_b32", k_bitop3_b32}, {"v_lshrrev_b32", k_lshrrev_b32},
    {"v_perm_b32", k_perm_b32},
    // the MAD again at the end, after the clock has ramped (the first kernel
    // of the run can start below the sustained clock)
    {"v_mad_u64_u32", k_mad_u64_u32},
  };
  int blocks = 256 * 8;
  uint32_t* d;
  hipMalloc(&d, blocks * 256 * 4);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  double ops = (double)blocks * 256 * CHAINS * UNROLL * ITERS;
  printf("{\"results\": [\n");
  for (size_t i = 0; i < sizeof(ks) / sizeof(ks[0]); ++i) {
    hipLaunchKernelGGL(ks[i].f, dim3(blocks), dim3(256), 0, 0, d, 1u);
    hipDeviceSynchronize();
    float best = 1e30f;
    for (int r = 0; r < 5; ++r) {
      hipEventRecord(e0);
      hipLaunchKernelGGL(ks[i].f, dim3(blocks), dim3(256), 0, 0, d, (uint32_t)r);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms;
      hipEventElapsedTime(&ms, e0, e1);
      if (ms < best) best = ms;
    }
    double rate = ops / (best * 1e-3);
    // lane-ops per clock per CU at the nominal 2.4 GHz
    double per_clk_cu = rate / 2.4e9 / 256.0;
    printf("  {\"insn\": \"%s\", \"lane_ops_per_s\": %.4e, \"lane_ops_per_clk_per_cu_at_2.4GHz\": %.2f, \"ms\": %.3f}%s\n",
           ks[i].name, rate, per_clk_cu, best, i + 1 < sizeof(ks) / sizeof(ks[0]) ? "," : "");
  }
  printf("]}\n");
  hipError_t err = hipGetLastError();
  if (err != hipSuccess) { fprintf(stderr, "HIP error %s\n", hipGetErrorString(err)); return 1; }
  return 0;
}
