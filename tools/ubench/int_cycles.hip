// Cycles per wave64 VALU instruction on gfx950, measured in-kernel with
// s_memtime (shader-clock ticks), at 1, 2 and 4 waves per SIMD.
// Complements int_rates.hip (which depends on the clock the chip held):
// these are clock-independent issue costs for the instruction mix of the
// field arithmetic.  Output: JSON, one row per (instruction, waves/SIMD).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define CHAINS 8
#define UNROLL 16
#define ITERS 64

#define KERNEL(NAME, T, INIT, BODY)                                                      \
  __global__ __launch_bounds__(256) void k_##NAME(uint64_t* cyc, uint32_t* sink, uint32_t s) { \
    T acc[CHAINS];                                                                       \
    uint32_t a = threadIdx.x * 2654435761u + s, b = a ^ 0x9e3779b9u;                     \
    _Pragma("unroll") for (int c = 0; c < CHAINS; ++c) acc[c] = INIT;                    \
    uint64_t t0 = __builtin_amdgcn_s_memtime();                                          \
    for (int it = 0; it < ITERS; ++it) {                                                 \
      _Pragma("unroll") for (int u = 0; u < UNROLL; ++u) {                               \
        _Pragma("unroll") for (int c = 0; c < CHAINS; ++c) { BODY; }                     \
      }                                                                                  \
    }                                                                                    \
    uint64_t t1 = __builtin_amdgcn_s_memtime();                                          \
    uint32_t r = 0;                                                                      \
    _Pragma("unroll") for (int c = 0; c < CHAINS; ++c) r ^= (uint32_t)acc[c];            \
    sink[blockIdx.x * 256 + threadIdx.x] = r;                                            \
    if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * 4 + threadIdx.x / 64] = t1 - t0;       \
  }

KERNEL(mad_u64_u32, uint64_t, (uint64_t)(a + c),
       { uint64_t cc; asm volatile("v_mad_u64_u32 %0, %1, %2, %3, %0" : "+v"(acc[c]), "=s"(cc) : "v"(a), "v"(b)); })
KERNEL(mul_lo_u32, uint32_t, a + c, { asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(acc[c]) : "v"(b)); })
KERNEL(add_u32, uint32_t, a + c, { asm volatile("v_add_u32 %0, %0, %1" : "+v"(acc[c]) : "v"(b)); })
KERNEL(and_b32, uint32_t, a + c, { asm volatile("v_and_b32 %0, %0, %1" : "+v"(acc[c]) : "v"(b)); })
KERNEL(lshlrev_b32, uint32_t, a + c, { asm volatile("v_lshlrev_b32 %0, 3, %0" : "+v"(acc[c])); })
KERNEL(add3_u32, uint32_t, a + c, { asm volatile("v_add3_u32 %0, %0, %1, %2" : "+v"(acc[c]) : "v"(a), "v"(b)); })
KERNEL(alignbit_b32, uint32_t, a + c, { asm volatile("v_alignbit_b32 %0, %0, %1, 7" : "+v"(acc[c]) : "v"(b)); })
KERNEL(lshl_add_u64, uint64_t, (uint64_t)(a + c),
       { asm volatile("v_lshl_add_u64 %0, %0, 0, %1" : "+v"(acc[c]) : "v"((uint64_t)b)); })
KERNEL(lshrrev_b64, uint64_t, (uint64_t)(a + c), { asm volatile("v_lshrrev_b64 %0, 3, %0" : "+v"(acc[c])); })
KERNEL(mov_b32, uint32_t, a + c, { asm volatile("v_mov_b32 %0, %1" : "=v"(acc[c]) : "v"(acc[(c + 1) % CHAINS])); })
KERNEL(cndmask_b32, uint32_t, a + c,
       { asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(acc[c]) : "v"(b) : "vcc"); })
KERNEL(mad_u32_u24, uint32_t, a + c, { asm volatile("v_mad_u32_u24 %0, %1, %2, %0" : "+v"(acc[c]) : "v"(a), "v"(b)); })

typedef void (*kfn)(uint64_t*, uint32_t*, uint32_t);

int main() {
  struct { const char* name; kfn f; } ks[] = {
    {"v_mad_u64_u32", k_mad_u64_u32}, {"v_mul_lo_u32", k_mul_lo_u32}, {"v_add_u32", k_add_u32},
    {"v_and_b32", k_and_b32}, {"v_lshlrev_b32", k_lshlrev_b32}, {"v_add3_u32", k_add3_u32},
    {"v_alignbit_b32", k_alignbit_b32}, {"v_lshl_add_u64", k_lshl_add_u64}, {"v_lshrrev_b64", k_lshrrev_b64},
    {"v_mov_b32", k_mov_b32}, {"v_cndmask_b32", k_cndmask_b32}, {"v_mad_u32_u24", k_mad_u32_u24},
  };
  const int nk = sizeof(ks) / sizeof(ks[0]);
  int cus = 256;
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, 0) == hipSuccess) cus = prop.multiProcessorCount;
  uint64_t* cyc;
  uint32_t* sink;
  const int maxblocks = cus * 8;
  if (hipMalloc(&cyc, maxblocks * 4 * sizeof(uint64_t)) != hipSuccess) return 1;
  if (hipMalloc(&sink, maxblocks * 256 * sizeof(uint32_t)) != hipSuccess) return 1;
  uint64_t* h = new uint64_t[maxblocks * 4];
  const double insts = (double)CHAINS * UNROLL * ITERS;
  printf("{\"cycles_per_wave_instruction\": [\n");
  bool first = true;
  for (int i = 0; i < nk; ++i) {
    for (int w : {1, 2, 4}) {
      const int blocks = cus * w;  // 256-thread blocks: one wave per SIMD per block
      hipLaunchKernelGGL(ks[i].f, dim3(blocks), dim3(256), 0, 0, cyc, sink, 1u);
      hipLaunchKernelGGL(ks[i].f, dim3(blocks), dim3(256), 0, 0, cyc, sink, 2u);
      if (hipDeviceSynchronize() != hipSuccess) return 2;
      if (hipMemcpy(h, cyc, blocks * 4 * sizeof(uint64_t), hipMemcpyDeviceToHost) != hipSuccess) return 3;
      double sum = 0;
      for (int k = 0; k < blocks * 4; ++k) sum += (double)h[k];
      const double per_wave = sum / (blocks * 4) / insts;  // cycles one wave spends per instruction
      printf("%s  {\"insn\": \"%s\", \"waves_per_simd\": %d, \"cycles_per_insn_per_wave\": %.3f, "
             "\"simd_cycles_per_insn\": %.3f}",
             first ? "" : ",\n", ks[i].name, w, per_wave, per_wave / w);
      first = false;
    }
  }
  printf("\n]}\n");
  return 0;
}
