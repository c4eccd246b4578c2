// Latency-regime instruction costs on gfx950: ONE wave per CU, a single
// dependent chain, with the wave's EXEC mask cut to N of its 64 lanes.
// Question it answers (round 5, the lane-split square-root chains): does a
// wave with fewer live lanes issue a dependent v_mad_u64_u32 faster, and
// what does a cross-lane exchange (DPP quad_perm / row_ror, ds_swizzle,
// ds_bpermute, v_readlane) cost inside a dependent chain?
// Output: JSON, one row per (chain, live lanes).
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

#define ITERS 256
#define UNROLL 16

#define KERNEL(NAME, BODY)                                                                          \
  __global__ __launch_bounds__(64) void k_##NAME(uint64_t* cyc, uint32_t* sink, uint32_t s, int live) { \
    const int lane = (int)threadIdx.x;                                                              \
    uint64_t acc = (uint64_t)(lane * 2654435761u + s);                                              \
    uint32_t x = (uint32_t)acc, a = x ^ 0x9e3779b9u, b = a * 3u + 1u;                               \
    uint64_t t0 = 0, t1 = 0;                                                                        \
    if (lane < live) {                                                                              \
      t0 = __builtin_amdgcn_s_memtime();                                                            \
      for (int it = 0; it < ITERS; ++it) {                                                          \
        _Pragma("unroll") for (int u = 0; u < UNROLL; ++u) { BODY; }                                \
      }                                                                                             \
      t1 = __builtin_amdgcn_s_memtime();                                                            \
    }                                                                                               \
    sink[blockIdx.x * 64 + lane] = (uint32_t)acc ^ x;                                               \
    if (lane == 0) cyc[blockIdx.x] = t1 - t0;                                                       \
  }

// dependent 64-bit MAD chain (the field arithmetic's column chains)
KERNEL(mad_dep, { asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, %0" : "+v"(acc) : "v"(a), "v"(b) : "vcc"); })
// four independent MAD chains round-robin (per-wave issue limit, not latency)
KERNEL(mad_ind4, {
  asm volatile(
      "v_mad_u64_u32 %0, vcc, %1, %2, %0\n"
      "v_mad_u64_u32 v[10:11], vcc, %1, %2, v[10:11]\n"
      "v_mad_u64_u32 v[12:13], vcc, %1, %2, v[12:13]\n"
      "v_mad_u64_u32 v[14:15], vcc, %1, %2, v[14:15]"
      : "+v"(acc) : "v"(a), "v"(b) : "vcc", "v10", "v11", "v12", "v13", "v14", "v15");
})
// dependent 32-bit add chain
KERNEL(add_dep, { asm volatile("v_add_u32 %0, %0, %1" : "+v"(x) : "v"(a)); })
// DPP quad_perm move feeding a dependent add (an operand exchange inside a quad)
KERNEL(dpp_quad, {
  asm volatile(
      "s_nop 1\n"
      "v_mov_b32_dpp %0, %0 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n"
      "v_add_u32 %0, %0, %1"
      : "+v"(x) : "v"(a));
})
// DPP row_ror:4 (rotation inside a 16-lane row)
KERNEL(dpp_ror, {
  asm volatile(
      "s_nop 1\n"
      "v_mov_b32_dpp %0, %0 row_ror:4 row_mask:0xf bank_mask:0xf\n"
      "v_add_u32 %0, %0, %1"
      : "+v"(x) : "v"(a));
})
// ds_swizzle (xor 4 inside 32 lanes) round trip
KERNEL(swizzle, {
  asm volatile(
      "ds_swizzle_b32 %0, %0 offset:swizzle(BITMASK_PERM, \"iiiii\") \n"
      "s_waitcnt lgkmcnt(0)\n"
      "v_add_u32 %0, %0, %1"
      : "+v"(x) : "v"(a));
})
// ds_bpermute round trip (arbitrary source lane)
KERNEL(bpermute, {
  asm volatile(
      "ds_bpermute_b32 %0, %2, %0\n"
      "s_waitcnt lgkmcnt(0)\n"
      "v_add_u32 %0, %0, %1"
      : "+v"(x) : "v"(a), "v"(b & 0xfcu));
})
// v_readlane into an SGPR feeding the next VALU (a broadcast of one lane)
KERNEL(readlane, {
  asm volatile(
      "v_readlane_b32 s40, %0, 1\n"
      "s_nop 4\n"
      "v_add_u32 %0, s40, %1"
      : "+v"(x) : "v"(a) : "s40");
})
// v_permlane32_swap (gfx950): swap the two 32-lane halves
KERNEL(permlane32, {
  asm volatile(
      "v_mov_b32 v16, %0\n"
      "v_permlane32_swap_b32 %0, v16\n"
      "v_add_u32 %0, %0, %1"
      : "+v"(x) : "v"(a) : "v16");
})

typedef void (*kfn)(uint64_t*, uint32_t*, uint32_t, int);

int main() {
  struct {
    const char* name;
    kfn f;
    int per_body;   // instructions counted per body
  } ks[] = {
      {"mad_dep", k_mad_dep, 1},   {"mad_ind4", k_mad_ind4, 4}, {"add_dep", k_add_dep, 1},
      {"dpp_quad+add", k_dpp_quad, 1}, {"dpp_ror+add", k_dpp_ror, 1}, {"swizzle+add", k_swizzle, 1},
      {"bpermute+add", k_bpermute, 1}, {"readlane+add", k_readlane, 1}, {"permlane32+add", k_permlane32, 1},
  };
  const int nk = sizeof(ks) / sizeof(ks[0]);
  int cus = 256;
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, 0) == hipSuccess) cus = prop.multiProcessorCount;
  uint64_t* cyc;
  uint32_t* sink;
  if (hipMalloc(&cyc, cus * sizeof(uint64_t)) != hipSuccess) return 1;
  if (hipMalloc(&sink, cus * 64 * sizeof(uint32_t)) != hipSuccess) return 1;
  uint64_t* h = new uint64_t[cus];
  printf("{\"latency_regime_cycles\": [\n");
  bool first = true;
  for (int i = 0; i < nk; ++i) {
    for (int live : {64, 32, 16, 8, 4, 1}) {
      hipLaunchKernelGGL(ks[i].f, dim3(cus), dim3(64), 0, 0, cyc, sink, 1u, live);
      hipLaunchKernelGGL(ks[i].f, dim3(cus), dim3(64), 0, 0, cyc, sink, 2u, live);
      if (hipDeviceSynchronize() != hipSuccess) return 2;
      if (hipMemcpy(h, cyc, cus * sizeof(uint64_t), hipMemcpyDeviceToHost) != hipSuccess) return 3;
      double sum = 0;
      for (int k = 0; k < cus; ++k) sum += (double)h[k];
      const double per = sum / cus / ((double)ITERS * UNROLL * ks[i].per_body);
      printf("%s  {\"chain\": \"%s\", \"live_lanes\": %d, \"cycles_per_step\": %.2f}", first ? "" : ",\n", ks[i].name,
             live, per);
      first = false;
    }
  }
  printf("\n]}\n");
  return 0;
}
