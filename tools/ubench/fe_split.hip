// A lone wave's squaring with each column's products split over TWO dependent
// MAD chains (one seeded with the incoming carry, one from zero, joined by one
// v_lshl_add_u64) against the shipped carry-seeded single chain (fe_sq): the
// split halves the dependent-MAD depth of a column (~10 cycles per dependent MAD
// against ~5.5 for independent ones on a lone wave, profiles/r05_lane_exec.json)
// for one extra 64-bit add per column.  The same column sums, so the same limbs.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -o fe_split fe_split.hip
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include "../../indy-plenum_amd/csrc/pv_field.h"

using namespace pv;
constexpr int N = 254;

__device__ __forceinline__ uint64_t split6(uint64_t c, bool first, const uint32_t a[6], const uint32_t b[6]) {
  uint64_t x = first ? 0 : c, y;
  asm("v_mad_u64_u32 %0, vcc, %2, %3, %0\n"
      "v_mad_u64_u32 %1, vcc, %4, %5, 0\n"
      "v_mad_u64_u32 %0, vcc, %6, %7, %0\n"
      "v_mad_u64_u32 %1, vcc, %8, %9, %1\n"
      "v_mad_u64_u32 %0, vcc, %10, %11, %0\n"
      "v_mad_u64_u32 %1, vcc, %12, %13, %1\n"
      "s_nop 0\n"
      "v_lshl_add_u64 %0, %0, 0, %1"
      : "+v"(x), "=&v"(y)
      : "v"(a[0]), "v"(b[0]), "v"(a[1]), "v"(b[1]), "v"(a[2]), "v"(b[2]), "v"(a[3]), "v"(b[3]), "v"(a[4]), "v"(b[4]),
        "v"(a[5]), "v"(b[5])
      : "vcc");
  return x;
}
__device__ __forceinline__ uint64_t split5(uint64_t c, const uint32_t a[6], const uint32_t b[6]) {
  uint64_t x = c, y;
  asm("v_mad_u64_u32 %0, vcc, %2, %3, %0\n"
      "v_mad_u64_u32 %1, vcc, %4, %5, 0\n"
      "v_mad_u64_u32 %0, vcc, %6, %7, %0\n"
      "v_mad_u64_u32 %1, vcc, %8, %9, %1\n"
      "v_mad_u64_u32 %0, vcc, %10, %11, %0\n"
      "s_nop 0\n"
      "v_lshl_add_u64 %0, %0, 0, %1"
      : "+v"(x), "=&v"(y)
      : "v"(a[0]), "v"(b[0]), "v"(a[1]), "v"(b[1]), "v"(a[2]), "v"(b[2]), "v"(a[3]), "v"(b[3]), "v"(a[4]), "v"(b[4])
      : "vcc");
  return x;
}
__device__ __forceinline__ void fe_sq_split(fe& h, const fe& f) {
  sq_ops o;
  sq_prepare(o, f);
  uint64_t carry = 0;
  uint32_t out[10];
#pragma unroll
  for (int k = 0; k < 10; ++k) {
    uint32_t as[6], bs[6];
    sq_column<1>(o, k, as, bs);
    const uint64_t acc = (k & 1) ? split5(carry, as, bs) : split6(carry, k == 0, as, bs);
    carry = acc >> ((k & 1) ? 25 : 26);
    out[k] = (uint32_t)acc & ((k & 1) ? M25 : M26);
  }
  fe_finish_columns(h, carry, out);
}

template <int V>
__global__ __launch_bounds__(64) void k_chain(uint64_t* cyc, uint32_t* out, uint32_t s) {
  const int lane = (int)threadIdx.x;
  fe a;
#pragma unroll
  for (int i = 0; i < 10; ++i) a.v[i] = ((lane + 1) * 2654435761u + s * (i + 3)) & ((i & 1) ? M25 : M26);
  const uint64_t t0 = __builtin_amdgcn_s_memtime();
#pragma unroll 1
  for (int i = 0; i < N; ++i) {
    if (V == 0) fe_sq(a, a);
    else fe_sq_split(a, a);
  }
  const uint64_t t1 = __builtin_amdgcn_s_memtime();
  if (lane == 0) cyc[V] = t1 - t0;
  for (int i = 0; i < 10; ++i) out[V * 640 + lane * 10 + i] = a.v[i];
}

int main() {
  uint64_t* cyc;
  uint32_t* out;
  if (hipMalloc(&cyc, 16) || hipMalloc(&out, 2 * 640 * 4)) return 1;
  double best[2] = {1e30, 1e30};
  uint32_t h[1280];
  uint64_t c[2];
  for (int rep = 0; rep < 5; ++rep) {
    hipLaunchKernelGGL(k_chain<0>, dim3(1), dim3(64), 0, 0, cyc, out, 12345u);
    hipLaunchKernelGGL(k_chain<1>, dim3(1), dim3(64), 0, 0, cyc, out, 12345u);
    if (hipDeviceSynchronize()) return 2;
    if (hipMemcpy(c, cyc, 16, hipMemcpyDeviceToHost) || hipMemcpy(h, out, sizeof h, hipMemcpyDeviceToHost)) return 3;
    for (int k = 0; k < 2; ++k) best[k] = best[k] < c[k] / (double)N ? best[k] : c[k] / (double)N;
  }
  int mism = 0;
  for (int i = 0; i < 640; ++i) mism += h[i] != h[640 + i];
  printf("{\"cycles_per_fe_sq_seeded\": %.1f, \"cycles_per_fe_sq_split_columns\": %.1f, \"limb_mismatches\": %d}\n",
         best[0], best[1], mism);
  return 0;
}
