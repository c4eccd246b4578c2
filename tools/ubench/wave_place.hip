// Where the waves of one small workgroup run, and whether they slow each other
// down (the latency kernels' regime: k_verify_quad_keyed is ONE block of three
// waves -- hash, comb, square root -- per 8 signatures).  One block of W waves
// (W = 1..4) on an otherwise idle GPU; every wave runs the same serial chain of
// fe_sq (the square root's inner loop) and records its SIMD (HW_ID bits 5:4),
// its CU (bits 11:8) and its cycles (s_memtime).  Output: JSON.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -o wave_place wave_place.hip
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include "../../indy-plenum_amd/csrc/pv_field.h"

using namespace pv;

__global__ __launch_bounds__(256) void k_place(uint64_t* out, uint32_t* sink, int iters) {
  const int lane = (int)threadIdx.x;
  fe a;
#pragma unroll
  for (int i = 0; i < 10; ++i) a.v[i] = ((lane + 1) * 2654435761u + 7u * (i + 3)) & ((i & 1) ? M25 : M26);
  uint32_t hw;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
  const uint64_t t0 = __builtin_amdgcn_s_memtime();
#pragma unroll 1
  for (int i = 0; i < iters; ++i) fe_sq(a, a);
  const uint64_t t1 = __builtin_amdgcn_s_memtime();
  sink[blockIdx.x * 256 + lane] = a.v[0] ^ a.v[9];
  if ((lane & 63) == 0) {
    const int w = lane >> 6;
    out[(blockIdx.x * 4 + w) * 2] = hw;
    out[(blockIdx.x * 4 + w) * 2 + 1] = t1 - t0;
  }
}

int main() {
  uint64_t* out;
  uint32_t* sink;
  if (hipMalloc(&out, 64 * sizeof(uint64_t)) != hipSuccess) return 1;
  if (hipMalloc(&sink, 4 * 256 * sizeof(uint32_t)) != hipSuccess) return 1;
  uint64_t h[64];
  printf("{\"one_block_waves\": [\n");
  bool first = true;
  for (int w = 1; w <= 4; ++w) {
    for (int rep = 0; rep < 3; ++rep) {
      hipMemset(out, 0, 64 * sizeof(uint64_t));
      hipLaunchKernelGGL(k_place, dim3(1), dim3(64 * w), 0, 0, out, sink, 254);
      if (hipDeviceSynchronize() != hipSuccess) return 2;
      if (hipMemcpy(h, out, 64 * sizeof(uint64_t), hipMemcpyDeviceToHost) != hipSuccess) return 3;
      for (int k = 0; k < w; ++k) {
        const uint32_t hw = (uint32_t)h[2 * k];
        printf("%s  {\"waves\": %d, \"rep\": %d, \"wave\": %d, \"simd\": %u, \"cu\": %u, \"cycles_per_fe_sq\": %.1f}",
               first ? "" : ",\n", w, rep, k, (hw >> 4) & 3u, (hw >> 8) & 15u, (double)h[2 * k + 1] / 254.0);
        first = false;
      }
    }
  }
  printf("\n]}\n");
  return 0;
}
