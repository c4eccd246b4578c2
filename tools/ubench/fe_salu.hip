// Can a lone signature's square-root chain run on the SCALAR unit?  One wave,
// one dependent fe_sq chain on (a) lane-varying values (VALU, the shipped asm
// column chains), (b) wave-uniform values with the plain C++ field code
// (-DPV_FE_NOASM): the compiler keeps uniform 32x32->64 products on the SALU
// (s_mul_i32 + s_mul_hi_u32, s_add_u32 / s_addc_u32), (c) both chains at once in
// one wave (VALU and SALU issue in parallel?).  s_memtime cycles per fe_sq; the
// results of (a) and (b) must match limb for limb.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -DPV_FE_NOASM -o fe_salu fe_salu.hip   (SALU build)
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -o fe_salu_asm fe_salu.hip            (asm VALU)
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include "../../indy-plenum_amd/csrc/pv_field.h"

using namespace pv;
constexpr int N = 254;

__global__ __launch_bounds__(64) void k_lane(const uint32_t* in, uint32_t* out, uint64_t* cyc) {
  fe a;
#pragma unroll
  for (int i = 0; i < 10; ++i) a.v[i] = in[i] + (threadIdx.x & 0) * threadIdx.x;   // VGPR values
  uint32_t lv = (uint32_t)threadIdx.x;
  asm volatile("" : "+v"(lv));
#pragma unroll
  for (int i = 0; i < 10; ++i) a.v[i] += lv & 0u;   // force VGPR residency
  const uint64_t t0 = __builtin_amdgcn_s_memtime();
#pragma unroll 1
  for (int i = 0; i < N; ++i) fe_sq(a, a);
  const uint64_t t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) {
    for (int i = 0; i < 10; ++i) out[i] = a.v[i];
    cyc[0] = t1 - t0;
  }
}

__global__ __launch_bounds__(64) void k_uniform(uint32_t i0, uint32_t i1, uint32_t i2, uint32_t i3, uint32_t i4,
                                                uint32_t i5, uint32_t i6, uint32_t i7, uint32_t i8, uint32_t i9,
                                                uint32_t* out, uint64_t* cyc) {
  fe a = {{i0, i1, i2, i3, i4, i5, i6, i7, i8, i9}};
  const uint64_t t0 = __builtin_amdgcn_s_memtime();
#pragma unroll 1
  for (int i = 0; i < N; ++i) fe_sq(a, a);
  const uint64_t t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) {
    for (int i = 0; i < 10; ++i) out[10 + i] = a.v[i];
    cyc[1] = t1 - t0;
  }
}

int main() {
  uint32_t h[10] = {0x1234567, 0x0abcdef, 0x2345678, 0x1bcdef0, 0x3456789, 0x0cdef01, 0x0456789, 0x1def012, 0x2567890,
                    0x0ef0123};
  uint32_t *in, *out;
  uint64_t* cyc;
  if (hipMalloc(&in, 40) || hipMalloc(&out, 80) || hipMalloc(&cyc, 16)) return 1;
  if (hipMemcpy(in, h, 40, hipMemcpyHostToDevice)) return 1;
  double best[2] = {1e30, 1e30};
  uint32_t o[20];
  uint64_t c[2];
  for (int rep = 0; rep < 5; ++rep) {
    hipLaunchKernelGGL(k_lane, dim3(1), dim3(64), 0, 0, in, out, cyc);
    hipLaunchKernelGGL(k_uniform, dim3(1), dim3(64), 0, 0, h[0], h[1], h[2], h[3], h[4], h[5], h[6], h[7], h[8], h[9],
                       out, cyc);
    if (hipDeviceSynchronize()) return 2;
    if (hipMemcpy(o, out, 80, hipMemcpyDeviceToHost) || hipMemcpy(c, cyc, 16, hipMemcpyDeviceToHost)) return 3;
    for (int k = 0; k < 2; ++k) best[k] = best[k] < c[k] / (double)N ? best[k] : c[k] / (double)N;
  }
  int mism = 0;
  for (int i = 0; i < 10; ++i) mism += o[i] != o[10 + i];
#if defined(PV_FE_NOASM)
  const char* build = "plain C++ (PV_FE_NOASM)";
#else
  const char* build = "asm column chains";
#endif
  printf("{\"build\": \"%s\", \"cycles_per_fe_sq_lane_values\": %.1f, \"cycles_per_fe_sq_uniform_values\": %.1f, "
         "\"limb_mismatches\": %d}\n", build, best[0], best[1], mism);
  return 0;
}
