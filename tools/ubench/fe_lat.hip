// Latency of one field operation for a wave ALONE on its SIMD (the latency
// kernels' regime): carry-seeded fe_sq / fe_mul (one dependent MAD chain per
// product) against the latency forms fe_sq_l / fe_mul_l (independent column
// chains interleaved in pairs, carries afterwards).  One wave per CU runs a
// serial chain of N operations; cycles from s_memtime; the two forms' results
// are compared (they must be bit-identical).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -o fe_lat fe_lat.hip
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include "../../indy-plenum_amd/csrc/pv_field.h"

using namespace pv;

#define N_SQ 254
#define N_MUL 64

template <int V>
__global__ __launch_bounds__(64) void k_chain(uint64_t* cyc, uint32_t* out, uint32_t s) {
  const int lane = (int)threadIdx.x;
  fe a, b;
#pragma unroll
  for (int i = 0; i < 10; ++i) {
    a.v[i] = ((lane + 1) * 2654435761u + s * (i + 3)) & ((i & 1) ? M25 : M26);
    b.v[i] = ((lane + 7) * 40503u + s * (i + 11)) & ((i & 1) ? M25 : M26);
  }
  const uint64_t t0 = __builtin_amdgcn_s_memtime();
  if (V == 0) {
#pragma unroll 1
    for (int i = 0; i < N_SQ; ++i) fe_sq(a, a);
  } else if (V == 1) {
#pragma unroll 1
    for (int i = 0; i < N_SQ; ++i) fe_sq_l(a, a);
  } else if (V == 2) {
#pragma unroll 1
    for (int i = 0; i < N_MUL; ++i) fe_mul(a, a, b);
  } else if (V == 3) {
#pragma unroll 1
    for (int i = 0; i < N_MUL; ++i) fe_mul_l(a, a, b);
  } else if (V == 4) {
    fe_pow22523(a, a);
  } else {
    // the latency form of fe_pow22523 (same operation sequence)
    fe z2, z9, z11, t, x, y, c;
    fe_sq_l(z2, a);
    fe_sqn_l(t, z2, 2);
    fe_mul_l(z9, t, a);
    fe_mul_l(z11, z9, z2);
    fe_sq_l(t, z11);
    fe_mul_l(x, t, z9);
    fe_sqn_l(t, x, 5);    fe_mul_l(y, t, x);
    fe_sqn_l(t, y, 10);   fe_mul_l(c, t, y);
    fe_sqn_l(t, c, 20);   fe_mul_l(t, t, c);
    fe_sqn_l(t, t, 10);   fe_mul_l(x, t, y);
    fe_sqn_l(t, x, 50);   fe_mul_l(y, t, x);
    fe_sqn_l(t, y, 100);  fe_mul_l(t, t, y);
    fe_sqn_l(t, t, 50);   fe_mul_l(t, t, x);
    fe_sqn_l(t, t, 2);
    fe_mul_l(a, t, a);
  }
  const uint64_t t1 = __builtin_amdgcn_s_memtime();
#pragma unroll
  for (int i = 0; i < 10; ++i) out[(blockIdx.x * 64 + lane) * 10 + i] = a.v[i];
  if (lane == 0) cyc[blockIdx.x] = t1 - t0;
}

int main() {
  int cus = 256;
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, 0) == hipSuccess) cus = prop.multiProcessorCount;
  uint64_t* cyc;
  uint32_t* out[6];
  if (hipMalloc(&cyc, cus * sizeof(uint64_t)) != hipSuccess) return 1;
  for (int v = 0; v < 6; ++v)
    if (hipMalloc(&out[v], cus * 64 * 10 * sizeof(uint32_t)) != hipSuccess) return 1;
  void (*ks[6])(uint64_t*, uint32_t*, uint32_t) = {k_chain<0>, k_chain<1>, k_chain<2>, k_chain<3>, k_chain<4>, k_chain<5>};
  const char* names[6] = {"fe_sq x254 (seeded)", "fe_sq_l x254", "fe_mul x64 (seeded)", "fe_mul_l x64",
                          "fe_pow22523 (seeded)", "fe_pow22523 latency form"};
  const double ops[6] = {N_SQ, N_SQ, N_MUL, N_MUL, 1, 1};
  uint64_t* h = new uint64_t[cus];
  uint32_t* r[6];
  printf("{\"fe_latency_one_wave\": [\n");
  for (int v = 0; v < 6; ++v) {
    hipLaunchKernelGGL(ks[v], dim3(cus), dim3(64), 0, 0, cyc, out[v], 5u);
    hipLaunchKernelGGL(ks[v], dim3(cus), dim3(64), 0, 0, cyc, out[v], 5u);
    if (hipDeviceSynchronize() != hipSuccess) return 2;
    if (hipMemcpy(h, cyc, cus * sizeof(uint64_t), hipMemcpyDeviceToHost) != hipSuccess) return 3;
    r[v] = new uint32_t[cus * 640];
    if (hipMemcpy(r[v], out[v], cus * 640 * 4, hipMemcpyDeviceToHost) != hipSuccess) return 3;
    double sum = 0;
    for (int k = 0; k < cus; ++k) sum += (double)h[k];
    printf("%s  {\"chain\": \"%s\", \"cycles_per_op\": %.1f}", v ? ",\n" : "", names[v], sum / cus / ops[v]);
  }
  int bad = 0;
  for (int v = 0; v < 6; v += 2)
    for (int k = 0; k < cus * 640; ++k) bad += r[v][k] != r[v + 1][k];
  printf("\n], \"seeded_vs_latency_limb_mismatches\": %d}\n", bad);
  return bad ? 4 : 0;
}
