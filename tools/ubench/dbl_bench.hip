// Doubling-chain throughput at 2/3/4 waves per SIMD (gfx950): the hot op of
// the curve kernel's Horner loop (ge_p2_dbl + ge_p1p1_to_p2), one independent
// point per lane, field code from pv_field.h / pv_curve.h (or a variant).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -o dbl_bench dbl_bench.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstring>
#include "../../indy-plenum_amd/csrc/pv_curve.h"

using namespace pv;

template <int W>
__global__ __launch_bounds__(256, W) void k_dbl(const uint32_t* in, uint32_t* out, int iters) {
  const int t = blockIdx.x * 256 + threadIdx.x;
  ge_p2 r;
#pragma unroll
  for (int i = 0; i < 10; ++i) {
    r.X.v[i] = in[(t % 4096) * 30 + i];
    r.Y.v[i] = in[(t % 4096) * 30 + 10 + i];
    r.Z.v[i] = in[(t % 4096) * 30 + 20 + i];
  }
  ge_p1p1 p;
#pragma unroll 1
  for (int k = 0; k < iters; ++k) {
    ge_p2_dbl(p, r);
    ge_p1p1_to_p2(r, p);
  }
  uint32_t w[8];
  fe_tobytes_w(w, r.Y);
#pragma unroll
  for (int i = 0; i < 8; ++i) out[t * 8 + i] = w[i];
}

template <int W>
double run(const uint32_t* in, uint32_t* out, int cus, int iters) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const int blocks = cus * W;
  hipLaunchKernelGGL((k_dbl<W>), dim3(blocks), dim3(256), 0, 0, in, out, 8);
  float best = 1e30f;
  for (int r = 0; r < 3; ++r) {
    hipEventRecord(e0);
    hipLaunchKernelGGL((k_dbl<W>), dim3(blocks), dim3(256), 0, 0, in, out, iters);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    best = ms < best ? ms : best;
  }
  return (double)blocks * 256 * iters / (best * 1e-3);
}

int main() {
  int cus = 256;
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, 0) == hipSuccess) cus = prop.multiProcessorCount;
  const int nin = 4096 * 30;
  uint32_t* hin = new uint32_t[nin];
  uint32_t s = 12345;
  for (int i = 0; i < nin; ++i) {
    s = s * 1664525u + 1013904223u;
    hin[i] = s & ((i % 2) ? M25 : M26);
  }
  uint32_t *in, *out;
  hipMalloc(&in, nin * 4);
  hipMalloc(&out, (size_t)cus * 8 * 256 * 8 * 4);
  hipMemcpy(in, hin, nin * 4, hipMemcpyHostToDevice);
  const int iters = 2048;
  double r2 = run<2>(in, out, cus, iters), r3 = run<3>(in, out, cus, iters), r4 = run<4>(in, out, cus, iters),
         r5 = run<5>(in, out, cus, iters);
  // 4 sq + 3 mul per doubling
  printf("{\"dbl_per_s\": {\"w2\": %.4e, \"w3\": %.4e, \"w4\": %.4e, \"w5\": %.4e}, \"mad_per_s\": {\"w2\": %.4e, "
         "\"w3\": %.4e, \"w4\": %.4e, \"w5\": %.4e}}\n", r2, r3, r4, r5, r2 * 520, r3 * 520, r4 * 520, r5 * 520);
  return 0;
}
