// Instruction-level parallelism in the field code of k_curve_half (gfx950).
//  1. v_mad_u64_u32 result latency: ONE dependent chain per wave vs 2 and 8
//     interleaved chains, at 1 and 2 waves per SIMD (cycles per MAD per wave
//     from s_memtime).
//  2. The Horner doubling (ge_p2_dbl + ge_p1p1_to_p2: 4 squarings + 3
//     multiplies) with the production one-chain-per-product field code vs the
//     fused forms (fe_sq2 / fe_mul2 / fe_mul3: C products' column chains
//     interleaved in one asm block), 2 waves per SIMD, results cross-checked.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -o fe_ilp fe_ilp.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstring>
#include "../../indy-plenum_amd/csrc/pv_curve.h"

using namespace pv;

template <int CH>
__global__ __launch_bounds__(256) void k_chain(uint64_t* cyc, uint32_t* sink, uint32_t s, int iters) {
  uint64_t acc[CH];
  uint32_t a = threadIdx.x * 2654435761u + s, b = a ^ 0x9e3779b9u;
#pragma unroll
  for (int c = 0; c < CH; ++c) acc[c] = a + c;
  const uint64_t t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int u = 0; u < 64 / CH; ++u) {
#pragma unroll
      for (int c = 0; c < CH; ++c) asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, %0" : "+v"(acc[c]) : "v"(a), "v"(b) : "vcc");
    }
  }
  const uint64_t t1 = __builtin_amdgcn_s_memtime();
  uint32_t r = 0;
#pragma unroll
  for (int c = 0; c < CH; ++c) r ^= (uint32_t)acc[c];
  sink[blockIdx.x * 256 + threadIdx.x] = r;
  if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * 4 + threadIdx.x / 64] = t1 - t0;
}

template <int CH>
void chain(int cus, int wps) {
  uint64_t* cyc;
  uint32_t* sink;
  const int blocks = cus * wps, iters = 2000;
  hipMalloc(&cyc, blocks * 4 * 8);
  hipMalloc(&sink, blocks * 256 * 4);
  hipLaunchKernelGGL(k_chain<CH>, dim3(blocks), dim3(256), 0, 0, cyc, sink, 1u, 10);
  hipLaunchKernelGGL(k_chain<CH>, dim3(blocks), dim3(256), 0, 0, cyc, sink, 1u, iters);
  hipDeviceSynchronize();
  uint64_t* h = new uint64_t[blocks * 4];
  hipMemcpy(h, cyc, blocks * 4 * 8, hipMemcpyDeviceToHost);
  double sum = 0;
  for (int i = 0; i < blocks * 4; ++i) sum += h[i];
  // s_memtime ticks at the shader clock on gfx9
  const double per = sum / (blocks * 4) / ((double)iters * 64);
  printf("{\"test\": \"mad_chain\", \"chains\": %d, \"waves_per_simd\": %d, \"cycles_per_mad_per_wave\": %.3f}\n", CH, wps,
         per);
  delete[] h;
  hipFree(cyc);
  hipFree(sink);
}

template <int V>
__device__ __forceinline__ void dbl(ge_p2& r2) {
  if constexpr (V == 0) {
    ge_p1p1 p;
    ge_p2_dbl(p, r2);
    ge_p1p1_to_p2(r2, p);
  } else {
    fe xx, yy, zz2, xy2, t, X, Y, Z, T;
    fe_add(t, r2.X, r2.Y);
    fe_sq2(xx, r2.X, yy, r2.Y);
    fe_sq2(zz2, r2.Z, xy2, t);
    fe_add(Y, yy, xx);
    fe_sub(Z, yy, xx);
    fe_sub4(X, xy2, Y);
    fe_add(t, zz2, zz2);
    fe_sub4(T, t, Z);
    fe_carry(T);
    if constexpr (V == 1) {
      fe_mul3(r2.X, X, T, r2.Y, Y, Z, r2.Z, Z, T);
    } else {
      fe_mul2(r2.X, X, T, r2.Y, Y, Z);
      fe_mul(r2.Z, Z, T);
    }
  }
}

template <int V>
__global__ __launch_bounds__(256, 2) void k_dbl(const uint32_t* in, uint32_t* out, int iters) {
  const int t = blockIdx.x * 256 + threadIdx.x;
  ge_p2 r;
#pragma unroll
  for (int i = 0; i < 10; ++i) {
    r.X.v[i] = in[(t % 4096) * 30 + i];
    r.Y.v[i] = in[(t % 4096) * 30 + 10 + i];
    r.Z.v[i] = in[(t % 4096) * 30 + 20 + i];
  }
#pragma unroll 1
  for (int k = 0; k < iters; ++k) dbl<V>(r);
  uint32_t w[8];
  fe_tobytes_w(w, r.Y);
#pragma unroll
  for (int i = 0; i < 8; ++i) out[t * 8 + i] = w[i];
}

template <int V>
void run(const char* name, const uint32_t* in, uint32_t* out, int cus, const uint32_t* ref, uint32_t* host) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const int blocks = cus * 2, iters = 512;
  hipLaunchKernelGGL(k_dbl<V>, dim3(blocks), dim3(256), 0, 0, in, out, 8);
  float best = 1e30f;
  for (int r = 0; r < 3; ++r) {
    hipEventRecord(e0);
    hipLaunchKernelGGL(k_dbl<V>, dim3(blocks), dim3(256), 0, 0, in, out, iters);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    best = ms < best ? ms : best;
  }
  hipLaunchKernelGGL(k_dbl<V>, dim3(64), dim3(256), 0, 0, in, out, 37);
  hipMemcpy(host, out, 64 * 256 * 8 * 4, hipMemcpyDeviceToHost);
  const bool ok = memcmp(host, ref, 64 * 256 * 8 * 4) == 0;
  const double dps = (double)blocks * 256 * iters / (best * 1e-3);
  printf("{\"test\": \"dbl\", \"variant\": \"%s\", \"waves_per_simd\": 2, \"ok\": %s, \"dbl_per_s\": %.4e, "
         "\"mad_per_s\": %.4e}\n", name, ok ? "true" : "false", dps, dps * 520.0);
}

// two independent squaring chains (the two pow22523 of decompressing -A and
// -R): one after the other (production) vs interleaved with fe_sq2
template <int V>
__global__ __launch_bounds__(256, 2) void k_sqc(const uint32_t* in, uint32_t* out, int iters) {
  const int t = blockIdx.x * 256 + threadIdx.x;
  fe x, y;
#pragma unroll
  for (int i = 0; i < 10; ++i) {
    x.v[i] = in[(t % 4096) * 30 + i];
    y.v[i] = in[(t % 4096) * 30 + 10 + i];
  }
  if constexpr (V == 0) {
#pragma unroll 1
    for (int k = 0; k < iters; ++k) fe_sq(x, x);
#pragma unroll 1
    for (int k = 0; k < iters; ++k) fe_sq(y, y);
  } else {
#pragma unroll 1
    for (int k = 0; k < iters; ++k) fe_sq2(x, x, y, y);
  }
  uint32_t w[8];
  fe_add(x, x, y);
  fe_tobytes_w(w, x);
#pragma unroll
  for (int i = 0; i < 8; ++i) out[t * 8 + i] = w[i];
}

template <int V>
void run_sq(const char* name, const uint32_t* in, uint32_t* out, int cus, const uint32_t* ref, uint32_t* host) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const int blocks = cus * 2, iters = 1024;
  float best = 1e30f;
  for (int r = 0; r < 4; ++r) {
    hipEventRecord(e0);
    hipLaunchKernelGGL(k_sqc<V>, dim3(blocks), dim3(256), 0, 0, in, out, iters);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    best = ms < best ? ms : best;
  }
  hipLaunchKernelGGL(k_sqc<V>, dim3(64), dim3(256), 0, 0, in, out, 37);
  hipMemcpy(host, out, 64 * 256 * 8 * 4, hipMemcpyDeviceToHost);
  const bool ok = memcmp(host, ref, 64 * 256 * 8 * 4) == 0;
  const double sps = 2.0 * blocks * 256 * iters / (best * 1e-3);
  printf("{\"test\": \"sq_chains\", \"variant\": \"%s\", \"waves_per_simd\": 2, \"ok\": %s, \"sq_per_s\": %.4e, "
         "\"mad_per_s\": %.4e}\n", name, ok ? "true" : "false", sps, sps * 55.0);
}

int main() {
  int cus = 256;
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, 0) == hipSuccess) cus = prop.multiProcessorCount;
  chain<1>(cus, 1);
  chain<2>(cus, 1);
  chain<8>(cus, 1);
  chain<1>(cus, 2);
  chain<2>(cus, 2);
  chain<8>(cus, 2);
  const int nin = 4096 * 30;
  uint32_t* hin = new uint32_t[nin];
  uint32_t s = 12345;
  for (int i = 0; i < nin; ++i) {
    s = s * 1664525u + 1013904223u;
    hin[i] = s & ((i % 2) ? M25 : M26);
  }
  uint32_t *in, *out;
  hipMalloc(&in, nin * 4);
  hipMalloc(&out, (size_t)cus * 2 * 256 * 8 * 4);
  hipMemcpy(in, hin, nin * 4, hipMemcpyHostToDevice);
  uint32_t* ref = new uint32_t[64 * 256 * 8];
  uint32_t* host = new uint32_t[64 * 256 * 8];
  hipLaunchKernelGGL(k_sqc<0>, dim3(64), dim3(256), 0, 0, in, out, 37);
  hipMemcpy(ref, out, 64 * 256 * 8 * 4, hipMemcpyDeviceToHost);
  for (int rep = 0; rep < 2; ++rep) {
    run_sq<0>("serial", in, out, cus, ref, host);
    run_sq<1>("sq2", in, out, cus, ref, host);
  }
  hipLaunchKernelGGL(k_dbl<0>, dim3(64), dim3(256), 0, 0, in, out, 37);
  hipMemcpy(ref, out, 64 * 256 * 8 * 4, hipMemcpyDeviceToHost);
  for (int rep = 0; rep < 2; ++rep) {
    run<0>("production", in, out, cus, ref, host);
    run<1>("sq2_mul3", in, out, cus, ref, host);
    run<2>("sq2_mul2", in, out, cus, ref, host);
  }
  return 0;
}
