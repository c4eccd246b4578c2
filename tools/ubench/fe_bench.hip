// Field-multiply / square variant benchmark (gfx950): time per fe op for
// alternative formulations of the radix-2^25.5 multiply, at a fixed number of
// waves per SIMD, with outputs cross-checked against the production fe_mul.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -o fe_bench fe_bench.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstring>
#include "../../indy-plenum_amd/csrc/pv_field.h"

using namespace pv;

#define FENCE() __builtin_amdgcn_sched_barrier(0)

__device__ __forceinline__ uint32_t dbl32(uint32_t x) {
  uint32_t r;
  asm volatile("v_add_u32 %0, %1, %1" : "=v"(r) : "v"(x));
  return r;
}

// V1: production product, doublings as v_add instead of v_lshlrev
__device__ __forceinline__ void mul_v1(fe& h, const fe& f, const fe& g) {
  uint32_t g19[10], f2[10];
#pragma unroll
  for (int j = 1; j < 10; ++j) g19[j] = 19u * g.v[j];
#pragma unroll
  for (int i = 1; i < 10; i += 2) f2[i] = dbl32(f.v[i]);
  uint64_t acc[10];
#pragma unroll
  for (int k = 0; k < 10; ++k) acc[k] = 0;
#pragma unroll
  for (int i = 0; i < 10; ++i)
#pragma unroll
    for (int j = 0; j < 10; ++j) {
      const bool oo = (i & 1) && (j & 1);
      const uint32_t a = oo ? f2[i] : f.v[i];
      const int k = i + j;
      if (k < 10) acc[k] += mul32x32(a, g.v[j]);
      else acc[k - 10] += mul32x32(a, g19[j]);
    }
  fe_carry_wide(h, acc);
  FENCE();
}

// V2: serial 11-step carry chain (0..9, wrap, 0) instead of the interleaved 12
__device__ __forceinline__ void carry_serial(fe& out, uint64_t h[10]) {
  uint64_t c;
#pragma unroll
  for (int k = 0; k < 9; ++k) {
    const int r = (k & 1) ? 25 : 26;
    c = h[k] >> r;
    h[k + 1] += c;
    h[k] &= (k & 1) ? M25 : M26;
  }
  c = h[9] >> 25; h[9] &= M25; h[0] += c * 19;
  c = h[0] >> 26; h[0] &= M26; h[1] += c;
#pragma unroll
  for (int i = 0; i < 10; ++i) out.v[i] = (uint32_t)h[i];
}
__device__ __forceinline__ void mul_v2(fe& h, const fe& f, const fe& g) {
  uint32_t g19[10], f2[10];
#pragma unroll
  for (int j = 1; j < 10; ++j) g19[j] = 19u * g.v[j];
#pragma unroll
  for (int i = 1; i < 10; i += 2) f2[i] = dbl32(f.v[i]);
  uint64_t acc[10];
#pragma unroll
  for (int k = 0; k < 10; ++k) acc[k] = 0;
#pragma unroll
  for (int i = 0; i < 10; ++i)
#pragma unroll
    for (int j = 0; j < 10; ++j) {
      const bool oo = (i & 1) && (j & 1);
      const uint32_t a = oo ? f2[i] : f.v[i];
      const int k = i + j;
      if (k < 10) acc[k] += mul32x32(a, g.v[j]);
      else acc[k - 10] += mul32x32(a, g19[j]);
    }
  carry_serial(h, acc);
  FENCE();
}

// V3: columns in order, each column's first product takes the previous
// column's carry as the 64-bit addend (the carry add rides in a v_mad_u64_u32)
__device__ __forceinline__ void mul_v3(fe& h, const fe& f, const fe& g) {
  uint32_t g19[10], f2[10];
#pragma unroll
  for (int j = 1; j < 10; ++j) g19[j] = 19u * g.v[j];
#pragma unroll
  for (int i = 1; i < 10; i += 2) f2[i] = dbl32(f.v[i]);
  uint64_t carry = 0;
  uint32_t out[10];
#pragma unroll
  for (int k = 0; k < 10; ++k) {
    uint64_t acc = carry;
#pragma unroll
    for (int i = 0; i < 10; ++i) {
      const int j = (k - i + 10) % 10;
      const bool wrap = i + j >= 10;
      const bool oo = (i & 1) && (j & 1);
      const uint32_t a = oo ? f2[i] : f.v[i];
      acc += mul32x32(a, wrap ? g19[j] : g.v[j]);
    }
    const int r = (k & 1) ? 25 : 26;
    carry = acc >> r;
    out[k] = (uint32_t)acc & ((k & 1) ? M25 : M26);
  }
  // wrap: out0 += 19 * carry (carry < 2^39), then one more carry into out1
  uint64_t t = (uint64_t)out[0] + carry * 19u;
  out[0] = (uint32_t)t & M26;
  out[1] += (uint32_t)(t >> 26);
#pragma unroll
  for (int i = 0; i < 10; ++i) h.v[i] = out[i];
  FENCE();
}

template <int V>
__device__ __forceinline__ void mulv(fe& h, const fe& f, const fe& g) {
  if (V == 0) fe_mul(h, f, g);
  else if (V == 1) mul_v1(h, f, g);
  else if (V == 2) mul_v2(h, f, g);
  else mul_v3(h, f, g);
}

template <int V, int W>
__global__ __launch_bounds__(256, W) void k_mul(const uint32_t* in, uint32_t* out, int iters) {
  const int t = blockIdx.x * 256 + threadIdx.x;
  fe a, b, c;
#pragma unroll
  for (int i = 0; i < 10; ++i) {
    a.v[i] = in[(t % 4096) * 30 + i];
    b.v[i] = in[(t % 4096) * 30 + 10 + i];
    c.v[i] = in[(t % 4096) * 30 + 20 + i];
  }
#pragma unroll 1
  for (int k = 0; k < iters; ++k) {
    mulv<V>(a, a, b);   // a <- a*b
    mulv<V>(b, b, c);   // b <- b*c   (independent second chain)
  }
  uint32_t w[8];
  fe_tobytes_w(w, a);
#pragma unroll
  for (int i = 0; i < 8; ++i) out[t * 16 + i] = w[i];
  fe_tobytes_w(w, b);
#pragma unroll
  for (int i = 0; i < 8; ++i) out[t * 16 + 8 + i] = w[i];
}

template <int V, int W>
float run(const uint32_t* in, uint32_t* out, int blocks, int iters, hipEvent_t e0, hipEvent_t e1) {
  hipLaunchKernelGGL((k_mul<V, W>), dim3(blocks), dim3(256), 0, 0, in, out, 4);
  hipEventRecord(e0);
  hipLaunchKernelGGL((k_mul<V, W>), dim3(blocks), dim3(256), 0, 0, in, out, iters);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  return ms;
}

template <int V>
void one(const char* name, const uint32_t* in, uint32_t* out, uint32_t* ref, uint32_t* host, int cus) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const int iters = 256;
  float ms2 = run<V, 2>(in, out, cus * 2, iters, e0, e1);
  float ms3 = run<V, 3>(in, out, cus * 3, iters, e0, e1);
  float ms4 = run<V, 4>(in, out, cus * 4, iters, e0, e1);
  // correctness: fixed grid, compare with V0 output
  hipLaunchKernelGGL((k_mul<V, 2>), dim3(64), dim3(256), 0, 0, in, out, 37);
  hipMemcpy(host, out, 64 * 256 * 16 * 4, hipMemcpyDeviceToHost);
  const bool ok = memcmp(host, ref, 64 * 256 * 16 * 4) == 0;
  auto per = [&](float ms, int w) { return ms * 1e6 / ((double)cus * w * 256 * iters * 2); };  // ns per mul per lane
  printf("  {\"variant\": \"%s\", \"ok\": %s, \"ns_per_mul_lane_w2\": %.5f, \"w3\": %.5f, \"w4\": %.5f, "
         "\"chip_muls_per_s_w2\": %.4e, \"w3\": %.4e, \"w4\": %.4e},\n",
         name, ok ? "true" : "false", per(ms2, 2), per(ms3, 3), per(ms4, 4),
         (double)cus * 2 * 256 * iters * 2 / (ms2 * 1e-3), (double)cus * 3 * 256 * iters * 2 / (ms3 * 1e-3),
         (double)cus * 4 * 256 * iters * 2 / (ms4 * 1e-3));
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
    hin[i] = s & ((i % 2) ? M25 : M26);  // TIGHT random limbs
  }
  uint32_t *in, *out;
  hipMalloc(&in, nin * 4);
  hipMalloc(&out, (size_t)cus * 4 * 256 * 16 * 4);
  hipMemcpy(in, hin, nin * 4, hipMemcpyHostToDevice);
  uint32_t* ref = new uint32_t[64 * 256 * 16];
  uint32_t* host = new uint32_t[64 * 256 * 16];
  hipLaunchKernelGGL((k_mul<0, 2>), dim3(64), dim3(256), 0, 0, in, out, 37);
  hipMemcpy(ref, out, 64 * 256 * 16 * 4, hipMemcpyDeviceToHost);
  printf("{\"fe_mul_variants\": [\n");
  one<0>("v0_production", in, out, ref, host, cus);
  one<1>("v1_add_doubling", in, out, ref, host, cus);
  one<2>("v2_serial_carry", in, out, ref, host, cus);
  one<3>("v3_column_carry_in_mad", in, out, ref, host, cus);
  printf("  {}\n]}\n");
  return 0;
}
