// Field-multiply / square formulations inside the hot op of k_curve_half (a
// p2 doubling + p1p1 -> p2, the 128-doubling Horner chain), gfx950.
// One independent point per lane, 2 or 3 waves per SIMD (the curve kernel's
// register budget), doublings/s and the implied v_mad_u64_u32 rate, outputs
// cross-checked against the production field code (pv_field.h).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -o fe_variants fe_variants.hip
//   ./fe_variants        -> one JSON line per (variant, waves)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstring>
#include "../../indy-plenum_amd/csrc/pv_curve.h"

using namespace pv;

// 64-bit accumulate of a 32x32 product as ONE v_mad_u64_u32 whose addend is
// the running sum: the compiler cannot reassociate an asm statement, so the
// column's carry stays the first addend instead of becoming a trailing
// v_lshl_add_u64.
__device__ __forceinline__ uint64_t mad(uint32_t a, uint32_t b, uint64_t c) {
  uint64_t d;
  asm("v_mad_u64_u32 %0, vcc, %1, %2, %3" : "=v"(d) : "v"(a), "v"(b), "v"(c) : "vcc");
  return d;
}
__device__ __forceinline__ uint64_t mul0(uint32_t a, uint32_t b) {
  uint64_t d;
  asm("v_mad_u64_u32 %0, vcc, %1, %2, 0" : "=v"(d) : "v"(a), "v"(b) : "vcc");
  return d;
}

// ---- variant A: production products, columns as asm chains seeded by the carry
__device__ __forceinline__ void mul_a(fe& h, const fe& f, const fe& g) {
  uint32_t g19[10], f2[10];
#pragma unroll
  for (int j = 1; j < 10; ++j) g19[j] = 19u * g.v[j];
#pragma unroll
  for (int i = 1; i < 10; i += 2) f2[i] = 2u * f.v[i];
  uint64_t carry = 0;
  uint32_t out[10];
#pragma unroll
  for (int k = 0; k < 10; ++k) {
    uint64_t acc = 0;
#pragma unroll
    for (int i = 0; i < 10; ++i) {
      const int j = (k - i + 10) % 10;
      const bool oo = (i & 1) && (j & 1);
      const uint32_t a = oo ? f2[i] : f.v[i];
      const uint32_t b = i + j >= 10 ? g19[j] : g.v[j];
      acc = (k == 0 && i == 0) ? mul0(a, b) : mad(a, b, i == 0 ? carry : acc);
    }
    carry = acc >> ((k & 1) ? 25 : 26);
    out[k] = (uint32_t)acc & ((k & 1) ? M25 : M26);
  }
  fe_finish_columns(h, carry, out);
  PV_FE_FENCE();
}

__device__ __forceinline__ void sq_a(fe& h, const fe& f) {
  uint32_t f2[10], f19[10], f4[10];
#pragma unroll
  for (int i = 0; i < 10; ++i) f2[i] = 2u * f.v[i];
#pragma unroll
  for (int i = 5; i < 10; ++i) f19[i] = 19u * f.v[i];
#pragma unroll
  for (int i = 1; i < 10; i += 2) f4[i] = 4u * f.v[i];
  uint64_t carry = 0;
  uint32_t out[10];
#pragma unroll
  for (int k = 0; k < 10; ++k) {
    uint64_t acc = 0;
    bool first = true;
#pragma unroll
    for (int i = 0; i < 10; ++i) {
#pragma unroll
      for (int j = i; j < 10; ++j) {
        if ((i + j) % 10 != k) continue;
        const bool oo = (i & 1) && (j & 1);
        const bool wrap = i + j >= 10;
        uint32_t a, b;
        if (i == j) {
          if (!wrap) { a = f.v[i]; b = oo ? f2[i] : f.v[i]; }
          else { a = oo ? f2[i] : f.v[i]; b = f19[i]; }
        } else {
          a = oo ? f4[i] : f2[i];
          b = wrap ? f19[j] : f.v[j];
        }
        acc = (k == 0 && first) ? mul0(a, b) : mad(a, b, first ? carry : acc);
        first = false;
      }
    }
    carry = acc >> ((k & 1) ? 25 : 26);
    out[k] = (uint32_t)acc & ((k & 1) ? M25 : M26);
  }
  fe_finish_columns(h, carry, out);
  PV_FE_FENCE();
}

// ---- variant B: A without the per-op scheduling fence (the compiler may
// interleave consecutive independent field ops)
__device__ __forceinline__ void mul_b(fe& h, const fe& f, const fe& g) {
  uint32_t g19[10], f2[10];
#pragma unroll
  for (int j = 1; j < 10; ++j) g19[j] = 19u * g.v[j];
#pragma unroll
  for (int i = 1; i < 10; i += 2) f2[i] = 2u * f.v[i];
  uint64_t carry = 0;
  uint32_t out[10];
#pragma unroll
  for (int k = 0; k < 10; ++k) {
    uint64_t acc = 0;
#pragma unroll
    for (int i = 0; i < 10; ++i) {
      const int j = (k - i + 10) % 10;
      const bool oo = (i & 1) && (j & 1);
      const uint32_t a = oo ? f2[i] : f.v[i];
      const uint32_t b = i + j >= 10 ? g19[j] : g.v[j];
      acc = (k == 0 && i == 0) ? mul0(a, b) : mad(a, b, i == 0 ? carry : acc);
    }
    carry = acc >> ((k & 1) ? 25 : 26);
    out[k] = (uint32_t)acc & ((k & 1) ? M25 : M26);
  }
  fe_finish_columns(h, carry, out);
}

// ---- the doubling with a pluggable field layer (same sequence as pv_curve.h)
template <int V>
__device__ __forceinline__ void MUL(fe& h, const fe& f, const fe& g) {
  if constexpr (V == 0) fe_mul(h, f, g);
  else if constexpr (V == 1) mul_a(h, f, g);
  else mul_b(h, f, g);
}
template <int V>
__device__ __forceinline__ void SQ(fe& h, const fe& f) {
  if constexpr (V == 0) fe_sq(h, f);
  else sq_a(h, f);
}

template <int V>
__device__ __forceinline__ void dbl(ge_p2& r2) {
  fe xx, yy, zz2, xy2, t, X, Y, Z, T;
  SQ<V>(xx, r2.X);
  SQ<V>(yy, r2.Y);
  SQ<V>(zz2, r2.Z);
  fe_add(t, r2.X, r2.Y);
  SQ<V>(xy2, t);
  fe_add(Y, yy, xx);
  fe_sub(Z, yy, xx);
  fe_sub4(X, xy2, Y);
  fe_add(t, zz2, zz2);
  fe_sub4(T, t, Z);
  fe_carry(T);
  MUL<V>(r2.X, X, T);
  MUL<V>(r2.Y, Y, Z);
  MUL<V>(r2.Z, Z, T);
}

template <int V, int W>
__global__ __launch_bounds__(256, W) void k_dbl(const uint32_t* in, uint32_t* out, int iters) {
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

template <int V, int W>
void run(const char* name, const uint32_t* in, uint32_t* out, int cus, const uint32_t* ref, uint32_t* host) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const int blocks = cus * W, iters = 512;
  hipLaunchKernelGGL((k_dbl<V, W>), dim3(blocks), dim3(256), 0, 0, in, out, 8);
  float best = 1e30f;
  for (int r = 0; r < 3; ++r) {
    hipEventRecord(e0);
    hipLaunchKernelGGL((k_dbl<V, W>), dim3(blocks), dim3(256), 0, 0, in, out, iters);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    best = ms < best ? ms : best;
  }
  hipLaunchKernelGGL((k_dbl<V, W>), dim3(64), dim3(256), 0, 0, in, out, 37);
  hipMemcpy(host, out, 64 * 256 * 8 * 4, hipMemcpyDeviceToHost);
  const bool ok = memcmp(host, ref, 64 * 256 * 8 * 4) == 0;
  const double dps = (double)blocks * 256 * iters / (best * 1e-3);
  printf("{\"variant\": \"%s\", \"waves_per_simd\": %d, \"ok\": %s, \"dbl_per_s\": %.4e, \"mad_per_s\": %.4e}\n", name,
         W, ok ? "true" : "false", dps, dps * 520.0);
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
  hipMalloc(&out, (size_t)cus * 4 * 256 * 8 * 4);
  hipMemcpy(in, hin, nin * 4, hipMemcpyHostToDevice);
  uint32_t* ref = new uint32_t[64 * 256 * 8];
  uint32_t* host = new uint32_t[64 * 256 * 8];
  hipLaunchKernelGGL((k_dbl<0, 2>), dim3(64), dim3(256), 0, 0, in, out, 37);
  hipMemcpy(ref, out, 64 * 256 * 8 * 4, hipMemcpyDeviceToHost);
  run<0, 2>("production", in, out, cus, ref, host);
  run<1, 2>("asm_carry_chain", in, out, cus, ref, host);
  run<2, 2>("asm_carry_chain_nofence_mul", in, out, cus, ref, host);
  run<0, 3>("production", in, out, cus, ref, host);
  run<1, 3>("asm_carry_chain", in, out, cus, ref, host);
  return 0;
}
