// HIP kernels for gfx950 (MI355X): batch Ed25519 verification with
// libsodium-1.0.18 verdict semantics, batch keygen/sign, n-f quorum tally.
//
// Verify = two launches, one lane per signature:
//   k_hash  : pre-checks (S < L, R/A not small order, A canonical) and
//             h = SHA-512(R || A || M) mod L                  
//   k_curve : -A = decompress(A), R' = h(-A) + S B by a FIXED signed-digit
//             schedule (A: radix 16, 9-entry per-lane table in scratch;
//             B: radix 256, 129-entry niels table in LDS), then
//             encode(R') == R                                 (steps 4, 6, 7)
// Every lane runs the same window schedule (digit 0 adds the identity), so
// a wavefront never diverges inside the scalar multiplication.  The
// per-signature algorithms live in pv_verify_core.h.
#include <hip/hip_runtime.h>
#include "pv_verify_core.h"
#include "pv_quad.h"
#include "pv_sha256.h"
#include "pv_kernels.h"

namespace pv {

// waves per SIMD the curve kernel is compiled for (register budget 512 / w);
// its hot Horner loop needs ~165 VGPRs; 2 waves/SIMD (<= 256 VGPRs) measured
// fastest (tools/variant_bench.py: 2 > 3 > 4 waves once spills appear)
#ifndef PV_HALF_LS
// lane interleave of k_curve_half's per-lane tables: 1 = lane-contiguous (the
// compiler loads a field element with dwordx4/x2); 64 = [word][lane] measured
// 40 % slower (10 dword loads + address arithmetic per field element,
// tools/variant_bench.py, profiles/r01_ab_layout.json)
#define PV_HALF_LS 1
#endif
#ifndef PV_CURVE_WAVES
#define PV_CURVE_WAVES 2
#endif

static_assert(KEYTAB_WIDE_WORDS == KEYW_WORDS && KEYTAB_WIDE_SCRATCH == KEYW_SCRATCH && KEYTAB_WORDS == KEY_WORDS &&
                  KEYTAB_WIDE_LANES == COMB_Q * KW_SLICES && KEYTAB_WIDE_LANES % 64 == 0,
              "prepared-key layouts");
static_assert(BT_ENTRIES == BTAB_ENTRIES && BT_WORDS == BTAB_WORDS && LANE_WORDS == ATAB_WORDS &&
                  AT_WORDS == ATAB_LAT_WORDS &&
                  KEY_WORDS == KEYTAB_WORDS && KEY_SCRATCH == KEYTAB_SCRATCH && BT_CHUNKS == BTAB_CHUNKS &&
                  HREC_WORDS == HSREC_WORDS && HALF_LANE_WORDS == HALF_SCRATCH_WORDS &&
                  BW_ENTRIES == BWTAB_ENTRIES,
              "table layout");

// ------------------------------------------------------------- hash kernel
// Persistent lanes with per-lane refill: each lane runs ONE SHA-512
// compression of its current message per loop trip and, when that message is
// done, stores the digest and takes the next message index from a
// wave-private chunk of the global queue (wq_take below).  Ragged message
// lengths (C4: 2..33 blocks) then cost no SIMD divergence: a lane never waits
// for a longer message in its wavefront, only the final drain is ragged.
__device__ __forceinline__ uint64_t readlane64(unsigned long long v, int lane) {
  return ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), lane) << 32) |
         (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, lane);
}

// Base index of a wave's __popcll(m) entries appended at *counter (m = the
// wave's nonzero ballot; call with the whole wavefront active): the first
// set lane adds, every lane reads its result with v_readlane at that
// (uniform) lane index -- no cross-lane shuffle through LDS.
__device__ __forceinline__ uint64_t wave_append(unsigned long long* counter, uint64_t m) {
  const int leader = __ffsll((unsigned long long)m) - 1;
  unsigned long long b = 0;
  if ((int)(threadIdx.x & 63u) == leader) b = atomicAdd(counter, (unsigned long long)__popcll(m));
  return readlane64(b, leader);
}

// Wave-private chunks of the global message queue: the wave takes a chunk of
// indices with one atomic and hands them out to its lanes by ballot rank; the
// atomic for the NEXT chunk is issued when a chunk is opened and its result is
// only read (v_readlane of lane 0) when that chunk is exhausted, so no lane
// ever waits for an atomic round trip (k_hash refilled on nearly every trip on
// C4 and waited for take_index's atomic each time).  Must be called with the
// whole wavefront active (convergent code).
// Chunk sizes (PV_HASH_GUIDED = 1) follow the batch's mean message length and
// what is left.  A chunk holds about 16 x 64 blocks of work: 64 x max(1, 16 /
// (mean blocks per message)) indices (mean from off[0], off[n]), so short
// messages (C3: one SHA-512 block each -- at a fixed 64, one atomic per wave
// per trip, all on one counter) take up to 1024 indices per atomic, while long
// ones (C4: ~17 blocks) keep 64 and the waves' chunks in flight stay in a
// narrow window of the blob; and never more than (indices left) / (2 x waves
// of the grid), so the last chunks are 64 and the grid's tail stays one
// message per lane.  Measured (profiles/r06_ab_hash_chunk.jsonl,
// r06_ab_hash_guided.jsonl): a fixed 256 cut C3's k_hash 0.62 -> 0.41 ms but
// made C2's 0.46 -> 0.58 ms (1M / 256 chunks are ~1.3 per wave); sizing by
// what is left alone (up to 1024 from the start) gave C3 0.42, C2 0.43, f3's
// leaf kernel 0.41 -> 0.38 ms, but C4 15.1 -> 16.3 ms (every wave streaming
// its own far-apart MBs of a 17 GB blob); a trip-count estimate of the length
// misjudged every wave's first chunk.  PV_HASH_GUIDED = 0: fixed chunks of
// PV_HASH_CHUNK.  k_sha256 keeps fixed chunks (G = false): its f3 leaf kernel
// (5-block messages) measured 0.41 ms with them and 0.44-0.45 with the sized
// ones (profiles/r06_ab_f3_queue.jsonl).
#ifndef PV_HASH_CHUNK
#define PV_HASH_CHUNK 64
#endif
#ifndef PV_HASH_GUIDED
#define PV_HASH_GUIDED 1
#endif
struct WaveQueue {
  uint64_t cb;     // current chunk base
  uint32_t cs;     // current chunk size
  uint32_t cu;     // indices of the current chunk already handed out
  uint64_t nbv;    // lane 0: base of the next chunk (atomic in flight)
  uint32_t ns;     // size of the next chunk (wave-uniform)
  uint32_t fit;    // chunk size for the batch's mean message length
  uint64_t n;      // queue length
  float rw2;       // 1 / (2 x waves of the grid)
};

// chunk size for a mean of `blocks` compressions per message
__device__ __forceinline__ uint32_t wq_fit(uint64_t blocks) {
  const uint64_t per = 16 / (blocks < 1 ? 1 : blocks);
  return 64u * (uint32_t)(per < 1 ? 1 : per);
}

// size of a chunk starting at `base`: q.fit capped by what is left (G), or a
// fixed PV_HASH_CHUNK
template <bool G>
__device__ __forceinline__ uint32_t wq_size(const WaveQueue& q, uint64_t base) {
  if (G) {
    const uint64_t left = q.n > base ? q.n - base : 0;
    uint64_t g = (uint64_t)((float)left * q.rw2) & ~63ull;   // a heuristic: no exact division needed
    if (g > q.fit) g = q.fit;
    return (uint32_t)(g < 64 ? 64 : (g > 1024 ? 1024 : g));
  }
  return (uint32_t)PV_HASH_CHUNK;
}

template <bool G>
__device__ __forceinline__ void wq_init(WaveQueue& q, unsigned long long* counter, uint64_t n, uint32_t fit) {
  const int lane = (int)(threadIdx.x & 63u);
  q.n = n;
  q.rw2 = 1.0f / (float)(2u * gridDim.x * (blockDim.x / 64u));
  q.fit = __builtin_amdgcn_readfirstlane(fit);   // wave-uniform (every lane computed the same value)
  const uint32_t s0 = wq_size<G>(q, 0);
  unsigned long long b = 0, nb = 0;
  if (lane == 0) {
    b = atomicAdd(counter, (unsigned long long)s0);
    nb = atomicAdd(counter, (unsigned long long)s0);
  }
  q.cb = ((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(b >> 32)) << 32) |
         __builtin_amdgcn_readfirstlane((uint32_t)b);
  q.cs = s0;
  q.cu = 0;
  q.nbv = nb;
  q.ns = s0;
}

// index for every lane with `want` (others get an unused value)
template <bool G>
__device__ __forceinline__ uint64_t wq_take(WaveQueue& q, bool want, unsigned long long* counter) {
  const int lane = (int)(threadIdx.x & 63u);
  const uint64_t m = __ballot(want);
  const uint32_t cnt = (uint32_t)__popcll(m);
  const uint32_t rank = (uint32_t)__popcll(m & ((1ull << lane) - 1ull));
  if (q.cu + cnt <= q.cs) {
    const uint64_t idx = q.cb + q.cu + rank;
    q.cu += cnt;
    return idx;
  }
  const uint32_t first = q.cs - q.cu;
  const uint64_t nb = ((uint64_t)__builtin_amdgcn_readlane((uint32_t)(q.nbv >> 32), 0) << 32) |
                      __builtin_amdgcn_readlane((uint32_t)q.nbv, 0);
  const uint64_t idx = rank < first ? q.cb + q.cu + rank : nb + (rank - first);
  q.cb = nb;
  q.cs = q.ns;
  q.cu = cnt - first;   // <= 64 <= every chunk size
  q.ns = wq_size<G>(q, nb + q.cs);
  if (lane == 0) q.nbv = atomicAdd(counter, (unsigned long long)q.ns);
  return idx;
}

// Next wave task from a global counter, as a wave-UNIFORM value: every lane
// takes part in the atomic (lane 0 adds 1, the others 0, so lane 0's return is
// the task) and the result is read with v_readfirstlane, so a loop exit on it
// is a uniform branch.  (An `if (lane == 0) atomicAdd` + __shfl made the
// compiler treat the exit as divergent; with the grouped k_curve it then
// structurized the loop so that the shuffle re-read a stale value and the
// wave never left it.)  Call with the whole wavefront active.
__device__ __forceinline__ uint64_t wave_task(unsigned long long* tasks) {
  const unsigned long long v = atomicAdd(tasks, (threadIdx.x & 63u) == 0 ? 1ull : 0ull);
  return ((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(v >> 32)) << 32) |
         __builtin_amdgcn_readfirstlane((uint32_t)v);
}

#ifndef PV_HASH_WAVES
#define PV_HASH_WAVES 2
#endif
#ifndef PV_HASH_LDS
#define PV_HASH_LDS 0
#endif
// 16-byte groups of the next block's message window loaded one compression
// ahead (0 = none)
#ifndef PV_HASH_PF
#define PV_HASH_PF 0
#endif
// libsodium's pre-checks on (R, S, A), one
// lane per signature, ahead of the hash: keeps the branchy, load-dependent
// check out of k_hash's refill path (which every ragged C4 iteration hit).
__global__ __launch_bounds__(256) void k_precheck(const uint8_t* __restrict__ pk, const uint8_t* __restrict__ sig,
                                                   uint64_t n, uint8_t* __restrict__ pre,
                                                   const uint32_t* __restrict__ kidx) {
  const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  pre[i] = precheck(pk + 32 * (kidx ? (uint64_t)kidx[i] : i), sig + 64 * i) ? 1 : 0;
}

// SHA-512(R || A || M) for the signatures that passed the pre-checks (pre =
// null: every signature; the half-size path runs the pre-checks in k_lattice
// instead and never reads the digests of rejected ones).  The next message of
// a lane is taken from the queue one message ahead: its offsets, pre-check
// verdict and key index are loaded while the current message is hashed, so a
// refill finds them in registers.
__global__ __launch_bounds__(HASH_BLOCK, PV_HASH_WAVES) void k_hash(const uint8_t* __restrict__ pk, const uint8_t* __restrict__ sig,
                                                     const uint8_t* __restrict__ blob,
                                                     const uint64_t* __restrict__ off, uint64_t n,
                                                     unsigned long long* __restrict__ counter,
                                                     uint32_t* __restrict__ dig, const uint8_t* __restrict__ pre,
                                                     const uint32_t* __restrict__ kidx) {
  uint64_t idx = n, blk = 0, nblk = 0, mo = 0, ml = 0;
  uint64_t hs[8];
  uint32_t ra[16];   // R || A of the current message (block 0's prefix)
  // prefetched next message: offsets, pre-check verdict, R || A
  WaveQueue q;
  // mean SHA-512 blocks per message from the blob's extent
  wq_init<PV_HASH_GUIDED>(q, counter, n, PV_HASH_GUIDED ? wq_fit(n ? hram_blocks((off[n] - off[0]) / n) : 1) : 64);
  uint64_t nidx = wq_take<PV_HASH_GUIDED>(q, true, counter), nmo = 0, nme = 0;
  uint32_t nok = 0, nra[16];
  auto prefetch = [&]() {
    if (nidx < n) {
      nmo = off[nidx];
      nme = off[nidx + 1];
      nok = pre ? pre[nidx] : 1u;
      load8(nra, sig + 64 * nidx);
      load8(nra + 8, pk + 32 * (kidx ? (uint64_t)kidx[nidx] : nidx));
    }
  };
  prefetch();
#if PV_HASH_PF
  // first groups of the next block's window (tagged by message offset + block)
  uint32_t ypf[4 * PV_HASH_PF];
  uint64_t pf_mo = ~0ull, pf_blk = 0;
#endif
#if PV_HASH_LDS
  // Message blocks are staged through LDS by the whole wavefront: lane l's
  // 144-byte window (9 groups of 16 B) is cut into 9 parts and part p is
  // loaded by lane (9 l + p) % 64 in pass (9 l + p) / 64, so one load
  // instruction of the wave covers ~7 consecutive windows (2 cache lines each)
  // instead of 64 scattered ones (~4.5x fewer L1 tag lookups per block).
  // Measured slower than per-lane loads (profiles/r02_ab_hash_queue.json):
  // the kernel is not bound by the L1 tag rate.
  constexpr int WB = 144;   // window bytes per lane
  __shared__ uint4 win[HASH_BLOCK / 64][64 * WB / 16];
  __shared__ uint4 desc[HASH_BLOCK / 64][64];
  const int lane = (int)(threadIdx.x & 63u), wv = (int)(threadIdx.x >> 6);
#endif
  // Convergent loop: every lane runs every trip (queue takes are wave-wide);
  // a lane without a block in progress idles through the compression.
  while (true) {
    // a lane whose message is done promotes its prefetched next message (a
    // message that failed the pre-checks leaves it idle for one trip) and
    // takes a new next index
    const bool promote = blk == nblk && nidx < n;
    if (promote) {
      idx = nidx;
      mo = nmo;
      ml = nme - nmo;
#pragma unroll
      for (int j = 0; j < 16; ++j) ra[j] = nra[j];
      if (nok != 0) {
        nblk = hram_blocks(ml);
        blk = 0;
        sha512_init(hs);
      }
    }
    const uint64_t t = wq_take<PV_HASH_GUIDED>(q, promote, counter);
    if (promote) {
      nidx = t;
      prefetch();
    }
    const bool active = blk < nblk;
    if (!__any(active || nidx < n)) break;   // nothing in progress, nothing queued
    uint64_t w[16];
#if PV_HASH_LDS
    {
      // this lane's window: aligned-down start of block blk and the number of
      // 16-byte groups holding message bytes (msg_fetch's rule)
      const uint64_t qb = hram_q(blk);
      const uint8_t* m = blob + mo;
      const uint32_t mis = (uint32_t)((reinterpret_cast<uintptr_t>(m) + qb) & 3u);
      const int64_t rem = (int64_t)ml - (int64_t)qb;
      int ng = 0;
      if (active && rem + (int64_t)mis > 0) {
        const int64_t g = (rem + (int64_t)mis + 15) / 16;
        ng = (int)(g < (blk == 0 ? 5 : 9) ? g : (blk == 0 ? 5 : 9));
      }
      const uint64_t wa = reinterpret_cast<uint64_t>(m + qb - mis);
      desc[wv][lane] = make_uint4((uint32_t)wa, (uint32_t)(wa >> 32), (uint32_t)ng, 0u);
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
      for (int k = 0; k < 9; ++k) {
        const int gi = 64 * k + lane, owner = gi / 9, part = gi - 9 * (gi / 9);
        const uint4 d = desc[wv][owner];
        uint4 v = make_uint4(0u, 0u, 0u, 0u);
        if (part < (int)d.z) {
          const uint64_t a = ((uint64_t)d.y << 32 | d.x) + 16u * (uint32_t)part;
          const uint32_t* p = reinterpret_cast<const uint32_t*>(a);
          v = make_uint4(p[0], p[1], p[2], p[3]);
        }
        win[wv][gi] = v;
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      uint32_t y[MSG_Y];
#pragma unroll
      for (int g = 0; g < 9; ++g) {
        const uint4 v = win[wv][9 * lane + g];
        y[4 * g] = v.x;
        y[4 * g + 1] = v.y;
        y[4 * g + 2] = v.z;
        y[4 * g + 3] = v.w;
      }
      __builtin_amdgcn_wave_barrier();   // the next trip's stores come after these reads
      if (active) hram_assemble_ra(w, y, ra, m, ml, blk, nblk);
    }
#endif
    if (active) {
#if !PV_HASH_LDS
      uint32_t y[MSG_Y];
#if PV_HASH_PF
      // the window's first PV_HASH_PF groups were loaded during the previous
      // compression when the tag matches; the rest now
      if (pf_mo == mo && pf_blk == blk) {
#pragma unroll
        for (int k = 0; k < 4 * PV_HASH_PF; ++k) y[k] = ypf[k];
        msg_fetch_part(y + 4 * PV_HASH_PF, blob + mo, ml, hram_q(blk), blk == 0, PV_HASH_PF, 9);
      } else {
        msg_fetch(y, blob + mo, ml, hram_q(blk), blk == 0);
      }
#else
      msg_fetch(y, blob + mo, ml, hram_q(blk), blk == 0);
#endif
      hram_assemble_ra(w, y, ra, blob + mo, ml, blk, nblk);
#if PV_HASH_PF
      // next trip's block: blk + 1 of this message, or block 0 of the queued one
      if (blk + 1 < nblk) {
        pf_mo = mo;
        pf_blk = blk + 1;
        msg_fetch_part(ypf, blob + mo, ml, hram_q(blk + 1), false, 0, PV_HASH_PF);
      } else if (nidx < n) {
        pf_mo = nmo;
        pf_blk = 0;
        msg_fetch_part(ypf, blob + nmo, nme - nmo, 0, true, 0, PV_HASH_PF);
      }
#endif
#endif
      sha512_compress(hs, w);
      if (++blk == nblk) {
        uint32_t d[16];
        sha512_digest_words(d, hs);
        uint32_t* o = dig + 16 * idx;
#pragma unroll
        for (int k = 0; k < 16; ++k) o[k] = d[k];
      }
    }
  }
}

hipError_t hash_occupancy(int* blocks_per_cu) {
  return hipOccupancyMaxActiveBlocksPerMultiprocessor(blocks_per_cu, reinterpret_cast<const void*>(k_hash),
                                                      HASH_BLOCK, 0);
}

hipError_t launch_hash(const uint8_t* pk, const uint8_t* sig, const uint8_t* blob, const uint64_t* off, uint64_t n,
                       unsigned long long* counter, uint32_t* dig, uint8_t* pre, int blocks, hipStream_t s,
                       const uint32_t* kidx) {
  if (n == 0) return hipSuccess;
  hipError_t e = hipMemsetAsync(counter, 0, sizeof(unsigned long long), s);
  if (e != hipSuccess) return e;
  if (pre) {
    hipLaunchKernelGGL(k_precheck, dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, s, pk, sig, n, pre, kidx);
    e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  const uint64_t need = (n + HASH_BLOCK - 1) / HASH_BLOCK;
  const uint64_t b = (uint64_t)blocks < need ? (uint64_t)blocks : need;
  hipLaunchKernelGGL(k_hash, dim3((uint32_t)b), dim3(HASH_BLOCK), 0, s, pk, sig, blob, off, n, counter, dig, pre,
                     kidx);
  return hipGetLastError();
}

// ---------------------------------------------------------- base-point table
// BTAB_CHUNKS tables, q-major: entry k of table q = k * 2^(32 q) * B
__global__ void k_btable_init(uint32_t* btab) {
  const int g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g < BTAB_CHUNKS * BTAB_ENTRIES) btable_entry(btab + g * BTAB_WORDS, g % BTAB_ENTRIES, g / BTAB_ENTRIES);
}

hipError_t launch_btable_init(uint32_t* btab, hipStream_t s) {
  const int n = BTAB_CHUNKS * BTAB_ENTRIES;
  hipLaunchKernelGGL(k_btable_init, dim3((n + 63) / 64), dim3(64), 0, s, btab);
  return hipGetLastError();
}

// ------------------------------------------------------------ curve kernel
// Persistent grid: lane gid owns scratch slot gid (its A table and the
// points awaiting the shared inversion) and takes CURVE_K signatures per round:
// gid, gid + nthreads, ... , gid + (K-1) nthreads.  Each wavefront covers 64
// consecutive signatures per k, so each ballot is one aligned bitmap word.
template <bool KEYED, int KF>
__global__ __launch_bounds__(CURVE_BLOCK, PV_CURVE_WAVES) void k_curve(const uint8_t* __restrict__ pk,
                                                                        const uint8_t* __restrict__ sig,
                                                                        const uint32_t* __restrict__ hin,
                                                                        const uint8_t* __restrict__ pre,
                                                                        const uint32_t* __restrict__ btab_g,
                                                                        uint32_t* __restrict__ scratch,
                                                                        uint8_t* __restrict__ verdict,
                                                                        uint64_t* __restrict__ bitmap, uint64_t n,
                                                                        const uint32_t* __restrict__ ktab,
                                                                        const uint32_t* __restrict__ kidx,
                                                                        const uint32_t* __restrict__ bw,
                                                                        unsigned long long* __restrict__ tasks) {
  // generic kernel: radix-256 table q = 0 in LDS (16.5 KB); the comb kernel of
  // prepared keys reads the radix-2^16 chunk tables bw from L2/MALL
  constexpr int TW = BTAB_ENTRIES * BTAB_WORDS;
  __shared__ uint32_t btab[KEYED ? 1 : TW];
  // keyed: the comb's 16 digit words per lane, lane-interleaved
  __shared__ uint32_t dg[KEYED ? 16 * CURVE_BLOCK : 1];
  if constexpr (!KEYED) {
    for (int j = threadIdx.x; j < TW; j += CURVE_BLOCK) btab[j] = btab_g[j];
    __syncthreads();
  }
  // persistent waves over a queue of wave tasks: task t = signatures
  // [64 CURVE_K t, 64 CURVE_K (t + 1)), lane l holding t's signatures l, l + 64,
  // ... (coalesced per k).  A dynamic queue (one atomic per task) instead of a
  // static grid stride: the grid's tail is one task per wave, and a block that
  // starts late (its CU busy with another stream's kernel) delays nothing.
  const int ln = (int)(threadIdx.x & 63u);
  const uint64_t gid = (uint64_t)blockIdx.x * CURVE_BLOCK + threadIdx.x;
  uint32_t* lane = scratch + gid * LANE_WORDS;
  constexpr uint64_t PER = 64ull * CURVE_K;
  const uint64_t ntasks = (n + PER - 1) / PER;
  for (;;) {
    const uint64_t t = wave_task(tasks);
    if (t >= ntasks) break;
    const uint64_t i0 = t * PER + (uint64_t)ln;
    const uint32_t okm = curve_group<KEYED, KEYED ? CURVE_BLOCK : 1, KF>(pk, sig, hin, pre, i0, 64, n, lane, btab,
                                                                          ktab, kidx, bw, dg + threadIdx.x);
#pragma unroll
    for (int k = 0; k < CURVE_K; ++k) {
      const uint64_t i = i0 + 64ull * (uint64_t)k;
      const bool ok = (okm >> k) & 1u;
      const uint64_t ball = __ballot(ok);
      if (i < n) {
        verdict[i] = ok ? 1 : 0;
        if (ln == 0) bitmap[i >> 6] = ball;
      }
    }
  }
}

hipError_t curve_occupancy(int* blocks_per_cu, bool keyed) {
  return keyed ? hipOccupancyMaxActiveBlocksPerMultiprocessor(blocks_per_cu,
                                                              reinterpret_cast<const void*>(k_curve<true, 0>),
                                                              CURVE_BLOCK, 0)
               : hipOccupancyMaxActiveBlocksPerMultiprocessor(blocks_per_cu,
                                                              reinterpret_cast<const void*>(k_curve<false, 0>),
                                                              CURVE_BLOCK, 0);
}

hipError_t launch_curve(const uint8_t* pk, const uint8_t* sig, const uint32_t* h, const uint8_t* pre,
                        const uint32_t* btab, uint32_t* scratch, uint64_t scratch_lanes, uint8_t* verdict,
                        uint64_t* bitmap, uint64_t n, int blocks, hipStream_t s, const uint32_t* ktab,
                        const uint32_t* kidx, const uint32_t* bw, unsigned long long* tasks, bool wide) {
  if (n == 0) return hipSuccess;
  // one wave task = 64 * CURVE_K signatures, CURVE_BLOCK / 64 waves per block
  const uint64_t ntasks = (n + 64ull * CURVE_K - 1) / (64ull * CURVE_K);
  uint64_t need = (ntasks + CURVE_BLOCK / 64 - 1) / (CURVE_BLOCK / 64);
  uint64_t b = (uint64_t)blocks < need ? (uint64_t)blocks : need;
  if (b * CURVE_BLOCK > scratch_lanes) b = scratch_lanes / CURVE_BLOCK;
  if (b == 0) return hipErrorInvalidValue;
  if (ktab && !bw) return hipErrorInvalidValue;
  if (!tasks) return hipErrorInvalidValue;
  hipError_t e = hipMemsetAsync(tasks, 0, sizeof(unsigned long long), s);
  if (e != hipSuccess) return e;
  if (ktab && wide)
    hipLaunchKernelGGL((k_curve<true, 1>), dim3((uint32_t)b), dim3(CURVE_BLOCK), 0, s, pk, sig, h, pre, btab, scratch,
                       verdict, bitmap, n, ktab, kidx, bw, tasks);
  else if (ktab)
    hipLaunchKernelGGL((k_curve<true, 0>), dim3((uint32_t)b), dim3(CURVE_BLOCK), 0, s, pk, sig, h, pre, btab, scratch,
                       verdict, bitmap, n, ktab, kidx, bw, tasks);
  else
    hipLaunchKernelGGL((k_curve<false, 0>), dim3((uint32_t)b), dim3(CURVE_BLOCK), 0, s, pk, sig, h, pre, btab, scratch,
                       verdict, bitmap, n, nullptr, nullptr, nullptr, tasks);
  return hipGetLastError();
}

// ------------------------------------------------ half-size scalar path
// k_lattice: one lane per signature.  h = digest mod L, Euclid on (8L, h) ->
// (c, d), s' = d S mod L, written as the record the curve kernel reads;
// deferred indices (~0.2 %) are appended to `dlist` (wave-aggregated atomic).
__global__ __launch_bounds__(256) void k_lattice(const uint8_t* __restrict__ pk, const uint8_t* __restrict__ sig,
                                                  const uint32_t* __restrict__ dig, uint8_t* __restrict__ pre, uint64_t n,
                                                  uint32_t* __restrict__ rec, uint32_t* __restrict__ dlist,
                                                  unsigned long long* __restrict__ dcount,
                                                  unsigned long long* __restrict__ bitmap, int force_full) {
  const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  uint32_t st = HS_NONE;
  if (i < n) {
    // the verdict bitmap the curve kernel ORs into (one word per 64 signatures)
    if ((i & 63) == 0) bitmap[i >> 6] = 0;
    // libsodium's pre-checks (App. C.2 steps 1-3) here, one lane per
    // signature: k_hash hashed every message of the half-size path
    const bool ok = precheck(pk + 32 * i, sig + 64 * i);
    pre[i] = ok ? 1 : 0;
    st = lattice_one(rec + HREC_WORDS * i, ok, dig + 16 * i, sig + 64 * i, force_full != 0);
  }
  const bool defer = st == HS_DEFER;
  const uint64_t m = __ballot(defer);
  if (m) {
    const int lane = (int)(threadIdx.x & 63u);
    const uint64_t base = wave_append(dcount, m);
    if (defer) dlist[base + (uint64_t)__popcll(m & ((1ull << lane) - 1ull))] = (uint32_t)i;
  }
}

// k_curve_half: persistent grid over a wave-granular work queue.  Tasks
// [0, F) are full-length verdicts of 64 deferred records each (taken first:
// they are the longest), tasks [F, F + ceil(n/64)) are 64 consecutive
// signatures on the half-size path (lanes of deferred or pre-rejected
// records idle).  Every task ORs its accepted bits into the bitmap (zeroed
// before the launch), so the two kinds never overwrite each other's words.
// LDS: tables of B and 2^128 B (2 x 16.5 KB).
__global__ __launch_bounds__(CURVE_BLOCK, PV_CURVE_WAVES) void k_curve_half(
    const uint8_t* __restrict__ pk, const uint8_t* __restrict__ sig, const uint32_t* __restrict__ dig,
    const uint32_t* __restrict__ rec, const uint32_t* __restrict__ btab, const uint32_t* __restrict__ bw,
    uint32_t* __restrict__ scratch, uint8_t* __restrict__ verdict, unsigned long long* __restrict__ bitmap,
    uint64_t n, const uint32_t* __restrict__ dlist, const unsigned long long* __restrict__ dcount,
    unsigned long long* __restrict__ tasks) {
  // base-point tables stay in global memory (L2/MALL): btab (radix 256, q = 0)
  // for the deferred full-length tasks, bw (radix 2^16, B and 2^128 B) for the
  // half-size verdicts; their entries are fetched ahead of use
  const int lane = (int)(threadIdx.x & 63u);
  // per-lane tables interleaved by PV_HALF_LS lanes ([word][lane] inside each
  // group of PV_HALF_LS consecutive lanes): coalesced table loads
  const uint64_t gl = (uint64_t)blockIdx.x * CURVE_BLOCK + threadIdx.x;
  uint32_t* scr = scratch + (gl / PV_HALF_LS) * (uint64_t)(HALF_LANE_WORDS * PV_HALF_LS) + gl % PV_HALF_LS;
  const uint64_t nd = *dcount;
  const uint64_t full_tasks = (nd + 63) / 64;
  const uint64_t all_tasks = full_tasks + (n + 63) / 64;
  for (;;) {
    const uint64_t t = wave_task(tasks);
    if (t >= all_tasks) break;
    if (t < full_tasks) {
      const uint64_t j = t * 64 + lane;
      if (j < nd) {
        const uint64_t i = dlist[j];
        const bool ok = verify_full_one<PV_HALF_LS>(pk + 32 * i, sig + 64 * i, dig + 16 * i, scr, btab);
        verdict[i] = ok ? 1 : 0;
        if (ok) atomicOr(&bitmap[i >> 6], 1ull << (i & 63));
      }
    } else {
      const uint64_t i = (t - full_tasks) * 64 + lane;
      uint32_t st = HS_NONE;
      if (i < n) st = rec[HREC_WORDS * i + HREC_FLAGS] & 0xffu;
      bool ok = false;
      if (st == HS_HALF)
        ok = curve_half<PV_HALF_LS>(pk + 32 * i, sig + 64 * i, rec + HREC_WORDS * i, scr, bw, bw + 4 * BW_TABLE);
      const uint64_t ball = __ballot(ok);
      if (i < n && st != HS_DEFER) verdict[i] = ok ? 1 : 0;
      if (lane == 0 && ball) atomicOr(&bitmap[t - full_tasks], (unsigned long long)ball);
    }
  }
}

// k_curve_lat: half-size verdicts of a SMALL batch on lane pairs (latency
// mode; pv_verify_core.h side_point / msm_side): signature i runs on lanes 2i
// (side 0: +-A and s'_lo B) and 2i + 1 (side 1: -R and s'_hi 2^128 B); side 1's
// point reaches side 0 through a lane shuffle, side 0 adds and tests for the
// identity.  Deferred records take the full-length verdict on side 0.  Each
// lane's chain is one decompression, one table and 33 + 8 adds around the 128
// doublings instead of k_curve_half's two, two and 66 + 16: batches of a few
// waves (one per SIMD) finish sooner.  Per-lane scratch: one table (AT_WORDS).
// The bitmap is zeroed before the launch (k_lattice) and ORed into here.
__global__ __launch_bounds__(64) void k_curve_lat(const uint8_t* __restrict__ pk, const uint8_t* __restrict__ sig,
                                                  const uint32_t* __restrict__ dig, const uint32_t* __restrict__ rec,
                                                  const uint32_t* __restrict__ btab, const uint32_t* __restrict__ bw,
                                                  uint32_t* __restrict__ scratch, uint8_t* __restrict__ verdict,
                                                  unsigned long long* __restrict__ bitmap, uint64_t n) {
  const uint64_t gl = (uint64_t)blockIdx.x * 64 + threadIdx.x;
  const uint64_t i = gl >> 1;
  const int side = (int)(gl & 1);
  uint32_t* scr = scratch + gl * AT_WORDS;
  const uint32_t st = i < n ? (rec[HREC_WORDS * i + HREC_FLAGS] & 0xffu) : HS_NONE;
  bool ok = false;
  ge_p3 Q;
  ge_p3_0(Q);
  if (st == HS_HALF) {
    const uint32_t* r = rec + HREC_WORDS * i;
    ok = side_point(Q, pk + 32 * i, sig + 64 * i, r, side);
    if (ok) {
      build_atab(scr, Q);
      ge_p1p1 t;
      msm_side(t, r, scr, side ? bw + 4 * BW_TABLE : bw, side);
      ge_p1p1_to_p3(Q, t);
    }
  }
  // side 1 -> side 0 (every lane shuffles: the exchange is convergent)
  ge_p3 Q1;
#pragma unroll
  for (int k = 0; k < 10; ++k) {
    Q1.X.v[k] = __shfl_xor(Q.X.v[k], 1, 64);
    Q1.Y.v[k] = __shfl_xor(Q.Y.v[k], 1, 64);
    Q1.Z.v[k] = __shfl_xor(Q.Z.v[k], 1, 64);
    Q1.T.v[k] = __shfl_xor(Q.T.v[k], 1, 64);
  }
  const bool ok1 = __shfl_xor(ok ? 1 : 0, 1, 64) != 0;
  if (side == 0 && i < n) {
    bool v = false;
    if (st == HS_HALF) {
      if (ok && ok1) {
        ge_cached c;
        ge_p3_to_cached(c, Q1);
        ge_p1p1 t;
        ge_add_cached(t, Q, c, false);
        v = p1p1_is_identity(t);
      }
    } else if (st == HS_DEFER) {
      v = verify_full_one(pk + 32 * i, sig + 64 * i, dig + 16 * i, scr, btab);
    }
    verdict[i] = v ? 1 : 0;
    if (v) atomicOr(&bitmap[i >> 6], 1ull << (i & 63));
  }
}

hipError_t launch_curve_lat(const uint8_t* pk, const uint8_t* sig, const uint32_t* dig, const uint32_t* rec,
                            const uint32_t* btab, const uint32_t* bw, uint32_t* scratch, uint64_t scratch_lanes,
                            uint8_t* verdict, uint64_t* bitmap, uint64_t n, hipStream_t s) {
  if (n == 0) return hipSuccess;
  const uint64_t blocks = (2 * n + 63) / 64;
  if (blocks * 64 > scratch_lanes) return hipErrorInvalidValue;
  hipLaunchKernelGGL(k_curve_lat, dim3((uint32_t)blocks), dim3(64), 0, s, pk, sig, dig, rec, btab, bw, scratch,
                     verdict, reinterpret_cast<unsigned long long*>(bitmap), n);
  return hipGetLastError();
}

// small calls (signatures per launch): k_verify_quad's schedule lanes, the keyed
// kernel's 4-signature blocks (host-buffer list calls)
#ifndef KQ_SMALL_MAX
#define KQ_SMALL_MAX 256
#endif
// PV_QUAD_PHASE (timing variants only, wrong verdicts): 1 skips the hash +
// lattice wave, 2 the decompressions + tables, 3 the windows
#ifndef PV_QUAD_PHASE
#define PV_QUAD_PHASE 0
#endif
// PV_QUAD_LDS_PAD (A/B variants only): extra LDS words per block, to cap the
// blocks a CU holds
#ifndef PV_QUAD_LDS_PAD
#define PV_QUAD_LDS_PAD 0
#endif
// k_verify_quad: the whole verify of a small batch in ONE launch (latency
// mode: pre-checks, SHA-512(R||A||M), the scalar stage and the lane-quad
// curve stage).  A block of 128 threads takes 8 signatures: wave 1 (one lane
// per signature) runs the pre-checks, the hash and the lattice stage into an
// LDS record while wave 0 (8 lanes per signature, lane quads) decodes -A and
// -R and builds their tables, which do not depend on the scalars; after one
// barrier wave 0 runs the windows.  Replaces 2 memsets + k_hash + k_lattice +
// the curve launch: the serial one-lane hash and lattice chains (~25 + 40 us
// per call) run under the decompressions.  Verdict bits are stored as the
// block's byte of the bitmap (8 signatures), so nothing needs zeroing; the
// deferred count (pv_curve_stats) is added to *dcount (zeroed by the caller).
// SCHED (calls up to KQ_SMALL_MAX signatures): the hash wave's message schedules
// on their own lanes first, as in k_verify_quad_keyed (pv_quad.h keyed_hash);
// larger calls keep hash_one (the 20 KB of schedules would halve the blocks per CU)
template <bool SCHED>
__global__ __launch_bounds__(128) void k_verify_quad(const uint8_t* __restrict__ pk, const uint8_t* __restrict__ sig,
                                                     const uint8_t* __restrict__ blob, const uint64_t* __restrict__ off,
                                                     uint64_t n, const uint32_t* __restrict__ bw,
                                                     uint8_t* __restrict__ verdict, uint8_t* __restrict__ bitmap_bytes,
                                                     uint64_t bitmap_len, unsigned long long* __restrict__ dcount,
                                                     int force_full) {
  __shared__ uint32_t tabs[16 * QTAB_WORDS + PV_QUAD_LDS_PAD];
  __shared__ uint32_t recs[8 * HREC_WORDS];
  __shared__ uint64_t kws[SCHED ? 80 * 8 * KQ_SCHED_BLOCKS : 1];
  const int t = (int)threadIdx.x;
  const uint64_t i0 = (uint64_t)blockIdx.x * 8;
  if (PV_QUAD_LDS_PAD && t == 0) tabs[16 * QTAB_WORDS] = 0;   // (keeps the padding allocated)
  const int side = (t >> 2) & 1;
  const QRole q = qrole_of((uint32_t)t & 3u);
  const uint64_t i = i0 + (uint64_t)((t & 63) >> 3);
  const uint64_t ic = i < n ? i : n - 1;   // lanes past the batch run on the last signature (results dropped)
  qfe Q;
  bool ok = false;
  if (t >= 64) {
    // wave 1: the scalar stage, lane k for signature i0 + k
    const int k = t - 64;
    uint32_t st = HS_NONE;
    if constexpr (SCHED) {
      const int sb = k & 7, bb = k >> 3;   // lane 8 b + s: block b's schedule of signature s
      const uint64_t js = i0 + (uint64_t)sb;
      if (bb < KQ_SCHED_BLOCKS && js < n && PV_QUAD_PHASE != 1) {
        const uint64_t ml = off[js + 1] - off[js];
        if ((uint64_t)bb < hram_blocks(ml))
          keyed_sched_block(kws + k, 8 * KQ_SCHED_BLOCKS, sig + 64 * js, pk + 32 * js, blob + off[js], ml,
                            (uint64_t)bb);
      }
      __threadfence_block();   // the schedules in LDS before the hashing lanes read them (same wave)
      __builtin_amdgcn_wave_barrier();
    }
    if (k < 8) {
      uint32_t* r = recs + HREC_WORDS * k;
      r[HREC_FLAGS] = HS_NONE;
      const uint64_t j = i0 + (uint64_t)k;
      if (j < n && PV_QUAD_PHASE != 1) {
        uint32_t dig[16];
        const uint64_t ml = off[j + 1] - off[j];
        const bool pre = SCHED ? keyed_hash(dig, kws + k, 8 * KQ_SCHED_BLOCKS, 8, sig + 64 * j, pk + 32 * j,
                                            blob + off[j], ml)
                               : hash_one(dig, pk + 32 * j, sig + 64 * j, blob + off[j], ml);
        st = lattice_one(r, pre, dig, sig + 64 * j, force_full != 0);
      }
    }
    const uint64_t dm = __ballot(st == HS_DEFER);
    if (k == 0 && dm) atomicAdd(dcount, (unsigned long long)__popcll(dm));
  } else {
    // wave 0: the points and their tables
    if (PV_QUAD_PHASE != 2) ok = q_side_table(Q, pk + 32 * ic, sig + 64 * ic, side, tabs + (t >> 2) * QTAB_WORDS, q);
  }
  __syncthreads();
  if (t >= 64) return;
  const uint32_t* r = recs + HREC_WORDS * (t >> 3);
  const uint32_t st = r[HREC_FLAGS] & 0xffu;
  if (PV_QUAD_PHASE != 3) q_side_msm(Q, r, side, tabs + (t >> 2) * QTAB_WORDS, side ? bw + 4 * BW_TABLE : bw, q);
  qfe e, e1;
  q_to_cached(e, Q, q);
#pragma unroll
  for (int k = 0; k < 10; ++k) e1.l[0].v[k] = __shfl_xor(e.l[0].v[k], 4, 64);   // side 1 -> side 0
  const bool ok1 = __shfl_xor(ok ? 1 : 0, 4, 64) != 0;
  const bool id = q_sum_is_identity(Q, e1, q);
  const bool v = (st == HS_HALF || st == HS_DEFER) && ok && ok1 && id;
  const bool mine = side == 0 && (t & 3) == 0 && i < n;
  if (mine) verdict[i] = v ? 1 : 0;
  const uint64_t ball = __ballot(mine && v);   // bits 8k: signature i0 + k
  if (t == 0) {
    uint32_t bits = 0;
#pragma unroll
    for (int k = 0; k < 8; ++k) bits |= (uint32_t)((ball >> (8 * k)) & 1ull) << k;
    bitmap_bytes[blockIdx.x] = (uint8_t)bits;
    // the last block also clears the rest of the last bitmap word
    if ((uint64_t)blockIdx.x + 1 == gridDim.x)
      for (uint64_t b = (uint64_t)blockIdx.x + 1; b < bitmap_len; ++b) bitmap_bytes[b] = 0;
  }
}

hipError_t launch_verify_quad(const uint8_t* pk, const uint8_t* sig, const uint8_t* blob, const uint64_t* off, uint64_t n,
                              const uint32_t* bw, uint8_t* verdict, uint64_t* bitmap, unsigned long long* dcount,
                              bool force_full, hipStream_t s) {
  if (n == 0) return hipSuccess;
  const uint64_t blocks = (n + 7) / 8;
  if (blocks > 0x7fffffffull) return hipErrorInvalidValue;
  const uint64_t bytes = (n + 63) / 64 * 8;
  if (n <= KQ_SMALL_MAX)
    hipLaunchKernelGGL(k_verify_quad<true>, dim3((uint32_t)blocks), dim3(128), 0, s, pk, sig, blob, off, n, bw,
                       verdict, reinterpret_cast<uint8_t*>(bitmap), bytes, dcount, force_full ? 1 : 0);
  else
    hipLaunchKernelGGL(k_verify_quad<false>, dim3((uint32_t)blocks), dim3(128), 0, s, pk, sig, blob, off, n, bw,
                       verdict, reinterpret_cast<uint8_t*>(bitmap), bytes, dcount, force_full ? 1 : 0);
  return hipGetLastError();
}

// k_verify_quad_list: k_verify_quad over a device-side LIST of signature
// indices (the records k_chunk_half deferred), count in *lcount (known only
// on the device): a fixed grid of blocks loops over groups of 8 entries, so
// the launch needs no read-back.  Verdicts go to verdict[index]; no bitmap
// (host-buffer calls return verdicts only).  The listed records are the
// deferred ones, so most take the quad kernel's full-length form (64 windows
// of h): ~0.4 ms per pass, about twice a half-size group.
__global__ __launch_bounds__(128) void k_verify_quad_list(const uint8_t* __restrict__ pk,
                                                          const uint8_t* __restrict__ sig,
                                                          const uint8_t* __restrict__ blob,
                                                          const uint64_t* __restrict__ off,
                                                          const uint32_t* __restrict__ list,
                                                          const unsigned long long* __restrict__ lcount,
                                                          const uint32_t* __restrict__ bw, uint8_t* __restrict__ verdict,
                                                          int force_full) {
  __shared__ uint32_t tabs[16 * QTAB_WORDS];
  __shared__ uint32_t recs[8 * HREC_WORDS];
  const int t = (int)threadIdx.x;
  const uint64_t cnt = *lcount;
  const int side = (t >> 2) & 1;
  const QRole q = qrole_of((uint32_t)t & 3u);
  for (uint64_t g = blockIdx.x; g * 8 < cnt; g += gridDim.x) {
    const uint64_t e = g * 8 + (uint64_t)((t & 63) >> 3);
    const uint64_t ic = list[e < cnt ? e : cnt - 1];   // lanes past the list repeat its last entry (dropped)
    qfe Q;
    bool ok = false;
    if (t >= 64) {
      const int k = t - 64;
      if (k < 8) {
        uint32_t* r = recs + HREC_WORDS * k;
        r[HREC_FLAGS] = HS_NONE;
        if (g * 8 + (uint64_t)k < cnt) {
          const uint64_t j = list[g * 8 + (uint64_t)k];
          uint32_t dig[16];
          const bool pre = hash_one(dig, pk + 32 * j, sig + 64 * j, blob + off[j], off[j + 1] - off[j]);
          (void)lattice_one(r, pre, dig, sig + 64 * j, force_full != 0);
        }
      }
    } else {
      ok = q_side_table(Q, pk + 32 * ic, sig + 64 * ic, side, tabs + (t >> 2) * QTAB_WORDS, q);
    }
    __syncthreads();
    if (t < 64) {
      const uint32_t* r = recs + HREC_WORDS * (t >> 3);
      const uint32_t st = r[HREC_FLAGS] & 0xffu;
      q_side_msm(Q, r, side, tabs + (t >> 2) * QTAB_WORDS, side ? bw + 4 * BW_TABLE : bw, q);
      qfe x, x1;
      q_to_cached(x, Q, q);
#pragma unroll
      for (int k = 0; k < 10; ++k) x1.l[0].v[k] = __shfl_xor(x.l[0].v[k], 4, 64);   // side 1 -> side 0
      const bool ok1 = __shfl_xor(ok ? 1 : 0, 4, 64) != 0;
      const bool id = q_sum_is_identity(Q, x1, q);
      const bool v = (st == HS_HALF || st == HS_DEFER) && ok && ok1 && id;
      if (side == 0 && (t & 3) == 0 && e < cnt) verdict[ic] = v ? 1 : 0;
    }
    __syncthreads();   // LDS tables and records are rewritten by the next group
  }
}

// the scalar stage of one k_chunk_half lane, out of line: inlined beside
// curve_half the compiler interleaved the two and spilled ~580 VGPRs
__device__ __attribute__((noinline)) uint32_t chunk_scalar_stage(uint32_t* rec, const uint8_t* pk, const uint8_t* sig,
                                                                 const uint8_t* m, uint64_t mlen, int force_full) {
  uint32_t dig[16];
  const bool pre = hash_one(dig, pk, sig, m, mlen);
  return lattice_one(rec, pre, dig, sig, force_full != 0);
}

hipError_t launch_verify_quad_list(const uint8_t* pk, const uint8_t* sig, const uint8_t* blob, const uint64_t* off,
                                   const uint32_t* list, const unsigned long long* lcount, uint64_t max_count,
                                   int blocks, const uint32_t* bw, uint8_t* verdict, bool force_full, hipStream_t s) {
  if (max_count == 0) return hipSuccess;
  const uint64_t need = (max_count + 7) / 8;
  const uint64_t b = (uint64_t)blocks < need ? (uint64_t)blocks : need;
  if (b == 0) return hipErrorInvalidValue;
  hipLaunchKernelGGL(k_verify_quad_list, dim3((uint32_t)b), dim3(128), 0, s, pk, sig, blob, off, list, lcount, bw,
                     verdict, force_full ? 1 : 0);
  return hipGetLastError();
}

// k_chunk_half: one launch per chunk of a host-buffer call (pv_verify_batch).
// Persistent grid over 64-signature wave tasks; a task runs the pre-checks,
// SHA-512(R||A||M) and the lattice stage (one lane per signature, record in
// `rec`) and then the half-size curve stage on the same lanes.  With no hash /
// lattice launches between the chunks' curve grids, chunk c + 1's waves
// (other stream) take the slots chunk c's waves release as they finish.
// Deferred records (~0.2 %) are appended to `dlist` as base + i (the shard
// index) for one k_verify_quad_list pass after the last chunk; their verdicts
// are not written here.  No bitmap.
__global__ __launch_bounds__(CURVE_BLOCK, PV_CURVE_WAVES) void k_chunk_half(
    const uint8_t* __restrict__ pk, const uint8_t* __restrict__ sig, const uint8_t* __restrict__ blob,
    const uint64_t* __restrict__ off, uint64_t n, uint32_t* __restrict__ rec, const uint32_t* __restrict__ bw,
    uint32_t* __restrict__ scratch, uint8_t* __restrict__ verdict, uint32_t* __restrict__ dlist,
    unsigned long long* __restrict__ dcount, uint64_t base, unsigned long long* __restrict__ tasks, int force_full) {
  const int lane = (int)(threadIdx.x & 63u);
  const uint64_t gl = (uint64_t)blockIdx.x * CURVE_BLOCK + threadIdx.x;
  uint32_t* scr = scratch + (gl / PV_HALF_LS) * (uint64_t)(HALF_LANE_WORDS * PV_HALF_LS) + gl % PV_HALF_LS;
  const uint64_t ntask = (n + 63) / 64;
  for (;;) {
    const uint64_t t = wave_task(tasks);
    if (t >= ntask) break;
    const uint64_t i = t * 64 + lane;
    uint32_t* r = rec + HREC_WORDS * (i < n ? i : 0);
    uint32_t st = HS_NONE;
    if (i < n) {
      st = chunk_scalar_stage(r, pk + 32 * i, sig + 64 * i, blob + off[i], off[i + 1] - off[i], force_full);
    }
    const bool defer = st == HS_DEFER;
    const uint64_t m = __ballot(defer);
    if (m) {
      const uint64_t b = wave_append(dcount, m);
      if (defer) dlist[b + (uint64_t)__popcll(m & ((1ull << lane) - 1ull))] = (uint32_t)(base + i);
    }
    bool ok = false;
    if (st == HS_HALF) ok = curve_half<PV_HALF_LS>(pk + 32 * i, sig + 64 * i, r, scr, bw, bw + 4 * BW_TABLE);
    if (i < n && !defer) verdict[i] = ok ? 1 : 0;
  }
}

hipError_t launch_chunk_half(const uint8_t* pk, const uint8_t* sig, const uint8_t* blob, const uint64_t* off,
                             uint64_t n, uint32_t* rec, const uint32_t* bw, uint32_t* scratch, uint64_t scratch_lanes,
                             uint8_t* verdict, uint32_t* dlist, unsigned long long* dcount, uint64_t base,
                             unsigned long long* tasks, int blocks, bool force_full, hipStream_t s) {
  if (n == 0) return hipSuccess;
  if (base + n > 0xffffffffull) return hipErrorInvalidValue;   // deferred indices are 32-bit
  hipError_t e = hipMemsetAsync(tasks, 0, sizeof(unsigned long long), s);
  if (e != hipSuccess) return e;
  const uint64_t need = (n + CURVE_BLOCK - 1) / CURVE_BLOCK;
  uint64_t b = (uint64_t)blocks < need ? (uint64_t)blocks : need;
  if (b * CURVE_BLOCK > scratch_lanes) b = scratch_lanes / CURVE_BLOCK;
  if (b == 0) return hipErrorInvalidValue;
  hipLaunchKernelGGL(k_chunk_half, dim3((uint32_t)b), dim3(CURVE_BLOCK), 0, s, pk, sig, blob, off, n, rec, bw, scratch,
                     verdict, dlist, dcount, base, tasks, force_full ? 1 : 0);
  return hipGetLastError();
}

hipError_t curve_half_occupancy(int* blocks_per_cu) {
  return hipOccupancyMaxActiveBlocksPerMultiprocessor(blocks_per_cu, reinterpret_cast<const void*>(k_curve_half),
                                                      CURVE_BLOCK, 0);
}

hipError_t launch_lattice(const uint8_t* pk, const uint8_t* sig, const uint32_t* dig, uint8_t* pre, uint64_t n,
                          uint32_t* rec, uint32_t* dlist, unsigned long long* dcount, unsigned long long* tasks,
                          uint64_t* bitmap, bool force_full, hipStream_t s) {
  if (n == 0) return hipSuccess;
  if (n > 0xffffffffull) return hipErrorInvalidValue;  // deferred indices are 32-bit
  // the counters (one memset when adjacent) and the bitmap the curve kernel
  // ORs into (zeroed by k_lattice itself) are reset here, so that the curve
  // launch is a single kernel (its HIP-event time == rocprof's)
  hipError_t e = tasks == dcount + 1 ? hipMemsetAsync(dcount, 0, 2 * sizeof(unsigned long long), s)
                                     : hipMemsetAsync(dcount, 0, sizeof(unsigned long long), s);
  if (e == hipSuccess && tasks != dcount + 1) e = hipMemsetAsync(tasks, 0, sizeof(unsigned long long), s);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(k_lattice, dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, s, pk, sig, dig, pre, n, rec, dlist,
                     dcount, reinterpret_cast<unsigned long long*>(bitmap), force_full ? 1 : 0);
  return hipGetLastError();
}

__global__ __launch_bounds__(64) void k_bw_init(uint32_t* bw) {
  const int g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g < BW_CHUNKS * BW_ENTRIES) btable_entry(bw + (uint64_t)g * BT_WORDS, g % BW_ENTRIES, g / BW_ENTRIES, 16);
}

hipError_t launch_bw_init(uint32_t* bw, hipStream_t s) {
  hipLaunchKernelGGL(k_bw_init, dim3((BW_CHUNKS * BW_ENTRIES + 63) / 64), dim3(64), 0, s, bw);
  return hipGetLastError();
}

hipError_t launch_curve_half(const uint8_t* pk, const uint8_t* sig, const uint32_t* dig, const uint32_t* rec,
                             const uint32_t* btab, const uint32_t* bw, uint32_t* scratch, uint64_t scratch_lanes,
                             uint8_t* verdict, uint64_t* bitmap, uint64_t n, const uint32_t* dlist,
                             const unsigned long long* dcount, unsigned long long* tasks, int blocks, hipStream_t s) {
  if (n == 0) return hipSuccess;
  const uint64_t need = (n + CURVE_BLOCK - 1) / CURVE_BLOCK;
  uint64_t b = (uint64_t)blocks < need ? (uint64_t)blocks : need;
  if (b * CURVE_BLOCK > scratch_lanes) b = scratch_lanes / CURVE_BLOCK;
  if (b == 0) return hipErrorInvalidValue;
  hipLaunchKernelGGL(k_curve_half, dim3((uint32_t)b), dim3(CURVE_BLOCK), 0, s, pk, sig, dig, rec, btab, bw, scratch,
                     verdict, reinterpret_cast<unsigned long long*>(bitmap), n, dlist, dcount, tasks);
  return hipGetLastError();
}

// -------------------------------------------------------------- key cache
// waves per SIMD k_keys is compiled for: 3 (168 VGPRs, 248 B of spills) measured
// 1 % slower on C4 than 2 (profiles/r02_ab_keys_waves_notadopted.jsonl)
#ifndef PV_KEYS_WAVES
#define PV_KEYS_WAVES 2
#endif
__global__ __launch_bounds__(256, PV_KEYS_WAVES) void k_keys(const uint8_t* __restrict__ pk, uint64_t k, uint32_t* __restrict__ ktab,
                                               uint32_t* __restrict__ scr) {
  const uint64_t j = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  // scratch lane-interleaved per wave: word w of key j at [(j / 64) * KEY_SCRATCH + w] * 64 + j % 64
  if (j < k) key_prepare<64>(ktab + j * KEY_WORDS, scr + (j / 64) * (uint64_t)(KEY_SCRATCH * 64) + j % 64, pk + 32 * j);
}

hipError_t launch_keys(const uint8_t* pk, uint64_t k, uint32_t* ktab, uint32_t* scr, hipStream_t s) {
  if (k == 0) return hipSuccess;
  hipLaunchKernelGGL(k_keys, dim3((uint32_t)((k + 255) / 256)), dim3(256), 0, s, pk, k, ktab, scr);
  return hipGetLastError();
}

// k_keys_wide: 128 lanes per key, lane g builds slice g % 16 of table
// (g / 16) % 8 of key g / 128 (key_prepare_wide_slice: the doublings of A_q,
// 8 multiples, one inversion); scratch lane-interleaved per 64 lanes
__global__ __launch_bounds__(64) void k_keys_wide(const uint8_t* __restrict__ pk, uint64_t k, uint32_t* __restrict__ ktab,
                                                  uint32_t* __restrict__ scr) {
  const uint64_t g = (uint64_t)blockIdx.x * 64 + threadIdx.x;
  const uint64_t key = g / (COMB_Q * KW_SLICES);
  if (key < k)
    key_prepare_wide_slice<64>(ktab + key * (uint64_t)KEYW_WORDS, scr + (g / 64) * (uint64_t)(KEYW_SCRATCH * 64) + g % 64,
                               pk + 32 * key, (int)((g / KW_SLICES) % COMB_Q), (int)(g % KW_SLICES));
}

hipError_t launch_keys_wide(const uint8_t* pk, uint64_t k, uint32_t* ktab, uint32_t* scr, hipStream_t s) {
  if (k == 0) return hipSuccess;
  hipLaunchKernelGGL(k_keys_wide, dim3((uint32_t)(KEYTAB_WIDE_LANES * k / 64)), dim3(64), 0, s, pk, k, ktab, scr);
  return hipGetLastError();
}

// k_verify_quad_keyed: the latency verdict of signatures whose key is
// prepared (pv_quad.h q_comb_side).  A block of 64 (KQ_CW + 2) threads takes 8
// signatures (4 in the small-call form, with 8 comb sides each: SIG below):
// the hash wave (one lane per signature) runs the pre-checks,
// SHA-512 and h mod L into an LDS record; the root wave (one lane per
// signature) decodes -R -- the 250-squaring square-root chain -- and leaves it
// in cached form in LDS; the KQ_CW comb waves (16 lanes per signature:
// KQ_SIDES = 4 lane quads, two comb tables and two base-point chunks each) sum
// S's base-point chunks, then run the comb of h as soon as the record is there.
// The sides' points are then summed over exchanges (shfl_xor 4, 8, ...) and side 0
// tests the total plus -R for the identity.  One wave per
// SIMD (four waves): no two paths share an issue port.
// Round 5: four sides instead of two -- a comb lane's chain 28 (sq + mul) +
// 2 x 34 mul -> 28 (sq + mul) + 2 x 20 mul + one more exchange level
// (profiles/r05_keyed_phase_kernel_stats.txt: hash -> comb was the critical path);
// and the hand-offs are LDS flags, not block barriers: a barrier after the hash
// held the root wave's chain until the hash was done (~7 us of a lone verify),
// now the root chain runs uninterrupted and only the comb waves wait (kq_wait).
// LIST: signature e of the launch is list[e] (host-buffer calls whose batch
// mixes cached and uncached keys); else e itself, and the verdict bits also
// go to the bitmap as the block's byte.
constexpr int KQ_NR = 41;   // -R cached in add order (Y-X, Y+X, 2dT, 2Z) + decode verdict
constexpr int KQ_CW = 2;   // comb waves per block: 8 signatures x 4 sides, or 4 x 8 (small calls)
constexpr int KQ_THREADS = 64 * (KQ_CW + 2);
static_assert(KQ_SCHED_BLOCKS >= 1 && 8 * KQ_SCHED_BLOCKS <= 64, "one lane per (signature, block) of the hash wave");
// PV_KEYED_PHASE (timing variants only, wrong verdicts), a bit mask: 1 skips the
// -R square root (root wave), 2 the comb (comb waves), 4 the hash (hash wave)
#ifndef PV_KEYED_PHASE
#define PV_KEYED_PHASE 0
#endif
// a wave's LDS writes done, then the flag (lane 0); the waiting waves spin on it.
// Every wave of the block is resident (one block = four waves on four SIMDs), so a
// waiting wave never holds up the one it waits for.
__device__ __forceinline__ void kq_signal(uint32_t* f) {
  __threadfence_block();
  if ((threadIdx.x & 63u) == 0) __hip_atomic_store(f, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void kq_wait(uint32_t* f) {
  while (__hip_atomic_load(f, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) == 0u) __builtin_amdgcn_s_sleep(1);
}
// SIG signatures per block: 8 (SIDES = 4 lane quads each) or, for small host
// calls, 4 (SIDES = 8: a comb lane adds one key table and one base-point chunk);
// the bitmap form (no LIST) needs 8 (one bitmap byte per block)
template <bool LIST, int SIG>
__global__ __launch_bounds__(KQ_THREADS) void k_verify_quad_keyed(const uint8_t* __restrict__ pk, int pk_by_key,
                                                                  const uint8_t* __restrict__ sig,
                                                                  const uint8_t* __restrict__ blob,
                                                                  const uint64_t* __restrict__ off, uint64_t n,
                                                                  const uint32_t* __restrict__ list,
                                                                  const uint32_t* __restrict__ ktab,
                                                                  const uint32_t* __restrict__ kidx,
                                                                  const uint32_t* __restrict__ bw,
                                                                  uint8_t* __restrict__ verdict,
                                                                  uint8_t* __restrict__ bitmap_bytes,
                                                                  uint64_t bitmap_len, uint32_t* __restrict__ done,
                                                                  uint32_t* __restrict__ flag, uint32_t seq) {
  constexpr int SIDES = 32 / SIG;      // lane quads per signature
  constexpr int LPS = 4 * SIDES;       // comb lanes per signature
  constexpr int KSL = SIG * KQ_SCHED_BLOCKS;   // schedule lanes of the hash wave
  static_assert((SIG == 8 || (SIG == 4 && LIST)) && SIG * LPS == 64 * KQ_CW, "8, or 4 with a list");
  __shared__ uint32_t recs[SIG * KQ_WORDS];
  __shared__ uint32_t negr[SIG * KQ_NR];
  __shared__ uint32_t vbits[KQ_CW];
  __shared__ uint32_t ready[2];   // 0: the records (hash wave), 1: -R (root wave)
  // the hash wave's message schedules: block b < KQ_SCHED_BLOCKS of signature s at
  // lane SIG b + s, K_t + W_t at kws[t * KSL + lane]
  __shared__ uint64_t kws[80 * KSL];
  const int t = (int)threadIdx.x;
  const int wave = t >> 6;
  const bool comb = wave < KQ_CW;
  const uint64_t e0 = (uint64_t)blockIdx.x * SIG;
  const int side = (t >> 2) & (SIDES - 1);
  const QRole q = qrole_of((uint32_t)t & 3u);
  const int cs = comb ? t / LPS : 0;   // comb waves: the block's signature of this lane
  const uint64_t e = e0 + (uint64_t)cs;
  const int k = (t & 63);                 // hash / root wave: lane k < SIG serves signature e0 + k
  const uint64_t ek = e0 + (uint64_t)k;
  const bool serve = !comb && k < SIG && ek < n;
  uint64_t j = 0;
  if (serve) j = LIST ? list[ek] : ek;
  if (t < 2) ready[t] = 0;
  __syncthreads();
  if (wave == KQ_CW) {
    // SHA-512(R || A || M) with the message schedules of the first
    // KQ_SCHED_BLOCKS blocks computed by one lane per block first (all blocks'
    // loads in flight at once), then the hashing lane runs only the rounds of
    // those blocks (round 5: the hash -> comb path is the kernel's critical path)
    const int sb = k % SIG, bb = k / SIG;   // this lane's signature and block
    const uint64_t es = e0 + (uint64_t)sb;
    const bool serve_s = !(PV_KEYED_PHASE & 4) && bb < KQ_SCHED_BLOCKS && es < n;
    uint64_t js = 0;
    if (serve_s) js = LIST ? list[es] : es;
    const uint8_t* as = pk + 32 * (pk_by_key ? (uint64_t)kidx[js] : js);
    const uint64_t mlen_s = serve_s ? off[js + 1] - off[js] : 0;
    const uint64_t nb_s = hram_blocks(mlen_s);
    if (serve_s && (uint64_t)bb < nb_s)
      keyed_sched_block(kws + k, KSL, sig + 64 * js, as, blob + off[js], mlen_s, (uint64_t)bb);
    __threadfence_block();   // the schedules in LDS before the hashing lanes read them (same wave)
    __builtin_amdgcn_wave_barrier();
    if (k < SIG) {
      uint32_t dig[16];
      bool pre = false;
      if (serve && !(PV_KEYED_PHASE & 4))
        pre = keyed_hash(dig, kws + k, KSL, SIG, sig + 64 * j, as, blob + off[j], mlen_s);
      keyed_record(recs + KQ_WORDS * k, pre, dig);
    }
    kq_signal(ready);
  } else if (wave == KQ_CW + 1) {
    if (k < SIG) {
      uint32_t* o = negr + KQ_NR * k;
      bool ok = false;
      ge_p3 P;
      if (serve && !(PV_KEYED_PHASE & 1)) {
        uint32_t enc[8];
        load8(enc, sig + 64 * j);
        ok = ge_frombytes_negate(P, enc) && y_is_canonical(enc);
      } else {
        ge_p3_0(P);
      }
      ge_cached c;
      ge_p3_to_cached(c, P);
      fe_carry(c.YmX);
      fe_carry(c.YpX);
      fe_carry(c.Z2);
      store_fe(o, c.YmX);
      store_fe(o + 10, c.YpX);
      store_fe(o + 20, c.T2d);
      store_fe(o + 30, c.Z2);
      o[40] = ok ? 1u : 0u;
    }
    kq_signal(ready + 1);
  } else {
    const uint64_t ec = e < n ? e : n - 1;   // lanes past the batch run on the last signature (results dropped)
    const uint64_t ic = LIST ? list[ec] : ec;
    qfe acc, e_hi, e_lo;
    if (!(PV_KEYED_PHASE & 2)) q_comb_base<SIDES>(e_hi, e_lo, sig + 64 * ic, side, bw, q);   // S B: no hash needed
    const uint32_t* kt = ktab + (uint64_t)kidx[ic] * KEY_WORDS;
    const uint32_t* r = recs + KQ_WORDS * cs;
    kq_wait(ready);
    if (!(PV_KEYED_PHASE & 2)) q_comb_side<SIDES>(acc, r, side, kt, e_hi, e_lo, q);
    // the sides' sum before -R is needed: side s + 1 -> s for even s (xor 4), then
    // side 2 -> 0 (xor 8) ..., so that only one add-and-test follows the root
    // wave's flag (round 5: the root chain is the longer path)
    qfe eR, x, xo;
#pragma unroll
    for (int step = 1; step < SIDES; step <<= 1) {
      q_to_cached(x, acc, q);
#pragma unroll
      for (int i = 0; i < 10; ++i) xo.l[0].v[i] = __shfl_xor(x.l[0].v[i], 4 * step, 64);
      q_add(acc, xo, false, q);   // meaningful on sides s % (2 step) == 0; the others compute alike, unused
    }
    kq_wait(ready + 1);
    const uint32_t* nr = negr + KQ_NR * cs;
    q_load_cached(eR, nr, false, q);
    const bool id = q_sum_is_identity(acc, eR, q);   // R' + (-R) = O on side 0
    const bool v = r[KQ_OK] != 0 && kt[KEY_STATUS] != 0 && nr[40] != 0 && id;
    const bool mine = side == 0 && (t & 3) == 0 && e < n;
    if (mine) verdict[ic] = v ? 1 : 0;
    if (flag) __threadfence_system();   // the verdicts out before the completion word
    if constexpr (!LIST) {
      const uint64_t ball = __ballot(mine && v);   // bit LPS m: signature 64 wave / LPS + m
      if ((t & 63) == 0) {
        uint32_t bits = 0;
#pragma unroll
        for (int m = 0; m < 64 / LPS; ++m) bits |= (uint32_t)((ball >> (LPS * m)) & 1ull) << m;
        vbits[wave] = bits;
      }
    }
  }
  if constexpr (!LIST) {
    __syncthreads();   // every wave (the hash and root waves too): the comb waves' bits are in LDS
    if (t == 0 && bitmap_bytes) {
      uint32_t bits = 0;
#pragma unroll
      for (int w = 0; w < KQ_CW; ++w) bits |= vbits[w] << (w * (64 / LPS));
      bitmap_bytes[blockIdx.x] = (uint8_t)bits;
      if ((uint64_t)blockIdx.x + 1 == gridDim.x)
        for (uint64_t b = (uint64_t)blockIdx.x + 1; b < bitmap_len; ++b) bitmap_bytes[b] = 0;
    }
  }
  if (flag) {
    // completion word of a zero-copy host call (run_small): the last block to
    // finish writes seq into fine-grained host memory and re-arms the counter
    // (instead of a k_signal launch behind the kernel)
    if constexpr (LIST) __syncthreads();
    if (t == 0) {
      __threadfence_system();
      if (atomicAdd(done, 1u) + 1u == gridDim.x) {
        done[0] = 0;
        __threadfence_system();
        __hip_atomic_store(flag, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
      }
    }
  }
}

hipError_t launch_verify_quad_keyed(const uint8_t* pk, bool pk_by_key, const uint8_t* sig, const uint8_t* blob,
                                    const uint64_t* off, uint64_t n, const uint32_t* list, const uint32_t* ktab,
                                    const uint32_t* kidx, const uint32_t* bw, uint8_t* verdict, uint64_t* bitmap,
                                    hipStream_t s, uint32_t* done, uint32_t* flag, uint32_t seq) {
  if ((flag != nullptr) != (done != nullptr)) return hipErrorInvalidValue;
  if (n == 0) return hipSuccess;
  const uint64_t blocks = (n + 7) / 8;
  if (blocks > 0x7fffffffull) return hipErrorInvalidValue;
  if (list && bitmap) return hipErrorInvalidValue;
  const uint64_t bytes = (n + 63) / 64 * 8;
  if (list && n <= KQ_SMALL_MAX)   // small host calls: 4 signatures per block, 8 comb sides each
    hipLaunchKernelGGL((k_verify_quad_keyed<true, 4>), dim3((uint32_t)((n + 3) / 4)), dim3(KQ_THREADS), 0, s, pk,
                       pk_by_key ? 1 : 0, sig, blob, off, n, list, ktab, kidx, bw, verdict, nullptr, 0, done, flag,
                       seq);
  else if (list)
    hipLaunchKernelGGL((k_verify_quad_keyed<true, 8>), dim3((uint32_t)blocks), dim3(KQ_THREADS), 0, s, pk,
                       pk_by_key ? 1 : 0, sig, blob, off, n, list, ktab, kidx, bw, verdict, nullptr, 0, done, flag,
                       seq);
  else
    hipLaunchKernelGGL((k_verify_quad_keyed<false, 8>), dim3((uint32_t)blocks), dim3(KQ_THREADS), 0, s, pk,
                       pk_by_key ? 1 : 0, sig, blob, off, n, nullptr, ktab, kidx, bw, verdict,
                       reinterpret_cast<uint8_t*>(bitmap), bytes, done, flag, seq);
  return hipGetLastError();
}

__global__ __launch_bounds__(64) void k_signal(uint32_t* __restrict__ flag, uint32_t seq) {
  if (threadIdx.x == 0) {
    __threadfence_system();
    __hip_atomic_store(flag + threadIdx.x, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

hipError_t launch_signal(uint32_t* flag, uint32_t seq, hipStream_t s) {
  hipLaunchKernelGGL(k_signal, dim3(1), dim3(64), 0, s, flag, seq);
  return hipGetLastError();
}

// ------------------------------------------------------------- batch signer
__global__ __launch_bounds__(256) void k_sign(const uint8_t* __restrict__ seeds, const uint8_t* __restrict__ blob,
                                               const uint64_t* __restrict__ off, uint64_t n,
                                               const uint32_t* __restrict__ btab_g, uint8_t* __restrict__ pk_out,
                                               uint8_t* __restrict__ sig_out) {
  __shared__ uint32_t btab[BTAB_ENTRIES * BTAB_WORDS];
  for (int j = threadIdx.x; j < BTAB_ENTRIES * BTAB_WORDS; j += 256) btab[j] = btab_g[j];
  __syncthreads();
  const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const uint64_t o = off[i];
  sign_one(pk_out + 32 * i, sig_out + 64 * i, seeds + 32 * i, blob + o, off[i + 1] - o, btab);
}

hipError_t launch_sign(const uint8_t* seeds, const uint8_t* blob, const uint64_t* off, uint64_t n,
                       const uint32_t* btab, uint8_t* pk_out, uint8_t* sig_out, hipStream_t s) {
  if (n == 0) return hipSuccess;
  const uint64_t blocks = (n + 255) / 256;
  hipLaunchKernelGGL(k_sign, dim3((uint32_t)blocks), dim3(256), 0, s, seeds, blob, off, n, btab, pk_out, sig_out);
  return hipGetLastError();
}

// ------------------------------------------------------------------- tally
// One wavefront per 3PC batch: lanes OR (1 << sender) of valid votes into the
// voter set (duplicates collapse), popcount, compare with the quorum.  A sender
// index >= n_nodes is an argument error: it sets *bad (the API reports it)
// instead of silently losing the vote.
// plenum/server/models.py:24-45,91-114 ; plenum/server/quorums.py:15-39
__global__ __launch_bounds__(256) void k_tally(const uint8_t* __restrict__ verdict, const uint32_t* __restrict__ sender,
                                                const uint64_t* __restrict__ batch_off, uint64_t n_batches,
                                                uint32_t n_nodes, uint32_t quorum, uint32_t* __restrict__ votes,
                                                uint8_t* __restrict__ reached, uint32_t* __restrict__ bad) {
  const uint64_t b = ((uint64_t)blockIdx.x * 256 + threadIdx.x) >> 6;
  const int lane = threadIdx.x & 63;
  if (b >= n_batches) return;
  const uint64_t s0 = batch_off[b], s1 = batch_off[b + 1];
  const uint32_t words = (n_nodes + 63) / 64;  // voter-set words; n_nodes <= 1024 (16 words)
  uint32_t count = 0;
  bool oob = false;
  for (uint32_t w = 0; w < words; ++w) {
    uint64_t mine = 0;
    for (uint64_t m = s0 + lane; m < s1; m += 64) {
      const uint32_t snd = sender[m];
      oob = oob || snd >= n_nodes;
      if (verdict[m] && snd < n_nodes && (snd >> 6) == w) mine |= 1ull << (snd & 63);
    }
    // wave OR-reduction
#pragma unroll
    for (int sh = 1; sh < 64; sh <<= 1) {
      const uint32_t lo = __shfl_xor((uint32_t)mine, sh, 64);
      const uint32_t hi = __shfl_xor((uint32_t)(mine >> 32), sh, 64);
      mine |= ((uint64_t)hi << 32) | lo;
    }
    count += __popcll(mine);
  }
  if (__ballot(oob) && lane == 0) atomicOr(bad, 1u);
  if (lane == 0) {
    votes[b] = count;
    reached[b] = count >= quorum ? 1 : 0;
  }
}

hipError_t launch_tally(const uint8_t* verdict, const uint32_t* sender, const uint64_t* batch_off, uint64_t n_batches,
                        uint32_t n_nodes, uint32_t quorum, uint32_t* votes, uint8_t* reached, uint32_t* bad,
                        hipStream_t s) {
  if (n_batches == 0) return hipSuccess;
  const uint64_t blocks = (n_batches * 64 + 255) / 256;
  hipLaunchKernelGGL(k_tally, dim3((uint32_t)blocks), dim3(256), 0, s, verdict, sender, batch_off, n_batches, n_nodes,
                     quorum, votes, reached, bad);
  return hipGetLastError();
}

// SURVEY.md §8(b) bitmap form: batch b's voter set is already a bitmap
// (bit j of word w = node 32 w + j has a valid vote), words_per = ceil(n_nodes/32)
// words per batch; dup_mask (may be null) clears the nodes whose votes must
// not count.  One lane per batch: popcount of (bits & ~dup) over the words,
// bits >= n_nodes ignored.
__global__ __launch_bounds__(256) void k_tally_bits(const uint32_t* __restrict__ bits, const uint32_t* __restrict__ dup,
                                                     uint64_t n_batches, uint32_t n_nodes, uint32_t quorum,
                                                     uint32_t* __restrict__ votes, uint8_t* __restrict__ reached) {
  const uint64_t b = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (b >= n_batches) return;
  const uint32_t wp = (n_nodes + 31) / 32;
  uint32_t count = 0;
  for (uint32_t w = 0; w < wp; ++w) {
    uint32_t x = bits[b * wp + w];
    if (dup) x &= ~dup[b * wp + w];
    const uint32_t top = n_nodes - 32 * w;    // nodes in this word
    if (top < 32) x &= (1u << top) - 1u;
    count += __popc(x);
  }
  if (votes) votes[b] = count;
  reached[b] = count >= quorum ? 1 : 0;
}

hipError_t launch_tally_bits(const uint32_t* bits, const uint32_t* dup, uint64_t n_batches, uint32_t n_nodes,
                             uint32_t quorum, uint32_t* votes, uint8_t* reached, hipStream_t s) {
  if (n_batches == 0) return hipSuccess;
  hipLaunchKernelGGL(k_tally_bits, dim3((uint32_t)((n_batches + 255) / 256)), dim3(256), 0, s, bits, dup, n_batches,
                     n_nodes, quorum, votes, reached);
  return hipGetLastError();
}

// ----------------------------------------------- SHA-256 / Merkle (row f3)
// PV_SHA256_PREFETCH = 1: each lane's next block window is loaded during the
// current compression (one trip ahead) instead of right before it
#ifndef PV_SHA256_PREFETCH
#define PV_SHA256_PREFETCH 1
#endif
// Batch SHA-256 of (prefix || M_i): persistent lanes with per-lane refill, the
// same work-queue scheme as k_hash (ragged messages cost no divergence;
// wave-private index chunks, next message's offsets loaded one message ahead).
__global__ __launch_bounds__(256) void k_sha256(const uint8_t* __restrict__ blob, const uint64_t* __restrict__ off,
                                                 uint64_t n, uint32_t plen, uint32_t prefix,
                                                 unsigned long long* __restrict__ counter, uint32_t* __restrict__ out) {
  WaveQueue q;
  wq_init<false>(q, counter, n, 64);
  uint64_t idx = n, blk = 0, nblk = 0, mo = 0, ml = 0;
  uint64_t nidx = wq_take<false>(q, true, counter), nmo = 0, nme = 0;
  if (nidx < n) {
    nmo = off[nidx];
    nme = off[nidx + 1];
  }
  uint32_t hs[8];
#if PV_SHA256_PREFETCH
  uint32_t y[SHA256_Y];   // the window of the block this lane compresses next
  if (nidx < n) sha256_window(y, blob + nmo, nme - nmo, plen, 0);
#endif
  while (true) {
    const bool promote = blk == nblk && nidx < n;
    if (promote) {
      idx = nidx;
      mo = nmo;
      ml = nme - nmo;
      nblk = sha256_blocks(ml, plen);
      blk = 0;
      sha256_init(hs);
    }
    const uint64_t t = wq_take<false>(q, promote, counter);
    if (promote) {
      nidx = t;
      if (nidx < n) {
        nmo = off[nidx];
        nme = off[nidx + 1];
      }
    }
    const bool active = blk < nblk;
    if (!__any(active)) break;   // every message promotes on the trip it is taken
    if (active) {
      uint32_t w[16];
#if PV_SHA256_PREFETCH
      sha256_assemble(w, y, blob + mo, ml, plen, prefix, blk, nblk);
      // the next trip's window in flight during this compression: block blk + 1,
      // or block 0 of the queued message (whose offsets are already loaded)
      if (blk + 1 < nblk) sha256_window(y, blob + mo, ml, plen, blk + 1);
      else if (nidx < n) sha256_window(y, blob + nmo, nme - nmo, plen, 0);
#else
      sha256_block(w, blob + mo, ml, plen, prefix, blk, nblk);
#endif
      sha256_compress(hs, w);
      if (++blk == nblk) {
        uint32_t* o = out + 8 * idx;
#pragma unroll
        for (int k = 0; k < 8; ++k) o[k] = bswap32_(hs[k]);
      }
    }
  }
}

hipError_t launch_sha256(const uint8_t* blob, const uint64_t* off, uint64_t n, uint32_t plen, uint32_t prefix,
                         unsigned long long* counter, uint32_t* out, int blocks, hipStream_t s) {
  if (n == 0) return hipSuccess;
  hipError_t e = hipMemsetAsync(counter, 0, sizeof(unsigned long long), s);
  if (e != hipSuccess) return e;
  const uint64_t need = (n + 255) / 256;
  const uint64_t b = (uint64_t)blocks < need ? (uint64_t)blocks : need;
  hipLaunchKernelGGL(k_sha256, dim3((uint32_t)b), dim3(256), 0, s, blob, off, n, plen, prefix, counter, out);
  return hipGetLastError();
}

// one Merkle level: out[i] = SHA-256(0x01 || in[2i] || in[2i+1]); an odd last
// node moves up unchanged (== RFC 6962 / ledger/tree_hasher.py MTH split at
// the largest power of two below n)
__global__ __launch_bounds__(256) void k_merkle_level(const uint32_t* __restrict__ in, uint64_t m,
                                                      uint32_t* __restrict__ out) {
  const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  const uint64_t half = m / 2;
  if (i < half) {
    uint32_t lr[16], h[8];
    const uint32_t* p = in + 16 * i;
#pragma unroll
    for (int k = 0; k < 16; ++k) lr[k] = p[k];
    sha256_node(h, lr);
#pragma unroll
    for (int k = 0; k < 8; ++k) out[8 * i + k] = h[k];
  } else if (i == half && (m & 1)) {
#pragma unroll
    for (int k = 0; k < 8; ++k) out[8 * i + k] = in[8 * (m - 1) + k];
  }
}

hipError_t launch_merkle_level(const uint32_t* in, uint64_t m, uint32_t* out, hipStream_t s) {
  const uint64_t outs = (m + 1) / 2;
  if (outs == 0) return hipSuccess;
  hipLaunchKernelGGL(k_merkle_level, dim3((uint32_t)((outs + 255) / 256)), dim3(256), 0, s, in, m, out);
  return hipGetLastError();
}

// the last levels of a tree in ONE workgroup: m <= MERKLE_TAIL nodes staged in
// LDS, one node per thread and level, a barrier between levels (replaces one
// launch per level below MERKLE_TAIL nodes; same pairing and odd-node rule).
// Measured: from 2048 nodes on one CU the 1024- and 512-node levels ran slower
// than their own multi-block launches (profiles/r06_ab_merkle_tail.jsonl)
static_assert(MERKLE_TAIL <= 512, "k_merkle_tail: one node per thread of 256 and level");
__global__ __launch_bounds__(256) void k_merkle_tail(const uint32_t* __restrict__ in, uint32_t m,
                                                       uint32_t* __restrict__ root) {
  __shared__ uint32_t lv[MERKLE_TAIL * 8];
  const uint32_t tid = threadIdx.x;
  for (uint32_t i = tid; i < 8 * m; i += 256) lv[i] = in[i];
  __syncthreads();
  while (m > 1) {
    const uint32_t half = m / 2;
    uint32_t h[8];
    if (tid < half) {
      uint32_t lr[16];
#pragma unroll
      for (int k = 0; k < 16; ++k) lr[k] = lv[16 * tid + k];
      sha256_node(h, lr);
    } else if (tid == half && (m & 1)) {
#pragma unroll
      for (int k = 0; k < 8; ++k) h[k] = lv[8 * (m - 1) + k];
    }
    __syncthreads();
    if (tid < half || (tid == half && (m & 1))) {
#pragma unroll
      for (int k = 0; k < 8; ++k) lv[8 * tid + k] = h[k];
    }
    __syncthreads();
    m = (m + 1) / 2;
  }
  if (tid < 8) root[tid] = lv[tid];
}

hipError_t launch_merkle_tail(const uint32_t* in, uint64_t m, uint32_t* root, hipStream_t s) {
  if (m < 2 || m > (uint64_t)MERKLE_TAIL) return hipErrorInvalidValue;
  hipLaunchKernelGGL(k_merkle_tail, dim3(1), dim3(256), 0, s, in, (uint32_t)m, root);
  return hipGetLastError();
}

hipError_t sha256_occupancy(int* blocks_per_cu) {
  return hipOccupancyMaxActiveBlocksPerMultiprocessor(blocks_per_cu, reinterpret_cast<const void*>(k_sha256), 256,
                                                      0);
}

// ------------------------------------------------------- synthetic workload
// Deterministic generator, spec in plenum_gpu/synth.py.
// Three layouts: FIXED (C2: every M mlen bytes), RANGE (C4: len uniform in
// [mlen_min, mlen_max] by hash), COMMIT (C3: 3PC batches of n_nodes COMMIT
// votes, M = serialize_msg_for_signing(COMMIT) of the batch).

// decimal digits of v >= 1
PV_HD uint32_t ndigits(uint64_t v) {
  uint32_t d = 1;
  while (v >= 10) { v /= 10; ++d; }
  return d;
}

// per-batch COMMIT parameters: bad run start r, bad count k, duplicate slot/sender
struct C3Batch { uint32_t r, k, dup_on, victim, dup; };

PV_HD C3Batch c3_batch(uint64_t b, uint32_t n_nodes) {
  // k_b from SHA-512("plenum-gpu/k" || u64le(b)) (no cfg byte: synth.c3_invalid_count)
  uint32_t w[16], d[16];
  const char* tag = "plenum-gpu/k";
#pragma unroll
  for (int k = 0; k < 16; ++k) w[k] = 0;
  for (int k = 0; k < 12; ++k) w[k >> 2] |= (uint32_t)(uint8_t)tag[k] << (8 * (k & 3));
  for (int k = 0; k < 8; ++k) w[(12 + k) >> 2] |= (uint32_t)(uint8_t)(b >> (8 * k)) << (8 * ((12 + k) & 3));
  int nb = 20;
  sha512_short(d, w, nb);
  C3Batch c;
  c.k = (d[0] & 0xffu) % 13u;
  nb = put_tag(w, "plenum-gpu/c3", 13, 3, b, false, 0);
  sha512_short(d, w, nb);
  const uint32_t b0 = d[0] & 0xffu, b1 = (d[0] >> 8) & 0xffu, b2 = (d[0] >> 16) & 0xffu;
  const uint32_t b3 = d[0] >> 24, b4 = d[1] & 0xffu;
  c.r = b0 % n_nodes;
  c.dup_on = ((b1 | (b2 << 8)) < 655u && n_nodes > 1) ? 1u : 0u;
  c.victim = b3 % n_nodes;
  c.dup = n_nodes > 1 ? (c.victim + 1u + b4 % (n_nodes - 1u)) % n_nodes : 0u;
  return c;
}

PV_HD uint32_t synth_len(uint32_t cfg, uint32_t mode, uint64_t i, uint32_t mlen_min, uint32_t mlen_max,
                         uint32_t n_nodes) {
  if (mode == 0) return mlen_min;
  if (mode == 2) return 36u + ndigits(i / n_nodes + 1);  // "instId:0|op:COMMIT|ppSeqNo:" <n> "|viewNo:0"
  uint32_t w[16], d[16];
  const int nb = put_tag(w, "plenum-gpu/len", 14, cfg, i, false, 0);
  sha512_short(d, w, nb);
  return mlen_min + d[0] % (mlen_max - mlen_min + 1u);
}

// lens[j] = len(M_{first+j}), j < n
__global__ void k_synth_len(uint32_t cfg, uint32_t mode, uint64_t first, uint64_t n, uint32_t mlen_min,
                            uint32_t mlen_max, uint32_t n_nodes, uint64_t* __restrict__ lens) {
  const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j < n) lens[j] = synth_len(cfg, mode, first + j, mlen_min, mlen_max, n_nodes);
}

// Exclusive prefix sum in place over x[0..n] (x[n] becomes the total):
// SCAN_ITEMS per thread, block sums, one-block scan of block sums, add back.
constexpr int SCAN_BLOCK = 256, SCAN_ITEMS = 8, SCAN_TILE = SCAN_BLOCK * SCAN_ITEMS;

__device__ uint64_t block_exclusive_scan(uint64_t v, uint64_t* total) {
  __shared__ uint64_t sh[SCAN_BLOCK];
  sh[threadIdx.x] = v;
  __syncthreads();
  for (int o = 1; o < SCAN_BLOCK; o <<= 1) {
    const uint64_t t = threadIdx.x >= (unsigned)o ? sh[threadIdx.x - o] : 0;
    __syncthreads();
    sh[threadIdx.x] += t;
    __syncthreads();
  }
  const uint64_t incl = sh[threadIdx.x];
  *total = sh[SCAN_BLOCK - 1];
  __syncthreads();
  return incl - v;
}

__global__ __launch_bounds__(SCAN_BLOCK) void k_scan_tiles(uint64_t* __restrict__ x, uint64_t m,
                                                           uint64_t* __restrict__ sums) {
  const uint64_t base = (uint64_t)blockIdx.x * SCAN_TILE + (uint64_t)threadIdx.x * SCAN_ITEMS;
  uint64_t v[SCAN_ITEMS], run = 0;
#pragma unroll
  for (int k = 0; k < SCAN_ITEMS; ++k) {
    v[k] = base + k < m ? x[base + k] : 0;
    const uint64_t t = v[k];
    v[k] = run;
    run += t;
  }
  uint64_t total;
  const uint64_t pre = block_exclusive_scan(run, &total);
#pragma unroll
  for (int k = 0; k < SCAN_ITEMS; ++k)
    if (base + k < m) x[base + k] = v[k] + pre;
  if (threadIdx.x == 0) sums[blockIdx.x] = total;
}

__global__ __launch_bounds__(SCAN_BLOCK) void k_scan_sums(uint64_t* __restrict__ sums, uint64_t nt) {
  uint64_t carry = 0;
  for (uint64_t b0 = 0; b0 < nt; b0 += SCAN_BLOCK) {
    const uint64_t j = b0 + threadIdx.x;
    const uint64_t v = j < nt ? sums[j] : 0;
    uint64_t total;
    const uint64_t pre = block_exclusive_scan(v, &total);
    if (j < nt) sums[j] = carry + pre;
    carry += total;
  }
}

__global__ __launch_bounds__(SCAN_BLOCK) void k_scan_add(uint64_t* __restrict__ x, uint64_t m,
                                                         const uint64_t* __restrict__ sums) {
  const uint64_t base = (uint64_t)blockIdx.x * SCAN_TILE;
  const uint64_t add = sums[blockIdx.x];
  for (int k = threadIdx.x; k < SCAN_TILE; k += SCAN_BLOCK)
    if (base + k < m) x[base + k] += add;
}

hipError_t launch_exclusive_scan(uint64_t* x, uint64_t m, uint64_t* sums, hipStream_t s) {
  if (m == 0) return hipSuccess;
  const uint64_t tiles = (m + SCAN_TILE - 1) / SCAN_TILE;
  hipLaunchKernelGGL(k_scan_tiles, dim3((uint32_t)tiles), dim3(SCAN_BLOCK), 0, s, x, m, sums);
  hipLaunchKernelGGL(k_scan_sums, dim3(1), dim3(SCAN_BLOCK), 0, s, sums, tiles);
  hipLaunchKernelGGL(k_scan_add, dim3((uint32_t)tiles), dim3(SCAN_BLOCK), 0, s, x, m, sums);
  return hipGetLastError();
}

uint64_t scan_sums_words(uint64_t m) { return (m + SCAN_TILE - 1) / SCAN_TILE + 1; }

hipError_t launch_synth_layout(uint32_t cfg, uint32_t mode, uint64_t first, uint64_t n, uint32_t mlen_min,
                               uint32_t mlen_max, uint32_t n_nodes, uint64_t* off, uint64_t* sums, hipStream_t s) {
  hipError_t e = hipMemsetAsync(off + n, 0, 8, s);
  if (e != hipSuccess) return e;
  if (n) {
    hipLaunchKernelGGL(k_synth_len, dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, s, cfg, mode, first, n,
                       mlen_min, mlen_max, n_nodes, off);
    e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  return launch_exclusive_scan(off, n + 1, sums, s);
}

// seeds, tamper flags and (COMMIT) senders for signature first + j
__global__ void k_synth(uint32_t cfg, uint32_t mode, uint64_t first, uint64_t n, uint32_t key_mod, uint32_t n_nodes,
                        uint8_t* __restrict__ seeds_out, uint8_t* __restrict__ tamper_out,
                        uint32_t* __restrict__ sender_out) {
  const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= n) return;
  const uint64_t i = first + j;
  uint32_t w[16], d[16];
  uint64_t key;
  uint8_t bad;
  if (mode == 2) {
    const uint64_t b = i / n_nodes;
    const uint32_t slot = (uint32_t)(i % n_nodes);
    const C3Batch c = c3_batch(b, n_nodes);
    const uint32_t snd = (c.dup_on && slot == c.victim) ? c.dup : slot;
    key = snd;
    bad = ((slot + n_nodes - c.r) % n_nodes) < c.k ? 1 : 0;
    if (sender_out) sender_out[j] = snd;
  } else {
    key = key_mod ? i % key_mod : i;
    const int nb = put_tag(w, "plenum-gpu/tamper", 17, cfg, i, false, 0);
    sha512_short(d, w, nb);
    bad = d[0] < 214748365u ? 1 : 0;
    if (sender_out) sender_out[j] = 0;
  }
  const int nb = put_tag(w, "plenum-gpu/key", 14, cfg, key, false, 0);
  sha512_short(d, w, nb);
  store8(seeds_out + 32 * j, d);
  tamper_out[j] = bad;
}

// message bytes of signature first + j at blob[off[j] - off[0] ...]
__global__ void k_synth_fill(uint32_t cfg, uint32_t mode, uint64_t first, uint64_t n, uint32_t n_nodes,
                             const uint64_t* __restrict__ off, uint8_t* __restrict__ blob) {
  const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= n) return;
  const uint64_t i = first + j;
  const uint64_t o = off[j], len = off[j + 1] - o;
  if (mode == 2) {
    const char* head = "instId:0|op:COMMIT|ppSeqNo:";
    const char* tail = "|viewNo:0";
    uint64_t q = 0;
    for (int k = 0; k < 27; ++k) blob[o + q++] = (uint8_t)head[k];
    const uint64_t v = i / n_nodes + 1;
    const uint32_t nd = ndigits(v);
    uint64_t t = v;
    for (int k = (int)nd - 1; k >= 0; --k) {
      blob[o + q + k] = (uint8_t)('0' + t % 10);
      t /= 10;
    }
    q += nd;
    for (int k = 0; k < 9; ++k) blob[o + q++] = (uint8_t)tail[k];
    return;
  }
  uint32_t w[16], d[16];
  for (uint64_t c = 0; c * 64 < len; ++c) {
    const int nb = put_tag(w, "plenum-gpu/msg", 14, cfg, i, true, c);
    sha512_short(d, w, nb);
    const uint64_t lim = len - c * 64 < 64 ? len - c * 64 : 64;
    if (lim == 64 && ((o + c * 64) & 3) == 0) {
      uint32_t* q = reinterpret_cast<uint32_t*>(blob + o + c * 64);
#pragma unroll
      for (int k = 0; k < 16; ++k) q[k] = d[k];
    } else {
      for (uint64_t k = 0; k < lim; ++k) blob[o + c * 64 + k] = (uint8_t)(d[k >> 2] >> (8 * (k & 3)));
    }
  }
}

__global__ void k_tamper(uint64_t first, uint64_t n, const uint8_t* __restrict__ tamper,
                         const uint64_t* __restrict__ off, uint8_t* __restrict__ blob, uint8_t* __restrict__ sig) {
  const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= n || !tamper[j]) return;
  const uint64_t i = first + j;
  const uint64_t o = off[j], len = off[j + 1] - o;
  const uint8_t bit = (uint8_t)(1u << (i % 8));
  const uint64_t kind = i % 3;
  if (kind == 0 && len > 0) blob[o + (i / 3) % len] ^= bit;
  else if (kind == 1 || (kind == 0 && len == 0)) sig[64 * j + (i / 3) % 32] ^= bit;
  else sig[64 * j + 32 + (i / 3) % 16] ^= bit;
}

hipError_t launch_synth(uint32_t cfg, uint32_t mode, uint64_t first, uint64_t n, uint32_t key_mod, uint32_t n_nodes,
                        uint8_t* seeds_out, uint8_t* tamper_out, uint32_t* sender_out, hipStream_t s) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_synth, dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, s, cfg, mode, first, n, key_mod,
                     n_nodes, seeds_out, tamper_out, sender_out);
  return hipGetLastError();
}

hipError_t launch_synth_fill(uint32_t cfg, uint32_t mode, uint64_t first, uint64_t n, uint32_t n_nodes,
                             const uint64_t* off, uint8_t* blob, hipStream_t s) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_synth_fill, dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, s, cfg, mode, first, n, n_nodes,
                     off, blob);
  return hipGetLastError();
}

hipError_t launch_tamper(uint64_t first, uint64_t n, const uint8_t* tamper, const uint64_t* off, uint8_t* blob,
                         uint8_t* sig, hipStream_t s) {
  if (n == 0) return hipSuccess;
  const uint64_t blocks = (n + 255) / 256;
  hipLaunchKernelGGL(k_tamper, dim3((uint32_t)blocks), dim3(256), 0, s, first, n, tamper, off, blob, sig);
  return hipGetLastError();
}

}  // namespace pv
