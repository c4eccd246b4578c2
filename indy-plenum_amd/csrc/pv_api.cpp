// C-ABI layer of libplenum_verify.so (include/plenum_verify.h).
//
// Owns per-device state (stream, base-point table, workspaces), shards host
// batches over the devices in a mask (contiguous index ranges, SURVEY.md
// §8(e)), and launches the kernels in pv_kernels.hip.  No exceptions cross
// the ABI: every entry point returns 0 or a negative code and records a
// message for pv_last_error().
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <atomic>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <condition_variable>
#include <memory>
#include <random>
#include <mutex>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#include "../../include/plenum_verify.h"
#include "pv_kernels.h"

static_assert(PV_KEY_WORDS == (unsigned)pv::KEYTAB_WORDS, "prepared-key layout");
static_assert(PV_KEY_WORDS_WIDE == (unsigned)pv::KEYTAB_WIDE_WORDS, "wide prepared-key layout");

namespace pvbls {
void set_quad_max(uint64_t n);   // pv_bls.hip
void set_oct_max(uint64_t n);
}

namespace {

thread_local std::string g_err;

int fail(int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  g_err = buf;
  return code;
}

// host-buffer pipeline (pv_verify_batch): a shard runs as leading ramp
// chunks and then at most PV_HOST_CHUNKS chunks of at least PV_HOST_CHUNK_MIN
// signatures
#define PV_HOST_CHUNKS 8
#define PV_HOST_CHUNK_MIN 32768
// ramp: leading chunks of 32768, 65536, ... signatures (below a regular
// chunk), so the first grid starts after a ~12 MB DMA (C2 end to end with
// fused chunks 11.6 vs 12.1 ms, profiles/r02_ab_fused_chunking.jsonl)
#define PV_HOST_RAMP 32768
// generic batches of at most this many signatures run the latency-mode curve
// kernel (k_verify_quad: one launch, lane quads per point); tuning.lat_max (0 disables)
#define PV_LAT_MAX 32768
// keyed batches (prepared keys) of at most this many signatures run the keyed
// latency kernel (k_verify_quad_keyed); tuning.lat_keyed_max (0 disables)
#define PV_LAT_KEYED_MAX 8192
// BLS calls of at most this many checks run the lane-quad check kernel
// (pv_bls.hip; the same default as its PV_BLS_QUAD_MAX); tuning.bls_quad_max
#define PV_BLS_QUAD_MAX_DEFAULT 32768
// ... and calls of at most this many the lane-octet kernel; tuning.bls_oct_max
#define PV_BLS_OCT_MAX_DEFAULT 4096
// host-buffer calls of at most this many signatures skip the H2D / D2H copies:
// the latency kernel reads the gathered inputs from, and writes the verdicts
// to, fine-grained page-locked host memory (one launch per call instead of
// copy + launch + copy); tuning.small_zc_max (0 = always copy)
#define PV_SMALL_ZC_MAX 2048
// shards of at least this many signatures decide PV_FLAG_DEDUP_KEYS from a sample
#define PV_DEDUP_SAMPLE_MIN 262144
// chunk gathers into the pinned staging ring use up to this many host threads
// (tuning.host_copy_threads); gathers under PV_HOST_PAR_MIN bytes stay on
// the calling thread
#define PV_HOST_COPY_THREADS 8
#define PV_HOST_PAR_MIN (4u << 20)
// largest page-locked staging slot (two per device, plus the shard's verdicts):
// at most ~1 GiB of locked host memory per device while pinned staging is on
#define PV_HOST_PIN_MAX (size_t(512) << 20)

#define HIP_OK(expr)                                                                          \
  do {                                                                                        \
    hipError_t e_ = (expr);                                                                   \
    if (e_ != hipSuccess)                                                                     \
      return fail(e_ == hipErrorOutOfMemory ? PV_ENOMEM : PV_EIO, "%s failed: %s (%s:%d)", #expr, \
                  hipGetErrorString(e_), __FILE__, __LINE__);                                 \
  } while (0)

template <typename T>
struct DevBuf {
  T* p = nullptr;
  size_t cap = 0;  // elements
  hipError_t ensure(size_t n) {
    if (n <= cap && p) return hipSuccess;
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
    size_t want = n < 64 ? 64 : n;
    hipError_t e = hipMalloc(reinterpret_cast<void**>(&p), want * sizeof(T));
    if (e == hipSuccess) cap = want;
    return e;
  }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
  }
};

// page-locked host buffer (one slot of the host-buffer staging ring)
struct PinBuf {
  uint8_t* p = nullptr;
  size_t cap = 0;  // bytes
  unsigned flags = hipHostMallocDefault;
  uint8_t* dev = nullptr;  // device address of a mapped buffer (looked up once per allocation)
  hipError_t ensure(size_t n) {
    if (n <= cap && p) return hipSuccess;
    if (p) (void)hipHostFree(p);
    p = nullptr;
    dev = nullptr;
    cap = 0;
    hipError_t e = hipHostMalloc(reinterpret_cast<void**>(&p), n, flags);
    if (e == hipSuccess && (flags & hipHostMallocMapped)) {
      void* a = nullptr;
      e = hipHostGetDevicePointer(&a, p, 0);
      if (e != hipSuccess) {
        (void)hipHostFree(p);
        p = nullptr;
        return e;
      }
      dev = static_cast<uint8_t*>(a);
    }
    if (e == hipSuccess) cap = n;
    return e;
  }
  void release() {
    if (p) (void)hipHostFree(p);
    p = nullptr;
    dev = nullptr;
    cap = 0;
  }
};

// host -> host copies of one chunk's inputs, split over `threads` threads by
// byte range of the concatenated jobs.  A job with `rebase` set copies u64
// values minus `rebase` (the chunk's message offsets made shard-relative while
// they are gathered: no separate pass over all offsets before the first DMA);
// it must be the FIRST job, so that the 8-byte-multiple piece boundaries never
// split one of its values between two threads.
struct CopyJob {
  uint8_t* dst;
  const uint8_t* src;
  size_t n;            // bytes (a multiple of 8 for rebased jobs)
  uint64_t rebase = 0;
  bool u64 = false;
};

// rebased u64 jobs also check that the values never decrease (message
// offsets): *bad is set, the caller refuses the chunk before any kernel reads it
void copy_part(const CopyJob& j, size_t lo, size_t hi, std::atomic<bool>* bad) {
  if (!j.u64) {
    memcpy(j.dst + lo, j.src + lo, hi - lo);
    return;
  }
  const uint64_t* a = reinterpret_cast<const uint64_t*>(j.src + lo);
  uint64_t* b = reinterpret_cast<uint64_t*>(j.dst + lo);
  uint64_t prev = lo ? a[-1] : a[0];
  bool dec = false;
  for (size_t k = 0; k < (hi - lo) / 8; ++k) {
    dec |= a[k] < prev;
    prev = a[k];
    b[k] = a[k] - j.rebase;
  }
  if (dec && bad) bad->store(true, std::memory_order_relaxed);
}

void gather_range(const CopyJob* jobs, int nj, size_t a, size_t b, std::atomic<bool>* bad) {
  size_t base = 0;
  for (int j = 0; j < nj && base < b; base += jobs[j].n, ++j) {
    const size_t lo = std::max(a, base) - base, hi = std::min(b, base + jobs[j].n) - base;
    if (lo < hi) copy_part(jobs[j], lo, hi, bad);
  }
}

// Persistent gather threads of one device (the host pipeline gathers every
// chunk: starting threads per chunk cost ~20 us each).  run() splits the
// concatenated jobs into `threads` pieces of 8-byte multiples; piece 0 runs on
// the caller.  Threads are started lazily; one that cannot be started leaves
// its pieces to the caller (no exception crosses the ABI).  Used by one
// thread at a time (a device's shard worker).
struct GatherPool {
  std::vector<std::thread> th;
  std::mutex mu;
  std::condition_variable cv, cv_done;
  const CopyJob* jobs = nullptr;
  int nj = 0, pieces = 0;
  size_t total = 0, piece = 0;
  std::atomic<bool>* bad = nullptr;
  uint64_t gen = 0;
  int pending = 0;
  bool stop = false;

  void worker(int t) {
    uint64_t seen = 0;
    std::unique_lock<std::mutex> lk(mu);
    for (;;) {
      cv.wait(lk, [&] { return stop || gen != seen; });
      if (stop) return;
      seen = gen;
      const bool mine = t < pieces;
      const size_t a = std::min(total, piece * t), b = std::min(total, piece * (t + 1));
      const CopyJob* J = jobs;
      const int n = nj;
      std::atomic<bool>* flag = bad;
      lk.unlock();
      if (mine) gather_range(J, n, a, b, flag);
      lk.lock();
      if (--pending == 0) cv_done.notify_one();
    }
  }

  void run(const CopyJob* js, int n, int threads, std::atomic<bool>* flag) {
    size_t tot = 0;
    for (int j = 0; j < n; ++j) tot += js[j].n;
    if (threads <= 1 || tot < PV_HOST_PAR_MIN) {
      gather_range(js, n, 0, tot, flag);
      return;
    }
    while ((int)th.size() < threads - 1) {
      try {
        th.emplace_back(&GatherPool::worker, this, (int)th.size() + 1);
      } catch (...) {
        break;
      }
    }
    const int p = (int)th.size() + 1;
    const size_t pc = ((tot + p - 1) / p + 7) & ~size_t(7);
    {
      std::lock_guard<std::mutex> lk(mu);
      jobs = js;
      nj = n;
      total = tot;
      piece = pc;
      pieces = p;
      bad = flag;
      pending = (int)th.size();
      ++gen;
    }
    cv.notify_all();
    gather_range(js, n, 0, std::min(tot, pc), flag);
    std::unique_lock<std::mutex> lk(mu);
    cv_done.wait(lk, [&] { return pending == 0; });
  }

  void shutdown() {
    {
      std::lock_guard<std::mutex> lk(mu);
      stop = true;
    }
    cv.notify_all();
    for (auto& t : th) t.join();
    th.clear();
    stop = false;
  }
  ~GatherPool() { shutdown(); }  // idle threads never outlive the pool (process exit included)
};

// Distinct 32-byte keys of a host batch (PV_FLAG_DEDUP_KEYS): open addressing
// with linear probing over 32-bit slots (0 = empty, else 1 + distinct index),
// hashed from the key's first 16 bytes; no per-key allocation.
struct KeyIndex {
  std::vector<uint32_t> slot;
  uint64_t mask = 0;
  const uint8_t* base = nullptr;  // key j at base + 32 * first[j]
  std::vector<uint64_t> first;    // position of each distinct key's first use
  void reset(const uint8_t* keys, uint64_t n) {
    uint64_t cap = 64;
    while (cap < 2 * n) cap <<= 1;
    slot.assign(cap, 0);
    mask = cap - 1;
    base = keys;
    first.clear();
  }
  // distinct index of key i (inserted on first sight)
  uint32_t insert(uint64_t i) {
    const uint8_t* k = base + 32 * i;
    uint64_t a, b;
    memcpy(&a, k, 8);
    memcpy(&b, k + 8, 8);
    uint64_t h = (a ^ (b * 0x9E3779B97F4A7C15ull)) * 0xBF58476D1CE4E5B9ull;
    for (uint64_t p = (h >> 17) & mask;; p = (p + 1) & mask) {
      const uint32_t v = slot[p];
      if (!v) {
        first.push_back(i);
        slot[p] = (uint32_t)first.size();
        return v + (uint32_t)first.size() - 1;
      }
      if (!memcmp(base + 32 * first[v - 1], k, 32)) return v - 1;
    }
  }
};

// Persistent verifying-key cache (pv_keycache_add): host-side index of the
// cached 32-byte keys; key j's comb tables sit in slot j of every device's
// `kc` table.  Open addressing over all 32 bytes with a per-process random
// seed (keys come from the ledger, so their first bytes are attacker-chosen).
struct KeyCache {
  std::vector<uint8_t> keys;      // 32 bytes per cached key, slot order
  std::vector<uint32_t> slot;     // 0 = empty, else 1 + slot
  uint64_t mask = 0;
  uint64_t seed = 0;
  uint64_t count() const { return keys.size() / 32; }
  uint64_t hash(const uint8_t* k) const {
    uint64_t h = seed;
    for (int i = 0; i < 4; ++i) {
      uint64_t w;
      memcpy(&w, k + 8 * i, 8);
      h = (h ^ w) * 0x9E3779B97F4A7C15ull;
      h ^= h >> 29;
    }
    return h;
  }
  // slot of key k, or UINT32_MAX
  uint32_t find(const uint8_t* k) const {
    if (slot.empty()) return UINT32_MAX;
    for (uint64_t p = hash(k) & mask;; p = (p + 1) & mask) {
      const uint32_t v = slot[p];
      if (!v) return UINT32_MAX;
      if (!memcmp(keys.data() + 32 * (uint64_t)(v - 1), k, 32)) return v - 1;
    }
  }
  void rehash(uint64_t cap) {
    slot.assign(cap, 0);
    mask = cap - 1;
    for (uint64_t j = 0; j < count(); ++j)
      for (uint64_t p = hash(keys.data() + 32 * j) & mask;; p = (p + 1) & mask)
        if (!slot[p]) {
          slot[p] = (uint32_t)(j + 1);
          break;
        }
  }
  // append keys (already known to be absent and distinct) as new slots
  void commit(const std::vector<uint8_t>& add) {
    if (!seed) seed = ((uint64_t)std::random_device{}() << 32 | std::random_device{}()) | 1;
    keys.insert(keys.end(), add.begin(), add.end());
    uint64_t cap = slot.size() ? slot.size() : 64;
    while (cap < 2 * count()) cap <<= 1;
    rehash(cap);
  }
  void clear() {
    keys.clear();
    slot.clear();
    mask = 0;
  }
};
KeyCache g_kc;

// PV_CURVE_MODE (read at pv_init): "half" (default) = half-size scalars with
// full-length tasks for deferred records; "full" = every record deferred
// (full-length verdicts through the same kernel: A/B timing and tests);
// "grouped" = the previous generic kernel (k_curve, 8 signatures per lane
// sharing one inversion).  Verdicts are identical in every mode.
enum class CurveMode { Half, Full, Grouped };

// Verify workspaces and the compute stream they are used on.  Device-pointer
// calls use ws[0] (stream = the device stream or the caller's; pv_*_async:
// ws[slot]); the host-buffer pipeline alternates chunks over ws[0] and ws[1]
// on their two streams, so the kernels of chunk c + 1 fill the tail of chunk
// c's persistent grid
// instead of waiting for it (the scratch of concurrently running curve grids
// must not alias: one per workspace).
struct Workspace {
  hipStream_t stream = nullptr;
  DevBuf<uint32_t> scratch;            // per-lane A / -R tables for the persistent curve grid
  DevBuf<uint32_t> h;                  // SHA-512 digest, 16 words per signature
  DevBuf<unsigned long long> counter;  // hash-kernel work queue
  DevBuf<uint8_t> pre;
  DevBuf<uint64_t> bitmap;
  DevBuf<uint32_t> hrec, dlist;        // lattice records, deferred indices (half-size path)
  DevBuf<unsigned long long> qc;       // [0] deferred count, [1] curve task queue
  bool half_ran = false;               // qc[0] holds the last generic batch's deferred count
  // last use: recorded after every enqueue on this workspace (whatever stream
  // it ran on); the next use on another stream waits for it, so an async batch
  // still running on a caller's stream never shares scratch / h / hrec / qc /
  // counter / bitmap with a later sync, host-buffer or async call
  hipEvent_t done = nullptr;
  hipStream_t done_on = nullptr;
  void release() {
    scratch.release(); h.release(); counter.release(); pre.release(); bitmap.release();
    hrec.release(); dlist.release(); qc.release();
    if (done) (void)hipEventDestroy(done);
    done = nullptr;
    done_on = nullptr;
  }
};

// order a use of workspace w on stream s after its previous use
int ws_begin(Workspace& w, hipStream_t s) {
  if (w.done_on && w.done_on != s) HIP_OK(hipStreamWaitEvent(s, w.done, 0));
  return PV_OK;
}

int ws_end(Workspace& w, hipStream_t s) {
  HIP_OK(hipEventRecord(w.done, s));
  w.done_on = s;
  return PV_OK;
}

struct Device {
  int id = -1;   // engine device id: the device_mask bit and the `device` argument
  int ord = -1;  // HIP ordinal (== id, except under pv_test_init_dup)
  hipStream_t stream = nullptr;
  hipStream_t copy = nullptr;   // host-buffer calls: H2D of chunk c+1 overlaps the kernels of chunk c
  hipEvent_t copied = nullptr;  // recorded on `copy` after each chunk's inputs, waited on by `stream`
  // tuning.host_staging: PV_STAGING_PINNED (default) gathers chunk c of a
  // host-buffer call into page-locked slot c & 1 and DMAs it from there;
  // PV_STAGING_PAGEABLE hands the caller's buffers to hipMemcpyAsync (runtime staging)
  bool pinned = true;
  int copy_threads = PV_HOST_COPY_THREADS;
  int host_chunks = PV_HOST_CHUNKS;  // tuning.host_chunks (1..256)
  int first_pct = 50;                // first chunk, % of a regular one; tuning.host_first_pct (10..100)
  // leading chunks r, 2r, 4r, ... below a regular chunk instead of one first
  // chunk (tuning.host_ramp; 0 = off, first_pct then sizes the first chunk)
  uint64_t ramp = PV_HOST_RAMP;
  size_t pin_max = PV_HOST_PIN_MAX;  // largest page-locked slot; tuning.host_pin_max_mb (16..4096)
  uint64_t lat_max = PV_LAT_MAX;     // generic batches up to this size use the latency kernel; tuning.lat_max (0 = off)
  uint64_t lat_keyed_max = PV_LAT_KEYED_MAX;  // keyed batches up to this size: k_verify_quad_keyed
  uint64_t zc_max = PV_SMALL_ZC_MAX;          // host calls up to this size: zero-copy (tuning.small_zc_max)
  PinBuf zc_in, zc_out;                       // fine-grained page-locked image / verdicts of zero-copy calls
  PinBuf zc_flag;                             // completion word of zero-copy calls, polled by the host
  uint32_t zc_seq = 0;
  DevBuf<uint32_t> zc_done;                   // block counter of a keyed kernel that writes the word itself
  bool zc_done_armed = false;                 // zc_done zeroed (the kernel's last block re-arms it)
  bool lat_quad = true;              // latency kernel: k_verify_quad (lane quads); PV_LAT_PAIR: k_curve_lat
  // host-buffer chunks of generic batches: one k_chunk_half launch per chunk
  // + one k_verify_quad_list pass for the deferred records; tuning.host_fused 0:
  // k_hash + k_lattice + k_curve_half per chunk (the device-resident schedule)
  bool chunk_fused = true;
  DevBuf<uint32_t> dl;               // shard indices deferred by k_chunk_half
  DevBuf<unsigned long long> dlc;    // their count
  hipEvent_t joined = nullptr;       // ws[1] drained into ws[0] (deferred pass)
  PinBuf pin[2];
  std::shared_ptr<GatherPool> pool = std::make_shared<GatherPool>();  // host gather threads
  PinBuf vout;  // page-locked verdicts of the shard (D2H target; copied to the caller after the drain)
  hipEvent_t staged[2] = {nullptr, nullptr};  // slot i's H2D has finished
  hipEvent_t keys_ready = nullptr;            // prepared-key table built (host pipeline, ws[0] -> ws[1])
  // pv_verify_keys_device_async: slot i's key preparation runs on kside[i],
  // forked from the caller's stream after the workspace's previous use (kfork)
  // and joined back before the curve kernel (kjoin), so it overlaps the hash stage
  hipStream_t kside[2] = {nullptr, nullptr};
  hipEvent_t kfork[2] = {nullptr, nullptr}, kjoin[2] = {nullptr, nullptr};
  int cu_count = 0;
  int curve_blocks = 0;
  int hash_blocks = 0;
  DevBuf<uint32_t> btab;
  DevBuf<uint32_t> bw;        // radix-2^16 base-point chunk tables (half-size path, keyed comb)
  Workspace ws[2];
  int last_ws = 0;            // workspace of the last generic verify (pv_curve_stats)
  size_t scratch_words = 0;   // per-workspace curve scratch
  DevBuf<unsigned long long> counter;  // SHA-256 work queue
  // staging for host-memory calls
  DevBuf<uint8_t> pk, sig, blob, verdict, tamper;
  DevBuf<uint8_t> stage;      // small host-buffer calls: device image of pinned slot 0 (run_small)
  DevBuf<uint64_t> off, batch_off;
  DevBuf<uint32_t> sender, votes;
  DevBuf<uint32_t> tflag, tbits;  // tally: out-of-range sender flag; staged voter bitmaps
  DevBuf<uint8_t> reached;
  DevBuf<uint64_t> scan;      // block sums of the device prefix scan
  DevBuf<uint32_t> ktab, kidx;  // prepared keys + per-signature key index (deduplicated host batches)
  DevBuf<uint32_t> kscr, kscr2;  // key-preparation scratch (kscr2: async slot 1)
  DevBuf<uint32_t> mk0, mk1;    // Merkle level ping-pong / leaf digests
  DevBuf<uint32_t> kc;          // persistent key cache: slot j = comb tables of g_kc key j
  uint64_t kc_count = 0;        // slots prepared on this device
  DevBuf<uint8_t> kcpk;         // staging of keys being added
  int sha256_blocks = 0;
  int curve_blocks_keyed = 0;
  int curve_half_blocks = 0;
  CurveMode mode = CurveMode::Half;
  // pv_kernel_timing: HIP-event times of every verify launch while enabled
  bool live_timing = false;
  float live_hash = 0, live_curve = 0;
  float live_sha = 0;   // the SHA-512 part of the hash interval (pre-checks + k_hash, no k_lattice)
  uint64_t live_launches = 0;
  // live timing records four events per launch without waiting (pipelined
  // callers keep launches in flight); they are resolved when the pool fills
  // up and when timing stops
  struct LiveRec {
    hipEvent_t e[4] = {nullptr, nullptr, nullptr, nullptr};   // start, prep end, curve end, k_hash end
  };
  std::vector<LiveRec> live_pool;
  size_t live_used = 0;
  hipEvent_t ev[4] = {nullptr, nullptr, nullptr, nullptr};
};

// restores the caller's current HIP device on scope exit (torch shares it)
struct DeviceGuard {
  int prev = -1;
  DeviceGuard() { (void)hipGetDevice(&prev); }
  ~DeviceGuard() {
    if (prev >= 0) (void)hipSetDevice(prev);
  }
};

std::mutex g_mu;
std::vector<Device> g_devs;

Device* find_dev(int id) {
  for (auto& d : g_devs)
    if (d.id == id) return &d;
  return nullptr;
}

// the process's schedule tuning (include/plenum_verify.h, pv_set_tuning):
// defaults only, never the environment
pv_tuning default_tuning() {
  pv_tuning t{};
  t.struct_size = sizeof(pv_tuning);
  t.curve_mode = PV_CURVE_HALF;
  t.lat_max = PV_LAT_MAX;
  t.lat_keyed_max = PV_LAT_KEYED_MAX;
  t.small_zc_max = PV_SMALL_ZC_MAX;
  t.lat_kernel = PV_LAT_QUAD;
  t.host_fused = 1;
  t.host_staging = PV_STAGING_PINNED;
  t.host_chunks = PV_HOST_CHUNKS;
  t.host_first_pct = 50;
  t.host_copy_threads = PV_HOST_COPY_THREADS;
  t.host_ramp = PV_HOST_RAMP;
  t.host_pin_max_mb = (uint32_t)(PV_HOST_PIN_MAX >> 20);
  t.bls_quad_max = PV_BLS_QUAD_MAX_DEFAULT;
  t.bls_oct_max = PV_BLS_OCT_MAX_DEFAULT;
  return t;
}
pv_tuning g_tune = default_tuning();
int g_dup = 0;   // pv_test_init_dup: engine devices sharing HIP device 0 (test only)

int check_tuning(const pv_tuning& t) {
  if (t.struct_size != sizeof(pv_tuning))
    return fail(PV_EINVAL, "struct_size %u != sizeof(pv_tuning) %zu", t.struct_size, sizeof(pv_tuning));
  if (t.curve_mode > PV_CURVE_GROUPED) return fail(PV_EINVAL, "unknown curve mode %u", t.curve_mode);
  if (t.lat_max > (1ull << 20) || t.lat_keyed_max > (1ull << 20) || t.small_zc_max > (1ull << 20))
    return fail(PV_EINVAL, "lat_max / lat_keyed_max / small_zc_max must be <= 2^20");
  if (t.lat_kernel > PV_LAT_PAIR) return fail(PV_EINVAL, "unknown latency kernel %u", t.lat_kernel);
  if (t.host_fused > 1) return fail(PV_EINVAL, "host_fused must be 0 or 1");
  if (t.host_staging > PV_STAGING_PAGEABLE) return fail(PV_EINVAL, "unknown staging mode %u", t.host_staging);
  if (t.host_chunks < 1 || t.host_chunks > 256) return fail(PV_EINVAL, "host_chunks must be in 1..256");
  if (t.host_first_pct < 10 || t.host_first_pct > 100) return fail(PV_EINVAL, "host_first_pct must be in 10..100");
  if (t.host_copy_threads < 1 || t.host_copy_threads > 64) return fail(PV_EINVAL, "host_copy_threads must be in 1..64");
  if (t.host_ramp != 0 && (t.host_ramp < 1024 || t.host_ramp > (1ull << 20)))
    return fail(PV_EINVAL, "host_ramp must be 0 or in 1024..2^20");
  if (t.host_pin_max_mb < 16 || t.host_pin_max_mb > 4096) return fail(PV_EINVAL, "host_pin_max_mb must be in 16..4096");
  if (t.host_trace > 1) return fail(PV_EINVAL, "host_trace must be 0 or 1");
  if (t.bls_quad_max > (1u << 20) || t.bls_oct_max > (1u << 20))
    return fail(PV_EINVAL, "bls_quad_max / bls_oct_max must be <= 2^20");
  if (t.reserved != 0) return fail(PV_EINVAL, "reserved must be 0");
  return PV_OK;
}

void apply_tuning(Device& d, const pv_tuning& t) {
  const CurveMode m = t.curve_mode == PV_CURVE_HALF ? CurveMode::Half
                      : t.curve_mode == PV_CURVE_FULL ? CurveMode::Full : CurveMode::Grouped;
  if (m != d.mode)
    for (auto& w : d.ws) w.half_ran = false;
  d.mode = m;
  d.lat_max = t.lat_max;
  d.lat_keyed_max = t.lat_keyed_max;
  d.zc_max = t.small_zc_max;
  d.lat_quad = t.lat_kernel == PV_LAT_QUAD;
  d.chunk_fused = t.host_fused != 0;
  d.host_chunks = (int)t.host_chunks;
  d.first_pct = (int)t.host_first_pct;
  d.copy_threads = (int)t.host_copy_threads;
  d.ramp = t.host_ramp;
  d.pin_max = size_t(t.host_pin_max_mb) << 20;
  const bool pinned = t.host_staging == PV_STAGING_PINNED;
  if (d.pinned && !pinned && d.copy) {   // pageable staging holds no page-locked memory
    (void)hipSetDevice(d.ord);
    (void)hipStreamSynchronize(d.copy);
    d.pin[0].release();
    d.pin[1].release();
    d.vout.release();
  }
  d.pinned = pinned;
}

int init_device(Device& d) {
  HIP_OK(hipSetDevice(d.ord));
  HIP_OK(hipStreamCreateWithFlags(&d.stream, hipStreamNonBlocking));
  d.ws[0].stream = d.stream;
  HIP_OK(hipStreamCreateWithFlags(&d.ws[1].stream, hipStreamNonBlocking));
  HIP_OK(hipStreamCreateWithFlags(&d.copy, hipStreamNonBlocking));
  HIP_OK(hipEventCreateWithFlags(&d.copied, hipEventDisableTiming));
  for (auto& e : d.staged) HIP_OK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  HIP_OK(hipEventCreateWithFlags(&d.keys_ready, hipEventDisableTiming));
  HIP_OK(hipEventCreateWithFlags(&d.joined, hipEventDisableTiming));
  for (auto& w : d.ws) HIP_OK(hipEventCreateWithFlags(&w.done, hipEventDisableTiming));
  for (int i = 0; i < 2; ++i) {
    HIP_OK(hipStreamCreateWithFlags(&d.kside[i], hipStreamNonBlocking));
    HIP_OK(hipEventCreateWithFlags(&d.kfork[i], hipEventDisableTiming));
    HIP_OK(hipEventCreateWithFlags(&d.kjoin[i], hipEventDisableTiming));
  }
  d.zc_in.flags = d.zc_out.flags = d.zc_flag.flags = hipHostMallocCoherent | hipHostMallocMapped;
  apply_tuning(d, g_tune);
  hipDeviceProp_t prop;
  HIP_OK(hipGetDeviceProperties(&prop, d.ord));
  d.cu_count = prop.multiProcessorCount;
  HIP_OK(d.btab.ensure(pv::BTAB_CHUNKS * pv::BTAB_ENTRIES * pv::BTAB_WORDS));
  HIP_OK(pv::launch_btable_init(d.btab.p, d.stream));
  HIP_OK(d.bw.ensure(pv::BWTAB_WORDS));
  HIP_OK(pv::launch_bw_init(d.bw.p, d.stream));
  // persistent curve grid: resident blocks per CU from the occupancy query
  // (kept <= 4 blocks of 256 threads per CU, see cdna_hip_programming.md §1)
  int per_cu = 0;
  HIP_OK(pv::curve_occupancy(&per_cu));
  if (per_cu < 1) per_cu = 1;
  if (per_cu > 4) per_cu = 4;
  d.curve_blocks = d.cu_count * per_cu;
  int halfper = 0;
  HIP_OK(pv::curve_half_occupancy(&halfper));
  if (halfper < 1) halfper = 1;
  if (halfper > 4) halfper = 4;
  d.curve_half_blocks = d.cu_count * halfper;
  {
    const size_t a = (size_t)d.curve_blocks * pv::ATAB_WORDS, b = (size_t)d.curve_half_blocks * pv::HALF_SCRATCH_WORDS;
    d.scratch_words = (a > b ? a : b) * pv::CURVE_BLOCK;
    HIP_OK(d.ws[0].scratch.ensure(d.scratch_words));
  }
  HIP_OK(d.ws[0].qc.ensure(2));
  int kper = 0;
  HIP_OK(pv::curve_occupancy(&kper, true));
  if (kper < 1) kper = 1;
  if (kper > per_cu) kper = per_cu;
  d.curve_blocks_keyed = d.cu_count * kper;
  int sper = 0;
  HIP_OK(pv::sha256_occupancy(&sper));
  d.sha256_blocks = d.cu_count * (sper < 1 ? 1 : sper);
  int hper = 0;
  HIP_OK(pv::hash_occupancy(&hper));
  if (hper < 1) hper = 1;
  d.hash_blocks = d.cu_count * hper;
  HIP_OK(d.counter.ensure(1));
  HIP_OK(d.ws[0].counter.ensure(1));
  for (auto& e : d.ev) HIP_OK(hipEventCreate(&e));
  HIP_OK(hipStreamSynchronize(d.stream));
  return PV_OK;
}

void release_device(Device& d) {
  if (d.id < 0) return;
  (void)hipSetDevice(d.ord);
  for (auto& w : d.ws)
    if (w.stream) (void)hipStreamSynchronize(w.stream);
  for (int i = 0; i < 2; ++i) {
    if (d.kside[i]) (void)hipStreamSynchronize(d.kside[i]), (void)hipStreamDestroy(d.kside[i]);
    if (d.kfork[i]) (void)hipEventDestroy(d.kfork[i]);
    if (d.kjoin[i]) (void)hipEventDestroy(d.kjoin[i]);
    d.kside[i] = nullptr;
    d.kfork[i] = d.kjoin[i] = nullptr;
  }
  d.btab.release(); d.bw.release(); d.counter.release();
  for (auto& w : d.ws) w.release();
  if (d.ws[1].stream) (void)hipStreamDestroy(d.ws[1].stream);
  for (auto& w : d.ws) w.stream = nullptr;
  d.pk.release(); d.sig.release(); d.blob.release(); d.verdict.release(); d.tamper.release(); d.stage.release();
  d.off.release(); d.batch_off.release();
  d.sender.release(); d.votes.release(); d.reached.release(); d.scan.release(); d.tflag.release(); d.tbits.release();
  d.ktab.release(); d.kidx.release(); d.kscr.release(); d.kscr2.release(); d.mk0.release(); d.mk1.release();
  d.kc.release(); d.kcpk.release();
  d.kc_count = 0;
  for (auto& e : d.ev)
    if (e) (void)hipEventDestroy(e), e = nullptr;
  for (auto& r : d.live_pool)
    for (auto& e : r.e)
      if (e) (void)hipEventDestroy(e), e = nullptr;
  d.live_pool.clear();
  d.live_used = 0;
  if (d.copied) (void)hipEventDestroy(d.copied);
  d.copied = nullptr;
  if (d.copy) (void)hipStreamSynchronize(d.copy), (void)hipStreamDestroy(d.copy);
  for (auto& e : d.staged)
    if (e) (void)hipEventDestroy(e), e = nullptr;
  if (d.keys_ready) (void)hipEventDestroy(d.keys_ready);
  d.keys_ready = nullptr;
  if (d.joined) (void)hipEventDestroy(d.joined);
  d.joined = nullptr;
  d.dl.release(); d.dlc.release();
  d.pin[0].release();
  d.pin[1].release();
  d.zc_in.release();
  d.zc_out.release();
  d.zc_flag.release();
  d.zc_done.release();
  d.zc_done_armed = false;
  d.vout.release();
  if (d.pool) d.pool->shutdown();
  d.copy = nullptr;
  if (d.stream) (void)hipStreamDestroy(d.stream);
  d.stream = nullptr;
  d.id = -1;
}

// fold the recorded live-timing events into the sums (waits for them)
int resolve_live(Device& d) {
  for (size_t k = 0; k < d.live_used; ++k) {
    hipEvent_t* e = d.live_pool[k].e;
    HIP_OK(hipEventSynchronize(e[2]));
    float a = 0, b = 0, c = 0;
    HIP_OK(hipEventElapsedTime(&a, e[0], e[1]));
    HIP_OK(hipEventElapsedTime(&b, e[1], e[2]));
    HIP_OK(hipEventElapsedTime(&c, e[0], e[3]));
    d.live_hash += a;
    d.live_sha += c;
    d.live_curve += b;
  }
  d.live_used = 0;
  return PV_OK;
}

// The two stages of a verify for device-resident inputs, on stream s with
// workspace w.  prep: pre-checks + SHA-512 (+ the lattice stage of the
// half-size path); curve: the curve kernel writing verdicts + bitmap.
// `bm` = the caller's bitmap or null (then w.bitmap).
uint64_t* stage_bitmap(Workspace& w, uint64_t* bitmap, uint64_t n, int& rc) {
  rc = PV_OK;
  if (bitmap) return bitmap;
  const hipError_t e = w.bitmap.ensure((n + 63) / 64);
  if (e != hipSuccess)
    rc = fail(e == hipErrorOutOfMemory ? PV_ENOMEM : PV_EIO, "bitmap allocation failed: %s", hipGetErrorString(e));
  return w.bitmap.p;
}

// small generic batches: the whole verify is one k_verify_quad launch
bool lat_fused(const Device& d, const uint32_t* ktab, uint64_t n) {
  return !ktab && d.mode != CurveMode::Grouped && n <= d.lat_max && d.lat_quad;
}
// small keyed batches: one k_verify_quad_keyed launch
bool lat_keyed(const Device& d, const uint32_t* ktab, uint64_t n, bool wide) {
  return ktab && !wide && n <= d.lat_keyed_max && d.lat_quad;
}

int enqueue_prep(Device& d, Workspace& w, const uint8_t* pk, const uint8_t* sig, const uint8_t* blob,
                 const uint64_t* off, uint64_t n, uint64_t* bm, hipStream_t s, const uint32_t* ktab,
                 const uint32_t* kidx, bool wide, hipEvent_t sha_ev = nullptr) {
  if (lat_keyed(d, ktab, n, wide)) {   // k_verify_quad_keyed runs the whole verify
    if (sha_ev) HIP_OK(hipEventRecord(sha_ev, s));
    return PV_OK;
  }
  if (lat_fused(d, ktab, n)) {
    // k_verify_quad runs the whole verify; only the deferred counter is reset
    HIP_OK(w.qc.ensure(2));
    HIP_OK(hipMemsetAsync(w.qc.p, 0, sizeof(unsigned long long), s));
    if (sha_ev) HIP_OK(hipEventRecord(sha_ev, s));
    return PV_OK;
  }
  HIP_OK(w.h.ensure(n * 16));
  HIP_OK(w.pre.ensure(n));
  HIP_OK(w.counter.ensure(1));
  HIP_OK(w.qc.ensure(2));
  HIP_OK(w.scratch.ensure(d.scratch_words));
  const bool half = !ktab && d.mode != CurveMode::Grouped;
  if (half) {
    if (n > 0xffffffffull) return fail(PV_EINVAL, "at most 2^32-1 signatures per device call");
    HIP_OK(w.hrec.ensure(n * pv::HSREC_WORDS));
    HIP_OK(w.dlist.ensure(n));
  }
  // the half-size path runs the pre-checks in k_lattice (k_hash hashes every
  // signature); keyed and grouped batches in k_precheck before the hash
  HIP_OK(pv::launch_hash(pk, sig, blob, off, n, w.counter.p, w.h.p, half ? nullptr : w.pre.p, d.hash_blocks, s, kidx));
  // live timing: the SHA-512 stage alone (its roofline in bench.py), before the lattice
  if (sha_ev) HIP_OK(hipEventRecord(sha_ev, s));
  if (half)
    HIP_OK(pv::launch_lattice(pk, sig, w.h.p, w.pre.p, n, w.hrec.p, w.dlist.p, w.qc.p, w.qc.p + 1, bm,
                              d.mode == CurveMode::Full, s));
  return PV_OK;
}

int enqueue_curve(Device& d, Workspace& w, const uint8_t* pk, const uint8_t* sig, const uint8_t* blob,
                  const uint64_t* off, uint64_t n, uint8_t* verdict, uint64_t* bm, hipStream_t s, const uint32_t* ktab,
                  const uint32_t* kidx, bool wide) {
  const bool half = !ktab && d.mode != CurveMode::Grouped;
  if (lat_keyed(d, ktab, n, wide)) {
    // small keyed batch: one launch, the comb split over the signature's two
    // lane quads (the hashed key bytes are pk[kidx[i]])
    HIP_OK(pv::launch_verify_quad_keyed(pk, true, sig, blob, off, n, nullptr, ktab, kidx, d.bw.p, verdict, bm, s));
  } else if (lat_fused(d, ktab, n)) {
    // small batch: one launch, 8 lanes per signature (each point on a lane
    // quad) plus one hashing lane per signature in a second wave
    HIP_OK(pv::launch_verify_quad(pk, sig, blob, off, n, d.bw.p, verdict, bm, w.qc.p, d.mode == CurveMode::Full, s));
    w.half_ran = true;
    d.last_ws = (int)(&w - d.ws);
  } else if (half && n <= d.lat_max) {
    // (PV_LAT_PAIR) lane pairs per signature, one table of scratch per lane
    HIP_OK(w.scratch.ensure(std::max<size_t>(d.scratch_words, (size_t)((2 * n + 63) / 64 * 64) * pv::ATAB_LAT_WORDS)));
    HIP_OK(pv::launch_curve_lat(pk, sig, w.h.p, w.hrec.p, d.btab.p, d.bw.p, w.scratch.p,
                                w.scratch.cap / pv::ATAB_LAT_WORDS, verdict, bm, n, s));
    w.half_ran = true;
    d.last_ws = (int)(&w - d.ws);
  } else if (half) {
    HIP_OK(pv::launch_curve_half(pk, sig, w.h.p, w.hrec.p, d.btab.p, d.bw.p, w.scratch.p,
                                 w.scratch.cap / pv::HALF_SCRATCH_WORDS, verdict, bm, n, w.dlist.p, w.qc.p, w.qc.p + 1,
                                 d.curve_half_blocks, s));
    w.half_ran = true;
    d.last_ws = (int)(&w - d.ws);
  } else {
    HIP_OK(pv::launch_curve(pk, sig, w.h.p, w.pre.p, d.btab.p, w.scratch.p, w.scratch.cap / pv::ATAB_WORDS, verdict,
                            bm, n, ktab ? d.curve_blocks_keyed : d.curve_blocks, s, ktab, kidx, d.bw.p, w.qc.p + 1,
                            wide));
  }
  return PV_OK;
}

// enqueue hash + curve for device-resident inputs on stream s with workspace w
int enqueue_verify(Device& d, Workspace& w, const uint8_t* pk, const uint8_t* sig, const uint8_t* blob,
                   const uint64_t* off, uint64_t n, uint8_t* verdict, uint64_t* bitmap, hipStream_t s, bool timed,
                   float* ms_hash, float* ms_curve, const uint32_t* ktab = nullptr, const uint32_t* kidx = nullptr,
                   bool wide = false, hipEvent_t curve_after = nullptr) {
  if (n == 0) return PV_OK;
  const bool live = !timed && d.live_timing;
  hipEvent_t* lev = nullptr;
  if (live) {
    if (d.live_used == d.live_pool.size() && d.live_used >= 256) {
      const int rc = resolve_live(d);
      if (rc) return rc;
    }
    if (d.live_used == d.live_pool.size()) {
      d.live_pool.emplace_back();
      for (auto& e : d.live_pool.back().e) HIP_OK(hipEventCreate(&e));
    }
    lev = d.live_pool[d.live_used++].e;
    ++d.live_launches;
  }
  int rc = ws_begin(w, s);
  if (rc) return rc;
  uint64_t* bm = stage_bitmap(w, bitmap, n, rc);
  if (rc) return rc;
  if (timed) HIP_OK(hipEventRecord(d.ev[0], s));
  if (lev) HIP_OK(hipEventRecord(lev[0], s));
  rc = enqueue_prep(d, w, pk, sig, blob, off, n, bm, s, ktab, kidx, wide, lev ? lev[3] : nullptr);
  if (rc) return rc;
  // the "hash" interval also holds the scalar stage of the half-size path
  if (timed) HIP_OK(hipEventRecord(d.ev[1], s));
  if (lev) HIP_OK(hipEventRecord(lev[1], s));
  // keys prepared on a side stream (pv_verify_keys_device_async): the curve
  // kernel reads their tables
  if (curve_after) HIP_OK(hipStreamWaitEvent(s, curve_after, 0));
  rc = enqueue_curve(d, w, pk, sig, blob, off, n, verdict, bm, s, ktab, kidx, wide);
  if (rc) return rc;
  rc = ws_end(w, s);
  if (rc) return rc;
  if (lev) HIP_OK(hipEventRecord(lev[2], s));
  if (timed) {
    HIP_OK(hipEventRecord(d.ev[2], s));
    HIP_OK(hipEventSynchronize(d.ev[2]));
    float a = 0, b = 0;
    HIP_OK(hipEventElapsedTime(&a, d.ev[0], d.ev[1]));
    HIP_OK(hipEventElapsedTime(&b, d.ev[1], d.ev[2]));
    if (ms_hash) *ms_hash += a;
    if (ms_curve) *ms_curve += b;
  }
  return PV_OK;
}

struct HostBatch {
  const uint8_t* pk;
  const uint8_t* sig;
  const uint8_t* blob;
  const uint64_t* off;
  uint8_t* verdict;
  uint32_t flags;
};

// One device's shard [s, e) of a host-buffer batch (pv_verify_batch), on the
// calling thread: key dedup and buffers, then a pipeline of chunks.  Chunk c's
// inputs are gathered by host threads into page-locked slot c & 1 (its
// offsets rebased to the shard and checked while they are copied), DMA'd on
// the copy stream, and verified on workspace c & 1's stream (see the loop).
// Verdicts come back through a page-locked buffer.  Returns after every verdict of the
// shard is in hb.verdict (or on error, after the device has drained).
// A shard of a Looper-pass size (m <= lat_max: the one-launch latency kernel).
// The inputs are gathered into page-locked slot 0 in the layout off | pk | sig
// | blob | 16 zero bytes, DMA'd with ONE copy into the device image `stage`,
// verified by one k_verify_quad launch and the verdicts copied back, all on
// workspace 0's stream (no copy stream, no cross-stream events).  Keys are
// never deduplicated here: the latency kernel beats preparing them (same
// verdicts).  Returns 1 when the shard does not fit the path (caller falls
// back to the pipeline).
// [p, p + n) lies inside one page-locked host allocation (hipHostMalloc'd or
// registered by the caller, e.g. torch pin_memory()), so the copy engine can
// read it directly and the gather into the staging ring can be skipped
bool host_locked(const void* p, size_t n) {
  if (n == 0) return true;
  if (!p) return false;
  hipPointerAttribute_t a;
  if (hipPointerGetAttributes(&a, p) != hipSuccess) {
    (void)hipGetLastError();
    return false;
  }
  if (a.type != hipMemoryTypeHost) return false;
  void* start = nullptr;
  size_t size = 0;
  hipDeviceptr_t dp = const_cast<void*>(p);
  if (hipPointerGetAttribute(&start, HIP_POINTER_ATTRIBUTE_RANGE_START_ADDR, dp) != hipSuccess ||
      hipPointerGetAttribute(&size, HIP_POINTER_ATTRIBUTE_RANGE_SIZE, dp) != hipSuccess || !start) {
    (void)hipGetLastError();
    return false;
  }
  return static_cast<const char*>(p) >= static_cast<const char*>(start) &&
         static_cast<const char*>(p) + n <= static_cast<const char*>(start) + size;
}

uint64_t small_bytes(const HostBatch& hb, uint64_t s, uint64_t e) {
  const uint64_t m = e - s;
  // + the key-cache tail: 8-byte alignment, list count, kidx and the two lists
  return (m + 1) * 8 + m * 96 + (hb.off[e] - hb.off[s]) + 16 + 16 + 8 * m;
}

// PV_ZC_POLL = 0 builds the stream-synchronize completion (A/B variant)
#ifndef PV_ZC_POLL
#define PV_ZC_POLL 1
#endif
// all-cached zero-copy calls up to this size complete by the keyed kernel's own
// word: 64 signatures = the 16 blocks of 4 that profiles/r05_ab_completion_word.jsonl
// measured faster than a k_signal launch (125 blocks measured slower)
constexpr uint64_t ZC_SELF_MAX = 64;
// spin budget of the completion word before the stream synchronize takes over
// (pv_test_set_spin_ns shortens it so a test reaches the fallback)
std::atomic<int64_t> g_zc_spin_ns{20'000'000};
// spins until *w == v (acquire) or `ns` nanoseconds have passed
bool spin_wait_word(const uint32_t* w, uint32_t v, int64_t ns) {
  const auto t0 = std::chrono::steady_clock::now();
  for (uint32_t i = 0;; ++i) {
    if (__atomic_load_n(w, __ATOMIC_ACQUIRE) == v) return true;
    if ((i & 255u) == 255u &&
        std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - t0).count() > ns)
      return false;
  }
}

int run_small(Device& d, const HostBatch& hb, uint64_t s, uint64_t e) {
  const uint64_t m = e - s;
  HIP_OK(hipSetDevice(d.ord));
  Workspace& w = d.ws[0];
  struct Drain {
    Device& d;
    bool done = false;   // the call's work is known complete (zero-copy completion word)
    ~Drain() {
      if (done) return;
      (void)hipSetDevice(d.ord);
      (void)hipStreamSynchronize(d.ws[0].stream);
    }
  } drain{d};
  const uint64_t b0 = hb.off[s], bytes = hb.off[e] - b0;
  const size_t o_pk = (m + 1) * 8, o_sig = o_pk + m * 32, o_blob = o_sig + m * 64, total = small_bytes(hb, s, e);
  // zero-copy: the kernels read the image from and write the verdicts to
  // fine-grained host memory (no copy launches); else one H2D into `stage`
  // and one D2H of the verdicts
  const bool zc = m <= d.zc_max;
  PinBuf& pin = zc ? d.zc_in : d.pin[0];
  PinBuf& vout = zc ? d.zc_out : d.vout;
  if (pin.ensure(total) != hipSuccess || vout.ensure(m) != hipSuccess) {
    (void)hipGetLastError();
    return 1;
  }
  uint8_t* base = pin.p;
  const uint8_t* g = nullptr;
  uint8_t* vdst = nullptr;
  if (zc) {
    g = pin.dev;
    vdst = vout.dev;
  } else {
    HIP_OK(d.stage.ensure(total));
    HIP_OK(d.verdict.ensure(m));
    g = d.stage.p;
    vdst = d.verdict.p;
  }
  std::atomic<bool> bad{false};
  const CopyJob jobs[4] = {{base, reinterpret_cast<const uint8_t*>(hb.off + s), (m + 1) * 8, b0, true},
                           {base + o_pk, hb.pk + 32 * s, m * 32},
                           {base + o_sig, hb.sig + 64 * s, m * 64},
                           {base + o_blob, hb.blob ? hb.blob + b0 : nullptr, bytes}};
  d.pool->run(jobs, 4, d.copy_threads, &bad);
  if (bad.load())
    return fail(PV_EINVAL, "msg_off not monotone in [%llu, %llu]", (unsigned long long)s, (unsigned long long)e);
  memset(base + o_blob + bytes, 0, 16);   // the hash reads aligned words past the last message
  // keys in the persistent key cache (pv_keycache_add): those signatures run
  // the keyed latency kernel over a list, the others k_verify_quad_list; the
  // image gets a tail of the uncached count, kidx[m] and the two lists (cached
  // indices from the front, uncached from the back)
  const size_t o_ext = (o_blob + bytes + 16 + 7) & ~size_t(7);
  uint64_t nk = 0, ng = 0;
  if (g_kc.count() && d.kc_count == g_kc.count() && d.lat_keyed_max && d.lat_quad) {
    uint32_t* kidx = reinterpret_cast<uint32_t*>(base + o_ext + 8);
    uint32_t* kl = kidx + m;
    for (uint64_t i = 0; i < m; ++i) {
      const uint32_t sl = g_kc.find(hb.pk + 32 * (s + i));
      kidx[i] = sl == UINT32_MAX ? 0u : sl;
      if (sl != UINT32_MAX) kl[nk++] = (uint32_t)i;
      else kl[m - 1 - ng++] = (uint32_t)i;
    }
    *reinterpret_cast<uint64_t*>(base + o_ext) = ng;
  }
  // zero-copy calls complete by a word in fine-grained host memory that the host
  // polls (~5 us below a stream synchronize, tools/ubench/sync_lat.hip): an
  // all-cached call's keyed kernel writes it from its last block, other calls
  // end with a k_signal launch
  const bool poll = zc && PV_ZC_POLL;
  uint32_t seq = 0;
  bool signalled = false;
  if (poll) {
    const bool fresh = d.zc_flag.p == nullptr;
    HIP_OK(d.zc_flag.ensure(64));
    // hipHostMalloc leaves the contents unspecified (recycled pinned pages after a
    // shutdown / init cycle): a stale word equal to the first seq would complete
    // the call before the kernel ran
    if (fresh) {
      __atomic_store_n(reinterpret_cast<uint32_t*>(d.zc_flag.p), 0u, __ATOMIC_RELEASE);
      d.zc_seq = 0;
    }
    if (++d.zc_seq == 0) d.zc_seq = 1;
    seq = d.zc_seq;
  }
  if (nk) {
    const size_t total_ext = o_ext + 8 + 8 * m;
    if (!zc) HIP_OK(hipMemcpyAsync(d.stage.p, base, total_ext, hipMemcpyHostToDevice, w.stream));
    int rc = ws_begin(w, w.stream);
    if (rc) return rc;
    const uint64_t* goff = reinterpret_cast<const uint64_t*>(g);
    const uint32_t* kidx = reinterpret_cast<const uint32_t*>(g + o_ext + 8);
    // up to 16 blocks: measured 2-3 us faster than a k_signal launch; at 125
    // blocks 3-4 us slower (every comb wave's system-scope fence and the
    // counter), profiles/r05_ab_completion_word.jsonl
    const bool self = poll && ng == 0 && nk <= ZC_SELF_MAX;
    if (self && !d.zc_done_armed) {
      HIP_OK(d.zc_done.ensure(1));
      HIP_OK(hipMemsetAsync(d.zc_done.p, 0, sizeof(uint32_t), w.stream));
      d.zc_done_armed = true;
    }
    HIP_OK(pv::launch_verify_quad_keyed(g + o_pk, false, g + o_sig, g + o_blob, goff, nk, kidx + m, d.kc.p, kidx,
                                        d.bw.p, vdst, nullptr, w.stream, self ? d.zc_done.p : nullptr,
                                        self ? reinterpret_cast<uint32_t*>(d.zc_flag.dev) : nullptr, seq));
    signalled = self;
    if (ng)
      HIP_OK(pv::launch_verify_quad_list(g + o_pk, g + o_sig, g + o_blob, goff, kidx + 2 * m - ng,
                                         reinterpret_cast<const unsigned long long*>(g + o_ext), ng, (int)((ng + 7) / 8),
                                         d.bw.p, vdst, d.mode == CurveMode::Full, w.stream));
    rc = ws_end(w, w.stream);
    if (rc) return rc;
  } else {
    if (!zc) HIP_OK(hipMemcpyAsync(d.stage.p, base, total, hipMemcpyHostToDevice, w.stream));
    const int rc = enqueue_verify(d, w, g + o_pk, g + o_sig, g + o_blob, reinterpret_cast<const uint64_t*>(g), m,
                                  vdst, nullptr, w.stream, false, nullptr, nullptr);
    if (rc) return rc;
  }
  if (poll) {
    // past the spin budget (a fault, a long queue) the synchronize reports /
    // waits as before
    if (!signalled) HIP_OK(pv::launch_signal(reinterpret_cast<uint32_t*>(d.zc_flag.dev), seq, w.stream));
    drain.done = spin_wait_word(reinterpret_cast<const uint32_t*>(d.zc_flag.p), seq,
                                 g_zc_spin_ns.load(std::memory_order_relaxed));
    if (!drain.done) HIP_OK(hipStreamSynchronize(w.stream));
  } else {
    if (!zc) HIP_OK(hipMemcpyAsync(vout.p, d.verdict.p, m, hipMemcpyDeviceToHost, w.stream));
    HIP_OK(hipStreamSynchronize(w.stream));
  }
  memcpy(hb.verdict + s, vout.p, m);
  return PV_OK;
}

int run_shard(Device& d, const HostBatch& hb, uint64_t s, uint64_t e) {
  // before any size arithmetic: a shard whose end offset lies below its start
  // would wrap bytes + 16 (the per-chunk checks come later)
  if (hb.off[e] < hb.off[s])
    return fail(PV_EINVAL, "msg_off not monotone in [%llu, %llu]", (unsigned long long)s, (unsigned long long)e);
  const uint64_t m = e - s;
  if (m == 0) return PV_OK;
  if (m <= d.lat_max && d.lat_quad && d.mode != CurveMode::Grouped && d.pinned &&
      small_bytes(hb, s, e) <= d.pin_max) {
    const int rc = run_small(d, hb, s, e);
    if (rc != 1) return rc;
  }
  HIP_OK(hipSetDevice(d.ord));
  // on every exit (errors included) wait for the work that reads host memory
  struct Drain {
    Device& d;
    ~Drain() {
      (void)hipSetDevice(d.ord);
      (void)hipStreamSynchronize(d.copy);
      for (auto& w : d.ws) (void)hipStreamSynchronize(w.stream);
    }
  } drain{d};
  // async batches may still hold either workspace on a caller's stream
  for (auto& w : d.ws) {
    const int rc = ws_begin(w, w.stream);
    if (rc) return rc;
  }
  const uint8_t* pk = hb.pk;
  const uint64_t b0 = hb.off[s], bytes = hb.off[e] - b0;
  // PV_FLAG_DEDUP_KEYS: prepare each distinct key once (cached multiples of
  // -A) when at least half of the shard's signatures repeat a key
  std::vector<uint8_t> upk;
  std::vector<uint32_t> idx;
  uint64_t nk = m;
  if (hb.flags & PV_FLAG_DEDUP_KEYS) {
    // a sample first: s keys (one at a pseudo-random position in each of s
    // equal strides, so positions never repeat) from a pool of <= m/2
    // distinct keys in even use repeat ~s^2/m times; a sample with under a
    // quarter of that means mostly distinct keys, and the full pass is
    // skipped (the choice only affects speed, never verdicts)
    KeyIndex ki;
    bool dedup = true;
    if (m >= PV_DEDUP_SAMPLE_MIN) {
      uint64_t smp = 8;
      while (smp * smp < 64 * m) smp <<= 1;  // s >= 8 sqrt(m): ~64 expected repeats at the threshold
      const uint64_t stride = m / smp;
      ki.reset(pk + 32 * s, m);
      for (uint64_t j = 0; j < smp; ++j) {
        uint64_t x = (j + 1) * 0x9E3779B97F4A7C15ull;
        x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
        x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
        ki.insert(j * stride + (x ^ (x >> 31)) % stride);
      }
      dedup = 4 * (smp - ki.first.size()) * m >= smp * smp;
    }
    if (dedup) {
      ki.reset(pk + 32 * s, m);
      idx.resize(m);
      for (uint64_t k = 0; k < m && 2 * ki.first.size() <= m; ++k) idx[k] = ki.insert(k);
      nk = ki.first.size();
      if (2 * nk > m) {
        nk = m;
        idx.clear();
      } else {
        upk.resize(nk * 32);
        for (uint64_t j = 0; j < nk; ++j) memcpy(upk.data() + 32 * j, pk + 32 * (s + ki.first[j]), 32);
      }
    }
  }
  const bool keyed = !idx.empty();
  HIP_OK(d.pk.ensure((keyed ? nk : m) * 32));
  HIP_OK(d.sig.ensure(m * 64));
  HIP_OK(d.blob.ensure(bytes + 16));
  HIP_OK(d.off.ensure(m + 1));
  HIP_OK(d.verdict.ensure(m));
  // chunk bounds: short leading chunks so the kernels start early -- the
  // ramp r, 2r, ... below a regular chunk (default), or with host_ramp 0
  // one first chunk of first_pct % of a regular one (>= PV_HOST_CHUNK_MIN) --
  // then the rest in equal chunks.  With pinned
  // staging the chunk count doubles until a chunk's inputs fit one
  // pin_max slot; a shard whose PV_HOST_CHUNK_MIN-signature chunks still do not
  // fit (or whose page-locked allocation fails) uses pageable staging.
  auto chunk_bytes = [&](uint64_t c0, uint64_t c1) -> size_t {
    return (c1 - c0 + 1) * 8 + (keyed ? 0 : (c1 - c0) * 32) + (c1 - c0) * 64 + (hb.off[s + c1] - hb.off[s + c0]);
  };
  std::vector<uint64_t> bounds;
  size_t cap = 0;
  for (uint64_t hc = d.host_chunks;; hc *= 2) {
    const uint64_t reg = std::max<uint64_t>(PV_HOST_CHUNK_MIN, (m + hc - 1) / hc);
    const uint64_t first = std::min(m, std::max<uint64_t>(PV_HOST_CHUNK_MIN, reg * (uint64_t)d.first_pct / 100));
    bounds.assign(1, 0);
    if (hc > 1 && d.ramp) {
      // tuning.host_ramp = r: leading chunks of r, 2r, 4r, ... signatures (< a
      // regular chunk), so the first kernels start after a short DMA
      for (uint64_t r = d.ramp; r < reg && bounds.back() + r < m; r *= 2) bounds.push_back(bounds.back() + r);
    } else if (hc > 1 && first < m) {
      bounds.push_back(first);
    }
    const uint64_t rest = m - bounds.back();
    const uint64_t k = std::max<uint64_t>(1, std::min<uint64_t>((rest + reg - 1) / reg, rest / PV_HOST_CHUNK_MIN));
    const uint64_t c0 = bounds.back();
    for (uint64_t j = 1; j <= k; ++j) bounds.push_back(c0 + rest * j / k);
    cap = 0;
    for (size_t j = 1; j < bounds.size(); ++j) cap = std::max(cap, chunk_bytes(bounds[j - 1], bounds[j]));
    if (!d.pinned || cap <= d.pin_max || reg == PV_HOST_CHUNK_MIN || hc >= 4096) break;
  }
  const size_t nch = bounds.size() - 1;
  // chunk sizes come from the offsets at the chunk bounds: check those before
  // anything is sized from them (each chunk's offsets are checked as they are copied)
  for (size_t j = 1; j < bounds.size(); ++j)
    if (hb.off[s + bounds[j]] < hb.off[s + bounds[j - 1]])
      return fail(PV_EINVAL, "msg_off not monotone in [%llu, %llu]", (unsigned long long)(s + bounds[j - 1]),
                  (unsigned long long)(s + bounds[j]));
  bool pinned = d.pinned && cap <= d.pin_max;
  if (pinned && (d.pin[0].ensure(cap) != hipSuccess || d.pin[1].ensure(cap) != hipSuccess ||
                 d.vout.ensure(m) != hipSuccess)) {
    (void)hipGetLastError();
    d.pin[0].release();
    d.pin[1].release();
    d.vout.release();
    pinned = false;
  }
  std::vector<uint64_t> offs;  // pageable staging: the shard's rebased offsets (read by in-flight copies)
  if (!pinned) offs.resize(m + 1);
  // caller buffers already page-locked: DMA pk / sig / blob straight from them,
  // only the offsets (rebased, checked) go through the staging ring
  const bool direct = pinned && !keyed && host_locked(pk + 32 * s, m * 32) && host_locked(hb.sig + 64 * s, m * 64) &&
                      host_locked(hb.blob ? hb.blob + b0 : nullptr, bytes);
  HIP_OK(hipMemsetAsync(d.blob.p + bytes, 0, 16, d.copy));
  // generic batches: one fused launch per chunk, deferred records listed for
  // one lane-quad pass at the end (its count is zeroed on the copy stream,
  // which every chunk's kernels wait for)
  // (PV_CURVE_MODE=full: every record deferred, i.e. verified by the list pass)
  const bool fused = !keyed && d.chunk_fused && d.mode != CurveMode::Grouped;
  if (fused) {
    if (m > 0xffffffffull) return fail(PV_EINVAL, "at most 2^32-1 signatures per device call");
    HIP_OK(d.dl.ensure(m));
    HIP_OK(d.dlc.ensure(1));
    HIP_OK(hipMemsetAsync(d.dlc.p, 0, sizeof(unsigned long long), d.copy));
    for (auto& w : d.ws) w.half_ran = false;   // pv_curve_stats describes device-resident calls
  }
  if (keyed) {
    HIP_OK(d.ktab.ensure(nk * pv::KEYTAB_WORDS));
    HIP_OK(d.kidx.ensure(m));
    HIP_OK(d.kscr.ensure((nk + 63) / 64 * 64 * pv::KEYTAB_SCRATCH));   // lane-interleaved per 64 keys
    HIP_OK(hipMemcpyAsync(d.pk.p, upk.data(), nk * 32, hipMemcpyHostToDevice, d.copy));
    HIP_OK(hipMemcpyAsync(d.kidx.p, idx.data(), m * 4, hipMemcpyHostToDevice, d.copy));
    HIP_OK(hipEventRecord(d.copied, d.copy));
    HIP_OK(hipStreamWaitEvent(d.ws[0].stream, d.copied, 0));
    HIP_OK(pv::launch_keys(d.pk.p, nk, d.ktab.p, d.kscr.p, d.ws[0].stream));
    HIP_OK(hipEventRecord(d.keys_ready, d.ws[0].stream));
    HIP_OK(hipStreamWaitEvent(d.ws[1].stream, d.keys_ready, 0));
  }
  // tuning.host_trace: per-chunk host timings on stderr (pipeline diagnostics)
  const bool trace = g_tune.host_trace != 0;
  const auto tstart = std::chrono::steady_clock::now();
  auto us = [&] { return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - tstart).count(); };
  if (trace) fprintf(stderr, "[pv host] dev %d shard %llu sigs: setup %.1f us, %zu chunks, pinned %d, direct %d\n", d.id,
                     (unsigned long long)m, us(), nch, (int)pinned, (int)direct);
  // chunk c is verified on workspace c & 1 and its stream, so chunk c + 1's
  // kernels start while chunk c's curve grid drains.  (A separate prep stream
  // for every chunk's hash + lattice with three workspaces measured no better:
  // squeezed into the slots the curve grids leave, the prep kernels of a chunk
  // take ~1.1 ms either way -- profiles/r02_e2e_timeline_prepstream_notadopted.txt.)
  for (size_t c = 0; c < nch; ++c) {
    const uint64_t c0 = bounds[c], c1 = bounds[c + 1], mc = c1 - c0;
    Workspace& w = d.ws[c & 1];
    const double t_begin = trace ? us() : 0;
    double t_slot = 0, t_gather = 0;
    const uint64_t cb0 = hb.off[s + c0] - b0, cbytes = hb.off[s + c1] - hb.off[s + c0];
    const uint8_t* src_pk = pk + 32 * (s + c0);
    const uint8_t* src_sig = hb.sig + 64 * (s + c0);
    const uint8_t* src_blob = hb.blob ? hb.blob + b0 + cb0 : nullptr;
    const uint8_t* src_off;
    std::atomic<bool> bad{false};
    if (pinned) {
      // gather the chunk into slot c & 1 once its previous H2D (chunk c - 2) is done
      const int slot = (int)(c & 1);
      if (c >= 2) HIP_OK(hipEventSynchronize(d.staged[slot]));
      if (trace) t_slot = us();
      uint8_t* base = d.pin[slot].p;
      uint8_t *p_off = base, *p_pk = p_off + (mc + 1) * 8, *p_sig = p_pk + (keyed ? 0 : mc * 32),
              *p_blob = p_sig + mc * 64;
      const CopyJob jobs[4] = {{p_off, reinterpret_cast<const uint8_t*>(hb.off + s + c0), (mc + 1) * 8, b0, true},
                               {p_pk, src_pk, keyed ? 0 : mc * 32},
                               {p_sig, src_sig, mc * 64},
                               {p_blob, src_blob, cbytes}};
      d.pool->run(jobs, direct ? 1 : 4, d.copy_threads, &bad);
      if (trace) t_gather = us();
      src_off = p_off;
      if (!direct) {
        src_pk = p_pk;
        src_sig = p_sig;
        src_blob = p_blob;
      }
    } else {
      const CopyJob job{reinterpret_cast<uint8_t*>(offs.data() + c0), reinterpret_cast<const uint8_t*>(hb.off + s + c0),
                        (mc + 1) * 8, b0, true};
      gather_range(&job, 1, 0, job.n, &bad);
      src_off = reinterpret_cast<const uint8_t*>(offs.data() + c0);
    }
    if (bad.load()) return fail(PV_EINVAL, "msg_off not monotone in [%llu, %llu]", (unsigned long long)(s + c0),
                                (unsigned long long)(s + c1));
    if (!keyed) HIP_OK(hipMemcpyAsync(d.pk.p + 32 * c0, src_pk, mc * 32, hipMemcpyHostToDevice, d.copy));
    HIP_OK(hipMemcpyAsync(d.sig.p + 64 * c0, src_sig, mc * 64, hipMemcpyHostToDevice, d.copy));
    if (cbytes) HIP_OK(hipMemcpyAsync(d.blob.p + cb0, src_blob, cbytes, hipMemcpyHostToDevice, d.copy));
    HIP_OK(hipMemcpyAsync(d.off.p + c0, src_off, (mc + 1) * 8, hipMemcpyHostToDevice, d.copy));
    if (pinned) HIP_OK(hipEventRecord(d.staged[c & 1], d.copy));
    HIP_OK(hipEventRecord(d.copied, d.copy));
    HIP_OK(hipStreamWaitEvent(w.stream, d.copied, 0));
    // blob base + shard-relative offsets: the hash kernel reads blob + off[i]
    if (fused) {
      HIP_OK(w.hrec.ensure(mc * pv::HSREC_WORDS));
      HIP_OK(w.qc.ensure(2));
      HIP_OK(w.scratch.ensure(d.scratch_words));
      HIP_OK(pv::launch_chunk_half(d.pk.p + 32 * c0, d.sig.p + 64 * c0, d.blob.p, d.off.p + c0, mc, w.hrec.p, d.bw.p,
                                   w.scratch.p, w.scratch.cap / pv::HALF_SCRATCH_WORDS, d.verdict.p + c0, d.dl.p,
                                   d.dlc.p, c0, w.qc.p + 1, d.curve_half_blocks, d.mode == CurveMode::Full, w.stream));
      if (const int rc = ws_end(w, w.stream)) return rc;
      if (trace)
        fprintf(stderr, "[pv host] chunk %zu (%llu sigs): begin %.1f slot-free %.1f gathered %.1f enqueued %.1f us\n", c,
                (unsigned long long)mc, t_begin, t_slot, t_gather, us());
      continue;
    }
    int rc = enqueue_verify(d, w, keyed ? d.pk.p : d.pk.p + 32 * c0, d.sig.p + 64 * c0, d.blob.p, d.off.p + c0, mc,
                            d.verdict.p + c0, nullptr, w.stream, false, nullptr, nullptr, keyed ? d.ktab.p : nullptr,
                            keyed ? d.kidx.p + c0 : nullptr);
    if (rc) return rc;
    HIP_OK(hipMemcpyAsync(pinned ? d.vout.p + c0 : hb.verdict + s + c0, d.verdict.p + c0, mc, hipMemcpyDeviceToHost,
                          w.stream));
    if (trace)
      fprintf(stderr, "[pv host] chunk %zu (%llu sigs): begin %.1f slot-free %.1f gathered %.1f enqueued %.1f us\n", c,
              (unsigned long long)mc, t_begin, t_slot, t_gather, us());
  }
  if (fused) {
    // the deferred records of every chunk (ws[1]'s chunks joined into ws[0]),
    // then all verdicts in one copy
    Workspace& w0 = d.ws[0];
    HIP_OK(hipEventRecord(d.joined, d.ws[1].stream));
    HIP_OK(hipStreamWaitEvent(w0.stream, d.joined, 0));
    HIP_OK(pv::launch_verify_quad_list(d.pk.p, d.sig.p, d.blob.p, d.off.p, d.dl.p, d.dlc.p, m, d.cu_count * 8, d.bw.p,
                                       d.verdict.p, d.mode == CurveMode::Full, w0.stream));
    HIP_OK(hipMemcpyAsync(pinned ? d.vout.p : hb.verdict + s, d.verdict.p, m, hipMemcpyDeviceToHost, w0.stream));
  }
  HIP_OK(hipStreamSynchronize(d.copy));
  for (auto& w : d.ws) HIP_OK(hipStreamSynchronize(w.stream));
  if (pinned) memcpy(hb.verdict + s, d.vout.p, m);
  if (trace) fprintf(stderr, "[pv host] drained %.1f us\n", us());
  return PV_OK;
}

// prepare keys[0 .. count) (32 bytes each) into key-cache slots [first,
// first + count) of device d, growing its table (existing slots are kept);
// synchronous.  d.kc_count is left to the caller.
int kc_prepare(Device& d, const uint8_t* keys, uint64_t first, uint64_t count) {
  if (count == 0) return PV_OK;
  HIP_OK(hipSetDevice(d.ord));
  const uint64_t need = (first + count) * (uint64_t)pv::KEYTAB_WORDS;
  if (need > d.kc.cap) {
    size_t cap = d.kc.cap ? d.kc.cap : 64 * (size_t)pv::KEYTAB_WORDS;
    while (cap < need) cap *= 2;
    DevBuf<uint32_t> nb;
    HIP_OK(nb.ensure(cap));
    if (first) {
      const hipError_t e = hipMemcpy(nb.p, d.kc.p, first * pv::KEYTAB_WORDS * sizeof(uint32_t), hipMemcpyDeviceToDevice);
      if (e != hipSuccess) {
        nb.release();
        HIP_OK(e);
      }
    }
    d.kc.release();
    d.kc = nb;
  }
  int rc = ws_begin(d.ws[0], d.stream);
  if (rc) return rc;
  HIP_OK(d.kcpk.ensure(32 * count));
  HIP_OK(hipMemcpyAsync(d.kcpk.p, keys, 32 * count, hipMemcpyHostToDevice, d.stream));
  HIP_OK(d.kscr.ensure((count + 63) / 64 * 64 * pv::KEYTAB_SCRATCH));
  HIP_OK(pv::launch_keys(d.kcpk.p, count, d.kc.p + first * pv::KEYTAB_WORDS, d.kscr.p, d.stream));
  rc = ws_end(d.ws[0], d.stream);
  if (rc) return rc;
  HIP_OK(hipStreamSynchronize(d.stream));
  return PV_OK;
}

std::vector<Device*> select_devs(uint32_t mask) {
  std::vector<Device*> v;
  for (auto& d : g_devs)
    if (mask == 0 || (mask >> d.id) & 1u) v.push_back(&d);
  return v;
}

}  // namespace

extern "C" {

// engine devices 0..dup-1 all on HIP device 0 (pv_test_init_dup), else one per HIP device
static int init_devices(uint32_t device_mask, int dup) {
  DeviceGuard dg;
  int count = 0;
  hipError_t e = hipGetDeviceCount(&count);
  if (e != hipSuccess || count <= 0) return fail(PV_ENODEV, "no HIP device available (%s)", hipGetErrorString(e));
  const int n_ids = dup ? dup : count;
  for (int id = 0; id < n_ids && id < 32; ++id) {
    if (device_mask && !((device_mask >> id) & 1u)) continue;
    if (find_dev(id)) continue;
    g_devs.emplace_back();
    g_devs.back().id = id;
    g_devs.back().ord = dup ? 0 : id;
    int rc = init_device(g_devs.back());
    if (rc == PV_OK && g_kc.count()) {   // a device added after keys were cached gets them too
      rc = kc_prepare(g_devs.back(), g_kc.keys.data(), 0, g_kc.count());
      if (rc == PV_OK) g_devs.back().kc_count = g_kc.count();
    }
    if (rc != PV_OK) {
      release_device(g_devs.back());
      g_devs.pop_back();
      return rc;
    }
  }
  if (g_devs.empty()) return fail(PV_ENODEV, "device_mask 0x%x selects no visible device", device_mask);
  return PV_OK;
}

int pv_init(uint32_t device_mask) {
  std::lock_guard<std::mutex> lk(g_mu);
  return init_devices(device_mask, g_dup);
}

int pv_test_init_dup(uint32_t k) {
  std::lock_guard<std::mutex> lk(g_mu);
  if (k < 2 || k > 8) return fail(PV_EINVAL, "pv_test_init_dup: k must be in 2..8 (got %u)", k);
  if (!g_devs.empty()) return fail(PV_EINVAL, "pv_test_init_dup: devices already initialised (call pv_shutdown first)");
  g_dup = (int)k;
  const int rc = init_devices(0, g_dup);
  if (rc != PV_OK) g_dup = 0;
  return rc;
}

int pv_test_set_spin_ns(int64_t ns) {
  if (ns < 0) return fail(PV_EINVAL, "pv_test_set_spin_ns: ns must be >= 0 (got %lld)", (long long)ns);
  g_zc_spin_ns.store(ns, std::memory_order_relaxed);
  return PV_OK;
}

void pv_shutdown(void) {
  std::lock_guard<std::mutex> lk(g_mu);
  DeviceGuard dg;
  for (auto& d : g_devs) release_device(d);
  g_devs.clear();
  g_kc.clear();
  g_dup = 0;
}

int pv_keycache_add(const uint8_t* pk, uint64_t k) {
  std::lock_guard<std::mutex> lk(g_mu);
  DeviceGuard dg;
  if (g_devs.empty()) return fail(PV_ENOTINIT, "pv_init has not been called");
  if (k == 0) return PV_OK;
  if (!pk) return fail(PV_EINVAL, "null buffer");
  if (g_kc.count() + k > 0xfffffffeull) return fail(PV_EINVAL, "key cache limited to 2^32 - 2 keys");
  // keys not cached yet, first occurrence only
  std::vector<uint8_t> add;
  {
    KeyIndex seen;
    seen.reset(pk, k);
    for (uint64_t i = 0; i < k; ++i) {
      const size_t before = seen.first.size();
      (void)seen.insert(i);
      if (seen.first.size() != before && g_kc.find(pk + 32 * i) == UINT32_MAX)
        add.insert(add.end(), pk + 32 * i, pk + 32 * i + 32);
    }
  }
  if (add.empty()) return PV_OK;
  const uint64_t first = g_kc.count(), cnt = add.size() / 32;
  for (auto& d : g_devs) {
    const int rc = kc_prepare(d, add.data(), first, cnt);
    if (rc) return rc;   // committed nowhere: every device keeps its previous slots
  }
  g_kc.commit(add);
  for (auto& d : g_devs) d.kc_count = g_kc.count();
  return PV_OK;
}

int pv_keycache_clear(void) {
  std::lock_guard<std::mutex> lk(g_mu);
  DeviceGuard dg;
  g_kc.clear();
  for (auto& d : g_devs) {
    (void)hipSetDevice(d.ord);
    (void)hipStreamSynchronize(d.stream);
    d.kc.release();
    d.kc_count = 0;
  }
  return PV_OK;
}

int pv_keycache_size(uint64_t* count) {
  std::lock_guard<std::mutex> lk(g_mu);
  if (!count) return fail(PV_EINVAL, "null buffer");
  *count = g_kc.count();
  return PV_OK;
}

const char* pv_last_error(void) { return g_err.c_str(); }

int pv_device_count(void) {
  std::lock_guard<std::mutex> lk(g_mu);
  DeviceGuard dg;
  return (int)g_devs.size();
}

int pv_verify_batch(const uint8_t* pk, const uint8_t* sig, const uint8_t* msg_blob, const uint64_t* msg_off,
                    uint64_t n, uint8_t* verdict, uint32_t device_mask, uint32_t flags) {
  if (flags & ~PV_FLAG_DEDUP_KEYS) return fail(PV_EINVAL, "unknown flags 0x%x", flags);
  std::lock_guard<std::mutex> lk(g_mu);
  DeviceGuard dg;
  if (g_devs.empty()) return fail(PV_ENOTINIT, "pv_init has not been called");
  if (n == 0) return PV_OK;
  if (!pk || !sig || !msg_off || !verdict || (!msg_blob && msg_off[n] != msg_off[0]))
    return fail(PV_EINVAL, "null buffer");
  if (msg_off[n] < msg_off[0]) return fail(PV_EINVAL, "msg_off not monotone");
  std::vector<Device*> devs = select_devs(device_mask);
  if (devs.empty()) return fail(PV_ENODEV, "device_mask 0x%x selects no initialised device", device_mask);
  const HostBatch hb{pk, sig, msg_blob, msg_off, verdict, flags};
  const uint64_t G = devs.size();
  if (G == 1) return run_shard(*devs[0], hb, 0, n);
  // O(G) pre-check of the shard boundaries (each shard also checks its own
  // range first, and every chunk its offsets while they are copied)
  for (uint64_t g = 0; g < G; ++g)
    if (msg_off[n * (g + 1) / G] < msg_off[n * g / G])
      return fail(PV_EINVAL, "msg_off not monotone in shard %llu [%llu, %llu]", (unsigned long long)g,
                  (unsigned long long)(n * g / G), (unsigned long long)(n * (g + 1) / G));
  // one worker thread per device: each gathers, stages and launches its own
  // shard, so no device waits on another's host gathers (errors come back as
  // codes + messages; no exception crosses the ABI)
  std::vector<int> rc(G, PV_OK);
  std::vector<std::string> err(G);
  std::vector<std::thread> ts;
  auto work = [&](uint64_t g) {
    rc[g] = run_shard(*devs[g], hb, n * g / G, n * (g + 1) / G);
    if (rc[g]) err[g] = g_err;
  };
  std::vector<uint64_t> inline_g;
  try {
    ts.reserve(G);
  } catch (...) {
  }
  for (uint64_t g = 1; g < G; ++g) {
    try {
      ts.emplace_back(work, g);
    } catch (...) {
      inline_g.push_back(g);
    }
  }
  work(0);
  for (uint64_t g : inline_g) work(g);
  for (auto& t : ts) t.join();
  for (uint64_t g = 0; g < G; ++g)
    if (rc[g]) return fail(rc[g], "device %d: %s", devs[g]->id, err[g].c_str());
  return PV_OK;
}

int pv_verify_batch_device(const uint8_t* pk, const uint8_t* sig, const uint8_t* msg_blob, const uint64_t* msg_off,
                           uint64_t n, uint8_t* verdict, uint64_t* bitmap, int device, void* stream) {
  std::lock_guard<std::mutex> lk(g_mu);
  DeviceGuard dg;
  Device* d = find_dev(device);
  if (!d) return fail(PV_ENOTINIT, "device %d not initialised (call pv_init)", device);
  if (n == 0) return PV_OK;
  if (!pk || !sig || !msg_blob || !msg_off || !verdict) return fail(PV_EINVAL, "null device buffer");
  HIP_OK(hipSetDevice(d->ord));
  hipStream_t s = stream ? reinterpret_cast<hipStream_t>(stream) : d->stream;
  int rc = enqueue_verify(*d, d->ws[0], pk, sig, msg_blob, msg_off, n, verdict, bitmap, s, false, nullptr, nullptr);
  if (rc) return rc;
  HIP_OK(hipStreamSynchronize(s));
  return PV_OK;
}

int pv_verify_batch_device_async(const uint8_t* pk, const uint8_t* sig, const uint8_t* msg_blob,
                                 const uint64_t* msg_off, uint64_t n, uint8_t* verdict, uint64_t* bitmap, int device,
                                 void* stream, int slot) {
  std::lock_guard<std::mutex> lk(g_mu);
  DeviceGuard dg;
  Device* d = find_dev(device);
  if (!d) return fail(PV_ENOTINIT, "device %d not initialised (call pv_init)", device);
  if (slot < 0 || slot > 1) return fail(PV_EINVAL, "slot must be 0 or 1");
  if (n == 0) return PV_OK;
  if (!pk || !sig || !msg_blob || !msg_off || !verdict || !bitmap) return fail(PV_EINVAL, "null device buffer");
  HIP_OK(hipSetDevice(d->ord));
  hipStream_t s = stream ? reinterpret_cast<hipStream_t>(stream) : d->ws[slot].stream;
  return enqueue_verify(*d, d->ws[slot], pk, sig, msg_blob, msg_off, n, verdict, bitmap, s, false, nullptr, nullptr);
}

int pv_verify_keyed_device_async(const uint32_t* ktab, const uint32_t* key_idx, const uint8_t* pk, const uint8_t* sig,
                                 const uint8_t* msg_blob, const uint64_t* msg_off, uint64_t n, uint8_t* verdict,
                                 uint64_t* bitmap, int device, void* stream, int slot) {
  std::lock_guard<std::mutex> lk(g_mu);
  DeviceGuard dg;
  Device* d = find_dev(device);
  if (!d) return fail(PV_ENOTINIT, "device %d not initialised (call pv_init)", device);
  if (slot < 0 || slot > 1) return fail(PV_EINVAL, "slot must be 0 or 1");
  if (n == 0) return PV_OK;
  if (!ktab || !key_idx || !pk || !sig || !msg_blob || !msg_off || !verdict || !bitmap)
    return fail(PV_EINVAL, "null device buffer");
  HIP_OK(hipSetDevice(d->ord));
  hipStream_t s = stream ? reinterpret_cast<hipStream_t>(stream) : d->ws[slot].stream;
  return enqueue_verify(*d, d->ws[slot], pk, sig, msg_blob, msg_off, n, verdict, bitmap, s, false, nullptr, nullptr,
                        ktab, key_idx);
}

int pv_keys_prepare_device_async(const uint8_t* pk, uint64_t k, uint32_t* ktab, int device, void* stream, int slot) {
  std::lock_guard<std::mutex> lk(g_mu);
  DeviceGuard dg;
  Device* d = find_dev(device);
  if (!d) return fail(PV_ENOTINIT, "device %d not initialised (call pv_init)", device);
  if (slot < 0 || slot > 1) return fail(PV_EINVAL, "slot must be 0 or 1");
  if (k == 0) return PV_OK;
  if (!pk || !ktab) return fail(PV_EINVAL, "null device buffer");
  HIP_OK(hipSetDevice(d->ord));
  hipStream_t s = stream ? reinterpret_cast<hipStream_t>(stream) : d->ws[slot].stream;
  // the key scratch of slot i is ordered like workspace i (the host pipeline
  // prepares keys in kscr on ws[0]'s stream)
  int rc = ws_begin(d->ws[slot], s);
  if (rc) return rc;
  DevBuf<uint32_t>& scr = slot ? d->kscr2 : d->kscr;
  HIP_OK(scr.ensure((k + 63) / 64 * 64 * pv::KEYTAB_SCRATCH));
  HIP_OK(pv::launch_keys(pk, k, ktab, scr.p, s));
  return ws_end(d->ws[slot], s);
}

int pv_keys_prepare_device(const uint8_t* pk, uint64_t k, uint32_t* ktab, int device, void* stream) {
  std::lock_guard<std::mutex> lk(g_mu);
  DeviceGuard dg;
  Device* d = find_dev(device);
  if (!d) return fail(PV_ENOTINIT, "device %d not initialised (call pv_init)", device);
  if (k == 0) return PV_OK;
  if (!pk || !ktab) return fail(PV_EINVAL, "null device buffer");
  HIP_OK(hipSetDevice(d->ord));
  hipStream_t s = stream ? reinterpret_cast<hipStream_t>(stream) : d->stream;
  int rc = ws_begin(d->ws[0], s);
  if (rc) return rc;
  HIP_OK(d->kscr.ensure((k + 63) / 64 * 64 * pv::KEYTAB_SCRATCH));
  HIP_OK(pv::launch_keys(pk, k, ktab, d->kscr.p, s));
  rc = ws_end(d->ws[0], s);
  if (rc) return rc;
  HIP_OK(hipStreamSynchronize(s));
  return PV_OK;
}

int pv_verify_keyed_device(const uint32_t* ktab, const uint32_t* key_idx, const uint8_t* pk, const uint8_t* sig,
                           const uint8_t* msg_blob, const uint64_t* msg_off, uint64_t n, uint8_t* verdict,
                           uint64_t* bitmap, int device, void* stream) {
  std::lock_guard<std::mutex> lk(g_mu);
  DeviceGuard dg;
  Device* d = find_dev(device);
  if (!d) return fail(PV_ENOTINIT, "device %d not initialised (call pv_init)", device);
  if (n == 0) return PV_OK;
  if (!ktab || !key_idx || !pk || !sig || !msg_blob || !msg_off || !verdict) return fail(PV_EINVAL, "null device buffer");
  HIP_OK(hipSetDevice(d->ord));
  hipStream_t s = stream ? reinterpret_cast<hipStream_t>(stream) : d->stream;
  int rc = enqueue_verify(*d, d->ws[0], pk, sig, msg_blob, msg_off, n, verdict, bitmap, s, false, nullptr, nullptr, ktab,
                          key_idx);
  if (rc) return rc;
  HIP_OK(hipStreamSynchronize(s));
  return PV_OK;
}

// wide key format (radix-256 comb): preparation on KEYTAB_WIDE_LANES (128) lanes
// per key into kscr / kscr2 (the slot's key scratch, 160 KB per key), verification
// through k_curve<true, 1>
static int keys_prepare_wide(Device& d, const uint8_t* pk, uint64_t k, uint32_t* ktab, hipStream_t s, int slot) {
  int rc = ws_begin(d.ws[slot], s);
  if (rc) return rc;
  DevBuf<uint32_t>& scr = slot ? d.kscr2 : d.kscr;
  HIP_OK(scr.ensure(k * pv::KEYTAB_WIDE_LANES * (uint64_t)pv::KEYTAB_WIDE_SCRATCH));
  HIP_OK(pv::launch_keys_wide(pk, k, ktab, scr.p, s));
  return ws_end(d.ws[slot], s);
}

int pv_keys_prepare_wide_device(const uint8_t* pk, uint64_t k, uint32_t* ktab, int device, void* stream) {
  std::lock_guard<std::mutex> lk(g_mu);
  DeviceGuard dg;
  Device* d = find_dev(device);
  if (!d) return fail(PV_ENOTINIT, "device %d not initialised (call pv_init)", device);
  if (k == 0) return PV_OK;
  if (!pk || !ktab) return fail(PV_EINVAL, "null device buffer");
  HIP_OK(hipSetDevice(d->ord));
  hipStream_t s = stream ? reinterpret_cast<hipStream_t>(stream) : d->stream;
  const int rc = keys_prepare_wide(*d, pk, k, ktab, s, 0);
  if (rc) return rc;
  HIP_OK(hipStreamSynchronize(s));
  return PV_OK;
}

int pv_keys_prepare_wide_device_async(const uint8_t* pk, uint64_t k, uint32_t* ktab, int device, void* stream,
                                      int slot) {
  std::lock_guard<std::mutex> lk(g_mu);
  DeviceGuard dg;
  Device* d = find_dev(device);
  if (!d) return fail(PV_ENOTINIT, "device %d not initialised (call pv_init)", device);
  if (slot < 0 || slot > 1) return fail(PV_EINVAL, "slot must be 0 or 1");
  if (k == 0) return PV_OK;
  if (!pk || !ktab) return fail(PV_EINVAL, "null device buffer");
  HIP_OK(hipSetDevice(d->ord));
  hipStream_t s = stream ? reinterpret_cast<hipStream_t>(stream) : d->ws[slot].stream;
  return keys_prepare_wide(*d, pk, k, ktab, s, slot);
}

int pv_verify_keyed_wide_device(const uint32_t* ktab, const uint32_t* key_idx, const uint8_t* pk, const uint8_t* sig,
                                const uint8_t* msg_blob, const uint64_t* msg_off, uint64_t n, uint8_t* verdict,
                                uint64_t* bitmap, int device, void* stream) {
  std::lock_guard<std::mutex> lk(g_mu);
  DeviceGuard dg;
  Device* d = find_dev(device);
  if (!d) return fail(PV_ENOTINIT, "device %d not initialised (call pv_init)", device);
  if (n == 0) return PV_OK;
  if (!ktab || !key_idx || !pk || !sig || !msg_blob || !msg_off || !verdict) return fail(PV_EINVAL, "null device buffer");
  HIP_OK(hipSetDevice(d->ord));
  hipStream_t s = stream ? reinterpret_cast<hipStream_t>(stream) : d->stream;
  int rc = enqueue_verify(*d, d->ws[0], pk, sig, msg_blob, msg_off, n, verdict, bitmap, s, false, nullptr, nullptr, ktab,
                          key_idx, true);
  if (rc) return rc;
  HIP_OK(hipStreamSynchronize(s));
  return PV_OK;
}

int pv_verify_keyed_wide_device_async(const uint32_t* ktab, const uint32_t* key_idx, const uint8_t* pk,
                                      const uint8_t* sig, const uint8_t* msg_blob, const uint64_t* msg_off, uint64_t n,
                                      uint8_t* verdict, uint64_t* bitmap, int device, void* stream, int slot) {
  std::lock_guard<std::mutex> lk(g_mu);
  DeviceGuard dg;
  Device* d = find_dev(device);
  if (!d) return fail(PV_ENOTINIT, "device %d not initialised (call pv_init)", device);
  if (slot < 0 || slot > 1) return fail(PV_EINVAL, "slot must be 0 or 1");
  if (n == 0) return PV_OK;
  if (!ktab || !key_idx || !pk || !sig || !msg_blob || !msg_off || !verdict || !bitmap)
    return fail(PV_EINVAL, "null device buffer");
  HIP_OK(hipSetDevice(d->ord));
  hipStream_t s = stream ? reinterpret_cast<hipStream_t>(stream) : d->ws[slot].stream;
  return enqueue_verify(*d, d->ws[slot], pk, sig, msg_blob, msg_off, n, verdict, bitmap, s, false, nullptr, nullptr,
                        ktab, key_idx, true);
}

// key preparation beside the hash stage: the keys are built on the slot's side
// stream while k_hash runs on `s`; the keyed curve waits for both
int pv_verify_keys_device_async(const uint8_t* pk, uint64_t k, uint32_t* ktab, const uint32_t* key_idx,
                                const uint8_t* sig, const uint8_t* msg_blob, const uint64_t* msg_off, uint64_t n,
                                uint8_t* verdict, uint64_t* bitmap, uint32_t wide, int device, void* stream, int slot) {
  std::lock_guard<std::mutex> lk(g_mu);
  DeviceGuard dg;
  Device* d = find_dev(device);
  if (!d) return fail(PV_ENOTINIT, "device %d not initialised (call pv_init)", device);
  if (slot < 0 || slot > 1) return fail(PV_EINVAL, "slot must be 0 or 1");
  if (wide > 1) return fail(PV_EINVAL, "wide must be 0 or 1");
  if (k == 0 && n == 0) return PV_OK;
  if (n > 0 && k == 0) return fail(PV_EINVAL, "signatures without keys");
  if (!pk || !ktab || (n > 0 && (!key_idx || !sig || !msg_blob || !msg_off || !verdict || !bitmap)))
    return fail(PV_EINVAL, "null device buffer");
  HIP_OK(hipSetDevice(d->ord));
  hipStream_t s = stream ? reinterpret_cast<hipStream_t>(stream) : d->ws[slot].stream;
  Workspace& w = d->ws[slot];
  // the slot's key table and key scratch were last used by its previous batch:
  // fork after that (ws_begin orders s), join before the curve
  int rc = ws_begin(w, s);
  if (rc) return rc;
  // beside the hash stage only when the key grid is small (less than one wave
  // per SIMD: C3's 25 wide node keys, a latency-bound 50-wave grid): a key
  // grid that fills the GPU (C4's 2^20 keys) competes with k_hash for the
  // same issue slots and ran 1.3 % slower beside it
  // (profiles/r06_ab_keys_beside.jsonl), so it stays in line on `s`
  const uint64_t lanes = wide ? k * (uint64_t)pv::KEYTAB_WIDE_LANES : k;
  const bool side = lanes <= 64ull * 4 * (uint64_t)d->cu_count;
  hipStream_t ks = side ? d->kside[slot] : s;
  if (side) {
    HIP_OK(hipEventRecord(d->kfork[slot], s));
    HIP_OK(hipStreamWaitEvent(ks, d->kfork[slot], 0));
  }
  DevBuf<uint32_t>& scr = slot ? d->kscr2 : d->kscr;
  if (wide) {
    HIP_OK(scr.ensure(k * pv::KEYTAB_WIDE_LANES * (uint64_t)pv::KEYTAB_WIDE_SCRATCH));
    HIP_OK(pv::launch_keys_wide(pk, k, ktab, scr.p, ks));
  } else {
    HIP_OK(scr.ensure((k + 63) / 64 * 64 * pv::KEYTAB_SCRATCH));
    HIP_OK(pv::launch_keys(pk, k, ktab, scr.p, ks));
  }
  if (side) HIP_OK(hipEventRecord(d->kjoin[slot], ks));
  if (n == 0) {
    if (side) HIP_OK(hipStreamWaitEvent(s, d->kjoin[slot], 0));
    return ws_end(w, s);
  }
  return enqueue_verify(*d, w, pk, sig, msg_blob, msg_off, n, verdict, bitmap, s, false, nullptr, nullptr, ktab, key_idx,
                        wide != 0, side ? d->kjoin[slot] : nullptr);
}

int pv_time_verify_keyed_device(const uint32_t* ktab, const uint32_t* key_idx, const uint8_t* pk, const uint8_t* sig,
                                const uint8_t* msg_blob, const uint64_t* msg_off, uint64_t n, uint8_t* verdict,
                                uint64_t* bitmap, int device, void* stream, int iters, float* ms_hash,
                                float* ms_curve) {
  std::lock_guard<std::mutex> lk(g_mu);
  DeviceGuard dg;
  Device* d = find_dev(device);
  if (!d) return fail(PV_ENOTINIT, "device %d not initialised (call pv_init)", device);
  if (iters <= 0) return fail(PV_EINVAL, "iters must be > 0");
  HIP_OK(hipSetDevice(d->ord));
  hipStream_t s = stream ? reinterpret_cast<hipStream_t>(stream) : d->stream;
  float a = 0, b = 0;
  for (int it = 0; it < iters; ++it) {
    int rc = enqueue_verify(*d, d->ws[0], pk, sig, msg_blob, msg_off, n, verdict, bitmap, s, true, &a, &b, ktab, key_idx);
    if (rc) return rc;
  }
  if (ms_hash) *ms_hash = a / iters;
  if (ms_curve) *ms_curve = b / iters;
  return PV_OK;
}

int pv_time_verify_device(const uint8_t* pk, const uint8_t* sig, const uint8_t* msg_blob, const uint64_t* msg_off,
                          uint64_t n, uint8_t* verdict, uint64_t* bitmap, int device, void* stream, int iters,
                          float* ms_hash, float* ms_curve) {
  std::lock_guard<std::mutex> lk(g_mu);
  DeviceGuard dg;
  Device* d = find_dev(device);
  if (!d) return fail(PV_ENOTINIT, "device %d not initialised (call pv_init)", device);
  if (iters <= 0) return fail(PV_EINVAL, "iters must be > 0");
  HIP_OK(hipSetDevice(d->ord));
  hipStream_t s = stream ? reinterpret_cast<hipStream_t>(stream) : d->stream;
  float a = 0, b = 0;
  for (int it = 0; it < iters; ++it) {
    int rc = enqueue_verify(*d, d->ws[0], pk, sig, msg_blob, msg_off, n, verdict, bitmap, s, true, &a, &b);
    if (rc) return rc;
  }
  if (ms_hash) *ms_hash = a / iters;
  if (ms_curve) *ms_curve = b / iters;
  return PV_OK;
}

int pv_kernel_timing(int device, int enable, float* hash_ms, float* curve_ms, uint64_t* launches) {
  std::lock_guard<std::mutex> lk(g_mu);
  Device* d = find_dev(device);
  if (!d) return fail(PV_ENOTINIT, "device %d not initialised (call pv_init)", device);
  DeviceGuard dg;
  HIP_OK(hipSetDevice(d->ord));
  {
    const int rc = resolve_live(*d);
    if (rc) return rc;
  }
  if (enable) {
    d->live_hash = d->live_curve = d->live_sha = 0;
    d->live_launches = 0;
  }
  if (hash_ms) *hash_ms = d->live_hash;
  if (curve_ms) *curve_ms = d->live_curve;
  if (launches) *launches = d->live_launches;
  d->live_timing = enable != 0;
  return PV_OK;
}

int pv_kernel_timing_sha(int device, float* sha_ms) {
  std::lock_guard<std::mutex> lk(g_mu);
  Device* d = find_dev(device);
  if (!d) return fail(PV_ENOTINIT, "device %d not initialised (call pv_init)", device);
  DeviceGuard dg;
  HIP_OK(hipSetDevice(d->ord));
  const int rc = resolve_live(*d);
  if (rc) return rc;
  if (sha_ms) *sha_ms = d->live_sha;
  return PV_OK;
}

int pv_get_tuning(pv_tuning* t) {
  std::lock_guard<std::mutex> lk(g_mu);
  if (!t) return fail(PV_EINVAL, "null pointer");
  if (t->struct_size != sizeof(pv_tuning))
    return fail(PV_EINVAL, "struct_size %u != sizeof(pv_tuning) %zu", t->struct_size, sizeof(pv_tuning));
  *t = g_tune;
  return PV_OK;
}

int pv_set_tuning(const pv_tuning* t) {
  std::lock_guard<std::mutex> lk(g_mu);
  if (!t) return fail(PV_EINVAL, "null pointer");
  if (int rc = check_tuning(*t)) return rc;
  g_tune = *t;
  pvbls::set_quad_max(g_tune.bls_quad_max);
  pvbls::set_oct_max(g_tune.bls_oct_max);
  DeviceGuard dg;
  for (auto& d : g_devs) apply_tuning(d, g_tune);
  return PV_OK;
}

int pv_curve_stats(int device, uint32_t* mode, uint64_t* deferred) {
  std::lock_guard<std::mutex> lk(g_mu);
  DeviceGuard dg;
  Device* d = find_dev(device);
  if (!d) return fail(PV_ENOTINIT, "device %d not initialised (call pv_init)", device);
  if (mode) *mode = d->mode == CurveMode::Half ? PV_CURVE_HALF : d->mode == CurveMode::Full ? PV_CURVE_FULL
                                                                                             : PV_CURVE_GROUPED;
  if (deferred) {
    *deferred = 0;
    Workspace& w = d->ws[d->last_ws];
    if (w.half_ran) {
      HIP_OK(hipSetDevice(d->ord));
      HIP_OK(w.done_on ? hipEventSynchronize(w.done) : hipStreamSynchronize(w.stream));
      HIP_OK(hipMemcpy(deferred, w.qc.p, sizeof(uint64_t), hipMemcpyDeviceToHost));
    }
  }
  return PV_OK;
}

int pv_tally_votes_device(const uint8_t* verdict, const uint32_t* sender, const uint64_t* batch_off,
                          uint64_t n_batches, uint32_t n_nodes, uint32_t quorum, uint32_t* votes, uint8_t* reached,
                          int device, void* stream) {
  std::lock_guard<std::mutex> lk(g_mu);
  DeviceGuard dg;
  Device* d = find_dev(device);
  if (!d) return fail(PV_ENOTINIT, "device %d not initialised (call pv_init)", device);
  if (n_nodes == 0 || n_nodes > 1024) return fail(PV_EINVAL, "n_nodes must be in 1..1024");
  if (n_batches == 0) return PV_OK;
  if (!verdict || !sender || !batch_off || !votes || !reached) return fail(PV_EINVAL, "null device buffer");
  HIP_OK(hipSetDevice(d->ord));
  hipStream_t s = stream ? reinterpret_cast<hipStream_t>(stream) : d->stream;
  HIP_OK(d->tflag.ensure(1));
  HIP_OK(hipMemsetAsync(d->tflag.p, 0, 4, s));
  HIP_OK(pv::launch_tally(verdict, sender, batch_off, n_batches, n_nodes, quorum, votes, reached, d->tflag.p, s));
  uint32_t bad = 0;
  HIP_OK(hipMemcpyAsync(&bad, d->tflag.p, 4, hipMemcpyDeviceToHost, s));
  HIP_OK(hipStreamSynchronize(s));
  if (bad) return fail(PV_EINVAL, "a sender index is >= n_nodes (%u)", n_nodes);
  return PV_OK;
}

int pv_tally_votes_device_async(const uint8_t* verdict, const uint32_t* sender, const uint64_t* batch_off,
                                uint64_t n_batches, uint32_t n_nodes, uint32_t quorum, uint32_t* votes,
                                uint8_t* reached, uint32_t* bad, int device, void* stream) {
  std::lock_guard<std::mutex> lk(g_mu);
  DeviceGuard dg;
  Device* d = find_dev(device);
  if (!d) return fail(PV_ENOTINIT, "device %d not initialised (call pv_init)", device);
  if (n_nodes == 0 || n_nodes > 1024) return fail(PV_EINVAL, "n_nodes must be in 1..1024");
  if (!bad) return fail(PV_EINVAL, "null device buffer");
  if (n_batches == 0) return PV_OK;
  if (!verdict || !sender || !batch_off || !votes || !reached) return fail(PV_EINVAL, "null device buffer");
  HIP_OK(hipSetDevice(d->ord));
  hipStream_t s = stream ? reinterpret_cast<hipStream_t>(stream) : d->stream;
  HIP_OK(pv::launch_tally(verdict, sender, batch_off, n_batches, n_nodes, quorum, votes, reached, bad, s));
  return PV_OK;
}

int pv_tally_votes(const uint8_t* verdict, const uint32_t* sender, const uint64_t* batch_off, uint64_t n_batches,
                   uint32_t n_nodes, uint32_t quorum, uint32_t* votes, uint8_t* reached) {
  std::lock_guard<std::mutex> lk(g_mu);
  DeviceGuard dg;
  if (g_devs.empty()) return fail(PV_ENOTINIT, "pv_init has not been called");
  if (n_nodes == 0 || n_nodes > 1024) return fail(PV_EINVAL, "n_nodes must be in 1..1024");
  if (n_batches == 0) return PV_OK;
  if (!verdict || !sender || !batch_off || !votes || !reached) return fail(PV_EINVAL, "null buffer");
  Device& d = g_devs[0];
  HIP_OK(hipSetDevice(d.ord));
  const uint64_t b0 = batch_off[0], m = batch_off[n_batches] - b0;
  std::vector<uint64_t> offs(n_batches + 1);
  for (uint64_t k = 0; k <= n_batches; ++k) {
    if (k && batch_off[k] < batch_off[k - 1]) return fail(PV_EINVAL, "batch_off not monotone");
    offs[k] = batch_off[k] - b0;
  }
  for (uint64_t k = 0; k < m; ++k)
    if (sender[b0 + k] >= n_nodes)
      return fail(PV_EINVAL, "sender[%llu] = %u is >= n_nodes (%u)", (unsigned long long)(b0 + k), sender[b0 + k],
                  n_nodes);
  HIP_OK(d.verdict.ensure(m ? m : 1));
  HIP_OK(d.sender.ensure(m ? m : 1));
  HIP_OK(d.batch_off.ensure(n_batches + 1));
  HIP_OK(d.votes.ensure(n_batches));
  HIP_OK(d.reached.ensure(n_batches));
  HIP_OK(d.tflag.ensure(1));
  if (m) {
    HIP_OK(hipMemcpyAsync(d.verdict.p, verdict + b0, m, hipMemcpyHostToDevice, d.stream));
    HIP_OK(hipMemcpyAsync(d.sender.p, sender + b0, m * 4, hipMemcpyHostToDevice, d.stream));
  }
  HIP_OK(hipMemcpyAsync(d.batch_off.p, offs.data(), (n_batches + 1) * 8, hipMemcpyHostToDevice, d.stream));
  HIP_OK(pv::launch_tally(d.verdict.p, d.sender.p, d.batch_off.p, n_batches, n_nodes, quorum, d.votes.p, d.reached.p,
                          d.tflag.p, d.stream));
  HIP_OK(hipMemcpyAsync(votes, d.votes.p, n_batches * 4, hipMemcpyDeviceToHost, d.stream));
  HIP_OK(hipMemcpyAsync(reached, d.reached.p, n_batches, hipMemcpyDeviceToHost, d.stream));
  HIP_OK(hipStreamSynchronize(d.stream));
  return PV_OK;
}

int pv_tally_device(const uint32_t* verdict_bits, const uint32_t* dup_mask, uint64_t n_batches, uint32_t n_nodes,
                    uint32_t quorum, uint8_t* reached, uint32_t* votes, int device, void* stream) {
  std::lock_guard<std::mutex> lk(g_mu);
  DeviceGuard dg;
  Device* d = find_dev(device);
  if (!d) return fail(PV_ENOTINIT, "device %d not initialised (call pv_init)", device);
  if (n_nodes == 0) return fail(PV_EINVAL, "n_nodes must be >= 1");
  if (n_batches == 0) return PV_OK;
  if (!verdict_bits || !reached) return fail(PV_EINVAL, "null device buffer");
  HIP_OK(hipSetDevice(d->ord));
  hipStream_t s = stream ? reinterpret_cast<hipStream_t>(stream) : d->stream;
  HIP_OK(pv::launch_tally_bits(verdict_bits, dup_mask, n_batches, n_nodes, quorum, votes, reached, s));
  HIP_OK(hipStreamSynchronize(s));
  return PV_OK;
}

int pv_tally(const uint32_t* verdict_bits, const uint32_t* dup_mask, uint64_t n_batches, uint32_t n_nodes,
             uint32_t quorum, uint8_t* reached) {
  std::lock_guard<std::mutex> lk(g_mu);
  DeviceGuard dg;
  if (g_devs.empty()) return fail(PV_ENOTINIT, "pv_init has not been called");
  if (n_nodes == 0) return fail(PV_EINVAL, "n_nodes must be >= 1");
  if (n_batches == 0) return PV_OK;
  if (!verdict_bits || !reached) return fail(PV_EINVAL, "null buffer");
  Device& d = g_devs[0];
  HIP_OK(hipSetDevice(d.ord));
  const uint64_t words = n_batches * ((n_nodes + 31) / 32);
  HIP_OK(d.tbits.ensure(2 * words));
  HIP_OK(d.reached.ensure(n_batches));
  HIP_OK(hipMemcpyAsync(d.tbits.p, verdict_bits, words * 4, hipMemcpyHostToDevice, d.stream));
  if (dup_mask) HIP_OK(hipMemcpyAsync(d.tbits.p + words, dup_mask, words * 4, hipMemcpyHostToDevice, d.stream));
  HIP_OK(pv::launch_tally_bits(d.tbits.p, dup_mask ? d.tbits.p + words : nullptr, n_batches, n_nodes, quorum, nullptr,
                               d.reached.p, d.stream));
  HIP_OK(hipMemcpyAsync(reached, d.reached.p, n_batches, hipMemcpyDeviceToHost, d.stream));
  HIP_OK(hipStreamSynchronize(d.stream));
  return PV_OK;
}

int pv_sign_batch_device(const uint8_t* seeds, const uint8_t* msg_blob, const uint64_t* msg_off, uint64_t n,
                         uint8_t* pk_out, uint8_t* sig_out, int device, void* stream) {
  std::lock_guard<std::mutex> lk(g_mu);
  DeviceGuard dg;
  Device* d = find_dev(device);
  if (!d) return fail(PV_ENOTINIT, "device %d not initialised (call pv_init)", device);
  if (n == 0) return PV_OK;
  HIP_OK(hipSetDevice(d->ord));
  hipStream_t s = stream ? reinterpret_cast<hipStream_t>(stream) : d->stream;
  HIP_OK(pv::launch_sign(seeds, msg_blob, msg_off, n, d->btab.p, pk_out, sig_out, s));
  HIP_OK(hipStreamSynchronize(s));
  return PV_OK;
}

int pv_sign_batch(const uint8_t* seeds, const uint8_t* msg_blob, const uint64_t* msg_off, uint64_t n,
                  uint8_t* pk_out, uint8_t* sig_out) {
  std::lock_guard<std::mutex> lk(g_mu);
  DeviceGuard dg;
  if (g_devs.empty()) return fail(PV_ENOTINIT, "pv_init has not been called");
  if (n == 0) return PV_OK;
  if (!seeds || !msg_off || !pk_out || !sig_out) return fail(PV_EINVAL, "null buffer");
  Device& d = g_devs[0];
  HIP_OK(hipSetDevice(d.ord));
  const uint64_t b0 = msg_off[0], bytes = msg_off[n] - b0;
  std::vector<uint64_t> offs(n + 1);
  for (uint64_t k = 0; k <= n; ++k) offs[k] = msg_off[k] - b0;
  HIP_OK(d.tamper.ensure(n * 32));  // seeds staging
  HIP_OK(d.blob.ensure(bytes + 16));
  HIP_OK(d.off.ensure(n + 1));
  HIP_OK(d.pk.ensure(n * 32));
  HIP_OK(d.sig.ensure(n * 64));
  HIP_OK(hipMemcpyAsync(d.tamper.p, seeds, n * 32, hipMemcpyHostToDevice, d.stream));
  if (bytes) HIP_OK(hipMemcpyAsync(d.blob.p, msg_blob + b0, bytes, hipMemcpyHostToDevice, d.stream));
  HIP_OK(hipMemsetAsync(d.blob.p + bytes, 0, 16, d.stream));
  HIP_OK(hipMemcpyAsync(d.off.p, offs.data(), (n + 1) * 8, hipMemcpyHostToDevice, d.stream));
  HIP_OK(pv::launch_sign(d.tamper.p, d.blob.p, d.off.p, n, d.btab.p, d.pk.p, d.sig.p, d.stream));
  HIP_OK(hipMemcpyAsync(pk_out, d.pk.p, n * 32, hipMemcpyDeviceToHost, d.stream));
  HIP_OK(hipMemcpyAsync(sig_out, d.sig.p, n * 64, hipMemcpyDeviceToHost, d.stream));
  HIP_OK(hipStreamSynchronize(d.stream));
  return PV_OK;
}

}  // extern "C"

namespace {
// leaf digests (n x 8 words) -> root (8 words) on stream s, all device memory
// PV_MERKLE_TAIL_ON = 0: one k_merkle_level launch per level down to the root (A/B)
#ifndef PV_MERKLE_TAIL_ON
#define PV_MERKLE_TAIL_ON 1
#endif
int enqueue_merkle(Device& d, const uint8_t* blob, const uint64_t* off, uint64_t n, uint32_t* leaves, uint32_t* root,
                   hipStream_t s) {
  if (n == 0) {  // hash_empty(): SHA-256 of the empty string (ledger/tree_hasher.py:17-19)
    static const uint32_t empty[8] = {0x42c4b0e3u, 0x141cfc98u, 0xc8f4fb9au, 0x24b96f99u,
                                      0xe441ae27u, 0x4c939b64u, 0x1b9995a4u, 0x55b85278u};
    HIP_OK(hipMemcpyAsync(root, empty, 32, hipMemcpyHostToDevice, s));
    return PV_OK;
  }
  HIP_OK(pv::launch_sha256(blob, off, n, 1, 0x00, d.counter.p, leaves, d.sha256_blocks, s));
  const uint32_t* in = leaves;
  uint64_t m = n;
  int which = 0;
  while (m > 1) {
    if (PV_MERKLE_TAIL_ON && m <= (uint64_t)pv::MERKLE_TAIL) {   // the last levels: one launch
      HIP_OK(pv::launch_merkle_tail(in, m, root, s));
      break;
    }
    uint32_t* out = (m + 1) / 2 == 1 ? root : (which ? d.mk1.p : d.mk0.p);
    HIP_OK(pv::launch_merkle_level(in, m, out, s));
    in = out;
    m = (m + 1) / 2;
    which ^= 1;
  }
  if (n == 1) HIP_OK(hipMemcpyAsync(root, leaves, 32, hipMemcpyDeviceToDevice, s));
  return PV_OK;
}
}  // namespace

extern "C" {

int pv_sha256_batch_device(const uint8_t* blob, const uint64_t* off, uint64_t n, int32_t prefix, uint8_t* digests,
                           int device, void* stream) {
  std::lock_guard<std::mutex> lk(g_mu);
  DeviceGuard dg;
  Device* d = find_dev(device);
  if (!d) return fail(PV_ENOTINIT, "device %d not initialised (call pv_init)", device);
  if (n == 0) return PV_OK;
  if (!blob || !off || !digests) return fail(PV_EINVAL, "null device buffer");
  if (prefix > 255) return fail(PV_EINVAL, "prefix must be -1 (none) or a byte value");
  HIP_OK(hipSetDevice(d->ord));
  hipStream_t s = stream ? reinterpret_cast<hipStream_t>(stream) : d->stream;
  HIP_OK(pv::launch_sha256(blob, off, n, prefix < 0 ? 0 : 1, prefix < 0 ? 0 : (uint32_t)prefix, d->counter.p,
                           reinterpret_cast<uint32_t*>(digests), d->sha256_blocks, s));
  HIP_OK(hipStreamSynchronize(s));
  return PV_OK;
}

int pv_merkle_root_device(const uint8_t* blob, const uint64_t* off, uint64_t n, uint8_t* leaf_hashes, uint8_t* root,
                          int device, void* stream) {
  std::lock_guard<std::mutex> lk(g_mu);
  DeviceGuard dg;
  Device* d = find_dev(device);
  if (!d) return fail(PV_ENOTINIT, "device %d not initialised (call pv_init)", device);
  if (!root || (n && (!blob || !off))) return fail(PV_EINVAL, "null device buffer");
  HIP_OK(hipSetDevice(d->ord));
  hipStream_t s = stream ? reinterpret_cast<hipStream_t>(stream) : d->stream;
  uint32_t* leaves = reinterpret_cast<uint32_t*>(leaf_hashes);
  if (!leaves && n) {
    HIP_OK(d->mk1.ensure((n + 1) / 2 * 8 + n * 8));
    leaves = d->mk1.p + (n + 1) / 2 * 8;
  }
  HIP_OK(d->mk0.ensure((n + 1) / 2 * 8 + 8));
  if (leaf_hashes) HIP_OK(d->mk1.ensure((n + 1) / 2 * 8 + 8));
  int rc = enqueue_merkle(*d, blob, off, n, leaves, reinterpret_cast<uint32_t*>(root), s);
  if (rc) return rc;
  HIP_OK(hipStreamSynchronize(s));
  return PV_OK;
}

int pv_merkle_root(const uint8_t* blob, const uint64_t* off, uint64_t n, uint8_t* root, uint8_t* leaf_hashes) {
  std::lock_guard<std::mutex> lk(g_mu);
  DeviceGuard dg;
  if (g_devs.empty()) return fail(PV_ENOTINIT, "pv_init has not been called");
  if (!root || (n && (!off || (!blob && off[n] != off[0])))) return fail(PV_EINVAL, "null buffer");
  for (uint64_t i = 0; i < n; ++i)
    if (off[i + 1] < off[i]) return fail(PV_EINVAL, "off not monotone at %llu", (unsigned long long)i);
  Device& d = g_devs[0];
  HIP_OK(hipSetDevice(d.ord));
  const uint64_t b0 = n ? off[0] : 0, bytes = n ? off[n] - b0 : 0;
  std::vector<uint64_t> offs(n + 1);
  for (uint64_t k = 0; k <= n; ++k) offs[k] = n ? off[k] - b0 : 0;
  HIP_OK(d.blob.ensure(bytes + 16));
  HIP_OK(d.off.ensure(n + 1));
  HIP_OK(d.mk0.ensure((n + 1) / 2 * 8 + 8));
  HIP_OK(d.mk1.ensure((n + 1) / 2 * 8 + n * 8 + 8));
  uint32_t* leaves = d.mk1.p + (n + 1) / 2 * 8;
  uint32_t* droot = d.mk0.p + (n + 1) / 2 * 8;
  if (bytes) HIP_OK(hipMemcpyAsync(d.blob.p, blob + b0, bytes, hipMemcpyHostToDevice, d.stream));
  HIP_OK(hipMemsetAsync(d.blob.p + bytes, 0, 16, d.stream));
  HIP_OK(hipMemcpyAsync(d.off.p, offs.data(), (n + 1) * 8, hipMemcpyHostToDevice, d.stream));
  int rc = enqueue_merkle(d, d.blob.p, d.off.p, n, leaves, droot, d.stream);
  if (rc) return rc;
  HIP_OK(hipMemcpyAsync(root, droot, 32, hipMemcpyDeviceToHost, d.stream));
  if (leaf_hashes && n) HIP_OK(hipMemcpyAsync(leaf_hashes, leaves, n * 32, hipMemcpyDeviceToHost, d.stream));
  HIP_OK(hipStreamSynchronize(d.stream));
  return PV_OK;
}

int pv_sha256_batch(const uint8_t* blob, const uint64_t* off, uint64_t n, int32_t prefix, uint8_t* digests) {
  std::lock_guard<std::mutex> lk(g_mu);
  DeviceGuard dg;
  if (g_devs.empty()) return fail(PV_ENOTINIT, "pv_init has not been called");
  if (n == 0) return PV_OK;
  if (!off || !digests || (!blob && off[n] != off[0])) return fail(PV_EINVAL, "null buffer");
  if (prefix > 255) return fail(PV_EINVAL, "prefix must be -1 (none) or a byte value");
  for (uint64_t i = 0; i < n; ++i)
    if (off[i + 1] < off[i]) return fail(PV_EINVAL, "off not monotone at %llu", (unsigned long long)i);
  Device& d = g_devs[0];
  HIP_OK(hipSetDevice(d.ord));
  const uint64_t b0 = off[0], bytes = off[n] - b0;
  std::vector<uint64_t> offs(n + 1);
  for (uint64_t k = 0; k <= n; ++k) offs[k] = off[k] - b0;
  HIP_OK(d.blob.ensure(bytes + 16));
  HIP_OK(d.off.ensure(n + 1));
  HIP_OK(d.mk0.ensure(n * 8));
  if (bytes) HIP_OK(hipMemcpyAsync(d.blob.p, blob + b0, bytes, hipMemcpyHostToDevice, d.stream));
  HIP_OK(hipMemsetAsync(d.blob.p + bytes, 0, 16, d.stream));
  HIP_OK(hipMemcpyAsync(d.off.p, offs.data(), (n + 1) * 8, hipMemcpyHostToDevice, d.stream));
  HIP_OK(pv::launch_sha256(d.blob.p, d.off.p, n, prefix < 0 ? 0 : 1, prefix < 0 ? 0 : (uint32_t)prefix, d.counter.p,
                           d.mk0.p, d.sha256_blocks, d.stream));
  HIP_OK(hipMemcpyAsync(digests, d.mk0.p, n * 32, hipMemcpyDeviceToHost, d.stream));
  HIP_OK(hipStreamSynchronize(d.stream));
  return PV_OK;
}

int pv_synth_layout_device(uint32_t cfg, uint32_t mode, uint64_t first, uint64_t n, uint32_t mlen_min,
                           uint32_t mlen_max, uint32_t n_nodes, uint64_t* off, int device, void* stream) {
  std::lock_guard<std::mutex> lk(g_mu);
  DeviceGuard dg;
  Device* d = find_dev(device);
  if (!d) return fail(PV_ENOTINIT, "device %d not initialised (call pv_init)", device);
  if (!off) return fail(PV_EINVAL, "null device buffer");
  if (mode > PV_SYNTH_COMMIT) return fail(PV_EINVAL, "unknown synth mode %u", mode);
  if (mode == PV_SYNTH_RANGE && mlen_max < mlen_min) return fail(PV_EINVAL, "mlen_max < mlen_min");
  if (mode == PV_SYNTH_COMMIT && (n_nodes == 0 || n_nodes > 1024))
    return fail(PV_EINVAL, "n_nodes must be in 1..1024");
  HIP_OK(hipSetDevice(d->ord));
  hipStream_t s = stream ? reinterpret_cast<hipStream_t>(stream) : d->stream;
  HIP_OK(d->scan.ensure(pv::scan_sums_words(n + 1)));
  HIP_OK(pv::launch_synth_layout(cfg, mode, first, n, mlen_min, mlen_max, n_nodes, off, d->scan.p, s));
  HIP_OK(hipStreamSynchronize(s));
  return PV_OK;
}

int pv_synth_fill_device(uint32_t cfg, uint32_t mode, uint64_t first, uint64_t n, uint32_t key_mod,
                         uint32_t n_nodes, const uint64_t* off, uint8_t* blob, uint8_t* seeds, uint8_t* pk,
                         uint8_t* sig, uint8_t* tamper, uint32_t* sender, int device, void* stream) {
  std::lock_guard<std::mutex> lk(g_mu);
  DeviceGuard dg;
  Device* d = find_dev(device);
  if (!d) return fail(PV_ENOTINIT, "device %d not initialised (call pv_init)", device);
  if (!off || !blob || !seeds || !pk || !sig || !tamper) return fail(PV_EINVAL, "null device buffer");
  if (mode > PV_SYNTH_COMMIT) return fail(PV_EINVAL, "unknown synth mode %u", mode);
  if (mode == PV_SYNTH_COMMIT && (n_nodes == 0 || n_nodes > 1024))
    return fail(PV_EINVAL, "n_nodes must be in 1..1024");
  HIP_OK(hipSetDevice(d->ord));
  hipStream_t s = stream ? reinterpret_cast<hipStream_t>(stream) : d->stream;
  uint64_t total = 0;
  HIP_OK(hipMemcpyAsync(&total, off + n, 8, hipMemcpyDeviceToHost, s));
  HIP_OK(hipStreamSynchronize(s));
  HIP_OK(pv::launch_synth(cfg, mode, first, n, key_mod, n_nodes, seeds, tamper, sender, s));
  HIP_OK(pv::launch_synth_fill(cfg, mode, first, n, n_nodes, off, blob, s));
  HIP_OK(hipMemsetAsync(blob + total, 0, 16, s));
  HIP_OK(pv::launch_sign(seeds, blob, off, n, d->btab.p, pk, sig, s));
  HIP_OK(pv::launch_tamper(first, n, tamper, off, blob, sig, s));
  HIP_OK(hipStreamSynchronize(s));
  return PV_OK;
}

int pv_synth_device(uint32_t cfg, uint64_t first, uint64_t n, uint32_t key_mod, uint32_t mlen, uint64_t* off,
                    uint8_t* blob, uint8_t* seeds, uint8_t* pk, uint8_t* sig, uint8_t* tamper, int device,
                    void* stream) {
  int rc = pv_synth_layout_device(cfg, PV_SYNTH_FIXED, first, n, mlen, mlen, 0, off, device, stream);
  if (rc) return rc;
  return pv_synth_fill_device(cfg, PV_SYNTH_FIXED, first, n, key_mod, 0, off, blob, seeds, pk, sig, tamper, nullptr,
                              device, stream);
}

}  // extern "C"
