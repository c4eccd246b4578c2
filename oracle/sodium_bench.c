/*
 * CPU BASELINE TIMER (bench.py cpu_baseline leg / tests only — never part of
 * the product path).
 *
 * Times the native call Plenum's verify path ends in — libsodium 1.0.18
 * crypto_sign_verify_detached, reached through libnacl.crypto_sign_open
 * (stp_core/crypto/nacl_wrappers.py:86-108) — on `threads` host threads over
 * a caller-provided sample, for at least `min_seconds`.  libsodium is loaded
 * with dlopen from the path given (the image's /opt/conda/lib/libsodium.so.23);
 * if it cannot be loaded, the C restatement in ed25519_oracle.c is timed
 * instead and the function reports kind = 1 ("port").
 */
#include <dlfcn.h>
#include <pthread.h>
#include <stdint.h>
#include <string.h>
#include <time.h>

int oracle_verify_detached(const uint8_t sig[64], const uint8_t *m, uint64_t mlen, const uint8_t pk[32]);

typedef int (*verify_fn)(const unsigned char *, const unsigned char *, unsigned long long, const unsigned char *);

static verify_fn g_sodium = 0;

static int port_verify(const unsigned char *s, const unsigned char *m, unsigned long long n, const unsigned char *pk) {
  return oracle_verify_detached(s, m, n, pk);
}

typedef struct {
  const uint8_t *pk, *sig, *blob;
  const uint64_t *off;
  uint64_t n, start;
  double min_seconds;
  verify_fn fn;
  uint64_t done;
  uint64_t accepted;
} job_t;

static double now_s(void) {
  struct timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return ts.tv_sec + ts.tv_nsec * 1e-9;
}

static void *worker(void *arg) {
  job_t *j = (job_t *)arg;
  const double t0 = now_s();
  uint64_t i = j->start;
  do {
    for (int k = 0; k < 64; ++k) {
      const uint64_t o = j->off[i];
      j->accepted += j->fn(j->sig + 64 * i, j->blob + o, j->off[i + 1] - o, j->pk + 32 * i) == 0;
      j->done++;
      if (++i == j->n) i = 0;
    }
  } while (now_s() - t0 < j->min_seconds);
  return 0;
}

/* returns verifies/s; *kind = 0 libsodium, 1 port; *accepted = accepted count */
double cpu_baseline_rate(const char *sodium_path, const uint8_t *pk, const uint8_t *sig, const uint8_t *blob,
                         const uint64_t *off, uint64_t n, int threads, double min_seconds, int *kind,
                         uint64_t *accepted) {
  if (!g_sodium && sodium_path) {
    void *h = dlopen(sodium_path, RTLD_NOW | RTLD_LOCAL);
    if (h) {
      int (*init)(void) = (int (*)(void))dlsym(h, "sodium_init");
      g_sodium = (verify_fn)dlsym(h, "crypto_sign_verify_detached");
      if (init) init();
    }
  }
  *kind = g_sodium ? 0 : 1;
  verify_fn fn = g_sodium ? g_sodium : port_verify;
  if (threads < 1) threads = 1;
  if (threads > 256) threads = 256;
  pthread_t th[256];
  job_t jobs[256];
  const double t0 = now_s();
  for (int t = 0; t < threads; ++t) {
    memset(&jobs[t], 0, sizeof jobs[t]);
    jobs[t].pk = pk; jobs[t].sig = sig; jobs[t].blob = blob; jobs[t].off = off;
    jobs[t].n = n; jobs[t].start = (n * (uint64_t)t) / (uint64_t)threads;
    jobs[t].min_seconds = min_seconds; jobs[t].fn = fn;
    pthread_create(&th[t], 0, worker, &jobs[t]);
  }
  uint64_t done = 0, acc = 0;
  for (int t = 0; t < threads; ++t) {
    pthread_join(th[t], 0);
    done += jobs[t].done;
    acc += jobs[t].accepted;
  }
  const double dt = now_s() - t0;
  *accepted = acc;
  return done / dt;
}
