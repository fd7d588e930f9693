/* Bench infrastructure (config 5, BASELINE.json configs[4]): a native multi-threaded caller.
 *
 * The reference verifies blocks inline in one tokio task per peer (net_sync.rs:214-221,
 * 314-386): many threads each verifying the block or two a message carries. Driving that
 * from Python threads would cap both legs at the interpreter, so this driver runs `callers`
 * pthreads that each call a verify function back to back on `per_call` consecutive blocks of
 * a packed buffer (thread t takes calls t, t + callers, ...), records every call's latency
 * and stops at `seconds` or after `max_calls` calls per thread.
 *
 *   kind 0: mv_verify_blocks(ctx, buf, off, len, n, status, NULL, NULL)   (the product C ABI)
 *   kind 1: orc_block_verify_batch_c(ctx, buf, off, len, n, status, NULL, NULL, inner_threads)
 *           (the oracle's CPU StatementBlock::verify, committee keys decoded once)
 *
 * Function pointers come from the caller (ctypes), so this file links neither library.
 */
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

typedef int32_t (*mv_verify_blocks_fn)(void* ctx, const uint8_t* buf, const uint64_t* off, const uint64_t* len,
                                       uint32_t n, uint8_t* status, uint8_t* msg_digest, uint8_t* block_digest);
typedef void (*orc_verify_batch_c_fn)(const void* committee, const uint8_t* buf, const uint64_t* off,
                                      const uint64_t* len, size_t n, uint8_t* status, uint8_t* msg_digests,
                                      uint8_t* block_digests, int threads);

typedef struct {
  int kind;
  void* fn;
  void* ctx;
  const uint8_t* buf;
  const uint64_t *off, *len;
  uint32_t nblocks, per_call;
  int callers, inner_threads;
  double seconds;
  uint64_t max_calls;
  pthread_barrier_t start;
  double t_stop;
} job_t;

typedef struct {
  job_t* j;
  int t;
  double* lat;
  uint64_t n, cap, bad, err;
} thr_t;

static double now(void) {
  struct timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return (double)ts.tv_sec + 1e-9 * (double)ts.tv_nsec;
}

static void* run(void* arg) {
  thr_t* r = (thr_t*)arg;
  job_t* j = r->j;
  uint8_t* st = (uint8_t*)malloc(j->per_call + 1);
  const uint32_t ncalls_in_corpus = j->nblocks / j->per_call;
  pthread_barrier_wait(&j->start);
  for (uint64_t c = (uint64_t)r->t;; c += (uint64_t)j->callers) {
    if (j->max_calls && r->n >= j->max_calls) break;
    const double t0 = now();
    if (j->seconds > 0 && t0 >= j->t_stop) break;
    const uint32_t first = (uint32_t)(c % ncalls_in_corpus) * j->per_call;
    memset(st, 0xff, j->per_call);
    if (j->kind == 0) {
      if (((mv_verify_blocks_fn)j->fn)(j->ctx, j->buf, j->off + first, j->len + first, j->per_call, st, NULL, NULL))
        r->err++;
    } else {
      ((orc_verify_batch_c_fn)j->fn)(j->ctx, j->buf, j->off + first, j->len + first, j->per_call, st, NULL, NULL,
                                     j->inner_threads);
    }
    const double dt = now() - t0;
    for (uint32_t i = 0; i < j->per_call; i++) r->bad += st[i] != 0;
    if (r->n == r->cap) {
      r->cap = r->cap ? 2 * r->cap : 4096;
      r->lat = (double*)realloc(r->lat, r->cap * sizeof(double));
    }
    r->lat[r->n++] = dt;
  }
  free(st);
  return NULL;
}

/* Returns the number of calls made (all threads); lat_out[0 .. min(calls, lat_cap)) receives
 * their latencies in seconds (thread by thread), *wall the seconds from the common start to the
 * last thread's end, *bad the blocks whose status was not OK, *errors the calls that failed. */
uint64_t mvb_concurrent(int kind, void* fn, void* ctx, const uint8_t* buf, const uint64_t* off, const uint64_t* len,
                        uint32_t nblocks, uint32_t per_call, int callers, int inner_threads, double seconds,
                        uint64_t max_calls, double* lat_out, uint64_t lat_cap, double* wall, uint64_t* bad,
                        uint64_t* errors) {
  if (callers < 1 || per_call < 1 || nblocks < per_call || (seconds <= 0 && max_calls == 0)) return 0;
  job_t j = {kind, fn, ctx, buf, off, len, nblocks, per_call, callers, inner_threads, seconds, max_calls};
  pthread_barrier_init(&j.start, NULL, (unsigned)callers + 1);
  pthread_t* th = (pthread_t*)calloc((size_t)callers, sizeof(pthread_t));
  thr_t* r = (thr_t*)calloc((size_t)callers, sizeof(thr_t));
  for (int t = 0; t < callers; t++) {
    r[t].j = &j;
    r[t].t = t;
    pthread_create(&th[t], NULL, run, &r[t]);
  }
  const double t0 = now();
  j.t_stop = t0 + seconds;
  pthread_barrier_wait(&j.start);
  for (int t = 0; t < callers; t++) pthread_join(th[t], NULL);
  *wall = now() - t0;
  uint64_t total = 0, k = 0;
  *bad = 0;
  *errors = 0;
  for (int t = 0; t < callers; t++) {
    for (uint64_t i = 0; i < r[t].n && k < lat_cap; i++) lat_out[k++] = r[t].lat[i];
    total += r[t].n;
    *bad += r[t].bad;
    *errors += r[t].err;
    free(r[t].lat);
  }
  free(r);
  free(th);
  pthread_barrier_destroy(&j.start);
  return total;
}
