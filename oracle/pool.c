/* ORACLE / TEST INFRASTRUCTURE ONLY: a persistent worker pool for the CPU legs.
 *
 * orc_parallel_for(n, threads, fn, ctx) runs fn(ctx, i) for i in [0, n) on `threads`
 * threads: the caller plus threads - 1 pool workers that live for the process. Items are
 * handed out one grain at a time from an atomic counter (dynamic balance for ragged
 * blocks). Workers spin briefly on the job generation before sleeping on a condition
 * variable, so back-to-back small batches (the config-5 latency path: 64 blocks, a few
 * hundred microseconds of work) pay neither thread creation nor a sleep/wake per batch.
 * Replaces the thread-per-batch pthread_create/join of round 1.
 */
#include <pthread.h>
#include <stdatomic.h>
#include <stddef.h>
#include <stdint.h>
#include <stdlib.h>
#include <unistd.h>

#include "oracle.h"

#define POOL_MAX 256
#define SPIN_ITERS 200000 /* ~50-100 us of pause loops before a worker sleeps */

typedef struct {
  pthread_mutex_t mu;
  pthread_cond_t cv;
  pthread_mutex_t submit_mu; /* one job at a time */
  int nworkers;
  _Atomic uint64_t gen;
  /* current job */
  orc_item_fn fn;
  void* ctx;
  size_t n, grain;
  int active; /* workers (by index) taking part */
  _Atomic size_t next;
  _Atomic int finished;
} pool_t;

static pool_t g_pool = {PTHREAD_MUTEX_INITIALIZER, PTHREAD_COND_INITIALIZER, PTHREAD_MUTEX_INITIALIZER, 0, 0,
                        NULL, NULL, 0, 1, 0, 0, 0};

static void run_items(pool_t* p) {
  for (;;) {
    size_t i = atomic_fetch_add(&p->next, p->grain);
    if (i >= p->n) break;
    size_t e = i + p->grain < p->n ? i + p->grain : p->n;
    for (; i < e; i++) p->fn(p->ctx, i);
  }
}

static inline void cpu_relax(void) {
#if defined(__x86_64__)
  __builtin_ia32_pause();
#endif
}

/* arg = worker index (low 16 bits) | the job generation current when it was created (the
 * next job, not yet published, is the first one it must take) */
static void* worker(void* arg) {
  const uint64_t a = (uint64_t)(uintptr_t)arg;
  const int idx = (int)(a & 0xffff);
  pool_t* p = &g_pool;
  uint64_t seen = a >> 16;
  for (;;) {
    uint64_t g;
    int spins = 0;
    while ((g = atomic_load_explicit(&p->gen, memory_order_acquire)) == seen && spins < SPIN_ITERS) {
      cpu_relax();
      spins++;
    }
    if (g == seen) {
      pthread_mutex_lock(&p->mu);
      while ((g = atomic_load(&p->gen)) == seen) pthread_cond_wait(&p->cv, &p->mu);
      pthread_mutex_unlock(&p->mu);
    }
    seen = g;
    if (idx < p->active) {
      run_items(p);
      atomic_fetch_add_explicit(&p->finished, 1, memory_order_release);
    }
  }
  return NULL;
}

void orc_parallel_for(size_t n, int threads, size_t grain, orc_item_fn fn, void* ctx) {
  if (threads <= 0) threads = (int)sysconf(_SC_NPROCESSORS_ONLN);
  if (threads > POOL_MAX) threads = POOL_MAX;
  if (grain == 0) grain = 1;
  if ((size_t)threads > (n + grain - 1) / grain) threads = n ? (int)((n + grain - 1) / grain) : 1;
  pool_t* p = &g_pool;
  pthread_mutex_lock(&p->submit_mu);
  if (threads == 1) {
    for (size_t i = 0; i < n; i++) fn(ctx, i);
    pthread_mutex_unlock(&p->submit_mu);
    return;
  }
  while (p->nworkers < threads - 1) {
    pthread_t t;
    pthread_attr_t a;
    pthread_attr_init(&a);
    pthread_attr_setdetachstate(&a, PTHREAD_CREATE_DETACHED);
    const uint64_t arg = ((uint64_t)atomic_load(&p->gen) << 16) | (uint64_t)p->nworkers;
    if (pthread_create(&t, &a, worker, (void*)(uintptr_t)arg) != 0) break;
    pthread_attr_destroy(&a);
    p->nworkers++;
  }
  const int helpers = threads - 1 < p->nworkers ? threads - 1 : p->nworkers;
  p->fn = fn;
  p->ctx = ctx;
  p->n = n;
  p->grain = grain;
  p->active = helpers;
  atomic_store(&p->next, 0);
  atomic_store(&p->finished, 0);
  pthread_mutex_lock(&p->mu);
  atomic_fetch_add_explicit(&p->gen, 1, memory_order_release);
  pthread_cond_broadcast(&p->cv);
  pthread_mutex_unlock(&p->mu);
  run_items(p);
  while (atomic_load_explicit(&p->finished, memory_order_acquire) < helpers) cpu_relax();
  pthread_mutex_unlock(&p->submit_mu);
}
