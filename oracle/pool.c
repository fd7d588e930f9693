/* ORACLE / TEST INFRASTRUCTURE ONLY: a persistent worker pool for the CPU legs.
 *
 * orc_parallel_for(n, threads, grain, fn, ctx) runs fn(ctx, i) for i in [0, n) on `threads`
 * threads: the caller plus threads - 1 pool workers that live for the process. Items are
 * handed out one grain at a time from an atomic counter (dynamic balance for ragged blocks).
 * Every worker has its own mailbox: the caller posts the job's generation to the mailboxes of
 * exactly the helpers it wants and waits for each of them to post it back, so a worker can
 * never act on another job's parameters. Workers spin briefly on their mailbox before
 * sleeping on a condition variable, so back-to-back small batches (the config-5 latency path:
 * 64 blocks, a few hundred microseconds of work) pay neither thread creation nor a sleep and
 * wake per batch. Replaces the thread-per-batch pthread_create/join of round 1.
 */
#include <pthread.h>
#include <sched.h>
#include <stdatomic.h>
#include <stddef.h>
#include <stdint.h>
#include <stdlib.h>
#include <unistd.h>

#include "oracle.h"

#define POOL_MAX 256
#define SPIN_ITERS 2000 /* ~30 us of pause loops before a worker sleeps */

typedef struct {
  _Atomic uint64_t post; /* generation of the job this worker must take part in */
  _Atomic uint64_t done; /* generation it has finished */
  char pad[48];
} mailbox_t;

static struct {
  pthread_mutex_t mu;
  pthread_cond_t cv;
  pthread_mutex_t submit_mu; /* one job at a time */
  int nworkers;
  uint64_t gen;
  /* the current job, written before any mailbox is posted */
  orc_item_fn fn;
  void* ctx;
  size_t n, grain;
  _Atomic size_t next;
  mailbox_t box[POOL_MAX];
} g_pool = {.mu = PTHREAD_MUTEX_INITIALIZER, .cv = PTHREAD_COND_INITIALIZER, .submit_mu = PTHREAD_MUTEX_INITIALIZER};

static inline void cpu_relax(void) {
#if defined(__x86_64__)
  __builtin_ia32_pause();
#endif
}

static void run_items(void) {
  for (;;) {
    size_t i = atomic_fetch_add(&g_pool.next, g_pool.grain);
    if (i >= g_pool.n) break;
    size_t e = i + g_pool.grain < g_pool.n ? i + g_pool.grain : g_pool.n;
    for (; i < e; i++) g_pool.fn(g_pool.ctx, i);
  }
}

static void* worker(void* arg) {
  mailbox_t* mb = &g_pool.box[(int)(intptr_t)arg];
  uint64_t seen = 0; /* posts start at generation 1: a job posted before this thread ran is still seen */
  for (;;) {
    uint64_t g;
    int spins = 0;
    while ((g = atomic_load_explicit(&mb->post, memory_order_acquire)) == seen && spins < SPIN_ITERS) {
      cpu_relax();
      spins++;
    }
    if (g == seen) {
      pthread_mutex_lock(&g_pool.mu);
      while ((g = atomic_load(&mb->post)) == seen) pthread_cond_wait(&g_pool.cv, &g_pool.mu);
      pthread_mutex_unlock(&g_pool.mu);
    }
    seen = g;
    run_items();
    atomic_store_explicit(&mb->done, g, memory_order_release);
  }
  return NULL;
}

void orc_parallel_for(size_t n, int threads, size_t grain, orc_item_fn fn, void* ctx) {
  if (threads <= 0) threads = (int)sysconf(_SC_NPROCESSORS_ONLN);
  if (threads > POOL_MAX) threads = POOL_MAX;
  if (grain == 0) grain = 1;
  const size_t chunks = (n + grain - 1) / grain;
  if ((size_t)threads > chunks) threads = chunks ? (int)chunks : 1;
  if (threads == 1) {
    /* inline on the caller's thread, without the pool: concurrent single-threaded callers
     * (one per peer, the config-5 "own core" leg) must run side by side, not one at a time */
    for (size_t i = 0; i < n; i++) fn(ctx, i);
    return;
  }
  pthread_mutex_lock(&g_pool.submit_mu);
  while (g_pool.nworkers < threads - 1) {
    pthread_t t;
    pthread_attr_t a;
    pthread_attr_init(&a);
    pthread_attr_setdetachstate(&a, PTHREAD_CREATE_DETACHED);
    const int ok = pthread_create(&t, &a, worker, (void*)(intptr_t)g_pool.nworkers) == 0;
    pthread_attr_destroy(&a);
    if (!ok) break;
    g_pool.nworkers++;
  }
  const int helpers = threads - 1 < g_pool.nworkers ? threads - 1 : g_pool.nworkers;
  const uint64_t g = ++g_pool.gen;
  g_pool.fn = fn;
  g_pool.ctx = ctx;
  g_pool.n = n;
  g_pool.grain = grain;
  atomic_store(&g_pool.next, 0);
  pthread_mutex_lock(&g_pool.mu);
  for (int w = 0; w < helpers; w++) atomic_store_explicit(&g_pool.box[w].post, g, memory_order_release);
  pthread_cond_broadcast(&g_pool.cv);
  pthread_mutex_unlock(&g_pool.mu);
  run_items();
  for (int w = 0; w < helpers; w++)
    for (int spins = 0; atomic_load_explicit(&g_pool.box[w].done, memory_order_acquire) != g; spins++) {
      if (spins < SPIN_ITERS) cpu_relax();
      else sched_yield();  /* more threads than free cores: let the helper run */
    }
  pthread_mutex_unlock(&g_pool.submit_mu);
}
