/* The secondary CPU speed reference of BASELINE.md §2: OpenSSL libcrypto's Ed25519 verify
 * (EVP_DigestVerify, one-shot Ed25519 with a 32-byte message) over n signatures on `threads`
 * pthreads, each thread a contiguous shard. A speed reference only: OpenSSL implements RFC 8032's
 * strict, cofactorless check, not ZIP-215 (the reference's ed25519-consensus), so its verdicts
 * are compared with the GPU's on valid signatures alone (bench.py cpu_baseline "openssl").
 * Every signature is checked against its own public key, so the key is decoded per call, as the
 * reference's VerificationKey::try_from + verify does for a key it has not cached.
 *   gcc -O2 -fPIC -shared -pthread -o libmv_openssl.so openssl_ed25519.c -lcrypto */
#include <openssl/evp.h>
#include <pthread.h>
#include <stddef.h>
#include <stdint.h>

struct shard {
  const uint8_t *pk, *sig, *msg;
  uint8_t* status;
  size_t lo, hi;
};

static void* run(void* arg) {
  struct shard* s = (struct shard*)arg;
  EVP_MD_CTX* ctx = EVP_MD_CTX_new();
  for (size_t i = s->lo; i < s->hi; i++) {
    uint8_t ok = 0;
    EVP_PKEY* key = EVP_PKEY_new_raw_public_key(EVP_PKEY_ED25519, NULL, s->pk + 32 * i, 32);
    if (key && ctx && EVP_DigestVerifyInit(ctx, NULL, NULL, NULL, key) == 1)
      ok = EVP_DigestVerify(ctx, s->sig + 64 * i, 64, s->msg + 32 * i, 32) == 1;
    s->status[i] = ok ? 0 : 1;
    EVP_PKEY_free(key);
    if (ctx) EVP_MD_CTX_reset(ctx);
  }
  EVP_MD_CTX_free(ctx);
  return NULL;
}

/* status[i] = 0 if OpenSSL accepts signature i, else 1. Returns 0, or -1 if a thread failed to
 * start (then the shards that did start have been joined). */
int mvb_openssl_verify(const uint8_t* pk, const uint8_t* sig, const uint8_t* msg, size_t n, uint8_t* status,
                       int threads) {
  if (threads < 1) threads = 1;
  if (threads > 256) threads = 256;
  pthread_t tid[256];
  struct shard sh[256];
  int started = 0, rc = 0;
  for (int t = 0; t < threads; t++) {
    sh[t] = (struct shard){pk, sig, msg, status, n * (size_t)t / (size_t)threads, n * (size_t)(t + 1) / (size_t)threads};
    if (pthread_create(&tid[t], NULL, run, &sh[t]) != 0) {
      rc = -1;
      break;
    }
    started++;
  }
  for (int t = 0; t < started; t++) pthread_join(tid[t], NULL);
  return rc;
}
