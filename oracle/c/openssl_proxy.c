/* TEST INFRASTRUCTURE ONLY (bench.py cpu_baseline): OpenSSL 3 Ed25519
 * single-verify throughput on the host cores, the strict-semantics CPU proxy
 * SURVEY §8(d) names when Go / curve25519-voi cannot run (RFC 8032,
 * cofactorless, rejects non-canonical encodings: it agrees with ZIP-215 on
 * honest signatures only, so the bench feeds it honest ones).  Never part of
 * the product path and never a parity checker. */
#include <openssl/evp.h>
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>

typedef struct {
  const uint8_t *pk, *sig, *msg;
  const uint32_t *off, *key_idx;
  EVP_PKEY **keys;  /* decoded once per distinct key (voi caches expanded keys too) */
  uint8_t *out;
  uint32_t lo, hi;
} job_t;

static void *run(void *arg) {
  job_t *j = (job_t *)arg;
  EVP_MD_CTX *ctx = EVP_MD_CTX_new();
  for (uint32_t i = j->lo; i < j->hi; i++) {
    EVP_PKEY *key = j->keys ? j->keys[j->key_idx[i]]
                            : EVP_PKEY_new_raw_public_key(EVP_PKEY_ED25519, NULL, j->pk + 32ull * i, 32);
    int ok = 0;
    if (key && EVP_DigestVerifyInit(ctx, NULL, NULL, NULL, key) == 1)
      ok = EVP_DigestVerify(ctx, j->sig + 64ull * i, 64, j->msg + j->off[i], j->off[i + 1] - j->off[i]) == 1;
    j->out[i] = (uint8_t)ok;
    if (!j->keys) EVP_PKEY_free(key);
    EVP_MD_CTX_reset(ctx);
  }
  EVP_MD_CTX_free(ctx);
  return NULL;
}

/* key_idx / n_keys / keys32: optional (NULL, 0, NULL) table of distinct keys,
 * entry i signed by keys32[key_idx[i]]; without it every entry decodes its key. */
int openssl_ed25519_verify_batch(const uint8_t *pk, const uint8_t *sig, const uint8_t *msg, const uint32_t *off,
                                 uint32_t n, uint8_t *out, int threads, const uint8_t *keys32,
                                 const uint32_t *key_idx, uint32_t n_keys) {
  if (threads < 1) threads = 1;
  if (threads > 256) threads = 256;
  EVP_PKEY **keys = NULL;
  if (keys32 && key_idx && n_keys) {
    keys = (EVP_PKEY **)calloc(n_keys, sizeof(EVP_PKEY *));
    for (uint32_t k = 0; k < n_keys; k++)
      keys[k] = EVP_PKEY_new_raw_public_key(EVP_PKEY_ED25519, NULL, keys32 + 32ull * k, 32);
  }
  pthread_t th[256];
  job_t jobs[256];
  for (int t = 0; t < threads; t++) {
    jobs[t] = (job_t){pk, sig, msg, off, key_idx, keys, out, (uint32_t)((uint64_t)n * t / threads),
                      (uint32_t)((uint64_t)n * (t + 1) / threads)};
    pthread_create(&th[t], NULL, run, &jobs[t]);
  }
  int all = 1;
  for (int t = 0; t < threads; t++) pthread_join(th[t], NULL);
  for (uint32_t i = 0; i < n; i++) all &= out[i];
  if (keys) {
    for (uint32_t k = 0; k < n_keys; k++) EVP_PKEY_free(keys[k]);
    free(keys);
  }
  return all;
}
