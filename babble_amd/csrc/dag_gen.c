/*
 * dag_gen.c -- deterministic synthetic gossip DAG generator (see dag_gen.h).
 * Host-side input generation only; never part of a timed region.
 */
#define OPENSSL_SUPPRESS_DEPRECATED 1
#include "dag_gen.h"

#include <openssl/bn.h>
#include <openssl/ec.h>
#include <openssl/obj_mac.h>
#include <openssl/sha.h>
#include <pthread.h>
#include <sched.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

/* SHA-256 through the low-level interface: OpenSSL 3's one-shot SHA256()
 * fetches the digest under a global lock on every call, which serialises
 * the worker threads */
static void sha256(const uint8_t *in, size_t len, uint8_t *out) {
  SHA256_CTX c;
  SHA256_Init(&c);
  SHA256_Update(&c, in, len);
  SHA256_Final(out, &c);
}

uint32_t bg_fnv1a32(const uint8_t *data, int64_t len) {
  uint32_t h = 2166136261u;
  for (int64_t i = 0; i < len; i++) {
    h ^= data[i];
    h *= 16777619u;
  }
  return h;
}

/* ---- xoshiro256** ---- */
typedef struct { uint64_t s[4]; } rng_t;
static uint64_t splitmix64(uint64_t *x) {
  uint64_t z = (*x += 0x9E3779B97F4A7C15ull);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
static inline uint64_t rotl(uint64_t x, int k) { return (x << k) | (x >> (64 - k)); }
static uint64_t rng_next(rng_t *r) {
  uint64_t *s = r->s;
  uint64_t res = rotl(s[1] * 5, 7) * 9, t = s[1] << 17;
  s[2] ^= s[0]; s[3] ^= s[1]; s[1] ^= s[2]; s[0] ^= s[3]; s[2] ^= t; s[3] = rotl(s[3], 45);
  return res;
}
static uint64_t rng_below(rng_t *r, uint64_t m) { /* unbiased */
  uint64_t lim = UINT64_MAX - UINT64_MAX % m, v;
  do v = rng_next(r); while (v >= lim);
  return v % m;
}
static double rng_unit(rng_t *r) { return (rng_next(r) >> 11) * (1.0 / 9007199254740992.0); }

/* ---- Go encoding helpers ---- */
static const char B64[] = "ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789+/";
static int b64enc(const uint8_t *in, int len, char *out) {
  int o = 0, i = 0;
  for (; i + 2 < len; i += 3) {
    uint32_t v = (uint32_t)in[i] << 16 | (uint32_t)in[i + 1] << 8 | in[i + 2];
    out[o++] = B64[v >> 18]; out[o++] = B64[(v >> 12) & 63];
    out[o++] = B64[(v >> 6) & 63]; out[o++] = B64[v & 63];
  }
  if (len - i == 1) {
    uint32_t v = (uint32_t)in[i] << 16;
    out[o++] = B64[v >> 18]; out[o++] = B64[(v >> 12) & 63]; out[o++] = '='; out[o++] = '=';
  } else if (len - i == 2) {
    uint32_t v = (uint32_t)in[i] << 16 | (uint32_t)in[i + 1] << 8;
    out[o++] = B64[v >> 18]; out[o++] = B64[(v >> 12) & 63]; out[o++] = B64[(v >> 6) & 63];
    out[o++] = '=';
  }
  return o;
}
/* fmt.Sprintf("0x%X", hash) (event.go:239-245) */
static int hexup(const uint8_t *h, char *out) {
  static const char HX[] = "0123456789ABCDEF";
  out[0] = '0'; out[1] = 'x';
  for (int i = 0; i < 32; i++) { out[2 + 2 * i] = HX[h[i] >> 4]; out[3 + 2 * i] = HX[h[i] & 15]; }
  return 66;
}

int32_t bg_tx_bytes(const bg_dag *d, int64_t e, uint8_t *buf64) {
  if (!d->ntx[e]) return 0;
  char tmp[96];
  int l = snprintf(tmp, sizeof tmp, "babble p%03d tx %010d", d->creator[e], d->index[e]);
  memcpy(buf64, tmp, (size_t)l);
  return l;
}

/* json.NewEncoder(&b).Encode(EventBody) (event.go:32-39): field order
 * Transactions, Parents, Creator, Index, BlockSignatures; nil slices encode as
 * null, empty non-nil slices as [] (initial events carry nil payloads,
 * Core.AddSelfEvent empty pools, node/core.go:295-310). */
int32_t bg_body_json(const bg_dag *d, int64_t e, char *buf) {
  int o = 0;
  int initial = d->index[e] == 0;
  o += sprintf(buf + o, "{\"Transactions\":");
  if (initial && !d->ntx[e]) o += sprintf(buf + o, "null");
  else if (!d->ntx[e]) o += sprintf(buf + o, "[]");
  else {
    uint8_t tx[64];
    int32_t l = bg_tx_bytes(d, e, tx);
    buf[o++] = '['; buf[o++] = '"';
    o += b64enc(tx, l, buf + o);
    buf[o++] = '"'; buf[o++] = ']';
  }
  o += sprintf(buf + o, ",\"Parents\":[\"");
  int32_t sp = d->self_parent[e], op = d->other_parent[e];
  if (sp < 0) o += sprintf(buf + o, "Root%lld", (long long)d->participant_ids[d->creator[e]]);
  else o += hexup(d->hash + (size_t)sp * 32, buf + o);
  o += sprintf(buf + o, "\",\"");
  if (op >= 0) o += hexup(d->hash + (size_t)op * 32, buf + o);
  o += sprintf(buf + o, "\"],\"Creator\":\"");
  o += b64enc(d->pubkeys + (size_t)d->creator[e] * 65, 65, buf + o);
  o += sprintf(buf + o, "\",\"Index\":%d,\"BlockSignatures\":%s}\n", d->index[e],
               initial ? "null" : "[]");
  return o;
}

/* big.Int.Text(36) of a 32-byte big-endian value */
static int base36(const uint8_t *be, char *out) {
  uint8_t v[32];
  memcpy(v, be, 32);
  char t[64];
  int k = 0, nz = 1;
  while (nz) {
    uint32_t rem = 0;
    nz = 0;
    for (int i = 0; i < 32; i++) {
      const uint32_t cur = rem << 8 | v[i];
      v[i] = (uint8_t)(cur / 36);
      rem = cur % 36;
      nz |= v[i];
    }
    t[k++] = "0123456789abcdefghijklmnopqrstuvwxyz"[rem];
  }
  for (int i = 0; i < k; i++) out[i] = t[k - 1 - i];
  return k;
}

int32_t bg_sig_string(const bg_dag *d, int64_t e, char *buf) {
  int o = base36(d->sig_r + (size_t)e * 32, buf);
  buf[o++] = '|';
  return o + base36(d->sig_s + (size_t)e * 32, buf + o);
}

typedef struct {
  const bg_dag *d;
  int64_t first, lo, hi;
  uint8_t *bodies, *sigs;
  int64_t *bo, *so;  /* per-event lengths first, offsets after the scan */
  int pass;
} bytes_job;

static void *bytes_worker(void *arg) {
  bytes_job *j = (bytes_job *)arg;
  char jb[1024];
  for (int64_t i = j->lo; i < j->hi; i++) {
    const int64_t e = j->first + i;
    if (j->pass == 0) {
      j->bo[i + 1] = bg_body_json(j->d, e, jb);
      j->so[i + 1] = bg_sig_string(j->d, e, jb);
    } else {  /* through jb: sprintf's terminator must not land in the next body */
      memcpy(j->bodies + j->bo[i], jb, (size_t)bg_body_json(j->d, e, jb));
      memcpy(j->sigs + j->so[i], jb, (size_t)bg_sig_string(j->d, e, jb));
    }
  }
  return NULL;
}

void bg_event_bytes(const bg_dag *d, int64_t first, int64_t count, uint8_t *bodies, int64_t *body_offsets,
                    uint8_t *sigs, int64_t *sig_offsets) {
  enum { T = 16 };
  pthread_t th[T];
  bytes_job jobs[T];
  body_offsets[0] = sig_offsets[0] = 0;
  for (int pass = 0; pass < 2; pass++) {
    for (int t = 0; t < T; t++) {
      jobs[t] = (bytes_job){d, first, count * t / T, count * (t + 1) / T, bodies, sigs, body_offsets, sig_offsets, pass};
      pthread_create(&th[t], NULL, bytes_worker, &jobs[t]);
    }
    for (int t = 0; t < T; t++) pthread_join(th[t], NULL);
    if (pass == 0)
      for (int64_t i = 0; i < count; i++) {
        body_offsets[i + 1] += body_offsets[i];
        sig_offsets[i + 1] += sig_offsets[i];
      }
  }
}

/* ---- ECDSA (P-256) ---- */
typedef struct {
  const bg_dag *d;
  uint64_t seed;
  int sig_mode;
  int64_t lo, hi;
  const BIGNUM *const *priv; /* [n] */
} sig_job;

static void *sig_worker(void *arg) {
  sig_job *j = (sig_job *)arg;
  const bg_dag *d = j->d;
  uint8_t buf[64];
  memcpy(buf, &j->seed, 8);
  if (j->sig_mode == 0) {
    for (int64_t e = j->lo; e < j->hi; e++) {
      uint8_t in[41];
      in[0] = 'r';
      memcpy(in + 1, &j->seed, 8);
      memcpy(in + 9, d->hash + (size_t)e * 32, 32);
      sha256(in, sizeof in, d->sig_r + (size_t)e * 32);
      d->sig_r[(size_t)e * 32] &= 0x7F; /* < q */
      in[0] = 's';
      sha256(in, sizeof in, d->sig_s + (size_t)e * 32);
      d->sig_s[(size_t)e * 32] &= 0x7F;
    }
    return NULL;
  }
  EC_GROUP *g = EC_GROUP_new_by_curve_name(NID_X9_62_prime256v1);
  BN_CTX *ctx = BN_CTX_new();
  BIGNUM *q = BN_new(), *k = BN_new(), *kinv = BN_new(), *r = BN_new(), *s = BN_new(),
         *e_bn = BN_new(), *x = BN_new(), *t = BN_new();
  EC_POINT *R = EC_POINT_new(g);
  EC_GROUP_get_order(g, q, ctx);
  for (int64_t e = j->lo; e < j->hi; e++) {
    const uint8_t *hsh = d->hash + (size_t)e * 32;
    memcpy(buf + 8, hsh, 32);
    uint8_t kb[32];
    sha256(buf, 40, kb);
    BN_bin2bn(kb, 32, k);
    BN_nnmod(k, k, q, ctx);
    if (BN_is_zero(k)) BN_one(k);
    EC_POINT_mul(g, R, k, NULL, NULL, ctx);
    EC_POINT_get_affine_coordinates(g, R, x, NULL, ctx);
    BN_nnmod(r, x, q, ctx);
    BN_bin2bn(hsh, 32, e_bn);
    BN_mod_mul(t, r, j->priv[d->creator[e]], q, ctx);
    BN_mod_add(t, t, e_bn, q, ctx);
    BN_mod_inverse(kinv, k, q, ctx);
    BN_mod_mul(s, kinv, t, q, ctx);
    BN_bn2binpad(r, d->sig_r + (size_t)e * 32, 32);
    BN_bn2binpad(s, d->sig_s + (size_t)e * 32, 32);
  }
  EC_POINT_free(R);
  BN_free(q); BN_free(k); BN_free(kinv); BN_free(r); BN_free(s); BN_free(e_bn); BN_free(x); BN_free(t);
  BN_CTX_free(ctx);
  EC_GROUP_free(g);
  return NULL;
}

typedef struct {
  bg_dag *d;
  uint8_t *done;
  int t, T;
} hash_job;

static void *hash_worker(void *arg) {
  hash_job *j = (hash_job *)arg;
  bg_dag *d = j->d;
  char jb[1024];
  for (int64_t e = j->t; e < d->N; e += j->T) {
    const int32_t sp = d->self_parent[e], op = d->other_parent[e];
    while ((sp >= 0 && !__atomic_load_n(&j->done[sp], __ATOMIC_ACQUIRE)) ||
           (op >= 0 && !__atomic_load_n(&j->done[op], __ATOMIC_ACQUIRE)))
      sched_yield();
    int32_t l = bg_body_json(d, e, jb);
    sha256((const uint8_t *)jb, (size_t)l, d->hash + (size_t)e * 32);
    __atomic_store_n(&j->done[e], 1, __ATOMIC_RELEASE);
  }
  return NULL;
}

typedef struct { int64_t id; int32_t key; } pid_sort;
static int cmp_pid(const void *a, const void *b) {
  int64_t x = ((const pid_sort *)a)->id, y = ((const pid_sort *)b)->id;
  return x < y ? -1 : x > y;
}

int bg_generate(const bg_params *p, bg_dag *out) {
  memset(out, 0, sizeof *out);
  int32_t n = p->n;
  int64_t N = p->N;
  if (n < 2 || N < n) return -1;
  out->n = n; out->N = N;
  out->participant_ids = (int64_t *)calloc((size_t)n, 8);
  out->pubkeys = (uint8_t *)calloc((size_t)n, 65);
  out->creator = (int32_t *)malloc((size_t)N * 4);
  out->index = (int32_t *)malloc((size_t)N * 4);
  out->self_parent = (int32_t *)malloc((size_t)N * 4);
  out->other_parent = (int32_t *)malloc((size_t)N * 4);
  out->ntx = (int32_t *)malloc((size_t)N * 4);
  out->hash = (uint8_t *)malloc((size_t)N * 32);
  out->sig_r = (uint8_t *)malloc((size_t)N * 32);
  out->sig_s = (uint8_t *)malloc((size_t)N * 32);
  if (!out->creator || !out->hash || !out->sig_r || !out->sig_s) return -2;

  /* keys -> ids -> ID-sorted slots */
  EC_GROUP *g = EC_GROUP_new_by_curve_name(NID_X9_62_prime256v1);
  BN_CTX *ctx = BN_CTX_new();
  BIGNUM *q = BN_new();
  EC_GROUP_get_order(g, q, ctx);
  BIGNUM **priv_raw = (BIGNUM **)calloc((size_t)n, sizeof(BIGNUM *));
  uint8_t *pub_raw = (uint8_t *)calloc((size_t)n, 65);
  pid_sort *ps = (pid_sort *)calloc((size_t)n, sizeof(pid_sort));
  EC_POINT *P = EC_POINT_new(g);
  for (int32_t i = 0; i < n; i++) {
    uint8_t in[22], d32[32];
    memcpy(in, "babble-hip", 10);
    memcpy(in + 10, &p->seed, 8);
    memcpy(in + 18, &i, 4);
    sha256(in, sizeof in, d32);
    priv_raw[i] = BN_bin2bn(d32, 32, NULL);
    BN_nnmod(priv_raw[i], priv_raw[i], q, ctx);
    if (BN_is_zero(priv_raw[i])) BN_one(priv_raw[i]);
    EC_POINT_mul(g, P, priv_raw[i], NULL, NULL, ctx);
    EC_POINT_point2oct(g, P, POINT_CONVERSION_UNCOMPRESSED, pub_raw + (size_t)i * 65, 65, ctx);
    ps[i].id = (int64_t)bg_fnv1a32(pub_raw + (size_t)i * 65, 65);
    ps[i].key = i;
  }
  qsort(ps, (size_t)n, sizeof(pid_sort), cmp_pid);
  BIGNUM **priv = (BIGNUM **)calloc((size_t)n, sizeof(BIGNUM *));
  for (int32_t s = 0; s < n; s++) {
    out->participant_ids[s] = ps[s].id;
    memcpy(out->pubkeys + (size_t)s * 65, pub_raw + (size_t)ps[s].key * 65, 65);
    priv[s] = priv_raw[ps[s].key];
  }
  EC_POINT_free(P);

  /* gossip process */
  rng_t rng;
  uint64_t sm = p->seed;
  for (int k = 0; k < 4; k++) rng.s[k] = splitmix64(&sm);
  int32_t *head = (int32_t *)malloc((size_t)n * 4), *seq = (int32_t *)malloc((size_t)n * 4),
          *last = (int32_t *)malloc((size_t)n * 4);
  double *w = (double *)malloc((size_t)n * sizeof(double));
  for (int32_t s = 0; s < n; s++) w[s] = p->lagging > 0 ? (double)(p->lag_div > 0 ? p->lag_div : 50) : 1.0;
  for (int32_t l = 0; l < p->lagging && l < n; l++) { /* pick lagging slots */
    int32_t s;
    do s = (int32_t)rng_below(&rng, (uint64_t)n); while (w[s] == 1.0);
    w[s] = 1.0;
  }
  for (int32_t s = 0; s < n; s++) {
    out->creator[s] = s; out->index[s] = 0; out->self_parent[s] = -1; out->other_parent[s] = -1;
    out->ntx[s] = 0;
    head[s] = s; seq[s] = 0; last[s] = -1;
  }
  double wsum = 0;
  for (int32_t s = 0; s < n; s++) wsum += w[s];
  for (int64_t e = n; e < N; e++) {
    int32_t to, from;
    if (p->lagging > 0) {
      double u = rng_unit(&rng) * wsum;
      for (to = 0; to < n - 1 && (u -= w[to]) >= 0; to++) {}
      double ws = wsum - w[to] - (last[to] >= 0 && n > 2 ? w[last[to]] : 0);
      do {
        u = rng_unit(&rng) * ws;
        for (from = 0; from < n; from++) {
          if (from == to || (n > 2 && from == last[to])) continue;
          if ((u -= w[from]) < 0) break;
        }
      } while (from >= n);
    } else {
      to = (int32_t)rng_below(&rng, (uint64_t)n);
      int32_t excl = (n > 2 && last[to] >= 0) ? 2 : 1;
      int32_t pick = (int32_t)rng_below(&rng, (uint64_t)(n - excl));
      for (from = 0; from < n; from++) {
        if (from == to || (excl == 2 && from == last[to])) continue;
        if (pick-- == 0) break;
      }
    }
    last[to] = from;
    out->creator[e] = to;
    out->index[e] = ++seq[to];
    out->self_parent[e] = head[to];
    out->other_parent[e] = head[from];
    out->ntx[e] = rng_unit(&rng) < p->tx_prob ? 1 : 0;
    head[to] = (int32_t)e;
  }
  free(head); free(seq); free(last); free(w);

  int T = p->threads > 0 ? p->threads : (int)sysconf(_SC_NPROCESSORS_ONLN);
  if (T > 16) T = 16;
  if (T < 1) T = 1;
  pthread_t th[16];

  /* hashes: a body holds its parents' hex hashes, so event e waits for its
   * parents' (always lower ids).  Thread t hashes e = t, t + T, ... in
   * order, spinning on the parents' done flags: the lowest unfinished
   * event always has its parents done, so the threads cannot deadlock. */
  hash_job hj[16];
  uint8_t *done = (uint8_t *)calloc((size_t)N, 1);
  for (int t = 0; t < T; t++) {
    hj[t].d = out; hj[t].done = done; hj[t].t = t; hj[t].T = T;
    pthread_create(&th[t], NULL, hash_worker, &hj[t]);
  }
  for (int t = 0; t < T; t++) pthread_join(th[t], NULL);
  free(done);

  /* signatures, in parallel */
  sig_job jobs[16];
  for (int t = 0; t < T; t++) {
    jobs[t].d = out; jobs[t].seed = p->seed; jobs[t].sig_mode = p->sig_mode;
    jobs[t].lo = N * t / T; jobs[t].hi = N * (t + 1) / T;
    jobs[t].priv = (const BIGNUM *const *)priv;
    pthread_create(&th[t], NULL, sig_worker, &jobs[t]);
  }
  for (int t = 0; t < T; t++) pthread_join(th[t], NULL);

  for (int32_t i = 0; i < n; i++) BN_free(priv_raw[i]);
  free(priv_raw); free(priv); free(pub_raw); free(ps);
  BN_free(q); BN_CTX_free(ctx); EC_GROUP_free(g);
  return 0;
}

void bg_free(bg_dag *d) {
  free(d->participant_ids); free(d->pubkeys); free(d->creator); free(d->index);
  free(d->self_parent); free(d->other_parent); free(d->ntx); free(d->hash);
  free(d->sig_r); free(d->sig_s);
  memset(d, 0, sizeof *d);
}
