/*
 * oracle/cdc_ref.c -- CPU restatement of restic's content-defined chunker and
 * SHA-256 blob IDs.
 *
 * TEST INFRASTRUCTURE ONLY.  This file is the parity checker and the CPU
 * baseline ("port").  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load it.  The product path (volsync_amd/csrc) never
 * links, loads or calls anything in oracle/.
 *
 * The reference repository does not contain the chunker: restic v0.13.1 is
 * git-cloned at image build time (/root/reference/mover-restic/Dockerfile:8-11)
 * and pins github.com/restic/chunker v0.4.0; blob IDs are Go crypto/sha256
 * (patched in by /root/reference/mover-restic/patch-sources.sh:16-27).  Neither
 * source tree is present offline, so this is a restatement of the published
 * algorithm, function by function:
 *
 *   ref_pol_deg / ref_pol_mod  <- chunker polynomials.go  Pol.Deg, Pol.Mod
 *   ref_tables                 <- chunker.go fillTables + appendByte
 *   ref_chunker_*              <- chunker.go Chunker{Reset,reset,Next}
 *   ref_sha256                 <- FIPS 180-4 (== Go crypto/sha256.Sum256,
 *                                 restic internal/restic/id.go Hash)
 *   ref_synth_fill             <- SURVEY.md 8(d) synthetic volume generator
 *
 * Parity pinning: SHA-256 is checked against FIPS 180-4 vectors, hashlib and
 * OpenSSL (tests/test_oracle.py).  The chunker is checked against the upstream
 * zero-data known answer (chunker_test.go: 4 x MinSize zero bytes -> four
 * MinSize chunks, Cut 0, SHA-256 07854d2f...) and against an independent
 * Python restatement that uses a different algorithm (closed-form windowed
 * fingerprint, oracle/cdc_ref.py).  Upstream's random-data vectors need Go's
 * math/rand stream and cannot be regenerated offline: the random-data chunk
 * boundaries are therefore "parity partially pinned" (DESIGN.md section 5).
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <pthread.h>
#include <dlfcn.h>

#define WINDOW 64
#define READBUF (512u * 1024u) /* chunkerBufSize = 512 KiB */

/* ------------------------------------------------------------------ */
/* GF(2)[x] polynomial helpers (chunker polynomials.go)               */
/* ------------------------------------------------------------------ */
int ref_pol_deg(uint64_t p) {
    for (int i = 63; i >= 0; --i)
        if ((p >> i) & 1) return i;
    return -1;
}

uint64_t ref_pol_mod(uint64_t x, uint64_t d) {
    if (x == 0) return 0;
    int dd = ref_pol_deg(d);
    while (ref_pol_deg(x) >= dd) x ^= d << (ref_pol_deg(x) - dd);
    return x;
}

static uint64_t append_byte(uint64_t h, uint8_t b, uint64_t pol) {
    h <<= 8;
    h |= b;
    return ref_pol_mod(h, pol);
}

/* out[b] = Hash(b || 63 zero bytes); mod[b] = (b*x^k mod P) | (b << k) */
void ref_tables(uint64_t pol, uint64_t out[256], uint64_t mod[256]) {
    int k = ref_pol_deg(pol);
    for (int b = 0; b < 256; ++b) {
        uint64_t h = append_byte(0, (uint8_t)b, pol);
        for (int i = 0; i < WINDOW - 1; ++i) h = append_byte(h, 0, pol);
        out[b] = h;
    }
    for (int b = 0; b < 256; ++b)
        mod[b] = ref_pol_mod((uint64_t)b << k, pol) | ((uint64_t)b << k);
}

/* ------------------------------------------------------------------ */
/* Chunker state machine (chunker.go Next)                            */
/* ------------------------------------------------------------------ */
typedef struct {
    /* config */
    uint64_t pol, min_size, max_size, splitmask;
    unsigned pol_shift;
    uint64_t tab_out[256], tab_mod[256];
    /* reader: an in-memory io.Reader */
    const uint8_t *src;
    uint64_t src_len, src_off;
    /* state */
    uint8_t window[WINDOW];
    unsigned wpos;
    uint8_t buf[READBUF];
    uint64_t bpos, bmax;
    uint64_t start, count, pos, pre;
    int closed;
    uint64_t digest;
} ref_chunker;

static uint64_t slide(ref_chunker *c, uint64_t digest, uint8_t b) {
    uint8_t out = c->window[c->wpos];
    c->window[c->wpos] = b;
    digest ^= c->tab_out[out];
    c->wpos = (c->wpos + 1) % WINDOW;
    uint64_t index = digest >> c->pol_shift;
    digest <<= 8;
    digest |= b;
    digest ^= c->tab_mod[index & 0xff];
    return digest;
}

static void chunker_reset_state(ref_chunker *c) {
    memset(c->window, 0, sizeof c->window);
    c->closed = 0;
    c->digest = 0;
    c->wpos = 0;
    c->count = 0;
    c->digest = slide(c, c->digest, 1);
    c->start = c->pos;
    c->pre = c->min_size - WINDOW;
}

/* io.ReadFull over the memory source: n bytes (n < cap only at the end), 0 = EOF */
static uint64_t read_full(ref_chunker *c, uint8_t *dst, uint64_t cap) {
    uint64_t n = c->src_len - c->src_off;
    if (n > cap) n = cap;
    if (n) memcpy(dst, c->src + c->src_off, n);   /* an empty source may be NULL */
    c->src_off += n;
    return n;
}

ref_chunker *ref_chunker_new(const uint8_t *src, uint64_t len, uint64_t pol,
                             uint64_t min_size, uint64_t max_size, int avg_bits) {
    if (pol == 0 || min_size < WINDOW || max_size < min_size) return NULL;
    ref_chunker *c = (ref_chunker *)calloc(1, sizeof *c);
    c->pol = pol;
    c->min_size = min_size;
    c->max_size = max_size;
    c->splitmask = (avg_bits >= 64) ? ~0ull : ((1ull << avg_bits) - 1);
    c->pol_shift = (unsigned)(ref_pol_deg(pol) - 8);
    ref_tables(pol, c->tab_out, c->tab_mod);
    c->src = src;
    c->src_len = len;
    c->src_off = 0;
    c->pos = 0;
    c->bpos = c->bmax = 0;
    chunker_reset_state(c);
    return c;
}

void ref_chunker_free(ref_chunker *c) { free(c); }

/* Returns 1 and fills (start,length,cut) for a chunk, 0 at io.EOF. */
int ref_chunker_next(ref_chunker *c, uint64_t *start, uint64_t *length, uint64_t *cut) {
    for (;;) {
        if (c->bpos >= c->bmax) {
            uint64_t n = read_full(c, c->buf, READBUF);
            if (n == 0 && !c->closed) { /* io.EOF */
                c->closed = 1;
                if (c->count > 0) {
                    *start = c->start;
                    *length = c->count;
                    *cut = c->digest;
                    return 1;
                }
            }
            if (n == 0) return 0;
            c->bpos = 0;
            c->bmax = n;
        }
        if (c->pre > 0) {
            uint64_t n = c->bmax - c->bpos;
            if (c->pre > n) {
                c->pre -= n;
                c->count += n;
                c->pos += n;
                c->bpos = c->bmax;
                continue;
            }
            c->bpos += c->pre;
            c->count += c->pre;
            c->pos += c->pre;
            c->pre = 0;
        }
        uint64_t add = c->count;
        uint64_t digest = c->digest;
        for (uint64_t i = c->bpos; i < c->bmax; ++i) {
            uint8_t b = c->buf[i];
            digest = slide(c, digest, b);
            add++;
            if (add < c->min_size) continue;
            if ((digest & c->splitmask) == 0 || add >= c->max_size) {
                uint64_t step = add - c->count;
                c->count = add;
                c->pos += step;
                c->bpos += step;
                *start = c->start;
                *length = c->count;
                *cut = digest;
                chunker_reset_state(c);
                return 1;
            }
        }
        c->digest = digest;
        uint64_t steps = c->bmax - c->bpos;
        c->count += steps;
        c->pos += steps;
        c->bpos = c->bmax;
    }
}

/* Chunk a whole buffer.  Returns the number of chunks (<= cap written), or
 * -1 on a configuration error (restic: "tables ... not initialized"). */
int64_t ref_chunk_all(const uint8_t *src, uint64_t len, uint64_t pol, uint64_t min_size,
                      uint64_t max_size, int avg_bits, uint64_t *starts, uint64_t *lens,
                      uint64_t *cuts, uint64_t cap) {
    ref_chunker *c = ref_chunker_new(src, len, pol, min_size, max_size, avg_bits);
    if (!c) return -1;
    uint64_t n = 0, s, l, k;
    while (ref_chunker_next(c, &s, &l, &k)) {
        if (n < cap) {
            starts[n] = s;
            lens[n] = l;
            cuts[n] = k;
        }
        n++;
    }
    ref_chunker_free(c);
    return (int64_t)n;
}

/* Canonical windowed fingerprint of the 64 bytes ending at p (p >= 63):
 * (sum_i B[p-63+i] x^(8(63-i))) mod P.  Used to cross-check candidates. */
uint64_t ref_window_fp(const uint8_t *src, uint64_t p, uint64_t pol) {
    uint64_t h = 0;
    for (int i = 0; i < WINDOW; ++i) h = append_byte(h, src[p - 63 + i], pol);
    return h;
}

/* ------------------------------------------------------------------ */
/* SHA-256, FIPS 180-4 (portable; independent of OpenSSL)             */
/* ------------------------------------------------------------------ */
static const uint32_t K256[64] = {
    0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4,
    0xab1c5ed5, 0xd807aa98, 0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe,
    0x9bdc06a7, 0xc19bf174, 0xe49b69c1, 0xefbe4786, 0x0fc19dc6, 0x240ca1cc, 0x2de92c6f,
    0x4a7484aa, 0x5cb0a9dc, 0x76f988da, 0x983e5152, 0xa831c66d, 0xb00327c8, 0xbf597fc7,
    0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967, 0x27b70a85, 0x2e1b2138, 0x4d2c6dfc,
    0x53380d13, 0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85, 0xa2bfe8a1, 0xa81a664b,
    0xc24b8b70, 0xc76c51a3, 0xd192e819, 0xd6990624, 0xf40e3585, 0x106aa070, 0x19a4c116,
    0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a, 0x5b9cca4f, 0x682e6ff3,
    0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7,
    0xc67178f2};

#define ROTR(x, n) (((x) >> (n)) | ((x) << (32 - (n))))

static void sha256_block(uint32_t st[8], const uint8_t *p) {
    uint32_t w[64];
    for (int i = 0; i < 16; ++i)
        w[i] = (uint32_t)p[4 * i] << 24 | (uint32_t)p[4 * i + 1] << 16 |
               (uint32_t)p[4 * i + 2] << 8 | (uint32_t)p[4 * i + 3];
    for (int i = 16; i < 64; ++i) {
        uint32_t s0 = ROTR(w[i - 15], 7) ^ ROTR(w[i - 15], 18) ^ (w[i - 15] >> 3);
        uint32_t s1 = ROTR(w[i - 2], 17) ^ ROTR(w[i - 2], 19) ^ (w[i - 2] >> 10);
        w[i] = w[i - 16] + s0 + w[i - 7] + s1;
    }
    uint32_t a = st[0], b = st[1], c = st[2], d = st[3], e = st[4], f = st[5], g = st[6],
             h = st[7];
    for (int i = 0; i < 64; ++i) {
        uint32_t S1 = ROTR(e, 6) ^ ROTR(e, 11) ^ ROTR(e, 25);
        uint32_t ch = (e & f) ^ (~e & g);
        uint32_t t1 = h + S1 + ch + K256[i] + w[i];
        uint32_t S0 = ROTR(a, 2) ^ ROTR(a, 13) ^ ROTR(a, 22);
        uint32_t mj = (a & b) ^ (a & c) ^ (b & c);
        uint32_t t2 = S0 + mj;
        h = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
    }
    st[0] += a; st[1] += b; st[2] += c; st[3] += d;
    st[4] += e; st[5] += f; st[6] += g; st[7] += h;
}

void ref_sha256(const uint8_t *data, uint64_t len, uint8_t out[32]) {
    uint32_t st[8] = {0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a,
                      0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19};
    uint64_t full = len / 64;
    for (uint64_t i = 0; i < full; ++i) sha256_block(st, data + 64 * i);
    uint8_t tail[128];
    uint64_t rem = len - 64 * full;
    memset(tail, 0, sizeof tail);
    if (rem) memcpy(tail, data + 64 * full, rem);   /* len 0: data may be NULL */
    tail[rem] = 0x80;
    uint64_t tl = (rem < 56) ? 64 : 128;
    uint64_t bits = len * 8;
    for (int i = 0; i < 8; ++i) tail[tl - 1 - i] = (uint8_t)(bits >> (8 * i));
    sha256_block(st, tail);
    if (tl == 128) sha256_block(st, tail + 64);
    for (int i = 0; i < 8; ++i) {
        out[4 * i] = (uint8_t)(st[i] >> 24);
        out[4 * i + 1] = (uint8_t)(st[i] >> 16);
        out[4 * i + 2] = (uint8_t)(st[i] >> 8);
        out[4 * i + 3] = (uint8_t)st[i];
    }
}

/* ------------------------------------------------------------------ */
/* Synthetic volume generator                        */
/* ------------------------------------------------------------------ */
static inline uint64_t splitmix_word(uint64_t seed, uint64_t i) {
    uint64_t z = seed + (i + 1) * 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

/* bytes [off, off+n) of the little-endian word stream w_0, w_1, ... */
void ref_synth_fill(uint64_t seed, uint64_t off, uint64_t n, uint8_t *out) {
    uint64_t k = 0;
    for (; k < n && ((off + k) & 7); ++k) {   /* head: up to the next word */
        const uint64_t pos = off + k;
        out[k] = (uint8_t)(splitmix_word(seed, pos >> 3) >> (8 * (pos & 7)));
    }
    for (; k + 8 <= n; k += 8) {               /* whole words, little-endian */
        const uint64_t w = splitmix_word(seed, (off + k) >> 3);
        for (int b = 0; b < 8; ++b) out[k + b] = (uint8_t)(w >> (8 * b));
    }
    for (; k < n; ++k) {                        /* tail */
        const uint64_t pos = off + k;
        out[k] = (uint8_t)(splitmix_word(seed, pos >> 3) >> (8 * (pos & 7)));
    }
}

/* ------------------------------------------------------------------ */
/* CPU baseline: restic's archiver shape (one chunker goroutine per   */
/* file, NumCPU BlobSaver goroutines hashing).  SHA-256 through        */
/* OpenSSL (SHA-NI, the analogue of Go crypto/sha256's asm path) when  */
/* libcrypto is loadable, else the portable ref_sha256.               */
/* ------------------------------------------------------------------ */
typedef unsigned char *(*sha256_fn)(const unsigned char *, size_t, unsigned char *);
static sha256_fn g_ossl_sha256 = NULL;
static int g_ossl_probed = 0;

int ref_have_openssl(void) {
    if (!g_ossl_probed) {
        g_ossl_probed = 1;
        void *h = dlopen("libcrypto.so.3", RTLD_NOW | RTLD_LOCAL);
        if (!h) h = dlopen("libcrypto.so", RTLD_NOW | RTLD_LOCAL);
        if (h) g_ossl_sha256 = (sha256_fn)dlsym(h, "SHA256");
    }
    return g_ossl_sha256 != NULL;
}

void ref_sha256_fast(const uint8_t *data, uint64_t len, uint8_t out[32]) {
    if (ref_have_openssl())
        g_ossl_sha256(data, (size_t)len, out);
    else
        ref_sha256(data, len, out);
}

typedef struct {
    const uint8_t *src;
    uint64_t *starts, *lens;
    uint8_t *ids;
    int64_t produced;          /* chunks published by the chunker thread (guarded by mu) */
    int done;                  /* the chunker has finished (guarded by mu) */
    int64_t next;              /* next chunk to claim (guarded by mu) */
    pthread_mutex_t mu;
    pthread_cond_t cv;         /* a chunk was published, or the chunker finished */
} hash_queue;

/* A hasher blocks while no chunk is published, as restic's BlobSaver
 * goroutines block on their channel: idle hashers take no CPU from the
 * chunker thread however many there are. */
static void *hash_worker(void *arg) {
    hash_queue *q = (hash_queue *)arg;
    for (;;) {
        int64_t i;
        pthread_mutex_lock(&q->mu);
        while (q->next >= q->produced && !q->done) pthread_cond_wait(&q->cv, &q->mu);
        if (q->next >= q->produced) {   /* done and drained */
            pthread_mutex_unlock(&q->mu);
            return NULL;
        }
        i = q->next++;
        pthread_mutex_unlock(&q->mu);
        ref_sha256_fast(q->src + q->starts[i], q->lens[i], q->ids + 32 * i);
    }
}

/* SHA-256 of blobs src[off[i], off[i] + len[i]) on `threads` threads (an
 * atomic work counter, 64 blobs per claim): restic's BlobSaver goroutines
 * hashing a chunk list, the all-core CPU baseline (bench.py).  TEST / BASELINE
 * INFRASTRUCTURE only.  Every blob is hashed; returns the threads that ran
 * (fewer than asked when pthread_create fails), -1 without memory. */
typedef struct {
    const uint8_t *src;
    const uint64_t *off, *len;
    uint8_t *ids;
    int64_t n, next;
} list_queue;

static void *list_worker(void *arg) {
    list_queue *q = (list_queue *)arg;
    for (;;) {
        const int64_t i0 = __atomic_fetch_add(&q->next, 64, __ATOMIC_RELAXED);
        if (i0 >= q->n) return NULL;
        const int64_t i1 = i0 + 64 < q->n ? i0 + 64 : q->n;
        for (int64_t i = i0; i < i1; ++i) ref_sha256_fast(q->src + q->off[i], q->len[i], q->ids + 32 * i);
    }
}

int ref_sha256_list(const uint8_t *src, const uint64_t *off, const uint64_t *len, int64_t n,
                    uint8_t *ids, int threads) {
    list_queue q = {src, off, len, ids, n, 0};
    if (threads < 1) threads = 1;
    if (threads > 1024) threads = 1024;
    pthread_t *th = (pthread_t *)malloc(sizeof(pthread_t) * (size_t)threads);
    if (!th) return -1;
    int started = 0;
    for (; started < threads; ++started)
        if (pthread_create(&th[started], NULL, list_worker, &q) != 0) break;
    if (started == 0) list_worker(&q);
    for (int t = 0; t < started; ++t) pthread_join(th[t], NULL);
    free(th);
    return started ? started : 1;
}

/* 1 chunker thread + n_hash hashing threads (n_hash 0: hash inline). */
int64_t ref_cdc_hash(const uint8_t *src, uint64_t len, uint64_t pol, uint64_t min_size,
                     uint64_t max_size, int avg_bits, int n_hash, uint64_t *starts,
                     uint64_t *lens, uint64_t *cuts, uint8_t *ids, uint64_t cap) {
    ref_chunker *c = ref_chunker_new(src, len, pol, min_size, max_size, avg_bits);
    if (!c) return -1;
    hash_queue q;
    memset(&q, 0, sizeof q);
    q.src = src; q.starts = starts; q.lens = lens; q.ids = ids;
    pthread_mutex_init(&q.mu, NULL);
    pthread_cond_init(&q.cv, NULL);
    pthread_t th[256];
    if (n_hash > 256) n_hash = 256;
    for (int t = 0; t < n_hash; ++t) pthread_create(&th[t], NULL, hash_worker, &q);
    uint64_t n = 0, s, l, k;
    int64_t rc = 0;
    while (ref_chunker_next(c, &s, &l, &k)) {
        if (n >= cap) { rc = -2; break; }
        starts[n] = s; lens[n] = l; cuts[n] = k;
        if (n_hash == 0) ref_sha256_fast(src + s, l, ids + 32 * n);
        n++;
        if (n_hash) {
            pthread_mutex_lock(&q.mu);
            q.produced = (int64_t)n;
            pthread_cond_signal(&q.cv);
            pthread_mutex_unlock(&q.mu);
        }
    }
    pthread_mutex_lock(&q.mu);
    q.done = 1;
    pthread_cond_broadcast(&q.cv);
    pthread_mutex_unlock(&q.mu);
    for (int t = 0; t < n_hash; ++t) pthread_join(th[t], NULL);
    pthread_cond_destroy(&q.cv);
    pthread_mutex_destroy(&q.mu);
    ref_chunker_free(c);
    return rc ? rc : (int64_t)n;
}

/* ------------------------------------------------------------------ */
/* Multi-threaded checker for the synthetic stream at full config      */
/* sizes (C2: 64 GiB).  TEST INFRASTRUCTURE (checker only).            */
/* ------------------------------------------------------------------ */
/* The chunker's digest at every position where Next() tests the cut
 * condition has slid >= 64 bytes since the last reset, so it equals the
 * canonical fingerprint of the 64-byte window ending there (checked against
 * ref_chunker_next by tests/test_oracle.py): candidate positions are a
 * property of the bytes alone and are found in parallel over byte ranges
 * (each warmed up on the 64 bytes before it).  The min/max rule then selects
 * cuts sequentially over the sorted candidates; the final chunk (EOF) is
 * re-chunked by ref_chunker_next from its start, which yields its Cut value
 * exactly; chunks are hashed in parallel.  The stream bytes are generated
 * on the fly (ref_synth_fill), so no thread holds more than a few MiB. */
typedef struct {
    uint64_t seed, lo, hi, mask;
    unsigned shift;
    const uint64_t *tab_out, *tab_mod;
    uint64_t *pos;   /* found candidate positions */
    uint64_t n, cap;
} cand_job;

static void *cand_worker(void *arg) {
    cand_job *j = (cand_job *)arg;
    enum { BLK = 1 << 20 };
    uint8_t *buf = (uint8_t *)malloc(BLK + WINDOW);
    uint8_t win[WINDOW];
    memset(win, 0, sizeof win);
    unsigned wpos = 0;
    uint64_t digest = 0;
    const uint64_t w0 = j->lo >= WINDOW ? j->lo - WINDOW : 0;
    for (uint64_t b = w0; b < j->hi; b += BLK) {
        const uint64_t n = (j->hi - b < BLK) ? j->hi - b : BLK;
        ref_synth_fill(j->seed, b, n, buf);
        for (uint64_t i = 0; i < n; ++i) {
            const uint8_t x = buf[i];
            const uint8_t out = win[wpos];
            win[wpos] = x;
            wpos = (wpos + 1) % WINDOW;
            digest ^= j->tab_out[out];
            const uint64_t idx = digest >> j->shift;
            digest = (digest << 8 | x) ^ j->tab_mod[idx & 0xff];
            const uint64_t p = b + i;
            if (p >= j->lo && p >= WINDOW - 1 && (digest & j->mask) == 0) {
                if (j->n == j->cap) {
                    j->cap = j->cap ? 2 * j->cap : 1024;
                    j->pos = (uint64_t *)realloc(j->pos, j->cap * sizeof(uint64_t));
                }
                j->pos[j->n++] = p;
            }
        }
    }
    free(buf);
    return NULL;
}

typedef struct {
    uint64_t seed;
    const uint64_t *starts, *lens;
    uint8_t *ids;
    int64_t n;
    int64_t next;
    pthread_mutex_t mu;
} synth_hash_queue;

static void *synth_hash_worker(void *arg) {
    synth_hash_queue *q = (synth_hash_queue *)arg;
    uint8_t *buf = NULL;
    uint64_t bcap = 0;
    for (;;) {
        pthread_mutex_lock(&q->mu);
        const int64_t i = q->next < q->n ? q->next++ : -1;
        pthread_mutex_unlock(&q->mu);
        if (i < 0) break;
        if (q->lens[i] > bcap) {
            bcap = q->lens[i];
            buf = (uint8_t *)realloc(buf, bcap);
        }
        ref_synth_fill(q->seed, q->starts[i], q->lens[i], buf);
        ref_sha256_fast(buf, q->lens[i], q->ids + 32 * i);
    }
    free(buf);
    return NULL;
}

/* Chunk list + blob IDs of bytes [0, len) of the synthetic stream `seed`,
 * with `threads` threads.  Returns #chunks (<= cap written) or < 0. */
int64_t ref_cdc_synth_mt(uint64_t seed, uint64_t len, uint64_t pol, uint64_t min_size,
                         uint64_t max_size, int avg_bits, int threads, uint64_t *starts,
                         uint64_t *lens, uint64_t *cuts, uint8_t *ids, uint64_t cap) {
    if (pol == 0 || min_size < WINDOW || max_size < min_size || threads < 1) return -1;
    if (threads > 256) threads = 256;
    uint64_t tab_out[256], tab_mod[256];
    ref_tables(pol, tab_out, tab_mod);
    const uint64_t mask = (avg_bits >= 64) ? ~0ull : ((1ull << avg_bits) - 1);
    cand_job jobs[256];
    pthread_t th[256];
    for (int t = 0; t < threads; ++t) {
        memset(&jobs[t], 0, sizeof jobs[t]);
        jobs[t].seed = seed;
        jobs[t].lo = len * (uint64_t)t / (uint64_t)threads;
        jobs[t].hi = len * (uint64_t)(t + 1) / (uint64_t)threads;
        jobs[t].mask = mask;
        jobs[t].shift = (unsigned)(ref_pol_deg(pol) - 8);
        jobs[t].tab_out = tab_out;
        jobs[t].tab_mod = tab_mod;
        pthread_create(&th[t], NULL, cand_worker, &jobs[t]);
    }
    for (int t = 0; t < threads; ++t) pthread_join(th[t], NULL);
    /* selection: Chunker.Next's min/max rule over the sorted candidates */
    uint64_t n = 0, s = 0;
    int jt = 0;
    uint64_t ji = 0;
    int64_t rc = 0;
    while (s < len) {
        const uint64_t lo = s + min_size - 1, lim = s + max_size - 1;
        while (jt < threads && (ji >= jobs[jt].n || jobs[jt].pos[ji] < lo)) {
            if (ji < jobs[jt].n) { ++ji; continue; }
            ++jt;
            ji = 0;
        }
        uint64_t cut;
        int eof = 0;
        if (jt < threads && jobs[jt].pos[ji] <= lim && jobs[jt].pos[ji] < len) {
            cut = jobs[jt].pos[ji];
        } else if (lim < len) {
            cut = lim;   /* forced at MaxSize */
        } else {
            cut = len - 1;
            eof = 1;
        }
        if (n >= cap) { rc = -2; break; }
        starts[n] = s;
        lens[n] = cut - s + 1;
        if (!eof) {
            uint8_t w[WINDOW];
            ref_synth_fill(seed, cut - (WINDOW - 1), WINDOW, w);
            cuts[n] = ref_window_fp(w, WINDOW - 1, pol);
        } else {
            /* the final chunk: Next() from its start gives its Cut value */
            uint8_t *tail = (uint8_t *)malloc(lens[n] ? lens[n] : 1);
            ref_synth_fill(seed, s, lens[n], tail);
            ref_chunker *c = ref_chunker_new(tail, lens[n], pol, min_size, max_size, avg_bits);
            uint64_t ts, tl, tk;
            if (!c || !ref_chunker_next(c, &ts, &tl, &tk) || tl != lens[n]) rc = -3;
            cuts[n] = tk;
            if (c) ref_chunker_free(c);
            free(tail);
        }
        ++n;
        s = cut + 1;
    }
    for (int t = 0; t < threads; ++t) free(jobs[t].pos);
    if (rc) return rc;
    synth_hash_queue q;
    memset(&q, 0, sizeof q);
    q.seed = seed;
    q.starts = starts;
    q.lens = lens;
    q.ids = ids;
    q.n = (int64_t)n;
    pthread_mutex_init(&q.mu, NULL);
    for (int t = 0; t < threads; ++t) pthread_create(&th[t], NULL, synth_hash_worker, &q);
    for (int t = 0; t < threads; ++t) pthread_join(th[t], NULL);
    pthread_mutex_destroy(&q.mu);
    return (int64_t)n;
}
