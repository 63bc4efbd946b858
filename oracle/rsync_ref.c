/*
 * oracle/rsync_ref.c -- CPU restatement of rsync 3.2.3's delta-matching
 * arithmetic.  TEST INFRASTRUCTURE ONLY (see cdc_ref.c header for the rule).
 *
 * The reference installs rsync as the UBI9 distro binary
 * (/root/reference/mover-rsync/Dockerfile:5-13) and runs it from
 * mover-rsync/source.sh:54 and kubectl-volsync/cmd/migration_rsync.go:185-186.
 * No rsync source is present offline; this restates the published behaviour
 * (SURVEY.md 8(a) rows R1-R7):
 *
 *   ref_rsync_checksum1   <- checksum.c get_checksum1 (signed bytes, CHAR_OFFSET 0)
 *   ref_rsync_checksum2   <- checksum.c get_checksum2 (xxh128 / xxh3 / xxh64 /
 *                            md5 with the protocol>=31 seed order)
 *   ref_rsync_sum_sizes   <- generator.c sum_sizes_sqroot (protocol >= 30)
 *   ref_rsync_signatures  <- generator.c generate_and_send_sums (sum1, sum2[s2len])
 *   ref_rsync_match       <- match.c match_sums -> build_hash_table + hash_search
 *                            (updating_basis_file = 0: no --inplace, source.sh:54)
 * XXH3/XXH64 come from the system libxxhash (dlopen; xxhash 0.8.x, the
 * library rsync 3.2.3 links); MD5 is restated here (RFC 1321).
 */
#include <dlfcn.h>
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

/* get_checksum1: s1 = sum b_j, s2 = sum (len - j) b_j over signed bytes. */
uint32_t ref_rsync_checksum1(const uint8_t *buf1, int32_t len) {
    const int8_t *buf = (const int8_t *)buf1;
    int32_t i;
    uint32_t s1 = 0, s2 = 0;
    for (i = 0; i < len - 4; i += 4) {
        s2 += 4 * (s1 + buf[i]) + 3 * buf[i + 1] + 2 * buf[i + 2] + buf[i + 3];
        s1 += (buf[i + 0] + buf[i + 1] + buf[i + 2] + buf[i + 3]);
    }
    for (; i < len; i++) {
        s1 += buf[i];
        s2 += s1;
    }
    return (s1 & 0xffff) + (s2 << 16);
}

#define RS_BLOCK_SIZE 700
#define RS_MAX_BLOCK_SIZE (1 << 17)
#define RS_BLOCKSUM_BIAS 10
#define RS_SUM_LENGTH 16
#define RS_SHORT_SUM_LENGTH 2

/* sum_sizes_sqroot for protocol >= 30 (rsync 3.2.3 <-> 3.2.3 speaks 31). */
int ref_rsync_sum_sizes(int64_t len, int32_t block_size, int32_t *blength_out,
                        int32_t *s2length_out, int32_t *count_out, int32_t *remainder_out) {
    int32_t blength;
    int s2length;
    int64_t l;
    if (len < 0) return -1;
    if (block_size)
        blength = block_size;
    else if (len <= (int64_t)RS_BLOCK_SIZE * RS_BLOCK_SIZE)
        blength = RS_BLOCK_SIZE;
    else {
        int32_t max_blength = RS_MAX_BLOCK_SIZE;
        int32_t c;
        for (c = 1, l = len; l >>= 2; c <<= 1) {
        }
        if (c < 0 || c >= max_blength)
            blength = max_blength;
        else {
            blength = 0;
            do {
                blength |= c;
                if (len < (int64_t)blength * blength) blength &= ~c;
                c >>= 1;
            } while (c >= 8);
            if (blength < RS_BLOCK_SIZE) blength = RS_BLOCK_SIZE;
        }
    }
    {
        int32_t c;
        int b = RS_BLOCKSUM_BIAS;
        for (l = len; l >>= 1; b += 2) {
        }
        for (c = blength; (c >>= 1) && b; b--) {
        }
        s2length = (b + 1 - 32 + 7) / 8;
        if (s2length < RS_SHORT_SUM_LENGTH) s2length = RS_SHORT_SUM_LENGTH;
        if (s2length > RS_SUM_LENGTH) s2length = RS_SUM_LENGTH;
    }
    int32_t remainder = (int32_t)(len % blength);
    int64_t count = len / blength + (remainder != 0);
    if ((int64_t)(int32_t)count != count) return -1;
    *blength_out = blength;
    *s2length_out = s2length;
    *remainder_out = remainder;
    *count_out = (int32_t)count;
    return 0;
}

/* ------------------------------------------------------------------ */
/* strong sums (checksum.c get_checksum2)                             */
/* ------------------------------------------------------------------ */
#define CSUM_MD5 5
#define CSUM_XXH64 6
#define CSUM_XXH3_64 7
#define CSUM_XXH3_128 8

typedef struct { uint64_t low64, high64; } xxh128_t;
typedef xxh128_t (*xxh3_128_seed_fn)(const void *, size_t, uint64_t);
typedef uint64_t (*xxh3_64_seed_fn)(const void *, size_t, uint64_t);
typedef uint64_t (*xxh64_fn)(const void *, size_t, uint64_t);
static xxh3_128_seed_fn g_x128;
static xxh3_64_seed_fn g_x3;
static xxh64_fn g_x64;
/* streaming API (the whole-file oracle at sizes no host buffer holds) */
typedef void *(*xxh3_new_fn)(void);
typedef int (*xxh3_free_fn)(void *);
typedef int (*xxh3_reset_fn)(void *);
typedef int (*xxh3_update_fn)(void *, const void *, size_t);
typedef xxh128_t (*xxh3_128_digest_fn)(const void *);
typedef uint64_t (*xxh3_64_digest_fn)(const void *);
static xxh3_new_fn g_xnew;
static xxh3_free_fn g_xfree;
static xxh3_reset_fn g_xreset128, g_xreset64;
static xxh3_update_fn g_xupd128, g_xupd64;
static xxh3_128_digest_fn g_xdig128;
static xxh3_64_digest_fn g_xdig64;

int ref_have_xxhash(void) {
    static int probed = 0;
    if (!probed) {
        probed = 1;
        void *h = dlopen("libxxhash.so.0", RTLD_NOW | RTLD_LOCAL);
        if (!h) h = dlopen("libxxhash.so", RTLD_NOW | RTLD_LOCAL);
        if (h) {
            g_x128 = (xxh3_128_seed_fn)dlsym(h, "XXH3_128bits_withSeed");
            g_x3 = (xxh3_64_seed_fn)dlsym(h, "XXH3_64bits_withSeed");
            g_x64 = (xxh64_fn)dlsym(h, "XXH64");
            g_xnew = (xxh3_new_fn)dlsym(h, "XXH3_createState");
            g_xfree = (xxh3_free_fn)dlsym(h, "XXH3_freeState");
            g_xreset128 = (xxh3_reset_fn)dlsym(h, "XXH3_128bits_reset");
            g_xreset64 = (xxh3_reset_fn)dlsym(h, "XXH3_64bits_reset");
            g_xupd128 = (xxh3_update_fn)dlsym(h, "XXH3_128bits_update");
            g_xupd64 = (xxh3_update_fn)dlsym(h, "XXH3_64bits_update");
            g_xdig128 = (xxh3_128_digest_fn)dlsym(h, "XXH3_128bits_digest");
            g_xdig64 = (xxh3_64_digest_fn)dlsym(h, "XXH3_64bits_digest");
        }
    }
    return g_x128 && g_x3 && g_x64;
}

/* MD5 (RFC 1321) */
typedef struct { uint32_t a, b, c, d; uint64_t len; uint8_t buf[64]; uint32_t fill; } md5_ctx;
static const uint32_t MD5_T[64] = {
    0xd76aa478, 0xe8c7b756, 0x242070db, 0xc1bdceee, 0xf57c0faf, 0x4787c62a, 0xa8304613, 0xfd469501,
    0x698098d8, 0x8b44f7af, 0xffff5bb1, 0x895cd7be, 0x6b901122, 0xfd987193, 0xa679438e, 0x49b40821,
    0xf61e2562, 0xc040b340, 0x265e5a51, 0xe9b6c7aa, 0xd62f105d, 0x02441453, 0xd8a1e681, 0xe7d3fbc8,
    0x21e1cde6, 0xc33707d6, 0xf4d50d87, 0x455a14ed, 0xa9e3e905, 0xfcefa3f8, 0x676f02d9, 0x8d2a4c8a,
    0xfffa3942, 0x8771f681, 0x6d9d6122, 0xfde5380c, 0xa4beea44, 0x4bdecfa9, 0xf6bb4b60, 0xbebfbc70,
    0x289b7ec6, 0xeaa127fa, 0xd4ef3085, 0x04881d05, 0xd9d4d039, 0xe6db99e5, 0x1fa27cf8, 0xc4ac5665,
    0xf4292244, 0x432aff97, 0xab9423a7, 0xfc93a039, 0x655b59c3, 0x8f0ccc92, 0xffeff47d, 0x85845dd1,
    0x6fa87e4f, 0xfe2ce6e0, 0xa3014314, 0x4e0811a1, 0xf7537e82, 0xbd3af235, 0x2ad7d2bb, 0xeb86d391};
static const uint8_t MD5_S[64] = {7, 12, 17, 22, 7, 12, 17, 22, 7, 12, 17, 22, 7, 12, 17, 22,
                                  5, 9,  14, 20, 5, 9,  14, 20, 5, 9,  14, 20, 5, 9,  14, 20,
                                  4, 11, 16, 23, 4, 11, 16, 23, 4, 11, 16, 23, 4, 11, 16, 23,
                                  6, 10, 15, 21, 6, 10, 15, 21, 6, 10, 15, 21, 6, 10, 15, 21};
static void md5_block(md5_ctx *c, const uint8_t *p) {
    uint32_t m[16];
    for (int i = 0; i < 16; ++i)
        m[i] = (uint32_t)p[4 * i] | (uint32_t)p[4 * i + 1] << 8 | (uint32_t)p[4 * i + 2] << 16 |
               (uint32_t)p[4 * i + 3] << 24;
    uint32_t a = c->a, b = c->b, cc = c->c, d = c->d;
    for (int i = 0; i < 64; ++i) {
        uint32_t f;
        int g;
        if (i < 16) { f = (b & cc) | (~b & d); g = i; }
        else if (i < 32) { f = (d & b) | (~d & cc); g = (5 * i + 1) & 15; }
        else if (i < 48) { f = b ^ cc ^ d; g = (3 * i + 5) & 15; }
        else { f = cc ^ (b | ~d); g = (7 * i) & 15; }
        uint32_t t = a + f + MD5_T[i] + m[g];
        a = d; d = cc; cc = b;
        b = b + ((t << MD5_S[i]) | (t >> (32 - MD5_S[i])));
    }
    c->a += a; c->b += b; c->c += cc; c->d += d;
}
static void md5_init(md5_ctx *c) {
    c->a = 0x67452301; c->b = 0xefcdab89; c->c = 0x98badcfe; c->d = 0x10325476;
    c->len = 0; c->fill = 0;
}
static void md5_update(md5_ctx *c, const uint8_t *p, uint64_t n) {
    c->len += n;
    while (n) {
        uint32_t take = 64 - c->fill;
        if (take > n) take = (uint32_t)n;
        memcpy(c->buf + c->fill, p, take);
        c->fill += take; p += take; n -= take;
        if (c->fill == 64) { md5_block(c, c->buf); c->fill = 0; }
    }
}
static void md5_final(md5_ctx *c, uint8_t out[16]) {
    uint64_t bits = c->len * 8;
    uint8_t pad = 0x80;
    md5_update(c, &pad, 1);
    uint8_t z = 0;
    while (c->fill != 56) md5_update(c, &z, 1);
    uint8_t lb[8];
    for (int i = 0; i < 8; ++i) lb[i] = (uint8_t)(bits >> (8 * i));
    md5_update(c, lb, 8);
    uint32_t v[4] = {c->a, c->b, c->c, c->d};
    for (int i = 0; i < 16; ++i) out[i] = (uint8_t)(v[i / 4] >> (8 * (i % 4)));
}

/* get_checksum2: 16-byte sum (only the first s2length bytes are compared) */
int ref_rsync_checksum2(const uint8_t *buf, int32_t len, int csum_type, uint32_t seed,
                        uint8_t sum[16]) {
    memset(sum, 0, 16);
    if (csum_type == CSUM_MD5) {
        md5_ctx c;
        md5_init(&c);
        if (seed) {  /* proper_seed_order (protocol >= 31): seed first */
            uint8_t sb[4] = {(uint8_t)seed, (uint8_t)(seed >> 8), (uint8_t)(seed >> 16),
                             (uint8_t)(seed >> 24)};
            md5_update(&c, sb, 4);
        }
        md5_update(&c, buf, (uint64_t)len);
        md5_final(&c, sum);
        return 0;
    }
    if (!ref_have_xxhash()) return -1;
    if (csum_type == CSUM_XXH3_128) {
        xxh128_t d = g_x128(buf, (size_t)len, seed);
        for (int i = 0; i < 8; ++i) sum[i] = (uint8_t)(d.low64 >> (8 * i));
        for (int i = 0; i < 8; ++i) sum[8 + i] = (uint8_t)(d.high64 >> (8 * i));
    } else if (csum_type == CSUM_XXH3_64) {
        uint64_t d = g_x3(buf, (size_t)len, seed);
        for (int i = 0; i < 8; ++i) sum[i] = (uint8_t)(d >> (8 * i));
    } else if (csum_type == CSUM_XXH64) {
        uint64_t d = g_x64(buf, (size_t)len, seed);
        for (int i = 0; i < 8; ++i) sum[i] = (uint8_t)(d >> (8 * i));
    } else {
        return -1;
    }
    return 0;
}

/* generate_and_send_sums: per basis block, sum1 and the first s2length bytes of sum2 */
int ref_rsync_signatures(const uint8_t *basis, int64_t len, int32_t blength, int32_t s2length,
                         int csum_type, uint32_t seed, uint32_t *sum1, uint8_t *sum2) {
    int64_t count = (len + blength - 1) / blength;
    for (int64_t i = 0; i < count; ++i) {
        int64_t off = i * (int64_t)blength;
        int32_t n = (int32_t)((len - off < blength) ? len - off : blength);
        sum1[i] = ref_rsync_checksum1(basis + off, n);
        uint8_t s[16];
        if (ref_rsync_checksum2(basis + off, n, csum_type, seed, s) < 0) return -1;
        memcpy(sum2 + i * (int64_t)s2length, s, (size_t)s2length);
    }
    return 0;
}

/* generate_and_send_sums over the synthetic stream `dseed` (cdc_ref.c
 * ref_synth_fill) of len bytes, on `threads` threads: each thread generates
 * and sums whole blocks, so a destination far larger than host memory (C4's
 * 256 GiB) is signed without ever existing in one buffer.  Same output as
 * ref_rsync_signatures over the materialised stream. */
void ref_synth_fill(uint64_t seed, uint64_t off, uint64_t n, uint8_t *out);

typedef struct {
    uint64_t dseed;
    int64_t len, count, next;
    int32_t blength, s2length;
    int csum_type;
    uint32_t seed;
    uint32_t *sum1;
    uint8_t *sum2;
    int err;
} sig_job;

static void *sig_worker(void *arg) {
    sig_job *j = (sig_job *)arg;
    uint8_t *buf = (uint8_t *)malloc((size_t)j->blength);
    if (!buf) {
        __atomic_store_n(&j->err, 1, __ATOMIC_RELAXED);
        return NULL;
    }
    for (;;) {
        const int64_t b0 = __atomic_fetch_add(&j->next, 64, __ATOMIC_RELAXED);
        if (b0 >= j->count) break;
        const int64_t b1 = b0 + 64 < j->count ? b0 + 64 : j->count;
        for (int64_t i = b0; i < b1; ++i) {
            const int64_t off = i * (int64_t)j->blength;
            const int32_t n = (int32_t)((j->len - off < j->blength) ? j->len - off : j->blength);
            ref_synth_fill(j->dseed, (uint64_t)off, (uint64_t)n, buf);
            j->sum1[i] = ref_rsync_checksum1(buf, n);
            uint8_t s[16];
            if (ref_rsync_checksum2(buf, n, j->csum_type, j->seed, s) < 0) {
                __atomic_store_n(&j->err, 1, __ATOMIC_RELAXED);
                break;
            }
            memcpy(j->sum2 + i * (int64_t)j->s2length, s, (size_t)j->s2length);
        }
    }
    free(buf);
    return NULL;
}

int ref_rsync_signatures_synth_mt(uint64_t dseed, int64_t len, int32_t blength, int32_t s2length,
                                  int csum_type, uint32_t seed, int threads, uint32_t *sum1,
                                  uint8_t *sum2) {
    if (len < 0 || blength <= 0 || s2length < 1 || s2length > 16) return -1;
    if (threads < 1) threads = 1;
    if (threads > 256) threads = 256;
    if (csum_type != CSUM_MD5 && !ref_have_xxhash()) return -1;   /* resolve before the threads */
    sig_job j = {dseed, len, (len + blength - 1) / blength, 0, blength, s2length, csum_type, seed,
                 sum1, sum2, 0};
    pthread_t th[256];
    int started = 0;
    for (int t = 0; t < threads; ++t)
        if (pthread_create(&th[t], NULL, sig_worker, &j) == 0) ++started;
    if (!started) sig_worker(&j);
    for (int t = 0; t < started; ++t) pthread_join(th[t], NULL);
    return j.err ? -1 : 0;
}

/* checksum.c sum_init/sum_update/sum_end (xxh128 / xxh3, unseeded) over the
 * synthetic stream `dseed`'s first len bytes, through libxxhash's streaming
 * API: the R7 oracle at C2/C4 sizes.  Pieces of 64 MiB are generated by
 * `threads` threads, a batch ahead of the (serial) hashing. */
typedef struct {
    uint64_t dseed, off, n;
    uint8_t *buf;
} gen_job;

static void *gen_worker(void *arg) {
    gen_job *g = (gen_job *)arg;
    ref_synth_fill(g->dseed, g->off, g->n, g->buf);
    return NULL;
}

int ref_xxh3_synth(uint64_t dseed, uint64_t len, int csum_type, int threads, uint8_t out[16]) {
    if (!ref_have_xxhash() || !g_xnew || !g_xupd128 || !g_xdig128) return -1;
    if (csum_type != CSUM_XXH3_128 && csum_type != CSUM_XXH3_64) return -1;
    if (threads < 1) threads = 1;
    if (threads > 64) threads = 64;
    const uint64_t piece = 64ull << 20, batch = piece * (uint64_t)threads;
    uint8_t *buf[2];
    buf[0] = (uint8_t *)malloc(batch);
    buf[1] = (uint8_t *)malloc(batch);
    void *st = g_xnew();
    if (!buf[0] || !buf[1] || !st) {
        free(buf[0]);
        free(buf[1]);
        if (st) g_xfree(st);
        return -1;
    }
    const int x128 = csum_type == CSUM_XXH3_128;
    (x128 ? g_xreset128 : g_xreset64)(st);
    gen_job jobs[2][64];
    pthread_t th[2][64];
    int nth[2] = {0, 0};
    /* generate batch k+1 while batch k is hashed */
    uint64_t boff = 0;
    int cur = 0;
    for (uint64_t b = 0; b * batch < len + batch; ++b) {
        /* start batch b (if any) into buf[cur] */
        nth[cur] = 0;
        if (boff < len) {
            for (int t = 0; t < threads && boff + (uint64_t)t * piece < len; ++t) {
                const uint64_t o = boff + (uint64_t)t * piece;
                gen_job *g = &jobs[cur][t];
                g->dseed = dseed;
                g->off = o;
                g->n = len - o < piece ? len - o : piece;
                g->buf = buf[cur] + (uint64_t)t * piece;
                if (pthread_create(&th[cur][t], NULL, gen_worker, g) != 0) gen_worker(g), th[cur][t] = 0;
                nth[cur]++;
            }
        }
        /* hash batch b-1 from buf[cur ^ 1] */
        const int prv = cur ^ 1;
        for (int t = 0; t < nth[prv]; ++t) {
            if (th[prv][t]) pthread_join(th[prv][t], NULL);
            (x128 ? g_xupd128 : g_xupd64)(st, jobs[prv][t].buf, (size_t)jobs[prv][t].n);
        }
        nth[prv] = 0;
        if (boff >= len) break;
        boff += batch;
        cur ^= 1;
    }
    for (int k = 0; k < 2; ++k)
        for (int t = 0; t < nth[k]; ++t)
            if (th[k][t]) pthread_join(th[k][t], NULL);
    memset(out, 0, 16);
    if (x128) {
        const xxh128_t d = g_xdig128(st);
        for (int i = 0; i < 8; ++i) out[i] = (uint8_t)(d.low64 >> (8 * i));
        for (int i = 0; i < 8; ++i) out[8 + i] = (uint8_t)(d.high64 >> (8 * i));
    } else {
        const uint64_t d = g_xdig64(st);
        for (int i = 0; i < 8; ++i) out[i] = (uint8_t)(d >> (8 * i));
    }
    g_xfree(st);
    free(buf[0]);
    free(buf[1]);
    return 0;
}

/* match_sums -> build_hash_table + hash_search.  Emits the ordered match list
 * (source offset, block index); literals are the gaps.  Returns #matches, or
 * -1 on error.  blens: per-block lengths (blength, remainder for the last). */
int64_t ref_rsync_match(const uint8_t *src, int64_t len, int32_t count, int32_t blength,
                        int32_t remainder, int32_t s2length, const uint32_t *sum1,
                        const uint8_t *sum2, int csum_type, uint32_t seed, int64_t *m_off,
                        int32_t *m_idx, int64_t cap, int64_t *false_alarms) {
    int64_t nm = 0, fa = 0;
    if (len <= 0 || count <= 0) {
        if (false_alarms) *false_alarms = 0;
        return 0;
    }
    /* build_hash_table */
    uint32_t tablesize = (uint32_t)(count / 8) * 10 + 11;
    const int trad = tablesize < (1u << 16);
    if (trad) tablesize = 1u << 16;
    int32_t *table = (int32_t *)malloc(sizeof(int32_t) * tablesize);
    int32_t *chain = (int32_t *)malloc(sizeof(int32_t) * (size_t)count);
    if (!table || !chain) { free(table); free(chain); return -1; }
    memset(table, 0xff, sizeof(int32_t) * tablesize);
    for (int32_t i = 0; i < count; ++i) {
        uint32_t t = trad ? (((sum1[i] & 0xffff) + (sum1[i] >> 16)) & 0xffff) : sum1[i] % tablesize;
        chain[i] = table[t];
        table[t] = i;
    }
#define BLEN(i) (((i) == count - 1 && remainder) ? remainder : blength)
    /* hash_search */
    const int8_t *map = (const int8_t *)src;
    int32_t want_i = 0;
    int64_t k = len < blength ? len : blength;
    uint32_t sum = ref_rsync_checksum1(src, (int32_t)k);
    uint32_t s1 = sum & 0xffff, s2 = sum >> 16;
    int64_t offset = 0;
    int64_t end = len + 1 - BLEN(count - 1);
    uint8_t sum2buf[16];
    do {  /* do-while: offset 0 is probed even when end <= 0 */
        int done_csum2 = 0;
        int32_t i;
        uint32_t hash_entry;
        if (trad) {
            hash_entry = (s1 + s2) & 0xffff;
            if ((i = table[hash_entry]) < 0) goto null_hash;
            sum = (s1 & 0xffff) | (s2 << 16);
        } else {
            sum = (s1 & 0xffff) | (s2 << 16);
            hash_entry = sum % tablesize;
            if ((i = table[hash_entry]) < 0) goto null_hash;
        }
        do {
            if (sum != sum1[i]) continue;
            int32_t l = (int32_t)((len - offset < blength) ? len - offset : blength);
            if (l != BLEN(i)) continue;
            if (!done_csum2) {
                if (ref_rsync_checksum2(src + offset, l, csum_type, seed, sum2buf) < 0) {
                    free(table); free(chain); return -1;
                }
                done_csum2 = 1;
            }
            if (memcmp(sum2buf, sum2 + (int64_t)i * s2length, (size_t)s2length) != 0) {
                fa++;
                continue;
            }
            if (i != want_i && want_i < count && sum == sum1[want_i] &&
                memcmp(sum2buf, sum2 + (int64_t)want_i * s2length, (size_t)s2length) == 0)
                i = want_i;
            want_i = i + 1;
            if (nm < cap) { m_off[nm] = offset; m_idx[nm] = i; }
            nm++;
            offset += BLEN(i) - 1;
            k = (len - offset < blength) ? len - offset : blength;
            sum = ref_rsync_checksum1(src + offset, (int32_t)k);
            s1 = sum & 0xffff;
            s2 = sum >> 16;
            break;
        } while ((i = chain[i]) >= 0);
    null_hash:;
        /* trim the first byte, add the next one (if any) */
        int more = offset + k < len;
        s1 -= (uint32_t)(int32_t)map[offset];
        s2 -= (uint32_t)k * (uint32_t)(int32_t)map[offset];
        if (more) {
            s1 += (uint32_t)(int32_t)map[offset + k];
            s2 += s1;
        } else {
            --k;
        }
    } while (++offset < end);
#undef BLEN
    free(table);
    free(chain);
    if (false_alarms) *false_alarms = fa;
    return nm;
}

/* ------------------------------------------------------------------ */
/* hash_search restricted to one shard of the source (multi-GPU walk  */
/* stitch).  TEST INFRASTRUCTURE: the checker of the     */
/* sharded device walk, and the test double of the gloo protocol.     */
/* ------------------------------------------------------------------ */
/* The greedy walk of hash_search (above), started from the state (entry,
 * want_i) instead of (0, 0), over the offsets of [entry, hi): it visits
 * offset o iff o < hi and (o < end or o == 0) -- the do-while visits offset 0
 * unconditionally -- and stops at the first offset >= hi.  *exit_off /
 * *exit_want = that state (exit_off = hi when the walk ran out at `end`), which
 * is the next shard's entry.  win points at file offset win_lo and must cover
 * [entry, min(hi + blength - 1, len)).  Offsets are file offsets; len is the
 * whole source file's length.  Matches with offset in [entry, hi) are
 * emitted in order; returns #matches or -1.  Walking [0, len) from (0, 0)
 * reproduces ref_rsync_match exactly. */
/* ref_rsync_walk_fab: the same walk; m_fab (optional, cap entries) receives
 * the false alarms counted before each match's offset was visited -- what the
 * full-size golden script (tests/golden/make_golden_full.py) needs to merge a
 * walk from the true entry into a speculative one. */
int64_t ref_rsync_walk_fab(const uint8_t *win, int64_t win_lo, int64_t len, int64_t hi,
                           int64_t entry, int32_t entry_want, int32_t count, int32_t blength,
                           int32_t remainder, int32_t s2length, const uint32_t *sum1,
                           const uint8_t *sum2, int csum_type, uint32_t seed, int64_t *m_off,
                           int32_t *m_idx, int64_t *m_fab, int64_t cap, int64_t *false_alarms,
                           int64_t *exit_off, int32_t *exit_want);

int64_t ref_rsync_walk(const uint8_t *win, int64_t win_lo, int64_t len, int64_t hi, int64_t entry,
                       int32_t entry_want, int32_t count, int32_t blength, int32_t remainder,
                       int32_t s2length, const uint32_t *sum1, const uint8_t *sum2, int csum_type,
                       uint32_t seed, int64_t *m_off, int32_t *m_idx, int64_t cap,
                       int64_t *false_alarms, int64_t *exit_off, int32_t *exit_want) {
    return ref_rsync_walk_fab(win, win_lo, len, hi, entry, entry_want, count, blength, remainder,
                              s2length, sum1, sum2, csum_type, seed, m_off, m_idx, NULL, cap,
                              false_alarms, exit_off, exit_want);
}

int64_t ref_rsync_walk_fab(const uint8_t *win, int64_t win_lo, int64_t len, int64_t hi,
                           int64_t entry, int32_t entry_want, int32_t count, int32_t blength,
                           int32_t remainder, int32_t s2length, const uint32_t *sum1,
                           const uint8_t *sum2, int csum_type, uint32_t seed, int64_t *m_off,
                           int32_t *m_idx, int64_t *m_fab, int64_t cap, int64_t *false_alarms,
                           int64_t *exit_off, int32_t *exit_want) {
    int64_t nm = 0, fa = 0;
    *exit_off = entry > hi ? entry : hi;
    *exit_want = entry_want;
    if (false_alarms) *false_alarms = 0;
    if (len <= 0 || count <= 0 || entry >= hi) return 0;
#define BLEN(i) (((i) == count - 1 && remainder) ? remainder : blength)
    const int64_t end = len + 1 - BLEN(count - 1);
    if (!(entry < end || entry == 0)) return 0;
    uint32_t tablesize = (uint32_t)(count / 8) * 10 + 11;
    const int trad = tablesize < (1u << 16);
    if (trad) tablesize = 1u << 16;
    int32_t *table = (int32_t *)malloc(sizeof(int32_t) * tablesize);
    int32_t *chain = (int32_t *)malloc(sizeof(int32_t) * (size_t)count);
    if (!table || !chain) { free(table); free(chain); return -1; }
    memset(table, 0xff, sizeof(int32_t) * tablesize);
    for (int32_t i = 0; i < count; ++i) {
        uint32_t t = trad ? (((sum1[i] & 0xffff) + (sum1[i] >> 16)) & 0xffff) : sum1[i] % tablesize;
        chain[i] = table[t];
        table[t] = i;
    }
    const int8_t *map = (const int8_t *)(win - win_lo);   /* indexed by file offset */
    int32_t want_i = entry_want;
    int64_t offset = entry;
    int64_t k = (len - offset < blength) ? len - offset : blength;
    uint32_t sum = ref_rsync_checksum1((const uint8_t *)map + offset, (int32_t)k);
    uint32_t s1 = sum & 0xffff, s2 = sum >> 16;
    uint8_t sum2buf[16];
    for (;;) {
        int done_csum2 = 0;
        int32_t i;
        const int64_t fa_visit = fa;
        sum = (s1 & 0xffff) | (s2 << 16);
        uint32_t hash_entry = trad ? ((s1 + s2) & 0xffff) : sum % tablesize;
        if ((i = table[hash_entry]) < 0) goto null_hash;
        do {
            if (sum != sum1[i]) continue;
            int32_t l = (int32_t)((len - offset < blength) ? len - offset : blength);
            if (l != BLEN(i)) continue;
            if (!done_csum2) {
                if (ref_rsync_checksum2((const uint8_t *)map + offset, l, csum_type, seed,
                                        sum2buf) < 0) {
                    free(table); free(chain); return -1;
                }
                done_csum2 = 1;
            }
            if (memcmp(sum2buf, sum2 + (int64_t)i * s2length, (size_t)s2length) != 0) {
                fa++;
                continue;
            }
            if (i != want_i && want_i < count && sum == sum1[want_i] &&
                memcmp(sum2buf, sum2 + (int64_t)want_i * s2length, (size_t)s2length) == 0)
                i = want_i;
            want_i = i + 1;
            if (nm < cap) {
                m_off[nm] = offset;
                m_idx[nm] = i;
                if (m_fab) m_fab[nm] = fa_visit;
            }
            nm++;
            offset += BLEN(i) - 1;
            if (offset + 1 >= hi || offset + 1 >= end) {   /* next visit is past the shard */
                ++offset;
                goto done;
            }
            k = (len - offset < blength) ? len - offset : blength;
            sum = ref_rsync_checksum1((const uint8_t *)map + offset, (int32_t)k);
            s1 = sum & 0xffff;
            s2 = sum >> 16;
            break;
        } while ((i = chain[i]) >= 0);
    null_hash:;
        if (offset + 1 >= hi || offset + 1 >= end) {
            ++offset;
            goto done;
        }
        int more = offset + k < len;
        s1 -= (uint32_t)(int32_t)map[offset];
        s2 -= (uint32_t)k * (uint32_t)(int32_t)map[offset];
        if (more) {
            s1 += (uint32_t)(int32_t)map[offset + k];
            s2 += s1;
        } else {
            --k;
        }
        ++offset;
    }
done:
#undef BLEN
    free(table);
    free(chain);
    *exit_off = offset >= hi ? offset : hi;
    *exit_want = want_i;
    if (false_alarms) *false_alarms = fa;
    return nm;
}
