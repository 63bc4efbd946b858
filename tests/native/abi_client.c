/*
 * tests/native/abi_client.c -- a plain C client of include/vsgpu.h, the way
 * the cgo package (gpuchunker/) and rsync's match.c call site
 * drive it: no Python, no torch.  Built by __graft_entry__.build() against
 * volsync_amd/lib/libvsgpu.so; run by tests/test_native_abi.py (-m gpu), which
 * compares its output with the golden fixtures.
 *
 *   abi_client cdc <seed> <len> <read_size> <batch_bytes>
 *       Chunker.Next loop over the synthetic stream fed in
 *       read_size pieces through vs_cdc_feed, exactly as FileSaver.saveFile
 *       reads a file: prints "start length cut id" per chunk.
 *   abi_client rsync <file>
 *       file = [i64 basis_len][i64 src_len][i32 csum][u32 seed][i32 block]
 *              [basis][src]; vs_rsync_sizes + vs_rsync_signatures on the
 *       basis (generate_and_send_sums), vs_rsync_match of the source against
 *       that table (match_sums): prints "offset block" per match.
 *   abi_client rsync-plan <plan> <read_size> <piece> <ring>
 *       The streamed forms, as rsync's generator and sender read files
 *       through map_ptr: plan = [i64 dlen][i32 csum][u32 seed][i32 block]
 *       [u32 dseed][i64 nseg] then nseg x [i64 length][u64 stream seed]
 *       [i64 stream offset] -- the basis is the synthetic stream dseed, the
 *       source the concatenated segments (bench.py C4Plan).  Both are
 *       generated read_size bytes at a time into one host buffer and fed:
 *       vs_rsync_sig_begin/feed/next (sums collected after every read), then
 *       vs_rsync_load_sums + vs_rsync_match_begin/feed/next (matches drained
 *       after every read, as matched() would be called; the whole-file
 *       checksum computed as the source passes).  Prints "sizes ...",
 *       "offset block" per match, "file_sum <hex>", then "false_alarms N".
 */
#include <inttypes.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../../include/vsgpu.h"

static uint64_t splitmix_word(uint64_t seed, uint64_t i) {
    uint64_t z = seed + (i + 1) * 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

static void synth(uint64_t seed, uint64_t off, uint64_t n, uint8_t *out) {
    uint64_t k = 0;
    for (; k < n && ((off + k) & 7); ++k)
        out[k] = (uint8_t)(splitmix_word(seed, (off + k) >> 3) >> (8 * ((off + k) & 7)));
    for (; k + 8 <= n; k += 8) {   /* whole little-endian words */
        const uint64_t w = splitmix_word(seed, (off + k) >> 3);
        memcpy(out + k, &w, 8);
    }
    for (; k < n; ++k)
        out[k] = (uint8_t)(splitmix_word(seed, (off + k) >> 3) >> (8 * ((off + k) & 7)));
}

static int die(const char *what, int rc) {
    fprintf(stderr, "%s failed (%d): %s\n", what, rc, vs_last_error());
    return 1;
}

static int run_cdc(uint64_t seed, uint64_t len, uint64_t read_size, uint64_t batch) {
    vs_cdc *h = NULL;
    int rc = vs_cdc_open(0, VS_DEFAULT_POL, VS_MIN_SIZE, VS_MAX_SIZE, VS_AVG_BITS, &h);
    if (rc) return die("vs_cdc_open", rc);
    if ((rc = vs_cdc_set_batch_bytes(h, batch))) return die("vs_cdc_set_batch_bytes", rc);
    uint8_t *buf = (uint8_t *)malloc(read_size ? read_size : 1);
    vs_chunk out[16];
    uint64_t fed = 0, chunks = 0;
    for (;;) {
        size_t n = 0;
        rc = vs_cdc_next(h, out, 16, &n);
        if (rc == VS_EOF) break;
        if (rc < 0) return die("vs_cdc_next", rc);
        for (size_t i = 0; i < n; ++i, ++chunks) {
            printf("%" PRIu64 " %" PRIu64 " 0x%" PRIx64 " ", out[i].start, out[i].length, out[i].cut);
            for (int b = 0; b < 32; ++b) printf("%02x", out[i].id[b]);
            printf("\n");
        }
        if (n) continue;
        /* Next() needs input: the io.Reader's next read */
        const uint64_t take = (len - fed < read_size) ? len - fed : read_size;
        synth(seed, fed, take, buf);
        fed += take;
        if ((rc = vs_cdc_feed(h, buf, take, fed == len))) return die("vs_cdc_feed", rc);
    }
    free(buf);
    vs_cdc_close(h);
    fprintf(stderr, "cdc: %" PRIu64 " chunks over %" PRIu64 " bytes\n", chunks, len);
    return 0;
}

static int run_rsync(const char *path) {
    FILE *f = fopen(path, "rb");
    if (!f) return die("fopen", -1);
    int64_t blen = 0, slen = 0;
    int32_t csum = 0, block = 0;
    uint32_t seed = 0;
    if (fread(&blen, 8, 1, f) != 1 || fread(&slen, 8, 1, f) != 1 || fread(&csum, 4, 1, f) != 1 ||
        fread(&seed, 4, 1, f) != 1 || fread(&block, 4, 1, f) != 1)
        return die("read header", -1);
    uint8_t *basis = (uint8_t *)malloc(blen ? blen : 1), *src = (uint8_t *)malloc(slen ? slen : 1);
    if (fread(basis, 1, (size_t)blen, f) != (size_t)blen || fread(src, 1, (size_t)slen, f) != (size_t)slen)
        return die("read data", -1);
    fclose(f);
    int32_t bl = 0, s2 = 0, count = 0, rem = 0;
    int rc = vs_rsync_sizes(blen, block, &bl, &s2, &count, &rem);
    if (rc) return die("vs_rsync_sizes", rc);
    uint32_t *sum1 = (uint32_t *)malloc(sizeof(uint32_t) * (count ? count : 1));
    uint8_t *sum2 = (uint8_t *)malloc((size_t)s2 * (count ? count : 1));
    if ((rc = vs_rsync_signatures(0, basis, blen, bl, s2, csum, seed, sum1, sum2)))
        return die("vs_rsync_signatures", rc);
    vs_sigtable t = {count, bl, s2, rem, sum1, sum2};
    const size_t cap = (size_t)(slen / (rem && rem < bl ? rem : bl)) + 8;
    vs_match *m = (vs_match *)malloc(sizeof(vs_match) * cap);
    size_t nm = 0;
    if ((rc = vs_rsync_match(0, src, slen, &t, csum, seed, m, cap, &nm)))
        return die("vs_rsync_match", rc);
    printf("sizes %d %d %d %d\n", bl, s2, count, rem);
    for (size_t i = 0; i < nm; ++i) printf("%" PRId64 " %d\n", m[i].offset, m[i].block_index);
    fprintf(stderr, "rsync: %zu matches\n", nm);
    free(m);
    free(sum1);
    free(sum2);
    free(basis);
    free(src);
    return 0;
}

typedef struct {
    int64_t length;
    uint64_t seed;
    int64_t off;
} plan_seg;

/* bytes [pos, pos + n) of the plan's source into out */
static void plan_fill(const plan_seg *sg, int64_t nseg, int64_t pos, int64_t n, uint8_t *out) {
    int64_t start = 0;
    for (int64_t k = 0; k < nseg && n > 0; ++k) {
        const int64_t end = start + sg[k].length;
        if (pos < end) {
            const int64_t take = (end - pos < n) ? end - pos : n;
            synth(sg[k].seed, (uint64_t)(sg[k].off + (pos - start)), (uint64_t)take, out);
            out += take;
            pos += take;
            n -= take;
        }
        start = end;
    }
}

static int run_rsync_plan(const char *path, uint64_t read_size, uint64_t piece, uint32_t ring) {
    FILE *f = fopen(path, "rb");
    if (!f) return die("fopen", -1);
    int64_t dlen = 0, nseg = 0;
    int32_t csum = 0, block = 0;
    uint32_t seed = 0, dseed = 0;
    if (fread(&dlen, 8, 1, f) != 1 || fread(&csum, 4, 1, f) != 1 || fread(&seed, 4, 1, f) != 1 ||
        fread(&block, 4, 1, f) != 1 || fread(&dseed, 4, 1, f) != 1 || fread(&nseg, 8, 1, f) != 1)
        return die("read plan header", -1);
    plan_seg *sg = (plan_seg *)malloc(sizeof(plan_seg) * (nseg ? nseg : 1));
    if (fread(sg, sizeof(plan_seg), (size_t)nseg, f) != (size_t)nseg) return die("read plan", -1);
    fclose(f);
    int64_t slen = 0;
    for (int64_t k = 0; k < nseg; ++k) slen += sg[k].length;
    int32_t bl = 0, s2 = 0, count = 0, rem = 0;
    int rc = vs_rsync_sizes(dlen, block, &bl, &s2, &count, &rem);
    if (rc) return die("vs_rsync_sizes", rc);
    vs_rsync *h = NULL;
    if ((rc = vs_rsync_open(0, &h))) return die("vs_rsync_open", rc);
    uint8_t *buf = (uint8_t *)malloc(read_size);
    uint32_t *sum1 = (uint32_t *)malloc(sizeof(uint32_t) * (count ? count : 1));
    uint8_t *sum2 = (uint8_t *)malloc((size_t)s2 * (count ? count : 1));
    /* generate_and_send_sums: read the basis, send each block's sums */
    if ((rc = vs_rsync_sig_begin(h, dlen, bl, s2, csum, seed, piece, ring)))
        return die("vs_rsync_sig_begin", rc);
    int64_t got = 0;
    for (int64_t pos = 0;;) {
        for (;;) {   /* the sums finished so far (write_int / write_buf in rsync) */
            size_t n = 0;
            rc = vs_rsync_sig_next(h, sum1 + got, sum2 + (size_t)got * s2, (size_t)(count - got), &n);
            if (rc < 0) return die("vs_rsync_sig_next", rc);
            got += (int64_t)n;
            if (rc == VS_EOF || !n) break;
        }
        if (rc == VS_EOF) break;
        if (pos == dlen) continue;   /* every byte fed: next waits for the last pieces */
        const int64_t take = (dlen - pos < (int64_t)read_size) ? dlen - pos : (int64_t)read_size;
        synth(dseed, (uint64_t)pos, (uint64_t)take, buf);
        if ((rc = vs_rsync_sig_feed(h, buf, (size_t)take))) return die("vs_rsync_sig_feed", rc);
        pos += take;
    }
    if (got != count) return die("signature count", -1);
    /* match_sums: the table, then the source read in order */
    if ((rc = vs_rsync_load_sums(h, count, bl, s2, rem, sum1, sum2, csum, seed)))
        return die("vs_rsync_load_sums", rc);
    if ((rc = vs_rsync_match_begin(h, slen, csum, piece, ring))) return die("vs_rsync_match_begin", rc);
    printf("sizes %d %d %d %d\n", bl, s2, count, rem);
    vs_match m[256];
    int64_t nm = 0;
    for (int64_t pos = 0;;) {
        for (;;) {   /* matched() for every match found so far */
            size_t n = 0;
            rc = vs_rsync_match_next(h, m, 256, &n);
            if (rc < 0) return die("vs_rsync_match_next", rc);
            for (size_t i = 0; i < n; ++i) printf("%" PRId64 " %d\n", m[i].offset, m[i].block_index);
            nm += (int64_t)n;
            if (rc == VS_EOF || !n) break;
        }
        if (rc == VS_EOF) break;
        if (pos == slen) continue;
        const int64_t take = (slen - pos < (int64_t)read_size) ? slen - pos : (int64_t)read_size;
        plan_fill(sg, nseg, pos, take, buf);
        if ((rc = vs_rsync_match_feed(h, buf, (size_t)take))) return die("vs_rsync_match_feed", rc);
        pos += take;
    }
    int64_t total = 0, fa = 0;
    uint8_t fsum[16];
    if ((rc = vs_rsync_match_end(h, &total, &fa, fsum))) return die("vs_rsync_match_end", rc);
    if (total != nm) return die("match count", -1);
    printf("file_sum ");
    for (int b = 0; b < 16; ++b) printf("%02x", fsum[b]);
    printf("\nfalse_alarms %" PRId64 "\n", fa);
    fprintf(stderr, "rsync-plan: %" PRId64 " matches, %" PRId64 " false alarms over %" PRId64 " bytes\n",
            nm, fa, slen);
    vs_rsync_close(h);
    free(buf);
    free(sum1);
    free(sum2);
    free(sg);
    return 0;
}

int main(int argc, char **argv) {
    if (argc >= 6 && !strcmp(argv[1], "cdc"))
        return run_cdc(strtoull(argv[2], 0, 0), strtoull(argv[3], 0, 0), strtoull(argv[4], 0, 0),
                       strtoull(argv[5], 0, 0));
    if (argc >= 3 && !strcmp(argv[1], "rsync")) return run_rsync(argv[2]);
    if (argc >= 6 && !strcmp(argv[1], "rsync-plan"))
        return run_rsync_plan(argv[2], strtoull(argv[3], 0, 0), strtoull(argv[4], 0, 0),
                              (uint32_t)strtoul(argv[5], 0, 0));
    if (argc >= 2 && !strcmp(argv[1], "version")) {
        printf("%s devices=%d\n", vs_version(), vs_device_count());
        return 0;
    }
    fprintf(stderr, "usage: abi_client cdc <seed> <len> <read_size> <batch> | rsync <file> | "
                    "rsync-plan <plan> <read_size> <piece> <ring> | version\n");
    return 2;
}
