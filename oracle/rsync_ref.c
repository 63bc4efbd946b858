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
 *   ref_rsync_sum_sizes   <- generator.c sum_sizes_sqroot (protocol >= 30)
 */
#include <stdint.h>

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
