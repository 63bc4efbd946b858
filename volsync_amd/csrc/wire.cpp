// wire.cpp -- the byte formats around the hot path, so the
// device results interoperate with unmodified peers and repositories.  Host
// code: these are serialisations of results the kernels already produced.
//
//  * rsync 3.2.3 io.c write_sum_head + generator.c generate_and_send_sums:
//    the signature table on the wire: count, blength, s2length (protocol >=
//    27), remainder as 4-byte LE ints, then per block sum1 (4-byte LE int)
//    and the first s2length bytes of sum2.
//  * rsync 3.2.3 token.c simple_send_token (no -z): literal data in pieces of
//    at most CHUNK_SIZE = 32 KiB, each preceded by its length as a 4-byte LE
//    int, then the token -(i+1) for a copy of block i; match.c matched()
//    sends one token per match and the final send_token(-1) writes 0.
//  * restic v0.13.1 internal/pack: the pack header's plaintext -- per blob
//    its type (1 byte: 0 data, 1 tree), the length of its encrypted form
//    (4-byte LE) and its 32-byte ID.
#include <cstring>
#include <vector>

#include "internal.hpp"

#define VS_API extern "C" __attribute__((visibility("default")))

namespace {

constexpr int64_t kChunkSize = 32 * 1024;   // token.c CHUNK_SIZE

inline void put_i32(uint8_t *p, int32_t v) {
    const uint32_t u = (uint32_t)v;
    p[0] = (uint8_t)u;
    p[1] = (uint8_t)(u >> 8);
    p[2] = (uint8_t)(u >> 16);
    p[3] = (uint8_t)(u >> 24);
}
inline int32_t get_i32(const uint8_t *p) {
    return (int32_t)((uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) |
                     ((uint32_t)p[3] << 24));
}

}  // namespace

using vsgpu::fail;

VS_API int vs_rsync_write_sums(int32_t count, int32_t blength, int32_t s2length, int32_t remainder,
                               const uint32_t *sum1, const uint8_t *sum2, uint8_t *out, size_t cap,
                               size_t *n_out) {
    if (count < 0 || s2length < 0 || s2length > 16 || (count && (!sum1 || !sum2)) || !n_out)
        return fail(VS_ERR_ARG, "bad signature table");
    const size_t need = 16 + (size_t)count * (4 + (size_t)s2length);
    *n_out = need;
    if (!out) return 0;   // size query
    if (cap < need) return fail(VS_ERR_ARG, "output buffer too small");
    put_i32(out, count);
    put_i32(out + 4, blength);
    put_i32(out + 8, s2length);
    put_i32(out + 12, remainder);
    uint8_t *p = out + 16;
    for (int32_t i = 0; i < count; ++i) {
        put_i32(p, (int32_t)sum1[i]);
        memcpy(p + 4, sum2 + (size_t)i * s2length, (size_t)s2length);
        p += 4 + s2length;
    }
    return 0;
}

VS_API int vs_rsync_read_sums(const uint8_t *in, size_t n, int32_t *count, int32_t *blength,
                              int32_t *s2length, int32_t *remainder, uint32_t *sum1, uint8_t *sum2,
                              size_t cap_blocks) {
    if (!in || n < 16 || !count || !blength || !s2length || !remainder)
        return fail(VS_ERR_ARG, "truncated sum head");
    const int32_t c = get_i32(in), b = get_i32(in + 4), s2 = get_i32(in + 8), r = get_i32(in + 12);
    if (c < 0 || b < 0 || s2 < 0 || s2 > 16 || r < 0 || (c && r > b))
        return fail(VS_ERR_ARG, "invalid sum head");
    *count = c;
    *blength = b;
    *s2length = s2;
    *remainder = r;
    if (!sum1 && !sum2) return 0;   // header only
    if ((size_t)c > cap_blocks) return fail(VS_ERR_ARG, "output arrays too small");
    if (n < 16 + (size_t)c * (4 + (size_t)s2)) return fail(VS_ERR_ARG, "truncated sums");
    const uint8_t *p = in + 16;
    for (int32_t i = 0; i < c; ++i) {
        if (sum1) sum1[i] = (uint32_t)get_i32(p);
        if (sum2) memcpy(sum2 + (size_t)i * s2, p + 4, (size_t)s2);
        p += 4 + s2;
    }
    return 0;
}

VS_API int vs_rsync_write_tokens(const vs_match *matches, int64_t n_matches, int64_t file_len,
                                 int32_t blength, int64_t basis_len, const uint8_t *src,
                                 uint8_t *out, size_t cap, size_t *n_out) {
    if (n_matches < 0 || file_len < 0 || blength <= 0 || basis_len < 0 || !n_out ||
        (n_matches && !matches) || (file_len && !src))
        return fail(VS_ERR_ARG, "bad arguments");
    const int64_t count = (basis_len + blength - 1) / blength;
    // pass 1: size (and validation); pass 2: write
    for (int pass = 0; pass < 2; ++pass) {
        size_t w = 0;
        int64_t last = 0;
        auto literal = [&](int64_t from, int64_t to) {
            for (int64_t o = from; o < to; o += kChunkSize) {
                const int64_t k = std::min(kChunkSize, to - o);
                if (pass) {
                    put_i32(out + w, (int32_t)k);
                    memcpy(out + w + 4, src + o, (size_t)k);
                }
                w += 4 + (size_t)k;
            }
        };
        for (int64_t j = 0; j < n_matches; ++j) {
            const vs_match m = matches[j];
            if (m.offset < last || m.block_index < 0 || m.block_index >= count)
                return fail(VS_ERR_ARG, "match list out of order or block index out of range");
            const int64_t bl = std::min<int64_t>(blength, basis_len - (int64_t)m.block_index * blength);
            if (m.offset + bl > file_len) return fail(VS_ERR_ARG, "match past the end of the file");
            literal(last, m.offset);
            if (pass) put_i32(out + w, -(m.block_index + 1));
            w += 4;
            last = m.offset + bl;
        }
        literal(last, file_len);
        if (pass) put_i32(out + w, 0);   // send_token(-1): the end of the file's tokens
        w += 4;
        if (!pass) {
            *n_out = w;
            if (!out) return 0;
            if (cap < w) return fail(VS_ERR_ARG, "output buffer too small");
        }
    }
    return 0;
}

VS_API int vs_rsync_read_tokens(const uint8_t *in, size_t n, int32_t blength, int64_t basis_len,
                                vs_match *matches, size_t cap, size_t *n_matches,
                                uint8_t *literals, size_t lit_cap, size_t *n_literal,
                                int64_t *file_len) {
    if (!in || blength <= 0 || !n_matches || !n_literal || !file_len)
        return fail(VS_ERR_ARG, "bad arguments");
    size_t r = 0, nm = 0, nl = 0;
    int64_t pos = 0;
    const int64_t count = (basis_len + blength - 1) / blength;
    for (;;) {
        if (r + 4 > n) return fail(VS_ERR_ARG, "truncated token stream");
        const int32_t t = get_i32(in + r);
        r += 4;
        if (t == 0) break;
        if (t > 0) {
            if (r + (size_t)t > n) return fail(VS_ERR_ARG, "truncated literal data");
            if (literals) {
                if (nl + (size_t)t > lit_cap) return fail(VS_ERR_ARG, "literal buffer too small");
                memcpy(literals + nl, in + r, (size_t)t);
            }
            nl += (size_t)t;
            r += (size_t)t;
            pos += t;
            continue;
        }
        const int64_t i = -(int64_t)t - 1;
        if (i >= count) return fail(VS_ERR_ARG, "token names a block past the basis");
        if (matches) {
            if (nm >= cap) return fail(VS_ERR_ARG, "match buffer too small");
            matches[nm].offset = pos;
            matches[nm].block_index = (int32_t)i;
            matches[nm].reserved = 0;
        }
        ++nm;
        pos += std::min<int64_t>(blength, basis_len - i * blength);
    }
    *n_matches = nm;
    *n_literal = nl;
    *file_len = pos;
    return 0;
}

VS_API int vs_restic_pack_header(const uint8_t *types, const uint32_t *lengths,
                                 const uint8_t *ids, size_t n, uint8_t *out, size_t cap,
                                 size_t *n_out) {
    if (!n_out || (n && (!types || !lengths || !ids))) return fail(VS_ERR_ARG, "bad arguments");
    const size_t need = n * 37;
    *n_out = need;
    if (!out) return 0;
    if (cap < need) return fail(VS_ERR_ARG, "output buffer too small");
    for (size_t i = 0; i < n; ++i) {
        if (types[i] > 1) return fail(VS_ERR_ARG, "blob type must be 0 (data) or 1 (tree)");
        uint8_t *p = out + 37 * i;
        p[0] = types[i];
        put_i32(p + 1, (int32_t)lengths[i]);
        memcpy(p + 5, ids + 32 * i, 32);
    }
    return 0;
}
