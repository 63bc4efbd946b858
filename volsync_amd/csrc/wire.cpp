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
//  * rsync 3.2.3 token.c send_zstd_token / recv_zstd_token: the token
//    stream under -z (mover-rsync/source.sh:54 runs rsync -aAhHSxz) between
//    two UBI9 rsync 3.2.3 builds.  Those builds link libzstd and liblz4, and
//    compat.c's default compression list is "zstd lz4 zlibx zlib none", so
//    the negotiated choice is zstd.  Literal data goes
//    through one zstd stream per transfer (the contexts outlive the file:
//    rsync creates them once), flushed at every token, in DEFLATED_DATA
//    pieces of <= 16383 bytes; block tokens are run-length coded relative to
//    the last run's end (TOKEN_REL / TOKENRUN_REL / TOKEN_LONG /
//    TOKENRUN_LONG); END_FLAG closes the file.  libzstd.so.1 is loaded at
//    run time (no header in the image: the stable 1.4 ABI is declared below).
//  * restic v0.13.1 internal/pack: the pack header's plaintext -- per blob
//    its type (1 byte: 0 data, 1 tree), the length of its encrypted form
//    (4-byte LE) and its 32-byte ID.
#include <dlfcn.h>

#include <cstring>
#include <mutex>
#include <string>
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
    // io.c read_sum_head's checks (protocol >= 30: blength <= MAX_BLOCK_SIZE
    // = 2^17, s2length <= MAX_DIGEST_LEN = 16, 0 <= remainder <= blength),
    // plus a positive blength whenever there are blocks (every later use
    // divides by it)
    if (c < 0 || b < 0 || b > (1 << 17) || s2 < 0 || s2 > 16 || r < 0 || r > b || (c && !b))
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

// ---- rsync -z token stream (zstd) ------------------------------------------------
namespace {

// libzstd 1.4 stable ABI (zstd.h): streaming compression / decompression
struct ZIn {
    const void *src;
    size_t size, pos;
};
struct ZOut {
    void *dst;
    size_t size, pos;
};
enum { kZContinue = 0, kZFlush = 1 };
constexpr int kZLevelParam = 100;   // ZSTD_c_compressionLevel

struct ZstdApi {
    void *(*createC)();
    size_t (*freeC)(void *);
    size_t (*setParam)(void *, int, int);
    size_t (*compress2)(void *, ZOut *, ZIn *, int);
    void *(*createD)();
    size_t (*freeD)(void *);
    size_t (*decompress)(void *, ZOut *, ZIn *);
    size_t (*dOutSize)();
    unsigned (*isError)(size_t);
    const char *(*errName)(size_t);
    bool ok = false;
};

const ZstdApi &zstd() {
    static ZstdApi a;
    static std::once_flag once;
    std::call_once(once, [] {
        void *h = dlopen("libzstd.so.1", RTLD_NOW | RTLD_LOCAL);
        if (!h) return;
        a.createC = (void *(*)())dlsym(h, "ZSTD_createCCtx");
        a.freeC = (size_t(*)(void *))dlsym(h, "ZSTD_freeCCtx");
        a.setParam = (size_t(*)(void *, int, int))dlsym(h, "ZSTD_CCtx_setParameter");
        a.compress2 = (size_t(*)(void *, ZOut *, ZIn *, int))dlsym(h, "ZSTD_compressStream2");
        a.createD = (void *(*)())dlsym(h, "ZSTD_createDCtx");
        a.freeD = (size_t(*)(void *))dlsym(h, "ZSTD_freeDCtx");
        a.decompress = (size_t(*)(void *, ZOut *, ZIn *))dlsym(h, "ZSTD_decompressStream");
        a.dOutSize = (size_t(*)())dlsym(h, "ZSTD_DStreamOutSize");
        a.isError = (unsigned (*)(size_t))dlsym(h, "ZSTD_isError");
        a.errName = (const char *(*)(size_t))dlsym(h, "ZSTD_getErrorName");
        a.ok = a.createC && a.freeC && a.setParam && a.compress2 && a.createD && a.freeD &&
               a.decompress && a.dOutSize && a.isError && a.errName;
    });
    return a;
}

// token.c flag bytes
constexpr uint8_t kEndFlag = 0, kTokenLong = 0x20, kTokenRunLong = 0x21, kDeflated = 0x40,
                  kTokenRel = 0x80, kTokenRunRel = 0xc0;
constexpr size_t kMaxDataCount = 16383;

}  // namespace

// One rsync -z session's zstd state, both directions: the sender's
// compressor and token-run state, the receiver's decompressor.
struct vs_ztok {
    void *cctx = nullptr, *dctx = nullptr;
    // send_zstd_token's statics
    int32_t last_token = -1, run_start = 0, last_run_end = 0;
    bool flush_pending = false;
    uint8_t obuf[kMaxDataCount + 2];
    ZOut zout{nullptr, 0, 0};
    std::vector<uint8_t> out;       // the last file's stream
    // recv_zstd_token's state
    std::vector<uint8_t> dbuf;
};

namespace {

void w_byte(vs_ztok *z, uint8_t b) { z->out.push_back(b); }
void w_int(vs_ztok *z, int32_t v) {
    uint8_t b[4];
    put_i32(b, v);
    z->out.insert(z->out.end(), b, b + 4);
}

// token.c send_zstd_token(f, token, buf, offset, nb): nb literal bytes at
// data, then (deferred into the current run) token
int send_zstd_token(vs_ztok *z, int32_t token, const uint8_t *data, int32_t nb) {
    const ZstdApi &Z = zstd();
    if (z->last_token == -1) {
        z->last_run_end = 0;
        z->run_start = token;
        z->flush_pending = false;
    } else if (z->last_token == -2) {
        z->run_start = token;
    } else if (nb != 0 || token != z->last_token + 1 || token >= z->run_start + 65536) {
        // the previous run
        const int32_t r = z->run_start - z->last_run_end;
        const int32_t n = z->last_token - z->run_start;
        if (r >= 0 && r <= 63) {
            w_byte(z, (uint8_t)((n == 0 ? kTokenRel : kTokenRunRel) + r));
        } else {
            w_byte(z, n == 0 ? kTokenLong : kTokenRunLong);
            w_int(z, z->run_start);
        }
        if (n != 0) {
            w_byte(z, (uint8_t)n);
            w_byte(z, (uint8_t)(n >> 8));
        }
        z->last_run_end = z->last_token;
        z->run_start = token;
    }
    z->last_token = token;
    if (nb || z->flush_pending) {
        ZIn in{data, (size_t)nb, 0};
        int flush = kZContinue;
        size_t r = 0;
        do {
            if (z->zout.size == 0) {
                z->zout.size = kMaxDataCount;
                z->zout.pos = 0;
            }
            if (token != -2) flush = kZFlush;
            r = Z.compress2(z->cctx, &z->zout, &in, flush);
            if (Z.isError(r)) return fail(VS_ERR_STATE, std::string("ZSTD_compressStream2: ") + Z.errName(r));
            if (z->zout.pos == z->zout.size || flush == kZFlush) {
                const size_t n = z->zout.pos;
                z->obuf[0] = (uint8_t)(kDeflated + (n >> 8));
                z->obuf[1] = (uint8_t)n;
                z->out.insert(z->out.end(), z->obuf, z->obuf + n + 2);
                z->zout.size = 0;
            }
            // token.c: loop while the input is not consumed or the internal
            // state is not fully written out (in every flush mode)
        } while (in.pos < in.size || r > 0);
        z->flush_pending = token == -2;
    }
    if (token == -1) w_byte(z, kEndFlag);
    return 0;
}

}  // namespace

VS_API int vs_ztok_open(int level, vs_ztok **out) {
    if (!out) return fail(VS_ERR_ARG, "null out-pointer");
    *out = nullptr;
    const ZstdApi &Z = zstd();
    if (!Z.ok) return fail(VS_ERR_STATE, "libzstd.so.1 not loadable (rsync -z needs zstd)");
    vs_ztok *z = new vs_ztok();
    z->cctx = Z.createC();
    z->dctx = Z.createD();
    if (!z->cctx || !z->dctx || Z.isError(Z.setParam(z->cctx, kZLevelParam, level))) {
        vs_ztok_close(z);
        return fail(VS_ERR_NOMEM, "zstd contexts");
    }
    z->zout.dst = z->obuf + 2;
    z->dbuf.resize(Z.dOutSize() * 2);
    *out = z;
    return 0;
}

VS_API void vs_ztok_close(vs_ztok *z) {
    if (!z) return;
    const ZstdApi &Z = zstd();
    if (z->cctx) Z.freeC(z->cctx);
    if (z->dctx) Z.freeD(z->dctx);
    delete z;
}

VS_API int vs_rsync_write_tokens_zstd(vs_ztok *z, const vs_match *matches, int64_t n_matches,
                                      int64_t file_len, int32_t blength, int64_t basis_len,
                                      int32_t last_block_len, const uint8_t *src,
                                      const uint8_t **out, size_t *n_out) {
    if (!z || n_matches < 0 || file_len < 0 || blength <= 0 || basis_len < 0 || !out || !n_out ||
        (n_matches && !matches) || (file_len && !src))
        return fail(VS_ERR_ARG, "bad arguments");
    const int64_t count = (basis_len + blength - 1) / blength;
    for (int64_t j = 0; j < n_matches; ++j) {   // validate before any state changes
        const vs_match m = matches[j];
        if ((j && m.offset < matches[j - 1].offset) || m.block_index < 0 || m.block_index >= count)
            return fail(VS_ERR_ARG, "match list out of order or block index out of range");
    }
    z->out.clear();
    constexpr int64_t kChunk = kChunkSize;
    int64_t last = 0;
    // match.c: with sums, hash_search's rolling loop flushes a literal run
    // early (matched(offset - blength, -2)) whenever it is blength +
    // CHUNK_SIZE long and more than CHUNK_SIZE offsets remain before end; with
    // no sums, match_sums sends the file in CHUNK_SIZE pieces (-2 each)
    const bool walked = file_len > 0 && count > 0;
    const int64_t end = file_len + 1 - (count ? last_block_len : 0);
    auto gap = [&](int64_t upto) -> int {   // the -2 flushes before offset upto
        if (!walked) return 0;
        for (;;) {
            const int64_t o = last + blength + kChunk;   // the first offset with backup >= blength + CHUNK
            if (o >= upto || o >= end || end - o <= kChunk) return 0;
            VS_TRY(send_zstd_token(z, -2, src + last, (int32_t)(o - blength - last)));
            last = o - blength;
        }
    };
    for (int64_t j = 0; j < n_matches; ++j) {
        const vs_match m = matches[j];
        const int64_t bl = std::min<int64_t>(blength, basis_len - (int64_t)m.block_index * blength);
        if (m.offset < last || m.offset + bl > file_len)
            return fail(VS_ERR_ARG, "matches overlap or run past the end of the file");
        VS_TRY(gap(m.offset));
        VS_TRY(send_zstd_token(z, m.block_index, src + last, (int32_t)(m.offset - last)));
        last = m.offset + bl;
    }
    if (walked) {
        VS_TRY(gap(end));
    } else {
        for (int64_t j = last + kChunk; j < file_len; j += kChunk) {
            VS_TRY(send_zstd_token(z, -2, src + last, (int32_t)(j - last)));
            last = j;
        }
    }
    VS_TRY(send_zstd_token(z, -1, src + last, (int32_t)(file_len - last)));
    *out = z->out.data();
    *n_out = z->out.size();
    return 0;
}

VS_API int vs_rsync_read_tokens_zstd(vs_ztok *z, const uint8_t *in, size_t n, int32_t blength,
                                     int64_t basis_len, vs_match *matches, size_t cap,
                                     size_t *n_matches, uint8_t *literals, size_t lit_cap,
                                     size_t *n_literal, int64_t *file_len, size_t *consumed) {
    if (!z || !in || blength <= 0 || !n_matches || !n_literal || !file_len)
        return fail(VS_ERR_ARG, "bad arguments");
    const ZstdApi &Z = zstd();
    const int64_t count = (basis_len + blength - 1) / blength;
    size_t r = 0, nm = 0, nl = 0;
    int64_t pos = 0;
    int32_t rx_token = 0;   // recv_zstd_token r_init
    auto token = [&](int32_t t) -> int {
        if (t < 0 || t >= count) return fail(VS_ERR_ARG, "token names a block past the basis");
        if (matches) {
            if (nm >= cap) return fail(VS_ERR_ARG, "match buffer too small");
            matches[nm] = {pos, t, 0};
        }
        ++nm;
        pos += std::min<int64_t>(blength, basis_len - (int64_t)t * blength);
        return 0;
    };
    for (;;) {
        if (r >= n) return fail(VS_ERR_ARG, "truncated token stream");
        uint8_t flag = in[r++];
        if ((flag & 0xc0) == kDeflated) {
            if (r >= n) return fail(VS_ERR_ARG, "truncated DEFLATED_DATA header");
            const size_t k = ((size_t)(flag & 0x3f) << 8) + in[r++];
            if (r + k > n) return fail(VS_ERR_ARG, "truncated compressed data");
            ZIn zin{in + r, k, 0};
            r += k;
            // r_inflating until the piece is consumed and the output not full
            for (;;) {
                ZOut zo{z->dbuf.data(), z->dbuf.size(), 0};
                const size_t e = Z.decompress(z->dctx, &zo, &zin);
                if (Z.isError(e)) return fail(VS_ERR_ARG, std::string("ZSTD_decompressStream: ") + Z.errName(e));
                if (literals) {
                    if (nl + zo.pos > lit_cap) return fail(VS_ERR_ARG, "literal buffer too small");
                    memcpy(literals + nl, z->dbuf.data(), zo.pos);
                }
                nl += zo.pos;
                pos += (int64_t)zo.pos;
                if (zin.pos == zin.size && zo.pos < zo.size) break;
            }
            continue;
        }
        if (flag == kEndFlag) break;
        if (flag & kTokenRel) {
            rx_token += flag & 0x3f;
            flag >>= 6;
        } else {
            if (r + 4 > n) return fail(VS_ERR_ARG, "truncated token");
            rx_token = get_i32(in + r);
            r += 4;
        }
        VS_TRY(token(rx_token));
        if (flag & 1) {
            if (r + 2 > n) return fail(VS_ERR_ARG, "truncated run count");
            int32_t run = in[r] | (in[r + 1] << 8);
            r += 2;
            while (run-- > 0) VS_TRY(token(++rx_token));
        }
    }
    *n_matches = nm;
    *n_literal = nl;
    *file_len = pos;
    if (consumed) *consumed = r;
    return 0;
}
