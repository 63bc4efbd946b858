// rsync_api.hip -- C ABI (include/vsgpu.h, vs_rsync_*) of rsync 3.2.3 delta matching.
//
// Pipeline of vs_rsync_match_device:
//   1. device: coarse prefix sums of the source, weak scan of every offset
//      against the loaded table (filter -> directory -> entries), candidate
//      offsets radix-sorted (rsync.hip);
//   2. host: the greedy walk of match.c hash_search over the sorted
//      candidates -- sequential control only (SURVEY.md 8(e) allows host or
//      GPU for R6), every strong comparison it makes uses a strong sum the
//      device computed for that window;
//   3. verification rounds: the walk needs strong sums only for candidates it
//      visits.  Round 0 hashes "chained" candidates (another candidate one
//      block length away, the shape of runs of matching blocks) and those no
//      chained candidate in the block window before them covers (isolated
//      weak collisions in edited regions, which the walk visits); each walk
//      then treats a candidate without a strong sum as a non-match and
//      records it; the recorded windows are hashed on the device and the
//      walk repeats.  The final walk found every strong sum it needed, so it
//      made exactly rsync's decisions.
#include <chrono>
#include <cstring>
#include <vector>

#include <cstdio>
#include <cstdlib>

#include "internal.hpp"

#define VS_API extern "C" __attribute__((visibility("default")))

using namespace vsgpu;

// Page-locks a host vector's storage for the candidate read-backs (≈ 115 MB
// at C4 shape; a pageable copy goes through staging buffers at a fraction of
// the link rate).  Re-registered only when the vector's storage moves.  A
// failed registration (e.g. hipErrorHostMemoryAlreadyRegistered when a small
// vector shares a page with a registered one) is remembered for that storage,
// so it is not retried on every call: the copy just stays pageable.
struct HostReg {
    void *p = nullptr;
    size_t n = 0;
    bool registered = false;
    template <typename T>
    hipError_t cover(std::vector<T> &v) {
        const size_t bytes = v.capacity() * sizeof(T);
        if (!bytes || (v.data() == p && bytes <= n)) return hipSuccess;
        release();
        p = v.data();
        n = bytes;
        if (hipHostRegister(v.data(), bytes, hipHostRegisterDefault) == hipSuccess) {
            registered = true;
        } else {
            (void)hipGetLastError();  // not fatal; remembered until the storage moves
        }
        return hipSuccess;
    }
    // before the vector may reallocate (its old pages must not stay registered)
    template <typename T>
    void grow(std::vector<T> &v, size_t count) {
        if (count > v.capacity()) release();
        v.resize(count);
    }
    void release() {
        if (registered) (void)hipHostUnregister(p);
        registered = false;
        p = nullptr;
        n = 0;
    }
};

struct vs_rsync {
    int device = 0;
    int cus = 256;
    hipStream_t own = nullptr, stream = nullptr;
    hipEvent_t ev_null = nullptr;   // orders own-stream work after null-stream work
    // signature table
    bool loaded = false;
    int32_t count = 0, blength = 0, s2length = 0, remainder = 0;
    int csum_type = 0;
    uint32_t seed = 0;
    uint32_t dbits = 0, fbits = 0;
    std::vector<uint32_t> sum1;     // host copies for the walk
    std::vector<uint8_t> sum2;
    std::vector<uint64_t> tkey_h;   // sorted (sum1 << 32 | ~i)
    std::vector<uint32_t> dir_h;
    DevBuf d_sum1, d_keys, d_tkey, d_dir, d_filt, d_tmp;
    // scan
    DevBuf px, pt, pxs, pts, partials, c_off, c_sum, c_off2, c_sum2, n_cand, sort_tmp;
    // verification
    DevBuf v_off, v_len, v_out;
    // results
    std::vector<vs_match> matches;
    // host scratch of match_device, reused across calls
    std::vector<uint64_t> h_off, h_batch;
    std::vector<uint32_t> h_sum;
    std::vector<uint8_t> h_known, h_strong, h_flag;
    DevBuf d_flag;
    HostReg reg_off, reg_sum, reg_flag;
    std::vector<vs_match> h_out;
    int64_t st_cand = 0, st_fa = 0, st_hashed = 0;
    int32_t st_rounds = 0;
    double ms[5] = {0, 0, 0, 0, 0};
    uint64_t *pinned = nullptr;
};

namespace {

int rs_dev(vs_rsync *h) {
    if (hipSetDevice(h->device) != hipSuccess) {
        (void)hipGetLastError();
        return fail(VS_ERR_NO_DEVICE, "hipSetDevice failed");
    }
    return 0;
}

// The handle's own stream is non-blocking: an entry point that reads or
// writes caller device memory first waits for work the caller queued on the
// null stream (e.g. torch's zero-fill of the output, or the cat that built the
// table).  With vs_rsync_set_stream the caller's stream carries that order.
int order_after_null(vs_rsync *h) {
    if (h->stream != h->own) return 0;
    VS_HIP(hipEventRecord(h->ev_null, nullptr));
    VS_HIP(hipStreamWaitEvent(h->stream, h->ev_null, 0));
    return 0;
}

uint32_t ceil_log2(uint64_t x) {
    uint32_t b = 0;
    while ((1ull << b) < x) ++b;
    return b;
}

double now_ms() {
    return std::chrono::duration<double, std::milli>(
               std::chrono::steady_clock::now().time_since_epoch())
        .count();
}

// generator.c sum_sizes_sqroot, protocol >= 30 (rsync 3.2.3 <-> 3.2.3 speaks 31)
int sum_sizes(int64_t len, int32_t block_size, int32_t *bl, int32_t *s2, int32_t *cnt,
              int32_t *rem) {
    constexpr int32_t kBlock = 700, kMaxBlock = 1 << 17, kBias = 10, kSum = 16, kShort = 2;
    if (len < 0 || block_size < 0) return fail(VS_ERR_ARG, "negative length or block size");
    int32_t blength;
    if (block_size) {
        blength = block_size;
    } else if (len <= (int64_t)kBlock * kBlock) {
        blength = kBlock;
    } else {
        int32_t c = 1;
        for (int64_t l = len; l >>= 2;) c <<= 1;
        if (c >= kMaxBlock) {
            blength = kMaxBlock;
        } else {
            blength = 0;
            do {
                blength |= c;
                if (len < (int64_t)blength * blength) blength &= ~c;
                c >>= 1;
            } while (c >= 8);
            blength = std::max(blength, kBlock);
        }
    }
    int b = kBias;
    for (int64_t l = len; l >>= 1;) b += 2;
    for (int32_t c = blength; (c >>= 1) && b;) --b;
    int32_t s2length = std::min(std::max((b + 1 - 32 + 7) / 8, kShort), kSum);
    const int64_t count = len / blength + (len % blength != 0);
    if (count > INT32_MAX) return fail(VS_ERR_ARG, "block count overflows int32");
    *bl = blength;
    *s2 = s2length;
    *cnt = (int32_t)count;
    *rem = (int32_t)(len % blength);
    return 0;
}

int check_csum(int csum_type) {
    if (csum_type != VS_CSUM_MD5 && csum_type != VS_CSUM_XXH64 && csum_type != VS_CSUM_XXH3_64 &&
        csum_type != VS_CSUM_XXH3_128)
        return fail(VS_ERR_ARG, "csum_type must be VS_CSUM_MD5/XXH64/XXH3_64/XXH3_128");
    return 0;
}

// build_hash_table: device sort + directory + filter from h->d_sum1
int build_table(vs_rsync *h) {
    const uint32_t count = (uint32_t)h->count;
    h->dbits = std::min<uint32_t>(std::max<uint32_t>(ceil_log2(std::max<uint32_t>(count, 1)) + 1, 4),
                                  26);
    h->fbits = std::min<uint32_t>(std::max<uint32_t>(ceil_log2(std::max<uint32_t>(count, 1)) + 5, 10),
                                  28);
    const size_t n = std::max<uint32_t>(count, 1);
    VS_TRY(h->d_keys.ensure(n * 8));
    VS_TRY(h->d_tkey.ensure(n * 8));
    VS_TRY(h->d_dir.ensure(((1ull << h->dbits) + 1) * 4));
    VS_TRY(h->d_filt.ensure(rs_filter_bytes(h->fbits)));
    const size_t tb = rs_sort_tmp_bytes(n, false);
    VS_TRY(h->d_tmp.ensure(tb));
    VS_HIP(launch_rs_table(h->d_sum1.as<uint32_t>(), count, h->d_keys.as<uint64_t>(),
                           h->d_tkey.as<uint64_t>(), h->d_tmp.p, h->d_tmp.cap, h->dbits,
                           h->d_dir.as<uint32_t>(), h->fbits, h->d_filt.as<uint32_t>(),
                           h->stream));
    h->tkey_h.resize(count);
    h->dir_h.resize((1ull << h->dbits) + 1);
    if (count) {
        VS_HIP(hipMemcpyAsync(h->tkey_h.data(), h->d_tkey.p, (size_t)count * 8,
                              hipMemcpyDeviceToHost, h->stream));
        VS_HIP(hipMemcpyAsync(h->dir_h.data(), h->d_dir.p, h->dir_h.size() * 4,
                              hipMemcpyDeviceToHost, h->stream));
    }
    VS_HIP(hipStreamSynchronize(h->stream));
    h->loaded = true;
    return 0;
}

int load_common(vs_rsync *h, int32_t count, int32_t blength, int32_t s2length,
                int32_t remainder, int csum_type, uint32_t seed) {
    VS_TRY(check_csum(csum_type));
    if (count < 0 || blength <= 0 || s2length < 1 || s2length > 16 || remainder < 0 ||
        remainder >= blength)
        return fail(VS_ERR_ARG, "bad signature header (count, blength, s2length, remainder)");
    h->loaded = false;
    h->count = count;
    h->blength = blength;
    h->s2length = s2length;
    h->remainder = remainder;
    h->csum_type = csum_type;
    h->seed = seed;
    return 0;
}

inline int32_t blen(const vs_rsync *h, int32_t i) {
    return (i == h->count - 1 && h->remainder) ? h->remainder : h->blength;
}

// first sorted table position with sum1 == sum, or -1
inline int64_t group_start(const vs_rsync *h, uint32_t sum) {
    const uint32_t b = (uint32_t)(((uint64_t)sum) >> (32 - h->dbits));
    for (uint32_t p = h->dir_h[b], e = h->dir_h[b + 1]; p < e; ++p) {
        const uint32_t s = (uint32_t)(h->tkey_h[p] >> 32);
        if (s == sum) return p;
        if (s > sum) break;
    }
    return -1;
}

// Where a walk resumes: the walk is deterministic, and a verification round
// only adds strong sums, so everything before the first candidate whose sum
// was unknown replays identically -- the next round starts there.
struct WalkState {
    int64_t offset = 0;
    int32_t want_i = 0;
    size_t c = 0;
    size_t nout = 0;
    int64_t false_alarms = 0;
    int64_t end_false_alarms = 0;  // at the end of the (optimistic) walk
};

// After the walk's needs were hashed: did any of them strong-match a table
// entry the walk would have compared it with?  If none did, treating each as
// a non-match was exactly rsync's decision, so the walk's output stands and
// only its false-alarm count lacks their compares (`extra_fa`).
bool needs_match(vs_rsync *h, int64_t len, const std::vector<uint64_t> &off,
                 const std::vector<uint32_t> &sum, const std::vector<uint8_t> &strong,
                 const std::vector<uint64_t> &need, int64_t *extra_fa) {
    const uint32_t s2 = (uint32_t)h->s2length;
    int64_t fa = 0;
    for (const uint64_t c : need) {
        const int64_t k = std::min<int64_t>(h->blength, len - (int64_t)off[c]);
        const uint32_t s = sum[c];
        for (int64_t q = group_start(h, s); q >= 0 && q < h->count && (uint32_t)(h->tkey_h[q] >> 32) == s;
             ++q) {
            const int32_t i = (int32_t)~(uint32_t)h->tkey_h[q];
            if (blen(h, i) != k) continue;
            if (memcmp(strong.data() + c * s2, h->sum2.data() + (size_t)i * s2, s2) == 0) return true;
            ++fa;
        }
    }
    *extra_fa = fa;
    return false;
}

// match.c hash_search over the sorted candidates, from state `st`.  A
// candidate whose strong sum is unknown is treated as a non-match and
// reported in `need`; st then holds the state just before the first of them
// (else the final state).
void walk(vs_rsync *h, int64_t len, const std::vector<uint64_t> &off,
          const std::vector<uint32_t> &sum, const std::vector<uint8_t> &known,
          const std::vector<uint8_t> &strong, std::vector<uint64_t> &need,
          std::vector<vs_match> &out, WalkState &st) {
    const size_t nc = off.size();
    const uint32_t s2 = (uint32_t)h->s2length;
    const int64_t end = len + 1 - blen(h, h->count - 1);
    int64_t offset = st.offset;
    int32_t want_i = st.want_i;
    size_t c = st.c;
    int64_t false_alarms = st.false_alarms;
    out.resize(st.nout);
    bool resume_set = false;
    WalkState resume;
    while (c < nc) {
        if ((int64_t)off[c] < offset) {
            // after a match the walk jumps one block ahead, past the ~count /
            // 2^32 * blength weak collisions inside it: gallop from c (a few
            // nearby probes) instead of a binary search over the whole rest
            size_t step = 1, lo = c, hi = c + 1;
            while (hi < nc && off[hi] < (uint64_t)offset) {
                lo = hi;
                step <<= 1;
                hi = std::min(nc, hi + step);
            }
            c = std::lower_bound(off.begin() + lo, off.begin() + hi, (uint64_t)offset) - off.begin();
            continue;
        }
        const int64_t o = (int64_t)off[c];
        if (o >= end) break;
        const int64_t k = std::min<int64_t>(h->blength, len - o);
        const uint32_t s = sum[c];
        const int64_t p0 = group_start(h, s);
        bool matched = false;
        for (int64_t q = p0; q >= 0 && q < h->count && (uint32_t)(h->tkey_h[q] >> 32) == s; ++q) {
            int32_t i = (int32_t)~(uint32_t)h->tkey_h[q];
            if (blen(h, i) != k) continue;
            if (!known[c]) {
                if (!resume_set) {
                    resume = {offset, want_i, c, out.size(), false_alarms};
                    resume_set = true;
                }
                need.push_back(c);
                break;
            }
            const uint8_t *st = strong.data() + c * s2;
            if (memcmp(st, h->sum2.data() + (size_t)i * s2, s2) != 0) {
                ++false_alarms;
                continue;
            }
            if (i != want_i && want_i < h->count && s == h->sum1[want_i] &&
                memcmp(st, h->sum2.data() + (size_t)want_i * s2, s2) == 0)
                i = want_i;
            out.push_back({o, i, 0});
            want_i = i + 1;
            offset = o + blen(h, i);
            matched = true;
            break;
        }
        if (!matched) {
            offset = o + 1;
            ++c;
        }
    }
    st = resume_set ? resume : WalkState{offset, want_i, c, out.size(), false_alarms};
    st.end_false_alarms = false_alarms;
}

// strong sums of candidate windows idx[] on the device -> strong/known
int verify(vs_rsync *h, const void *dev_src, int64_t len, const std::vector<uint64_t> &off,
           const std::vector<uint64_t> &idx, std::vector<uint8_t> &known,
           std::vector<uint8_t> &strong) {
    const size_t n = idx.size();
    if (!n) return 0;
    const uint32_t s2 = (uint32_t)h->s2length;
    std::vector<uint64_t> vo(n);
    std::vector<uint32_t> vl(n);
    uint32_t min_len = 0xffffffffu;
    for (size_t j = 0; j < n; ++j) {
        vo[j] = off[idx[j]];
        vl[j] = (uint32_t)std::min<int64_t>(h->blength, len - (int64_t)vo[j]);
        min_len = std::min(min_len, vl[j]);
    }
    VS_TRY(h->v_off.ensure(n * 8));
    VS_TRY(h->v_len.ensure(n * 4));
    VS_TRY(h->v_out.ensure(n * s2));
    VS_HIP(hipMemcpyAsync(h->v_off.p, vo.data(), n * 8, hipMemcpyHostToDevice, h->stream));
    VS_HIP(hipMemcpyAsync(h->v_len.p, vl.data(), n * 4, hipMemcpyHostToDevice, h->stream));
    VS_HIP(launch_rs_strong((const uint8_t *)dev_src, h->v_off.as<uint64_t>(),
                            h->v_len.as<uint32_t>(), n, h->csum_type, h->seed, s2,
                            h->v_out.as<uint8_t>(), min_len, h->stream));
    std::vector<uint8_t> res(n * s2);
    VS_HIP(hipMemcpyAsync(res.data(), h->v_out.p, n * s2, hipMemcpyDeviceToHost, h->stream));
    VS_HIP(hipStreamSynchronize(h->stream));
    for (size_t j = 0; j < n; ++j) {
        memcpy(strong.data() + idx[j] * s2, res.data() + j * s2, s2);
        known[idx[j]] = 1;
    }
    h->st_hashed += (int64_t)n;
    return 0;
}

int match_device(vs_rsync *h, const void *dev_src, int64_t len, int64_t *n_matches) {
    if (!h->loaded) return fail(VS_ERR_STATE, "vs_rsync_match_device before vs_rsync_load_sums");
    if (len < 0 || (len && !dev_src)) return fail(VS_ERR_ARG, "bad source");
    VS_TRY(rs_dev(h));
    h->matches.clear();
    h->st_cand = h->st_fa = h->st_hashed = 0;
    h->st_rounds = 0;
    for (int i = 2; i < 5; ++i) h->ms[i] = 0;
    if (n_matches) *n_matches = 0;
    if (len == 0 || h->count == 0) return 0;  // match_sums: no sums -> all literal
    const double t0 = now_ms();
    VS_TRY(order_after_null(h));
    // 1. coarse prefixes
    const uint64_t nblk = ((uint64_t)len + kRsG - 1) / kRsG;
    VS_TRY(h->px.ensure(nblk * 4));
    VS_TRY(h->pt.ensure(nblk * 4));
    VS_TRY(h->pxs.ensure((nblk + 1) * 4));
    VS_TRY(h->pts.ensure((nblk + 1) * 4));
    VS_TRY(h->partials.ensure((nblk / 4096 + 2) * 4));
    VS_TRY(h->n_cand.ensure(16));
    VS_HIP(launch_rs_prefix((const uint8_t *)dev_src, (uint64_t)len, h->px.as<uint32_t>(),
                            h->pt.as<uint32_t>(), h->pxs.as<uint32_t>(), h->pts.as<uint32_t>(),
                            h->partials.as<uint32_t>(), h->stream));
    static const bool trace = getenv("VSGPU_RS_TRACE") != nullptr;
    if (trace) {
        VS_HIP(hipStreamSynchronize(h->stream));
        fprintf(stderr, "rs: prefix %.1f ms\n", now_ms() - t0);
    }
    // 2. weak scan (re-run once with an exact capacity on overflow)
    RsScanArgs a{};
    a.data = (const uint8_t *)dev_src;
    a.len = (uint64_t)len;
    a.blength = (uint64_t)h->blength;
    a.nfull = (a.len >= a.blength) ? a.len - a.blength + 1 : 0;
    a.count = (uint32_t)h->count;
    a.remainder = (uint32_t)h->remainder;
    a.px_scan = h->pxs.as<uint32_t>();
    a.pt_scan = h->pts.as<uint32_t>();
    a.tkey = h->d_tkey.as<uint64_t>();
    a.dir = h->d_dir.as<uint32_t>();
    a.filt = h->d_filt.as<uint32_t>();
    a.dbits = h->dbits;
    a.fbits = h->fbits;
    a.lbits = rs_lds_filter_bits(h->fbits);
    a.filt_l = h->d_filt.as<uint32_t>() + ((1ull << h->fbits) / 32);
    a.n_cand = (unsigned long long *)h->n_cand.p;
    // expected: weak collisions (count / 2^32 per offset) + one per matching block
    uint64_t cap = (uint64_t)((double)a.nfull * h->count / 4294967296.0 * 2.0) +
                   (uint64_t)len / h->blength * 2 + 65536;
    uint64_t nc = 0;
    for (int attempt = 0; attempt < 2; ++attempt) {
        VS_TRY(h->c_off.ensure(cap * 8));
        VS_TRY(h->c_sum.ensure(cap * 4));
        a.cap = cap;
        a.cand_off = h->c_off.as<uint64_t>();
        a.cand_sum = h->c_sum.as<uint32_t>();
        VS_HIP(hipMemsetAsync(h->n_cand.p, 0, 8, h->stream));
        VS_HIP(launch_rs_scan(a, h->cus, h->stream));
        VS_HIP(hipMemcpyAsync(h->pinned, h->n_cand.p, 8, hipMemcpyDeviceToHost, h->stream));
        VS_HIP(hipStreamSynchronize(h->stream));
        nc = h->pinned[0];
        if (trace) fprintf(stderr, "rs: scan done %.1f ms (%llu candidates)\n", now_ms() - t0,
                           (unsigned long long)nc);
        if (nc <= cap) break;
        cap = nc;
        if (attempt == 1) return fail(VS_ERR_STATE, "candidate buffer overflow");
    }
    // 3. sort candidates by offset
    // host scratch kept in the handle: first-touch page faults on ~160 MB of
    // fresh vectors per call (C4 shape) cost ~100 ms
    std::vector<uint64_t> &off = h->h_off;
    std::vector<uint32_t> &sum = h->h_sum;
    h->reg_off.grow(off, nc);
    h->reg_sum.grow(sum, nc);
    if (nc) {
        VS_TRY(h->c_off2.ensure(nc * 8));
        VS_TRY(h->c_sum2.ensure(nc * 4));
        VS_TRY(h->sort_tmp.ensure(rs_sort_tmp_bytes(nc, true)));
        const int end_bit = (int)std::max<uint32_t>(ceil_log2((uint64_t)len + 1), 1);
        VS_HIP(launch_rs_sort_cands(h->sort_tmp.p, h->sort_tmp.cap, h->c_off.as<uint64_t>(),
                                    h->c_off2.as<uint64_t>(), h->c_sum.as<uint32_t>(),
                                    h->c_sum2.as<uint32_t>(), nc, end_bit, h->stream));
        VS_HIP(h->reg_off.cover(off));
        VS_HIP(h->reg_sum.cover(sum));
        VS_HIP(hipMemcpyAsync(off.data(), h->c_off2.p, nc * 8, hipMemcpyDeviceToHost, h->stream));
        VS_HIP(hipMemcpyAsync(sum.data(), h->c_sum2.p, nc * 4, hipMemcpyDeviceToHost, h->stream));
        VS_HIP(hipStreamSynchronize(h->stream));
    }
    h->st_cand = (int64_t)nc;
    const double t1 = now_ms();
    if (trace) fprintf(stderr, "rs: sorted + copied %.1f ms\n", t1 - t0);
    h->ms[2] = t1 - t0;
    // 4. round 0: chained candidates (another candidate one block length
    // away) plus the uncovered ones (see rs_visit_kernel)
    std::vector<uint8_t> &known = h->h_known, &strong = h->h_strong;
    known.assign(nc, 0);
    strong.resize(nc * (size_t)h->s2length);
    std::vector<uint64_t> &batch = h->h_batch;
    batch.clear();
    if (nc) {
        // flags computed on the device over the sorted offsets (binary
        // searches for o - blength and o + blength); the host loop over
        // 8.9 M candidates took ~100 ms at C4 shape
        VS_TRY(h->d_flag.ensure(2 * nc));
        VS_HIP(launch_rs_chained(h->c_off2.as<uint64_t>(), nc, (uint64_t)h->blength,
                                 h->d_flag.as<uint8_t>(), h->stream));
        h->reg_flag.grow(h->h_flag, nc);
        VS_HIP(h->reg_flag.cover(h->h_flag));
        VS_HIP(hipMemcpyAsync(h->h_flag.data(), h->d_flag.as<uint8_t>() + nc, nc,
                              hipMemcpyDeviceToHost, h->stream));
        VS_HIP(hipStreamSynchronize(h->stream));
        const uint8_t *fl = h->h_flag.data();
        for (size_t c = 0; c < nc; ++c)
            if (fl[c]) batch.push_back(c);
    }
    if (trace) fprintf(stderr, "rs: chained batch %.1f ms (%zu)\n", now_ms() - t0, batch.size());
    double t_ver = 0, t_walk = 0;
    std::vector<vs_match> &out = h->h_out;
    out.clear();
    WalkState ws;
    for (;;) {
        double tv = now_ms();
        VS_TRY(verify(h, dev_src, len, off, batch, known, strong));
        t_ver += now_ms() - tv;
        ++h->st_rounds;
        double tw = now_ms();
        int64_t extra_fa = 0;
        if (h->st_rounds > 1 && !needs_match(h, len, off, sum, strong, batch, &extra_fa)) {
            // every need was a false alarm: no replay (out holds the whole walk)
            ws.false_alarms = ws.end_false_alarms + extra_fa;
            t_walk += now_ms() - tw;
            break;
        }
        batch.clear();
        walk(h, len, off, sum, known, strong, batch, out, ws);
        t_walk += now_ms() - tw;
        if (trace && !batch.empty()) {
            const uint64_t b0 = batch[0];
            fprintf(stderr,
                    "rs: round %d needs %zu (resume c=%zu of %llu, offset %lld; first need "
                    "c=%llu off=%llu chained=%d)\n",
                    h->st_rounds, batch.size(), ws.c, (unsigned long long)nc,
                    (long long)ws.offset, (unsigned long long)b0,
                    (unsigned long long)off[b0], (int)h->h_flag[b0]);
        }
        if (batch.empty()) break;
    }
    h->ms[3] = t_ver;
    h->ms[4] = t_walk;
    if (trace) fprintf(stderr, "rs: match done %.1f ms (verify %.1f, walk %.1f)\n", now_ms() - t0,
                       t_ver, t_walk);
    h->st_fa = ws.false_alarms;
    h->matches.assign(out.begin(), out.end());
    if (n_matches) *n_matches = (int64_t)h->matches.size();
    return 0;
}

}  // namespace

VS_API int vs_rsync_sizes(int64_t len, int32_t block_size, int32_t *blength, int32_t *s2length,
                          int32_t *count, int32_t *remainder) {
    if (!blength || !s2length || !count || !remainder) return fail(VS_ERR_ARG, "null output");
    return sum_sizes(len, block_size, blength, s2length, count, remainder);
}

VS_API int vs_rsync_open(int device, vs_rsync **out) {
    if (!out) return fail(VS_ERR_ARG, "null handle out-pointer");
    *out = nullptr;
    const int ndev = vs_device_count();
    if (ndev <= 0) return fail(VS_ERR_NO_DEVICE, "no HIP device available (no CPU fallback)");
    if (device < 0 || device >= ndev) return fail(VS_ERR_ARG, "device index out of range");
    vs_rsync *h = new vs_rsync();
    h->device = device;
    (void)hipDeviceGetAttribute(&h->cus, hipDeviceAttributeMultiprocessorCount, device);
    if (rs_dev(h) < 0 || hipStreamCreateWithFlags(&h->own, hipStreamNonBlocking) != hipSuccess ||
        hipEventCreateWithFlags(&h->ev_null, hipEventDisableTiming) != hipSuccess ||
        hipHostMalloc((void **)&h->pinned, 64, hipHostMallocDefault) != hipSuccess) {
        (void)hipGetLastError();
        vs_rsync_close(h);
        return fail(VS_ERR_HIP, "stream / pinned buffer creation failed");
    }
    h->stream = h->own;
    *out = h;
    return 0;
}

VS_API int vs_rsync_set_stream(vs_rsync *h, void *hip_stream) {
    if (!h) return fail(VS_ERR_ARG, "null handle");
    h->stream = hip_stream ? (hipStream_t)hip_stream : h->own;
    return 0;
}

VS_API void vs_rsync_close(vs_rsync *h) {
    if (!h) return;
    (void)hipSetDevice(h->device);
    if (h->stream) (void)hipStreamSynchronize(h->stream);
    for (DevBuf *b : {&h->d_sum1, &h->d_keys, &h->d_tkey, &h->d_dir, &h->d_filt, &h->d_tmp, &h->px,
                      &h->pt, &h->pxs, &h->pts, &h->partials, &h->c_off, &h->c_sum, &h->c_off2,
                      &h->c_sum2, &h->n_cand, &h->sort_tmp, &h->v_off, &h->v_len, &h->v_out,
                      &h->d_flag})
        b->release();
    if (h->pinned) (void)hipHostFree(h->pinned);
    for (HostReg *r : {&h->reg_off, &h->reg_sum, &h->reg_flag}) r->release();
    if (h->ev_null) (void)hipEventDestroy(h->ev_null);
    if (h->own) (void)hipStreamDestroy(h->own);
    delete h;
}

VS_API int vs_rsync_signatures_device(vs_rsync *h, const void *dev_basis, int64_t len,
                                      int32_t blength, int32_t s2length, int csum_type,
                                      uint32_t seed, uint32_t *dev_sum1, uint8_t *dev_sum2) {
    if (!h) return fail(VS_ERR_ARG, "null handle");
    VS_TRY(check_csum(csum_type));
    if (len < 0 || blength <= 0 || s2length < 1 || s2length > 16)
        return fail(VS_ERR_ARG, "bad length, blength or s2length");
    const int64_t count = len / blength + (len % blength != 0);
    if (count && (!dev_basis || !dev_sum1 || !dev_sum2)) return fail(VS_ERR_ARG, "null device pointer");
    VS_TRY(rs_dev(h));
    RsSigArgs a{};
    a.data = (const uint8_t *)dev_basis;
    a.len = (uint64_t)len;
    a.count = (uint64_t)count;
    a.blength = (uint32_t)blength;
    a.remainder = (uint32_t)(len % blength);
    a.s2length = (uint32_t)s2length;
    a.csum_type = csum_type;
    a.seed = seed;
    a.sum1 = dev_sum1;
    a.sum2 = dev_sum2;
    const double t0 = now_ms();
    VS_TRY(order_after_null(h));
    VS_HIP(launch_rs_signatures(a, h->stream));
    VS_HIP(hipStreamSynchronize(h->stream));
    h->ms[0] = now_ms() - t0;
    return 0;
}

VS_API int vs_rsync_load_sums(vs_rsync *h, int32_t count, int32_t blength, int32_t s2length,
                              int32_t remainder, const uint32_t *sum1, const uint8_t *sum2,
                              int csum_type, uint32_t seed) {
    if (!h) return fail(VS_ERR_ARG, "null handle");
    VS_TRY(load_common(h, count, blength, s2length, remainder, csum_type, seed));
    if (count && (!sum1 || !sum2)) return fail(VS_ERR_ARG, "null sum arrays");
    VS_TRY(rs_dev(h));
    const double t0 = now_ms();
    h->sum1.assign(sum1, sum1 + count);
    h->sum2.assign(sum2, sum2 + (size_t)count * s2length);
    VS_TRY(h->d_sum1.ensure((size_t)std::max(count, 1) * 4));
    if (count)
        VS_HIP(hipMemcpyAsync(h->d_sum1.p, sum1, (size_t)count * 4, hipMemcpyHostToDevice,
                              h->stream));
    VS_TRY(build_table(h));
    h->ms[1] = now_ms() - t0;
    return 0;
}

VS_API int vs_rsync_load_sums_device(vs_rsync *h, int32_t count, int32_t blength,
                                     int32_t s2length, int32_t remainder,
                                     const uint32_t *dev_sum1, const uint8_t *dev_sum2,
                                     int csum_type, uint32_t seed) {
    if (!h) return fail(VS_ERR_ARG, "null handle");
    VS_TRY(load_common(h, count, blength, s2length, remainder, csum_type, seed));
    if (count && (!dev_sum1 || !dev_sum2)) return fail(VS_ERR_ARG, "null sum arrays");
    VS_TRY(rs_dev(h));
    const double t0 = now_ms();
    h->sum1.resize(count);
    h->sum2.resize((size_t)count * s2length);
    VS_TRY(h->d_sum1.ensure((size_t)std::max(count, 1) * 4));
    VS_TRY(order_after_null(h));
    if (count) {
        VS_HIP(hipMemcpyAsync(h->d_sum1.p, dev_sum1, (size_t)count * 4, hipMemcpyDeviceToDevice,
                              h->stream));
        VS_HIP(hipMemcpyAsync(h->sum1.data(), dev_sum1, (size_t)count * 4,
                              hipMemcpyDeviceToHost, h->stream));
        VS_HIP(hipMemcpyAsync(h->sum2.data(), dev_sum2, h->sum2.size(), hipMemcpyDeviceToHost,
                              h->stream));
    }
    VS_TRY(build_table(h));
    h->ms[1] = now_ms() - t0;
    return 0;
}

VS_API int vs_rsync_match_device(vs_rsync *h, const void *dev_src, int64_t len,
                                 int64_t *n_matches) {
    if (!h) return fail(VS_ERR_ARG, "null handle");
    return match_device(h, dev_src, len, n_matches);
}

VS_API int vs_rsync_get_matches(vs_rsync *h, int64_t first, int64_t n, vs_match *out) {
    if (!h) return fail(VS_ERR_ARG, "null handle");
    if (first < 0 || n < 0 || first + n > (int64_t)h->matches.size())
        return fail(VS_ERR_ARG, "match range out of bounds");
    if (n && !out) return fail(VS_ERR_ARG, "null output");
    if (n) memcpy(out, h->matches.data() + first, (size_t)n * sizeof(vs_match));
    return 0;
}

VS_API int vs_rsync_stats(vs_rsync *h, int64_t *candidates, int64_t *false_alarms,
                          int64_t *strong_hashed, int32_t *rounds) {
    if (!h) return fail(VS_ERR_ARG, "null handle");
    if (candidates) *candidates = h->st_cand;
    if (false_alarms) *false_alarms = h->st_fa;
    if (strong_hashed) *strong_hashed = h->st_hashed;
    if (rounds) *rounds = h->st_rounds;
    return 0;
}

VS_API int vs_rsync_timing(vs_rsync *h, double ms_out[5]) {
    if (!h || !ms_out) return fail(VS_ERR_ARG, "null argument");
    for (int i = 0; i < 5; ++i) ms_out[i] = h->ms[i];
    return 0;
}

VS_API int vs_rsync_signatures(int device, const void *basis, int64_t len, int32_t blength,
                               int32_t s2length, int csum_type, uint32_t seed, uint32_t *sum1,
                               uint8_t *sum2) {
    if (len < 0 || (len && !basis) || blength <= 0) return fail(VS_ERR_ARG, "bad basis");
    const int64_t count = len / blength + (len % blength != 0);
    if (count && (!sum1 || !sum2)) return fail(VS_ERR_ARG, "null outputs");
    vs_rsync *h = nullptr;
    VS_TRY(vs_rsync_open(device, &h));
    DevBuf d, s1, s2;
    int r = 0;
    if ((r = d.ensure((size_t)std::max<int64_t>(len, 16))) < 0 ||
        (r = s1.ensure((size_t)std::max<int64_t>(count, 1) * 4)) < 0 ||
        (r = s2.ensure((size_t)std::max<int64_t>(count, 1) * s2length)) < 0) {
        vs_rsync_close(h);
        return r;
    }
    if (len && hipMemcpy(d.p, basis, (size_t)len, hipMemcpyHostToDevice) != hipSuccess)
        r = fail(VS_ERR_HIP, "basis upload failed");
    if (!r)
        r = vs_rsync_signatures_device(h, d.p, len, blength, s2length, csum_type, seed,
                                       s1.as<uint32_t>(), s2.as<uint8_t>());
    if (!r && count &&
        (hipMemcpy(sum1, s1.p, (size_t)count * 4, hipMemcpyDeviceToHost) != hipSuccess ||
         hipMemcpy(sum2, s2.p, (size_t)count * s2length, hipMemcpyDeviceToHost) != hipSuccess))
        r = fail(VS_ERR_HIP, "signature download failed");
    d.release();
    s1.release();
    s2.release();
    vs_rsync_close(h);
    return r;
}

VS_API int vs_rsync_match(int device, const void *src, int64_t len, const vs_sigtable *t,
                          int csum_type, uint32_t seed, vs_match *out, size_t cap,
                          size_t *n_out) {
    if (!t || !n_out) return fail(VS_ERR_ARG, "null argument");
    if (len < 0 || (len && !src)) return fail(VS_ERR_ARG, "bad source");
    vs_rsync *h = nullptr;
    VS_TRY(vs_rsync_open(device, &h));
    int r = vs_rsync_load_sums(h, t->count, t->blength, t->s2length, t->remainder, t->sum1,
                               t->sum2, csum_type, seed);
    DevBuf d;
    int64_t nm = 0;
    if (!r) r = d.ensure((size_t)std::max<int64_t>(len, 16));
    if (!r && len && hipMemcpy(d.p, src, (size_t)len, hipMemcpyHostToDevice) != hipSuccess)
        r = fail(VS_ERR_HIP, "source upload failed");
    if (!r) r = vs_rsync_match_device(h, d.p, len, &nm);
    if (!r) {
        *n_out = (size_t)nm;
        if ((size_t)nm > cap)
            r = fail(VS_ERR_ARG, "output capacity too small (need " + std::to_string(nm) + ")");
        else
            r = vs_rsync_get_matches(h, 0, nm, out);
    }
    d.release();
    vs_rsync_close(h);
    return r;
}
