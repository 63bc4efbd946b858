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
#include <condition_variable>
#include <cstring>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include <cstdio>
#include <cstdlib>

#include "internal.hpp"

#define VS_API extern "C" __attribute__((visibility("default")))

using namespace vsgpu;

// One sharded match run (vs_rsync_match_scan .. _finish).  Offsets in spec /
// fin are data-relative (file offset - origin).
struct RsRun {
    const uint8_t *dev = nullptr;  // device bytes at file offset `origin`
    int64_t dlen = 0, origin = 0, flen = 0, own_lo = 0, own_hi = 0;
    int64_t spec_entry = 0;
    int32_t spec_want = 0;
    std::vector<vs_match> spec;          // the speculative walk's matches
    std::vector<int64_t> spec_fa_before; // false alarms before each match's offset
    int64_t spec_fa = 0, spec_exit = 0;
    int32_t spec_exit_want = 0;
    std::vector<vs_match> fin;           // the walk from the true entry (use_spec: = spec)
    bool use_spec = true;
    int64_t fin_fa = 0, fin_exit = 0;
    int32_t fin_exit_want = 0;
    int state = 0;                       // 0 none, 1 scanned, 2 stitched, 3 finished
    // device-walk path (rsync_walk.hip): segments of the owned range, the
    // current stitched exit, and the walk's continuation past the last full
    // window (the short last block's one window, checked on the host)
    bool dev_walk = false;
    RsWalkArgs wa{};
    int xcur = 0;                        // which exit buffer holds the current exits
    std::vector<vs_match> tail;          // at most one match
    int64_t tail_fa = 0;
};

// One whole-file checksum in flight (R7).  XXH3 of a long
// file, rows first (round 5): one kernel computes every 1 KiB block's
// contribution row (64 B) into a device buffer of len / 16 bytes as soon as
// the job starts -- before the caller's walk takes the CUs -- and the rows
// come back on an SDMA engine (DmaD2H; a HIP copy in a PyTorch process is a
// blit kernel, which waits for CUs the persistent walk holds) into a pinned
// buffer of the same size, all of its chunks queued at once so that the
// engine serves jobs in order at its full rate, chained on a host thread as
// each chunk lands.  Without the DMA path,
// or for files whose rows exceed kRowsCap, contributions are computed one
// piece at a time into a 3-deep device ring instead.  MD5, XXH64 and XXH3 of
// <= 240 bytes are serial chains: the file's bytes come back through the same
// pinned ring and are hashed on the host thread.
struct FsJob {
    static constexpr uint64_t kRowsCap = 8ull << 30;   // rows of a 128 GiB file
    // pinned row copies per handle: three 64 GiB files in
    // flight fit; a job that would pass it takes the piece ring
    static constexpr uint64_t kPinnedRowsCap = 16ull << 30;
    DmaD2H dma;
    DevBuf rows;                          // rows-first: every block's row
    uint8_t *hrows = nullptr;             // rows-first: their pinned copy
    uint64_t hrows_cap = 0;
    static constexpr int kChunks = 16;    // rows-first read-back: copies queued per job
    bool rows_first = false;
    static constexpr int kRing = 3;
    uint64_t piece = 1ull << 18;          // blocks per piece (16 MiB of rows; serial: of bytes)
    hipStream_t s = nullptr;
    hipEvent_t ev[kRing] = {}, ev_in = nullptr, kev[kRing][2] = {};
    uint8_t *hC[kRing] = {};              // pinned ring (piece * 64 bytes each)
    uint8_t *hlast = nullptr;             // pinned: the file's last <= 1088 bytes
    DevBuf dC;                            // device ring of contribution rows
    const uint8_t *src = nullptr;
    std::thread th;
    bool active = false, whole = false, serial = false;
    int device = 0, csum = 0, rc = 0;
    std::string err;
    uint64_t len = 0, nb = 0;
    uint64_t acc[8] = {};
    uint8_t digest[16] = {};
    double host_ms = 0, dev_ms = 0;
    double t_call = 0;   // fs_start (VS_FS_TRACE builds report the job's timeline)
};

// ---- streamed forms: a file fed from host memory in order -------------------
// The sender's source (match_sums) and the generator's basis
// (generate_and_send_sums) reach rsync through map_ptr's sliding window, one
// read at a time: the library receives them piece by piece and keeps only a
// small ring of pieces on the device, so a file may be far larger than HBM.
//
// MatchStream: piece k owns the walk's visits to [k P, (k+1) P) and needs its
// bytes plus a blength - 1 halo (the first bytes of piece k+1, copied on the
// device when they arrive).  The walk is sequential, so each piece is walked
// from its TRUE entry -- the previous piece's exit -- with no speculation
// between pieces; inside a piece the segment walk of DESIGN.md 3.4 runs as
// usual.  Pieces are walked by a library thread while the caller feeds the
// next ones: the H2D copies (copy stream) overlap the walks (handle stream).
struct MatchStream {
    static constexpr uint32_t kMaxRing = 8;
    int64_t flen = 0, piece = 0, halo = 0, np = 0;
    uint32_t ring = 0;
    vsgpu::DevBuf slot[kMaxRing];
    hipEvent_t ev[kMaxRing] = {};     // piece k's bytes and halo are on the device
    hipStream_t cs = nullptr;          // copies of fed bytes
    vsgpu::Stager stage;               // pageable feeds (the walk thread uses the handle's)
    int64_t fed = 0, queued = 0;       // bytes received; pieces whose bytes are all queued
    uint64_t pinned_bytes = 0, staged_bytes = 0;
    double feed_wait_ms = 0;           // caller time waiting for a free slot
    std::thread th;
    std::mutex mu;
    std::condition_variable cv;
    int64_t complete = 0, walked = 0;  // (under mu) pieces queued / walked
    bool stop = false;
    int rc = 0;
    std::string err;
    std::vector<vs_match> out;         // (under mu) matches found, [head, size) not yet returned
    size_t head = 0;
    int64_t fa = 0, hashed = 0;        // (under mu)
    double walk_ms = 0, idle_ms = 0;   // (under mu) worker time walking / waiting for bytes
    // R7 as the file passes (file_csum != 0): XXH3 of a long file from each
    // piece's block contributions on the device, chained by the walk thread;
    // MD5 / XXH64 / short XXH3 on the host from the fed bytes; the file's
    // last <= 1088 bytes kept for the XXH3 finish
    int fcsum = 0;
    bool fs_xxh3 = false;
    uint64_t acc[8] = {};
    vsgpu::SerialSum ss{};
    vsgpu::DevBuf dC;
    uint64_t *hC = nullptr;            // pinned: one piece's contribution rows
    uint8_t last[1088] = {};
    double fs_ms = 0;                  // (under mu) walk-thread contributions + chain
};

// SigStream: pieces are whole blocks; each is signed as soon as its bytes are
// on the device, and the sums are read back into pinned host arrays in block
// order for vs_rsync_sig_next.
struct SigStream {
    static constexpr uint32_t kMaxRing = 8;
    int64_t len = 0, piece = 0, count = 0, np = 0;
    int32_t blength = 0, s2length = 0, remainder = 0;
    int csum = 0;
    uint32_t seed = 0, ring = 0;
    vsgpu::DevBuf slot[kMaxRing], d1, d2;
    hipEvent_t ev_in[kMaxRing] = {}, ev_done[kMaxRing] = {};
    hipStream_t cs = nullptr;
    vsgpu::Stager stage;
    uint32_t *h1 = nullptr;            // pinned [count]
    uint8_t *h2 = nullptr;             // pinned [count * s2length]
    int64_t fed = 0, launched = 0, done = 0;   // bytes; pieces signed; pieces read back
    int64_t returned = 0;              // blocks handed to the caller
    uint64_t pinned_bytes = 0, staged_bytes = 0;
};

struct vs_rsync {
    int device = 0;
    int cus = 256;
    hipStream_t own = nullptr, stream = nullptr;
    hipEvent_t ev_null = nullptr;   // orders own-stream work after null-stream work
    // device time of the kernels themselves (HIP events on h->stream around
    // each launch; every entry point synchronises right after): [0] weak scan
    // / device walk, [1] strong verification, [2] signatures
    hipEvent_t kev[2] = {nullptr, nullptr};
    double kms[5] = {0, 0, 0, 0, 0};
    int64_t kn[5] = {0, 0, 0, 0, 0};
    // signature table
    bool loaded = false;
    int32_t count = 0, blength = 0, s2length = 0, remainder = 0;
    int csum_type = 0;
    uint32_t seed = 0;
    uint32_t dbits = 0, fbits = 0, bbits = 0;
    // host copies for the host walk and the short-last-block tail, fetched
    // from the device table only when one of them runs (host_tables)
    bool host_ok = false;
    std::vector<uint32_t> sum1;
    std::vector<uint8_t> sum2;
    std::vector<uint64_t> tkey_h;   // sorted (sum1 << 32 | ~i)
    std::vector<uint32_t> dir_h;
    DevBuf d_sum1, d_keys, d_tkey, d_dir, d_filt, d_tmp, d_bkt;
    DevBuf d_sum2p, d_sum2tmp;      // zero-padded 16-byte strong sums (device walk)
    // device walk: per-segment results and two exit buffers
    DevBuf w_spec_off, w_spec_idx, w_spec_fab, w_spec_n, w_spec_fa, w_spec_exit, w_spec_exitw;
    DevBuf w_spec_fao, w_spec_fac, w_spec_nfa;
    DevBuf w_fin_entry, w_fin_entryw, w_fin_from, w_fin_n, w_fin_fa, w_fin_off, w_fin_idx,
        w_fin_fab;
    DevBuf w_exit[2], w_exitw[2], w_ctl, w_prof;
    // whole-file checksums in flight, FIFO: a file's chain may overlap the
    // next file's walk (and the next file's chain, on another host thread)
    static constexpr uint32_t kFsJobs = 4;
    FsJob fs[kFsJobs];
    uint32_t fs_head = 0, fs_tail = 0;   // jobs [head, tail) are in flight
    FsJob fs_sync;                       // the blocking vs_rsync_file_sum's own job
    // pinned row copies not held by a job (rows first): a job
    // takes one at its start and returns it once waited for, so the pinned
    // bytes follow the jobs in flight, at most FsJob::kPinnedRowsCap in all
    std::vector<std::pair<uint8_t *, uint64_t>> fs_pool;
    uint64_t fs_pinned = 0;              // bytes pinned for row copies (pool + jobs)
    double fs_dev_ms = 0, fs_host_ms = 0; // the last job waited for
    DevBuf rc_pieces;               // receiver reconstruction
    // scan
    DevBuf px, pt, pxs, pts, partials, c_off, c_sum, c_off2, c_sum2, n_cand, sort_tmp;
    // verification
    DevBuf v_off, v_len, v_out;
    // results
    std::vector<vs_match> matches;
    // host scratch of match_device, reused across calls
    // candidate read-backs (~115 MB at C4 shape): owned pinned pages, written
    // by the DMA engine directly (xfer.cpp: never register heap storage)
    PinnedVec<uint64_t> h_off;
    PinnedVec<uint32_t> h_sum;
    PinnedVec<uint8_t> h_flag;
    std::vector<uint64_t> h_batch;
    std::vector<uint8_t> h_known, h_strong;
    DevBuf d_flag;
    Stager stage;                   // copies of caller / heap host memory
    std::vector<vs_match> h_out;
    RsRun run;
    int64_t st_cand = 0, st_fa = 0, st_hashed = 0;
    int32_t st_rounds = 0;
    // options (vs_rsync_set_option; tests and measurement)
    uint32_t seg_blocks = 0;        // walk segment length in blocks (0: automatic)
    uint32_t opt_bbits = 0;         // membership bucket bits (0: automatic)
    int32_t opt_facap = -1;         // false-alarm windows recorded per segment (-1: automatic)
    bool opt_host_walk = false;     // the host walk for every checksum type
    bool opt_prefilter = true;      // the walk's LDS prefilter
    uint32_t opt_flushq = 0;        // STEP hits per flush (4: rows only; 16 or 0: wide passes)
    uint32_t opt_flushspan = 0;     // flush once the scan is this far past the first hit (0: none)
    bool opt_flushpredict = true;   // flush at a likely resync hit (weak sum of block want .. want + 2)
    int32_t opt_tailpct = -1;       // % of the walk range in quarter-length tail segments (-1: automatic)
    int64_t opt_seg_margin = -1;    // walk segments start this far before a block boundary (-1: automatic)
    uint64_t fs_piece = 0;          // file-sum piece in 1 KiB blocks (0: 2^18)
    // streamed forms (host-fed files): see the MatchStream / SigStream section
    MatchStream *mst = nullptr;
    SigStream *sst = nullptr;
    double ms[5] = {0, 0, 0, 0, 0};
    uint64_t *pinned = nullptr;
    // device walk's compacted match list (walk_collect)
    DevBuf wc_cnt, wc_pos, wc_part, wc_out;
    vs_match *wc_host = nullptr;    // pinned read-back
    size_t wc_host_cap = 0;
};

namespace {

int rs_dev(vs_rsync *h) { return enter_device(h->device); }

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

// brackets one kernel launch with the handle's two timing events; fold()
// after the stream synchronised adds the elapsed time to kms[which]
struct KernelTimer {
    vs_rsync *h;
    int which;
    bool on = false;
    KernelTimer(vs_rsync *h_, int w) : h(h_), which(w) {
        on = h->kev[0] && hipEventRecord(h->kev[0], h->stream) == hipSuccess;
    }
    void stop() {
        if (on) on = hipEventRecord(h->kev[1], h->stream) == hipSuccess;
    }
    void fold() {  // call after hipStreamSynchronize(h->stream)
        float ms = 0;
        if (on && hipEventElapsedTime(&ms, h->kev[0], h->kev[1]) == hipSuccess) {
            h->kms[which] += ms;
            h->kn[which] += 1;
        }
        on = false;
    }
};

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
    // Filter size: 32 bits per key, capped at 2^25 bits (4 MiB, one XCD's L2)
    // so the walk's gathers stay L2-resident.  At C4's 2 M blocks the cap
    // (16 bits per key) measured 745 -> 775-787 GB/s per rank; at 524 K
    // blocks 32 and 16 bits per key are within 1 % and 8 bits per key loses
    // 5 % (profiles/r02_walk_ab).
    const uint32_t lc = ceil_log2(std::max<uint32_t>(count, 1));
#ifndef VS_FBITS_CAP
// 2 MiB: half of one XCD's L2, so the walk's filter gathers stay in it beside
// the window bytes (at the real C4's 2 M blocks the 4 MiB filter's misses were
// half the walk's fetch: 5.5 -> 2.8 B per source byte)
#define VS_FBITS_CAP 24u
#endif
    h->fbits = std::min<uint32_t>(std::max<uint32_t>(std::min(lc + 5, VS_FBITS_CAP), 10), 28);
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
    // VS_OPT_BUCKET_BITS (tests): 2^k buckets, so that small tables overflow
    // buckets and exercise the directory fallback
    h->bbits = h->opt_bbits ? h->opt_bbits : rs_bucket_bits(count);
    const size_t bkt_bytes = ((size_t)kBucketWords * 4) << h->bbits;
    VS_TRY(h->d_bkt.ensure(bkt_bytes));
    VS_HIP(hipMemsetAsync(h->d_bkt.p, 0, bkt_bytes, h->stream));
    VS_HIP(launch_rs_buckets(h->d_tkey.as<uint64_t>(), count, (uint32_t)h->remainder, h->bbits,
                             h->d_bkt.as<uint32_t>(), h->stream));
    VS_HIP(hipStreamSynchronize(h->stream));
    h->host_ok = false;
    h->loaded = true;
    return 0;
}

// The table's host copies (sorted keys, directory, sum1, sum2 rows), read
// back once per loaded table and only by the paths that walk on the host: the
// device walk never needs them, and reading ~4 x count x 4 B through pageable
// copies cost the C4 step ~14 ms.
int host_tables(vs_rsync *h) {
    if (h->host_ok) return 0;
    const size_t count = (size_t)std::max(h->count, 0);
    const size_t s2 = (size_t)h->s2length;
    h->tkey_h.resize(count);
    h->dir_h.resize((1ull << h->dbits) + 1);
    h->sum1.resize(count);
    h->sum2.resize(count * s2);
    std::vector<uint64_t> pad(count * 2);
    if (count) {
        VS_TRY(h->stage.d2h(h->tkey_h.data(), h->d_tkey.p, count * 8, h->stream));
        VS_TRY(h->stage.d2h(h->dir_h.data(), h->d_dir.p, h->dir_h.size() * 4, h->stream));
        VS_TRY(h->stage.d2h(h->sum1.data(), h->d_sum1.p, count * 4, h->stream));
        VS_TRY(h->stage.d2h(pad.data(), h->d_sum2p.p, count * 16, h->stream));
    }
    // d_sum2p rows are the strong sums zero-padded to 16 bytes
    for (size_t i = 0; i < count; ++i) memcpy(h->sum2.data() + i * s2, pad.data() + 2 * i, s2);
    h->host_ok = true;
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
    int64_t exit_off = 0;          // first visited offset >= stop (final state)
    int32_t exit_want = 0;
};

// Offsets inside a walk are relative to the device data (file offset
// `origin`); F = file length - origin, so k = min(blength, F - o) and
// hash_search's end = F + 1 - len(last block), exactly as for a whole file.
struct WalkGeom {
    int64_t F = 0;      // file end, data-relative
    int64_t stop = 0;   // own_hi, data-relative: the walk stops at the first offset >= stop
};

// After the walk's needs were hashed: did any of them strong-match a table
// entry the walk would have compared it with?  If none did, treating each as
// a non-match was exactly rsync's decision, so the walk's output stands and
// only its false-alarm count lacks their compares (`extra_fa`).
bool needs_match(vs_rsync *h, int64_t F, const PinnedVec<uint64_t> &off,
                 const PinnedVec<uint32_t> &sum, const std::vector<uint8_t> &strong,
                 const std::vector<uint64_t> &need, int64_t *extra_fa) {
    const uint32_t s2 = (uint32_t)h->s2length;
    int64_t fa = 0;
    for (const uint64_t c : need) {
        const int64_t k = std::min<int64_t>(h->blength, F - (int64_t)off[c]);
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

// The speculative walk a re-walk may merge into: its matches
// (data-relative offsets), the false alarms counted before each match's
// offset was processed, its total and its exit state.
struct SpecWalk {
    const std::vector<vs_match> *m = nullptr;
    const std::vector<int64_t> *fa_before = nullptr;
    int64_t fa = 0, exit_off = 0;
    int32_t exit_want = 0;
};

// match.c hash_search over the sorted candidates, from state `st`, until the
// first offset >= g.stop.  A candidate whose strong sum is unknown is treated
// as a non-match and reported in `need`; st then holds the state just before
// the first of them (else the final state).  With `merge`, the walk ends at
// its first match that the speculative walk also made (same offset, same
// block): both walks continue identically from there, so the rest of the
// output, the false alarms and the exit are the speculative walk's.
void walk(vs_rsync *h, const WalkGeom &g, const PinnedVec<uint64_t> &off,
          const PinnedVec<uint32_t> &sum, const std::vector<uint8_t> &known,
          const std::vector<uint8_t> &strong, std::vector<uint64_t> &need,
          std::vector<vs_match> &out, std::vector<int64_t> &out_fa, WalkState &st,
          const SpecWalk *merge) {
    const size_t nc = off.size();
    const uint32_t s2 = (uint32_t)h->s2length;
    const int64_t end = g.F + 1 - blen(h, h->count - 1);
    int64_t offset = st.offset;
    int32_t want_i = st.want_i;
    size_t c = st.c;
    int64_t false_alarms = st.false_alarms;
    out.resize(st.nout);
    out_fa.resize(st.nout);
    bool resume_set = false, merged = false;
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
        if (o >= end || o >= g.stop) break;
        const int64_t k = std::min<int64_t>(h->blength, g.F - o);
        const uint32_t s = sum[c];
        const int64_t p0 = group_start(h, s);
        const int64_t fa_visit = false_alarms;
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
            const uint8_t *st2 = strong.data() + c * s2;
            if (memcmp(st2, h->sum2.data() + (size_t)i * s2, s2) != 0) {
                ++false_alarms;
                continue;
            }
            if (i != want_i && want_i < h->count && s == h->sum1[want_i] &&
                memcmp(st2, h->sum2.data() + (size_t)want_i * s2, s2) == 0)
                i = want_i;
            out.push_back({o, i, 0});
            out_fa.push_back(fa_visit);
            want_i = i + 1;
            offset = o + blen(h, i);
            matched = true;
            if (merge) {
                const std::vector<vs_match> &sm = *merge->m;
                auto it = std::lower_bound(sm.begin(), sm.end(), o,
                                           [](const vs_match &x, int64_t v) { return x.offset < v; });
                if (it != sm.end() && it->offset == o && it->block_index == i) {
                    const size_t j = (size_t)(it - sm.begin());
                    out.insert(out.end(), it + 1, sm.end());
                    for (size_t t = j + 1; t < sm.size(); ++t)
                        out_fa.push_back(fa_visit + (*merge->fa_before)[t] - (*merge->fa_before)[j]);
                    false_alarms = fa_visit + merge->fa - (*merge->fa_before)[j];
                    offset = merge->exit_off;
                    want_i = merge->exit_want;
                    merged = true;
                }
            }
            break;
        }
        if (merged) break;
        if (!matched) {
            offset = o + 1;
            ++c;
        }
    }
    const int64_t ex = std::max(offset, g.stop);
    st = resume_set ? resume : WalkState{offset, want_i, c, out.size(), false_alarms};
    st.end_false_alarms = false_alarms;
    st.exit_off = ex;
    st.exit_want = want_i;
}

// strong sums of candidate windows idx[] on the device -> strong/known
int verify(vs_rsync *h, const uint8_t *dev, int64_t F, const PinnedVec<uint64_t> &off,
           const std::vector<uint64_t> &idx, std::vector<uint8_t> &known,
           std::vector<uint8_t> &strong) {
    std::vector<uint64_t> todo;
    todo.reserve(idx.size());
    for (const uint64_t c : idx)
        if (!known[c]) todo.push_back(c);
    const size_t n = todo.size();
    if (!n) return 0;
    const uint32_t s2 = (uint32_t)h->s2length;
    std::vector<uint64_t> vo(n);
    std::vector<uint32_t> vl(n);
    uint32_t min_len = 0xffffffffu;
    for (size_t j = 0; j < n; ++j) {
        vo[j] = off[todo[j]];
        vl[j] = (uint32_t)std::min<int64_t>(h->blength, F - (int64_t)vo[j]);
        min_len = std::min(min_len, vl[j]);
    }
    VS_TRY(h->v_off.ensure(n * 8));
    VS_TRY(h->v_len.ensure(n * 4));
    VS_TRY(h->v_out.ensure(n * s2));
    VS_TRY(h->stage.h2d(h->v_off.p, vo.data(), n * 8, h->stream));
    VS_TRY(h->stage.h2d(h->v_len.p, vl.data(), n * 4, h->stream));
    KernelTimer kt(h, 1);
    VS_HIP(launch_rs_strong(dev, h->v_off.as<uint64_t>(), h->v_len.as<uint32_t>(), n,
                            h->csum_type, h->seed, s2, h->v_out.as<uint8_t>(), min_len, h->stream));
    kt.stop();
    std::vector<uint8_t> res(n * s2);
    VS_TRY(h->stage.d2h(res.data(), h->v_out.p, n * s2, h->stream));
    kt.fold();
    for (size_t j = 0; j < n; ++j) {
        memcpy(strong.data() + todo[j] * s2, res.data() + j * s2, s2);
        known[todo[j]] = 1;
    }
    h->st_hashed += (int64_t)n;
    return 0;
}

// Walks from (entry, want) (data-relative) with verification rounds until
// every strong sum the walk needed was known; the result is exactly
// hash_search's over [entry, stop).  batch: round 0's windows to hash first.
int run_walk(vs_rsync *h, int64_t entry, int32_t want, const SpecWalk *merge,
             std::vector<uint64_t> &batch, std::vector<vs_match> &out,
             std::vector<int64_t> &out_fa, WalkState &ws) {
    RsRun &r = h->run;
    const WalkGeom g{r.flen - r.origin, r.own_hi - r.origin};
    const PinnedVec<uint64_t> &off = h->h_off;
    ws = WalkState{};
    ws.offset = entry;
    ws.want_i = want;
    ws.c = std::lower_bound(off.begin(), off.end(), (uint64_t)std::max<int64_t>(entry, 0)) - off.begin();
    out.clear();
    out_fa.clear();
    double t_ver = 0, t_walk = 0;
    for (int round = 0;; ++round) {
        double tv = now_ms();
        VS_TRY(verify(h, r.dev, g.F, off, batch, h->h_known, h->h_strong));
        t_ver += now_ms() - tv;
        ++h->st_rounds;
        double tw = now_ms();
        int64_t extra_fa = 0;
        if (round > 0 && !needs_match(h, g.F, off, h->h_sum, h->h_strong, batch, &extra_fa)) {
            // every need was a false alarm: no replay (out holds the whole walk)
            ws.false_alarms = ws.end_false_alarms + extra_fa;
            t_walk += now_ms() - tw;
            break;
        }
        batch.clear();
        walk(h, g, off, h->h_sum, h->h_known, h->h_strong, batch, out, out_fa, ws, merge);
        t_walk += now_ms() - tw;
        if (batch.empty()) {
            ws.false_alarms = ws.end_false_alarms;
            break;
        }
    }
    h->ms[3] += t_ver;
    h->ms[4] += t_walk;
    return 0;
}

// Candidates of the owned offsets: coarse prefix sums, weak scan of every
// full-window offset in [own_lo, min(own_hi, F - blength + 1)) plus the one
// shrunk window that can match (the short last block), radix-sorted by
// offset and read back; round 0's "visit" predictions (rs_visit_kernel).
int scan_candidates(vs_rsync *h, std::vector<uint64_t> &batch) {
    RsRun &r = h->run;
    const int64_t dlen = r.dlen;
    const int64_t F = r.flen - r.origin;
    const int64_t lo = r.own_lo - r.origin, hi = r.own_hi - r.origin;
#ifdef VS_RS_TRACE
    constexpr bool trace = true;   // debug builds: stage times on stderr
#else
    constexpr bool trace = false;
#endif
    const double t0 = now_ms();
    // 1. coarse prefixes of the data
    const uint64_t nblk = ((uint64_t)dlen + kRsG - 1) / kRsG;
    VS_TRY(h->px.ensure(nblk * 4));
    VS_TRY(h->pt.ensure(nblk * 4));
    VS_TRY(h->pxs.ensure((nblk + 1) * 4));
    VS_TRY(h->pts.ensure((nblk + 1) * 4));
    VS_TRY(h->partials.ensure((nblk / 4096 + 2) * 4));
    VS_TRY(h->n_cand.ensure(16));
    VS_HIP(launch_rs_prefix(r.dev, (uint64_t)dlen, h->px.as<uint32_t>(), h->pt.as<uint32_t>(),
                            h->pxs.as<uint32_t>(), h->pts.as<uint32_t>(),
                            h->partials.as<uint32_t>(), h->stream));
    // 2. weak scan (re-run once with an exact capacity on overflow)
    RsScanArgs a{};
    a.data = r.dev;
    a.len = (uint64_t)dlen;
    a.blength = (uint64_t)h->blength;
    a.lo = (uint64_t)lo;
    const int64_t nfull_end = std::min<int64_t>(hi, F - h->blength + 1);
    a.nfull = nfull_end > lo ? (uint64_t)nfull_end : 0;
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
    const int64_t tail = F - h->remainder;   // the short last block's only window
    a.tail = (h->remainder && tail >= lo && tail < hi && tail >= 0) ? (int64_t)tail : -1;
    // expected: weak collisions (count / 2^32 per offset) + one per matching block
    const uint64_t span = a.nfull > a.lo ? a.nfull - a.lo : 0;
    uint64_t cap = (uint64_t)((double)span * h->count / 4294967296.0 * 2.0) +
                   span / h->blength * 2 + 65536;
    uint64_t nc = 0;
    for (int attempt = 0; attempt < 2; ++attempt) {
        VS_TRY(h->c_off.ensure(cap * 8));
        VS_TRY(h->c_sum.ensure(cap * 4));
        a.cap = cap;
        a.cand_off = h->c_off.as<uint64_t>();
        a.cand_sum = h->c_sum.as<uint32_t>();
        VS_HIP(hipMemsetAsync(h->n_cand.p, 0, 8, h->stream));
        KernelTimer kt(h, 0);
        VS_HIP(launch_rs_scan(a, h->cus, h->stream));
        kt.stop();
        VS_HIP(hipMemcpyAsync(h->pinned, h->n_cand.p, 8, hipMemcpyDeviceToHost, h->stream));
        VS_HIP(hipStreamSynchronize(h->stream));
        kt.fold();
        nc = h->pinned[0];
        if (trace) fprintf(stderr, "rs: scan done %.1f ms (%llu candidates)\n", now_ms() - t0,
                           (unsigned long long)nc);
        if (nc <= cap) break;
        cap = nc;
        if (attempt == 1) return fail(VS_ERR_STATE, "candidate buffer overflow");
    }
    // 3. sort candidates by offset; host scratch kept in the handle (first-touch
    // page faults on ~160 MB of fresh vectors per call cost ~100 ms at C4 shape)
    PinnedVec<uint64_t> &off = h->h_off;
    PinnedVec<uint32_t> &sum = h->h_sum;
    VS_TRY(pv_resize(off, nc));
    VS_TRY(pv_resize(sum, nc));
    if (nc) {
        VS_TRY(h->c_off2.ensure(nc * 8));
        VS_TRY(h->c_sum2.ensure(nc * 4));
        VS_TRY(h->sort_tmp.ensure(rs_sort_tmp_bytes(nc, true)));
        const int end_bit = (int)std::max<uint32_t>(ceil_log2((uint64_t)dlen + 1), 1);
        VS_HIP(launch_rs_sort_cands(h->sort_tmp.p, h->sort_tmp.cap, h->c_off.as<uint64_t>(),
                                    h->c_off2.as<uint64_t>(), h->c_sum.as<uint32_t>(),
                                    h->c_sum2.as<uint32_t>(), nc, end_bit, h->stream));
        VS_HIP(hipMemcpyAsync(off.data(), h->c_off2.p, nc * 8, hipMemcpyDeviceToHost, h->stream));
        VS_HIP(hipMemcpyAsync(sum.data(), h->c_sum2.p, nc * 4, hipMemcpyDeviceToHost, h->stream));
        VS_HIP(hipStreamSynchronize(h->stream));
    }
    h->st_cand = (int64_t)nc;
    h->h_known.assign(nc, 0);
    h->h_strong.resize(nc * (size_t)h->s2length);
    // 4. round 0: chained candidates (another candidate one block length
    // away) plus the uncovered ones (see rs_visit_kernel), flagged on the
    // device over the sorted offsets
    batch.clear();
    if (nc) {
        VS_TRY(h->d_flag.ensure(2 * nc));
        VS_HIP(launch_rs_chained(h->c_off2.as<uint64_t>(), nc, (uint64_t)h->blength,
                                 h->d_flag.as<uint8_t>(), h->stream));
        VS_TRY(pv_resize(h->h_flag, nc));
        VS_HIP(hipMemcpyAsync(h->h_flag.data(), h->d_flag.as<uint8_t>() + nc, nc,
                              hipMemcpyDeviceToHost, h->stream));
        VS_HIP(hipStreamSynchronize(h->stream));
        const uint8_t *fl = h->h_flag.data();
        for (size_t c = 0; c < nc; ++c)
            if (fl[c]) batch.push_back(c);
    }
    h->ms[2] += now_ms() - t0;
    if (trace) fprintf(stderr, "rs: candidates + round-0 batch %.1f ms (%zu)\n", now_ms() - t0,
                       batch.size());
    return 0;
}

// ---- device-walk path (rsync_walk.hip) -----------------------------------------
#ifdef VS_WALK_DEBUG
// debug builds: per-wave progress records in host-mapped memory, dumped by a
// watchdog thread if a walk launch has not finished after VSGPU_WALK_WATCH s
}  // namespace
#include <atomic>
#include <thread>
namespace {
uint64_t *g_walk_dbg = nullptr;
std::atomic<int> g_walk_gen{0};
void walk_watch_arm(vs_rsync *h, RsWalkArgs &a) {
    const char *e = getenv("VSGPU_WALK_WATCH");   // VS_WALK_DEBUG builds only
    if (!e) return;
    if (!g_walk_dbg && hipHostMalloc((void **)&g_walk_dbg, 4096 * 32, hipHostMallocMapped) != hipSuccess)
        return;
    memset(g_walk_dbg, 0xff, 4096 * 32);
    a.dbg = g_walk_dbg;
    const int gen = ++g_walk_gen;
    const double secs = atof(e);
    std::thread([gen, secs]() {
        std::this_thread::sleep_for(std::chrono::duration<double>(secs));
        if (g_walk_gen.load() != gen) return;
        fprintf(stderr, "walk watchdog: launch %d still running; per-wave phase/offset/extra:\n", gen);
        for (int w = 0; w < 4096; ++w) {
            const volatile uint64_t *r = g_walk_dbg + 4 * w;
            if (r[0] == ~0ull) continue;
            fprintf(stderr, "  wave %d phase %llu o %lld x %llx\n", w, (unsigned long long)r[0],
                    (long long)r[1], (unsigned long long)r[2]);
        }
        fflush(stderr);
    }).detach();
    (void)h;
}
void walk_watch_done() { ++g_walk_gen; }
#else
inline void walk_watch_arm(vs_rsync *, RsWalkArgs &) {}
inline void walk_watch_done() {}
#endif
bool walk_eligible(const vs_rsync *h) {
    return !h->opt_host_walk &&
           (h->csum_type == VS_CSUM_XXH3_128 || h->csum_type == VS_CSUM_XXH3_64) &&
           h->blength > 240;
}

// get_checksum1 on the host
uint32_t host_weak(const uint8_t *p, int64_t n) {
    uint32_t s1 = 0, s2 = 0;
    for (int64_t i = 0; i < n; ++i) {
        s1 += (uint32_t)(int32_t)(int8_t)p[i];
        s2 += s1;
    }
    return (s1 & 0xffffu) | (s2 << 16);
}

// Stitch passes until no segment's exit changes (Jacobi: a changed exit
// reaches the next segment in the next pass).  Returns the last segment's exit.
int walk_converge(vs_rsync *h, int64_t *x, int32_t *xw) {
    RsRun &r = h->run;
    RsWalkArgs &a = r.wa;
    for (uint32_t pass = 0;; ++pass) {
        if (pass > a.nseg + 2) return fail(VS_ERR_STATE, "device walk stitch did not converge");
        a.exit_old = h->w_exit[r.xcur].as<int64_t>();
        a.exitw_old = h->w_exitw[r.xcur].as<int32_t>();
        a.exit_new = h->w_exit[r.xcur ^ 1].as<int64_t>();
        a.exitw_new = h->w_exitw[r.xcur ^ 1].as<int32_t>();
        VS_HIP(hipMemsetAsync(a.flags, 0, 4, h->stream));
        KernelTimer kt(h, 3);
        walk_watch_arm(h, a);
        VS_HIP(launch_rs_walk(a, true, h->cus, h->stream));
        kt.stop();
        VS_HIP(hipMemcpyAsync(h->pinned, a.flags, 4, hipMemcpyDeviceToHost, h->stream));
        VS_HIP(hipStreamSynchronize(h->stream));
        walk_watch_done();
        kt.fold();
        r.xcur ^= 1;
        const uint32_t fl = (uint32_t)h->pinned[0];
        if (fl & 2u) return fail(VS_ERR_STATE, "device walk: segment match capacity exceeded");
        if (!(fl & 1u)) break;
    }
    VS_HIP(hipMemcpyAsync(h->pinned, h->w_exit[r.xcur].as<int64_t>() + (a.nseg - 1), 8,
                          hipMemcpyDeviceToHost, h->stream));
    VS_HIP(hipMemcpyAsync((int32_t *)(h->pinned + 1), h->w_exitw[r.xcur].as<int32_t>() + (a.nseg - 1),
                          4, hipMemcpyDeviceToHost, h->stream));
    VS_HIP(hipStreamSynchronize(h->stream));
    *x = (int64_t)h->pinned[0];
    *xw = *(const int32_t *)(h->pinned + 1);
    return 0;
}

// The walk's continuation past the last full window: of the offsets in
// [max(x, full_end), end) only F - remainder (the short last block's one
// window) can match.  x / xw: the device walk's exit.  Sets the range exit.
int walk_tail(vs_rsync *h, int64_t x, int32_t xw, int64_t *exit_off, int32_t *exit_want) {
    RsRun &r = h->run;
    const int64_t F = r.flen - r.origin, hi = r.own_hi - r.origin;
    r.tail.clear();
    r.tail_fa = 0;
    int64_t o = x;
    int32_t want = xw;
    const int64_t t = F - h->remainder;
#ifdef VS_RS_TRACE
    constexpr bool trace = true;   // debug builds: stage times on stderr
#else
    constexpr bool trace = false;
#endif
    if (trace)
        fprintf(stderr, "rs: walk tail: device exit %lld want %d, tail offset %lld, range end %lld\n",
                (long long)x, xw, (long long)t, (long long)hi);
    if (h->remainder && o <= t && t < hi && t >= 0) {
        VS_TRY(host_tables(h));
        std::vector<uint8_t> buf((size_t)h->remainder);
        VS_TRY(h->stage.d2h(buf.data(), r.dev + t, buf.size(), h->stream));
        const uint32_t sum = host_weak(buf.data(), h->remainder);
        const uint32_t s2 = (uint32_t)h->s2length;
        // the strong sum on the device (the same kernel the walk's windows use)
        uint8_t st[16] = {0};
        {
            const uint32_t vl = (uint32_t)h->remainder;
            VS_TRY(h->v_off.ensure(8));
            VS_TRY(h->v_len.ensure(4));
            VS_TRY(h->v_out.ensure(16));
            // through the handle's pinned words: [4] offset, [5] length, [6..7] sum
            h->pinned[4] = (uint64_t)t;
            h->pinned[5] = vl;
            VS_HIP(hipMemcpyAsync(h->v_off.p, h->pinned + 4, 8, hipMemcpyHostToDevice, h->stream));
            VS_HIP(hipMemcpyAsync(h->v_len.p, h->pinned + 5, 4, hipMemcpyHostToDevice, h->stream));
            VS_HIP(launch_rs_strong(r.dev, h->v_off.as<uint64_t>(), h->v_len.as<uint32_t>(), 1,
                                    h->csum_type, h->seed, s2, h->v_out.as<uint8_t>(), vl,
                                    h->stream));
            VS_HIP(hipMemcpyAsync(h->pinned + 6, h->v_out.p, s2, hipMemcpyDeviceToHost, h->stream));
            VS_HIP(hipStreamSynchronize(h->stream));
            memcpy(st, h->pinned + 6, s2);
            h->st_hashed += 1;
        }
        o = t + 1;   // no match: hash_search's loop ends (end = F + 1 - remainder)
        for (int64_t q = group_start(h, sum); q >= 0 && q < h->count &&
                                             (uint32_t)(h->tkey_h[q] >> 32) == sum;
             ++q) {
            int32_t i = (int32_t)~(uint32_t)h->tkey_h[q];
            if (blen(h, i) != h->remainder) continue;
            if (memcmp(st, h->sum2.data() + (size_t)i * s2, s2) != 0) {
                ++r.tail_fa;
                continue;
            }
            if (i != want && want < h->count && sum == h->sum1[want] &&
                memcmp(st, h->sum2.data() + (size_t)want * s2, s2) == 0)
                i = want;
            r.tail.push_back({t, i, 0});
            want = i + 1;
            o = t + blen(h, i);
            break;
        }
    }
    *exit_off = std::max(o, hi) + r.origin;
    *exit_want = want;
    return 0;
}

// match_scan on the device-walk path: segments, speculative walks, stitch
// from the range's speculative entry
int walk_scan(vs_rsync *h) {
    RsRun &r = h->run;
    RsWalkArgs &a = r.wa;
    a = RsWalkArgs{};
    const int64_t F = r.flen - r.origin;
    a.data = r.dev;
    a.dlen = (uint64_t)r.dlen;
    a.full_end = F - h->blength + 1;
    a.lo = r.own_lo - r.origin;
    a.hi = r.own_hi - r.origin;
    {
        // segment length: 48 blocks (6 MiB at C4; with the wide flushes 16,
        // 24, 32, 64 and 96 measured slower), shorter -- down
        // to 1 MiB -- when the range is too small to give every wave of the
        // grid two segments (a streamed piece of 256 MiB: 256 segments
        // instead of 43 idle-heavy ones).  VS_OPT_WALK_SEGMENT_BLOCKS
        // overrides it.
        const int64_t range = std::max<int64_t>(a.hi - a.lo, 1);
        const int64_t waves = (int64_t)std::max(h->cus, 1) * rs_walk_waves_per_cu();
        int64_t sl = (int64_t)h->blength * (h->seg_blocks ? h->seg_blocks : 48);
        if (!h->seg_blocks && range / sl < 2 * waves)
            sl = std::max<int64_t>(range / (2 * waves), h->blength);
        a.seg_len = std::max<int64_t>(sl, 1 << 20);
    }
    // Segment starts a margin before a block boundary of the file: a
    // speculative walk steps byte by byte from its segment's start to its
    // first match, on average half a block when the start is arbitrary; where
    // the source keeps the destination's block phase (in-place writes) or
    // drifts from it by short inserts and deletes (C4), the first match lies
    // about the margin past the start.  Segment 0 starts at lo.  Only when
    // the segments are whole blocks and the range holds several.
#ifndef VS_SEG_MARGIN
#define VS_SEG_MARGIN 24576
#endif
    a.segb = a.lo;
    {
        const int64_t L = (int64_t)h->blength, M = h->opt_seg_margin >= 0 ? h->opt_seg_margin : VS_SEG_MARGIN;
        if (M > 0 && a.seg_len % L == 0 && a.hi - a.lo >= 4 * a.seg_len) {
            const int64_t rr = ((a.lo + a.seg_len + r.origin + M) % L + L) % L;
            a.segb = a.lo - rr;   // segment 1 starts at lo + seg_len - rr, M before a boundary
        }
    }
    a.nseg = (uint32_t)((a.hi - a.segb + a.seg_len - 1) / a.seg_len);
    a.nseg1 = a.nseg;
    a.seg_len2 = a.seg_len;
    // the last tail % of the range in segments a quarter as long, handed out
    // last (waves take segments in index order), so the grid's last waves
    // finish closer together: 20 % when the grid gets fewer than four
    // segments per wave, else 10 % (the real C4's rank: walk 44.6 -> 41.2 ms;
    // the 64 GiB shape: 42.0 -> 41.1)
    const int64_t waves = (int64_t)std::max(h->cus, 1) * rs_walk_waves_per_cu();
    const int32_t tailpct = h->opt_tailpct >= 0 ? h->opt_tailpct : ((int64_t)a.nseg < 4 * waves ? 20 : 10);
    if (tailpct > 0) {
#ifndef VS_TAIL_DIV
#define VS_TAIL_DIV 4
#endif
        const int64_t range = a.hi - a.segb, L2 = std::max<int64_t>(a.seg_len / VS_TAIL_DIV, 1 << 20);
        if (L2 < a.seg_len) {
            // (at least segment 0 when it ends at an aligned start)
            const int64_t big = std::max<int64_t>(range * (100 - tailpct) / 100 / a.seg_len,
                                                  a.segb < a.lo ? 1 : 0);
            a.nseg1 = (uint32_t)big;
            a.seg_len2 = L2;
            a.nseg = (uint32_t)(big + (range - big * a.seg_len + L2 - 1) / L2);
        }
    }
    a.cap = (uint32_t)(a.seg_len / h->blength + 2);
    a.blength = (uint32_t)h->blength;
    a.count = (uint32_t)h->count;
    a.remainder = (uint32_t)h->remainder;
    a.csum_type = h->csum_type;
    a.seed = h->seed;
    const uint32_t s2 = (uint32_t)h->s2length;
    a.s2mask_lo = s2 >= 8 ? ~0ull : ((1ull << (8 * s2)) - 1);
    a.s2mask_hi = s2 <= 8 ? 0ull : (s2 >= 16 ? ~0ull : ((1ull << (8 * (s2 - 8))) - 1));
    a.sum2p = h->d_sum2p.as<uint64_t>();
    a.sum1 = h->d_sum1.as<uint32_t>();
    a.tkey = h->d_tkey.as<uint64_t>();
    a.dir = h->d_dir.as<uint32_t>();
    a.bkt = h->d_bkt.as<uint32_t>();
    a.bbits = h->bbits;
    a.filt = h->d_filt.as<uint32_t>();
    a.fbits = h->fbits;
    a.dbits = h->dbits;
    a.lbits = rs_lds_filter_bits(h->fbits);
    a.filt_l = h->d_filt.as<uint32_t>() + ((1ull << h->fbits) / 32);
    a.filt_b = (const uint64_t *)(a.filt_l + ((1ull << a.lbits) / 32));
    if (!h->opt_prefilter) a.lbits = 0;   // VS_OPT_WALK_PREFILTER 0: no LDS prefilter
    a.flushq = h->opt_flushq ? h->opt_flushq : 16u;   // wide flushes
    a.flushspan = h->opt_flushspan;
    a.flushpredict = h->opt_flushpredict ? 1u : 0u;
    const size_t ns = std::max<uint32_t>(a.nseg, 1), nc = ns * a.cap;
    VS_TRY(h->w_spec_off.ensure(nc * 8));
    VS_TRY(h->w_spec_idx.ensure(nc * 4));
    VS_TRY(h->w_spec_fab.ensure(nc * 8));
    VS_TRY(h->w_fin_off.ensure(nc * 8));
    VS_TRY(h->w_fin_idx.ensure(nc * 4));
    VS_TRY(h->w_fin_fab.ensure(nc * 8));
    VS_TRY(h->w_spec_n.ensure(ns * 4));
    // false-alarm windows of the speculative walks: up to 1024 per segment (a
    // 6 MiB segment of the real C4 averages ~300; more falls back to a
    // re-walk), at most 256 MiB of records per walk (small blocks, many
    // segments)
    a.facap = (uint32_t)std::max<uint64_t>(
        64, std::min<uint64_t>(1024, (256ull << 20) / (12ull * std::max<uint32_t>(a.nseg, 1))));
    // VS_OPT_FA_RECORD (tests): a smaller record, so stitches fall back to re-walks
    if (h->opt_facap >= 0) a.facap = (uint32_t)h->opt_facap;
    VS_TRY(h->w_spec_fao.ensure(ns * a.facap * 8));
    VS_TRY(h->w_spec_fac.ensure(ns * a.facap * 4));
    VS_TRY(h->w_spec_nfa.ensure(ns * 4));
    VS_TRY(h->w_spec_fa.ensure(ns * 8));
    VS_TRY(h->w_spec_exit.ensure(ns * 8));
    VS_TRY(h->w_spec_exitw.ensure(ns * 4));
    VS_TRY(h->w_fin_entry.ensure(ns * 8));
    VS_TRY(h->w_fin_entryw.ensure(ns * 4));
    VS_TRY(h->w_fin_from.ensure(ns * 4));
    VS_TRY(h->w_fin_n.ensure(ns * 4));
    VS_TRY(h->w_fin_fa.ensure(ns * 8));
    for (int i = 0; i < 2; ++i) {
        VS_TRY(h->w_exit[i].ensure(ns * 8));
        VS_TRY(h->w_exitw[i].ensure(ns * 4));
    }
    VS_TRY(h->w_ctl.ensure(64));
    a.prof = nullptr;
    a.work = h->w_ctl.as<uint32_t>();
    a.flags = h->w_ctl.as<uint32_t>() + 4;
    a.spec_off = h->w_spec_off.as<int64_t>();
    a.spec_idx = h->w_spec_idx.as<int32_t>();
    a.spec_fab = h->w_spec_fab.as<int64_t>();
    a.spec_n = h->w_spec_n.as<uint32_t>();
    a.spec_fa = h->w_spec_fa.as<uint64_t>();
    a.spec_exit = h->w_spec_exit.as<int64_t>();
    a.spec_exitw = h->w_spec_exitw.as<int32_t>();
    a.spec_fao = h->w_spec_fao.as<int64_t>();
    a.spec_fac = h->w_spec_fac.as<uint32_t>();
    a.spec_nfa = h->w_spec_nfa.as<uint32_t>();
    a.fin_entry = h->w_fin_entry.as<int64_t>();
    a.fin_entryw = h->w_fin_entryw.as<int32_t>();
    a.fin_from = h->w_fin_from.as<uint32_t>();
    a.fin_n = h->w_fin_n.as<uint32_t>();
    a.fin_fa = h->w_fin_fa.as<uint64_t>();
    a.fin_off = h->w_fin_off.as<int64_t>();
    a.fin_idx = h->w_fin_idx.as<int32_t>();
    a.fin_fab = h->w_fin_fab.as<int64_t>();
    a.e0 = r.spec_entry - r.origin;
    a.w0 = r.spec_want;
    a.spec_w0 = r.spec_want;
    // speculative walks -> w_exit[0]
    r.xcur = 0;
    a.exit_old = h->w_exit[1].as<int64_t>();
    a.exitw_old = h->w_exitw[1].as<int32_t>();
    a.exit_new = h->w_exit[0].as<int64_t>();
    a.exitw_new = h->w_exitw[0].as<int32_t>();
    const double t0 = now_ms();
    VS_HIP(hipMemsetAsync(a.flags, 0, 4, h->stream));
    // profiling builds (-DVS_WALK_PROF): per-wave phase cycles of the
    // speculative pass on stderr
#ifdef VS_WALK_PROF
    constexpr bool wprof = true;
#else
    constexpr bool wprof = false;
#endif
    constexpr int kPh = 16;   // phases (rsync_walk.hip kPrN): cycles, then counts
    const size_t nprof = (size_t)std::max(h->cus, 1) * 64 * 2 * kPh;
    if (wprof) {
        VS_TRY(h->w_prof.ensure(nprof * 8));
        VS_HIP(hipMemsetAsync(h->w_prof.p, 0, nprof * 8, h->stream));
        a.prof = h->w_prof.as<uint64_t>();
    }
    {
        KernelTimer kt(h, 0);
        walk_watch_arm(h, a);
        VS_HIP(launch_rs_walk(a, false, h->cus, h->stream));
        kt.stop();
        VS_HIP(hipMemcpyAsync(h->pinned, a.flags, 4, hipMemcpyDeviceToHost, h->stream));
        VS_HIP(hipStreamSynchronize(h->stream));
        walk_watch_done();
        kt.fold();
        if ((uint32_t)h->pinned[0] & 2u)
            return fail(VS_ERR_STATE, "device walk: segment match capacity exceeded");
    }
    if (wprof) {
        std::vector<uint64_t> pr(nprof);
        VS_TRY(h->stage.d2h(pr.data(), a.prof, nprof * 8, h->stream));
        const char *names[kPh] = {"run", "step", "flush", "chain", "segment", "band-fill",
                                  "band-pairs", "band-chain", "step:sums", "step:lds",
                                  "step:gather", "step:probe", "step:queue", "flush:iters",
                                  "flush:windows", ""};
        double cyc[kPh] = {0}, cnt[kPh] = {0}, mx = 0;
        int waves = 0;
        for (size_t w = 0; w < nprof / (2 * kPh); ++w) {
            const uint64_t *q = &pr[w * 2 * kPh];
            if (!q[kPh + 4]) continue;
            ++waves;
            for (int i = 0; i < kPh; ++i) {
                cyc[i] += (double)q[i];
                cnt[i] += (double)q[kPh + i];
            }
            mx = std::max(mx, (double)q[4]);
        }
        fprintf(stderr, "walk prof: %d waves; per wave:", waves);
        for (int i = 0; i < kPh; ++i)
            if (cnt[i] > 0)
                fprintf(stderr, " %s %.3g cyc / %.4g calls (%.3g cyc each);", names[i],
                    cyc[i] / std::max(waves, 1), cnt[i] / std::max(waves, 1),
                    cyc[i] / std::max(cnt[i], 1.0));
        fprintf(stderr, " max segment-total %.3g cyc\n", mx);
        a.prof = nullptr;
    }
    int64_t x = 0;
    int32_t xw = 0;
    VS_TRY(walk_converge(h, &x, &xw));
    VS_TRY(walk_tail(h, x, xw, &r.spec_exit, &r.spec_exit_want));
    h->ms[2] += now_ms() - t0;
    return 0;
}

// the device walk's result (matches data-relative, in order) and false alarms:
// compacted on the device (launch_rs_collect), read back through pinned memory
int walk_collect(vs_rsync *h, std::vector<vs_match> &out, int64_t *fa) {
    RsRun &r = h->run;
    const RsWalkArgs &a = r.wa;
    const size_t ns = a.nseg, nc = ns * a.cap;
    out.clear();
    int64_t total_fa = 0;
    if (ns) {
        VS_TRY(h->wc_cnt.ensure(ns * 4));
        VS_TRY(h->wc_pos.ensure((ns + 1) * 4 + 64));
        VS_TRY(h->wc_part.ensure((ns / 4096 + 2) * 4));
        VS_TRY(h->wc_out.ensure(nc * sizeof(vs_match)));
        static_assert(sizeof(vs_match) == 16, "vs_match is one 16-byte record");
        uint32_t *pos = h->wc_pos.as<uint32_t>();
        // the false-alarm total: 8-byte aligned, after pos[0, ns]
        unsigned long long *fat =
            (unsigned long long *)(((uintptr_t)(pos + ns + 1) + 7) & ~(uintptr_t)7);
        VS_HIP(launch_rs_collect(a, h->wc_cnt.as<uint32_t>(), pos, h->wc_part.as<uint32_t>(),
                                 h->wc_out.as<uint4>(), fat, h->stream));
        VS_HIP(hipMemcpyAsync(h->pinned, fat, 8, hipMemcpyDeviceToHost, h->stream));
        VS_HIP(hipMemcpyAsync((uint32_t *)(h->pinned + 1), pos + ns, 4, hipMemcpyDeviceToHost,
                              h->stream));
        VS_HIP(hipStreamSynchronize(h->stream));
        total_fa = (int64_t)h->pinned[0];
        const size_t n = *(const uint32_t *)(h->pinned + 1);
        if (n > nc) return fail(VS_ERR_STATE, "device walk: match list longer than its capacity");
        if (n > h->wc_host_cap) {
            if (h->wc_host) (void)hipHostFree(h->wc_host);
            h->wc_host = nullptr;
            h->wc_host_cap = 0;
            const size_t want = std::max(n, nc);
            if (hipHostMalloc((void **)&h->wc_host, want * sizeof(vs_match), hipHostMallocDefault) !=
                hipSuccess) {
                (void)hipGetLastError();
                h->wc_host = nullptr;
                return fail(VS_ERR_NOMEM, "pinned match read-back buffer");
            }
            h->wc_host_cap = want;
        }
        if (n) {
            VS_HIP(hipMemcpyAsync(h->wc_host, h->wc_out.p, n * sizeof(vs_match),
                                  hipMemcpyDeviceToHost, h->stream));
            VS_HIP(hipStreamSynchronize(h->stream));
        }
        out.assign(h->wc_host, h->wc_host + n);
    }
    for (const vs_match &m : r.tail) out.push_back(m);
    *fa = total_fa + r.tail_fa;
    return 0;
}

// ---- sharded match_sums: scan + speculative walk, stitch, finish
// entry / want: where the range's own walk starts -- the true entry when the
// caller knows it (the streamed walk: the previous piece's exit), else
// (has_entry false) hash_search's start at offset 0 or "no preference" (the
// speculative entry of a shard, stitched later)
int match_scan(vs_rsync *h, const void *dev_src, int64_t dlen, int64_t origin, int64_t flen,
               int64_t own_lo, int64_t own_hi, int64_t *exit_off, int32_t *exit_want,
               bool has_entry = false, int64_t entry = 0, int32_t want = 0) {
    if (!h->loaded) return fail(VS_ERR_STATE, "vs_rsync_match_scan before vs_rsync_load_sums");
    if (dlen < 0 || (dlen && !dev_src) || origin < 0 || flen < origin + dlen || own_lo < origin ||
        own_hi < own_lo || own_hi > flen)
        return fail(VS_ERR_ARG, "bad source range (need origin <= own_lo <= own_hi <= file_len)");
    const int64_t need_hi = std::min<int64_t>(own_hi + h->blength - 1, flen);
    if (own_hi > own_lo && origin + dlen < need_hi)
        return fail(VS_ERR_ARG, "source data must cover [own_lo, min(own_hi + blength - 1, file_len))");
    VS_TRY(rs_dev(h));
    RsRun &r = h->run;
    r = RsRun{};
    r.dev = (const uint8_t *)dev_src;
    r.dlen = dlen;
    r.origin = origin;
    r.flen = flen;
    r.own_lo = own_lo;
    r.own_hi = own_hi;
    h->st_cand = h->st_fa = h->st_hashed = 0;
    h->st_rounds = 0;
    for (int i = 2; i < 5; ++i) h->ms[i] = 0;
    // the speculative entry: hash_search's own start at offset 0, else
    // want_i = count ("no preference": want_i < count fails)
    if (has_entry && (entry < own_lo || want < 0))
        return fail(VS_ERR_ARG, "entry before the owned range or negative want_i");
    r.spec_entry = has_entry ? entry : own_lo;
    r.spec_want = has_entry ? want : (own_lo == 0 ? 0 : h->count);
    r.state = 1;
    if (own_hi <= r.spec_entry || flen == 0 || h->count == 0) {
        // match_sums: no sums (or no owned offsets) -> all literal
        r.spec_exit = std::max(r.spec_entry, own_hi);
        r.spec_exit_want = r.spec_want;
    } else if (walk_eligible(h)) {
        if (((uintptr_t)dev_src & 15) != 0)
            return fail(VS_ERR_ARG, "device source must be 16-byte aligned");
        VS_TRY(order_after_null(h));
        r.dev_walk = true;
        VS_TRY(walk_scan(h));
        int64_t fa = 0;
        VS_TRY(walk_collect(h, r.spec, &fa));
        r.spec_fa = fa;
    } else {
        VS_TRY(order_after_null(h));
        VS_TRY(host_tables(h));
        std::vector<uint64_t> &batch = h->h_batch;
        VS_TRY(scan_candidates(h, batch));
        WalkState ws;
        VS_TRY(run_walk(h, r.spec_entry - origin, r.spec_want, nullptr, batch, r.spec,
                        r.spec_fa_before, ws));
        r.spec_fa = ws.false_alarms;
        r.spec_exit = ws.exit_off + origin;
        r.spec_exit_want = ws.exit_want;
    }
    r.fin_exit = r.spec_exit;
    r.fin_exit_want = r.spec_exit_want;
    r.fin_fa = r.spec_fa;
    r.use_spec = true;
    h->st_fa = r.fin_fa;
    if (exit_off) *exit_off = r.spec_exit;
    if (exit_want) *exit_want = r.spec_exit_want;
    return 0;
}

int match_stitch(vs_rsync *h, int64_t entry, int32_t want, int64_t *exit_off, int32_t *exit_want) {
    RsRun &r = h->run;
    if (r.state < 1) return fail(VS_ERR_STATE, "vs_rsync_match_stitch before vs_rsync_match_scan");
    if (entry < r.own_lo) return fail(VS_ERR_ARG, "entry before the scanned own range");
    if (want < 0) return fail(VS_ERR_ARG, "negative want_i");
    VS_TRY(rs_dev(h));
    if (entry == r.spec_entry && want == r.spec_want) {
        r.use_spec = true;
        r.fin_exit = r.spec_exit;
        r.fin_exit_want = r.spec_exit_want;
        r.fin_fa = r.spec_fa;
    } else if (entry >= r.own_hi || h->count == 0 || r.flen == 0) {
        // a match of the previous shard spans this whole range: nothing to visit
        r.use_spec = false;
        r.fin.clear();
        r.fin_fa = 0;
        r.fin_exit = std::max(entry, r.own_hi);
        r.fin_exit_want = want;
    } else if (r.dev_walk) {
        r.wa.e0 = entry - r.origin;
        r.wa.w0 = want;
        int64_t x = 0;
        int32_t xw = 0;
        const double t0 = now_ms();
        VS_TRY(walk_converge(h, &x, &xw));
        VS_TRY(walk_tail(h, x, xw, &r.fin_exit, &r.fin_exit_want));
        int64_t fa = 0;
        VS_TRY(walk_collect(h, r.fin, &fa));
        h->ms[2] += now_ms() - t0;
        r.use_spec = false;
        r.fin_fa = fa;
    } else {
        SpecWalk sw{&r.spec, &r.spec_fa_before, r.spec_fa, r.spec_exit - r.origin, r.spec_exit_want};
        std::vector<uint64_t> &batch = h->h_batch;
        batch.clear();
        WalkState ws;
        std::vector<int64_t> fa_before;
        VS_TRY(run_walk(h, entry - r.origin, want, &sw, batch, r.fin, fa_before, ws));
        r.use_spec = false;
        r.fin_fa = ws.false_alarms;
        r.fin_exit = ws.exit_off + r.origin;
        r.fin_exit_want = ws.exit_want;
    }
    r.state = 2;
    h->st_fa = r.fin_fa;
    if (exit_off) *exit_off = r.fin_exit;
    if (exit_want) *exit_want = r.fin_exit_want;
    return 0;
}

int match_finish(vs_rsync *h, int64_t *n_matches) {
    RsRun &r = h->run;
    if (r.state < 1) return fail(VS_ERR_STATE, "vs_rsync_match_finish before vs_rsync_match_scan");
    const std::vector<vs_match> &src = r.use_spec ? r.spec : r.fin;
    h->matches.resize(src.size());
    for (size_t j = 0; j < src.size(); ++j)
        h->matches[j] = {src[j].offset + r.origin, src[j].block_index, 0};
    h->st_fa = r.fin_fa;
    r.state = 3;
    if (n_matches) *n_matches = (int64_t)h->matches.size();
    return 0;
}

int match_device(vs_rsync *h, const void *dev_src, int64_t len, int64_t *n_matches) {
    if (!h->loaded) return fail(VS_ERR_STATE, "vs_rsync_match_device before vs_rsync_load_sums");
    if (len < 0 || (len && !dev_src)) return fail(VS_ERR_ARG, "bad source");
    h->matches.clear();
    if (n_matches) *n_matches = 0;
    VS_TRY(match_scan(h, dev_src, len, 0, len, 0, len, nullptr, nullptr));
    return match_finish(h, n_matches);
}

// ---- whole-file checksum jobs (FsJob) ----------------------------------------
// The job's thread: piece i = contributions of blocks [i P, (i+1) P) into
// device slot i % R, read back into pinned slot i % R (serial types: the
// bytes themselves, P * 64 at a time), then chained / hashed on the host.
// Stream order on j->s keeps a device slot until its read-back is done; a
// pinned slot is refilled only after the host consumed it.
#ifndef VS_FS_TRACE
#define VS_FS_TRACE 0
#endif
void fs_thread(FsJob *j) {
    const bool serial = j->serial;
    const uint64_t unit = serial ? 1 : 1024;             // source bytes per item
    const uint64_t items = serial ? j->len : j->nb;       // bytes or blocks
    const uint64_t per = serial ? j->piece * 64 : j->piece;
    const uint64_t np = (items + per - 1) / per;
    double chain = 0, kms = 0;
    auto fail_here = [&](hipError_t e, const char *what) {
        j->rc = VS_ERR_HIP;
        j->err = std::string(what) + ": " + hipGetErrorName(e);
        (void)hipGetLastError();
    };
    if (hipSetDevice(j->device) != hipSuccess) return fail_here(hipGetLastError(), "hipSetDevice");
    if (j->rows_first) {
        // every row is on the device once the kernel's event fires; pieces come
        // back on the DMA engine, copy i overlapping the chain of piece i - 1
        const double t_thread = now_ms();
        double dwait = 0;
        (void)t_thread;
        const hipError_t e = hipEventSynchronize(j->kev[0][1]);
        const double t_rows = now_ms();
        (void)t_rows;
        if (e != hipSuccess) return fail_here(e, "file-sum rows kernel");
        float ms = 0;
        if (hipEventElapsedTime(&ms, j->kev[0][0], j->kev[0][1]) == hipSuccess) kms = ms;
        (void)hipGetLastError();
        const uint8_t *rows = j->rows.as<uint8_t>();
        // The whole read-back is queued at once, in kChunks copies (one
        // signal each): the engine then serves this job's chunks back to back
        // at its full rate, and the next job's after them.  With one copy in
        // flight per job (a 3-deep ring of 16 MiB pieces, round 5's first
        // form) three concurrent jobs shared the engine piece by piece; each
        // chain then waited on its own copies and the jobs stayed
        // overlapped: 240-266 ms of copy waits per job against 3-64 in the
        // runs where they happened to stagger (profiles/r05_r7/trace).
        const uint64_t total = items * 64;
        const uint64_t cb = ((total + FsJob::kChunks - 1) / FsJob::kChunks + 63) & ~63ull;
        const uint64_t nc = (total + cb - 1) / cb;
        if (j->whole) {   // the file's last <= 1088 bytes, for the finish
            const uint64_t keep = std::min<uint64_t>(j->len, 1088);
            if (!j->dma.start(FsJob::kChunks, j->hlast, j->src + j->len - keep, keep))
                return fail_here(hipErrorUnknown, "file-sum tail read-back (DMA)");
        }
        for (uint64_t c = 0; c < nc; ++c)
            if (!j->dma.start((int)c, j->hrows + c * cb, rows + c * cb, std::min(cb, total - c * cb))) {
                // copies already queued still write into hrows / hlast: they
                // must land before the job ends and its buffers can be freed
                for (uint64_t k = 0; k < c; ++k) (void)j->dma.wait((int)k);
                if (j->whole) (void)j->dma.wait(FsJob::kChunks);
                return fail_here(hipErrorUnknown, "file-sum rows read-back (DMA)");
            }
        bool copies_ok = true;
        for (uint64_t c = 0; c < nc; ++c) {
            const double w0 = now_ms();
            copies_ok &= j->dma.wait((int)c);
            dwait += now_ms() - w0;
            const uint64_t n = std::min(cb, total - c * cb) / 64;
            const double c0 = now_ms();
            xxh3_chain_rows((const uint64_t *)(j->hrows + c * cb), n, j->acc);
            chain += now_ms() - c0;
        }
        if (j->whole) copies_ok &= j->dma.wait(FsJob::kChunks);
        if (!copies_ok) return fail_here(hipErrorUnknown, "file-sum rows read-back (DMA copy error)");
        j->host_ms = chain;
        j->dev_ms = kms;
#if VS_FS_TRACE
        {
            static const double epoch = now_ms();
            fprintf(stderr, "fs trace: job %p call %.1f thread %.1f rows %.1f dmawait %.1f chain %.1f end %.1f ms\n",
                    (void *)j, j->t_call - epoch, t_thread - epoch, t_rows - epoch, dwait, chain,
                    now_ms() - epoch);
        }
#else
        (void)dwait;
#endif
        return;
    }
    SerialSum ss;
    if (serial) serial_sum_init(ss, j->csum);
    auto issue = [&](uint64_t i) -> bool {
        const int r = (int)(i % FsJob::kRing);
        const uint64_t i0 = i * per, n = std::min(per, items - i0);
        hipError_t e = hipSuccess;
        if (serial) {
            e = hipMemcpyAsync(j->hC[r], j->src + i0, n, hipMemcpyDeviceToHost, j->s);
        } else {
            uint64_t *dc = j->dC.as<uint64_t>() + (uint64_t)r * j->piece * 8;
            e = hipEventRecord(j->kev[r][0], j->s);
            if (e == hipSuccess) e = launch_fs_contrib(j->src + i0 * unit, n, dc, j->s);
            if (e == hipSuccess) e = hipEventRecord(j->kev[r][1], j->s);
            if (e == hipSuccess)
                e = hipMemcpyAsync(j->hC[r], dc, n * 64, hipMemcpyDeviceToHost, j->s);
        }
        if (e == hipSuccess) e = hipEventRecord(j->ev[r], j->s);
        if (e != hipSuccess) fail_here(e, "file-sum piece");
        return e == hipSuccess;
    };
    for (uint64_t i = 0; i < std::min<uint64_t>(np, FsJob::kRing); ++i)
        if (!issue(i)) return;
    for (uint64_t i = 0; i < np; ++i) {
        const int r = (int)(i % FsJob::kRing);
        const hipError_t e = hipEventSynchronize(j->ev[r]);
        if (e != hipSuccess) return fail_here(e, "file-sum piece wait");
        const uint64_t i0 = i * per, n = std::min(per, items - i0);
        const double c0 = now_ms();
        if (serial) {
            serial_sum_update(ss, j->hC[r], n);
        } else {
            xxh3_chain_rows((const uint64_t *)j->hC[r], n, j->acc);
            float ms = 0;
            if (hipEventElapsedTime(&ms, j->kev[r][0], j->kev[r][1]) == hipSuccess) kms += ms;
            (void)hipGetLastError();
        }
        chain += now_ms() - c0;
        if (i + FsJob::kRing < np && !issue(i + FsJob::kRing)) return;
    }
    if (serial) serial_sum_final(ss, j->digest);
    j->host_ms = chain;
    j->dev_ms = kms;
}

int fs_setup(FsJob &j, int device) {
    if (j.s) return 0;
    j.device = device;
    // the lowest priority: the contribution kernel fills what the walk and
    // signature kernels leave free rather than taking CUs from them
    int least = 0, greatest = 0;
    if (hipDeviceGetStreamPriorityRange(&least, &greatest) != hipSuccess) {
        (void)hipGetLastError();
        least = 0;
    }
    VS_HIP(hipStreamCreateWithPriority(&j.s, hipStreamNonBlocking, least));
    VS_HIP(hipEventCreateWithFlags(&j.ev_in, hipEventDisableTiming));
    for (auto &e : j.ev) VS_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    for (auto &k : j.kev)
        for (auto &e : k) VS_HIP(hipEventCreate(&e));
    if (!(j.hlast = (uint8_t *)pinned_alloc(2048))) return fail(VS_ERR_NOMEM, "pinned tail buffer");
    return 0;
}

// the job's rings, sized for its piece length (kept across jobs)
int fs_rings(FsJob &j, uint64_t piece, bool serial) {
    if (piece != j.piece || !j.hC[0]) {
        for (auto &p : j.hC) pinned_free(p), p = nullptr;
        j.piece = piece;
        for (auto &p : j.hC)
            if (!(p = (uint8_t *)pinned_alloc(j.piece * 64)))
                return fail(VS_ERR_NOMEM, "pinned file-sum ring");
    }
    // MD5 / XXH64 (and XXH3 of <= 240 bytes) read the source bytes back
    // through the pinned ring only: no device contribution rows
    if (serial) return 0;
    return 0;   // the device ring (piece mode only) is sized in fs_start
}

// waits for the job (if any); the job's status becomes the return value
int fs_finish(FsJob &j) {
    if (!j.active) return 0;
    if (j.th.joinable()) j.th.join();
    const hipError_t e = hipStreamSynchronize(j.s);
    (void)hipGetLastError();
    if (j.rc < 0) {
        const int rc = j.rc;
        j.rc = 0;
        j.active = false;
        return fail(rc, "whole-file checksum: " + j.err);
    }
    if (e != hipSuccess) {
        j.active = false;
        return fail_hip(e, "whole-file checksum stream", __FILE__, __LINE__);
    }
    return 0;
}

void fs_release(FsJob &j) {
    if (j.th.joinable()) j.th.join();
    if (j.s) (void)hipStreamSynchronize(j.s);
    j.dma.release();
    j.rows.release();
    pinned_free(j.hrows);   // a copy still held by the job (the pool frees the rest)
    j.hrows = nullptr;
    j.hrows_cap = 0;
    for (auto &p : j.hC) pinned_free(p), p = nullptr;
    pinned_free(j.hlast);
    j.hlast = nullptr;
    j.dC.release();
    for (auto &e : j.ev)
        if (e) (void)hipEventDestroy(e), e = nullptr;
    for (auto &k : j.kev)
        for (auto &e : k)
            if (e) (void)hipEventDestroy(e), e = nullptr;
    if (j.ev_in) (void)hipEventDestroy(j.ev_in), j.ev_in = nullptr;
    if (j.s) (void)hipStreamDestroy(j.s), j.s = nullptr;
    j.active = false;
}

void fs_account(vs_rsync *h, const FsJob &j) {
    h->kms[4] += j.dev_ms;
    h->kn[4] += 1;
    h->fs_dev_ms = j.dev_ms;
    h->fs_host_ms = j.host_ms;
}

// the job's pinned row copy back to the handle's pool (its thread has been
// joined: every DMA into it has landed)
void fs_rows_put(vs_rsync *h, FsJob &j) {
    if (!j.hrows) return;
    if (j.th.joinable()) j.th.join();
    h->fs_pool.push_back({j.hrows, j.hrows_cap});
    j.hrows = nullptr;
    j.hrows_cap = 0;
}

// whole: the digest of the file p[0, len); else the accumulators after the
// whole blocks p[0, len) (len a multiple of 1024) chained from acc_in.  The
// job is the FIFO's next slot, or sync (the blocking form's own job, outside
// the FIFO, so it neither waits for nor counts against the jobs in flight).
int fs_start(vs_rsync *h, const uint8_t *p, uint64_t len, int csum, bool whole,
             const uint64_t *acc_in, FsJob *sync = nullptr) {
    if (!sync && h->fs_tail - h->fs_head == vs_rsync::kFsJobs)
        return fail(VS_ERR_STATE, "4 whole-file checksums in flight: wait for one first");
    FsJob &j = sync ? *sync : h->fs[h->fs_tail % vs_rsync::kFsJobs];
    const bool xxh3 = csum == VS_CSUM_XXH3_64 || csum == VS_CSUM_XXH3_128;
    const bool serial = whole && (!xxh3 || len <= 240);
    VS_TRY(fs_setup(j, h->device));
    VS_TRY(fs_rings(j, h->fs_piece ? h->fs_piece : (1ull << 18), serial));
    j.whole = whole;
    j.csum = csum;
    j.len = len;
    j.src = p;
    j.rc = 0;
    j.err.clear();
    j.host_ms = j.dev_ms = 0;
    j.t_call = now_ms();
    j.serial = serial;
    // after the caller's null-stream work and this handle's queued work
    VS_HIP(hipEventRecord(j.ev_in, h->stream));
    VS_HIP(hipStreamWaitEvent(j.s, j.ev_in, 0));
    j.rows_first = false;
    if (j.serial) {
        j.nb = 0;
    } else {
        j.nb = whole ? (len - 1) / 1024 : len / 1024;
        if (whole || !acc_in) xxh3_init_acc(j.acc);
        else memcpy(j.acc, acc_in, 64);
        // rows first unless VS_OPT_FILE_SUM_PIECE asks for the piece ring (a
        // nonzero piece forces it: tests reach the ring path that files over
        // kRowsCap, a failed pin and hosts without the DMA path take)
        j.rows_first = h->fs_piece == 0 && j.nb > 0 && j.nb * 64 <= FsJob::kRowsCap &&
                       j.dma.init(j.device);
        if (j.rows_first) {
            // The pinned copy of the rows: the smallest pooled one that fits,
            // else a new one within the handle's bound, else the piece ring.
            // Page-locking 4 GiB takes ~175 ms on the caller's thread, so the
            // first allocation also pools copies for the jobs that usually
            // follow it in flight (profiles/r05_r7/queued), within the bound.
            const uint64_t need = j.nb * 64;
            fs_rows_put(h, j);   // (a job that was never waited for)
            size_t best = h->fs_pool.size();
            for (size_t i = 0; i < h->fs_pool.size(); ++i)
                if (h->fs_pool[i].second >= need &&
                    (best == h->fs_pool.size() || h->fs_pool[i].second < h->fs_pool[best].second))
                    best = i;
            if (best == h->fs_pool.size()) {
                // free pooled copies too small to serve, then pin within the bound
                for (size_t i = h->fs_pool.size(); i-- > 0;)
                    if (h->fs_pinned + need > FsJob::kPinnedRowsCap) {
                        pinned_free(h->fs_pool[i].first);
                        h->fs_pinned -= h->fs_pool[i].second;
                        h->fs_pool.erase(h->fs_pool.begin() + (long)i);
                    }
                const bool first = h->fs_pinned == 0;
                for (uint32_t k = 0; k < (first && !sync ? vs_rsync::kFsJobs - 1 : 1u); ++k) {
                    if (h->fs_pinned + need > FsJob::kPinnedRowsCap) break;
                    uint8_t *b = (uint8_t *)pinned_alloc((size_t)need);
                    if (!b) break;
                    h->fs_pinned += need;
                    h->fs_pool.push_back({b, need});
                }
                best = h->fs_pool.empty() || h->fs_pool.back().second < need ? h->fs_pool.size()
                                                                              : h->fs_pool.size() - 1;
            }
            if (best < h->fs_pool.size()) {
                j.hrows = h->fs_pool[best].first;
                j.hrows_cap = h->fs_pool[best].second;
                h->fs_pool.erase(h->fs_pool.begin() + (long)best);
            }
            j.rows_first = j.hrows != nullptr;   // else the bounded piece ring
        }
        if (j.rows_first) {
            // all rows now, on the handle's stream: after the caller's queued
            // work and ahead of whatever it queues next (the signatures, the
            // walk).  On the job's low-priority stream the kernel ran beside
            // the caller's next kernels and held CUs their small follow-up
            // launches then waited for (the sum-table copy: 1 -> 10 ms).
            VS_TRY(j.rows.ensure((size_t)j.nb * 64));
            VS_HIP(hipEventRecord(j.kev[0][0], h->stream));
            VS_HIP(launch_fs_contrib(p, j.nb, j.rows.as<uint64_t>(), h->stream));
            VS_HIP(hipEventRecord(j.kev[0][1], h->stream));
        } else {
            VS_TRY(j.dC.ensure((size_t)FsJob::kRing * j.piece * 64));
            if (whole) {   // the last partial block, last stripe: read back for the finish
                const uint64_t keep = std::min<uint64_t>(len, 1088);
                VS_HIP(hipMemcpyAsync(j.hlast, p + len - keep, keep, hipMemcpyDeviceToHost, j.s));
            }
        }
    }
    if (j.th.joinable()) j.th.join();   // (fs_finish joined it; never terminate())
    if (j.serial ? len > 0 : j.nb > 0) {
        j.th = std::thread(fs_thread, &j);
    } else if (j.serial) {   // an empty file: nothing to read back
        SerialSum ss;
        serial_sum_init(ss, csum);
        serial_sum_final(ss, j.digest);
    }
    j.active = true;
    if (!sync) h->fs_tail++;
    return 0;
}

// the finished job's digest (whole files)
void fs_digest(const FsJob &j, uint8_t out[16]) {
    memset(out, 0, 16);
    const int n = (j.csum == VS_CSUM_MD5 || j.csum == VS_CSUM_XXH3_128) ? 16 : 8;
    if (j.serial) {
        memcpy(out, j.digest, (size_t)n);
    } else {
        uint8_t o[16];
        xxh3_file_finish(j.hlast, j.len, j.acc, j.csum, o);
        memcpy(out, o, (size_t)n);
    }
}

// ---- streamed forms (MatchStream / SigStream) --------------------------------
// n caller bytes to device dst on copy stream cs: pinned caller memory by DMA
// (*dma set: the call waits for it before returning -- the caller owns the
// buffer), pageable memory through the stream's own staging buffers
int feed_copy(Stager &st, hipStream_t cs, uint8_t *dst, const uint8_t *src, size_t n, bool *dma,
              uint64_t *pinned_bytes, uint64_t *staged_bytes) {
    if (!n) return 0;
    if (host_range_pinned(src, n)) {
        VS_HIP(hipMemcpyAsync(dst, src, n, hipMemcpyHostToDevice, cs));
        *dma = true;
        *pinned_bytes += n;
        return 0;
    }
    *staged_bytes += n;
    return st.h2d(dst, src, n, cs);
}

int stream_mk(hipStream_t *cs, hipEvent_t *ev, uint32_t nev) {
    if (!*cs) VS_HIP(hipStreamCreateWithFlags(cs, hipStreamNonBlocking));
    for (uint32_t i = 0; i < nev; ++i)
        if (!ev[i]) VS_HIP(hipEventCreateWithFlags(&ev[i], hipEventDisableTiming));
    return 0;
}

void ms_release(vs_rsync *h) {
    MatchStream *m = h->mst;
    if (!m) return;
    {
        std::lock_guard<std::mutex> lk(m->mu);
        m->stop = true;
    }
    m->cv.notify_all();
    if (m->th.joinable()) m->th.join();
    if (m->cs) (void)hipStreamSynchronize(m->cs);
    for (auto &b : m->slot) b.release();
    for (auto &e : m->ev)
        if (e) (void)hipEventDestroy(e);
    m->stage.release();
    m->dC.release();
    pinned_free(m->hC);
    if (m->cs) (void)hipStreamDestroy(m->cs);
    delete m;
    h->mst = nullptr;
}

// the walk thread: piece k from the previous piece's exit, as its bytes arrive
void ms_worker(vs_rsync *h, MatchStream *m) {
    int64_t entry = 0;
    int32_t want = 0;
    for (int64_t k = 0; k < m->np; ++k) {
        {
            const double t0 = now_ms();
            std::unique_lock<std::mutex> lk(m->mu);
            m->cv.wait(lk, [&] { return m->stop || m->complete > k; });
            m->idle_ms += now_ms() - t0;
            if (m->stop) return;
        }
        const double t0 = now_ms();
        const int64_t lo = k * m->piece, hi = std::min(lo + m->piece, m->flen);
        const int64_t dhi = std::min(hi + m->halo, m->flen);
        int rc = rs_dev(h);
        int64_t nm = 0, fa = 0, hashed = 0;
        if (!rc && hipStreamWaitEvent(h->stream, m->ev[k % m->ring], 0) != hipSuccess)
            rc = fail_hip(hipGetLastError(), "hipStreamWaitEvent (streamed piece)", __FILE__,
                          __LINE__);
        double fms = 0;
        if (!rc && m->fs_xxh3) {   // R7: this piece's whole blocks of the file
            const double f0 = now_ms();
            const uint64_t nbf = (uint64_t)(m->flen - 1) / 1024;
            const uint64_t b0 = (uint64_t)lo / 1024, b1 = std::min<uint64_t>((uint64_t)hi / 1024, nbf);
            if (b1 > b0) {
                hipError_t e = launch_fs_contrib(m->slot[k % m->ring].as<uint8_t>(), b1 - b0,
                                                 m->dC.as<uint64_t>(), h->stream);
                if (e == hipSuccess)
                    e = hipMemcpyAsync(m->hC, m->dC.p, (b1 - b0) * 64, hipMemcpyDeviceToHost,
                                       h->stream);
                if (e == hipSuccess) e = hipStreamSynchronize(h->stream);
                if (e != hipSuccess) rc = fail_hip(e, "streamed file-sum piece", __FILE__, __LINE__);
                else xxh3_chain_rows(m->hC, b1 - b0, m->acc);
            }
            fms = now_ms() - f0;
        }
        if (!rc && entry < hi) {
            int64_t x = 0;
            int32_t xw = 0;
            if (!rc)
                rc = match_scan(h, m->slot[k % m->ring].p, dhi - lo, lo, m->flen, lo, hi, &x, &xw,
                                true, entry, want);
            if (!rc) rc = match_finish(h, &nm);
            if (!rc) {
                fa = h->st_fa;
                hashed = h->st_hashed;
                entry = x;
                want = xw;
            }
        }
        std::lock_guard<std::mutex> lk(m->mu);
        if (rc < 0) {
            m->rc = rc;
            m->err = vs_last_error();
            m->stop = true;
            m->cv.notify_all();
            return;
        }
        if (nm) m->out.insert(m->out.end(), h->matches.begin(), h->matches.begin() + nm);
        m->fa += fa;
        m->hashed += hashed;
        m->walked = k + 1;
        m->walk_ms += now_ms() - t0 - fms;
        m->fs_ms += fms;
        m->cv.notify_all();
    }
}

int ms_error(MatchStream *m) {
    std::lock_guard<std::mutex> lk(m->mu);
    if (m->rc < 0) return fail(m->rc, "streamed match walk: " + m->err);
    return 0;
}

int ms_build(vs_rsync *h, MatchStream *m, int64_t flen, int fcsum, uint64_t piece, uint32_t ring);

int ms_begin(vs_rsync *h, int64_t flen, int fcsum, uint64_t piece, uint32_t ring) {
    if (!h->loaded) return fail(VS_ERR_STATE, "vs_rsync_match_begin before vs_rsync_load_sums");
    if (flen < 0) return fail(VS_ERR_ARG, "negative file length");
    if (fcsum) VS_TRY(check_csum(fcsum));
    if (!piece) piece = 256ull << 20;
    if (!ring) ring = 3;
    if (ring < 2 || ring > MatchStream::kMaxRing || piece < (1u << 20) || (piece & 1023))
        return fail(VS_ERR_ARG, "piece must be >= 1 MiB and a multiple of 1024, ring 2..8");
    VS_TRY(rs_dev(h));
    ms_release(h);
    h->mst = new MatchStream();
    // a stream that fails to come up is released whole: no
    // half-built ring without its walk thread is left behind for _feed/_next
    const int rc = ms_build(h, h->mst, flen, fcsum, piece, ring);
    if (rc < 0) ms_release(h);
    return rc;
}

int ms_build(vs_rsync *h, MatchStream *m, int64_t flen, int fcsum, uint64_t piece, uint32_t ring) {
    m->flen = flen;
    m->halo = h->blength - 1;
    // a piece never shorter than the walk's halo; small files get one slot's worth
    m->piece = (int64_t)std::max<uint64_t>(piece, ((uint64_t)h->blength + 1023) & ~1023ull);
    m->np = flen ? (flen + m->piece - 1) / m->piece : 0;
    m->ring = ring;
    // slots k % ring for the pieces there are (a small file: one)
    const uint32_t nslot = (uint32_t)std::min<int64_t>(ring, std::max<int64_t>(m->np, 1));
    const size_t sb = (size_t)std::min<int64_t>(m->piece + m->halo, std::max<int64_t>(flen, 16)) + 16;
    VS_TRY(stream_mk(&m->cs, m->ev, nslot));
    for (uint32_t i = 0; i < nslot; ++i) VS_TRY(m->slot[i].ensure(sb));
    m->fcsum = fcsum;
    m->fs_xxh3 = (fcsum == VS_CSUM_XXH3_64 || fcsum == VS_CSUM_XXH3_128) && flen > 240;
    if (m->fs_xxh3) {
        xxh3_init_acc(m->acc);
        const uint64_t rows = (uint64_t)m->piece / 1024;
        VS_TRY(m->dC.ensure(rows * 64));
        if (!(m->hC = (uint64_t *)pinned_alloc(rows * 64)))
            return fail(VS_ERR_NOMEM, "pinned file-sum rows");
    } else if (fcsum) {
        serial_sum_init(m->ss, fcsum);
    }
    h->matches.clear();
    h->st_cand = h->st_fa = h->st_hashed = 0;
    h->st_rounds = 0;
    if (m->np) {
        try {
            m->th = std::thread(ms_worker, h, m);
        } catch (const std::exception &e) {
            return fail(VS_ERR_NOMEM, std::string("streamed match walk thread: ") + e.what());
        }
    }
    return 0;
}

int ms_feed(vs_rsync *h, const uint8_t *p, size_t n) {
    MatchStream *m = h->mst;
    if (!m) return fail(VS_ERR_STATE, "vs_rsync_match_feed before vs_rsync_match_begin");
    VS_TRY(ms_error(m));
    if (n && !p) return fail(VS_ERR_ARG, "null buffer");
    if ((int64_t)n > m->flen - m->fed) return fail(VS_ERR_ARG, "fed past the file length given to begin");
    VS_TRY(rs_dev(h));
    bool dma = false;
    while (n) {
        const int64_t k = m->fed / m->piece, off = m->fed - k * m->piece;
        const size_t take = (size_t)std::min<int64_t>((int64_t)n, m->piece - off);
        if (k >= m->ring) {   // slot k % ring: free once piece k - ring is walked
            const double t0 = now_ms();
            std::unique_lock<std::mutex> lk(m->mu);
            m->cv.wait(lk, [&] { return m->stop || m->walked > k - m->ring; });
            m->feed_wait_ms += now_ms() - t0;
            if (m->stop) {
                lk.unlock();
                VS_TRY(ms_error(m));
                return fail(VS_ERR_STATE, "streamed match stopped");
            }
        }
        uint8_t *dst = m->slot[k % m->ring].as<uint8_t>() + off;
        VS_TRY(feed_copy(m->stage, m->cs, dst, p, take, &dma, &m->pinned_bytes, &m->staged_bytes));
        if (m->fcsum && !m->fs_xxh3) serial_sum_update(m->ss, p, take);
        const int64_t keep = std::min<int64_t>(m->flen, 1088), t0 = m->flen - keep;
        if (m->fs_xxh3 && m->fed + (int64_t)take > t0) {   // the file's last bytes, for the finish
            const int64_t a = std::max(m->fed, t0);
            memcpy(m->last + (a - t0), p + (a - m->fed), (size_t)(m->fed + (int64_t)take - a));
        }
        if (k > 0 && off < m->halo) {   // also piece k-1's halo
            const size_t hn = (size_t)std::min<int64_t>((int64_t)take, m->halo - off);
            VS_HIP(hipMemcpyAsync(m->slot[(k - 1) % m->ring].as<uint8_t>() + m->piece + off, dst, hn,
                                  hipMemcpyDeviceToDevice, m->cs));
        }
        m->fed += (int64_t)take;
        p += take;
        n -= take;
        // pieces whose bytes and halo are now all queued
        int64_t q = m->queued;
        while (q < m->np && m->fed >= std::min((q + 1) * m->piece + m->halo, m->flen)) {
            VS_HIP(hipEventRecord(m->ev[q % m->ring], m->cs));
            ++q;
        }
        if (q != m->queued) {
            m->queued = q;
            {
                std::lock_guard<std::mutex> lk(m->mu);
                m->complete = q;
            }
            m->cv.notify_all();
        }
    }
    if (dma) VS_HIP(hipStreamSynchronize(m->cs));   // the caller's pinned bytes are copied
    return 0;
}

// matches found so far, in order; with wait: blocks until at least one is
// found or the walk is over.  VS_EOF once the last has been returned.
int ms_next(vs_rsync *h, vs_match *out, size_t cap, size_t *n_out, bool wait) {
    MatchStream *m = h->mst;
    *n_out = 0;
    if (!m) return fail(VS_ERR_STATE, "vs_rsync_match_next before vs_rsync_match_begin");
    std::unique_lock<std::mutex> lk(m->mu);
    if (wait)
        m->cv.wait(lk, [&] { return m->stop || m->head < m->out.size() || m->walked == m->np; });
    if (m->rc < 0) {
        lk.unlock();
        return ms_error(m);
    }
    const size_t n = std::min(cap, m->out.size() - m->head);
    if (n) memcpy(out, m->out.data() + m->head, n * sizeof(vs_match));
    m->head += n;
    *n_out = n;
    if (!n && m->walked == m->np && m->fed == m->flen) return VS_EOF;
    return 0;
}

int ms_end(vs_rsync *h, int64_t *n_matches, int64_t *false_alarms, uint8_t *file_sum) {
    MatchStream *m = h->mst;
    if (!m) return fail(VS_ERR_STATE, "vs_rsync_match_end before vs_rsync_match_begin");
    if (m->fed != m->flen)
        return fail(VS_ERR_STATE, "vs_rsync_match_end after " + std::to_string(m->fed) + " of " +
                                      std::to_string(m->flen) + " bytes");
    {
        std::unique_lock<std::mutex> lk(m->mu);
        m->cv.wait(lk, [&] { return m->stop || m->walked == m->np; });
    }
    if (m->th.joinable()) m->th.join();
    VS_TRY(ms_error(m));
    std::lock_guard<std::mutex> lk(m->mu);
    // the handle's counters and match list describe the whole file now
    h->st_fa = m->fa;
    h->st_hashed = m->hashed;
    h->matches.assign(m->out.begin(), m->out.end());
    if (n_matches) *n_matches = (int64_t)m->out.size();
    if (false_alarms) *false_alarms = m->fa;
    if (file_sum) {
        memset(file_sum, 0, 16);
        if (!m->fcsum) return fail(VS_ERR_STATE, "the stream was begun without a file checksum");
        uint8_t o[16];
        if (m->fs_xxh3) {
            xxh3_file_finish(m->last, (uint64_t)m->flen, m->acc, m->fcsum, o);
        } else {
            SerialSum ss = m->ss;   // _end may be called again
            serial_sum_final(ss, o);
        }
        memcpy(file_sum, o, (m->fcsum == VS_CSUM_MD5 || m->fcsum == VS_CSUM_XXH3_128) ? 16 : 8);
    }
    return 0;
}

void ss_release(vs_rsync *h) {
    SigStream *s = h->sst;
    if (!s) return;
    if (s->cs) (void)hipStreamSynchronize(s->cs);
    if (h->stream) (void)hipStreamSynchronize(h->stream);
    for (auto &b : s->slot) b.release();
    s->d1.release();
    s->d2.release();
    for (auto &e : s->ev_in)
        if (e) (void)hipEventDestroy(e);
    for (auto &e : s->ev_done)
        if (e) (void)hipEventDestroy(e);
    pinned_free(s->h1);
    pinned_free(s->h2);
    s->stage.release();
    if (s->cs) (void)hipStreamDestroy(s->cs);
    delete s;
    h->sst = nullptr;
}

int ss_build(SigStream *s, int64_t len, int32_t blength, int32_t s2length, int csum, uint32_t seed,
             uint64_t piece, uint32_t ring, int64_t count);

int ss_begin(vs_rsync *h, int64_t len, int32_t blength, int32_t s2length, int csum, uint32_t seed,
             uint64_t piece, uint32_t ring) {
    VS_TRY(check_csum(csum));
    if (len < 0 || blength <= 0 || s2length < 1 || s2length > 16)
        return fail(VS_ERR_ARG, "bad length, blength or s2length");
    if (!piece) piece = 256ull << 20;
    if (!ring) ring = 3;
    if (ring < 2 || ring > SigStream::kMaxRing) return fail(VS_ERR_ARG, "ring must be 2..8");
    const int64_t count = len / blength + (len % blength != 0);
    if (count > INT32_MAX) return fail(VS_ERR_ARG, "block count overflows int32");
    VS_TRY(rs_dev(h));
    ss_release(h);
    h->sst = new SigStream();
    const int rc = ss_build(h->sst, len, blength, s2length, csum, seed, piece, ring, count);
    if (rc < 0) ss_release(h);   // as ms_begin: nothing half-built stays on the handle
    return rc;
}

int ss_build(SigStream *s, int64_t len, int32_t blength, int32_t s2length, int csum, uint32_t seed,
             uint64_t piece, uint32_t ring, int64_t count) {
    s->len = len;
    s->blength = blength;
    s->s2length = s2length;
    s->remainder = (int32_t)(len % blength);
    s->csum = csum;
    s->seed = seed;
    s->count = count;
    s->piece = std::max<int64_t>((int64_t)piece / blength, 1) * blength;
    s->np = len ? (len + s->piece - 1) / s->piece : 0;
    s->ring = ring;
    const uint32_t nslot = (uint32_t)std::min<int64_t>(ring, std::max<int64_t>(s->np, 1));
    VS_TRY(stream_mk(&s->cs, s->ev_in, nslot));
    VS_TRY(stream_mk(&s->cs, s->ev_done, nslot));
    const size_t sb = (size_t)std::min<int64_t>(s->piece, std::max<int64_t>(len, 16)) + 16;
    for (uint32_t i = 0; i < nslot; ++i) VS_TRY(s->slot[i].ensure(sb));
    const size_t c = (size_t)std::max<int64_t>(count, 1);
    VS_TRY(s->d1.ensure(c * 4));
    VS_TRY(s->d2.ensure(c * s2length));
    if (!(s->h1 = (uint32_t *)pinned_alloc(c * 4)) || !(s->h2 = (uint8_t *)pinned_alloc(c * s2length)))
        return fail(VS_ERR_NOMEM, "pinned signature read-back arrays");
    return 0;
}

// piece k's bytes are queued: sign it on the handle's stream, read its sums back
int ss_launch(vs_rsync *h, SigStream *s, int64_t k) {
    const int64_t lo = k * s->piece, hi = std::min(lo + s->piece, s->len);
    const int64_t b0 = lo / s->blength;
    RsSigArgs a{};
    a.data = s->slot[k % s->ring].as<uint8_t>();
    a.len = (uint64_t)(hi - lo);
    a.count = (uint64_t)((hi - lo + s->blength - 1) / s->blength);
    a.blength = (uint32_t)s->blength;
    a.remainder = (uint32_t)((hi - lo) % s->blength);
    a.s2length = (uint32_t)s->s2length;
    a.csum_type = s->csum;
    a.seed = s->seed;
    a.sum1 = s->d1.as<uint32_t>() + b0;
    a.sum2 = s->d2.as<uint8_t>() + b0 * s->s2length;
    VS_HIP(hipEventRecord(s->ev_in[k % s->ring], s->cs));
    VS_HIP(hipStreamWaitEvent(h->stream, s->ev_in[k % s->ring], 0));
    VS_HIP(launch_rs_signatures(a, h->stream));
    VS_HIP(hipMemcpyAsync(s->h1 + b0, a.sum1, a.count * 4, hipMemcpyDeviceToHost, h->stream));
    VS_HIP(hipMemcpyAsync(s->h2 + b0 * s->s2length, a.sum2, a.count * s->s2length,
                          hipMemcpyDeviceToHost, h->stream));
    VS_HIP(hipEventRecord(s->ev_done[k % s->ring], h->stream));
    return 0;
}

// pieces whose sums are on the host: without wait, those that are done now
int ss_collect(SigStream *s, bool wait) {
    while (s->done < s->launched) {
        hipEvent_t e = s->ev_done[s->done % s->ring];
        if (wait) {
            VS_HIP(hipEventSynchronize(e));
        } else {
            const hipError_t q = hipEventQuery(e);
            if (q == hipErrorNotReady) {
                (void)hipGetLastError();
                break;
            }
            if (q != hipSuccess) return fail_hip(q, "signature piece", __FILE__, __LINE__);
        }
        ++s->done;
        if (wait) break;   // one piece per wait
    }
    return 0;
}

int ss_feed(vs_rsync *h, const uint8_t *p, size_t n) {
    SigStream *s = h->sst;
    if (!s) return fail(VS_ERR_STATE, "vs_rsync_sig_feed before vs_rsync_sig_begin");
    if (n && !p) return fail(VS_ERR_ARG, "null buffer");
    if ((int64_t)n > s->len - s->fed) return fail(VS_ERR_ARG, "fed past the length given to begin");
    VS_TRY(rs_dev(h));
    bool dma = false;
    while (n) {
        const int64_t k = s->fed / s->piece, off = s->fed - k * s->piece;
        const size_t take = (size_t)std::min<int64_t>((int64_t)n, s->piece - off);
        while (k >= s->done + s->ring) VS_TRY(ss_collect(s, true));   // slot k % ring is free
        VS_TRY(feed_copy(s->stage, s->cs, s->slot[k % s->ring].as<uint8_t>() + off, p, take, &dma,
                         &s->pinned_bytes, &s->staged_bytes));
        s->fed += (int64_t)take;
        p += take;
        n -= take;
        if (s->fed == std::min((k + 1) * s->piece, s->len)) {
            VS_TRY(ss_launch(h, s, k));
            s->launched = k + 1;
        }
    }
    if (dma) VS_HIP(hipStreamSynchronize(s->cs));
    return 0;
}

int ss_next(vs_rsync *h, uint32_t *sum1, uint8_t *sum2, size_t cap, size_t *n_out) {
    SigStream *s = h->sst;
    *n_out = 0;
    if (!s) return fail(VS_ERR_STATE, "vs_rsync_sig_next before vs_rsync_sig_begin");
    VS_TRY(rs_dev(h));
    VS_TRY(ss_collect(s, false));
    const int64_t per = s->piece / s->blength;
    // nothing ready but a piece in flight: wait for the oldest (with none in
    // flight, more input is needed first)
    if (std::min(s->done * per, s->count) == s->returned && s->done < s->launched)
        VS_TRY(ss_collect(s, true));
    const int64_t avail = std::min(s->done * per, s->count) - s->returned;
    const size_t n = (size_t)std::min<int64_t>((int64_t)cap, avail);
    if (n) {
        memcpy(sum1, s->h1 + s->returned, n * 4);
        memcpy(sum2, s->h2 + s->returned * s->s2length, n * (size_t)s->s2length);
        s->returned += (int64_t)n;
    }
    *n_out = n;
    if (!n && s->returned == s->count && s->fed == s->len) return VS_EOF;
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
        hipEventCreate(&h->kev[0]) != hipSuccess || hipEventCreate(&h->kev[1]) != hipSuccess ||
        !(h->pinned = (uint64_t *)pinned_alloc(64))) {
        const hipError_t e = hipGetLastError();
        vs_rsync_close(h);
        return fail(VS_ERR_HIP, std::string("stream / event / pinned word creation failed: ") +
                                    hipGetErrorName(e));
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
    ms_release(h);
    ss_release(h);
    for (FsJob &j : h->fs) fs_release(j);
    fs_release(h->fs_sync);
    for (auto &b : h->fs_pool) pinned_free(b.first);
    h->fs_pool.clear();
    h->fs_pinned = 0;
    if (h->stream) (void)hipStreamSynchronize(h->stream);
    for (DevBuf *b : {&h->d_sum1, &h->d_keys, &h->d_tkey, &h->d_dir, &h->d_filt, &h->d_tmp, &h->d_bkt, &h->px,
                      &h->pt, &h->pxs, &h->pts, &h->partials, &h->c_off, &h->c_sum, &h->c_off2,
                      &h->c_sum2, &h->n_cand, &h->sort_tmp, &h->v_off, &h->v_len, &h->v_out,
                      &h->d_flag, &h->d_sum2p, &h->d_sum2tmp, &h->w_spec_off, &h->w_spec_idx,
                      &h->w_spec_fab, &h->w_spec_n, &h->w_spec_fa, &h->w_spec_exit,
                      &h->w_spec_exitw, &h->w_fin_entry, &h->w_fin_entryw, &h->w_fin_from,
                      &h->w_fin_n, &h->w_fin_fa, &h->w_fin_off, &h->w_fin_idx, &h->w_fin_fab,
                      &h->w_exit[0], &h->w_exit[1], &h->w_exitw[0], &h->w_exitw[1], &h->w_ctl, &h->w_prof, &h->rc_pieces,
                      &h->wc_cnt, &h->wc_pos, &h->wc_part, &h->wc_out})
        b->release();
    pinned_free(h->pinned);
    if (h->wc_host) (void)hipHostFree(h->wc_host);
    h->stage.release();
    PinnedVec<uint64_t>().swap(h->h_off);
    PinnedVec<uint32_t>().swap(h->h_sum);
    PinnedVec<uint8_t>().swap(h->h_flag);
    if (h->ev_null) (void)hipEventDestroy(h->ev_null);
    for (hipEvent_t e : h->kev)
        if (e) (void)hipEventDestroy(e);
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
    KernelTimer kt(h, 2);
    VS_HIP(launch_rs_signatures(a, h->stream));
    kt.stop();
    VS_HIP(hipStreamSynchronize(h->stream));
    kt.fold();
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
    VS_TRY(h->d_sum1.ensure((size_t)std::max(count, 1) * 4));
    VS_TRY(h->d_sum2p.ensure((size_t)std::max(count, 1) * 16));
    VS_TRY(h->d_sum2tmp.ensure((size_t)std::max(count, 1) * s2length));
    if (count) {
        VS_TRY(h->stage.h2d(h->d_sum1.p, sum1, (size_t)count * 4, h->stream));
        VS_TRY(h->stage.h2d(h->d_sum2tmp.p, sum2, (size_t)count * s2length, h->stream));
        VS_HIP(launch_rs_pad_sum2(h->d_sum2tmp.as<uint8_t>(), (uint32_t)count, (uint32_t)s2length,
                                  h->d_sum2p.as<uint64_t>(), h->stream));
    }
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
    VS_TRY(h->d_sum1.ensure((size_t)std::max(count, 1) * 4));
    VS_TRY(order_after_null(h));
    VS_TRY(h->d_sum2p.ensure((size_t)std::max(count, 1) * 16));
    if (count)   // sum1 copied and sum2 padded in one kernel
        VS_HIP(launch_rs_pad_sum2(dev_sum2, (uint32_t)count, (uint32_t)s2length,
                                  h->d_sum2p.as<uint64_t>(), h->stream, dev_sum1,
                                  h->d_sum1.as<uint32_t>()));
    VS_TRY(build_table(h));
    h->ms[1] = now_ms() - t0;
    return 0;
}

VS_API int vs_rsync_match_device(vs_rsync *h, const void *dev_src, int64_t len,
                                 int64_t *n_matches) {
    if (!h) return fail(VS_ERR_ARG, "null handle");
    return match_device(h, dev_src, len, n_matches);
}

VS_API int vs_rsync_match_scan(vs_rsync *h, const void *dev_src, int64_t len, int64_t origin,
                               int64_t file_len, int64_t own_lo, int64_t own_hi,
                               int64_t *exit_off, int32_t *exit_want) {
    if (!h) return fail(VS_ERR_ARG, "null handle");
    return match_scan(h, dev_src, len, origin, file_len, own_lo, own_hi, exit_off, exit_want);
}

VS_API int vs_rsync_match_stitch(vs_rsync *h, int64_t entry, int32_t want_i, int64_t *exit_off,
                                 int32_t *exit_want) {
    if (!h) return fail(VS_ERR_ARG, "null handle");
    return match_stitch(h, entry, want_i, exit_off, exit_want);
}

VS_API int vs_rsync_match_finish(vs_rsync *h, int64_t *n_matches) {
    if (!h) return fail(VS_ERR_ARG, "null handle");
    return match_finish(h, n_matches);
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

VS_API int vs_rsync_file_sum_start(vs_rsync *h, const void *dev_src, int64_t len, int csum_type) {
    if (!h || len < 0 || (len && !dev_src)) return fail(VS_ERR_ARG, "bad arguments");
    if (csum_type != VS_CSUM_MD5 && csum_type != VS_CSUM_XXH64 && csum_type != VS_CSUM_XXH3_64 &&
        csum_type != VS_CSUM_XXH3_128)
        return fail(VS_ERR_ARG, "unsupported checksum type");
    VS_TRY(rs_dev(h));
    VS_TRY(order_after_null(h));
    return fs_start(h, (const uint8_t *)dev_src, (uint64_t)len, csum_type, true, nullptr);
}

VS_API int vs_rsync_file_sum_wait(vs_rsync *h, uint8_t out[16]) {
    if (!h || !out) return fail(VS_ERR_ARG, "bad arguments");
    if (h->fs_head == h->fs_tail) return fail(VS_ERR_STATE, "no whole-file checksum in flight");
    FsJob &j = h->fs[h->fs_head % vs_rsync::kFsJobs];
    if (!j.whole) return fail(VS_ERR_STATE, "the oldest checksum job is a block range");
    VS_TRY(rs_dev(h));
    h->fs_head++;
    const int rc = fs_finish(j);   // joins the job's thread, syncs its stream
    fs_rows_put(h, j);
    j.active = false;
    VS_TRY(rc);
    fs_account(h, j);
    fs_digest(j, out);
    return 0;
}

// the blocking form runs on its own job and waits for it only: jobs the
// caller already has in flight keep their FIFO order and their count
VS_API int vs_rsync_file_sum(vs_rsync *h, const void *dev_src, int64_t len, int csum_type,
                             uint8_t out[16]) {
    if (!out) return fail(VS_ERR_ARG, "bad arguments");
    if (!h || len < 0 || (len && !dev_src)) return fail(VS_ERR_ARG, "bad arguments");
    if (csum_type != VS_CSUM_MD5 && csum_type != VS_CSUM_XXH64 && csum_type != VS_CSUM_XXH3_64 &&
        csum_type != VS_CSUM_XXH3_128)
        return fail(VS_ERR_ARG, "unsupported checksum type");
    VS_TRY(rs_dev(h));
    VS_TRY(order_after_null(h));
    FsJob &j = h->fs_sync;
    VS_TRY(fs_start(h, (const uint8_t *)dev_src, (uint64_t)len, csum_type, true, nullptr, &j));
    const int rc = fs_finish(j);
    fs_rows_put(h, j);
    j.active = false;
    VS_TRY(rc);
    fs_account(h, j);
    fs_digest(j, out);
    return 0;
}

VS_API int vs_rsync_file_sum_blocks_start(vs_rsync *h, const void *dev_blocks, int64_t nblocks,
                                          const uint64_t acc_in[8]) {
    if (!h || nblocks < 0 || (nblocks && !dev_blocks)) return fail(VS_ERR_ARG, "bad arguments");
    VS_TRY(rs_dev(h));
    VS_TRY(order_after_null(h));
    return fs_start(h, (const uint8_t *)dev_blocks, (uint64_t)nblocks * 1024, VS_CSUM_XXH3_128,
                    false, acc_in);
}

VS_API int vs_rsync_file_sum_blocks_wait(vs_rsync *h, uint64_t acc_out[8]) {
    if (!h || !acc_out) return fail(VS_ERR_ARG, "bad arguments");
    if (h->fs_head == h->fs_tail) return fail(VS_ERR_STATE, "no block-range checksum in flight");
    FsJob &j = h->fs[h->fs_head % vs_rsync::kFsJobs];
    if (j.whole) return fail(VS_ERR_STATE, "the oldest checksum job is a whole file");
    VS_TRY(rs_dev(h));
    h->fs_head++;
    const int rc = fs_finish(j);   // joins the job's thread, syncs its stream
    fs_rows_put(h, j);
    j.active = false;
    VS_TRY(rc);
    fs_account(h, j);
    memcpy(acc_out, j.acc, 64);
    return 0;
}

VS_API int vs_rsync_file_sum_finish(const uint64_t acc[8], const uint8_t *last, int64_t len,
                                    int csum_type, uint8_t out[16]) {
    if (!acc || !last || !out || len <= 240 ||
        (csum_type != VS_CSUM_XXH3_64 && csum_type != VS_CSUM_XXH3_128))
        return fail(VS_ERR_ARG, "bad arguments (XXH3 of a file over 240 bytes)");
    uint8_t o[16];
    xxh3_file_finish(last, (uint64_t)len, acc, csum_type, o);
    memset(out, 0, 16);
    memcpy(out, o, csum_type == VS_CSUM_XXH3_128 ? 16 : 8);
    return 0;
}

VS_API int vs_rsync_file_sum_init(uint64_t acc[8]) {
    if (!acc) return fail(VS_ERR_ARG, "null accumulators");
    xxh3_init_acc(acc);
    return 0;
}

VS_API int vs_rsync_file_sum_timing(vs_rsync *h, double *device_ms, double *host_ms) {
    if (!h) return fail(VS_ERR_ARG, "null handle");
    if (device_ms) *device_ms = h->fs_dev_ms;
    if (host_ms) *host_ms = h->fs_host_ms;
    return 0;
}

VS_API int vs_rsync_reconstruct(vs_rsync *h, void *dev_out, int64_t out_len, const void *dev_basis,
                                int64_t basis_len, int32_t blength, const vs_match *matches,
                                int64_t n_matches, const void *dev_literals, int64_t literal_len) {
    if (!h || out_len < 0 || basis_len < 0 || blength <= 0 || n_matches < 0 || literal_len < 0 ||
        (out_len && !dev_out) || (n_matches && (!matches || !dev_basis)) ||
        (literal_len && !dev_literals))
        return fail(VS_ERR_ARG, "bad arguments");
    // the token stream as pieces, in order (receiver.c receive_data: literal
    // data is written as it comes, token i copies basis block i)
    std::vector<ReconPiece> pc;
    pc.reserve((size_t)n_matches * 2 + 1);
    int64_t pos = 0, lit = 0;
    const int64_t count = (basis_len + blength - 1) / blength;
    for (int64_t k = 0; k < n_matches; ++k) {
        const vs_match m = matches[k];
        if (m.offset < pos || m.block_index < 0 || m.block_index >= count)
            return fail(VS_ERR_ARG, "match list out of order or block index out of range");
        const int64_t bo = (int64_t)m.block_index * blength;
        const int64_t bl = std::min<int64_t>(blength, basis_len - bo);
        if (m.offset + bl > out_len) return fail(VS_ERR_ARG, "match past the end of the file");
        if (m.offset > pos) {
            pc.push_back({(uint64_t)pos, (uint64_t)lit, (uint64_t)(m.offset - pos), 1, 0});
            lit += m.offset - pos;
        }
        pc.push_back({(uint64_t)m.offset, (uint64_t)bo, (uint64_t)bl, 0, 0});
        pos = m.offset + bl;
    }
    if (pos < out_len) {
        pc.push_back({(uint64_t)pos, (uint64_t)lit, (uint64_t)(out_len - pos), 1, 0});
        lit += out_len - pos;
    }
    if (lit != literal_len) return fail(VS_ERR_ARG, "literal bytes do not fill the gaps between matches");
    if (pc.empty()) return 0;
    VS_TRY(rs_dev(h));
    VS_TRY(order_after_null(h));
    VS_TRY(h->rc_pieces.ensure(pc.size() * sizeof(ReconPiece)));
    VS_TRY(h->stage.h2d(h->rc_pieces.p, pc.data(), pc.size() * sizeof(ReconPiece), h->stream));
    VS_HIP(launch_recon((uint8_t *)dev_out, (const uint8_t *)dev_basis, (const uint8_t *)dev_literals,
                        h->rc_pieces.as<ReconPiece>(), pc.size(), h->cus, h->stream));
    VS_HIP(hipStreamSynchronize(h->stream));
    return 0;
}

VS_API int vs_rsync_kernel_time(vs_rsync *h, int which, int reset, double *ms,
                                int64_t *launches) {
    if (!h || which < 0 || which > 4) return fail(VS_ERR_ARG, "bad handle or kernel index");
    if (ms) *ms = h->kms[which];
    if (launches) *launches = h->kn[which];
    if (reset) {
        h->kms[which] = 0;
        h->kn[which] = 0;
    }
    return 0;
}

VS_API int vs_rsync_set_option(vs_rsync *h, int option, int64_t value) {
    if (!h) return fail(VS_ERR_ARG, "null handle");
    switch (option) {
        case VS_OPT_WALK_SEGMENT_BLOCKS:
            if (value < 0 || value > (1 << 20)) return fail(VS_ERR_ARG, "segment length out of range");
            h->seg_blocks = (uint32_t)value;
            return 0;
        case VS_OPT_FILE_SUM_PIECE:
            if (value < 0 || value > (1 << 24)) return fail(VS_ERR_ARG, "file-sum piece out of range");
            for (const FsJob &j : h->fs)
                if (j.active) return fail(VS_ERR_STATE, "file-sum jobs in flight");
            h->fs_piece = (uint64_t)value;
            return 0;
        case VS_OPT_BUCKET_BITS:
            if (value < 0 || value > 26) return fail(VS_ERR_ARG, "bucket bits out of range");
            h->opt_bbits = (uint32_t)value;   // applies to the next load_sums
            return 0;
        case VS_OPT_FA_RECORD:
            if (value < -1 || value > 4096) return fail(VS_ERR_ARG, "false-alarm record out of range");
            h->opt_facap = (int32_t)value;
            return 0;
        case VS_OPT_HOST_WALK:
            h->opt_host_walk = value != 0;
            return 0;
        case VS_OPT_WALK_FLUSH_WINDOWS:
            if (value != 0 && value != 4 && value != 16)
                return fail(VS_ERR_ARG, "flush windows: 0 (automatic), 4 or 16");
            h->opt_flushq = (uint32_t)value;
            return 0;
        case VS_OPT_WALK_FLUSH_SPAN:
            if (value < 0 || value > (1ll << 30)) return fail(VS_ERR_ARG, "flush span out of range");
            h->opt_flushspan = (uint32_t)value;
            return 0;
        case VS_OPT_WALK_TAIL_PCT:
            if (value < -1 || value > 90) return fail(VS_ERR_ARG, "tail share out of range");
            h->opt_tailpct = (int32_t)value;
            return 0;
        case VS_OPT_WALK_SEG_MARGIN:
            if (value < -1 || value > (1ll << 32)) return fail(VS_ERR_ARG, "segment margin out of range");
            h->opt_seg_margin = value;
            return 0;
        case VS_OPT_WALK_FLUSH_PREDICT:
            h->opt_flushpredict = value != 0;
            return 0;
        case VS_OPT_WALK_PREFILTER:
            h->opt_prefilter = value != 0;
            return 0;
        default:
            return fail(VS_ERR_ARG, "unknown vs_rsync option " + std::to_string(option));
    }
}

VS_API int vs_rsync_match_begin(vs_rsync *h, int64_t file_len, int file_csum,
                                uint64_t piece_bytes, uint32_t ring) {
    if (!h) return fail(VS_ERR_ARG, "null handle");
    return ms_begin(h, file_len, file_csum, piece_bytes, ring);
}

VS_API int vs_rsync_match_feed(vs_rsync *h, const void *buf, size_t n) {
    if (!h) return fail(VS_ERR_ARG, "null handle");
    return ms_feed(h, (const uint8_t *)buf, n);
}

VS_API int vs_rsync_match_next(vs_rsync *h, vs_match *out, size_t cap, size_t *n_out) {
    if (!h || !n_out || (cap && !out)) return fail(VS_ERR_ARG, "bad arguments");
    // once every byte is fed the caller can only wait for the walk
    const bool all = h->mst && h->mst->fed == h->mst->flen;
    return ms_next(h, out, cap, n_out, all);
}

VS_API int vs_rsync_match_end(vs_rsync *h, int64_t *n_matches, int64_t *false_alarms,
                              uint8_t file_sum[16]) {
    if (!h) return fail(VS_ERR_ARG, "null handle");
    return ms_end(h, n_matches, false_alarms, file_sum);
}

VS_API int vs_rsync_match_stream_stats(vs_rsync *h, double out[10]) {
    if (!h || !out) return fail(VS_ERR_ARG, "bad arguments");
    for (int i = 0; i < 10; ++i) out[i] = 0;
    MatchStream *m = h->mst;
    if (!m) return 0;
    std::lock_guard<std::mutex> lk(m->mu);
    out[0] = (double)m->pinned_bytes;
    out[1] = (double)m->staged_bytes;
    out[2] = m->feed_wait_ms;
    out[3] = m->walk_ms;
    out[4] = m->idle_ms;
    out[5] = (double)m->walked;
    out[6] = (double)m->piece;
    out[7] = (double)m->ring;
    out[8] = m->fs_ms;
    out[9] = (double)m->fcsum;
    return 0;
}

VS_API int vs_rsync_sig_begin(vs_rsync *h, int64_t len, int32_t blength, int32_t s2length,
                              int csum_type, uint32_t seed, uint64_t piece_bytes, uint32_t ring) {
    if (!h) return fail(VS_ERR_ARG, "null handle");
    return ss_begin(h, len, blength, s2length, csum_type, seed, piece_bytes, ring);
}

VS_API int vs_rsync_sig_feed(vs_rsync *h, const void *buf, size_t n) {
    if (!h) return fail(VS_ERR_ARG, "null handle");
    return ss_feed(h, (const uint8_t *)buf, n);
}

VS_API int vs_rsync_sig_next(vs_rsync *h, uint32_t *sum1, uint8_t *sum2, size_t cap_blocks,
                             size_t *n_blocks) {
    if (!h || !n_blocks || (cap_blocks && (!sum1 || !sum2))) return fail(VS_ERR_ARG, "bad arguments");
    return ss_next(h, sum1, sum2, cap_blocks, n_blocks);
}

// The host one-shot forms run the streamed paths: a file of any size passes
// through a bounded device ring (SURVEY.md 8(b) signatures).
VS_API int vs_rsync_signatures(int device, const void *basis, int64_t len, int32_t blength,
                               int32_t s2length, int csum_type, uint32_t seed, uint32_t *sum1,
                               uint8_t *sum2) {
    if (len < 0 || (len && !basis) || blength <= 0) return fail(VS_ERR_ARG, "bad basis");
    const int64_t count = len / blength + (len % blength != 0);
    if (count && (!sum1 || !sum2)) return fail(VS_ERR_ARG, "null outputs");
    vs_rsync *h = nullptr;
    VS_TRY(vs_rsync_open(device, &h));
    int r = vs_rsync_sig_begin(h, len, blength, s2length, csum_type, seed, 0, 0);
    if (!r && len) r = vs_rsync_sig_feed(h, basis, (size_t)len);
    int64_t got = 0;
    while (!r) {
        size_t n = 0;
        r = vs_rsync_sig_next(h, sum1 + got, sum2 + got * s2length, (size_t)(count - got), &n);
        got += (int64_t)n;
    }
    if (r == VS_EOF) r = got == count ? 0 : fail(VS_ERR_STATE, "signature stream ended early");
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
    if (!r) r = vs_rsync_match_begin(h, len, 0, 0, 0);
    if (!r && len) r = vs_rsync_match_feed(h, src, (size_t)len);
    int64_t nm = 0;
    if (!r) r = vs_rsync_match_end(h, &nm, nullptr, nullptr);
    if (!r) {
        *n_out = (size_t)nm;
        if ((size_t)nm > cap)
            r = fail(VS_ERR_ARG, "output capacity too small (need " + std::to_string(nm) + ")");
        else
            r = vs_rsync_get_matches(h, 0, nm, out);
    }
    vs_rsync_close(h);
    return r;
}
