// api.hip -- the C ABI (include/vsgpu.h): handle, device buffers, pipeline
// orchestration and the streaming Chunker surface.
//
// Pipeline per batch:
//   fingerprint (fingerprint.hip) -> candidate compaction + speculative
//   segment walks + boundary stitch + emit (select.hip) -> Cut values ->
//   longest-first order -> SHA-256 blob IDs (sha256.hip).
#include <algorithm>
#include <cstdlib>
#include <chrono>
#include <cstring>
#include <deque>
#include <mutex>
#include <string>
#include <vector>

#include "internal.hpp"

#define VS_API extern "C" __attribute__((visibility("default")))

namespace vsgpu {

static thread_local std::string g_err;
void set_error(const std::string &msg) { g_err = msg; }
int fail(int code, const std::string &msg) {
    g_err = msg;
    return code;
}

// strip = 64 * G with G even and G < 256 (fingerprint.hip alternates two
// 64-byte group buffers and notes groups by 8-bit index)
constexpr uint32_t kStrip = 12288;

enum Stage { kStFp = 0, kStSel = 1, kStSha = 2, kStOther = 3 };

}  // namespace vsgpu

using namespace vsgpu;

struct vs_cdc {
    int device = 0;
    int cus = 256;  // compute units (persistent fingerprint grid)
    hipStream_t stream = nullptr;
    hipStream_t own = nullptr;
    // parameters
    uint64_t pol = 0;
    uint32_t min_size = 0, max_size = 0, avg_bits = 0;
    uint32_t idx_shift = 0;
    uint64_t out_h[256], mod_h[256], out8_h[256];
    DevBuf tabs;  // [mod 256][out8 256]
    // fingerprint / candidate index
    DevBuf counts, offs, dslot, pool, flags, cstart, partials, compact;
    uint32_t pool_cap = 0;
    uint64_t nstrips = 0, base = 0, scan_end = 0;
    const uint8_t *data = nullptr;
    uint64_t dlen = 0, origin = 0, own_lo = 0, own_hi = 0;  // data offsets for own_*
    bool final_ = false, final_eof = false;
    // segments
    uint32_t nseg = 0, maxc = 0;
    uint64_t seg_len = 0;
    DevBuf spec_cut, spec_n, spec_exit, st_cut, st_n, st_merge, st_total, exit_a, exit_b,
        seg_off;
    uint64_t *exit_old = nullptr, *exit_new = nullptr;
    uint64_t entry = 0;  // data offset
    // chunk batches: a ring of per-batch chunk arrays.  The
    // hash engine keeps hashing batch q's chunks (IDs into its slot) while
    // batches q+1, q+2, ... are chunked; a slot is reused only once every
    // chain of its previous batch is complete.
    struct Slot {
        DevBuf start, end, cut, id;
        uint64_t n = 0, origin = 0;
        uint64_t seq = ~0ull;     // batch number held, ~0 = never used
        uint64_t done_slice = 0;  // slice index after which its blob IDs are final
    };
    std::vector<Slot> slots;
    uint64_t seq = 0;             // batches finished so far
    int last = -1;                // slot of the last finished batch
    uint64_t n_chunks = 0;
    DevBuf n_out;
    // VS_OPT_FP_GENERIC: the generic fingerprint variant even where the FAST
    // one applies (A/B measurements; results are identical)
    bool fp_generic = false;
    // SHA-256: time-sliced engine on its own stream (hstream)
    ShaEngine sha;
    uint32_t hash_budget = 512;   // blocks per chain per slice (0xffffffff: unbounded)
    uint32_t chain_slices = 1;    // slices that finish any chain: ceil(max blocks / budget)
    uint64_t slices = 0;          // slices launched
    static constexpr int kSliceEv = 64;
    hipEvent_t slice_ev[kSliceEv] = {};  // event after slice i at [i % kSliceEv]
    hipStream_t hstream = nullptr;
    hipStream_t own_h = nullptr;
    hipEvent_t ev_ready = nullptr;   // main stream: a batch's chunk list written
    hipEvent_t ev_null = nullptr;    // orders a scan after prior null-stream work
    bool hash_pending = false;
    int state = 0;  // 0 idle, 1 scanned, 2 stitched, 3 finished
    // host staging
    uint64_t *pinned = nullptr;  // 8 u64 of pinned host memory
    PinnedVec<uint8_t> rb;       // chunk-list read-back: start | end | cut | id per batch range
    // streaming (vs_cdc_feed / vs_cdc_next): one device batch
    // buffer per ring slot -- the hash engine reads a batch's chunks from its
    // buffer until their blob IDs are final -- filled by H2D copies on a copy
    // stream; finished batches are collected in order once their IDs are final
    static constexpr size_t kStreamSlots = 32;
    std::vector<DevBuf> sbufs;
    uint64_t sorigin = 0, batch_bytes = 512ull << 20;
    bool streaming = false;          // the handle is in streaming mode (first feed .. reset)
    uint32_t pre_stream_budget = 0;  // hash_budget before streaming changed it
    uint32_t pre_stream_isolate = 1; // the engine's isolated-drain setting before streaming
    std::deque<uint64_t> spend;      // batches whose chunks are not yet collected
    std::deque<vs_chunk> ready;
    bool final_fed = false;
    hipStream_t cstream = nullptr;   // H2D copies
    hipStream_t own_hm = nullptr;    // hash stream masked to half the CUs (streaming)
    hipEvent_t ev_copy = nullptr;    // after the last copy into the filling buffer
    bool copy_pending = false;
    bool dma_wait = false;           // a copy from pinned caller memory is in flight
    uint64_t fill_seq = 0, fill_new = 0, carry = 0, skip = 0;   // the batch being filled
    bool scanned = false;            // a batch is scanned, its cut selection pending
    bool scan_final = false;
    uint64_t scan_len = 0, scan_skip = 0;
    uint8_t *scan_buf = nullptr;
    uint8_t *stage[2] = {nullptr, nullptr};   // pinned staging for pageable input
    size_t stage_cap = 0;
    hipEvent_t stage_ev[2] = {nullptr, nullptr};
    bool stage_busy[2] = {false, false};
    int stage_i = 0;
    // bytes direct, bytes staged, collect waits, batches, then host ms spent
    // waiting for DMAs, processing batches, collecting chunks, staging memcpy
    double feed_stats[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    double dbg_ms[3] = {0, 0, 0};    // VSGPU_STREAM_TRACE: stitch, finish, scan host ms
    // timing
    bool timing = false;
    struct Pend {
        int stage;
        hipEvent_t a, b;
    };
    std::vector<Pend> pend;
    std::vector<hipEvent_t> ev_pool;
    double ms[4] = {0, 0, 0, 0};
    uint64_t launches[4] = {0, 0, 0, 0};
    // the fingerprint and SHA-256 kernel windows of the timed region as
    // [start, end) ms after `anchor` (recorded on the main stream when timing
    // starts), so the SHA-256 time can be split into the part inside a
    // fingerprint window and the part outside (vs_cdc_timing_detail)
    hipEvent_t anchor = nullptr;
    bool anchored = false;
    std::vector<std::pair<double, double>> win_fp, win_sha;
    double detail[4] = {0, 0, 0, 0};
    uint64_t quad_chains = 0;  // chains the drains ran in latency mode (timed region)
};

namespace vsgpu {

static int set_dev(vs_cdc *h) { return enter_device(h->device); }

static hipEvent_t get_event(vs_cdc *h) {
    if (!h->ev_pool.empty()) {
        hipEvent_t e = h->ev_pool.back();
        h->ev_pool.pop_back();
        return e;
    }
    hipEvent_t e = nullptr;
    if (hipEventCreate(&e) != hipSuccess) return nullptr;
    return e;
}

struct StageTimer {
    vs_cdc *h;
    int st;
    hipStream_t s;
    hipEvent_t a = nullptr;
    StageTimer(vs_cdc *h_, int st_, hipStream_t s_ = nullptr) : h(h_), st(st_), s(s_ ? s_ : h_->stream) {
        if (h->timing) {
            a = get_event(h);
            if (a) (void)hipEventRecord(a, s);
        }
    }
    ~StageTimer() {
        if (a) {
            hipEvent_t b = get_event(h);
            if (b) {
                (void)hipEventRecord(b, s);
                h->pend.push_back({st, a, b});
            } else {
                h->ev_pool.push_back(a);
            }
        }
    }
};

// call after a stream sync: fold completed event pairs into the totals
static void drain_timers(vs_cdc *h) {
    for (auto &p : h->pend) {
        float ms = 0;
        if (hipEventElapsedTime(&ms, p.a, p.b) == hipSuccess) {
            h->ms[p.stage] += ms;
            h->launches[p.stage] += 1;
            float t0 = 0;
            if (h->anchored && (p.stage == kStFp || p.stage == kStSha) &&
                hipEventElapsedTime(&t0, h->anchor, p.a) == hipSuccess)
                (p.stage == kStFp ? h->win_fp : h->win_sha).push_back({t0, (double)t0 + ms});
        }
        h->ev_pool.push_back(p.a);
        h->ev_pool.push_back(p.b);
    }
    h->pend.clear();
}

// waits for the main stream; also for the hash stream when `all`
static int sync_stream(vs_cdc *h, bool all = false) {
    VS_HIP(hipStreamSynchronize(h->stream));
    if (all && h->hash_pending) {
        VS_HIP(hipStreamSynchronize(h->hstream));
        h->hash_pending = false;
    }
    if (all || !h->hash_pending) drain_timers(h);
    return 0;
}


// one slice of the hash engine on the hash stream, followed by its event.
// Flow control: before slice i reuses event slot i % kSliceEv the host waits
// for slice i - kSliceEv, so "c + kSliceEv <= slices" implies slice c is done.
static int run_slice(vs_cdc *h, uint32_t budget) {
    if (h->sha.idle()) return 0;
    const uint64_t i = h->slices + 1;
    hipEvent_t &e = h->slice_ev[i % vs_cdc::kSliceEv];
    if (!e) {
        VS_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    } else if (i > (uint64_t)vs_cdc::kSliceEv) {
        VS_HIP(hipEventSynchronize(e));
    }
    // stage "sha256" = the hash kernels alone, bracketed inside the engine
    // (comparable with a rocprofv3 kernel trace); its bookkeeping launches
    // (histogram, scan, scatter) are not timed
    if (h->timing) h->sha.ev_get = [h] { return get_event(h); };
    h->sha.last_quad_chains = 0;
    const int rc = h->sha.slice(budget, h->hstream);
    h->quad_chains += h->sha.last_quad_chains;
    h->sha.ev_get = nullptr;
    for (auto &p : h->sha.kernel_pairs) h->pend.push_back({kStSha, p.first, p.second});
    h->sha.kernel_pairs.clear();
    VS_TRY(rc);
    VS_HIP(hipEventRecord(e, h->hstream));
    h->slices = i;
    if (budget == 0xffffffffu)
        for (auto &s : h->slots)
            if (s.seq != ~0ull && s.done_slice > i) s.done_slice = i;
    return 0;
}

// hash every queued chain to the end (one unbounded slice)
static int drain_hash(vs_cdc *h) { return run_slice(h, 0xffffffffu); }

// make the main stream wait until slot k's previous batch is fully hashed
static int slot_free(vs_cdc *h, size_t k) {
    vs_cdc::Slot &s = h->slots[k];
    if (s.seq == ~0ull) return 0;
    if (s.done_slice > h->slices) VS_TRY(drain_hash(h));  // ring shorter than a chain's slices
    const uint64_t c = s.done_slice;
    if (c == 0 || c + vs_cdc::kSliceEv <= h->slices) return 0;
    VS_HIP(hipStreamWaitEvent(h->stream, h->slice_ev[c % vs_cdc::kSliceEv], 0));
    return 0;
}

// (re)size the batch ring for the current parameters and slice budget
static int size_ring(vs_cdc *h) {
    const uint64_t mb = sha_blocks(h->max_size);
    const uint64_t L = (h->hash_budget == 0xffffffffu) ? 1 : (mb + h->hash_budget - 1) / h->hash_budget;
    h->chain_slices = (uint32_t)std::min<uint64_t>(L, 1u << 30);
    // one slot per batch still hashing: a chain of max_size finishes L slices
    // (= batches) after its own, so L + 2 slots never make the host wait
    const size_t want = (size_t)std::min<uint64_t>(L + 2, 256);
    if (h->slots.size() != want) {
        // budgeted chains of earlier batches still point into the old slots'
        // id arrays: hash them to the end before the slots are released
        VS_TRY(drain_hash(h));
        VS_TRY(sync_stream(h, true));
        for (auto &s : h->slots) {
            s.start.release();
            s.end.release();
            s.cut.release();
            s.id.release();
        }
        h->slots.assign(want, vs_cdc::Slot());
        h->last = -1;
    }
    return 0;
}

static int set_params(vs_cdc *h, uint64_t pol, uint32_t min_size, uint32_t max_size,
                      uint32_t avg_bits) {
    if (pol == 0) return fail(VS_ERR_POLY, "tables for polynomial computation not initialized");
    const int deg = pol_deg(pol);
    if (deg < 40 || deg > 53)
        return fail(VS_ERR_POLY, "polynomial degree " + std::to_string(deg) +
                                     " outside [40, 53] (restic draws degree 53)");
    if (min_size < 64 || max_size < min_size)
        return fail(VS_ERR_ARG, "need 64 <= min_size <= max_size");
    if (avg_bits < 1 || avg_bits > 53) return fail(VS_ERR_ARG, "avg_bits must be in [1, 53]");
    h->pol = pol;
    h->min_size = min_size;
    h->max_size = max_size;
    h->avg_bits = avg_bits;
    h->idx_shift = (uint32_t)(deg - 40);
    pol_tables(pol, h->out_h, h->mod_h);
    pol_out8(pol, h->out_h, h->out8_h);
    VS_TRY(h->tabs.ensure(512 * sizeof(uint64_t)));
    VS_HIP(hipMemcpyAsync(h->tabs.as<uint64_t>(), h->mod_h, 256 * 8, hipMemcpyHostToDevice,
                          h->stream));
    VS_HIP(hipMemcpyAsync(h->tabs.as<uint64_t>() + 256, h->out8_h, 256 * 8,
                          hipMemcpyHostToDevice, h->stream));
    VS_TRY(sync_stream(h));
    return 0;
}

static FpArgs fp_args(vs_cdc *h) {
    FpArgs a{};
    a.data = h->data;
    a.dlen = h->dlen;
    a.base = h->base;
    a.scan_end = h->scan_end;
    a.strip = kStrip;
    a.idx_shift = h->idx_shift;
    const uint64_t mask = (h->avg_bits >= 64) ? ~0ull : ((1ull << h->avg_bits) - 1);
    a.mask_lo = (uint32_t)mask;
    a.mask_hi = (uint32_t)(mask >> 32);
    a.counts = h->counts.as<uint32_t>();
    a.offs = h->offs.as<uint32_t>();
    a.dense_slot = h->dslot.as<uint32_t>();
    a.pool = h->pool.as<uint32_t>();
    a.pool_cap = h->pool_cap;
    a.flags = h->flags.as<uint32_t>();
    a.pool_next = h->flags.as<uint32_t>() + 1;
    a.mod_tab = h->tabs.as<uint64_t>();
    a.out8_tab = h->tabs.as<uint64_t>() + 256;
    return a;
}

static SelArgs sel_args(vs_cdc *h) {
    SelArgs a{};
    a.base = h->base;
    a.strip = kStrip;
    a.nstrips = h->nstrips;
    a.counts = h->counts.as<uint32_t>();
    a.offs = h->offs.as<uint32_t>();
    a.dense_slot = h->dslot.as<uint32_t>();
    a.pool = h->pool.as<uint32_t>();
    a.cstart = h->cstart.as<uint32_t>();
    a.compact = h->compact.as<uint64_t>();
    a.flags = h->flags.as<uint32_t>();
    a.min_size = h->min_size;
    a.max_size = h->max_size;
    a.scan_end = h->scan_end;
    a.dlen = h->dlen;
    a.final_eof = h->final_eof ? 1 : 0;
    a.own_lo = h->own_lo;
    a.own_hi = h->own_hi;
    a.seg_len = h->seg_len;
    a.nseg = h->nseg;
    a.maxc = h->maxc;
    a.spec_cut = h->spec_cut.as<uint64_t>();
    a.spec_n = h->spec_n.as<uint32_t>();
    a.spec_exit = h->spec_exit.as<uint64_t>();
    a.st_cut = h->st_cut.as<uint64_t>();
    a.st_n = h->st_n.as<uint32_t>();
    a.st_merge = h->st_merge.as<uint32_t>();
    a.st_total = h->st_total.as<uint32_t>();
    a.exit_old = h->exit_old;
    a.exit_new = h->exit_new;
    a.entry = h->entry;
    return a;
}

// fingerprint pass + candidate index + speculative walks
static int run_scan_kernels(vs_cdc *h) {
    const size_t words = kStrip / 32;
    VS_TRY(h->pool.ensure((size_t)h->pool_cap * words * 4));
    VS_HIP(hipMemsetAsync(h->flags.p, 0, 4 * sizeof(uint32_t), h->stream));
    {
        StageTimer t(h, kStFp);
        FpArgs a = fp_args(h);
        const bool wide = h->avg_bits > 32;
        // strips whose reads stay inside [0, dlen) need no bounds checks; the
        // rest (at most a few) run bounds-checked inside the same launch
        uint64_t k_lo = (h->base >= 64) ? 0 : 1;
        uint64_t k_hi = (h->dlen >= h->base) ? (h->dlen - h->base) / kStrip : 0;
        k_hi = std::min(k_hi, h->nstrips);
        k_lo = std::min(k_lo, h->nstrips);
        if (k_hi < k_lo) k_hi = k_lo;
        a.k_lo = k_lo;
        a.k_hi = k_hi;
        a.n_edge = k_lo + (h->nstrips - k_hi);
        a.work = h->flags.as<uint32_t>() + 3;  // zeroed with the flags above
        const bool fast = !wide && h->idx_shift >= 8 && !h->fp_generic;
        // a fed stream's hash slices hold up to a few hundred workgroups for
        // ~10 ms on the masked half of the CUs: a persistent grid of one
        // workgroup per CU would wait for them before it could complete, so
        // streaming batches get a grid that fits beside them
        VS_HIP(launch_fingerprint(a, wide, fast, h->streaming ? std::max(h->cus / 2, 1) : h->cus,
                                  h->stream));
    }
    {
        StageTimer t(h, kStSel);
        SelArgs s = sel_args(h);
        VS_HIP(launch_compact(s, h->partials.as<uint32_t>(), h->compact.as<uint64_t>(),
                              h->cstart.as<uint32_t>(), h->stream));
        VS_HIP(launch_spec_walk(s, h->stream));
    }
    return 0;
}

static int cdc_scan(vs_cdc *h, const void *dev_data, uint64_t len, uint64_t origin,
                    uint64_t own_lo, uint64_t own_hi, int final) {
    if (!h) return fail(VS_ERR_ARG, "null handle");
    if (!dev_data && len) return fail(VS_ERR_ARG, "null device data");
    if (((uintptr_t)dev_data & 15) != 0) return fail(VS_ERR_ARG, "device data must be 16-byte aligned");
    if (own_lo < origin || own_hi < own_lo || own_hi > origin + len)
        return fail(VS_ERR_ARG, "own range must lie inside [origin, origin + len)");
    VS_TRY(set_dev(h));
    if (h->stream == h->own && !h->streaming) {
        // the handle's own stream is non-blocking: order the scan after work the
        // caller queued on the null stream (e.g. the kernel that wrote the data).
        // With vs_cdc_set_stream the caller's stream carries that order instead;
        // a fed stream's bytes come from the handle's own copies.
        VS_HIP(hipEventRecord(h->ev_null, nullptr));
        VS_HIP(hipStreamWaitEvent(h->stream, h->ev_null, 0));
    }
    h->data = (const uint8_t *)dev_data;
    h->dlen = len;
    h->origin = origin;
    h->own_lo = own_lo - origin;
    h->own_hi = own_hi - origin;
    h->final_ = final != 0;
    h->scan_end = std::min<uint64_t>(h->own_hi + h->max_size - 1, len);
    h->final_eof = h->final_ && h->scan_end == len;
    h->base = h->own_lo & ~63ull;
    h->nstrips = (h->scan_end > h->base) ? (h->scan_end - h->base + kStrip - 1) / kStrip : 0;
    const uint64_t ns = std::max<uint64_t>(h->nstrips, 1);
    VS_TRY(h->counts.ensure(ns * 4));
    VS_TRY(h->offs.ensure(ns * kSlots * 4));
    VS_TRY(h->dslot.ensure(ns * 4));
    VS_TRY(h->flags.ensure(16));
    VS_TRY(h->cstart.ensure((ns + 1) * 4));
    VS_TRY(h->partials.ensure((ns / 4096 + 2) * 4));
    VS_TRY(h->compact.ensure(ns * kSlots * 8));
    h->pool_cap = (uint32_t)std::max<uint64_t>({(uint64_t)h->pool_cap, 16, h->nstrips / 256});
    // segments
    const uint64_t own = h->own_hi - h->own_lo;
    h->seg_len = std::min<uint64_t>(std::max<uint64_t>((uint64_t)h->min_size * 64, 1ull << 20),
                                    64ull << 20);
    h->nseg = (uint32_t)((own + h->seg_len - 1) / h->seg_len);
    h->maxc = (uint32_t)(h->seg_len / h->min_size + 3);
    const uint64_t sg = std::max<uint32_t>(h->nseg, 1);
    VS_TRY(h->spec_cut.ensure(sg * h->maxc * 8));
    VS_TRY(h->st_cut.ensure(sg * h->maxc * 8));
    VS_TRY(h->spec_n.ensure(sg * 4));
    VS_TRY(h->spec_exit.ensure(sg * 8));
    VS_TRY(h->st_n.ensure(sg * 4));
    VS_TRY(h->st_merge.ensure(sg * 4));
    VS_TRY(h->st_total.ensure(sg * 4));
    VS_TRY(h->exit_a.ensure(sg * 8));
    VS_TRY(h->exit_b.ensure(sg * 8));
    VS_TRY(h->seg_off.ensure((sg + 1 + sg / 4096 + 2) * 4));
    VS_TRY(run_scan_kernels(h));
    h->state = 1;
    return 0;
}

static int cdc_stitch(vs_cdc *h, uint64_t entry, uint64_t *exit_pos, int *complete) {
    if (!h || h->state < 1) return fail(VS_ERR_STATE, "vs_cdc_stitch before vs_cdc_scan");
    if (entry < h->origin + h->own_lo)
        return fail(VS_ERR_ARG, "entry before the scanned own range");
    // entry >= own_hi is legal: a chunk of the previous shard spans this whole
    // range, so this shard owns no chunk start and its exit is the entry
    VS_TRY(set_dev(h));
    h->entry = entry - h->origin;
    for (int attempt = 0;; ++attempt) {
        h->exit_old = h->exit_a.as<uint64_t>();
        h->exit_new = h->exit_b.as<uint64_t>();
        if (h->nseg)
            VS_HIP(hipMemcpyAsync(h->exit_old, h->spec_exit.p, (size_t)h->nseg * 8,
                                  hipMemcpyDeviceToDevice, h->stream));
        bool redo = false;
        for (uint32_t pass = 0; pass <= h->nseg + 1; ++pass) {
            {
                StageTimer t(h, kStSel);
                // clear only the per-pass word; scan errors in flags[0] persist
                VS_HIP(hipMemsetAsync(h->flags.as<uint32_t>() + 2, 0, 4, h->stream));
                SelArgs s = sel_args(h);
                VS_HIP(launch_stitch(s, h->stream));
            }
            VS_HIP(hipMemcpyAsync(h->pinned, h->flags.p, 16, hipMemcpyDeviceToHost, h->stream));
            VS_TRY(sync_stream(h));
            const uint32_t *fw = (const uint32_t *)h->pinned;
            if (fw[0] & (kFlagPoolOverflow | kFlagDenseMissing)) {
                redo = true;
                break;
            }
            std::swap(h->exit_old, h->exit_new);  // exit_old = latest exits
            if (!(fw[2] & kFlagChanged)) break;
        }
        if (!redo) break;
        if (attempt > 0) return fail(VS_ERR_STATE, "dense candidate pool still overflowing");
        // some strips were dense beyond the pool: size it for the worst case
        h->pool_cap = (uint32_t)std::max<uint64_t>(h->nstrips, 16);
        VS_TRY(run_scan_kernels(h));
    }
    // after the loop exit_old holds the converged exits (== exit_new)
    uint64_t ex;
    if (h->nseg) {
        VS_HIP(hipMemcpyAsync(h->pinned, h->exit_old + (h->nseg - 1), 8, hipMemcpyDeviceToHost,
                              h->stream));
        VS_TRY(sync_stream(h));
        ex = h->pinned[0];
    } else {
        ex = h->entry;
    }
    const bool done = ex != kIncomplete;
    if (exit_pos) *exit_pos = done ? ex + h->origin : ~0ull;
    if (complete) *complete = done ? 1 : 0;
    h->state = 2;
    return 0;
}

static int cdc_finish(vs_cdc *h, uint64_t *n_chunks) {
    if (!h || h->state < 2) return fail(VS_ERR_STATE, "vs_cdc_finish before vs_cdc_stitch");
    VS_TRY(set_dev(h));
    VS_TRY(h->n_out.ensure(16));
    VS_TRY(size_ring(h));
    const size_t k = (size_t)(h->seq % h->slots.size());
    vs_cdc::Slot &sl = h->slots[k];
    // the slot's previous batch must be fully hashed before emit rewrites it
    VS_TRY(slot_free(h, k));
    SelArgs s = sel_args(h);
    // upper bound of chunks: every segment's capacity
    const uint64_t cap = std::max<uint64_t>((uint64_t)h->nseg * h->maxc, 1);
    if (sl.start.cap < cap * 8 || sl.end.cap < cap * 8) {
        VS_TRY(sync_stream(h, true));  // growing arrays the hash stream may read
        VS_TRY(sl.start.ensure(cap * 8));
        VS_TRY(sl.end.ensure(cap * 8));
    }
    {
        StageTimer t(h, kStSel);
        VS_HIP(launch_emit(s, h->seg_off.as<uint32_t>(), sl.start.as<uint64_t>(),
                           sl.end.as<uint64_t>(), h->n_out.as<uint64_t>(), h->stream));
    }
    VS_HIP(hipMemcpyAsync(h->pinned, h->n_out.p, 8, hipMemcpyDeviceToHost, h->stream));
    VS_TRY(sync_stream(h));
    const uint64_t n = h->pinned[0];
    if (sl.cut.cap < n * 8 || sl.id.cap < n * 32) {
        VS_TRY(sync_stream(h, true));
        VS_TRY(sl.cut.ensure(std::max<uint64_t>(n, 1) * 8));
        VS_TRY(sl.id.ensure(std::max<uint64_t>(n, 1) * 32));
    }
    if (n) {
        {
            StageTimer t(h, kStOther);
            VS_HIP(launch_cut_fp(h->data, n, sl.start.as<uint64_t>(), sl.end.as<uint64_t>(),
                                 h->min_size, h->tabs.as<uint64_t>(), h->tabs.as<uint64_t>() + 256,
                                 h->idx_shift, sl.cut.as<uint64_t>(), h->stream));
        }
        // the hash stream picks the chunk list up once emit has written it
        VS_HIP(hipEventRecord(h->ev_ready, h->stream));
        VS_HIP(hipStreamWaitEvent(h->hstream, h->ev_ready, 0));
        VS_TRY(h->sha.append_chunks(h->data, sl.start.as<uint64_t>(), sl.end.as<uint64_t>(), n,
                                    sl.id.as<uint8_t>(), (uint32_t)sha_blocks(h->max_size),
                                    h->hstream));
        VS_TRY(run_slice(h, h->hash_budget));
        h->hash_pending = true;
    }
    sl.n = n;
    sl.origin = h->origin;
    sl.seq = h->seq;
    sl.done_slice = n ? h->slices + h->chain_slices - 1 : 0;
    h->last = (int)k;
    h->n_chunks = n;
    h->seq++;
    // Cut values and blob IDs stay queued: results are waited for by
    // vs_cdc_wait / vs_cdc_get_chunks, so the next batch's fingerprint pass
    // runs beside this batch's hashing.
    if (n_chunks) *n_chunks = n;
    h->state = 3;
    return 0;
}

static int cdc_wait(vs_cdc *h) {
    if (!h) return fail(VS_ERR_ARG, "null handle");
    VS_TRY(set_dev(h));
    VS_TRY(drain_hash(h));
    return sync_stream(h, true);
}

// chunks [first, first+n) of a slot, read back into the handle's pinned
// buffer on its own (non-blocking) stream -- a null-stream copy would wait for
// every blocking stream, the masked hash stream included
static int read_chunks(vs_cdc *h, const vs_cdc::Slot &sl, uint64_t first, uint64_t n,
                       vs_chunk *out) {
    VS_TRY(pv_resize(h->rb, n * 56));
    uint64_t *st = (uint64_t *)h->rb.data(), *en = st + n, *cu = en + n;
    uint8_t *id = (uint8_t *)(cu + n);
    VS_HIP(hipMemcpyAsync(st, sl.start.as<uint64_t>() + first, n * 8, hipMemcpyDeviceToHost, h->stream));
    VS_HIP(hipMemcpyAsync(en, sl.end.as<uint64_t>() + first, n * 8, hipMemcpyDeviceToHost, h->stream));
    VS_HIP(hipMemcpyAsync(cu, sl.cut.as<uint64_t>() + first, n * 8, hipMemcpyDeviceToHost, h->stream));
    VS_HIP(hipMemcpyAsync(id, sl.id.as<uint8_t>() + first * 32, n * 32, hipMemcpyDeviceToHost,
                          h->stream));
    VS_HIP(hipStreamSynchronize(h->stream));
    for (uint64_t i = 0; i < n; ++i) {
        out[i].start = sl.origin + st[i];
        out[i].length = (en[i] & kPosMask) - st[i] + 1;
        out[i].cut = cu[i];
        memcpy(out[i].id, id + i * 32, 32);
    }
    return 0;
}

// chunks [first, first+n) of batch `seq` (while its ring slot still holds it)
static int cdc_get_batch(vs_cdc *h, uint64_t seq, uint64_t first, uint64_t n, vs_chunk *out) {
    if (!h || h->slots.empty() || seq >= h->seq) return fail(VS_ERR_STATE, "no such finished batch");
    const vs_cdc::Slot &sl = h->slots[seq % h->slots.size()];
    if (sl.seq != seq) return fail(VS_ERR_STATE, "batch already recycled (ring holds the last " +
                                                     std::to_string(h->slots.size()) + ")");
    if (first + n > sl.n) return fail(VS_ERR_ARG, "chunk range out of bounds");
    if (!n) return 0;
    VS_TRY(cdc_wait(h));
    VS_TRY(read_chunks(h, sl, first, n, out));
    return 0;
}

static int cdc_get_chunks(vs_cdc *h, uint64_t first, uint64_t n, vs_chunk *out) {
    if (!h || h->state < 3 || h->last < 0) return fail(VS_ERR_STATE, "no finished batch");
    if (first + n > h->n_chunks) return fail(VS_ERR_ARG, "chunk range out of bounds");
    return cdc_get_batch(h, h->seq - 1, first, n, out);
}

static int cdc_process(vs_cdc *h, const void *dev_data, uint64_t len, uint64_t origin, int final,
                       uint64_t *n_chunks, uint64_t *consumed) {
    VS_TRY(cdc_scan(h, dev_data, len, origin, origin, origin + len, final));
    uint64_t ex = 0;
    int complete = 0;
    VS_TRY(cdc_stitch(h, origin, &ex, &complete));
    uint64_t n = 0;
    VS_TRY(cdc_finish(h, &n));
    if (n_chunks) *n_chunks = n;
    if (consumed) {
        if (complete) {
            *consumed = ex - origin;
        } else if (n) {
            VS_HIP(hipMemcpyAsync(h->pinned, h->slots[h->last].end.as<uint64_t>() + (n - 1), 8,
                                  hipMemcpyDeviceToHost, h->stream));
            VS_HIP(hipStreamSynchronize(h->stream));
            *consumed = (h->pinned[0] & kPosMask) + 1;
        } else {
            *consumed = 0;
        }
    }
    return 0;
}

// ---- streaming ------------------------------------------------------------
static double now_ms() {
    return std::chrono::duration<double, std::milli>(
               std::chrono::steady_clock::now().time_since_epoch())
        .count();
}

// Batch s lives in ring slot / device buffer s % R.  A batch's chunks become
// `ready` once the slice that finishes its longest chain has completed.
static bool batch_done(vs_cdc *h, uint64_t s) {
    const vs_cdc::Slot &sl = h->slots[s % h->slots.size()];
    const uint64_t c = sl.done_slice;
    if (sl.n == 0 || c == 0) return true;
    if (c > h->slices) return false;
    if (c + vs_cdc::kSliceEv <= h->slices) return true;
    const hipError_t e = hipEventQuery(h->slice_ev[c % vs_cdc::kSliceEv]);
    if (e == hipErrorNotReady) {
        (void)hipGetLastError();
        return false;
    }
    return e == hipSuccess;
}

// move batch s (the oldest pending one) to `ready`; block = wait for its IDs
static int collect_batch(vs_cdc *h, uint64_t s, bool block) {
    vs_cdc::Slot &sl = h->slots[s % h->slots.size()];
    if (sl.seq != s) return fail(VS_ERR_STATE, "streaming batch recycled before collection");
    if (!batch_done(h, s)) {
        if (!block) return 1;
        h->feed_stats[2] += 1;
        if (sl.done_slice > h->slices) VS_TRY(drain_hash(h));
        VS_HIP(hipEventSynchronize(h->slice_ev[sl.done_slice % vs_cdc::kSliceEv]));
    }
    const uint64_t n = sl.n;
    if (n) {
        std::vector<vs_chunk> got(n);
        VS_TRY(read_chunks(h, sl, 0, n, got.data()));
        h->ready.insert(h->ready.end(), got.begin(), got.end());
    }
    h->spend.pop_front();
    return 0;
}

// collect finished batches in order (block: at least the oldest one)
static int collect_ready(vs_cdc *h, bool block) {
    const double t0 = now_ms();
    struct Acc {
        double *d, t0;
        ~Acc() { *d += now_ms() - t0; }
    } acc{&h->feed_stats[6], t0};
    while (!h->spend.empty()) {
        const int r = collect_batch(h, h->spend.front(), block);
        if (r < 0) return r;
        if (r == 1) break;
        block = false;
    }
    return 0;
}

// Batches of the stream: batch q is filled into device buffer q % R (R =
// ring slots): [kStreamPad - carry, kStreamPad) holds the bytes carried over
// from batch q - 1 (after its last determined cut), [kStreamPad, ...) the new
// bytes.  A full batch is scanned (fingerprint launched) at once; its cut
// selection, emit and hash queueing -- which wait for the GPU -- run when the
// next batch is full, so the fingerprint pass overlaps that batch's copies.
static uint64_t stream_pad(const vs_cdc *h) {
    return (2ull * h->max_size + (1 << 20) + 63) & ~63ull;
}
static uint64_t stream_new_bytes(const vs_cdc *h) {
    return std::max<uint64_t>(h->batch_bytes, 2ull * h->max_size + (1 << 20));
}

// buffer of batch q, free for writing: slot q % R's previous batch collected
// (backpressure: wait for it)
static int stream_buffer(vs_cdc *h, uint64_t q, DevBuf **out) {
    const size_t R = h->slots.size();
    while (!h->spend.empty() && h->spend.front() + R <= q) VS_TRY(collect_batch(h, h->spend.front(), true));
    DevBuf &b = h->sbufs[q % R];
    const uint64_t need = stream_pad(h) + stream_new_bytes(h) + (1 << 20);
    if (b.cap < need) VS_TRY(b.ensure(need));
    *out = &b;
    return 0;
}

// first feed of a stream: streaming mode (slice budget so that a MaxSize
// chain finishes within the ring), copy stream, staging buffers
static int stream_begin(vs_cdc *h) {
    if (h->streaming) return 0;
    if (!h->cstream) {
        VS_HIP(hipStreamCreateWithFlags(&h->cstream, hipStreamNonBlocking));
        VS_HIP(hipEventCreateWithFlags(&h->ev_copy, hipEventDisableTiming));
        for (int i = 0; i < 2; ++i) VS_HIP(hipEventCreateWithFlags(&h->stage_ev[i], hipEventDisableTiming));
    }
    VS_TRY(cdc_wait(h));
    // the hash slices of a stream run ~10 ms each (a MaxSize chain must finish
    // within the ring); spread over every CU they starve the next batch's
    // fingerprint pass, so the handle's own hash stream is swapped for one
    // masked to every other CU (across all XCDs) while streaming.  (That
    // stream is created blocking, so nothing in the streaming path orders
    // work through the null stream.)
    if (h->hstream == h->own_h) {
        if (!h->own_hm) {
            std::vector<uint32_t> mask(((size_t)std::max(h->cus, 1) + 31) / 32, 0x55555555u);
            if (hipExtStreamCreateWithCUMask(&h->own_hm, (uint32_t)mask.size(), mask.data()) !=
                hipSuccess) {
                (void)hipGetLastError();
                h->own_hm = nullptr;
            }
        }
        if (h->own_hm) h->hstream = h->own_hm;
    }
    h->pre_stream_budget = h->hash_budget;
    // no isolated drains while streaming: the fingerprint grid of the next
    // batch may hold CUs a quad tile would wait to take whole, and the hash
    // stream is masked to half the CUs
    h->pre_stream_isolate = h->sha.isolate;
    h->sha.isolate = 0;
    const uint64_t mb = sha_blocks(h->max_size);
    const uint64_t budget = (mb + vs_cdc::kStreamSlots - 3) / (vs_cdc::kStreamSlots - 2);
    h->hash_budget = (uint32_t)std::max<uint64_t>(budget, 1);
    VS_TRY(size_ring(h));
    h->sbufs.resize(h->slots.size());
    h->fill_seq = h->seq;
    h->fill_new = 0;
    h->carry = 0;
    h->skip = 0;
    h->scanned = false;
    h->streaming = true;
    return 0;
}

// issue the copy of n caller bytes to device dst on the copy stream.  Pinned
// caller memory is DMA'd directly (h->dma_wait: the call waits for it before
// returning -- the caller owns the buffer); pageable memory goes through two
// pinned staging buffers (the copy of each piece waits only for its buffer).
static int stream_copy(vs_cdc *h, uint8_t *dst, const uint8_t *src, size_t n) {
    if (!n) return 0;
    if (host_range_pinned(src, n)) {
        VS_HIP(hipMemcpyAsync(dst, src, n, hipMemcpyHostToDevice, h->cstream));
        VS_HIP(hipEventRecord(h->ev_copy, h->cstream));
        h->feed_stats[0] += (double)n;
        h->copy_pending = true;
        h->dma_wait = true;
        return 0;
    }
    const size_t piece = 64ull << 20;
    if (!h->stage[0]) {
        for (int i = 0; i < 2; ++i)
            if (hipHostMalloc((void **)&h->stage[i], piece, hipHostMallocDefault) != hipSuccess) {
                (void)hipGetLastError();
                return fail(VS_ERR_NOMEM, "pinned staging allocation failed");
            }
        h->stage_cap = piece;
    }
    for (size_t off = 0; off < n; off += piece) {
        const size_t k = std::min(piece, n - off);
        const int i = h->stage_i;
        const double t0 = now_ms();
        if (h->stage_busy[i]) VS_HIP(hipEventSynchronize(h->stage_ev[i]));
        const double t1 = now_ms();
        par_memcpy(h->stage[i], src + off, k);
        h->feed_stats[4] += t1 - t0;
        h->feed_stats[7] += now_ms() - t1;
        VS_HIP(hipMemcpyAsync(dst + off, h->stage[i], k, hipMemcpyHostToDevice, h->cstream));
        VS_HIP(hipEventRecord(h->stage_ev[i], h->cstream));
        h->stage_busy[i] = true;
        h->stage_i ^= 1;
    }
    VS_HIP(hipEventRecord(h->ev_copy, h->cstream));
    h->feed_stats[1] += (double)n;
    h->copy_pending = true;
    return 0;
}

// launch the fingerprint pass of the filling batch (bytes carried + new)
static int stream_scan(vs_cdc *h, bool final) {
    DevBuf *cur = nullptr;
    VS_TRY(stream_buffer(h, h->fill_seq, &cur));
    if (h->copy_pending) {
        VS_HIP(hipStreamWaitEvent(h->stream, h->ev_copy, 0));
        h->copy_pending = false;
    }
    // the scan starts `skip` bytes before the carried ones (16-byte aligned
    // data; those bytes belong to the previous batch's last chunk and are
    // outside the owned range)
    const uint64_t len = h->skip + h->carry + h->fill_new;
    const uint8_t *p = (const uint8_t *)cur->p + stream_pad(h) - h->carry - h->skip;
    const uint64_t origin = h->sorigin - h->skip;
    h->scan_len = len;
    h->scan_final = final;
    h->scan_buf = (uint8_t *)p;
    h->scan_skip = h->skip;
    const double t0 = now_ms();
    VS_TRY(cdc_scan(h, len ? p : (const uint8_t *)h->tabs.p, len, origin, h->sorigin,
                    origin + len, final ? 1 : 0));
    h->feed_stats[5] += now_ms() - t0;
    h->dbg_ms[2] += now_ms() - t0;
    h->scanned = true;
    h->fill_seq += 1;
    h->fill_new = 0;
    return 0;
}

// cut selection, emit and hash queueing of the scanned batch; its bytes
// after the last determined cut are carried into the filling buffer
static int stream_finish(vs_cdc *h) {
    if (!h->scanned) return 0;
    const double t0 = now_ms();
    uint64_t ex = 0, n = 0;
    int complete = 0;
    VS_TRY(cdc_stitch(h, h->sorigin, &ex, &complete));
    const double t1 = now_ms();
    const uint64_t q = h->seq;
    VS_TRY(cdc_finish(h, &n));
    h->dbg_ms[0] += t1 - t0;
    h->dbg_ms[1] += now_ms() - t1;
    // used = scanned bytes up to the last determined cut (skip included)
    uint64_t used = h->scan_skip;
    if (complete) {
        used = ex - (h->sorigin - h->scan_skip);
    } else if (n) {
        VS_HIP(hipMemcpyAsync(h->pinned, h->slots[h->last].end.as<uint64_t>() + (n - 1), 8,
                              hipMemcpyDeviceToHost, h->stream));
        VS_HIP(hipStreamSynchronize(h->stream));
        used = (h->pinned[0] & kPosMask) + 1;
    }
    h->spend.push_back(q);
    h->feed_stats[3] += 1;
    const uint64_t rest = h->scan_len - used;
    // the next scan starts 16-byte aligned: skip = the bytes before the
    // carried ones that align it (at most 15; a non-final batch uses at
    // least MinSize >= 64 bytes, so they exist)
    const uint64_t skip = (stream_pad(h) - rest) % 16;
    if (rest + skip > stream_pad(h) || (rest && used < skip))
        return fail(VS_ERR_STATE, "streaming carry exceeds its reserve");
    if (rest) {
        DevBuf *nxt = nullptr;
        VS_TRY(stream_buffer(h, h->fill_seq, &nxt));
        VS_HIP(hipMemcpyAsync((uint8_t *)nxt->p + stream_pad(h) - rest - skip,
                              h->scan_buf + used - skip, rest + skip, hipMemcpyDeviceToDevice,
                              h->stream));
    }
    h->carry = rest;
    h->skip = rest ? skip : 0;
    h->sorigin += used - h->scan_skip;
    h->scanned = false;
    h->feed_stats[5] += now_ms() - t0;
    return collect_ready(h, false);
}

}  // namespace vsgpu

// ============================================================================
// exported C ABI
// ============================================================================
VS_API const char *vs_last_error(void) { return g_err.c_str(); }
VS_API const char *vs_version(void) { return "volsync_amd vsgpu 0.1 (gfx950)"; }

VS_API int vs_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) {
        (void)hipGetLastError();
        return 0;
    }
    return n;
}

VS_API int vs_pol_deg(uint64_t pol) { return pol_deg(pol); }
VS_API int vs_pol_irreducible(uint64_t pol) { return pol_irreducible(pol) ? 1 : 0; }
VS_API int vs_pol_tables(uint64_t pol, uint64_t out_tab[256], uint64_t mod_tab[256]) {
    if (!pol) return fail(VS_ERR_POLY, "tables for polynomial computation not initialized");
    if (pol_deg(pol) > 56) return fail(VS_ERR_POLY, "polynomial degree > 56");
    pol_tables(pol, out_tab, mod_tab);
    return 0;
}

VS_API int vs_cdc_open(int device, uint64_t pol, uint32_t min_size, uint32_t max_size,
                       uint32_t avg_bits, vs_cdc **out) {
    if (!out) return fail(VS_ERR_ARG, "null handle out-pointer");
    *out = nullptr;
    int ndev = vs_device_count();
    if (ndev <= 0) return fail(VS_ERR_NO_DEVICE, "no HIP device available (no CPU fallback)");
    if (device < 0 || device >= ndev) return fail(VS_ERR_ARG, "device index out of range");
    vs_cdc *h = new vs_cdc();
    h->device = device;
    if (set_dev(h) < 0) {
        delete h;
        return VS_ERR_NO_DEVICE;
    }
    if (hipStreamCreateWithFlags(&h->own, hipStreamNonBlocking) != hipSuccess ||
        hipStreamCreateWithFlags(&h->own_h, hipStreamNonBlocking) != hipSuccess ||
        hipEventCreateWithFlags(&h->ev_ready, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&h->ev_null, hipEventDisableTiming) != hipSuccess ||
        !(h->pinned = (uint64_t *)pinned_alloc(64))) {
        const hipError_t e = hipGetLastError();
        vs_cdc_close(h);
        return fail(VS_ERR_HIP, std::string("stream / event / pinned word creation failed: ") +
                                    hipGetErrorName(e));
    }
    h->stream = h->own;
    h->hstream = h->own_h;
    if (hipDeviceGetAttribute(&h->cus, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess)
        h->cus = 256;
    if (h->sha.init(device) < 0) {
        std::string msg = g_err;
        vs_cdc_close(h);
        g_err = msg;
        return VS_ERR_NOMEM;
    }
    int r = set_params(h, pol, min_size, max_size, avg_bits);
    if (r < 0) {
        std::string msg = g_err;
        vs_cdc_close(h);
        g_err = msg;
        return r;
    }
    *out = h;
    return 0;
}

VS_API int vs_cdc_reset(vs_cdc *h, uint64_t pol, uint32_t min_size, uint32_t max_size,
                        uint32_t avg_bits) {
    if (!h) return fail(VS_ERR_ARG, "null handle");
    VS_TRY(set_dev(h));
    // drain the hash engine first: chains queued by earlier batches still
    // write blob IDs into their ring slots, which size_ring() releases when
    // the new max_size changes the ring length
    VS_TRY(cdc_wait(h));
    if (h->streaming) {
        h->hash_budget = h->pre_stream_budget;   // the device API's budget again
        h->sha.isolate = h->pre_stream_isolate;
        if (h->own_hm && h->hstream == h->own_hm) h->hstream = h->own_h;
    }
    VS_TRY(set_params(h, pol, min_size, max_size, avg_bits));
#ifdef VS_STREAM_TRACE
    constexpr bool trace = true;   // debug builds: host time split of a stream
#else
    constexpr bool trace = false;
#endif
    if (trace && h->streaming)
        fprintf(stderr, "stream: host ms stitch %.1f finish %.1f scan %.1f\n", h->dbg_ms[0],
                h->dbg_ms[1], h->dbg_ms[2]);
    h->state = 0;
    h->ready.clear();
    h->spend.clear();
    h->sorigin = 0;
    h->final_fed = false;
    h->copy_pending = false;
    h->dma_wait = false;
    h->scanned = false;
    h->fill_new = 0;
    h->carry = 0;
    h->skip = 0;
    if (h->cstream) VS_HIP(hipStreamSynchronize(h->cstream));
    h->streaming = false;   // the next feed re-derives the streaming slice budget
    return 0;
}

VS_API int vs_cdc_set_batch_bytes(vs_cdc *h, uint64_t bytes) {
    if (!h || bytes < 1) return fail(VS_ERR_ARG, "bad batch size");
    if (h->streaming) return fail(VS_ERR_STATE, "batch size is fixed while a stream is fed (vs_cdc_reset first)");
    h->batch_bytes = bytes;
    return 0;
}

VS_API int vs_cdc_feed(vs_cdc *h, const void *buf, size_t n, int final) {
    if (!h) return fail(VS_ERR_ARG, "null handle");
    if (h->final_fed) return fail(VS_ERR_STATE, "stream already finalised (call vs_cdc_reset)");
    if (n && !buf) return fail(VS_ERR_ARG, "null buffer");
    VS_TRY(set_dev(h));
    VS_TRY(stream_begin(h));
    const uint8_t *src = (const uint8_t *)buf;
    size_t left = n;
    const uint64_t batch = stream_new_bytes(h);
    while (left) {
        DevBuf *cur = nullptr;
        VS_TRY(stream_buffer(h, h->fill_seq, &cur));
        const uint64_t take = std::min<uint64_t>(batch - h->fill_new, left);
        VS_TRY(stream_copy(h, (uint8_t *)cur->p + stream_pad(h) + h->fill_new, src, take));
        h->fill_new += take;
        src += take;
        left -= take;
        // the previous batch's cut selection waits until this batch is full:
        // its fingerprint pass then had the whole batch's copies to finish in
        if (h->fill_new == batch) {
            VS_TRY(stream_finish(h));
            VS_TRY(stream_scan(h, false));
        }
    }
    if (final) {
        VS_TRY(stream_finish(h));
        VS_TRY(stream_scan(h, true));
        VS_TRY(stream_finish(h));
        h->final_fed = true;
    }
    if (h->dma_wait) {
        // pinned caller memory: its copies must be complete before returning
        const double t0 = now_ms();
        VS_HIP(hipStreamSynchronize(h->cstream));
        h->feed_stats[4] += now_ms() - t0;
        h->dma_wait = false;
    }
    return 0;
}

// wait_any: with no chunk ready, wait for the oldest batch in flight instead of
// asking for more input (the caller's bound on bytes held, vs_cdc_next_wait)
static int cdc_next(vs_cdc *h, vs_chunk *out, size_t cap, size_t *n_out, bool wait_any) {
    if (!h || (!out && cap)) return fail(VS_ERR_ARG, "bad arguments");
    if (n_out) *n_out = 0;
    if (h->streaming) {
        VS_TRY(set_dev(h));
        // after the final feed nothing else will advance the stream: wait
        VS_TRY(collect_ready(h, h->ready.empty() && (h->final_fed || wait_any)));
    }
    size_t k = 0;
    while (k < cap && !h->ready.empty()) {
        out[k++] = h->ready.front();
        h->ready.pop_front();
    }
    if (n_out) *n_out = k;
    if (k == 0 && h->final_fed && h->spend.empty()) return VS_EOF;
    return 0;
}

VS_API int vs_cdc_next(vs_cdc *h, vs_chunk *out, size_t cap, size_t *n_out) {
    return cdc_next(h, out, cap, n_out, false);
}

VS_API int vs_cdc_next_wait(vs_cdc *h, vs_chunk *out, size_t cap, size_t *n_out) {
    return cdc_next(h, out, cap, n_out, true);
}

VS_API int vs_cdc_inflight(vs_cdc *h, uint64_t *batches) {
    if (!h || !batches) return fail(VS_ERR_ARG, "bad arguments");
    *batches = h->spend.size();
    return 0;
}

VS_API int vs_cdc_stream_stats(vs_cdc *h, double out[8]) {
    if (!h || !out) return fail(VS_ERR_ARG, "bad arguments");
    for (int i = 0; i < 8; ++i) out[i] = h->feed_stats[i];
    return 0;
}

VS_API void vs_cdc_close(vs_cdc *h) {
    if (!h) return;
    (void)hipSetDevice(h->device);
    if (h->stream) (void)hipStreamSynchronize(h->stream);
    if (h->hstream) (void)hipStreamSynchronize(h->hstream);
    DevBuf *bufs[] = {&h->tabs,     &h->counts,    &h->offs,   &h->dslot,   &h->pool,
                      &h->flags,    &h->cstart,    &h->partials, &h->compact, &h->spec_cut,
                      &h->spec_n,   &h->spec_exit, &h->st_cut, &h->st_n,    &h->st_merge,
                      &h->st_total, &h->exit_a,    &h->exit_b, &h->seg_off, &h->n_out};
    for (DevBuf *b : bufs) b->release();
    for (DevBuf &b : h->sbufs) b.release();
    if (h->cstream) (void)hipStreamSynchronize(h->cstream);
    for (int i = 0; i < 2; ++i) {
        if (h->stage[i]) (void)hipHostFree(h->stage[i]);
        if (h->stage_ev[i]) (void)hipEventDestroy(h->stage_ev[i]);
    }
    if (h->ev_copy) (void)hipEventDestroy(h->ev_copy);
    if (h->cstream) (void)hipStreamDestroy(h->cstream);
    if (h->own_hm) {
        (void)hipStreamSynchronize(h->own_hm);
        (void)hipStreamDestroy(h->own_hm);
    }
    for (auto &s : h->slots) {
        s.start.release();
        s.end.release();
        s.cut.release();
        s.id.release();
    }
    h->sha.release();
    for (auto &p : h->pend) {
        (void)hipEventDestroy(p.a);
        (void)hipEventDestroy(p.b);
    }
    for (auto e : h->ev_pool) (void)hipEventDestroy(e);
    for (auto e : h->slice_ev)
        if (e) (void)hipEventDestroy(e);
    pinned_free(h->pinned);
    PinnedVec<uint8_t>().swap(h->rb);
    if (h->ev_ready) (void)hipEventDestroy(h->ev_ready);
    if (h->ev_null) (void)hipEventDestroy(h->ev_null);
    if (h->anchor) (void)hipEventDestroy(h->anchor);
    if (h->own_h) (void)hipStreamDestroy(h->own_h);
    if (h->own) (void)hipStreamDestroy(h->own);
    delete h;
}

VS_API int vs_cdc_set_stream(vs_cdc *h, void *hip_stream) {
    if (!h) return fail(VS_ERR_ARG, "null handle");
    h->stream = hip_stream ? (hipStream_t)hip_stream : h->own;
    return 0;
}

VS_API int vs_cdc_set_hash_stream(vs_cdc *h, void *hip_stream) {
    if (!h) return fail(VS_ERR_ARG, "null handle");
    VS_TRY(cdc_wait(h));  // the engine's queued work stays on the old stream
    h->hstream = hip_stream ? (hipStream_t)hip_stream : h->own_h;
    return 0;
}

VS_API int vs_cdc_set_hash_slice(vs_cdc *h, uint32_t blocks) {
    if (!h) return fail(VS_ERR_ARG, "null handle");
    if (h->streaming) return fail(VS_ERR_STATE, "slice budget is fixed while a stream is fed (vs_cdc_reset first)");
    VS_TRY(cdc_wait(h));
    h->hash_budget = blocks ? blocks : 0xffffffffu;
    return size_ring(h);
}

static void set_wide(ShaEngine &e, uint32_t min_chains, uint32_t drain_blocks) {
    e.wide_min = min_chains ? min_chains : e.wide_default;
    e.wide_budget = drain_blocks ? drain_blocks : 4096;
}

VS_API int vs_cdc_set_hash_wide(vs_cdc *h, uint32_t min_chains, uint32_t drain_blocks) {
    if (!h) return fail(VS_ERR_ARG, "null handle");
    VS_TRY(cdc_wait(h));
    set_wide(h->sha, min_chains, drain_blocks);
    return 0;
}

VS_API int vs_cdc_get_batch_chunks(vs_cdc *h, uint64_t batch, uint64_t first, uint64_t n,
                                   vs_chunk *out) {
    if (!h) return fail(VS_ERR_ARG, "null handle");
    VS_TRY(set_dev(h));
    return cdc_get_batch(h, batch, first, n, out);
}

VS_API int vs_cdc_batches(vs_cdc *h, uint64_t *finished, uint64_t *ring) {
    if (!h) return fail(VS_ERR_ARG, "null handle");
    if (finished) *finished = h->seq;
    if (ring) *ring = h->slots.size();
    return 0;
}

VS_API int vs_cdc_scan(vs_cdc *h, const void *dev_data, uint64_t len, uint64_t origin,
                       uint64_t own_lo, uint64_t own_hi, int final) {
    return cdc_scan(h, dev_data, len, origin, own_lo, own_hi, final);
}

VS_API int vs_cdc_stitch(vs_cdc *h, uint64_t entry, uint64_t *exit_pos, int *complete) {
    return cdc_stitch(h, entry, exit_pos, complete);
}

VS_API int vs_cdc_finish(vs_cdc *h, uint64_t *n_chunks) { return cdc_finish(h, n_chunks); }

VS_API int vs_cdc_process(vs_cdc *h, const void *dev_data, uint64_t len, uint64_t origin,
                          int final, uint64_t *n_chunks, uint64_t *consumed) {
    return cdc_process(h, dev_data, len, origin, final, n_chunks, consumed);
}

VS_API int vs_cdc_wait(vs_cdc *h) { return cdc_wait(h); }

VS_API int vs_cdc_fence(vs_cdc *h, uint64_t batch) {
    if (!h) return fail(VS_ERR_ARG, "null handle");
    if (batch >= h->seq) return fail(VS_ERR_STATE, "no such finished batch");
    VS_TRY(set_dev(h));
    if (h->slots.empty()) return 0;
    const size_t k = (size_t)(batch % h->slots.size());
    // a recycled slot's batch was waited for when its slot was reused
    if (h->slots[k].seq != batch) return 0;
    return slot_free(h, k);
}

VS_API int vs_cdc_get_chunks(vs_cdc *h, uint64_t first, uint64_t n, vs_chunk *out) {
    return cdc_get_chunks(h, first, n, out);
}

VS_API int vs_cdc_timing(vs_cdc *h, int enable, double ms_out[4], uint64_t launches_out[4]) {
    if (!h) return fail(VS_ERR_ARG, "null handle");
    VS_TRY(cdc_wait(h));
    if (ms_out)
        for (int i = 0; i < 4; ++i) ms_out[i] = h->ms[i];
    if (launches_out)
        for (int i = 0; i < 4; ++i) launches_out[i] = h->launches[i];
    // SHA-256 kernel time inside / outside the union of fingerprint windows
    {
        auto &f = h->win_fp;
        std::sort(f.begin(), f.end());
        std::vector<std::pair<double, double>> u;  // union of the fingerprint windows
        for (auto &w : f) {
            if (!u.empty() && w.first <= u.back().second) u.back().second = std::max(u.back().second, w.second);
            else u.push_back(w);
        }
        double sha = 0, inside = 0, fp = 0;
        for (auto &w : u) fp += w.second - w.first;
        for (auto &w : h->win_sha) {
            sha += w.second - w.first;
            for (auto &v : u) inside += std::max(0.0, std::min(w.second, v.second) - std::max(w.first, v.first));
        }
        h->detail[0] = sha;
        h->detail[1] = sha - inside;  // SHA-256 kernel time outside every fingerprint window
        h->detail[2] = inside;
        h->detail[3] = fp;            // the fingerprint windows' union
        h->win_fp.clear();
        h->win_sha.clear();
    }
    for (int i = 0; i < 4; ++i) {
        h->ms[i] = 0;
        h->launches[i] = 0;
    }
    h->timing = enable != 0;
    h->anchored = false;
    if (h->timing) h->quad_chains = 0;
    if (h->timing) {
        if (!h->anchor) VS_HIP(hipEventCreate(&h->anchor));
        VS_HIP(hipEventRecord(h->anchor, h->stream));
        h->anchored = true;
    }
    return 0;
}

VS_API int vs_cdc_timing_detail(vs_cdc *h, double out[4], uint64_t *quad_chains) {
    if (!h || !out) return fail(VS_ERR_ARG, "bad arguments");
    for (int i = 0; i < 4; ++i) out[i] = h->detail[i];
    if (quad_chains) *quad_chains = h->quad_chains;
    h->quad_chains = 0;
    return 0;
}

struct vs_sha {
    int device = 0;
    ShaEngine eng;
    DevBuf dd_tmp;                  // vs_blob_dedup scratch
    DevBuf dd_flag;                 // vs_blob_dedup_known: per-blob "in the index" flags
    DevBuf ix_tmp;                  // vs_blob_index_sort scratch
    uint64_t *dd_pinned = nullptr;
    DevBuf blk_off, blk_len;        // vs_sha256_blocks descriptors
    DevBuf vf_ids, vf_cnt;          // vs_blob_verify scratch
    hipEvent_t done = nullptr;  // after the last use of the handle's scratch, on its stream
    bool ran = false;
    Stager stage;                   // vs_sha256_batch: caller host buffers
};

VS_API int vs_sha256_open(int device, vs_sha **out) {
    if (!out) return fail(VS_ERR_ARG, "null handle out-pointer");
    *out = nullptr;
    const int ndev = vs_device_count();
    if (ndev <= 0) return fail(VS_ERR_NO_DEVICE, "no HIP device available (no CPU fallback)");
    if (device < 0 || device >= ndev) return fail(VS_ERR_ARG, "device index out of range");
    VS_TRY(enter_device(device));
    vs_sha *h = new vs_sha();
    h->device = device;
    // many independent blobs (C5): throughput mode from 384 active blobs per
    // CU (split mode saturates at 5 x 64 per CU).  vs_cdc
    // handles keep split mode: their long chunks' latency is the tail.
    const bool ok = h->eng.init(device) == 0;
    h->eng.wide_default = (uint32_t)std::max(h->eng.cus, 1) * 384;
    h->eng.wide_min = h->eng.wide_default;
    if (!ok ||
        hipEventCreateWithFlags(&h->done, hipEventDisableTiming) != hipSuccess) {
        std::string msg = g_err;
        vs_sha256_close(h);
        g_err = msg;
        return VS_ERR_NOMEM;
    }
    *out = h;
    return 0;
}

// blob IDs of n device blobs with the hash engine: append + one unbounded slice
static int sha_run(vs_sha *h, const uint8_t *buf, const uint64_t *off, const uint32_t *len,
                   size_t n, uint8_t *out, hipStream_t s) {
    if (h->ran) VS_HIP(hipStreamWaitEvent(s, h->done, 0));  // engine buffers of the last run
    VS_TRY(h->eng.append_blobs(buf, off, len, n, out, s));
    VS_TRY(h->eng.slice(0xffffffffu, s));
    VS_HIP(hipEventRecord(h->done, s));
    h->ran = true;
    return 0;
}

VS_API int vs_sha256_run_device(vs_sha *h, const void *dev_buf, const uint64_t *dev_off,
                                const uint32_t *dev_len, size_t n, uint8_t *dev_out,
                                void *hip_stream) {
    if (!h) return fail(VS_ERR_ARG, "null handle");
    if (n && (!dev_buf || !dev_off || !dev_len || !dev_out))
        return fail(VS_ERR_ARG, "null device pointer");
    if (!n) return 0;
    VS_TRY(enter_device(h->device));
    return sha_run(h, (const uint8_t *)dev_buf, dev_off, dev_len, n, dev_out,
                   (hipStream_t)hip_stream);
}

VS_API int vs_sha256_blocks(vs_sha *h, const void *dev_buf, uint64_t len, uint32_t block_size,
                            uint8_t *dev_out, void *hip_stream) {
    if (!h || !block_size || (len && (!dev_buf || !dev_out))) return fail(VS_ERR_ARG, "bad arguments");
    const uint64_t n = (len + block_size - 1) / block_size;
    if (!n) return 0;
    VS_TRY(enter_device(h->device));
    const hipStream_t s = (hipStream_t)hip_stream;
    if (h->ran) VS_HIP(hipStreamWaitEvent(s, h->done, 0));   // descriptors of the last run
    VS_TRY(h->blk_off.ensure(n * 8));
    VS_TRY(h->blk_len.ensure(n * 4));
    VS_HIP(launch_blk_desc(len, block_size, n, h->blk_off.as<uint64_t>(), h->blk_len.as<uint32_t>(), s));
    return sha_run(h, (const uint8_t *)dev_buf, h->blk_off.as<uint64_t>(), h->blk_len.as<uint32_t>(), n,
                   dev_out, s);
}

VS_API int vs_syncthing_block_size(int64_t file_size) {
    // lib/protocol BlockSize: the smallest of 128 KiB .. 16 MiB (powers of
    // two) that keeps the file under 2000 blocks, else 16 MiB
    int bs = 128 << 10;
    for (; bs < (16 << 20); bs *= 2)
        if (file_size < 2000ll * bs) break;
    return bs;
}

VS_API int vs_blob_verify(vs_sha *h, const void *dev_buf, const uint64_t *dev_off,
                          const uint32_t *dev_len, size_t n, const uint8_t *dev_want,
                          uint32_t *dev_bad, uint64_t *n_bad, void *hip_stream) {
    if (!h || (n && (!dev_buf || !dev_off || !dev_len || !dev_want)))
        return fail(VS_ERR_ARG, "bad arguments");
    if (n_bad) *n_bad = 0;
    if (!n) return 0;
    VS_TRY(enter_device(h->device));
    const hipStream_t s = (hipStream_t)hip_stream;
    if (h->ran) VS_HIP(hipStreamWaitEvent(s, h->done, 0));
    VS_TRY(h->vf_ids.ensure(n * 32));
    VS_TRY(h->vf_cnt.ensure(8));
    VS_TRY(sha_run(h, (const uint8_t *)dev_buf, dev_off, dev_len, n, h->vf_ids.as<uint8_t>(), s));
    VS_HIP(launch_verify(h->vf_ids.as<uint8_t>(), dev_want, n, dev_bad,
                         h->vf_cnt.as<unsigned long long>(), s));
    VS_HIP(hipEventRecord(h->done, s));   // vf_ids / vf_cnt are read until here
    if (n_bad) {
        if (!h->dd_pinned &&
            hipHostMalloc((void **)&h->dd_pinned, 64, hipHostMallocDefault) != hipSuccess) {
            (void)hipGetLastError();
            return fail(VS_ERR_NOMEM, "pinned read-back buffer");
        }
        VS_HIP(hipMemcpyAsync(h->dd_pinned, h->vf_cnt.p, 8, hipMemcpyDeviceToHost, s));
        VS_HIP(hipStreamSynchronize(s));
        *n_bad = h->dd_pinned[0];
    }
    return 0;
}

VS_API int vs_blob_dedup(vs_sha *h, const uint8_t *dev_ids, size_t n, uint32_t *dev_first,
                         uint64_t *n_unique, void *hip_stream) {
    if (!h || (n && (!dev_ids || !dev_first))) return fail(VS_ERR_ARG, "bad arguments");
    VS_TRY(enter_device(h->device));
    const hipStream_t s = (hipStream_t)hip_stream;
    // the distinct-ID counter takes the first 256 bytes: dd_first_kernel adds
    // to it with a 64-bit atomic, which faults unless 8-byte aligned (at the
    // buffer's end it sat wherever the sort's scratch size left it)
    if (n > 0x7fffffffull) return fail(VS_ERR_ARG, "more than 2^31 - 1 blobs per call (radix sort count)");
    if (((uintptr_t)dev_ids & 15) != 0) return fail(VS_ERR_ARG, "blob IDs must be 16-byte aligned");
    // dd_tmp may still be read by the previous dedup on another stream
    if (h->ran) VS_HIP(hipStreamWaitEvent(s, h->done, 0));
    VS_TRY(h->dd_tmp.ensure(dedup_tmp_bytes(std::max<size_t>(n, 1)) + 256));
    unsigned long long *cnt = (unsigned long long *)h->dd_tmp.p;
    VS_HIP(launch_dedup(dev_ids, n, dev_first, (uint8_t *)h->dd_tmp.p + 256, h->dd_tmp.cap - 256,
                        cnt, s));
    VS_HIP(hipEventRecord(h->done, s));
    h->ran = true;
    if (n_unique) {
        if (!h->dd_pinned &&
            hipHostMalloc((void **)&h->dd_pinned, 64, hipHostMallocDefault) != hipSuccess) {
            (void)hipGetLastError();
            return fail(VS_ERR_NOMEM, "pinned read-back buffer");
        }
        VS_HIP(hipMemcpyAsync(h->dd_pinned, cnt, 8, hipMemcpyDeviceToHost, s));
        VS_HIP(hipStreamSynchronize(s));
        *n_unique = h->dd_pinned[0];
    }
    return 0;
}

VS_API int vs_blob_dedup_known(vs_sha *h, const uint8_t *dev_ids, size_t n,
                               const uint8_t *dev_known, size_t n_known, uint32_t *dev_first,
                               uint64_t *n_new, void *hip_stream) {
    if (!h || (n_known && !dev_known)) return fail(VS_ERR_ARG, "bad arguments");
    if (((uintptr_t)dev_known & 15) != 0) return fail(VS_ERR_ARG, "known IDs must be 16-byte aligned");
    // the batch's own first occurrences (vs_blob_dedup), without its count
    VS_TRY(vs_blob_dedup(h, dev_ids, n, dev_first, nullptr, hip_stream));
    const hipStream_t s = (hipStream_t)hip_stream;
    VS_TRY(h->dd_flag.ensure(dedup_known_tmp_bytes(std::max<size_t>(n, 1))));
    unsigned long long *cnt = (unsigned long long *)h->dd_tmp.p + 8;   // its own 8-byte slot
    VS_HIP(launch_dedup_known(dev_ids, n, dev_known, n_known, dev_first, h->dd_flag.p, cnt, s));
    VS_HIP(hipEventRecord(h->done, s));
    if (n_new) {
        if (!h->dd_pinned &&
            hipHostMalloc((void **)&h->dd_pinned, 64, hipHostMallocDefault) != hipSuccess) {
            (void)hipGetLastError();
            return fail(VS_ERR_NOMEM, "pinned read-back buffer");
        }
        VS_HIP(hipMemcpyAsync(h->dd_pinned, cnt, 8, hipMemcpyDeviceToHost, s));
        VS_HIP(hipStreamSynchronize(s));
        *n_new = h->dd_pinned[0];
    }
    return 0;
}

VS_API int vs_blob_index_sort(vs_sha *h, uint8_t *dev_known, size_t n, void *hip_stream) {
    if (!h || (n && !dev_known)) return fail(VS_ERR_ARG, "bad arguments");
    if (n > 0x7fffffffull) return fail(VS_ERR_ARG, "more than 2^31 - 1 known IDs (radix sort count)");
    if (((uintptr_t)dev_known & 15) != 0) return fail(VS_ERR_ARG, "known IDs must be 16-byte aligned");
    VS_TRY(enter_device(h->device));
    const hipStream_t s = (hipStream_t)hip_stream;
    if (h->ran) VS_HIP(hipStreamWaitEvent(s, h->done, 0));
    VS_TRY(h->ix_tmp.ensure(index_sort_tmp_bytes(std::max<size_t>(n, 1)) + 256));
    VS_HIP(launch_index_sort(dev_known, n, h->ix_tmp.p, h->ix_tmp.cap, s));
    VS_HIP(hipEventRecord(h->done, s));
    h->ran = true;
    return 0;
}

// the options a vs_cdc / vs_sha handle takes (vsgpu.h); the engine's quad
// (latency-mode) share of the final drain: 0 = split mode only
static int sha_option(ShaEngine &e, int option, int64_t value) {
    if (option == VS_OPT_SHA_GRID_PER_CU) {
        if (value < 0 || value > 5) return fail(VS_ERR_ARG, "grid per CU out of range [0, 5]");
        e.grid_per_cu = (uint32_t)value;
        return 0;
    }
    if (option == VS_OPT_SHA_ISOLATE) {
        if (value < 0 || value > 1) return fail(VS_ERR_ARG, "isolate is 0 or 1");
        e.isolate = (uint32_t)value;
        return 0;
    }
    if (option != VS_OPT_SHA_QUAD_PCT) return fail(VS_ERR_ARG, "unknown option " + std::to_string(option));
    if (value < -1 || value > 1000) return fail(VS_ERR_ARG, "quad share out of range");
    e.quad_pct = value < 0 ? ShaEngine::kQuadAuto : (uint32_t)value;
    return 0;
}

VS_API int vs_cdc_set_option(vs_cdc *h, int option, int64_t value) {
    if (!h) return fail(VS_ERR_ARG, "null handle");
    VS_TRY(cdc_wait(h));
    if (option == VS_OPT_FP_GENERIC) {
        h->fp_generic = value != 0;
        return 0;
    }
    if (option == VS_OPT_SHA_ISOLATE && h->streaming) {   // applies once the stream ends
        const uint32_t cur = h->sha.isolate;
        VS_TRY(sha_option(h->sha, option, value));
        h->pre_stream_isolate = h->sha.isolate;
        h->sha.isolate = cur;
        return 0;
    }
    return sha_option(h->sha, option, value);
}

VS_API int vs_sha256_set_option(vs_sha *h, int option, int64_t value) {
    if (!h) return fail(VS_ERR_ARG, "null handle");
    if (h->ran) VS_HIP(hipEventSynchronize(h->done));
    return sha_option(h->eng, option, value);
}

VS_API int vs_sha256_drain_stats(vs_sha *h, uint64_t out[2]) {
    if (!h || !out) return fail(VS_ERR_ARG, "null argument");
    if (h->ran) VS_HIP(hipEventSynchronize(h->done));
    out[0] = h->eng.last_quad_chains;
    out[1] = h->eng.last_iso_chains;
    return 0;
}

VS_API int vs_sha256_set_wide(vs_sha *h, uint32_t min_chains, uint32_t drain_blocks) {
    if (!h) return fail(VS_ERR_ARG, "null handle");
    if (h->ran) VS_HIP(hipEventSynchronize(h->done));
    set_wide(h->eng, min_chains, drain_blocks);
    return 0;
}

VS_API void vs_sha256_close(vs_sha *h) {
    if (!h) return;
    (void)hipSetDevice(h->device);
    (void)hipDeviceSynchronize();
    h->dd_tmp.release();
    for (DevBuf *b : {&h->blk_off, &h->blk_len, &h->vf_ids, &h->vf_cnt}) b->release();
    if (h->dd_pinned) (void)hipHostFree(h->dd_pinned);
    h->stage.release();
    if (h->done) {
        (void)hipEventSynchronize(h->done);
        (void)hipEventDestroy(h->done);
    }
    h->eng.release();
    delete h;
}

VS_API int vs_sha256_batch(int device, const void *buf, size_t buf_len, const uint64_t *off,
                           const uint32_t *len, size_t n, uint8_t (*out)[32]) {
    if (vs_device_count() <= 0) return fail(VS_ERR_NO_DEVICE, "no HIP device available");
    if (n && (!buf || !off || !len || !out)) return fail(VS_ERR_ARG, "null pointer");
    for (size_t i = 0; i < n; ++i)
        if (off[i] + len[i] > buf_len) return fail(VS_ERR_ARG, "blob outside the buffer");
    if (!n) return 0;
    vs_sha *h = nullptr;
    VS_TRY(vs_sha256_open(device, &h));
    DevBuf d, o, l, r;
    int rc = 0;
    if ((rc = d.ensure(std::max<size_t>(buf_len, 16))) < 0 || (rc = o.ensure(n * 8)) < 0 ||
        (rc = l.ensure(n * 4)) < 0 || (rc = r.ensure(n * 32)) < 0) {
    } else if ((rc = h->stage.h2d(d.p, buf, buf_len, nullptr)) < 0 ||
               (rc = h->stage.h2d(o.p, off, n * 8, nullptr)) < 0 ||
               (rc = h->stage.h2d(l.p, len, n * 4, nullptr)) < 0) {
    } else if ((rc = sha_run(h, d.as<uint8_t>(), o.as<uint64_t>(), l.as<uint32_t>(), n,
                             r.as<uint8_t>(), nullptr)) == 0) {
        rc = h->stage.d2h(out, r.p, n * 32, nullptr);
    }
    vs_sha256_close(h);
    d.release();
    o.release();
    l.release();
    r.release();
    return rc;
}

VS_API int vs_synth_fill_device(int device, uint64_t seed, uint64_t off, uint64_t n,
                                void *dev_out, void *hip_stream) {
    if (vs_device_count() <= 0) return fail(VS_ERR_NO_DEVICE, "no HIP device available");
    VS_TRY(enter_device(device));
    VS_HIP(launch_synth(seed, off, n, (uint8_t *)dev_out, (hipStream_t)hip_stream));
    if (!hip_stream) VS_HIP(hipStreamSynchronize(nullptr));  // NULL stream: blocking fill
    return 0;
}
