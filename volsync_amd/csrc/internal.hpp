// internal.hpp -- shared declarations of the gfx950 CDC + SHA-256 pipeline.
// Public ABI: include/vsgpu.h.  Design: DESIGN.md.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <algorithm>
#include <string>
#include <functional>
#include <vector>

#include "../../include/vsgpu.h"
#include "filesum.hpp"

namespace vsgpu {

// ---- error plumbing -------------------------------------------------------
void set_error(const std::string &msg);
int fail(int code, const std::string &msg);
// VS_ERR_HIP with the call, hipGetErrorName, the numeric code, the message and
// the source line (xfer.cpp); clears the runtime's last error
int fail_hip(hipError_t e, const char *what, const char *file, int line);
#define VS_HIP(call)                                                                  \
    do {                                                                              \
        hipError_t e_ = (call);                                                       \
        if (e_ != hipSuccess) return ::vsgpu::fail_hip(e_, #call, __FILE__, __LINE__); \
    } while (0)
// every entry point that launches work: clears a stale last error the caller
// left on this thread, then hipSetDevice (VS_ERR_NO_DEVICE on failure)
int enter_device(int device);
#define VS_TRY(expr)                 \
    do {                             \
        int r_ = (expr);             \
        if (r_ < 0) return r_;       \
    } while (0)

// ---- device-to-host copies on an SDMA engine (xfer.cpp) --------------------------
// hsa_amd_memory_async_copy: runs beside kernels that hold every CU, where the
// HIP runtime's blit-kernel copies would queue behind them.  The caller orders
// it after the kernel that wrote the source (an event synchronisation).
struct DmaD2H {
    static constexpr int kSignals = 20;
    bool init(int device);                     // false: no DMA path (use hipMemcpyAsync)
    void release();
    bool start(int slot, void *dst, const void *src, size_t n);  // async; signal `slot`
    bool wait(int slot);                       // until copy `slot` has landed; false: it failed
    bool ready = false;

    int engine = -1;                           // the SDMA engine copies go to (-1: the runtime's pick)

  private:
    uint64_t gpu_ = 0, cpu_ = 0;               // hsa_agent_t handles
    uint64_t sig_[kSignals] = {};              // hsa_signal_t handles
};

// ---- host memory the DMA engines touch (xfer.cpp) -------------------------------
// The library page-locks only memory it allocated itself (hipHostMalloc):
// registering heap storage pins pages it shares with the caller's buffers.
void *pinned_alloc(size_t bytes);   // nullptr on failure
void pinned_free(void *p);
// [p, p + n) lies inside one page-locked host allocation (DMA it directly)
bool host_range_pinned(const void *p, size_t n);
// memcpy split over a few host threads for large copies (staging)
void par_memcpy(void *dst, const void *src, size_t n);

// std::vector storage in owned pinned pages: read-back targets the DMA engine
// writes directly (grows like any vector; every allocation is hipHostMalloc)
template <class T>
struct PinnedAlloc {
    using value_type = T;
    PinnedAlloc() = default;
    template <class U>
    PinnedAlloc(const PinnedAlloc<U> &) {}
    T *allocate(size_t n) {
        T *p = (T *)pinned_alloc(n * sizeof(T));
        if (!p) throw std::bad_alloc();
        return p;
    }
    void deallocate(T *p, size_t) { pinned_free(p); }
    template <class U>
    bool operator==(const PinnedAlloc<U> &) const { return true; }
    template <class U>
    bool operator!=(const PinnedAlloc<U> &) const { return false; }
};
template <class T>
using PinnedVec = std::vector<T, PinnedAlloc<T>>;
// resize without letting bad_alloc cross the C ABI
template <class V>
int pv_resize(V &v, size_t n) {
    try {
        v.resize(n);
    } catch (const std::bad_alloc &) {
        return fail(VS_ERR_NOMEM, "pinned host buffer of " + std::to_string(n) + " elements");
    }
    return 0;
}

// Copies between caller host memory (pageable or not) and the device through
// two owned pinned chunks.  h2d returns once the caller's bytes are staged
// (the DMA stays queued on s); d2h returns once dst holds the bytes.
struct Stager {
    static constexpr size_t kChunk = 8u << 20;
    uint8_t *buf[2] = {nullptr, nullptr};
    hipEvent_t ev[2] = {nullptr, nullptr};
    bool busy[2] = {false, false};
    int next = 0;
    int init();
    int wait(int i);
    int h2d(void *dst, const void *src, size_t n, hipStream_t s);
    int d2h(void *dst, const void *src, size_t n, hipStream_t s);
    void release();
};

// ---- device buffer that only grows ------------------------------------------
struct DevBuf {
    void *p = nullptr;
    size_t cap = 0;
    int ensure(size_t bytes) {
        if (bytes <= cap) return 0;
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
        size_t want = std::max<size_t>(bytes, 256);
        const hipError_t e = hipMalloc(&p, want);
        if (e != hipSuccess) {
            p = nullptr;
            (void)hipGetLastError();
            return fail(VS_ERR_NOMEM, "hipMalloc of " + std::to_string(want) + " bytes failed: " +
                                          hipGetErrorName(e));
        }
        cap = want;
        return 0;
    }
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
    }
    template <class T>
    T *as() const {
        return (T *)p;
    }
};

// ---- Rabin tables (chunker.go fillTables) ----------------------------------
int pol_deg(uint64_t p);
uint64_t pol_mod(uint64_t x, uint64_t d);
bool pol_irreducible(uint64_t p);
void pol_tables(uint64_t pol, uint64_t out_tab[256], uint64_t mod_tab[256]);
// out8[b] = b * x^512 mod P  (= appendByte(out[b], 0)): the evicted-byte term of
// the rolling window written against the shifted digest.
void pol_out8(uint64_t pol, const uint64_t out_tab[256], uint64_t out8[256]);

// ---- fingerprint pass ------------------------------------------------------
// 16 waves per CU (128 VGPRs; the hot loop spill-free, 78 spilled VGPRs in
// the rare re-roll / bounds-checked paths) against 12 (168 VGPRs): 21.4 vs
// 21.8 ms per 64 GiB in three interleaved rounds, C2 1033.7 vs 1023.3 GB/s
// (profiles/r05_fp); more chains per wave instead (3 or 4 strips per lane at
// 8 or 12 waves) measured 25.8-26.7 ms: the pass wants independent waves
// issuing, not deeper per-wave interleaving
#ifndef VS_FP_THREADS
#define VS_FP_THREADS 1024
#endif
constexpr int kFpThreads = VS_FP_THREADS;  // one workgroup per CU (LDS: 128 KiB tables)
constexpr int kFpCopies = 32;      // lane-private table copies: conflict-free ds_read_b64
constexpr int kSlots = 3;          // candidate offsets kept per strip (dense strips: bitmask)
constexpr uint32_t kNoSlot = 0xffffffffu;
// flags words: [0] scan errors (pool overflow, dense strip without bitmask),
// [1] dense pool bump cursor, [2] stitch pass "an exit changed"
constexpr uint32_t kFlagPoolOverflow = 1u;
constexpr uint32_t kFlagChanged = 2u;
constexpr uint32_t kFlagDenseMissing = 4u;

struct FpArgs {
    const uint8_t *data;   // device bytes, 16-byte aligned base
    uint64_t dlen;         // readable bytes at data
    uint64_t base;         // data offset of strip 0 (multiple of 64)
    uint64_t scan_end;     // candidates are recorded for positions < scan_end
    uint64_t k_lo, k_hi;   // interior strips [k_lo, k_hi): reads need no bounds checks
    uint64_t n_edge;       // the other strips ([0, k_lo), [k_hi, nstrips)): bounds-checked
    uint32_t *work;        // interior work-unit counter (zeroed before the launch)
    uint32_t strip;        // bytes per strip (multiple of 64)
    uint32_t idx_shift;    // digest bit of the table index, minus 32 (deg - 40)
    uint32_t mask_lo, mask_hi;
    uint32_t *counts;      // [nstrips] candidates per strip
    uint32_t *offs;        // [nstrips * kSlots] first offsets within the strip
    uint32_t *dense_slot;  // [nstrips] pool slot of dense strips
    uint32_t *pool;        // [pool_cap * strip/32] candidate bitmasks
    uint32_t pool_cap;
    uint32_t *pool_next;   // bump allocator
    uint32_t *flags;
    const uint64_t *mod_tab;   // [256]
    const uint64_t *out8_tab;  // [256]
};
// fast: the FAST variant (idx_shift >= 8, i.e. deg >= 48)
hipError_t launch_fingerprint(const FpArgs &a, bool wide_mask, bool fast, int cus, hipStream_t s);

// ---- selection -------------------------------------------------------------
constexpr uint64_t kPosMask = (1ull << 62) - 1;
constexpr uint64_t kCutNormal = 0, kCutForced = 1ull << 62, kCutEof = 2ull << 62;
constexpr uint64_t kIncomplete = ~0ull;   // exit marker: a cut needs more data

struct SelArgs {
    // candidate index (from the fingerprint pass)
    uint64_t base;
    uint32_t strip;
    uint64_t nstrips;
    const uint32_t *counts, *offs, *dense_slot, *pool;
    const uint32_t *cstart;   // [nstrips+1] exclusive scan of min(count, kSlots)
    const uint64_t *compact;  // [cstart[nstrips]] candidate positions (data offsets)
    uint32_t *flags;
    // chunk rule
    uint64_t min_size, max_size;
    uint64_t scan_end, dlen;
    int final_eof;            // 1: the stream ends at dlen and scan_end == dlen
    // segments tiling [own_lo, own_hi)
    uint64_t own_lo, own_hi, seg_len;
    uint32_t nseg, maxc;
    uint64_t *spec_cut;       // [nseg * maxc]
    uint32_t *spec_n;         // [nseg]
    uint64_t *spec_exit;      // [nseg]
    uint64_t *st_cut;         // [nseg * maxc]
    uint32_t *st_n, *st_merge, *st_total;  // [nseg]
    uint64_t *exit_old, *exit_new;         // [nseg]
    uint64_t entry;
};
hipError_t launch_compact(const SelArgs &a, uint32_t *cstart_partials, uint64_t *compact,
                          uint32_t *cstart, hipStream_t s);
hipError_t launch_spec_walk(const SelArgs &a, hipStream_t s);
hipError_t launch_stitch(const SelArgs &a, hipStream_t s);
// chunk list: starts/ends (data offsets) + cut type, in stream order
hipError_t launch_emit(const SelArgs &a, uint32_t *seg_off, uint64_t *ch_start,
                       uint64_t *ch_end, uint64_t *n_out, hipStream_t s);
hipError_t launch_cut_fp(const uint8_t *data, uint64_t n, const uint64_t *ch_start,
                         const uint64_t *ch_end, uint64_t min_size, const uint64_t *mod_tab,
                         const uint64_t *out8_tab, uint32_t idx_shift, uint64_t *cut_out,
                         hipStream_t s);

// ---- SHA-256 hash engine (sha256.hip) --------------------------
// One active hash chain: a blob data[ptr0 .. end) of len bytes, advanced to
// ptr (ptr - ptr0 is a multiple of 64; ptr > end while only the second
// padding block is left), midstate st, digest destination out.  64 bytes.
struct ShaChain {
    uint64_t ptr, end, len;
    uint8_t *out;
    uint32_t st[8];
};
static_assert(sizeof(ShaChain) == 64, "ShaChain is one 64-byte record");

struct ShaSliceArgs {
    const ShaChain *cur;
    ShaChain *next;
    const uint32_t *order;   // longest-first permutation of cur
    const uint32_t *n_cur;   // device counts
    uint32_t *n_next;
    uint32_t *tile_ctr;
    uint32_t budget;         // max blocks per chain in this slice (0xffffffff: all)
    uint32_t quad_chains;    // the first (longest) chains of the order run in latency mode
    uint32_t quad_lo;        // sha_slice_kernel: of those, the first quad_lo run in an isolated
                             // drain's sha_iso_kernel; its own latency tiles take the rest
    uint32_t *resident;      // sha_iso_kernel: host-visible count of resident workgroups
};

// Host side of the engine: a double-buffered active list on the device, fed by
// append_*() and advanced by slice(); every call queues on the given stream
// (always the same one) without synchronising.
enum { kShaSplit = 0, kShaWide = 1, kShaQuad = 2 };
struct ShaEngine {
    struct Group {
        uint64_t n;
        uint32_t max_blocks;  // upper bound on any chain's remaining blocks
    };
    int device = 0;
    int cus = 256;
    DevBuf list[2], order, hist, ctl;  // ctl: u32 counts [0], [1] (list parity), [2] tile counter
    int cur = 0;
    uint64_t cap = 0;  // chains per list
    uint64_t ub = 0;   // upper bound on the active chains
    std::vector<Group> groups;
    // throughput mode (sha_slice_wide_kernel) once this many chains are active;
    // a drain advances them by wide_budget blocks per slice until fewer remain
    uint32_t wide_min = 0xffffffffu;  // never, unless the handle sets it
    uint32_t wide_default = 0xffffffffu;
    uint32_t wide_budget = 4096;
    uint32_t *live_h = nullptr;  // pinned: active-chain count read back during a drain
    // optional timing of the hash kernels alone (no bookkeeping launches):
    // when ev_get is set, launch() brackets each slice kernel with two events
    std::function<hipEvent_t()> ev_get;
    std::vector<std::pair<hipEvent_t, hipEvent_t>> kernel_pairs;
    int init(int dev);
    // the final drain runs its longest chains in latency (quad) mode
    // (VS_OPT_SHA_QUAD_PCT): kQuadAuto = every chain that would otherwise
    // finish after the drain's floor; p = those with at least p % of the
    // longest chain's remaining blocks; 0 disables
    static constexpr uint32_t kQuadAuto = 0xffffffffu;
    uint32_t quad_pct = kQuadAuto;
    uint32_t last_quad_chains = 0;  // chains the last drain ran in quad mode (stats)
    uint32_t last_iso_chains = 0;   // of those, in isolated tiles (sha_iso_kernel)
    // Isolated latency drain (VS_OPT_SHA_ISOLATE, default on): the latency
    // tiles run in sha_iso_kernel, 32 chains per workgroup, each holding a
    // CU alone (it asks for the CU's whole LDS), resident before the split
    // tiles are launched, so the drain's critical chains never share a CU
    // with the bulk
    uint32_t isolate = 1;
    hipStream_t iso_q = nullptr;
    hipEvent_t iso_ev[2] = {nullptr, nullptr};   // fork, quad tiles done
    uint32_t *iso_res_h = nullptr, *iso_res_d = nullptr;   // residency counter (host / device view)
    int iso_setup();
    // persistent-grid cap (VS_OPT_SHA_GRID_PER_CU): split mode workgroups per
    // CU (default 5, the LDS limit), throughput mode waves per SIMD (default 3)
    uint32_t grid_per_cu = 0;
    uint32_t *hist_h = nullptr;  // pinned: the drain's bucket histogram
    int launch(uint32_t budget, int mode, hipStream_t s);
    void release();
    uint32_t *count(int which);
    int reserve(uint64_t n_new, hipStream_t s);
    // chunks [starts[i], (ends[i] & kPosMask)] of data; digest i -> ids + 32 i
    int append_chunks(const uint8_t *data, const uint64_t *starts, const uint64_t *ends, uint64_t n,
                      uint8_t *ids, uint32_t max_blocks, hipStream_t s);
    int append_blobs(const uint8_t *data, const uint64_t *off, const uint32_t *lens, uint64_t n,
                     uint8_t *ids, hipStream_t s);
    int slice(uint32_t budget, hipStream_t s);
    bool idle() const { return ub == 0; }
};
// SHA-256 blocks of a blob of len bytes (data + padding)
inline uint64_t sha_blocks(uint64_t len) { return (len >> 6) + ((len & 63) < 56 ? 1 : 2); }

// ---- synthetic data --------------------------------------------------------
hipError_t launch_synth(uint64_t seed, uint64_t off, uint64_t n, uint8_t *out, hipStream_t s);

// ---- misc ---------------------------------------------------------------------
hipError_t launch_scan_u32(const uint32_t *in, uint32_t *out, uint64_t n, uint32_t *partials,
                           uint32_t clamp, hipStream_t s);

// ---- rsync delta matching (rsync.hip) ------------------------------------------
constexpr uint64_t kRsG = 4096;       // coarse prefix granularity (bytes)
constexpr uint64_t kRsStrip = 4096;   // offsets per scan lane (multiple of kRsG and 16)

struct RsSigArgs {
    const uint8_t *data;   // basis bytes
    uint64_t len;
    uint64_t count;        // blocks
    uint32_t blength, remainder, s2length;
    int csum_type;
    uint32_t seed;
    uint32_t *sum1;        // [count]
    uint8_t *sum2;         // [count * s2length]
};
hipError_t launch_rs_signatures(const RsSigArgs &a, hipStream_t s);
hipError_t launch_rs_strong(const uint8_t *data, const uint64_t *offs, const uint32_t *lens,
                            uint64_t n, int csum_type, uint32_t seed, uint32_t s2length,
                            uint8_t *out, uint32_t min_len, hipStream_t s);
// sort keys (sum1 << 32 | ~index) -> tkey, directory over the top dbits of sum1
// (2^dbits + 1 entries) and a 2^fbits-bit filter over the top fbits
hipError_t launch_rs_table(const uint32_t *sum1, uint32_t count, uint64_t *keys, uint64_t *tkey,
                           void *tmp, size_t tmp_bytes, uint32_t dbits, uint32_t *dir,
                           uint32_t fbits, uint32_t *filt, hipStream_t s);
size_t rs_sort_tmp_bytes(uint64_t n_keys, bool pairs);
// coarse prefixes: px/pt per kRsG block, *_scan exclusive (n+1 entries)
hipError_t launch_rs_prefix(const uint8_t *data, uint64_t len, uint32_t *px, uint32_t *pt,
                            uint32_t *px_scan, uint32_t *pt_scan, uint32_t *partials,
                            hipStream_t s);

struct RsScanArgs {
    const uint8_t *data;   // source bytes (data-relative offsets below)
    uint64_t len;          // readable bytes at data
    uint64_t lo;           // first offset reported (offsets below lo are skipped)
    uint64_t nfull;        // end (exclusive) of the full-window offsets reported (<= len - blength + 1)
    int64_t tail;          // the one shrunk-window offset that can match the short last block, or -1
    uint64_t blength;
    uint32_t count, remainder;
    const uint32_t *px_scan, *pt_scan;
    const uint64_t *tkey;  // sorted (sum1 << 32 | ~index)
    const uint32_t *dir;
    const uint32_t *filt;
    uint32_t dbits, fbits;
    // LDS prefilter: bit (sum >> (32 - lbits)) set iff some block's sum1 has
    // those top bits; lives right after filt in the same allocation
    const uint32_t *filt_l;
    uint32_t lbits;
    unsigned long long *n_cand;
    uint64_t cap;
    uint64_t *cand_off;    // [cap]
    uint32_t *cand_sum;    // [cap]
};
// bits of the LDS-resident prefilter (2^20 bits = 128 KiB) for an fbits filter
__host__ __device__ inline uint32_t rs_lds_filter_bits(uint32_t fbits) {
    return fbits < 20 ? fbits : 20;
}
// the device walk's L2-resident filter: a blocked Bloom filter of 2^fbits
// bits in 64-bit words -- the word from a multiplicative hash of sum1, three
// bits in it from sum1's low 18 bits -- so one gather per offset rejects all
// but ~0.1 % of the offsets the LDS prefilter passes (about 2 keys per word)
__host__ __device__ inline uint32_t rs_bloom_word(uint32_t sum1, uint32_t fbits) {
    return (sum1 * 0x9E3779B1u) >> (32 - (fbits - 6));
}
#ifndef VS_BLOOM_K
#define VS_BLOOM_K 3
#endif
__host__ __device__ inline uint64_t rs_bloom_mask(uint32_t sum1) {
    uint64_t m = 0;
#pragma unroll
    for (int j = 0; j < VS_BLOOM_K; ++j) m |= 1ull << ((sum1 >> (6 * j)) & 63);
    return m;
}
// Membership buckets for the walk's probe ("is there a full-length block with
// sum1 == s?"): 2^bbits buckets of 32 bytes -- a count, then up to 7 distinct
// sums -- so a probe is one 32-byte load instead of the directory + sorted-key
// round trips; a bucket whose count passed 7 falls back to those.
constexpr uint32_t kBucketWords = 8;
constexpr uint32_t kBucketSlots = kBucketWords - 1;
__host__ __device__ inline uint32_t rs_bucket(uint32_t sum1, uint32_t bbits) {
    return (sum1 * 0x85EBCA77u) >> (32 - bbits);
}
__host__ __device__ inline uint32_t rs_bucket_bits(uint32_t count) {
    uint32_t lc = 0;
    while ((1ull << lc) < (uint64_t)(count ? count : 1)) ++lc;
    return lc < 5 ? 4 : lc - 1;   // ~2 distinct sums per bucket (P(> 7) ~ 0.1 %)
}
// layout: filter [2^fbits bits], LDS prefilter [2^lbits bits], blocked filter [2^fbits bits]
inline size_t rs_filter_bytes(uint32_t fbits) {
    return 2 * (((size_t)1 << fbits) / 8) + (((size_t)1 << rs_lds_filter_bits(fbits)) / 8);
}
hipError_t launch_rs_scan(const RsScanArgs &a, int cus, hipStream_t s);
// flag[0, n): some candidate sits exactly one block before or after off[c]
// (off sorted ascending); flag[n, 2n): chained, or not covered by a chained
// candidate in the block window before it -- the walk's likely strong-sum
// needs.  flag holds 2n bytes.
hipError_t launch_rs_chained(const uint64_t *off, uint64_t n, uint64_t blength, uint8_t *flag,
                             hipStream_t s);
// ---- device-resident greedy walk (rsync_walk.hip, XXH3, blength > 240) -----
// Offsets are data-relative.  The owned range [lo, hi) is cut into segments
// of seg_len; each wave walks one segment (spec kernel: from its own start;
// stitch kernel: from the previous segment's exit, merging into the spec).
struct RsWalkArgs {
    const uint8_t *data;   // source bytes, 16-byte aligned
    uint64_t dlen;
    int64_t full_end;      // offsets below it have a full window (F - blength + 1)
    int64_t lo, hi;        // the owned range
    int64_t seg_len;
    int64_t seg_len2;      // segments nseg1.. (the tail): this long
    int64_t segb;          // segment k >= 1 starts at segb + k seg_len (k <= nseg1); segment 0 at lo
    uint32_t nseg1;
    uint32_t nseg, cap;    // segments, match capacity per segment
    uint32_t blength, count, remainder;
    int csum_type;
    uint64_t seed;
    uint64_t s2mask_lo, s2mask_hi;   // the first s2length bytes of (lo64, hi64)
    const uint64_t *sum2p;           // [count][2] zero-padded strong sums
    const uint32_t *sum1;            // [count]
    const uint64_t *tkey;            // sorted (sum1 << 32 | ~index)
    const uint32_t *dir;
    const uint32_t *filt, *filt_l;
    const uint64_t *filt_b;          // blocked filter (rs_bloom_word / rs_bloom_mask)
    const uint32_t *bkt;             // membership buckets (rs_bucket): 32 B, a count + 7 sums
    uint32_t bbits;
    uint32_t dbits, fbits, lbits;
    int64_t e0;                      // segment 0's entry (offset, want_i)
    int32_t w0;
    int32_t spec_w0;                 // want_i of segment 0's speculative walk
    uint32_t *work;                  // segment work counter
    uint32_t *flags;                 // 1: an exit changed, 2: capacity overflow
    // speculative walks [nseg * cap] / [nseg]
    int64_t *spec_off;
    int32_t *spec_idx;
    int64_t *spec_fab;               // false alarms before the match's offset
    uint32_t *spec_n;
    uint64_t *spec_fa;
    int64_t *spec_exit;
    int32_t *spec_exitw;
    // the speculative walk's false-alarm windows (offset, running total after
    // the window), up to facap per segment; spec_nfa[k] > facap: overflowed.
    // A stitch whose entry the speculative walk visited merges there.
    int64_t *spec_fao;
    uint32_t *spec_fac;
    uint32_t *spec_nfa;
    uint32_t facap;
    // final walks: fin_off[0, fin_n) then spec[fin_from, spec_n) (fin_from
    // 0xffffffff: the final walk is the speculative one)
    int64_t *fin_entry;
    int32_t *fin_entryw;
    uint32_t *fin_from, *fin_n;
    uint64_t *fin_fa;
    int64_t *fin_off;
    int32_t *fin_idx;
    int64_t *fin_fab;
    // exits of the current final walks, double-buffered across stitch passes
    const int64_t *exit_old;
    const int32_t *exitw_old;
    int64_t *exit_new;
    int32_t *exitw_new;
    uint32_t flushq;                 // STEP hits queued per flush: 4 (rows) or 16 (wide)
    uint32_t flushspan;              // flush once the scan ran this far past the first hit (0: no bound)
    uint32_t flushpredict;           // flush at a hit whose weak sum is block want .. want + 2's
    uint64_t *dbg;                   // debug builds: per-wave progress records (host-mapped)
    uint64_t *prof;                  // VS_WALK_PROF builds: per-wave phase cycles/counts [waves][16]
};
int rs_walk_waves_per_cu();   // the device walk's resident waves per CU (one workgroup)
hipError_t launch_rs_walk(const RsWalkArgs &a, bool stitch, int cus, hipStream_t s);
// fill the membership buckets (zeroed by the caller) from the sorted keys:
// each distinct sum1 of a full-length block once (the short final block,
// index count-1 when remainder != 0, is left out)
hipError_t launch_rs_buckets(const uint64_t *tkey, uint32_t count, uint32_t remainder,
                             uint32_t bbits, uint32_t *bkt, hipStream_t s);
// the final walks' match list in order as 16-byte vs_match records (offset,
// block index, 0): cnt [nseg], pos [nseg + 1] (pos[nseg] = length),
// partials >= nseg / 4096 + 2, out >= nseg * cap records; *fa_total = the
// false alarms of the final walks
hipError_t launch_rs_collect(const RsWalkArgs &a, uint32_t *cnt, uint32_t *pos, uint32_t *partials,
                             uint4 *out, unsigned long long *fa_total, hipStream_t s);
hipError_t launch_rs_pad_sum2(const uint8_t *sum2, uint32_t count, uint32_t s2length,
                              uint64_t *out, hipStream_t s, const uint32_t *sum1_in = nullptr,
                              uint32_t *sum1_out = nullptr);
// whole-file checksum (filesum.hip + filesum_host.cpp):
// contributions of nb whole 1 KiB blocks -> C[nb][8] (block-major)
hipError_t launch_fs_contrib(const uint8_t *p, uint64_t nb, uint64_t *C, hipStream_t s);


// restic Key.Seal (crypto.hip)
struct SealArgs {
    const uint8_t *in;
    uint8_t *out;               // ciphertext at the same offsets
    const uint64_t *off;
    const uint32_t *len;
    uint64_t n;
    const uint8_t *nonces;      // [n][16]
    const uint64_t *prefix;     // [n + 1] exclusive prefix of 16-byte blocks per blob
    uint64_t total_blocks;
    const uint32_t *te0;        // [256] AES T-table (LE column words)
    const uint32_t *rk256;      // [60] AES-256 round keys (EncryptionKey)
    const uint32_t *rk128;      // [44] AES-128 round keys (MACKey.K)
    const uint32_t *rpow;       // [64][5] r^1..r^64 in 26-bit limbs (MACKey.R clamped)
    const uint32_t *rsq;        // [kSealSq][5] r^(64 * 2^j) (the fused MAC's long lifts)
    unsigned long long *acc;    // [n][5] fused MAC: per-blob limb sums of the lifted partials
    uint8_t *macs;              // [n][16] (kOpen: the expected tags)
    // where blob i's output bytes go (nullptr: off[i], i.e. in place /
    // same layout); kSealRecords writes nonce || ciphertext || mac around it
    const uint64_t *out_off;
    int mode;                   // kSealMacs, kSealRecords, kOpen
    bool fused;                 // kSealMacs: the MAC inside the CTR pass (else two kernels)
    uint32_t *bad;              // kOpen: [n] 1 where the stored tag does not match
    unsigned long long *n_bad;  // kOpen: their count
};
enum { kSealMacs = 0, kSealRecords = 1, kOpen = 2 };
constexpr int kSealSq = 24;     // r^(64 * 2^j), j < 24: lifts up to 2^30 blocks (16 GiB blobs)
hipError_t launch_seal_prefix(const uint32_t *len, uint64_t n, uint64_t *prefix, uint64_t *total,
                              hipStream_t s);
hipError_t launch_seal(const SealArgs &a, int cus, hipStream_t s, hipEvent_t *ev);
// kOpen inputs from stored records (nonce || ciphertext || mac at rec_off):
// nonces / tags gathered into 16-byte rows, ct_off = rec_off + 16
hipError_t launch_open_gather(const uint8_t *in, const uint64_t *rec_off, const uint32_t *len,
                              uint64_t n, uint8_t *nonces, uint8_t *macs, uint64_t *ct_off,
                              hipStream_t s);
// the 4-byte LE trailers of packs: out[pos[i]..+4) = val[i]
hipError_t launch_put_u32(uint8_t *out, const uint64_t *pos, const uint32_t *val, uint64_t n,
                          hipStream_t s);
// adjacent-mover kernels (movers.hip)
struct ReconPiece {
    uint64_t dst, src, len;
    uint32_t kind;   // 0: basis bytes, 1: literal bytes
    uint32_t pad;
};
hipError_t launch_blk_desc(uint64_t len, uint32_t bs, uint64_t n, uint64_t *off, uint32_t *lens,
                           hipStream_t s);
hipError_t launch_verify(const uint8_t *got, const uint8_t *want, uint64_t n, uint32_t *bad,
                         unsigned long long *count, hipStream_t s);
hipError_t launch_recon(uint8_t *dst, const uint8_t *basis, const uint8_t *lit,
                        const ReconPiece *pieces, uint64_t n, int cus, hipStream_t s);
// SaveBlob dedup (dedup.hip): first[i] = smallest index with ids[i]'s ID
size_t dedup_tmp_bytes(uint64_t n);
// vs_blob_dedup with the repository's index: first[i] = kDedupKnown for a
// blob whose ID the (vs_blob_index_sort-ed) known array holds
constexpr uint32_t kDedupKnown = 0xffffffffu;
size_t dedup_known_tmp_bytes(uint64_t n);
hipError_t launch_dedup_known(const uint8_t *ids, uint64_t n, const uint8_t *known,
                              uint64_t n_known, uint32_t *first, void *flag_tmp,
                              unsigned long long *n_new_dev, hipStream_t s);
size_t index_sort_tmp_bytes(uint64_t n);
hipError_t launch_index_sort(uint8_t *ids, uint64_t n, void *tmp, size_t tmp_bytes, hipStream_t s);
hipError_t launch_dedup(const uint8_t *ids, uint64_t n, uint32_t *first, void *tmp,
                        size_t tmp_bytes, unsigned long long *n_unique_dev, hipStream_t s);
hipError_t launch_rs_sort_cands(void *tmp, size_t tmp_bytes, const uint64_t *off_in,
                                uint64_t *off_out, const uint32_t *sum_in, uint32_t *sum_out,
                                uint64_t n, int end_bit, hipStream_t s);

}  // namespace vsgpu
