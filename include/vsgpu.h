/*
 * vsgpu.h -- C ABI of the MI355X data-movement hot path behind VolSync's
 * restic and rsync movers: content-defined chunking (restic chunker, Rabin
 * fingerprint over a 64-byte window) plus SHA-256 blob IDs, and rsync's
 * rolling weak checksum + strong-sum block matching, as hand-written gfx950
 * HIP kernels.
 *
 * The reference binds this path in Go.  The restic mover image
 * (/root/reference/mover-restic/Dockerfile:8-27) builds restic v0.13.1, whose
 * archiver calls github.com/restic/chunker@v0.4.0 and crypto/sha256 (patched
 * in by mover-restic/patch-sources.sh:16-27); restic runs from
 * mover-restic/entry.sh:60-65 ("restic backup").  The rsync mover image
 * (mover-rsync/Dockerfile:11-12) installs rsync 3.2.3, run by
 * mover-rsync/source.sh:54 (rsync -aAhHSxz --delete ...); its sender's
 * match.c/checksum.c/generator.c functions are the vs_rsync_* entry points.
 * Each entry point below names the upstream interface it replaces;
 * INTEGRATION.md shows the cgo binding.
 *
 * Conventions:
 *  - return 0 on success, a negative VS_ERR_* on failure, VS_EOF (1) when a
 *    chunk stream is exhausted; vs_last_error() gives a thread-local message;
 *  - the caller owns every buffer it passes; host buffers are copied before
 *    the call returns and never retained (cgo pointer rules);
 *  - a handle is single-threaded; different handles may run concurrently;
 *    each call makes the handle's device current (cgo calls hop OS threads);
 *  - there is no CPU fallback: without a usable gfx950 device every compute
 *    entry point fails with VS_ERR_NO_DEVICE.
 */
#ifndef VSGPU_H
#define VSGPU_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define VS_OK 0
#define VS_EOF 1
#define VS_ERR_ARG (-1)       /* bad argument */
#define VS_ERR_POLY (-2)      /* polynomial 0 ("tables ... not initialized") or degree > 53 */
#define VS_ERR_NO_DEVICE (-3) /* no HIP device / HIP runtime error */
#define VS_ERR_NOMEM (-4)     /* device or host allocation failed */
#define VS_ERR_STATE (-5)     /* call out of sequence */
#define VS_ERR_HIP (-6)       /* a HIP call or kernel launch failed */

#define VS_DEFAULT_POL 0x3DA3358B4DC173ull /* chunker_test.go testPol */
#define VS_MIN_SIZE (512u * 1024u)         /* chunker.go MinSize */
#define VS_MAX_SIZE (8u * 1024u * 1024u)   /* chunker.go MaxSize */
#define VS_AVG_BITS 20u                    /* splitmask = 2^20 - 1 */

/* One chunk: chunker.go `type Chunk struct { Start, Length uint; Cut uint64; Data []byte }`
 * plus restic's blob ID (internal/restic/id.go Hash = sha256.Sum256(Data)).
 * Data is not carried: it is data[start : start+length] of the caller's stream. */
typedef struct vs_chunk {
    uint64_t start;
    uint64_t length;
    uint64_t cut;
    uint8_t id[32];
} vs_chunk;

typedef struct vs_cdc vs_cdc;

/* ---- library / device ------------------------------------------------ */
const char *vs_last_error(void);
const char *vs_version(void);
/* number of usable gfx9xx devices (0 when none; never initialises a context) */
int vs_device_count(void);

/* ---- polynomial helpers (chunker polynomials.go) ---------------------- */
/* Pol.Deg */
int vs_pol_deg(uint64_t pol);
/* Pol.Irreducible (Ben-Or), 1 = irreducible */
int vs_pol_irreducible(uint64_t pol);
/* fillTables: out[b] = Hash(b || 63 zero bytes), mod[b] = (b x^k mod P) | (b << k) */
int vs_pol_tables(uint64_t pol, uint64_t out_tab[256], uint64_t mod_tab[256]);

/* ---- restic chunker stream (replaces chunker.New / NewWithBoundaries /
 *      Reset / SetAverageBits / Next + restic.Hash in FileSaver.saveFile) -- */
/* chunker.NewWithBoundaries(rd, pol, min, max) + SetAverageBits(avg_bits) */
int vs_cdc_open(int device, uint64_t pol, uint32_t min_size, uint32_t max_size,
                uint32_t avg_bits, vs_cdc **h);
/* Chunker.Reset / ResetWithBoundaries: new stream, same device buffers */
int vs_cdc_reset(vs_cdc *h, uint64_t pol, uint32_t min_size, uint32_t max_size,
                 uint32_t avg_bits);
/* Append n host bytes of the stream (the io.Reader's output); final = 1 at EOF.
 * Work is batched: chunks become available once their cut is determined. */
int vs_cdc_feed(vs_cdc *h, const void *buf, size_t n, int final);
/* Chunker.Next: copy up to cap ready chunks (with blob IDs) into out.
 * Returns VS_OK with *n_out > 0, VS_OK with *n_out == 0 when more input is
 * needed, or VS_EOF once the final chunk has been returned (io.EOF). */
int vs_cdc_next(vs_cdc *h, vs_chunk *out, size_t cap, size_t *n_out);
/* vs_cdc_next for a caller that bounds the stream bytes it holds: with no
 * chunk ready it waits for the oldest batch in flight (its blob IDs) instead
 * of returning *n_out == 0; *n_out == 0 then means no batch is in flight and
 * the stream needs more input.  Same chunks, same order as vs_cdc_next. */
int vs_cdc_next_wait(vs_cdc *h, vs_chunk *out, size_t cap, size_t *n_out);
/* batches whose cuts are selected and whose blob IDs are pending */
int vs_cdc_inflight(vs_cdc *h, uint64_t *batches);
void vs_cdc_close(vs_cdc *h);
/* Streaming pipeline: fed bytes are copied to the device on a
 * copy stream (pinned caller memory by DMA, waited for before the call
 * returns; pageable memory through two pinned 64 MiB staging buffers) and
 * chunked in batches of batch_bytes (default 512 MiB); up to 32 batches are
 * in flight while their blob IDs are computed, and vs_cdc_next returns chunks
 * in stream order as soon as theirs are final (after the final feed it waits
 * for them).  The batch size can only change between streams. */
int vs_cdc_set_batch_bytes(vs_cdc *h, uint64_t bytes);
/* Streaming counters: [0] bytes fed from pinned memory, [1] bytes fed through
 * the staging buffers, [2] times a call waited for a batch's IDs, [3] batches;
 * host milliseconds spent [4] waiting for H2D copies, [5] running batches
 * (fingerprint, cut selection, hash queueing), [6] collecting chunks, [7]
 * copying pageable input into the staging buffers. */
int vs_cdc_stream_stats(vs_cdc *h, double out[8]);

/* ---- device-resident batch API (data already in HBM) ------------------
 * Chunks a device byte range that begins at a chunk boundary.  dev_data
 * points at stream offset `origin`; own_lo/own_hi are stream offsets (the
 * byte range this call owns); data must cover [own_lo - 63, own_hi + max - 1)
 * clipped to the stream, and final = 1 when origin + len is the stream end.
 * Multi-GPU: each rank scans its own byte range, exchanges the exit offset of
 * its last chunk (vs_cdc_stitch) and finishes; see DESIGN.md section 6. */
/* Ordering: with the handle's own stream (default) a scan waits for work
 * already queued on the null stream; with vs_cdc_set_stream the caller's
 * stream must already order the producer of dev_data before the scan. */
int vs_cdc_set_stream(vs_cdc *h, void *hip_stream); /* NULL = handle's own stream */
/* Stream of the SHA-256 stage.  NULL (default) = the handle's own hash
 * stream, so batch k+1's fingerprint pass runs beside batch k's hashing. */
int vs_cdc_set_hash_stream(vs_cdc *h, void *hip_stream);
/* Time slicing of the SHA-256 engine: each vs_cdc_finish
 * advances every queued chunk by at most `blocks` 64-byte blocks and carries
 * the midstate of unfinished chunks to the next batch's launch; vs_cdc_wait
 * hashes the rest.  0 = unbounded (every batch hashed to the end in one
 * launch).  Default 512 (32 KiB per chunk per batch). */
int vs_cdc_set_hash_slice(vs_cdc *h, uint32_t blocks);
/* Throughput mode of the SHA-256 engine: once at least
 * min_chains chunks are being hashed, each wavefront hashes 64 chunks whole
 * instead of the producer/consumer split, and a drain advances them by
 * drain_blocks per launch until fewer than min_chains remain.  Results are
 * identical in both modes.  min_chains 0 = the handle's default (never for
 * vs_cdc, whose long chunks make the tail; 384 per CU for vs_sha), 0xffffffff
 * = never; drain_blocks 0 = default (4096). */
int vs_cdc_set_hash_wide(vs_cdc *h, uint32_t min_chains, uint32_t drain_blocks);
/* Pipelined batches: batch numbers count vs_cdc_finish calls from 0; the ring
 * keeps the last *ring batches' chunk lists.  Data passed to vs_cdc_scan must
 * stay valid until its batch's blob IDs are final (vs_cdc_wait). */
int vs_cdc_batches(vs_cdc *h, uint64_t *finished, uint64_t *ring);
int vs_cdc_get_batch_chunks(vs_cdc *h, uint64_t batch, uint64_t first, uint64_t n,
                            vs_chunk *out);
int vs_cdc_scan(vs_cdc *h, const void *dev_data, uint64_t len, uint64_t origin,
                uint64_t own_lo, uint64_t own_hi, int final);
/* Selects cuts given the true start of the first chunk (entry).  *exit_pos =
 * start of the first chunk at or beyond own_hi (or the stream end);
 * *complete = 0 when a chunk's cut depends on bytes not yet supplied. */
int vs_cdc_stitch(vs_cdc *h, uint64_t entry, uint64_t *exit_pos, int *complete);
/* Emits the chunk list (the count is known on return), queues the Cut values
 * and hands the chunks to the SHA-256 engine without waiting for their IDs. */
int vs_cdc_finish(vs_cdc *h, uint64_t *n_chunks);
/* Hashes every queued chunk to the end and waits until all blob IDs of all
 * finished batches are final. */
int vs_cdc_wait(vs_cdc *h);
/* scan + stitch(own_lo) + finish for a single device (own range = whole buffer). */
int vs_cdc_process(vs_cdc *h, const void *dev_data, uint64_t len, uint64_t origin, int final,
                   uint64_t *n_chunks, uint64_t *consumed);
/* Copy chunks [first, first+n) of the last finish() to host (waits). */
int vs_cdc_get_chunks(vs_cdc *h, uint64_t first, uint64_t n, vs_chunk *out);
/* Accumulated device time (ms) per pipeline stage since the last reset of the
 * timers, measured with HIP events on the handle's stream when enabled.
 * stage: 0 fingerprint, 1 select, 2 sha256 (the hash kernels alone; their
 * histogram / scan / scatter bookkeeping launches are not timed), 3 other. */
int vs_cdc_timing(vs_cdc *h, int enable, double ms_out[4], uint64_t launches_out[4]);
/* Order the handle's next scan (on its stream) after the blob IDs of finished
 * batch `batch` (0 = the first vs_cdc_finish of the handle) are final, as a
 * producer about to overwrite that batch's bytes needs; when the batch's
 * chunks are still queued beyond the slices already launched, the engine
 * drains (every queued chunk is hashed to its end).  Does not block the host
 * beyond that drain's set-up. */
int vs_cdc_fence(vs_cdc *h, uint64_t batch);
/* The SHA-256 kernel windows of the interval the last vs_cdc_timing call
 * closed, against the fingerprint windows (HIP events on both streams, as ms
 * after an anchor event recorded when timing was enabled): out[0] SHA-256
 * kernel time, out[1] the part outside every fingerprint window, out[2] the
 * part inside one, out[3] the fingerprint windows' union.  *quad_chains: the
 * chains the final drains ran in latency (quad) mode since the last call. */
int vs_cdc_timing_detail(vs_cdc *h, double out[4], uint64_t *quad_chains);

/* ---- batched SHA-256 (restic.Hash over many blobs; C5 small files) ----
 * A vs_sha handle owns the scratch of the work-queue kernel.  run_device:
 * dev_buf device bytes; dev_off/dev_len device arrays of n entries; dev_out a
 * device array of n*32 bytes.  Blob i = dev_buf[off[i] : off[i]+len[i]].
 * Asynchronous on hip_stream (NULL = default stream); one run in flight per
 * handle. */
typedef struct vs_sha vs_sha;
int vs_sha256_open(int device, vs_sha **h);
int vs_sha256_run_device(vs_sha *h, const void *dev_buf, const uint64_t *dev_off,
                         const uint32_t *dev_len, size_t n, uint8_t *dev_out, void *hip_stream);
/* The last drain of vs_sha256_run_device: out[0] = chains it ran in latency
 * mode (4 lanes per chain), out[1] = those of them in isolated tiles (a CU
 * each); the rest ran as latency tiles beside the split tiles.  Diagnostics
 * for tests and benches; the digests never depend on the split. */
int vs_sha256_drain_stats(vs_sha *h, uint64_t out[2]);
/* Same knob as vs_cdc_set_hash_wide for a vs_sha handle. */
int vs_sha256_set_wide(vs_sha *h, uint32_t min_chains, uint32_t drain_blocks);
void vs_sha256_close(vs_sha *h);
/* The SaveBlob dedup seam (restic Repository.SaveBlob: idx.Has / AddPending):
 * for n 32-byte blob IDs in stream order (device array dev_ids), dev_first[i]
 * = the smallest index whose ID equals ID i (i itself for the first, stored
 * blob; any other value marks a duplicate), and *n_unique (optional; waits
 * for the result) = the number of distinct IDs.  Queued on hip_stream (NULL =
 * default stream); scratch lives in the vs_sha handle. */
int vs_blob_dedup(vs_sha *h, const uint8_t *dev_ids, size_t n, uint32_t *dev_first,
                  uint64_t *n_unique, void *hip_stream);
/* The same against the repository's index as well (restic v0.13.1
 * Repository.SaveBlob: known = !idx.AddPending(BlobHandle{id, t}) -- a blob
 * the master index already holds is not stored again; a scheduled backup
 * re-runs `restic backup` into an initialised repository,
 * /root/reference/mover-restic/entry.sh:43-65, so most IDs are known):
 * dev_known holds n_known 32-byte IDs of one blob type, prepared once per
 * backup by vs_blob_index_sort.  dev_first[i] = VS_DEDUP_KNOWN when ID i is
 * in the index, else as vs_blob_dedup; *n_new (optional; waits) = the
 * distinct IDs the index does not hold, i.e. the blobs SaveBlob stores. */
#define VS_DEDUP_KNOWN 0xffffffffu
int vs_blob_dedup_known(vs_sha *h, const uint8_t *dev_ids, size_t n, const uint8_t *dev_known,
                        size_t n_known, uint32_t *dev_first, uint64_t *n_new, void *hip_stream);
/* Sorts n device-resident 32-byte IDs in place into the order
 * vs_blob_dedup_known searches (by the first 8 bytes, big-endian).  Queued on
 * hip_stream; scratch lives in the handle. */
int vs_blob_index_sort(vs_sha *h, uint8_t *dev_known, size_t n, void *hip_stream);
/* syncthing's scanner (lib/scanner; SURVEY.md 8(f)4, mover-syncthing/entry.sh:
 * 130-135): SHA-256 of every block_size block of a device buffer of len bytes
 * (the last block short), n = ceil(len / block_size) digests into dev_out.
 * Queued on hip_stream like vs_sha256_run_device. */
int vs_sha256_blocks(vs_sha *h, const void *dev_buf, uint64_t len, uint32_t block_size,
                     uint8_t *dev_out, void *hip_stream);
/* syncthing lib/protocol BlockSize: the smallest power of two from 128 KiB to
 * 16 MiB that keeps a file of file_size bytes under 2000 blocks (else 16 MiB). */
int vs_syncthing_block_size(int64_t file_size);
/* Restore-side check (restic Repository.LoadBlob, mover-restic/entry.sh:
 * 215-228): hash n device blobs and compare with their expected IDs
 * (dev_want, n*32 bytes); dev_bad[i] (optional) = 1 on mismatch, *n_bad
 * (optional; waits) = the mismatches. */
int vs_blob_verify(vs_sha *h, const void *dev_buf, const uint64_t *dev_off,
                   const uint32_t *dev_len, size_t n, const uint8_t *dev_want,
                   uint32_t *dev_bad, uint64_t *n_bad, void *hip_stream);
/* Host-memory convenience form (copies in and out). */
int vs_sha256_batch(int device, const void *buf, size_t buf_len, const uint64_t *off,
                    const uint32_t *len, size_t n, uint8_t (*out)[32]);

/* ---- rsync delta matching (rsync 3.2.3) -----
 * csum_type: the negotiated xfersum (checksum.c): VS_CSUM_MD5 (seed
 * prepended as LE u32 when non-zero), VS_CSUM_XXH64, VS_CSUM_XXH3_64,
 * VS_CSUM_XXH3_128 (the 3.2.3 <-> 3.2.3 default).  seed = checksum_seed. */
#define VS_CSUM_MD5 5
#define VS_CSUM_XXH64 6
#define VS_CSUM_XXH3_64 7
#define VS_CSUM_XXH3_128 8

/* One match: match.c matched(offset, i) -- source bytes [offset, offset +
 * len_i) equal destination block i; literals are the gaps between matches. */
typedef struct vs_match {
    int64_t offset;
    int32_t block_index;
    int32_t reserved;
} vs_match;

/* Replaces generator.c sum_sizes_sqroot (protocol >= 30): block length,
 * strong-sum bytes sent, block count and last-block remainder for a
 * destination of len bytes; block_size != 0 is --block-size. */
int vs_rsync_sizes(int64_t len, int32_t block_size, int32_t *blength, int32_t *s2length,
                   int32_t *count, int32_t *remainder);

typedef struct vs_rsync vs_rsync;
int vs_rsync_open(int device, vs_rsync **h);
/* Ordering: with the handle's own stream (default) every call that reads or
 * writes caller device memory first waits for work already queued on the null
 * stream (e.g. the fill of dev_sum1 or the kernel that wrote the source); with
 * vs_rsync_set_stream the caller's stream must already order those producers
 * before the call. */
int vs_rsync_set_stream(vs_rsync *h, void *hip_stream); /* NULL = handle's own stream */
void vs_rsync_close(vs_rsync *h);
/* Replaces generator.c generate_and_send_sums (get_checksum1 + get_checksum2
 * per block): signatures of a device-resident destination file.  dev_sum1
 * [count] u32 and dev_sum2 [count * s2length] bytes are device arrays.
 * Returns after queueing on the handle's stream. */
int vs_rsync_signatures_device(vs_rsync *h, const void *dev_basis, int64_t len, int32_t blength,
                               int32_t s2length, int csum_type, uint32_t seed,
                               uint32_t *dev_sum1, uint8_t *dev_sum2);
/* Replaces match.c build_hash_table: load the signature table the sender
 * received (read_sum_head + per-block sum1/sum2).  Host arrays (copied) or,
 * in the _device form, device arrays. */
int vs_rsync_load_sums(vs_rsync *h, int32_t count, int32_t blength, int32_t s2length,
                       int32_t remainder, const uint32_t *sum1, const uint8_t *sum2,
                       int csum_type, uint32_t seed);
int vs_rsync_load_sums_device(vs_rsync *h, int32_t count, int32_t blength, int32_t s2length,
                              int32_t remainder, const uint32_t *dev_sum1,
                              const uint8_t *dev_sum2, int csum_type, uint32_t seed);
/* Replaces match.c match_sums -> hash_search: the greedy match list of a
 * device-resident source against the loaded table (identical to rsync's,
 * including chain order, the want_i preference and false-alarm handling).
 * Blocks until done; *n_matches = number of matches. */
int vs_rsync_match_device(vs_rsync *h, const void *dev_src, int64_t len, int64_t *n_matches);
/* Sharded match_sums: one hash_search over a source file of
 * file_len bytes, split by byte range across devices/handles.  This handle
 * owns the walk's visits to offsets [own_lo, own_hi); dev_src points at file
 * offset `origin` (<= own_lo) and holds len bytes covering
 * [own_lo, min(own_hi + blength - 1, file_len)).  match_scan finds the
 * candidates and walks the range speculatively from own_lo (want_i 0 when
 * own_lo == 0, as hash_search starts; otherwise "no preference"), returning
 * that walk's exit state: the first offset >= own_hi it would visit, and
 * want_i there.  match_stitch re-walks from the true entry (the previous
 * range's exit) until it rejoins the speculative walk and returns the new
 * exit; it may be called again with another entry.  match_finish makes the
 * walk from the last entry given (the speculative one if none) the result:
 * matches with offsets in [entry, own_hi), file offsets, in order.  The
 * ranges' results concatenated equal one vs_rsync_match_device over the
 * whole file, false-alarm counts included (vs_rsync_stats). */
int vs_rsync_match_scan(vs_rsync *h, const void *dev_src, int64_t len, int64_t origin,
                        int64_t file_len, int64_t own_lo, int64_t own_hi, int64_t *exit_off,
                        int32_t *exit_want);
int vs_rsync_match_stitch(vs_rsync *h, int64_t entry, int32_t want_i, int64_t *exit_off,
                          int32_t *exit_want);
int vs_rsync_match_finish(vs_rsync *h, int64_t *n_matches);
/* Copy matches [first, first+n) of the last match run to host. */
int vs_rsync_get_matches(vs_rsync *h, int64_t first, int64_t n, vs_match *out);
/* Counters of the last match run: weak candidates found by the scan,
 * false alarms (strong mismatches the walk visited, rsync's stats), windows
 * strong-hashed on the device, walk rounds. */
int vs_rsync_stats(vs_rsync *h, int64_t *candidates, int64_t *false_alarms,
                   int64_t *strong_hashed, int32_t *rounds);
/* Device time (ms) of the last run's stages: 0 signatures, 1 table, 2 scan
 * (prefix + weak scan + sort), 3 strong verification, 4 host walk. */
int vs_rsync_timing(vs_rsync *h, double ms_out[5]);
/* Replaces checksum.c sum_init / sum_update / sum_end over one file (match.c
 * matched() streams every source byte into it; rsync 3.2.3 seeds none of the
 * xxhash / MD5 file sums): the whole-file checksum of a device-resident file,
 * as sum_end writes it -- xxh128: LE low64 then LE high64; xxh3 / xxh64: LE
 * 64-bit value (out[8..15] zeroed); md5: the digest.  XXH3 runs as parallel
 * block contributions on the device plus one serial scramble chain on a host
 * thread (for files up to 128 GiB the contribution rows,
 * len / 16 bytes, are held on the device and in pinned host memory); MD5 and
 * XXH64 -- serial chains with no parallel form -- are hashed on a library host
 * thread from the file's bytes read back through a pinned ring.  Any length.  Blocks until done.  It runs on
 * a job of its own: jobs other calls left in flight stay in flight, keep their
 * _wait order and do not limit it (nor does it count toward their 4). */
int vs_rsync_file_sum(vs_rsync *h, const void *dev_src, int64_t len, int csum_type,
                      uint8_t out[16]);
/* The same, asynchronous: _start queues the device part (after work queued on
 * the null stream and on the handle's stream) and returns; the host chain
 * runs on a library thread while the caller goes on (e.g. with the match walk
 * over the same file).  dev_src must stay valid and unchanged until its _wait.
 * Up to 4 jobs (whole files or block ranges) may be in flight per handle,
 * each with its own host thread and (XXH3 only) 3 pieces of device memory
 * for its contribution rows: _wait returns
 * the OLDEST job's digest (jobs complete in start order; the _blocks_ form
 * shares the queue). */
int vs_rsync_file_sum_start(vs_rsync *h, const void *dev_src, int64_t len, int csum_type);
int vs_rsync_file_sum_wait(vs_rsync *h, uint8_t out[16]);
/* A file split by byte range across ranks: the XXH3 state is a
 * relay.  _blocks_start chains the nblocks whole 1 KiB blocks at dev_blocks
 * (file offset a multiple of 1024) from acc_in (NULL: the initial state,
 * vs_rsync_file_sum_init); _blocks_wait returns the state after them, which
 * the next range's owner takes as its acc_in.  The ranks together must chain
 * exactly the file's first (len - 1) / 1024 whole blocks: the block holding
 * byte len - 1 is always the finish's partial block, even when len % 1024 ==
 * 0.  The owner of the file's last byte finishes with
 * vs_rsync_file_sum_finish over the file's last min(len, 1088) bytes (host
 * memory).  XXH3 only (xxh128 and xxh3 share the state; len > 240). */
int vs_rsync_file_sum_init(uint64_t acc[8]);
int vs_rsync_file_sum_blocks_start(vs_rsync *h, const void *dev_blocks, int64_t nblocks,
                                   const uint64_t acc_in[8]);
int vs_rsync_file_sum_blocks_wait(vs_rsync *h, uint64_t acc_out[8]);
int vs_rsync_file_sum_finish(const uint64_t acc[8], const uint8_t *last, int64_t len,
                             int csum_type, uint8_t out[16]);
/* The last file-sum job's device time (the contribution kernel, ms) and host
 * time (the scramble chain, ms). */
int vs_rsync_file_sum_timing(vs_rsync *h, double *device_ms, double *host_ms);
/* Replaces receiver.c receive_data: rebuild the new file
 * (out_len bytes, device dev_out) from the basis (device, basis_len bytes,
 * blocks of blength) and the token stream -- the match list (host array, in
 * order: block i copied to offset) and the literal bytes of the gaps between
 * matches, concatenated in order (device, literal_len bytes).  Blocks until
 * done; vs_rsync_file_sum over dev_out then checks it as receive_data does. */
int vs_rsync_reconstruct(vs_rsync *h, void *dev_out, int64_t out_len, const void *dev_basis,
                         int64_t basis_len, int32_t blength, const vs_match *matches,
                         int64_t n_matches, const void *dev_literals, int64_t literal_len);
/* Device time of one kernel class summed over its launches since the handle
 * was opened (or the last reset), from HIP events on the handle's stream:
 * which 0 = weak scan / speculative device walk, 1 = strong-sum verification,
 * 2 = signatures, 3 = device walk stitch passes, 4 = whole-file checksum.
 * reset != 0 zeroes the totals after reading them. */
int vs_rsync_kernel_time(vs_rsync *h, int which, int reset, double *ms, int64_t *launches);

/* ---- streamed forms: a file fed from host memory in order ---------------
 * rsync reads files through map_ptr (fileio.c), a sliding window with an
 * int32 length, never the whole file at once.  These entry points take the
 * file the same way -- any number of feeds of any size, in file order -- and
 * keep only a ring of `ring` pieces of `piece_bytes` on the device (0, 0 =
 * 256 MiB x 3), so files far larger than HBM pass.  Fed bytes are copied
 * before feed returns (pinned caller memory by DMA, pageable memory through
 * the library's staging buffers).  A handle runs one stream of each kind at
 * a time; while a match stream runs, call only its _feed / _next / _end on
 * the handle (its walk thread uses the handle's table and buffers).
 *
 * Replaces match.c match_sums -> hash_search over a file of file_len bytes
 * (the table from vs_rsync_load_sums[_device]).  Each piece is walked by a
 * library thread from the previous piece's exit state as soon as its bytes
 * and a blength - 1 halo are on the device, while the caller feeds the next
 * ones.  The match list is exactly vs_rsync_match_device's over the whole
 * file, false alarms included.
 * _next: matches found so far, in file order (*n_out may be 0 before the
 * last feed; after it, _next waits for the walk); VS_EOF once every match has
 * been returned.  _end waits for the walk and gives the totals (the match
 * list then also stays readable through vs_rsync_get_matches). */
/* file_csum (0 = none): the negotiated xfersum whose whole-file checksum
 * (R7: sum_update over every byte, which matched() does in match.c) the
 * stream also computes as the file passes -- XXH3 from each piece's block
 * contributions on the device, chained by the walk thread; MD5 / XXH64 on the
 * caller's thread from the fed bytes -- returned by _end in file_sum (as
 * vs_rsync_file_sum writes it; NULL: not wanted).  piece_bytes: a multiple of
 * 1024, >= 1 MiB. */
int vs_rsync_match_begin(vs_rsync *h, int64_t file_len, int file_csum, uint64_t piece_bytes,
                         uint32_t ring);
int vs_rsync_match_feed(vs_rsync *h, const void *buf, size_t n);
int vs_rsync_match_next(vs_rsync *h, vs_match *out, size_t cap, size_t *n_out);
int vs_rsync_match_end(vs_rsync *h, int64_t *n_matches, int64_t *false_alarms,
                       uint8_t file_sum[16]);
/* [0] bytes fed from pinned memory, [1] bytes staged, [2] caller ms waiting
 * for a free piece slot, [3] walk-thread ms walking, [4] walk-thread ms
 * waiting for bytes, [5] pieces walked, [6] piece bytes, [7] ring, [8]
 * walk-thread ms on the XXH3 file checksum, [9] file_csum */
int vs_rsync_match_stream_stats(vs_rsync *h, double out[10]);
/* Replaces generator.c generate_and_send_sums over a basis file of len bytes
 * read in order: pieces of whole blocks are signed as they arrive; _next
 * returns the sums of finished blocks in block order (sum1 [n] u32, sum2
 * [n * s2length]), waiting for the oldest piece in flight when none is
 * ready; VS_EOF after the last block. */
int vs_rsync_sig_begin(vs_rsync *h, int64_t len, int32_t blength, int32_t s2length,
                       int csum_type, uint32_t seed, uint64_t piece_bytes, uint32_t ring);
int vs_rsync_sig_feed(vs_rsync *h, const void *buf, size_t n);
int vs_rsync_sig_next(vs_rsync *h, uint32_t *sum1, uint8_t *sum2, size_t cap_blocks,
                      size_t *n_blocks);

/* Host-memory one-shot forms: the streamed forms above over
 * one host buffer (the device holds at most the piece ring, whatever len is). */
int vs_rsync_signatures(int device, const void *basis, int64_t len, int32_t blength,
                        int32_t s2length, int csum_type, uint32_t seed, uint32_t *sum1,
                        uint8_t *sum2);
typedef struct vs_sigtable {
    int32_t count, blength, s2length, remainder;
    const uint32_t *sum1; /* [count] */
    const uint8_t *sum2;  /* [count * s2length] */
} vs_sigtable;
int vs_rsync_match(int device, const void *src, int64_t len, const vs_sigtable *t,
                   int csum_type, uint32_t seed, vs_match *out, size_t cap, size_t *n_out);

/* ---- restic blob encryption (the pack stage) -----------
 * restic v0.13.1 internal/crypto Key.Seal per blob: ciphertext =
 * AES-256-CTR(enc_key, IV = the blob's 16-byte nonce, the whole block
 * incremented as a 128-bit big-endian counter), mac = Poly1305(ciphertext,
 * r = mac_r (clamped), s = AES-128(mac_k, nonce)).  The repository stores
 * nonce || ciphertext || mac.  A vs_seal handle holds one repository key. */
typedef struct vs_seal vs_seal;
int vs_seal_open(int device, const uint8_t enc_key[32], const uint8_t mac_k[16],
                 const uint8_t mac_r[16], vs_seal **h);
/* Blob i = dev_in[off[i] : off[i]+len[i]] (device arrays); its ciphertext is
 * written to dev_out at the same offset (dev_out may equal dev_in) and its
 * mac to dev_macs[16*i]; nonces: device array of n*16 bytes, 16-byte aligned.  Queued on
 * hip_stream after a short read-back of the block count. */
int vs_seal_run_device(vs_seal *h, const void *dev_in, const uint64_t *dev_off,
                       const uint32_t *dev_len, size_t n, const uint8_t *dev_nonces,
                       uint8_t *dev_out, uint8_t *dev_macs, void *hip_stream);
/* Kernel timing for measurement: when on, each run records HIP events around
 * its CTR and MAC kernels; vs_seal_kernel_ms waits for them and returns the
 * summed milliseconds (ms[0] CTR, ms[1] MAC) and the run count, then resets. */
int vs_seal_set_timing(vs_seal *h, int on);
int vs_seal_kernel_ms(vs_seal *h, double ms[2], int *runs);
/* Key.Seal into the pack layout: blob i's record nonce || ciphertext || tag
 * is written around dev_out + ct_off[i] (the nonce at ct_off - 16, the tag
 * at ct_off + len) -- restic Packer.Add of repository.saveAndEncrypt's
 * output. */
int vs_seal_records_device(vs_seal *h, const void *dev_in, const uint64_t *dev_off,
                           const uint32_t *dev_len, size_t n, const uint8_t *dev_nonces,
                           uint8_t *dev_out, const uint64_t *dev_ct_off, void *hip_stream);
/* restic internal/crypto Key.Open over a batch of stored blobs (restic
 * Repository.LoadBlob on restore, mover-restic/entry.sh:224): record i at
 * dev_in + rec_off[i] is nonce || ciphertext (len[i] bytes) || tag.  Every
 * tag is verified (Poly1305 over the ciphertext, as Open does before it
 * decrypts) and the ciphertext is decrypted to dev_out + out_off[i]
 * (out_off NULL: in the same layout, i.e. at rec_off[i] + 16 of dev_out;
 * dev_out == dev_in decrypts in place).  bad[i] (device) = 1 where the tag
 * does not match: that plaintext must be discarded (Open returns
 * ErrUnauthenticated); n_bad (host, optional: waits) counts them. */
int vs_open_run_device(vs_seal *h, const void *dev_in, const uint64_t *dev_rec_off,
                       const uint32_t *dev_len, size_t n, uint8_t *dev_out,
                       const uint64_t *dev_out_off, uint32_t *dev_bad, uint64_t *n_bad,
                       void *hip_stream);
/* restic v0.13.1 pack files from sealed blobs (internal/pack Packer +
 * internal/repository's packer managers): blobs (plaintext on the device at
 * off[i], len[i] bytes; host arrays, in save order, with their types 0 data /
 * 1 tree and 32-byte IDs) are appended to their type's open pack, finalised
 * once it holds >= min_pack_size bytes (v0.13.1: 4 MiB); at the end the data
 * pack, then the tree pack.  Each pack = the blob records, the header (per
 * blob: type, record length, ID; sealed with hdr_nonces[p]) and the sealed
 * header's length (4-byte LE).  dev_out receives the packs back to back;
 * packs[p] = {offset, length, first blob in pack order, n blobs}; pack_ids =
 * SHA-256 of each pack file (its name in the repository), by the vs_sha
 * engine.  dev_out NULL: *n_packs, *out_len (and packs, if given) only.
 * hdr_nonces needs one 16-byte row per pack (n rows always suffice). */
typedef struct {
    uint64_t offset, length;
    uint32_t first_blob, n_blobs;
} vs_pack;
int vs_restic_pack(vs_seal *h, vs_sha *sha, const void *dev_in, const uint64_t *off,
                   const uint32_t *len, const uint8_t *types, const uint8_t *ids, size_t n,
                   const uint8_t *blob_nonces, const uint8_t *hdr_nonces, uint64_t min_pack_size,
                   uint8_t *dev_out, uint64_t out_cap, vs_pack *packs, size_t pack_cap,
                   size_t *n_packs, uint64_t *out_len, uint8_t *pack_ids, void *hip_stream);
/* restic v0.13.1 internal/index Index.Encode + repository.SaveUnpacked: the
 * index file of the packs vs_restic_pack made from the same blobs (same len,
 * types, ids, n, min_pack_size; pack_ids as it returned them).  The JSON is
 * {"packs":[{"id":...,"blobs":[{"id":...,"type":"data"|"tree","offset":o,
 * "length":l}...]}...]} plus a newline, l = the stored record length
 * (plaintext + 32) and o its offset in the pack; packs in finalize order,
 * blobs in pack order (restic's own order follows a randomly seeded hash map;
 * its DecodeIndex reads any).  json_out (NULL: size only) receives it;
 * file_out (NULL: JSON only) the stored file nonce || Key.Seal(JSON) || tag
 * (*json_n + 32 bytes), file_id its SHA-256 (the name in the repository). */
int vs_restic_index(vs_seal *h, vs_sha *sha, const uint32_t *len, const uint8_t *types,
                    const uint8_t *ids, size_t n, uint64_t min_pack_size, const uint8_t *pack_ids,
                    const uint8_t nonce[16], uint8_t *json_out, size_t json_cap, size_t *json_n,
                    uint8_t *file_out, uint8_t file_id[32]);
void vs_seal_close(vs_seal *h);

/* ---- wire formats (host code, no device needed) -------
 * rsync 3.2.3 io.c write_sum_head + generate_and_send_sums: count, blength,
 * s2length, remainder (4-byte LE each), then per block sum1 (4-byte LE) and
 * s2length bytes of sum2.  out == NULL: *n_out = the size only. */
int vs_rsync_write_sums(int32_t count, int32_t blength, int32_t s2length, int32_t remainder,
                        const uint32_t *sum1, const uint8_t *sum2, uint8_t *out, size_t cap,
                        size_t *n_out);
/* read_sum_head + the per-block sums (sum1 / sum2 NULL: the header only). */
int vs_rsync_read_sums(const uint8_t *in, size_t n, int32_t *count, int32_t *blength,
                       int32_t *s2length, int32_t *remainder, uint32_t *sum1, uint8_t *sum2,
                       size_t cap_blocks);
/* token.c simple_send_token as match.c matched() drives it (no -z): literal
 * runs in <= 32 KiB pieces, each after its 4-byte LE length, the token
 * -(i+1) per match of block i, and 0 after the file's last literal.  src is
 * the source file (host).  out == NULL: *n_out = the size only. */
int vs_rsync_write_tokens(const vs_match *matches, int64_t n_matches, int64_t file_len,
                          int32_t blength, int64_t basis_len, const uint8_t *src, uint8_t *out,
                          size_t cap, size_t *n_out);
/* receiver.c's side: the match list (offsets in the new file) and the literal
 * bytes, concatenated, of a token stream; matches / literals may be NULL to
 * size them first. */
int vs_rsync_read_tokens(const uint8_t *in, size_t n, int32_t blength, int64_t basis_len,
                         vs_match *matches, size_t cap, size_t *n_matches, uint8_t *literals,
                         size_t lit_cap, size_t *n_literal, int64_t *file_len);
/* token.c send_zstd_token / recv_zstd_token: the token stream under rsync -z
 * between two rsync 3.2.3 (UBI9) peers, which negotiate zstd (DESIGN.md
 * 3.11).  A vs_ztok is one transfer's zstd state: rsync creates the
 * compressor / decompressor once per transfer and every file continues the
 * same stream, so write / read the files of a transfer through one handle,
 * in order (a receiver uses its own handle).  level: rsync's
 * --compress-level (3, ZSTD_CLEVEL_DEFAULT, when not given).
 * write: the stream of one file from its match list (as match.c drives
 * send_token, including hash_search's early literal flushes), into a buffer
 * owned by the handle (*out, valid until the next call); last_block_len is
 * sums[count - 1].len (the remainder, or blength).
 * read: one file's stream from in (*consumed bytes), as write's inputs. */
typedef struct vs_ztok vs_ztok;
int vs_ztok_open(int level, vs_ztok **out);
void vs_ztok_close(vs_ztok *z);
int vs_rsync_write_tokens_zstd(vs_ztok *z, const vs_match *matches, int64_t n_matches,
                               int64_t file_len, int32_t blength, int64_t basis_len,
                               int32_t last_block_len, const uint8_t *src, const uint8_t **out,
                               size_t *n_out);
int vs_rsync_read_tokens_zstd(vs_ztok *z, const uint8_t *in, size_t n, int32_t blength,
                              int64_t basis_len, vs_match *matches, size_t cap, size_t *n_matches,
                              uint8_t *literals, size_t lit_cap, size_t *n_literal,
                              int64_t *file_len, size_t *consumed);
/* restic v0.13.1 internal/pack header plaintext: per blob its type (0 data,
 * 1 tree), the length of its encrypted form (4-byte LE) and its 32-byte ID,
 * 37 bytes per entry.  out == NULL: *n_out = the size only. */
int vs_restic_pack_header(const uint8_t *types, const uint32_t *lengths, const uint8_t *ids,
                          size_t n, uint8_t *out, size_t cap, size_t *n_out);

/* ---- options -----------------------------------------------------------
 * The library reads no environment variables: the few settings a test or a
 * measurement needs to change are set per handle here.  The defaults are the
 * product settings; results are identical under every option (they change
 * which kernels run or how work is split, never what is computed). */
#define VS_OPT_WALK_SEGMENT_BLOCKS 1 /* rsync: device walk segment length in blocks
                                      * (0 = automatic: 48, shorter for ranges too
                                      * small to give every wave two segments) */
#define VS_OPT_FILE_SUM_PIECE 2      /* rsync: file-sum read-back piece in 1 KiB blocks
                                      * (0 = 2^18: 16 MiB of contribution rows) */
#define VS_OPT_BUCKET_BITS 3         /* rsync: log2 of the walk's membership buckets,
                                      * applied at the next load_sums (0 = automatic) */
#define VS_OPT_FA_RECORD 4           /* rsync: false-alarm windows recorded per walk
                                      * segment for stitch merges (-1 = automatic) */
#define VS_OPT_HOST_WALK 5           /* rsync: 1 = the host walk with device
                                      * verification for every checksum type */
#define VS_OPT_WALK_PREFILTER 6      /* rsync: 0 = the device walk without its LDS
                                      * prefilter (default 1) */
#define VS_OPT_WALK_FLUSH_WINDOWS 7  /* rsync: STEP weak hits hashed per flush: 16 =
                                      * address-lockstep passes over the resync span
                                      * (blocks > 1 KiB; 0 = default), 4 = four
                                      * windows per pass */
#define VS_OPT_WALK_FLUSH_SPAN 8     /* rsync: flush once the scan is this many bytes
                                      * past the first queued hit (0 = no bound; default) */
#define VS_OPT_WALK_FLUSH_PREDICT 9  /* rsync: 1 = flush the STEP queue at once at a hit
                                      * whose weak sum is that of block want_i .. want_i + 2,
                                      * the usual resync after an edit (default 1) */
#define VS_OPT_WALK_TAIL_PCT 10      /* rsync: % of the walk range cut into quarter-length
                                      * segments handed out last (-1 = automatic, the
                                      * default: 20 below four segments per wave, else 10) */
#define VS_OPT_WALK_SEG_MARGIN 11    /* rsync: device walk segments after the first start
                                      * this many bytes before a block boundary of the file
                                      * (-1 = automatic, the default: 24576; 0 = segments
                                      * from the range start, unaligned) */
#define VS_OPT_SHA_QUAD_PCT 16       /* cdc / sha: which chains of a latency-bound final
                                      * drain run in latency (quad) mode.  -1 (default):
                                      * every chain that would finish after the drain's
                                      * floor -- max(longest chain in quad mode, backlog
                                      * at split throughput) -- in split mode beside the
                                      * bulk; 1..1000: the chains within this % of the
                                      * longest; 0 = split mode only */
#define VS_OPT_SHA_GRID_PER_CU 18   /* cdc / sha: persistent hash grid per CU: split-mode
                                      * workgroups (default 5) / throughput-mode waves
                                      * per SIMD (default 3); 0 = default */
#define VS_OPT_SHA_ISOLATE 19         /* cdc / sha: 1 (default) = a latency-bound final
                                      * drain gives each quad tile a CU of its own (its
                                      * LDS padded to the whole CU), resident before the
                                      * split tiles start beside it; 0 = one launch */
#define VS_OPT_FP_GENERIC 17         /* cdc: 1 = the generic fingerprint address code
                                      * even where the FAST variant applies */
#define VS_OPT_SEAL_FUSED 32         /* seal: 0 = separate CTR and MAC kernels (default 1) */
int vs_rsync_set_option(vs_rsync *h, int option, int64_t value);
int vs_cdc_set_option(vs_cdc *h, int option, int64_t value);
int vs_sha256_set_option(vs_sha *h, int option, int64_t value);
int vs_seal_set_option(vs_seal *h, int option, int64_t value);

/* ---- device utilities for benches and tests --------------------------- */
/* Fill dev_out[0:n] with bytes [off, off+n) of the synthetic splitmix64
 * volume stream.  hip_stream NULL: returns when the fill is
 * complete; otherwise queued on that stream. */
int vs_synth_fill_device(int device, uint64_t seed, uint64_t off, uint64_t n, void *dev_out,
                         void *hip_stream);

#ifdef __cplusplus
}
#endif
#endif /* VSGPU_H */
