// dedup.hip -- the SaveBlob dedup seam on the device.
//
// restic v0.13.1 internal/repository Repository.SaveBlob looks the blob ID
// up in the index (idx.Has / AddPending): the first blob with a given ID is
// stored, every later one with the same ID is a duplicate.  For a batch of
// n blob IDs in stream order this kernel chain returns, per blob, the index
// of the first blob with the same ID (itself when it is new) and the number
// of distinct IDs: a stable radix sort of (first 8 ID bytes, index) pairs,
// then, within each run of equal 8-byte prefixes, a full 32-byte compare
// against the earlier members of the run (prefix collisions of distinct
// SHA-256 IDs are vanishingly rare, but the result does not rely on it).
#include <rocprim/device/device_radix_sort.hpp>

#include "internal.hpp"

namespace vsgpu {
namespace {

__global__ void dd_keys_kernel(const uint8_t *ids, uint64_t n, uint64_t *keys, uint32_t *idx) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint8_t *p = ids + 32 * i;
    uint64_t k = 0;
    for (int b = 0; b < 8; ++b) k = (k << 8) | p[b];   // big-endian: byte order = key order
    keys[i] = k;
    idx[i] = (uint32_t)i;
}

__device__ __forceinline__ bool id_eq(const uint8_t *ids, uint32_t a, uint32_t b) {
    const uint4 *x = (const uint4 *)(ids + 32 * (uint64_t)a);
    const uint4 *y = (const uint4 *)(ids + 32 * (uint64_t)b);
    const uint4 x0 = x[0], x1 = x[1], y0 = y[0], y1 = y[1];
    return x0.x == y0.x && x0.y == y0.y && x0.z == y0.z && x0.w == y0.w && x1.x == y1.x &&
           x1.y == y1.y && x1.z == y1.z && x1.w == y1.w;
}

// sorted position p: first[idx[p]] = the smallest index with the same ID.
// Equal IDs have equal keys, so they sit in one run of equal keys, in
// ascending index order (the sort is stable); the first equal member of the
// run is the first occurrence.  The run start is a binary search (a run of a
// million identical blobs costs log n per blob, not n); only a run that mixes
// distinct IDs with one 8-byte prefix is scanned member by member.
__global__ void dd_first_kernel(const uint8_t *ids, uint64_t n, const uint64_t *skeys,
                                const uint32_t *sidx, uint32_t *first,
                                unsigned long long *n_unique) {
    const uint64_t p = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    bool is_new = false;
    if (p < n) {
        const uint64_t k = skeys[p];
        uint64_t lo = 0, hi = p;
        while (lo < hi) {
            const uint64_t mid = (lo + hi) >> 1;
            if (skeys[mid] < k) lo = mid + 1;
            else hi = mid;
        }
        const uint32_t me = sidx[p];
        uint32_t f = me;
        for (uint64_t q = lo; q < p; ++q)
            if (id_eq(ids, sidx[q], me)) {
                f = sidx[q];
                break;
            }
        first[me] = f;
        is_new = f == me;
    }
    const uint64_t b = __ballot(is_new);
    if ((threadIdx.x & 63) == 0 && b) atomicAdd(n_unique, (unsigned long long)__popcll(b));
}

// ---- the repository's index (restic Repository.SaveBlob: idx.AddPending
// fails for a blob the master index already holds) ----------------------------
// The known IDs come as a device array sorted by their first 8 bytes read
// big-endian (vs_blob_index_sort; the order of IDs sharing a prefix is
// irrelevant): membership is a lower_bound on the prefix, then a full 32-byte
// compare over the run of equal prefixes.
__device__ __forceinline__ uint64_t id_key(const uint8_t *p) {
    const uint2 w = *(const uint2 *)p;
    return ((uint64_t)__builtin_bswap32(w.x) << 32) | __builtin_bswap32(w.y);
}

__device__ bool id_known(const uint8_t *id, const uint8_t *known, uint64_t n_known) {
    const uint64_t k = id_key(id);
    uint64_t lo = 0, hi = n_known;
    while (lo < hi) {
        const uint64_t mid = (lo + hi) >> 1;
        if (id_key(known + 32 * mid) < k) lo = mid + 1;
        else hi = mid;
    }
    const uint4 *x = (const uint4 *)id;
    const uint4 x0 = x[0], x1 = x[1];
    for (uint64_t q = lo; q < n_known && id_key(known + 32 * q) == k; ++q) {
        const uint4 *y = (const uint4 *)(known + 32 * q);
        const uint4 y0 = y[0], y1 = y[1];
        if (x0.x == y0.x && x0.y == y0.y && x0.z == y0.z && x0.w == y0.w && x1.x == y1.x &&
            x1.y == y1.y && x1.z == y1.z && x1.w == y1.w)
            return true;
    }
    return false;
}

// first occurrences only: flag[i] = 1 when blob i's ID is in the index
__global__ void dd_known_kernel(const uint8_t *ids, uint64_t n, const uint8_t *known,
                                uint64_t n_known, const uint32_t *first, uint8_t *flag) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    flag[i] = (first[i] == (uint32_t)i && id_known(ids + 32 * i, known, n_known)) ? 1 : 0;
}

// every blob whose first occurrence is known: first = kDedupKnown; the count
// becomes the distinct IDs the index does not hold (the blobs SaveBlob stores)
__global__ void dd_mark_known_kernel(uint64_t n, const uint8_t *flag, uint32_t *first,
                                     unsigned long long *n_new) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    bool is_new = false;
    if (i < n) {
        const uint32_t f = first[i];
        if (flag[f]) first[i] = kDedupKnown;
        else is_new = f == (uint32_t)i;
    }
    const uint64_t b = __ballot(is_new);
    if ((threadIdx.x & 63) == 0 && b) atomicAdd(n_new, (unsigned long long)__popcll(b));
}

__global__ void idx_keys_kernel(const uint8_t *ids, uint64_t n, uint64_t *keys, uint32_t *idx) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    keys[i] = id_key(ids + 32 * i);
    idx[i] = (uint32_t)i;
}

__global__ void idx_gather_kernel(const uint8_t *src, uint64_t n, const uint32_t *sidx,
                                  uint8_t *dst) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= 2 * n) return;   // two 16-byte halves per ID
    const uint64_t r = i >> 1, h = i & 1;
    ((uint4 *)dst)[2 * r + h] = ((const uint4 *)src)[2 * (uint64_t)sidx[r] + h];
}

}  // namespace

size_t dedup_known_tmp_bytes(uint64_t n) { return n + 256; }

hipError_t launch_dedup_known(const uint8_t *ids, uint64_t n, const uint8_t *known,
                              uint64_t n_known, uint32_t *first, void *flag_tmp,
                              unsigned long long *n_new_dev, hipStream_t s) {
    hipError_t e = hipMemsetAsync(n_new_dev, 0, 8, s);
    if (e != hipSuccess || !n) return e;
    const uint32_t blocks = (uint32_t)((n + 255) / 256);
    dd_known_kernel<<<blocks, 256, 0, s>>>(ids, n, known, n_known, first, (uint8_t *)flag_tmp);
    dd_mark_known_kernel<<<blocks, 256, 0, s>>>(n, (const uint8_t *)flag_tmp, first, n_new_dev);
    return hipGetLastError();
}

size_t index_sort_tmp_bytes(uint64_t n) {
    size_t b = 0;
    (void)rocprim::radix_sort_pairs(nullptr, b, (const uint64_t *)nullptr, (uint64_t *)nullptr,
                                    (const uint32_t *)nullptr, (uint32_t *)nullptr, (size_t)n, 0, 64);
    // keys, sorted keys, idx, sorted idx, a copy of the IDs, then the scratch
    return n * (8 + 8 + 4 + 4 + 32) + 512 + b;
}

hipError_t launch_index_sort(uint8_t *ids, uint64_t n, void *tmp, size_t tmp_bytes,
                             hipStream_t s) {
    if (n < 2) return hipSuccess;
    uint8_t *t = (uint8_t *)tmp;
    uint8_t *copy = (uint8_t *)(((uintptr_t)t + 15) & ~(uintptr_t)15);
    uint64_t *keys = (uint64_t *)(copy + 32 * n);
    uint64_t *skeys = keys + n;
    uint32_t *idx = (uint32_t *)(skeys + n);
    uint32_t *sidx = idx + n;
    uint8_t *scratch = (uint8_t *)(((uintptr_t)(sidx + n) + 255) & ~(uintptr_t)255);
    size_t sb = tmp_bytes - (size_t)(scratch - t);
    const uint32_t blocks = (uint32_t)((n + 255) / 256);
    idx_keys_kernel<<<blocks, 256, 0, s>>>(ids, n, keys, idx);
    hipError_t e = hipMemcpyAsync(copy, ids, 32 * n, hipMemcpyDeviceToDevice, s);
    if (e != hipSuccess) return e;
    e = rocprim::radix_sort_pairs(scratch, sb, keys, skeys, idx, sidx, (size_t)n, 0, 64, s);
    if (e != hipSuccess) return e;
    idx_gather_kernel<<<(uint32_t)((2 * n + 255) / 256), 256, 0, s>>>(copy, n, sidx, ids);
    return hipGetLastError();
}

size_t dedup_tmp_bytes(uint64_t n) {
    size_t b = 0;
    (void)rocprim::radix_sort_pairs(nullptr, b, (const uint64_t *)nullptr, (uint64_t *)nullptr,
                                    (const uint32_t *)nullptr, (uint32_t *)nullptr, (size_t)n, 0, 64);
    // keys, sorted keys, idx, sorted idx, counter, then the sort scratch
    return n * (8 + 8 + 4 + 4) + 512 + b;
}

hipError_t launch_dedup(const uint8_t *ids, uint64_t n, uint32_t *first, void *tmp,
                        size_t tmp_bytes, unsigned long long *n_unique_dev, hipStream_t s) {
    // the counter takes a 64-bit atomic: a misaligned one is a memory violation
    if (((uintptr_t)n_unique_dev & 7) || ((uintptr_t)tmp & 7)) return hipErrorInvalidValue;
    hipError_t e = hipMemsetAsync(n_unique_dev, 0, 8, s);
    if (e != hipSuccess || !n) return e;
    uint8_t *t = (uint8_t *)tmp;
    uint64_t *keys = (uint64_t *)t;
    uint64_t *skeys = keys + n;
    uint32_t *idx = (uint32_t *)(skeys + n);
    uint32_t *sidx = idx + n;
    // the sort's scratch 256-byte aligned (rocprim's look-back state is
    // updated with wide atomics)
    uint8_t *scratch = (uint8_t *)(((uintptr_t)(sidx + n) + 256 + 255) & ~(uintptr_t)255);
    size_t sb = tmp_bytes - (size_t)(scratch - t);
    const uint32_t blocks = (uint32_t)((n + 255) / 256);
    dd_keys_kernel<<<blocks, 256, 0, s>>>(ids, n, keys, idx);
    e = rocprim::radix_sort_pairs(scratch, sb, keys, skeys, idx, sidx, (size_t)n, 0, 64, s);
    if (e != hipSuccess) return e;
    dd_first_kernel<<<blocks, 256, 0, s>>>(ids, n, skeys, sidx, first, n_unique_dev);
    return hipGetLastError();
}

}  // namespace vsgpu
