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
#include <hipcub/hipcub.hpp>

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

}  // namespace

size_t dedup_tmp_bytes(uint64_t n) {
    size_t b = 0;
    (void)hipcub::DeviceRadixSort::SortPairs(nullptr, b, (const uint64_t *)nullptr,
                                             (uint64_t *)nullptr, (const uint32_t *)nullptr,
                                             (uint32_t *)nullptr, (int)n, 0, 64);
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
    e = hipcub::DeviceRadixSort::SortPairs(scratch, sb, keys, skeys, idx, sidx, (int)n, 0, 64, s);
    if (e != hipSuccess) return e;
    dd_first_kernel<<<blocks, 256, 0, s>>>(ids, n, skeys, sidx, first, n_unique_dev);
    return hipGetLastError();
}

}  // namespace vsgpu
