// sort.hip -- device scans and radix sorts on rocPRIM.
//
// Binning order.  Upstream sorts K (tile << 32 | depth bits) 64-bit keys over 32 + bits(T)
// bits (6 LSD passes of 8 bits at 1080p).  Here the same total order is produced with far less
// traffic: (1) the P Gaussians are stably sorted by their 32-bit depth bits, (2) instances are
// emitted in that order, (3) the K instances are stably sorted by tile id alone (bits(T) = 13 at
// 1080p: 2 passes over 2-byte keys).  Stability makes the result (tile, depth, id) order --
// exactly the upstream key order, tie-breaks included.  Kept in its own translation unit:
// rocPRIM's templates dominate compile time.
#include <cstring>
#include <rocprim/rocprim.hpp>
#include "gsr_launch.h"

namespace gsr {

namespace {
// rocPRIM routes radix sorts of up to 2^20 items through block-sort + 10 merge passes; for the
// P ~ 1M depth keys that is ~150 us/frame on MI355X vs a few onesweep passes.  Cap the merge path.
using OnesweepCfg = rocprim::radix_sort_config<rocprim::default_config, rocprim::default_config,
                                               rocprim::default_config, 8192>;

struct GatherTiles {
    const uint32_t *tiles;
    __host__ __device__ uint32_t operator()(uint32_t g) const { return tiles[g]; }
};
}  // namespace

size_t scan_temp_bytes(int P) {
    size_t bytes = 0;
    auto it = rocprim::make_transform_iterator((const uint32_t *)nullptr, GatherTiles{nullptr});
    rocprim::inclusive_scan(nullptr, bytes, it, (uint32_t *)nullptr, (size_t)(P > 0 ? P : 1),
                            rocprim::plus<uint32_t>());
    return bytes;
}

hipError_t inclusive_scan_gathered(void *tmp, size_t tmp_bytes, const uint32_t *order, const uint32_t *tiles,
                                   uint32_t *out, int P, hipStream_t s) {
    if (P == 0) return hipSuccess;
    auto it = rocprim::make_transform_iterator(order, GatherTiles{tiles});
    return rocprim::inclusive_scan(tmp, tmp_bytes, it, out, (size_t)P, rocprim::plus<uint32_t>(), s);
}

size_t depth_sort_temp_bytes(int P) {
    size_t bytes = 0;
    rocprim::radix_sort_pairs<OnesweepCfg>(nullptr, bytes, (const uint32_t *)nullptr, (uint32_t *)nullptr,
                                           (const uint32_t *)nullptr, (uint32_t *)nullptr, (size_t)(P > 0 ? P : 1),
                                           0, 32);
    return bytes;
}

hipError_t depth_sort(void *tmp, size_t tmp_bytes, const uint32_t *kin, uint32_t *kout, const uint32_t *vin,
                      uint32_t *vout, int P, hipStream_t s) {
    if (P == 0) return hipSuccess;
    return rocprim::radix_sort_pairs<OnesweepCfg>(tmp, tmp_bytes, kin, kout, vin, vout, (size_t)P, 0, 32, s);
}

size_t tile_sort_temp_bytes(int64_t K, int end_bit, bool wide) {
    size_t bytes = 0;
    const size_t n = (size_t)(K > 0 ? K : 1);
    if (wide)
        rocprim::radix_sort_pairs(nullptr, bytes, (const uint32_t *)nullptr, (uint32_t *)nullptr,
                                  (const uint32_t *)nullptr, (uint32_t *)nullptr, n, 0, end_bit);
    else
        rocprim::radix_sort_pairs(nullptr, bytes, (const uint16_t *)nullptr, (uint16_t *)nullptr,
                                  (const uint32_t *)nullptr, (uint32_t *)nullptr, n, 0, end_bit);
    return bytes;
}

hipError_t tile_sort(void *tmp, size_t tmp_bytes, const void *kin, void *kout, const uint32_t *vin, uint32_t *vout,
                     int64_t K, int end_bit, bool wide, hipStream_t s) {
    if (K == 0) return hipSuccess;
    if (wide)
        return rocprim::radix_sort_pairs(tmp, tmp_bytes, static_cast<const uint32_t *>(kin),
                                         static_cast<uint32_t *>(kout), vin, vout, (size_t)K, 0, end_bit, s);
    return rocprim::radix_sort_pairs(tmp, tmp_bytes, static_cast<const uint16_t *>(kin), static_cast<uint16_t *>(kout),
                                     vin, vout, (size_t)K, 0, end_bit, s);
}

size_t tile_order_temp_bytes(int T) {
    size_t bytes = 0;
    rocprim::radix_sort_pairs_desc(nullptr, bytes, (const uint32_t *)nullptr, (uint32_t *)nullptr,
                                   (const uint32_t *)nullptr, (uint32_t *)nullptr, (size_t)(T > 0 ? T : 1), 0, 16);
    return bytes;
}

// Stable descending sort of the T per-tile work estimates (clamped to 16 bits by the producer):
// equal-work tiles keep index order, so the launch order is deterministic.
hipError_t tile_order(void *tmp, size_t tmp_bytes, const uint32_t *work, uint32_t *work_sorted, const uint32_t *ids,
                      uint32_t *order, int T, hipStream_t s) {
    if (T == 0) return hipSuccess;
    return rocprim::radix_sort_pairs_desc(tmp, tmp_bytes, work, work_sorted, ids, order, (size_t)T, 0, 16, s);
}

}  // namespace gsr
