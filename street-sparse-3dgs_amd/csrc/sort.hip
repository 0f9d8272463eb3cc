// sort.hip -- device scan (tiles_touched -> offsets) and the LSD radix sort of the
// (tile << 32 | depth) keys, on rocPRIM.  Kept in its own
// translation unit: rocPRIM's templates dominate compile time.
#include <cstring>
#include <rocprim/rocprim.hpp>
#include "gsr_launch.h"

namespace gsr {

size_t scan_temp_bytes(int P) {
    size_t bytes = 0;
    rocprim::inclusive_scan(nullptr, bytes, (const uint32_t *)nullptr, (uint32_t *)nullptr, (size_t)(P > 0 ? P : 1),
                            rocprim::plus<uint32_t>());
    return bytes;
}

hipError_t inclusive_scan_u32(void *tmp, size_t tmp_bytes, const uint32_t *in, uint32_t *out, int P, hipStream_t s) {
    if (P == 0) return hipSuccess;
    return rocprim::inclusive_scan(tmp, tmp_bytes, in, out, (size_t)P, rocprim::plus<uint32_t>(), s);
}

size_t sort_temp_bytes(int64_t K, int end_bit) {
    size_t bytes = 0;
    rocprim::radix_sort_pairs(nullptr, bytes, (const uint64_t *)nullptr, (uint64_t *)nullptr,
                              (const uint32_t *)nullptr, (uint32_t *)nullptr, (size_t)(K > 0 ? K : 1), 0, end_bit);
    return bytes;
}

hipError_t sort_pairs_u64(void *tmp, size_t tmp_bytes, const uint64_t *kin, uint64_t *kout, const uint32_t *vin,
                          uint32_t *vout, int64_t K, int end_bit, hipStream_t s) {
    if (K == 0) return hipSuccess;
    return rocprim::radix_sort_pairs(tmp, tmp_bytes, kin, kout, vin, vout, (size_t)K, 0, end_bit, s);
}

}  // namespace gsr
