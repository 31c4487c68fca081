// sort.hpp -- stable LSD radix sorts of (key, value) pairs that always take rocprim's
// onesweep path.  rocprim's default config switches to block-sort + merge-path below 2^20
// items; for the ~1M-item sorts on the hot path (Morton order, Boruvka edge order) that
// took ~200 us per sort vs ~90-140 us for onesweep (profiles/r01).  Both are stable, so
// the results are identical.
#pragma once
#include <rocprim/device/device_radix_sort.hpp>

namespace hdb {

using OnesweepOnly = rocprim::radix_sort_config<rocprim::default_config, rocprim::default_config,
                                                rocprim::default_config, 0>;

template <class K, class V>
inline hipError_t sort_pairs(void *tmp, size_t &bytes, const K *kin, K *kout, const V *vin, V *vout, int64_t n,
                             int begin_bit, int end_bit, hipStream_t st) {
    return rocprim::radix_sort_pairs<OnesweepOnly>(tmp, bytes, kin, kout, vin, vout, (size_t)n, (unsigned)begin_bit,
                                                   (unsigned)end_bit, st);
}

template <class K, class V>
inline hipError_t sort_pairs_desc(void *tmp, size_t &bytes, const K *kin, K *kout, const V *vin, V *vout, int64_t n,
                                  int begin_bit, int end_bit, hipStream_t st) {
    return rocprim::radix_sort_pairs_desc<OnesweepOnly>(tmp, bytes, kin, kout, vin, vout, (size_t)n,
                                                        (unsigned)begin_bit, (unsigned)end_bit, st);
}

}  // namespace hdb
