// knn_d16.hip -- K1 instantiations for d = 16 (see knn_impl.hpp).
#include "knn_impl.hpp"

namespace hdb {

void knn_run_d16(hdb_ctx *ctx, int KC, bool excl, bool idx, const double *Xp, int64_t n, double *ov, int32_t *oi) {
    if (idx) {
        if (excl) dispatch_k<16, true, true>(ctx, KC, Xp, n, ov, oi);
        else dispatch_k<16, false, true>(ctx, KC, Xp, n, ov, oi);
    } else {
        if (excl) dispatch_k<16, true, false>(ctx, KC, Xp, n, ov, nullptr);
        else dispatch_k<16, false, false>(ctx, KC, Xp, n, ov, nullptr);
    }
}

}  // namespace hdb
