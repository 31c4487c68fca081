// knn_d2.hip -- K1 instantiations for d = 2 (see knn_impl.hpp).
#include "knn_impl.hpp"

namespace hdb {

void knn_run_d2(hdb_ctx *ctx, int KC, bool excl, bool idx, const double *Xp, int64_t n, double *ov, int32_t *oi) {
    if (idx) {
        if (excl) dispatch_k<2, true, true>(ctx, KC, Xp, n, ov, oi);
        else dispatch_k<2, false, true>(ctx, KC, Xp, n, ov, oi);
    } else {
        if (excl) dispatch_k<2, true, false>(ctx, KC, Xp, n, ov, nullptr);
        else dispatch_k<2, false, false>(ctx, KC, Xp, n, ov, nullptr);
    }
}

}  // namespace hdb
