// gb_spgemm_hash.hip -- entry of the hash Gustavson SpGEMM (gb_spgemm_hash.cuh): picks the
// semiring instantiation; the instantiations are compiled in gb_spgemm_hash_p*.hip.
#include "gb_dispatch.cuh"
#include "gb_internal.h"

namespace gbh {
template <class SRT, class X, class Z>
void spgemm_hash_run(gb_mat_result &T, gb_csr_view &A, gb_csr_view &B, const gb_sr_info &info, SRT srf,
                     bool vals_needed, const void *av, const void *bv, const int64_t *flops);
}  // namespace gbh

// C = A * B (no mask applied here): T gets sorted CSR rows.
void gb_spgemm_hash(gb_mat_result &T, gb_csr_view &A, gb_csr_view &B, GrB_Semiring sring, bool iso,
                    const void *av, const void *bv, const int64_t *flops) {
    const gb_sr_info info = gb_sr_describe(sring);
    gb_dispatch_sr(info, [&](auto srf, auto x, auto z) {
        gbh::spgemm_hash_run<decltype(srf), decltype(x), decltype(z)>(T, A, B, info, srf, !iso, av, bv, flops);
    });
}
