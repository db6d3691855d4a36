// gb_spgemm_hash_p1.hip -- instantiations of the hash Gustavson SpGEMM (gb_spgemm_hash.cuh),
// one file per group of semirings so the builds run in parallel.
#include "gb_spgemm_hash.cuh"

#define SS_DYN(X, Z) gb_sr_dyn<X, Z>
GB_SPGEMM_HASH_INST(gb_sr_min_plus<int64_t>, int64_t, int64_t)
GB_SPGEMM_HASH_INST(gb_sr_min_plus<int32_t>, int32_t, int32_t)
GB_SPGEMM_HASH_INST(gb_sr_min_plus<double>, double, double)
GB_SPGEMM_HASH_INST(gb_sr_any_pair<bool>, bool, bool)
GB_SPGEMM_HASH_INST(gb_sr_any_pair<int64_t>, int64_t, int64_t)
GB_SPGEMM_HASH_INST(gb_sr_any_pair<int32_t>, int32_t, int32_t)
GB_SPGEMM_HASH_INST(gb_sr_lor_land, bool, bool)
