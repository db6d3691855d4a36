// gb_spgemm_hash_p0.hip -- instantiations of the hash Gustavson SpGEMM (gb_spgemm_hash.cuh),
// one file per group of semirings so the builds run in parallel.
#include "gb_spgemm_hash.cuh"

#define SS_DYN(X, Z) gb_sr_dyn<X, Z>
GB_SPGEMM_HASH_INST(gb_sr_plus_times<double>, double, double)
GB_SPGEMM_HASH_INST(gb_sr_plus_times<float>, float, float)
GB_SPGEMM_HASH_INST(gb_sr_plus_times<int64_t>, int64_t, int64_t)
