// gb_spgemm_hash_p6.hip -- instantiations of the hash Gustavson SpGEMM (gb_spgemm_hash.cuh),
// one file per group of semirings so the builds run in parallel.
#include "gb_spgemm_hash.cuh"

#define SS_DYN(X, Z) gb_sr_dyn<X, Z>
GB_SPGEMM_HASH_INST(SS_DYN(uint32_t, bool), uint32_t, bool)
GB_SPGEMM_HASH_INST(SS_DYN(int64_t, bool), int64_t, bool)
GB_SPGEMM_HASH_INST(SS_DYN(uint64_t, bool), uint64_t, bool)
GB_SPGEMM_HASH_INST(SS_DYN(float, bool), float, bool)
GB_SPGEMM_HASH_INST(SS_DYN(double, bool), double, bool)
