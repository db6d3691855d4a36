// gb_spgemm_hash_p3.hip -- instantiations of the hash Gustavson SpGEMM (gb_spgemm_hash.cuh),
// one file per group of semirings so the builds run in parallel.
#include "gb_spgemm_hash.cuh"

#define SS_DYN(X, Z) gb_sr_dyn<X, Z>
GB_SPGEMM_HASH_INST(SS_DYN(uint16_t, uint16_t), uint16_t, uint16_t)
GB_SPGEMM_HASH_INST(SS_DYN(int32_t, int32_t), int32_t, int32_t)
GB_SPGEMM_HASH_INST(SS_DYN(uint32_t, uint32_t), uint32_t, uint32_t)
GB_SPGEMM_HASH_INST(SS_DYN(int64_t, int64_t), int64_t, int64_t)
