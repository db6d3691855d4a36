// gb_spgemm_hash_p2.hip -- instantiations of the hash Gustavson SpGEMM (gb_spgemm_hash.cuh),
// one file per group of semirings so the builds run in parallel.
#include "gb_spgemm_hash.cuh"

#define SS_DYN(X, Z) gb_sr_dyn<X, Z>
GB_SPGEMM_HASH_INST(SS_DYN(bool, bool), bool, bool)
GB_SPGEMM_HASH_INST(SS_DYN(int8_t, int8_t), int8_t, int8_t)
GB_SPGEMM_HASH_INST(SS_DYN(uint8_t, uint8_t), uint8_t, uint8_t)
GB_SPGEMM_HASH_INST(SS_DYN(int16_t, int16_t), int16_t, int16_t)
