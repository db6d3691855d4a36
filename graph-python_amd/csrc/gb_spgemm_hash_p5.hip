// gb_spgemm_hash_p5.hip -- instantiations of the hash Gustavson SpGEMM (gb_spgemm_hash.cuh),
// one file per group of semirings so the builds run in parallel.
#include "gb_spgemm_hash.cuh"

#define SS_DYN(X, Z) gb_sr_dyn<X, Z>
GB_SPGEMM_HASH_INST(SS_DYN(bool, bool), bool, bool)
GB_SPGEMM_HASH_INST(SS_DYN(int8_t, bool), int8_t, bool)
GB_SPGEMM_HASH_INST(SS_DYN(uint8_t, bool), uint8_t, bool)
GB_SPGEMM_HASH_INST(SS_DYN(int16_t, bool), int16_t, bool)
GB_SPGEMM_HASH_INST(SS_DYN(uint16_t, bool), uint16_t, bool)
GB_SPGEMM_HASH_INST(SS_DYN(int32_t, bool), int32_t, bool)
