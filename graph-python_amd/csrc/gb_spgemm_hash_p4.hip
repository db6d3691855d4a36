// gb_spgemm_hash_p4.hip -- instantiations of the hash Gustavson SpGEMM (gb_spgemm_hash.cuh),
// one file per group of semirings so the builds run in parallel.
#include "gb_spgemm_hash.cuh"

#define SS_DYN(X, Z) gb_sr_dyn<X, Z>
GB_SPGEMM_HASH_INST(SS_DYN(uint64_t, uint64_t), uint64_t, uint64_t)
GB_SPGEMM_HASH_INST(SS_DYN(float, float), float, float)
GB_SPGEMM_HASH_INST(SS_DYN(double, double), double, double)
