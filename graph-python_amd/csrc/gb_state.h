// gb_state.h -- layout of the persistent device state words (zeroed once per
// process by gb_device_state(); every user leaves its words as it found them).
#pragma once

#define GB_GRID_SHARDS 32
#define GB_GRID_STRIDE 32  // u64 words between counters (256 B)
#define GB_GRID_STATE_WORDS ((GB_GRID_SHARDS + 1) * GB_GRID_STRIDE)
#define GB_DIR_STATE_OFFSET GB_GRID_STATE_WORDS  // SpMV direction state (gb_mxv.hip)
#define GB_GRID2_OFFSET (GB_GRID_STATE_WORDS + 32)  // a second grid-sum area (two sums in one kernel)
#define GB_GRID3_OFFSET (GB_GRID2_OFFSET + GB_GRID_STATE_WORDS)  // a third one
#define GB_STATE_WORDS (GB_GRID3_OFFSET + GB_GRID_STATE_WORDS)
#define GB_HINT_PARTS GB_GRID_SHARDS  // parts of a vector's next-frontier edge hint (d_nvals[2..])
