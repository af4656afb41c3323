// lh_lk.h — pyramid level table shared by the LK kernels (lh_lk.hip) and the host side.
#pragma once
#include <stdint.h>

#define LH_LK_MAX_LEVELS 4

struct lh_lk_levels {
    const uint8_t* data[LH_LK_MAX_LEVELS];
    int32_t cols[LH_LK_MAX_LEVELS], rows[LH_LK_MAX_LEVELS];
    int64_t step[LH_LK_MAX_LEVELS];
};
