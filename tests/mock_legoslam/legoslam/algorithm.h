// Mock of include/legoslam/algorithm.h (TEST INFRASTRUCTURE): toVec2 only.
#pragma once
#include "legoslam/common_include.h"

namespace legoslam {
inline Vec2 toVec2(const cv::Point2f& p) { return Vec2{p.x, p.y}; }
}  // namespace legoslam
