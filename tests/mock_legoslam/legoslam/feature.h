// Mock of include/legoslam/feature.h (TEST INFRASTRUCTURE): frame / map point links, the key point,
// the outlier and image flags; and MapPoint::RemoveObservation (src/mappoint.cpp semantics: unlink the
// feature from the point and the point from the feature).
#pragma once
#include "legoslam/common_include.h"
#include "legoslam/frame.h"
#include "legoslam/mappoint.h"

namespace legoslam {
class Feature {
  public:
    typedef std::shared_ptr<Feature> Ptr;
    std::weak_ptr<Frame> frame_;
    std::weak_ptr<MapPoint> map_point_;
    cv::KeyPoint position_;
    bool is_outlier_ = false;
    bool is_on_left_image_ = true;
    bool is_on_right_image_ = false;
};

inline void MapPoint::RemoveObservation(std::shared_ptr<Feature> feat) {
    std::unique_lock<std::mutex> lck(data_mutex_);
    for (auto it = observations_.begin(); it != observations_.end(); ++it) {
        if (it->lock() == feat) {
            observations_.erase(it);
            feat->map_point_.reset();
            observed_times_--;
            break;
        }
    }
}
}  // namespace legoslam
