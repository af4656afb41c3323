// Mock of include/legoslam/mappoint.h (TEST INFRASTRUCTURE): position, outlier flag, observations.
#pragma once
#include "legoslam/common_include.h"

namespace legoslam {
class Feature;
class MapPoint {
  public:
    typedef std::shared_ptr<MapPoint> Ptr;
    unsigned long id_ = 0;
    bool is_outlier_ = false;
    int observed_times_ = 0;
    Vec3 Pos() {
        std::unique_lock<std::mutex> lck(data_mutex_);
        return pos_;
    }
    void SetPos(const Vec3& pos) {
        std::unique_lock<std::mutex> lck(data_mutex_);
        pos_ = pos;
    }
    void AddObservation(std::shared_ptr<Feature> feature) {
        std::unique_lock<std::mutex> lck(data_mutex_);
        observations_.push_back(feature);
        observed_times_++;
    }
    void RemoveObservation(std::shared_ptr<Feature> feat);   // defined after Feature (feature.h)
    std::list<std::weak_ptr<Feature>> GetObs() {
        std::unique_lock<std::mutex> lck(data_mutex_);
        return observations_;
    }

  private:
    Vec3 pos_;
    std::mutex data_mutex_;
    std::list<std::weak_ptr<Feature>> observations_;
};
}  // namespace legoslam
