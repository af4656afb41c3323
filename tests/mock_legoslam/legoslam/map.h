// Mock of include/legoslam/map.h (TEST INFRASTRUCTURE): keyframes (std::map by id) and landmarks
// (unordered_map by id); every inserted element is active.
#pragma once
#include "legoslam/common_include.h"
#include "legoslam/frame.h"
#include "legoslam/mappoint.h"

namespace legoslam {
class Map {
  public:
    typedef std::shared_ptr<Map> Ptr;
    typedef std::unordered_map<unsigned long, MapPoint::Ptr> LandmarksType;
    typedef std::map<unsigned long, Frame::Ptr> KeyframesType;
    void InsertKeyFrame(Frame::Ptr frame) {
        std::unique_lock<std::mutex> lck(data_mutex_);
        keyframes_[frame->keyframe_id_] = frame;
    }
    void InsertMapPoint(MapPoint::Ptr mp) {
        std::unique_lock<std::mutex> lck(data_mutex_);
        landmarks_[mp->id_] = mp;
    }
    LandmarksType GetActiveMapPoints() {   // BackendLoop reads the window here, once per pass
        const int pass = optimize_calls_.fetch_add(1);
        if (on_pass) on_pass(pass);
        std::unique_lock<std::mutex> lck(data_mutex_);
        return landmarks_;
    }
    KeyframesType GetActiveKeyFrames() {
        std::unique_lock<std::mutex> lck(data_mutex_);
        return keyframes_;
    }
    KeyframesType GetAllKeyFrames() {
        std::unique_lock<std::mutex> lck(data_mutex_);
        return keyframes_;
    }
    // mock only: backend loop passes that read the window, and a hook called at the start of each pass
    // (pass k > 0 sees the state pass k - 1 wrote back)
    std::atomic<int> optimize_calls_{0};
    std::function<void(int)> on_pass;

  private:
    std::mutex data_mutex_;
    LandmarksType landmarks_;
    KeyframesType keyframes_;
};
}  // namespace legoslam
