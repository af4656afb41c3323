// Mock of include/legoslam/backend.h (TEST INFRASTRUCTURE): the Backend class declaration
// backend_hip.cpp defines (same public and private members as the reference header).
#pragma once
#include "legoslam/common_include.h"
#include "legoslam/frame.h"
#include "legoslam/map.h"

namespace legoslam {
class Map;
class Backend {
  public:
    EIGEN_MAKE_ALIGNED_OPERATOR_NEW;
    typedef std::shared_ptr<Backend> Ptr;
    Backend();
    void SetCameras(Camera::Ptr left, Camera::Ptr right) {
        cam_left_ = left;
        cam_right_ = right;
    }
    void SetMap(Map::Ptr map) { map_ = map; }
    void UpdateMap();
    void Hang();
    void Restart();
    void Stop();

  private:
    void BackendLoop();
    void Optimize(Map::KeyframesType& keyframes, Map::LandmarksType& landmarks);
    Map::Ptr map_ = nullptr;
    std::thread backend_thread_;
    std::mutex data_mutex_;
    std::condition_variable map_update_;
    std::atomic<bool> backend_running_{};
    Camera::Ptr cam_left_ = nullptr, cam_right_ = nullptr;
};
}  // namespace legoslam
