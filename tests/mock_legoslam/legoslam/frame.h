// Mock of include/legoslam/frame.h (TEST INFRASTRUCTURE): keyframe id and the T_cw pose.
#pragma once
#include "legoslam/camera.h"
#include "legoslam/common_include.h"

namespace legoslam {
class Frame {
  public:
    typedef std::shared_ptr<Frame> Ptr;
    unsigned long id_ = 0, keyframe_id_ = 0;
    SE3 Pose() {
        std::unique_lock<std::mutex> lck(pose_mutex_);
        return pose_;
    }
    void SetPose(const SE3& pose) {
        std::unique_lock<std::mutex> lck(pose_mutex_);
        pose_ = pose;
    }

  private:
    SE3 pose_;
    std::mutex pose_mutex_;
};
}  // namespace legoslam
