// Mock of include/legoslam/camera.h (TEST INFRASTRUCTURE): intrinsics K() and extrinsics pose().
#pragma once
#include "legoslam/common_include.h"

namespace legoslam {
class Camera {
  public:
    typedef std::shared_ptr<Camera> Ptr;
    double fx_ = 0, fy_ = 0, cx_ = 0, cy_ = 0, baseline_ = 0;
    SE3 pose_;
    Camera(double fx, double fy, double cx, double cy, double baseline, const SE3& pose)
        : fx_(fx), fy_(fy), cx_(cx), cy_(cy), baseline_(baseline), pose_(pose) {}
    SE3 pose() const { return pose_; }
    Mat33 K() const {
        Mat33 k;
        k(0, 0) = fx_; k(0, 2) = cx_; k(1, 1) = fy_; k(1, 2) = cy_; k(2, 2) = 1.0;
        return k;
    }
};
}  // namespace legoslam
