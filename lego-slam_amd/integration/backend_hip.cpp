// backend_hip.cpp — legoslam::Backend on the MI355X bundle-adjustment library: the drop-in for
// src/backend_lego.cpp.  The reference selects its Backend implementation at link
// time (src/CMakeLists.txt:10-16 lists backend_lego.cpp or backend_g2o.cpp; both implement
// include/legoslam/backend.h:17-60): list this file instead, add lego-slam_amd/integration and include/ to
// the include path and link liblego_ba.so.
//
// Same class, same members, same thread protocol as backend_lego.cpp:
//   * the constructor starts the backend thread (:12-15); UpdateMap notifies it under data_mutex_
//     (:17-20), so the frontend's next keyframe insertion waits while a solve runs, as in the reference;
//   * BackendLoop (:38-54) optimises the active keyframes and landmarks on every notification.  The
//     thread owns one solver handle (lh_backend::ThreadSolver: created when the loop starts, destroyed
//     when it ends; a handle is single-threaded and the frontend thread would own its own);
//   * Optimize (:56-218): window assembly, problem.solve(10) -> lh_solve, the outlier threshold loop,
//     feature flags, RemoveObservation and the write-back, in lh_backend::optimize_window;
//   * Stop (:32-36) also writes the keyframe trajectory (KITTI pose format, T_wc per keyframe) to the file
//     named by LEGO_BA_TRAJECTORY, if set: the reference writes none, and the KITTI-00 comparison needs it.
//
// The reference's headers need Sophus, Eigen, OpenCV and glog (through common_include.h), none of which
// exist in the build image.  The CPU suite compiles this file unchanged against minimal mock headers of
// the legoslam types it touches (tests/mock_legoslam/legoslam/*.h), and the GPU suite links it into a
// driver that runs the Backend thread on a window through those types (tests/backend_hip_driver.cpp,
// tests/test_backend_loop.py).  The KITTI-00 end-to-end run (BASELINE config 5) stays untested: no
// dataset and no reference libraries here.
#include "legoslam/backend.h"

#include <cstdlib>
#include <functional>
#include <memory>

#include "legoslam/algorithm.h"   // toVec2 (backend_lego.cpp includes it too)
#include "legoslam/feature.h"
#include "legoslam/map.h"
#include "legoslam/mappoint.h"
#include "lh_backend.h"

namespace legoslam {

namespace {

// SE3 / Vec3 / cv::KeyPoint <-> the ABI's flat arrays
struct LegoTraits {
    static void pose12(const Frame::Ptr& f, double T[12]) {
        const Mat44 M = f->Pose().matrix();   // T_cw
        for (int r = 0; r < 3; ++r)
            for (int c = 0; c < 4; ++c) T[4 * r + c] = M(r, c);
    }
    static void set_pose(const Frame::Ptr& f, const double T[12]) {
        Mat44 M = Mat44::Identity();
        for (int r = 0; r < 3; ++r)
            for (int c = 0; c < 4; ++c) M(r, c) = T[4 * r + c];
        f->SetPose(SE3(M));   // as SE3(v0.second->getEstimate()), backend_lego.cpp:210
    }
    static void pos(const MapPoint::Ptr& mp, double x[3]) {
        const Vec3 p = mp->Pos();
        x[0] = p[0]; x[1] = p[1]; x[2] = p[2];
    }
    static void set_pos(const MapPoint::Ptr& mp, const double x[3]) { mp->SetPos(Vec3(x[0], x[1], x[2])); }
    static void pixel(const Feature::Ptr& feat, double& u, double& v) {
        const Vec2 z = toVec2(feat->position_.pt);   // algorithm.h:37
        u = z[0];
        v = z[1];
    }
};

void ext12(const SE3& T, double out[12]) {
    const Mat44 M = T.matrix();
    for (int r = 0; r < 3; ++r)
        for (int c = 0; c < 4; ++c) out[4 * r + c] = M(r, c);
}

}  // namespace

Backend::Backend() {
    backend_running_.store(true);
    backend_thread_ = std::thread(std::bind(&Backend::BackendLoop, this));
}

void Backend::UpdateMap() {
    std::unique_lock<std::mutex> lock(data_mutex_);
    map_update_.notify_one();
}

void Backend::Hang() {
    backend_running_.store(false);
    LOG(INFO) << "Backend is hanging. ";
}

void Backend::Restart() {
    backend_running_.store(true);
    LOG(INFO) << "Backend restart.";
}

void Backend::Stop() {
    backend_running_.store(false);
    map_update_.notify_one();
    backend_thread_.join();
    if (const char* path = std::getenv("LEGO_BA_TRAJECTORY")) {
        if (map_ && !lh_backend::write_keyframe_trajectory<LegoTraits>(path, map_->GetAllKeyFrames()))
            LOG(WARNING) << "lego_ba: cannot write " << path;
    }
}

void Backend::BackendLoop() {
    lh_backend::ThreadSolver solver;   // this thread's handle, for every window
    if (solver.status() != LH_OK) LOG(ERROR) << "lego_ba: lh_create: " << lh_strerror(solver.status());
    while (backend_running_.load()) {
        std::unique_lock<std::mutex> lock(data_mutex_);
        map_update_.wait(lock);
        // 1. just optimize active keyframes and landmarks
        Map::KeyframesType kfs_to_opti = map_->GetActiveKeyFrames();
        Map::LandmarksType landmarks_to_opti = map_->GetActiveMapPoints();
        Optimize(kfs_to_opti, landmarks_to_opti);
    }
}

void Backend::Optimize(Map::KeyframesType& keyframes, Map::LandmarksType& landmarks) {
    const Mat33 Km = cam_left_->K();
    const double K[4] = {Km(0, 0), Km(1, 1), Km(0, 2), Km(1, 2)};
    double left[12], right[12];
    ext12(cam_left_->pose(), left);
    ext12(cam_right_->pose(), right);
    lh_backend::Report rep;
    const int st = lh_backend::optimize_window<LegoTraits>(lh_backend::thread_solver(), keyframes, landmarks, K, left,
                                                           right, &rep);
    if (st != LH_OK && st != LH_E_EMPTY) {
        LOG(WARNING) << "lego_ba: " << lh_strerror(st);
        return;
    }
    LOG(INFO) << "Outlier/Inlier in optimization: " << rep.n_outlier << " / " << rep.n_inlier;
}

}  // namespace legoslam
