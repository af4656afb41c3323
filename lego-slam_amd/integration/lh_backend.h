// lh_backend.h — the logic of the MI355X legoslam::Backend (integration/backend_hip.cpp), independent of
// the SLAM types so that it compiles, and is tested, without the reference's headers.
//
// Backend::Optimize (src/backend_lego.cpp:56-218) around the C ABI (include/lego_ba.h):
//   * the window: every keyframe becomes a pose (ascending keyframe id, Map::KeyframesType is a
//     std::map, map.h:21); landmarks in ascending id (Map::LandmarksType is an unordered_map, map.h:19,
//     so the ids are sorted: Problem::setOrdering orders the landmark vertices by id,
//     problem.cpp:234-255); a landmark that is not an outlier becomes a vertex on its first edge
//     (:126-133); one edge per observation whose feature is live, not an outlier, on a live frame,
//     and on exactly one image (left -> camera 0, right -> camera 1, :101-124);
//   * problem.solve(10) (:161) -> lh_solve;
//   * the outlier threshold loop (:163-194) -> lh_result.is_outlier (the loop on the device), then the feature flags and
//     MapPoint::RemoveObservation for the outliers (:186-194);
//   * the write-back of every pose and landmark vertex (:198-217).
// The SLAM types enter through a traits class (pose / position / pixel conversions: Sophus and Eigen in
// the reference, plain arrays in tests/backend_loop_test.cpp) and through the member names Optimize
// itself uses: Frame::keyframe_id_, MapPoint::{id_, is_outlier_, GetObs(), RemoveObservation()},
// Feature::{frame_, map_point_, is_outlier_, is_on_left_image_, is_on_right_image_}.
//
// One handle per thread (lego_ba.h): ThreadSolver creates the backend thread's handle when the thread
// starts and destroys it when the thread ends; thread_solver() returns it to Optimize.
#pragma once

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <memory>
#include <unordered_map>
#include <vector>

#include "lego_ba.h"

namespace lh_backend {

// What one Optimize call did (the reference logs the outlier counts, backend_lego.cpp:196).
struct Report {
    int status = LH_OK;
    int iterations = 0, trials = 0;
    double chi2_initial = 0.0, chi2_final = 0.0, chi2_th = 0.0;
    int64_t n_poses = 0, n_landmarks = 0, n_edges = 0, n_inlier = 0, n_outlier = 0;
};

inline lh_handle*& thread_solver_slot() {
    static thread_local lh_handle* h = nullptr;
    return h;
}
inline lh_handle* thread_solver() { return thread_solver_slot(); }

// The backend thread's solver handle for the lifetime of the thread (BackendLoop's scope).  The device
// is LEGO_BA_DEVICE (default: the current HIP device).
class ThreadSolver {
public:
    explicit ThreadSolver(const lh_options* opt = nullptr) {
        lh_options o;
        if (opt) {
            o = *opt;
        } else {
            lh_default_options(&o);
            if (const char* d = std::getenv("LEGO_BA_DEVICE")) o.device = std::atoi(d);
        }
        status_ = lh_create(&h_, &o);
        if (status_ != LH_OK) h_ = nullptr;
        thread_solver_slot() = h_;
    }
    ~ThreadSolver() {
        thread_solver_slot() = nullptr;
        lh_destroy(h_);
    }
    ThreadSolver(const ThreadSolver&) = delete;
    ThreadSolver& operator=(const ThreadSolver&) = delete;
    int status() const { return status_; }
    lh_handle* get() const { return h_; }

private:
    lh_handle* h_ = nullptr;
    int status_ = LH_OK;
};

// Backend::Optimize(keyframes, landmarks) on handle h.  K = {fx, fy, cx, cy}; ext12: the left and right
// cameras' extrinsics (Camera::pose(), row-major [R | t]).  Returns an lh_status; on an error nothing is
// written back (LH_E_EMPTY is the reference's solve() returning false on an empty problem, after
// which it still runs the outlier pass and write-back on no edges: nothing changes either way).
template <class Traits, class KeyframesT, class LandmarksT>
int optimize_window(lh_handle* h, KeyframesT& keyframes, LandmarksT& landmarks, const double K[4],
                    const double left_ext12[12], const double right_ext12[12], Report* rep = nullptr,
                    double chi2_th0 = 5.991) {
    Report r;
    if (!h) {
        r.status = LH_E_STATE;
        if (rep) *rep = r;
        return r.status;
    }
    // ---- poses: every keyframe, ascending id (backend_lego.cpp:67-79) ----
    std::vector<unsigned long> kf_ids;
    std::unordered_map<unsigned long, uint32_t> kf_index;
    std::vector<double> pose12;
    kf_ids.reserve(keyframes.size());
    pose12.reserve(12 * keyframes.size());
    for (auto& kv : keyframes) {
        kf_index[kv.second->keyframe_id_] = (uint32_t)kf_ids.size();
        kf_ids.push_back(kv.first);
        double T[12];
        Traits::pose12(kv.second, T);
        pose12.insert(pose12.end(), T, T + 12);
    }
    // ---- landmarks (ascending id) and their edges (backend_lego.cpp:98-158) ----
    std::vector<unsigned long> ids;
    ids.reserve(landmarks.size());
    for (auto& kv : landmarks) ids.push_back(kv.first);
    std::sort(ids.begin(), ids.end());
    std::vector<unsigned long> lm_ids;
    std::vector<double> xyz;
    std::vector<uint32_t> obs_pose, obs_lm;
    std::vector<uint8_t> obs_cam;
    std::vector<double> obs_uv;
    using FeaturePtr = decltype(landmarks.begin()->second->GetObs().begin()->lock());
    std::vector<FeaturePtr> obs_feature;   // edge -> feature, for the outlier pass
    for (const unsigned long id : ids) {
        auto& mp = landmarks.at(id);
        if (mp->is_outlier_) continue;
        int32_t li = -1;
        for (auto& wk : mp->GetObs()) {
            auto feat = wk.lock();
            if (!feat) continue;
            auto frame = feat->frame_.lock();
            if (feat->is_outlier_ || !frame) continue;
            uint8_t cam;
            if (feat->is_on_left_image_ && !feat->is_on_right_image_) cam = 0;         // EdgeProjection(K, left_ext)
            else if (feat->is_on_right_image_ && !feat->is_on_left_image_) cam = 1;    // EdgeProjection(K, right_ext)
            else continue;
            const auto it = kf_index.find(frame->keyframe_id_);
            if (it == kf_index.end()) continue;   // the reference's vertices.at() would throw: not a window pose
            if (li < 0) {
                li = (int32_t)lm_ids.size();
                lm_ids.push_back(id);
                double x[3];
                Traits::pos(mp, x);
                xyz.insert(xyz.end(), x, x + 3);
            }
            double u, v;
            Traits::pixel(feat, u, v);   // toVec2 (algorithm.h:37): the float pixel widened
            obs_pose.push_back(it->second);
            obs_lm.push_back((uint32_t)li);
            obs_cam.push_back(cam);
            obs_uv.push_back(u);
            obs_uv.push_back(v);
            obs_feature.push_back(feat);
        }
    }
    double ext[24];
    std::copy(left_ext12, left_ext12 + 12, ext);
    std::copy(right_ext12, right_ext12 + 12, ext + 12);
    lh_window win{};
    win.n_poses = (int32_t)kf_ids.size();
    win.pose_Tcw = pose12.data();
    win.pose_fixed = nullptr;   // the reference fixes no vertex
    win.n_landmarks = (int32_t)lm_ids.size();
    win.lm_xyz = xyz.data();
    win.n_obs = (int64_t)obs_pose.size();
    win.obs_pose = obs_pose.data();
    win.obs_lm = obs_lm.data();
    win.obs_cam = obs_cam.data();
    win.obs_uv = obs_uv.data();
    for (int i = 0; i < 4; ++i) win.K[i] = K[i];
    win.n_cams = 2;
    win.cam_ext = ext;
    r.n_poses = win.n_poses;
    r.n_landmarks = win.n_landmarks;
    r.n_edges = win.n_obs;

    // ---- problem.solve(10) (:161) ----
    // ---- and the outlier pass (:163-194) on the device: only the flags come back (ABI 5) ----
    std::vector<double> pose_out(pose12.size()), xyz_out(xyz.size());
    std::vector<uint8_t> is_outlier(obs_pose.size());
    lh_result res{};
    res.pose_Tcw = pose_out.data();
    res.lm_xyz = xyz_out.data();
    res.is_outlier = is_outlier.data();
    res.outlier_chi2_th = chi2_th0;
    r.status = lh_solve(h, &win, &res);
    if (r.status != LH_OK) {
        if (rep) *rep = r;
        return r.status;
    }
    r.iterations = res.iterations;
    r.trials = res.trials;
    r.chi2_initial = res.chi2_initial;
    r.chi2_final = res.chi2_final;

    // ---- outliers (:163-194): the threshold loop ran on the device; the features' flags here ----
    r.chi2_th = res.outlier_th;
    r.n_inlier = res.n_inlier;
    r.n_outlier = res.n_outlier;
    for (size_t e = 0; e < obs_feature.size(); ++e) {
        auto& feat = obs_feature[e];
        if (is_outlier[e]) {
            feat->is_outlier_ = true;
            if (auto mp = feat->map_point_.lock()) mp->RemoveObservation(feat);
        } else {
            feat->is_outlier_ = false;
        }
    }
    // ---- write-back (:198-217) ----
    for (size_t i = 0; i < kf_ids.size(); ++i) Traits::set_pose(keyframes.at(kf_ids[i]), &pose_out[12 * i]);
    for (size_t i = 0; i < lm_ids.size(); ++i) Traits::set_pos(landmarks.at(lm_ids[i]), &xyz_out[3 * i]);
    if (rep) *rep = r;
    return LH_OK;
}

// The keyframe trajectory in the KITTI pose format the evaluation tools read: one line per keyframe,
// ascending id, "id r00 r01 r02 t0 r10 r11 r12 t1 r20 r21 r22 t2" of T_wc = T_cw^-1 (the reference stores
// T_cw, Frame::Pose, frame.h:49; it writes no trajectory, visual_odometry.cpp:46-70).
template <class Traits, class KeyframesT>
bool write_keyframe_trajectory(const char* path, const KeyframesT& keyframes) {
    FILE* f = std::fopen(path, "w");
    if (!f) return false;
    std::vector<std::pair<unsigned long, const typename KeyframesT::mapped_type*>> kfs;
    for (auto& kv : keyframes) kfs.emplace_back(kv.first, &kv.second);
    std::sort(kfs.begin(), kfs.end(), [](const auto& a, const auto& b) { return a.first < b.first; });
    for (auto& kv : kfs) {
        double T[12];
        Traits::pose12(*kv.second, T);
        double W[12];   // [R^T | -R^T t]
        for (int i = 0; i < 3; ++i) {
            for (int j = 0; j < 3; ++j) W[4 * i + j] = T[4 * j + i];
            W[4 * i + 3] = -(T[i] * T[3] + T[4 + i] * T[7] + T[8 + i] * T[11]);
        }
        std::fprintf(f, "%lu", kv.first);
        for (int k = 0; k < 12; ++k) std::fprintf(f, " %.12e", W[k]);
        std::fprintf(f, "\n");
    }
    return std::fclose(f) == 0;
}

}  // namespace lh_backend
