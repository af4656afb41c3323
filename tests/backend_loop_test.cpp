// backend_loop_test.cpp — the MI355X legoslam::Backend (lego-slam_amd/integration/backend_hip.cpp) as far as
// it can run without the reference's headers: lh_backend.h's Optimize and trajectory writer on stand-in
// SLAM types (frames, map points, features with the member names Backend::Optimize uses), driven by a
// backend thread with the reference's protocol (backend_lego.cpp:12-54: a condition variable under the
// data mutex, one solver handle owned by the thread).  Two keyframe notifications: the first window from
// a file, the second the written-back state with the first pass's outliers removed.
//
//   backend_loop_test <window.bin> <result.bin> <trajectory.txt>
//
// window.bin as tests/abi_caller.cpp (pose_fixed ignored: the Backend fixes no vertex).  result.bin:
//   int32 status, iterations, trials;  int64 n_edges, n_inlier, n_outlier;  double chi2_initial,
//   chi2_final, chi2_th;  double pose[P][12], lm[L][3];  uint8 is_outlier[O] (window order);
//   int32 status2, iterations2;  int64 n_edges2;  double chi2_initial2, chi2_final2
#include <condition_variable>
#include <cstdio>
#include <list>
#include <map>
#include <memory>
#include <mutex>
#include <thread>
#include <unordered_map>
#include <vector>

#include "lh_backend.h"

namespace {

struct MapPoint;
struct Frame {
    unsigned long keyframe_id_ = 0;
    double T[12];   // T_cw, row-major [R | t]
};
struct Feature {
    std::weak_ptr<Frame> frame_;
    std::weak_ptr<MapPoint> map_point_;
    float px = 0.f, py = 0.f;   // cv::KeyPoint::pt
    bool is_outlier_ = false, is_on_left_image_ = true, is_on_right_image_ = false;
};
struct MapPoint {
    unsigned long id_ = 0;
    bool is_outlier_ = false;
    double pos[3];
    std::list<std::weak_ptr<Feature>> obs;
    std::list<std::weak_ptr<Feature>> GetObs() { return obs; }
    void RemoveObservation(std::shared_ptr<Feature> feat) {   // mappoint.cpp:16-27
        for (auto it = obs.begin(); it != obs.end(); ++it)
            if (it->lock() == feat) {
                obs.erase(it);
                feat->map_point_.reset();
                break;
            }
    }
};
using FramePtr = std::shared_ptr<Frame>;
using MapPointPtr = std::shared_ptr<MapPoint>;
using FeaturePtr = std::shared_ptr<Feature>;

struct Traits {
    static void pose12(const FramePtr& f, double T[12]) { std::copy(f->T, f->T + 12, T); }
    static void set_pose(const FramePtr& f, const double T[12]) { std::copy(T, T + 12, f->T); }
    static void pos(const MapPointPtr& m, double x[3]) { std::copy(m->pos, m->pos + 3, x); }
    static void set_pos(const MapPointPtr& m, const double x[3]) { std::copy(x, x + 3, m->pos); }
    static void pixel(const FeaturePtr& f, double& u, double& v) { u = f->px; v = f->py; }
};

template <typename T>
bool rd(FILE* f, T* p, size_t n) { return n == 0 || fread(p, sizeof(T), n, f) == n; }
template <typename T>
void wr(FILE* f, const T* p, size_t n) { if (n) fwrite(p, sizeof(T), n, f); }

// the backend thread (backend_lego.cpp:12-54), with a job count instead of the active-window copies
struct BackendThread {
    std::mutex data_mutex_;
    std::condition_variable map_update_;
    bool pending_ = false, stop_ = false;
    int done_ = 0;
    std::condition_variable done_cv_;
    std::thread thread_;
    template <class Job>
    void start(Job job) {
        thread_ = std::thread([this, job]() {
            lh_backend::ThreadSolver solver;   // the thread's handle for every window
            std::unique_lock<std::mutex> lock(data_mutex_);
            for (;;) {
                map_update_.wait(lock, [this] { return pending_ || stop_; });
                if (stop_) break;
                pending_ = false;
                job(solver.status());
                ++done_;
                done_cv_.notify_all();
            }
        });
    }
    void update_map_and_wait(int n) {   // Backend::UpdateMap, then wait for that solve
        std::unique_lock<std::mutex> lock(data_mutex_);
        pending_ = true;
        map_update_.notify_one();
        done_cv_.wait(lock, [this, n] { return done_ >= n; });
    }
    void stop() {
        {
            std::unique_lock<std::mutex> lock(data_mutex_);
            stop_ = true;
            map_update_.notify_one();
        }
        thread_.join();
    }
};

}  // namespace

int main(int argc, char** argv) {
    if (argc != 4) { fprintf(stderr, "usage: %s window.bin result.bin trajectory.txt\n", argv[0]); return 2; }
    FILE* f = fopen(argv[1], "rb");
    if (!f) { perror(argv[1]); return 2; }
    int32_t P = 0, L = 0, ncam = 0, has_fixed = 0;
    int64_t O = 0;
    double K[4];
    bool ok = rd(f, &P, 1) && rd(f, &L, 1) && rd(f, &O, 1) && rd(f, &ncam, 1) && rd(f, &has_fixed, 1) && rd(f, K, 4);
    if (!ok || P < 1 || L < 0 || O < 0 || ncam < 1 || ncam > 2) { fprintf(stderr, "bad header\n"); return 2; }
    std::vector<double> pose(12 * (size_t)P), lm(3 * (size_t)L), uv(2 * (size_t)O), ext(12 * (size_t)ncam);
    std::vector<uint8_t> fixed(has_fixed ? P : 0), cam(O);
    std::vector<uint32_t> op(O), ol(O);
    ok = rd(f, pose.data(), pose.size()) && rd(f, fixed.data(), fixed.size()) && rd(f, lm.data(), lm.size()) &&
         rd(f, op.data(), op.size()) && rd(f, ol.data(), ol.size()) && rd(f, cam.data(), cam.size()) &&
         rd(f, uv.data(), uv.size()) && rd(f, ext.data(), ext.size());
    fclose(f);
    if (!ok) { fprintf(stderr, "short window file\n"); return 2; }
    double right[12];
    std::copy(ext.begin() + (ncam > 1 ? 12 : 0), ext.begin() + (ncam > 1 ? 24 : 12), right);

    // the map: keyframe ids 10, 13, 16, ... (Map::KeyframesType, a std::map), landmark ids 7 l + 2 in an
    // unordered_map (Map::LandmarksType), one feature per observation in window order
    std::map<unsigned long, FramePtr> keyframes;
    std::vector<FramePtr> frames(P);
    for (int p = 0; p < P; ++p) {
        frames[p] = std::make_shared<Frame>();
        frames[p]->keyframe_id_ = 10 + 3 * (unsigned long)p;
        std::copy(&pose[12 * p], &pose[12 * p] + 12, frames[p]->T);
        keyframes[frames[p]->keyframe_id_] = frames[p];
    }
    std::unordered_map<unsigned long, MapPointPtr> landmarks;
    std::vector<MapPointPtr> points(L);
    for (int l = 0; l < L; ++l) {
        points[l] = std::make_shared<MapPoint>();
        points[l]->id_ = 7 * (unsigned long)l + 2;
        std::copy(&lm[3 * l], &lm[3 * l] + 3, points[l]->pos);
        landmarks[points[l]->id_] = points[l];
    }
    std::vector<FeaturePtr> feats(O);
    for (int64_t o = 0; o < O; ++o) {
        auto ft = std::make_shared<Feature>();
        ft->frame_ = frames[op[o]];
        ft->map_point_ = points[ol[o]];
        ft->px = (float)uv[2 * o];   // the window's pixels are float-valued
        ft->py = (float)uv[2 * o + 1];
        ft->is_on_left_image_ = cam[o] == 0;
        ft->is_on_right_image_ = cam[o] == 1;
        points[ol[o]]->obs.push_back(ft);
        feats[o] = ft;
    }

    lh_backend::Report rep[2];
    int job_status[2] = {LH_E_STATE, LH_E_STATE};
    int njob = 0;
    std::vector<double> pose1, lm1;
    std::vector<uint8_t> out1(O);
    BackendThread bt;
    bt.start([&](int create_status) {
        const int j = njob++;
        if (create_status != LH_OK) { job_status[j] = create_status; return; }
        job_status[j] = lh_backend::optimize_window<Traits>(lh_backend::thread_solver(), keyframes, landmarks, K,
                                                            ext.data(), right, &rep[j]);
        if (j == 0) {   // the write-back values of the first window
            for (int p = 0; p < P; ++p) pose1.insert(pose1.end(), frames[p]->T, frames[p]->T + 12);
            for (int l = 0; l < L; ++l) lm1.insert(lm1.end(), points[l]->pos, points[l]->pos + 3);
            for (int64_t o = 0; o < O; ++o) out1[o] = feats[o]->is_outlier_ ? 1 : 0;
        }
    });
    bt.update_map_and_wait(1);
    bt.update_map_and_wait(2);
    bt.stop();
    const bool traj = lh_backend::write_keyframe_trajectory<Traits>(argv[3], keyframes);

    FILE* g = fopen(argv[2], "wb");
    if (!g) { perror(argv[2]); return 2; }
    const int32_t h1[3] = {job_status[0], rep[0].iterations, rep[0].trials};
    wr(g, h1, 3);
    const int64_t c1[3] = {rep[0].n_edges, rep[0].n_inlier, rep[0].n_outlier};
    wr(g, c1, 3);
    const double s1[3] = {rep[0].chi2_initial, rep[0].chi2_final, rep[0].chi2_th};
    wr(g, s1, 3);
    pose1.resize(12 * (size_t)P);
    lm1.resize(3 * (size_t)L);
    wr(g, pose1.data(), pose1.size());
    wr(g, lm1.data(), lm1.size());
    wr(g, out1.data(), out1.size());
    const int32_t h2[2] = {job_status[1], rep[1].iterations};
    wr(g, h2, 2);
    const int64_t c2[1] = {rep[1].n_edges};
    wr(g, c2, 1);
    const double s2[2] = {rep[1].chi2_initial, rep[1].chi2_final};
    wr(g, s2, 2);
    fclose(g);
    printf("backend_loop_test: windows %d/%d, edges %lld -> %lld, chi2 %.9g -> %.9g, then %.9g -> %.9g, "
           "outliers %lld, trajectory %s\n", job_status[0], job_status[1], (long long)rep[0].n_edges,
           (long long)rep[1].n_edges, rep[0].chi2_initial, rep[0].chi2_final, rep[1].chi2_initial, rep[1].chi2_final,
           (long long)rep[0].n_outlier, traj ? "ok" : "failed");
    return (job_status[0] == LH_OK && job_status[1] == LH_OK && traj) ? 0 : 1;
}
