// abi_caller.cpp — the INTEGRATION.md §3 flow as a compiled C++ caller of the C ABI: what
// Backend::Optimize (src/backend_lego.cpp:56-218) does around the solver once the block :57-161 is
// replaced.  It links liblego_ba.so directly (no ctypes), creates a handle, solves one window from a
// binary file, runs the reference's outlier pass (lh_classify_outliers, :163-194) and writes the
// write-back values (:198-217) to an output file the test compares with the oracle.
//
//   abi_caller <window.bin> <result.bin> [reps]
//
// With reps > 0 the same window is then solved reps more times into the same output buffers (the
// caller's own, as Backend::Optimize keeps them), and the median wall time of one lh_solve is printed:
// the drop-in call's cost as a C++ caller pays it (bench.py's host_buffer_path reports it).
//
// With reps > 0 it also times the call with the outlier pass on the device (lh_result.is_outlier, ABI 5:
// flags instead of the per-edge chi2) and checks those flags against the host pass.
//
// window.bin:  int32 P, int32 L, int64 O, int32 ncam, int32 has_fixed, double K[4],
//              double pose[P][12], uint8 fixed[P] (if has_fixed), double lm[L][3],
//              uint32 obs_pose[O], uint32 obs_lm[O], uint8 obs_cam[O], double obs_uv[O][2],
//              double cam_ext[ncam][12]
// result.bin:  int32 status, int32 iterations, int32 trials, int32 accepted, double chi2_initial,
//              double chi2_final, double chi2_th, int64 n_inlier, int64 n_outlier,
//              double pose[P][12], double lm[L][3], double edge_robust_chi2[O], uint8 is_outlier[O]
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "lego_ba.h"

namespace {
template <typename T>
bool rd(FILE* f, T* p, size_t n) { return n == 0 || fread(p, sizeof(T), n, f) == n; }
template <typename T>
void wr(FILE* f, const T* p, size_t n) { if (n) fwrite(p, sizeof(T), n, f); }
}  // namespace

int main(int argc, char** argv) {
    if (argc != 3 && argc != 4) { fprintf(stderr, "usage: %s window.bin result.bin [reps]\n", argv[0]); return 2; }
    const int reps = argc == 4 ? atoi(argv[3]) : 0;
    FILE* f = fopen(argv[1], "rb");
    if (!f) { perror(argv[1]); return 2; }
    int32_t P = 0, L = 0, ncam = 0, has_fixed = 0;
    int64_t O = 0;
    double K[4];
    bool ok = rd(f, &P, 1) && rd(f, &L, 1) && rd(f, &O, 1) && rd(f, &ncam, 1) && rd(f, &has_fixed, 1) && rd(f, K, 4);
    if (!ok || P < 0 || L < 0 || O < 0 || ncam < 0) { fprintf(stderr, "bad header\n"); return 2; }
    std::vector<double> pose(12 * (size_t)P), lm(3 * (size_t)L), uv(2 * (size_t)O), ext(12 * (size_t)ncam);
    std::vector<uint8_t> fixed(has_fixed ? P : 0), cam(O);
    std::vector<uint32_t> op(O), ol(O);
    ok = rd(f, pose.data(), pose.size()) && rd(f, fixed.data(), fixed.size()) && rd(f, lm.data(), lm.size()) &&
         rd(f, op.data(), op.size()) && rd(f, ol.data(), ol.size()) && rd(f, cam.data(), cam.size()) &&
         rd(f, uv.data(), uv.size()) && rd(f, ext.data(), ext.size());
    fclose(f);
    if (!ok) { fprintf(stderr, "short window file\n"); return 2; }

    // Backend::Backend: one handle, reused for every window
    lh_options opt;
    lh_default_options(&opt);
    opt.device = 0;
    lh_handle* h = nullptr;
    int st = lh_create(&h, &opt);
    if (st != LH_OK) { fprintf(stderr, "lh_create: %s\n", lh_strerror(st)); return 1; }

    lh_window win{};
    win.n_poses = P;
    win.pose_Tcw = pose.data();
    win.pose_fixed = has_fixed ? fixed.data() : nullptr;
    win.n_landmarks = L;
    win.lm_xyz = lm.data();
    win.n_obs = O;
    win.obs_pose = op.data();
    win.obs_lm = ol.data();
    win.obs_cam = cam.data();
    win.obs_uv = uv.data();
    for (int i = 0; i < 4; ++i) win.K[i] = K[i];
    win.n_cams = ncam;
    win.cam_ext = ncam ? ext.data() : nullptr;

    // problem.solve(10) (backend_lego.cpp:161)
    std::vector<double> pose_out(pose.size()), lm_out(lm.size()), rchi2(O);
    lh_result res{};
    res.pose_Tcw = pose_out.data();
    res.lm_xyz = lm_out.data();
    res.edge_robust_chi2 = rchi2.data();
    st = lh_solve(h, &win, &res);
    if (st == LH_OK && reps > 0) {
        std::vector<double> ms;
        for (int i = 0; i < reps && st == LH_OK; ++i) {
            const auto t0 = std::chrono::steady_clock::now();
            st = lh_solve(h, &win, &res);
            ms.push_back(std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count());
        }
        std::sort(ms.begin(), ms.end());
        printf("abi_caller: lh_solve median %.4f ms over %d (min %.4f): prep %.4f upload %.4f solve %.4f download %.4f\n",
               ms[ms.size() / 2], (int)ms.size(), ms[0], res.time_prep_ms, res.time_upload_ms, res.time_ms,
               res.time_download_ms);
        // the same call with the outlier pass on the device (ABI 5): the flags come back instead of the
        // per-edge chi2 (backend_lego.cpp:163-194 as Backend::Optimize runs it, integration/lh_backend.h)
        std::vector<uint8_t> dflag(O);
        lh_result rd5{};
        rd5.pose_Tcw = pose_out.data();
        rd5.lm_xyz = lm_out.data();
        rd5.is_outlier = dflag.data();
        rd5.outlier_chi2_th = 5.991;
        ms.clear();
        for (int i = 0; i < reps && st == LH_OK; ++i) {
            const auto t0 = std::chrono::steady_clock::now();
            st = lh_solve(h, &win, &rd5);
            ms.push_back(std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count());
        }
        if (st == LH_OK) {
            std::sort(ms.begin(), ms.end());
            std::vector<uint8_t> hflag(O);
            double th = 0.0;
            int64_t ni = 0, no = 0;
            lh_classify_outliers(rchi2.data(), O, 5.991, hflag.data(), &th, &ni, &no);
            const bool same = hflag == dflag && th == rd5.outlier_th && ni == rd5.n_inlier && no == rd5.n_outlier;
            printf("abi_caller (device outlier pass): lh_solve median %.4f ms over %d (min %.4f): prep %.4f upload %.4f "
                   "solve %.4f download %.4f; flags %s the host pass\n",
                   ms[ms.size() / 2], (int)ms.size(), ms[0], rd5.time_prep_ms, rd5.time_upload_ms, rd5.time_ms,
                   rd5.time_download_ms, same ? "equal" : "DIFFER from");
            if (!same) st = LH_E_STATE;
        }
    }

    // outlier pass (backend_lego.cpp:163-194)
    std::vector<uint8_t> is_outlier(O);
    double chi2_th = 0.0;
    int64_t n_in = 0, n_out = 0;
    if (st == LH_OK) lh_classify_outliers(rchi2.data(), O, 5.991, is_outlier.data(), &chi2_th, &n_in, &n_out);
    lh_destroy(h);

    FILE* g = fopen(argv[2], "wb");
    if (!g) { perror(argv[2]); return 2; }
    const int32_t hdr[4] = {st, res.iterations, res.trials, res.accepted};
    wr(g, hdr, 4);
    const double sc[3] = {res.chi2_initial, res.chi2_final, chi2_th};
    wr(g, sc, 3);
    const int64_t cnt[2] = {n_in, n_out};
    wr(g, cnt, 2);
    wr(g, pose_out.data(), pose_out.size());
    wr(g, lm_out.data(), lm_out.size());
    wr(g, rchi2.data(), rchi2.size());
    wr(g, is_outlier.data(), is_outlier.size());
    fclose(g);
    printf("abi_caller: status %d (%s), %d iterations, chi2 %.9g -> %.9g, outliers %lld / inliers %lld\n", st,
           lh_strerror(st), res.iterations, res.chi2_initial, res.chi2_final, (long long)n_out, (long long)n_in);
    return st == LH_OK ? 0 : 1;
}
