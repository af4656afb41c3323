// Mock of include/legoslam/common_include.h for compiling integration/backend_hip.cpp unchanged without
// Eigen, Sophus, OpenCV or glog (none are in this image).  TEST INFRASTRUCTURE: only the members
// backend_hip.cpp touches, with the reference's names and value semantics; nothing here is product code.
#pragma once

#include <atomic>
#include <condition_variable>
#include <functional>
#include <iostream>
#include <list>
#include <map>
#include <memory>
#include <mutex>
#include <set>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#define EIGEN_MAKE_ALIGNED_OPERATOR_NEW static_assert(true, "")

// a fixed-size, row-major double matrix with the Eigen calls the backend makes: (r, c), [i], Identity
template <int R, int C>
struct MockMat {
    double a[R * C] = {};
    MockMat() = default;
    template <class... T, class = typename std::enable_if<sizeof...(T) == R * C && (R == 1 || C == 1)>::type>
    MockMat(T... v) : a{static_cast<double>(v)...} {}
    double& operator()(int r, int c) { return a[r * C + c]; }
    double operator()(int r, int c) const { return a[r * C + c]; }
    double& operator[](int i) { return a[i]; }
    double operator[](int i) const { return a[i]; }
    static MockMat Identity() {
        MockMat m;
        for (int i = 0; i < (R < C ? R : C); ++i) m(i, i) = 1.0;
        return m;
    }
    static MockMat Zero() { return MockMat(); }
};
typedef MockMat<4, 4> Mat44;
typedef MockMat<3, 3> Mat33;
typedef MockMat<3, 1> Vec3;
typedef MockMat<2, 1> Vec2;

// Sophus::SE3d as the backend uses it: built from a 4x4 (SE3(Mat4), backend_lego.cpp:210) and read back
// with matrix()
class SE3 {
  public:
    SE3() : m_(Mat44::Identity()) {}
    explicit SE3(const Mat44& m) : m_(m) { m_(3, 0) = m_(3, 1) = m_(3, 2) = 0.0; m_(3, 3) = 1.0; }
    Mat44 matrix() const { return m_; }

  private:
    Mat44 m_;
};

namespace cv {
struct Point2f {
    float x = 0.f, y = 0.f;
};
struct KeyPoint {
    Point2f pt;
};
}  // namespace cv

// glog's LOG(severity) << ...: to stderr
struct MockLog {
    explicit MockLog(const char* sev) { std::cerr << "[" << sev << "] "; }
    ~MockLog() { std::cerr << std::endl; }
    template <class T>
    MockLog& operator<<(const T& v) {
        std::cerr << v;
        return *this;
    }
};
#define LOG(sev) MockLog(#sev)
