// gdf_objects.hpp - the object layer the ROS component reads from the engine after
// objectSegmentation / objectTracking (include/gpu_depthmap_fusion/gpu_depthmap_fusion.h:31-156 and
// filter/*.h of xaedes/ros_gpu_depthmap_fusion): CCObject with its contours and minimal shapes,
// the tracks (CCObjectTrack, CCObjectTrackComparison) with their gain filters, and the
// association step objectTracking (src/gpu_depthmap_fusion.cpp:2579-2944).  Host code: a few
// hundred objects per frame; the per-voxel work before it (labels, stats, contours, layer
// connections, label merge, object aggregates) runs on the GPU (gdf_segment.h).
//
// Geometry types: with GDF_WITH_OPENCV defined (the ROS build, where OpenCV is present) they are
// OpenCV's own (cv::Point2f, cv::RotatedRect, cv::Mat_) and the shapes come from cv::minAreaRect
// / cv::minEnclosingCircle - the reference's exact calls.  Without OpenCV, plain structs with the
// same member names and a restatement of OpenCV 4.2's algorithms (convex hull, rotating calipers,
// the iterative enclosing circle): parity of those two shapes with OpenCV is unpinned here (no
// OpenCV in this image), everything else follows the reference's arithmetic.
#pragma once

#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstdint>
#include <cstdlib>
#include <vector>

#ifdef GDF_WITH_OPENCV
#include <opencv2/core.hpp>
#include <opencv2/imgproc.hpp>
#endif

namespace gdf {

#ifdef GDF_WITH_OPENCV
using Point = cv::Point;
using Point2f = cv::Point2f;
using Size2f = cv::Size2f;
using RotatedRect = cv::RotatedRect;
template <class T>
using Mat_ = cv::Mat_<T>;
inline double norm(const Point2f& p) { return cv::norm(p); }
#else
struct Point {  // cv::Point
    int x = 0, y = 0;
};
struct Point2f {  // cv::Point2f
    float x = 0, y = 0;
    Point2f() = default;
    Point2f(float x_, float y_) : x(x_), y(y_) {}
    Point2f operator-(const Point2f& o) const { return Point2f(x - o.x, y - o.y); }
    Point2f operator+(const Point2f& o) const { return Point2f(x + o.x, y + o.y); }
};
struct Size2f {  // cv::Size2f
    float width = 0, height = 0;
    Size2f() = default;
    Size2f(float w, float h) : width(w), height(h) {}
    float area() const { return width * height; }
};
// cv::norm(Point_): sqrt in double of the float coordinates
inline double norm(const Point2f& p) { return std::sqrt((double)p.x * p.x + (double)p.y * p.y); }
struct RotatedRect {  // cv::RotatedRect
    Point2f center;
    Size2f size;
    float angle = 0;
    RotatedRect() = default;
    RotatedRect(const Point2f& c, const Size2f& s, float a) : center(c), size(s), angle(a) {}
    // cv::RotatedRect::points: bottomLeft, topLeft, topRight, bottomRight (angle 0, y down)
    template <class P>
    void points(P pts[]) const {
        const double a = angle * M_PI / 180.;
        const float b = (float)std::cos(a) * 0.5f;
        const float s = (float)std::sin(a) * 0.5f;
        pts[0].x = center.x - s * size.height - b * size.width;
        pts[0].y = center.y + b * size.height - s * size.width;
        pts[1].x = center.x + s * size.height - b * size.width;
        pts[1].y = center.y - b * size.height - s * size.width;
        pts[2].x = 2 * center.x - pts[0].x;
        pts[2].y = 2 * center.y - pts[0].y;
        pts[3].x = 2 * center.x - pts[1].x;
        pts[3].y = 2 * center.y - pts[1].y;
    }
};
// cv::Mat_ view: rows x cols elements at data (row-major, not owned)
template <class T>
struct Mat_ {
    int rows = 0, cols = 0;
    T* data = nullptr;
    Mat_() = default;
    Mat_(int r, int c, T* d) : rows(r), cols(c), data(d) {}
    T& operator()(int r, int c) const { return data[(size_t)r * cols + c]; }
    template <class U>
    U& at(int r, int c) const { return reinterpret_cast<U*>(data)[(size_t)r * cols + c]; }
};
#endif

struct vec3 {  // glm::vec3
    float x = 0, y = 0, z = 0;
    vec3() = default;
    vec3(float a, float b, float c) : x(a), y(b), z(c) {}
    float& operator[](int i) { return i == 0 ? x : i == 1 ? y : z; }
    float operator[](int i) const { return i == 0 ? x : i == 1 ? y : z; }
};
struct ivec3 {  // glm::ivec3
    int x = 0, y = 0, z = 0;
    ivec3() = default;
    ivec3(int a, int b, int c) : x(a), y(b), z(c) {}
    int& operator[](int i) { return i == 0 ? x : i == 1 ? y : z; }
    int operator[](int i) const { return i == 0 ? x : i == 1 ? y : z; }
};

// ---- minimal shapes (CCObject::MinShapes, gpu_depthmap_fusion.h:54-75) -------------------------
namespace detail {
#ifndef GDF_WITH_OPENCV
// Convex hull, clockwise in a y-up frame (minAreaRect's cv::convexHull(points, hull, true, true)),
// collinear points dropped, starting at the leftmost (then lowest) point: Andrew's monotone chain.
inline std::vector<Point2f> convex_hull(std::vector<Point2f> p) {
    std::sort(p.begin(), p.end(), [](const Point2f& a, const Point2f& b) {
        return a.x < b.x || (a.x == b.x && a.y < b.y);
    });
    p.erase(std::unique(p.begin(), p.end(),
                        [](const Point2f& a, const Point2f& b) { return a.x == b.x && a.y == b.y; }),
            p.end());
    if (p.size() < 3) return p;
    auto cross = [](const Point2f& o, const Point2f& a, const Point2f& b) {
        return ((double)a.x - o.x) * ((double)b.y - o.y) - ((double)a.y - o.y) * ((double)b.x - o.x);
    };
    std::vector<Point2f> h(2 * p.size());
    size_t k = 0;
    for (size_t i = 0; i < p.size(); ++i) {
        while (k >= 2 && cross(h[k - 2], h[k - 1], p[i]) <= 0) --k;
        h[k++] = p[i];
    }
    for (size_t i = p.size() - 1, t = k + 1; i-- > 0;) {
        while (k >= t && cross(h[k - 2], h[k - 1], p[i]) <= 0) --k;
        h[k++] = p[i];
    }
    h.resize(k - 1);
    std::reverse(h.begin() + 1, h.end());  // (the chain runs counter-clockwise)
    return h;
}

// OpenCV 4.2 rotatingCalipers(CALIPERS_MINAREARECT) over a convex polygon (imgproc/rotcalipers.cpp):
// out = corner, edge vector 1 (width), edge vector 2 (height)
inline void min_area_calipers(const std::vector<Point2f>& pt, Point2f out[3]) {
    const int n = (int)pt.size();
    std::vector<Point2f> vect(n);
    std::vector<float> inv_len(n);
    int left = 0, bottom = 0, right = 0, top = 0;
    float left_x = pt[0].x, right_x = pt[0].x, top_y = pt[0].y, bottom_y = pt[0].y;
    Point2f p0 = pt[0];
    for (int i = 0; i < n; ++i) {
        if (p0.x < left_x) left_x = p0.x, left = i;
        if (p0.x > right_x) right_x = p0.x, right = i;
        if (p0.y > top_y) top_y = p0.y, top = i;
        if (p0.y < bottom_y) bottom_y = p0.y, bottom = i;
        const Point2f p1 = pt[i + 1 < n ? i + 1 : 0];
        const double dx = p1.x - p0.x, dy = p1.y - p0.y;
        vect[i] = Point2f((float)dx, (float)dy);
        inv_len[i] = (float)(1. / std::sqrt(dx * dx + dy * dy));
        p0 = p1;
    }
    float orientation = 0;
    {
        double ax = vect[n - 1].x, ay = vect[n - 1].y;
        for (int i = 0; i < n; ++i) {
            const double bx = vect[i].x, by = vect[i].y;
            const double convexity = ax * by - ay * bx;
            if (convexity != 0) {
                orientation = convexity > 0 ? 1.f : -1.f;
                break;
            }
            ax = bx;
            ay = by;
        }
    }
    float base_a = orientation, base_b = 0;
    int seq[4] = {bottom, right, top, left};
    float minarea = FLT_MAX;
    int best_left = 0, best_bottom = 0;
    float best_a = 0, best_b = 0, best_w = 0, best_h = 0;
    for (int k = 0; k < n; ++k) {
        const float dp[4] = {
            +base_a * vect[seq[0]].x + base_b * vect[seq[0]].y,
            -base_b * vect[seq[1]].x + base_a * vect[seq[1]].y,
            -base_a * vect[seq[2]].x - base_b * vect[seq[2]].y,
            +base_b * vect[seq[3]].x - base_a * vect[seq[3]].y,
        };
        float maxcos = dp[0] * inv_len[seq[0]];
        int main_element = 0;
        for (int i = 1; i < 4; ++i) {
            const float cosalpha = dp[i] * inv_len[seq[i]];
            if (cosalpha > maxcos) {
                main_element = i;
                maxcos = cosalpha;
            }
        }
        const int pindex = seq[main_element];
        const float lead_x = vect[pindex].x * inv_len[pindex];
        const float lead_y = vect[pindex].y * inv_len[pindex];
        switch (main_element) {
            case 0: base_a = lead_x; base_b = lead_y; break;
            case 1: base_a = lead_y; base_b = -lead_x; break;
            case 2: base_a = -lead_x; base_b = -lead_y; break;
            default: base_a = -lead_y; base_b = lead_x; break;
        }
        seq[main_element] += 1;
        if (seq[main_element] == n) seq[main_element] = 0;
        float dx = pt[seq[1]].x - pt[seq[3]].x, dy = pt[seq[1]].y - pt[seq[3]].y;
        const float width = dx * base_a + dy * base_b;
        dx = pt[seq[2]].x - pt[seq[0]].x;
        dy = pt[seq[2]].y - pt[seq[0]].y;
        const float height = -dx * base_b + dy * base_a;
        const float area = width * height;
        if (area <= minarea) {
            minarea = area;
            best_left = seq[3];
            best_a = base_a;
            best_w = width;
            best_b = base_b;
            best_h = height;
            best_bottom = seq[0];
        }
    }
    const float A1 = best_a, B1 = best_b, A2 = -best_b, B2 = best_a;
    const float C1 = A1 * pt[best_left].x + pt[best_left].y * B1;
    const float C2 = A2 * pt[best_bottom].x + pt[best_bottom].y * B2;
    const float idet = 1.f / (A1 * B2 - A2 * B1);
    out[0] = Point2f((C1 * B2 - C2 * B1) * idet, (A1 * C2 - A2 * C1) * idet);
    out[1] = Point2f(A1 * best_w, B1 * best_w);
    out[2] = Point2f(A2 * best_h, B2 * best_h);
}

// cv::minAreaRect (OpenCV 4.2, imgproc/rotcalipers.cpp): angle in degrees in [-90, 0)
inline RotatedRect min_area_rect(const std::vector<Point2f>& points) {
    const std::vector<Point2f> h = convex_hull(points);
    RotatedRect box;
    const int n = (int)h.size();
    if (n > 2) {
        Point2f out[3];
        min_area_calipers(h, out);
        box.center.x = out[0].x + (out[1].x + out[2].x) * 0.5f;
        box.center.y = out[0].y + (out[1].y + out[2].y) * 0.5f;
        box.size.width = (float)std::sqrt((double)out[1].x * out[1].x + (double)out[1].y * out[1].y);
        box.size.height = (float)std::sqrt((double)out[2].x * out[2].x + (double)out[2].y * out[2].y);
        box.angle = (float)std::atan2((double)out[1].y, (double)out[1].x);
    } else if (n == 2) {
        box.center.x = (h[0].x + h[1].x) * 0.5f;
        box.center.y = (h[0].y + h[1].y) * 0.5f;
        const double dx = h[1].x - h[0].x, dy = h[1].y - h[0].y;
        box.size.width = (float)std::sqrt(dx * dx + dy * dy);
        box.size.height = 0;
        box.angle = (float)std::atan2(dy, dx);
    } else if (n == 1) {
        box.center = h[0];
    }
    box.angle = (float)(box.angle * 180 / M_PI);
    return box;
}

// cv::minEnclosingCircle (OpenCV 4.2, imgproc/shapedescr.cpp): the iterative 1-, 2-, 3-point
// construction in input order, radii padded by EPS
constexpr float kCircleEps = 1.0e-4f;
inline void circle_2(const Point2f& a, const Point2f& b, Point2f& c, float& r) {
    c.x = (a.x + b.x) / 2.0f;
    c.y = (a.y + b.y) / 2.0f;
    r = (float)(norm(Point2f(a.x - b.x, a.y - b.y)) / 2.0 + kCircleEps);
}
inline void circle_3(const Point2f& p1, const Point2f& p2, const Point2f& p3, Point2f& c, float& r) {
    const double x1 = p1.x, y1 = p1.y, x2 = p2.x, y2 = p2.y, x3 = p3.x, y3 = p3.y;
    const double d = 2.0 * (x1 * (y2 - y3) + x2 * (y3 - y1) + x3 * (y1 - y2));
    if (std::fabs(d) < 1e-12) {  // collinear: the farthest pair
        const double d12 = norm(p2 - p1), d13 = norm(p3 - p1), d23 = norm(p3 - p2);
        if (d12 >= d13 && d12 >= d23) circle_2(p1, p2, c, r);
        else if (d13 >= d23) circle_2(p1, p3, c, r);
        else circle_2(p2, p3, c, r);
        return;
    }
    const double a1 = x1 * x1 + y1 * y1, a2 = x2 * x2 + y2 * y2, a3 = x3 * x3 + y3 * y3;
    c.x = (float)((a1 * (y2 - y3) + a2 * (y3 - y1) + a3 * (y1 - y2)) / d);
    c.y = (float)((a1 * (x3 - x2) + a2 * (x1 - x3) + a3 * (x2 - x1)) / d);
    r = (float)(norm(Point2f((float)(x1 - c.x), (float)(y1 - c.y))) + kCircleEps);
}
inline void circle_third(const std::vector<Point2f>& p, int i, int j, Point2f& c, float& r) {
    circle_2(p[i], p[j], c, r);
    for (int k = 0; k < j; ++k) {
        if (norm(p[k] - c) < r) continue;
        circle_3(p[i], p[j], p[k], c, r);
    }
}
inline void circle_second(const std::vector<Point2f>& p, int i, Point2f& c, float& r) {
    circle_2(p[i], p[0], c, r);
    for (int j = 1; j < i; ++j) {
        if (norm(p[j] - c) < r) continue;
        circle_third(p, i, j, c, r);
    }
}
inline void min_enclosing_circle(const std::vector<Point2f>& p, Point2f& c, float& r) {
    const int n = (int)p.size();
    if (n == 0) {
        c = Point2f();
        r = 0;
        return;
    }
    if (n == 1) {
        c = p[0];
        r = kCircleEps;
        return;
    }
    circle_2(p[0], p[1], c, r);
    for (int i = 2; i < n; ++i) {
        if (norm(p[i] - c) < r) continue;
        circle_second(p, i, c, r);
    }
}
#endif

template <class P>
inline std::vector<Point2f> to_point2f(const std::vector<P>& pts) {
    std::vector<Point2f> v(pts.size());
    for (size_t i = 0; i < pts.size(); ++i) v[i] = Point2f((float)pts[i].x, (float)pts[i].y);
    return v;
}
}  // namespace detail

// ---- the gain filters (filter/filter.h, const_global_velocity_filter.h, orientation_2d_filter.h,
// wrap_pi.h, rotated_rect_filter.h) ----------------------------------------------------------------
template <class T, unsigned N>
struct GainFilter {
    T values[N] = {};
    T gain = 0.5;
    bool has_values = false;
    double reference_dt = 1;
    GainFilter() = default;
    GainFilter(T g, double ref_dt) : gain(g), reference_dt(ref_dt) {}
    // filter.h:70-84 (y_new = x_new * gain + (1 - gain) * y_old, gain scaled to dt)
    T gain_for_dt(double dt) const {
        if (std::abs(gain) < 1e-9) return 0;
        const T denom = (reference_dt / gain) + dt - reference_dt;
        if (std::abs(denom) < 1e-9) return 1;
        return dt / denom;
    }
    GainFilter& filter(const T* x) {
        if (has_values) {
            for (unsigned i = 0; i < N; ++i) values[i] = x[i] * gain + (1 - gain) * values[i];
        } else {
            std::copy(x, x + N, values);
            has_values = true;
        }
        return *this;
    }
    GainFilter& filter(double dt, const T* x) {
        if (has_values) {
            const T g = gain_for_dt(dt);
            for (unsigned i = 0; i < N; ++i) values[i] = x[i] * g + (1 - g) * values[i];
        } else {
            std::copy(x, x + N, values);
            has_values = true;
        }
        return *this;
    }
};

template <class T, unsigned N>
struct ObservePredictFilter {  // filter.h:95-155
    T values[N] = {};
    bool has_values = false;
    GainFilter<T, N> prediction_filter, correction_filter;
    ObservePredictFilter() : ObservePredictFilter(0.5, 1, 0.5, 1) {}
    ObservePredictFilter(T pg, double pg_dt, T cg, double cg_dt)
        : prediction_filter(pg, pg_dt), correction_filter(cg, cg_dt) {}
    void correct(double dt, const T* observed) { step(dt, observed, correction_filter); }
    void predict(double dt, const T* prediction) { step(dt, prediction, prediction_filter); }

private:
    void step(double dt, const T* x, GainFilter<T, N>& f) {
        if (has_values) {
            std::copy(values, values + N, f.values);
            f.filter(dt, x);
            std::copy(f.values, f.values + N, values);
        } else {
            has_values = true;
            std::copy(x, x + N, values);
            std::copy(values, values + N, correction_filter.values);
            std::copy(values, values + N, prediction_filter.values);
            correction_filter.has_values = true;
            prediction_filter.has_values = true;
        }
    }
};

template <class T, unsigned N>
struct ConstGlobalVelocityFilter {  // const_global_velocity_filter.h
    T values[N] = {}, velocity[N] = {};
    ObservePredictFilter<T, N> value_filter, velocity_filter;
    T last_measurement[N] = {};
    bool has_last_measurement = false;
    T predicted_velocity[N] = {};
    ConstGlobalVelocityFilter() = default;
    ConstGlobalVelocityFilter(T vpg, double vpg_dt, T vcg, double vcg_dt, T wpg, double wpg_dt,
                              T wcg, double wcg_dt)
        : value_filter(vpg, vpg_dt, vcg, vcg_dt), velocity_filter(wpg, wpg_dt, wcg, wcg_dt) {}
    void observe(double dt, const T* observed) {
        predict(dt);
        correct(dt, observed);
    }
    void correct(double dt, const T* observed) {
        if (has_last_measurement && std::abs(dt) > 1e-6) {
            T v[N];
            for (unsigned i = 0; i < N; ++i) v[i] = (observed[i] - last_measurement[i]) / dt;
            velocity_filter.correct(dt, v);
            std::copy(velocity_filter.values, velocity_filter.values + N, velocity);
        }
        value_filter.correct(dt, observed);
        std::copy(value_filter.values, value_filter.values + N, values);
        std::copy(observed, observed + N, last_measurement);
        has_last_measurement = true;
    }
    void predict(double dt) {
        if (!has_last_measurement) return;
        T p[N];
        for (unsigned i = 0; i < N; ++i) p[i] = values[i] + velocity[i] * dt;
        value_filter.predict(dt, p);
        velocity_filter.predict(dt, predicted_velocity);
        std::copy(value_filter.values, value_filter.values + N, values);
        std::copy(velocity_filter.values, velocity_filter.values + N, velocity);
    }
};

// wrap_pi.h
template <class T>
T wrapTo2Pi(T rad) {
    return std::fmod(rad, static_cast<T>(2 * M_PI)) + ((rad < 0) ? static_cast<T>(2 * M_PI) : 0);
}
template <class T>
T wrapToPi(T rad) {
    return wrapTo2Pi<T>(rad + static_cast<T>(M_PI)) - static_cast<T>(M_PI);
}
template <class T>
T wrapToPiSeq(T before, T now) {
    before = wrapToPi(before);
    now = wrapToPi(now);
    const T diff = now - before;
    if (diff > +static_cast<T>(M_PI)) now -= static_cast<T>(2 * M_PI);
    if (diff < -static_cast<T>(M_PI)) now += static_cast<T>(2 * M_PI);
    return now;
}
template <class T>
T angleDiff(T before, T now) {
    return wrapToPi<T>(wrapToPiSeq<T>(before, now) - before);
}

template <class T>
struct Orientation2DFilter {  // orientation_2d_filter.h (the correct / predict path)
    static const unsigned TNumOrientation = 1;
    T orientation[1] = {0}, turnrate[1] = {0};
    T rotation_wrap = 0;
    ConstGlobalVelocityFilter<T, 1> filter;
    Orientation2DFilter() : Orientation2DFilter(0.5, 1, 0.5, 1, 0.5, 1, 0.5, 1, 0) {}
    Orientation2DFilter(T vpg, double vpg_dt, T vcg, double vcg_dt, T wpg, double wpg_dt, T wcg,
                        double wcg_dt, T wrap)
        : rotation_wrap(wrap), filter(vpg, vpg_dt, vcg, vcg_dt, wpg, wpg_dt, wcg, wcg_dt) {}
    void observe(double dt, const T* observed) {
        predict(dt);
        correct(dt, observed);
    }
    void correct(double dt, const T* observed) {
        T unwrapped[1];
        if (filter.has_last_measurement) {
            T diff = angleDiff(filter.last_measurement[0], observed[0]);
            if (rotation_wrap != 0)
                diff = -rotation_wrap / 2 + std::fmod(diff + rotation_wrap / 2, rotation_wrap);
            unwrapped[0] = filter.last_measurement[0] + diff;
        } else {
            unwrapped[0] = observed[0];
        }
        filter.correct(dt, unwrapped);
        orientation[0] = filter.values[0];
        turnrate[0] = filter.velocity[0];
    }
    void predict(double dt) {
        filter.predict(dt);
        orientation[0] = filter.values[0];
        turnrate[0] = filter.velocity[0];
    }
};

class RotatedRectFilter {  // rotated_rect_filter.h
public:
    RotatedRectFilter() {
        const double ref_dt = 0.1;
        orientation_filter = Orientation2DFilter<double>(1.0, ref_dt, 0.5, ref_dt, 1.0, ref_dt, 0.5,
                                                         ref_dt, M_PI / 2);
        kinematic_filter = ConstGlobalVelocityFilter<double, 2>(1, ref_dt, 0.3, ref_dt, 1.0, ref_dt,
                                                                0.0, ref_dt);
        size_filter = GainFilter<double, 2>(0.2, ref_dt);
    }
    explicit RotatedRectFilter(const RotatedRect& r) : RotatedRectFilter() { filter(1, r); }
    void filter(double dt, const RotatedRect& r) {
        double pos[2] = {r.center.x, r.center.y};
        double angle = r.angle * M_PI / 180;
        const double size[2] = {r.size.width, r.size.height};
        kinematic_filter.observe(dt, pos);
        orientation_filter.correct(dt, &angle);
        size_filter.filter(dt, size);
        rrect = RotatedRect(Point2f((float)kinematic_filter.values[0], (float)kinematic_filter.values[1]),
                            Size2f((float)size_filter.values[0], (float)size_filter.values[1]),
                            (float)(orientation_filter.orientation[0] * 180 / M_PI));
    }
    RotatedRect rrect;

protected:
    ConstGlobalVelocityFilter<double, 2> kinematic_filter;
    Orientation2DFilter<double> orientation_filter;
    GainFilter<double, 2> size_filter;
};

// ---- CCObject (gpu_depthmap_fusion.h:33-113) --------------------------------------------------
class CCObject {
public:
    template <class TWorld, class TVoxel>
    struct Pair {
        TWorld world;
        TVoxel voxel;
    };
    template <class TWorld, class TVoxel>
    struct VectorPair {
        std::vector<TWorld> world;
        std::vector<TVoxel> voxel;
    };
    struct EnclosingCircle {
        Point2f center;
        float radius = 0;
    };
    struct MinShapes {
        RotatedRect box;
        EnclosingCircle circle;
        MinShapes() = default;
        explicit MinShapes(const std::vector<Point2f>& points) {
            if (points.empty()) return;
#ifdef GDF_WITH_OPENCV
            box = cv::minAreaRect(points);
            cv::minEnclosingCircle(points, circle.center, circle.radius);
#else
            box = detail::min_area_rect(points);
            detail::min_enclosing_circle(points, circle.center, circle.radius);
#endif
        }
        explicit MinShapes(const std::vector<Point>& points) : MinShapes(detail::to_point2f(points)) {}
    };
    typedef Pair<vec3, vec3> Pair_3f3f;
    typedef Pair<vec3, ivec3> Pair_3f3i;
    typedef VectorPair<Point2f, Point2f> VectorPair_Points;
    typedef VectorPair<vec3, vec3> VectorPair_3f3f;
    typedef Pair<MinShapes, MinShapes> Pair_Shapes;
    struct Component {
        VectorPair_Points contour2d;
        VectorPair_3f3f contour3d;
        Pair_Shapes shapes;
    };
    struct Layer {
        VectorPair_Points points2d;
        Pair_Shapes shapes;
    };

    Point2f centroid;
    uint32_t label = 0;
    unsigned num_components = 0;
    unsigned num_layers = 0;
    Pair_3f3f center_coord;
    Pair_3f3i min_coord;
    Pair_3f3i max_coord;
    Pair_3f3i aabb_size;  // axis aligned bounding box
    std::vector<Component> components;
    std::vector<Layer> layers;
    Layer topview;
};

// rolledRRect (gpu_depthmap_fusion.cpp:2650-2664)
inline RotatedRect rolledRRect(const RotatedRect& r, int roll) {
    if (roll % 2 == 0) return RotatedRect(r.center, r.size, r.angle + 90 * roll);
    return RotatedRect(r.center, Size2f(r.size.height, r.size.width), r.angle + 90 * roll);
}

class CCObjectTrack;
class CCObjectTrackComparison {  // gpu_depthmap_fusion.cpp:2667-2725
public:
    CCObjectTrackComparison() = default;
    CCObjectTrackComparison(const CCObjectTrack& track, const CCObject& object);
    const CCObjectTrack* track = nullptr;
    const CCObject* object = nullptr;
    RotatedRect trackBox, objectBox;
    Point2f center_diff;
    Point2f box_point_diffs[4];
    float center_dist = 0;
    float box_point_dists[4] = {};
    int best_roll = 0;
    float mean_box_point_dist = 0;
    float area_diff = 0;
    float score = 0;
};

class CCObjectTrack {  // gpu_depthmap_fusion.cpp:2579-2648
public:
    CCObjectTrack() : initialized(false), score_filter(0.5, 0.1, 0.9, 0.1), age(0) {}
    explicit CCObjectTrack(const CCObject& object)
        : initialized(true), lastObject(object), rrect_filter(object.topview.shapes.world.box),
          score_filter(0.25, 0.1, 0.9, 0.1), age(0) {
        const double new_track_score = 0.5;
        score_filter.correct(1, &new_track_score);
    }
    bool initialized;
    CCObject lastObject;
    RotatedRectFilter rrect_filter;
    ObservePredictFilter<double, 1> score_filter;
    float age;

    void advance(double dt) {
        age += dt;
        const double penalty_score = 0.0;
        score_filter.predict(dt, &penalty_score);
    }
    void merge(double dt, const CCObject& obj, const CCObjectTrackComparison& comp) {
        age += 1;
        rrect_filter.filter(dt, rolledRRect(obj.topview.shapes.world.box, comp.best_roll));
        lastObject = obj;
        const double merge_score = 1.0;
        score_filter.correct(dt, &merge_score);
    }
    bool isAcceptable(const CCObjectTrackComparison& comp) const {
        const double area = comp.trackBox.size.area();
        const float trackSize = comp.trackBox.size.width + comp.trackBox.size.height;
        const float objectSize = comp.objectBox.size.width + comp.objectBox.size.height;
        const float distUntilTrackBoundary = trackSize * 0.5;
        const float distUntilObjectBoundary = objectSize * 0.5;
        if (area > 0.5 && (comp.area_diff > area * 0.5)) return false;
        if (comp.center_dist > (distUntilTrackBoundary + distUntilObjectBoundary)) return false;
        if (comp.center_dist > 2.5) return false;
        if (comp.mean_box_point_dist > 2.5) return false;
        return true;
    }
    bool isDead() const { return (age > 0.06) && (score_filter.values[0] < 0.1); }
};

inline CCObjectTrackComparison::CCObjectTrackComparison(const CCObjectTrack& t, const CCObject& o)
    : track(&t), object(&o) {
    trackBox = t.rrect_filter.rrect;
    objectBox = o.topview.shapes.world.box;
    center_diff = trackBox.center - objectBox.center;
    center_dist = (float)norm(center_diff);
    Point2f a[4], b[4];
    trackBox.points(a);
    objectBox.points(b);
    for (int roll = 0; roll < 4; ++roll) {
        Point2f d[4];
        float dist[4];
        for (int i = 0; i < 4; ++i) {
            d[i] = a[i] - b[(i + roll) % 4];
            dist[i] = (float)norm(d[i]);
        }
        const float mean = 0.25 * (dist[0] + dist[1] + dist[2] + dist[3]);
        if (roll == 0 || mean < mean_box_point_dist) {
            best_roll = roll;
            mean_box_point_dist = mean;
            for (int i = 0; i < 4; ++i) {
                box_point_diffs[i] = d[i];
                box_point_dists[i] = dist[i];
            }
        }
    }
    area_diff = std::abs(trackBox.size.area() - objectBox.size.area());
    const float w_center = 0.0, w_pts = 0.1, w_area = 0.0;
    score = -(+w_center * center_dist + w_pts * mean_box_point_dist + w_area * area_diff);
}

// objectTracking (gpu_depthmap_fusion.cpp:2727-2944): associate this frame's objects with the
// tracks (best acceptable score per object, then the best object per track), merge, start new
// tracks, advance the others, drop the dead ones (the reference's diagnostics prints are omitted).
inline void object_tracking(const std::vector<CCObject>& objects, std::vector<CCObjectTrack>& tracks,
                            float min_area) {
    const double dt = 1.0 / 30.0;
    const int num_objects = (int)objects.size();
    int num_tracks = (int)tracks.size();
    std::vector<int> assigned(num_objects), numObjectsPerTrack(num_tracks, 0);
    std::vector<CCObjectTrackComparison> comparisons((size_t)num_objects * num_tracks);
    for (int o = 0; o < num_objects; ++o) {
        assigned[o] = -2;  // ignore
        if (o == 0) continue;  // background
        if (objects[o].topview.shapes.world.box.size.area() < min_area) continue;
        assigned[o] = -1;  // new track
        float best = 0;
        for (int t = 0; t < num_tracks; ++t) {
            CCObjectTrackComparison& comp = comparisons[(size_t)o * num_tracks + t];
            comp = CCObjectTrackComparison(tracks[t], objects[o]);
            if (!tracks[t].isAcceptable(comp)) continue;
            if (assigned[o] < 0 || comp.score > best) {
                best = comp.score;
                assigned[o] = t;
            }
        }
        if (assigned[o] >= 0) numObjectsPerTrack[assigned[o]] += 1;
    }
    std::vector<int> objectPerTrack(num_tracks, -1);
    std::vector<float> bestPerTrack(num_tracks, 0);
    for (int o = 1; o < num_objects; ++o) {
        const int t = assigned[o];
        if (t < 0) continue;
        const CCObjectTrackComparison& comp = comparisons[(size_t)o * num_tracks + t];
        if (objectPerTrack[t] == -1 || comp.score > bestPerTrack[t]) {
            objectPerTrack[t] = o;
            bestPerTrack[t] = comp.score;
        }
    }
    for (int o = 1; o < num_objects; ++o) {
        const int t = assigned[o];
        if (t < 0 || objectPerTrack[t] == o) continue;
        assigned[o] = -1;  // lost its track: a new one
    }
    int num_new = 0;
    for (int o = 1; o < num_objects; ++o) num_new += assigned[o] == -1;
    tracks.resize(num_tracks + num_new);
    std::vector<bool> advance(num_tracks + num_new, true);
    int next_new = num_tracks;
    for (int o = 1; o < num_objects; ++o) {
        const int t = assigned[o];
        if (t == -2) continue;
        if (t == -1) {
            tracks[next_new] = CCObjectTrack(objects[o]);
            advance[next_new] = false;
            ++next_new;
        } else {
            tracks[t].merge(dt, objects[o], comparisons[(size_t)o * num_tracks + t]);
            advance[t] = false;
        }
    }
    for (int t = 0; t < num_tracks + num_new; ++t)
        if (advance[t]) tracks[t].advance(dt);
    num_tracks += num_new;
    int remaining = 0;
    for (int t = 0; t < num_tracks; ++t) {
        if (tracks[t].isDead()) continue;
        if (t != remaining) tracks[remaining] = tracks[t];
        ++remaining;
    }
    tracks.resize(remaining);
}

}  // namespace gdf
