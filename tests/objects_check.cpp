// Checks of include/gdf_objects.hpp on the host (tests/test_objects.py builds and runs it): the
// restated minAreaRect / minEnclosingCircle on shapes with known answers, the gain filters'
// first-sample and dt behaviour, and objectTracking's association over a few synthetic frames
// (gpu_depthmap_fusion.cpp:2579-2944).  Prints "ok" or the first failed check.
#include <cmath>
#include <cstdio>
#include <vector>

#include "gdf_objects.hpp"

using gdf::Point2f;

static int fails = 0;
#define CHECK(c)                                                  \
    do {                                                          \
        if (!(c)) {                                               \
            std::printf("FAIL line %d: %s\n", __LINE__, #c);      \
            ++fails;                                              \
        }                                                         \
    } while (0)

static bool near(double a, double b, double tol) { return std::fabs(a - b) <= tol; }

static gdf::CCObject box_object(float cx, float cy, float w, float h, float angle) {
    gdf::CCObject o;
    o.topview.shapes.world.box = gdf::RotatedRect(Point2f(cx, cy), gdf::Size2f(w, h), angle);
    o.max_coord.world.z = 1.0f;
    return o;
}

int main() {
    // a 4 x 2 rectangle rotated by 30 degrees, its corners plus interior points
    {
        const double a = 30 * M_PI / 180;
        const double ux = std::cos(a), uy = std::sin(a), vx = -std::sin(a), vy = std::cos(a);
        std::vector<Point2f> pts;
        for (int i = 0; i <= 8; ++i)
            for (int j = 0; j <= 4; ++j) {
                const double s = -2 + 0.5 * i, t = -1 + 0.5 * j;
                pts.push_back(Point2f((float)(5 + s * ux + t * vx), (float)(3 + s * uy + t * vy)));
            }
        const gdf::RotatedRect r = gdf::detail::min_area_rect(pts);
        CHECK(near(r.size.area(), 8.0, 1e-3));
        CHECK(near(r.center.x, 5.0, 1e-4) && near(r.center.y, 3.0, 1e-4));
        CHECK(r.angle >= -90.0f && r.angle < 0.0f);
        Point2f c[4];
        r.points(c);
        for (int k = 0; k < 4; ++k) {  // every corner is one of the rectangle's
            bool hit = false;
            for (int sx = -1; sx <= 1; sx += 2)
                for (int sy = -1; sy <= 1; sy += 2)
                    hit |= near(c[k].x, 5 + 2 * sx * ux + sy * vx, 1e-3) &&
                           near(c[k].y, 3 + 2 * sx * uy + sy * vy, 1e-3);
            CHECK(hit);
        }
        // the enclosing circle of the rectangle: half its diagonal, at its center
        Point2f cc;
        float rad;
        gdf::detail::min_enclosing_circle(pts, cc, rad);
        CHECK(near(rad, std::sqrt(5.0), 1e-3));
        CHECK(near(cc.x, 5.0, 1e-3) && near(cc.y, 3.0, 1e-3));
    }
    // integer contour points (cv::Point): an axis-aligned 3 x 2 box
    {
        std::vector<gdf::Point> q = {{0, 0}, {1, 0}, {2, 0}, {3, 0}, {3, 1}, {3, 2}, {2, 2}, {0, 2}, {0, 1}};
        const gdf::CCObject::MinShapes sh(q);
        CHECK(near(sh.box.size.area(), 6.0, 1e-4));
        CHECK(near(sh.box.center.x, 1.5, 1e-5) && near(sh.box.center.y, 1.0, 1e-5));
        CHECK(near(sh.circle.radius, std::sqrt(13.0) / 2, 1e-3));
    }
    // degenerate inputs: one point, two points, collinear points, none
    {
        const gdf::RotatedRect r1 = gdf::detail::min_area_rect({Point2f(2, 3)});
        CHECK(r1.center.x == 2 && r1.center.y == 3 && r1.size.area() == 0);
        const gdf::RotatedRect r2 = gdf::detail::min_area_rect({Point2f(0, 0), Point2f(3, 4)});
        CHECK(near(r2.size.width, 5, 1e-6) && r2.size.height == 0);
        const gdf::RotatedRect r3 = gdf::detail::min_area_rect({Point2f(0, 0), Point2f(1, 1), Point2f(2, 2)});
        CHECK(near(r3.size.width, std::sqrt(8.0), 1e-5) && r3.size.height == 0);
        const gdf::CCObject::MinShapes none(std::vector<Point2f>{});
        CHECK(none.box.size.area() == 0 && none.circle.radius == 0);
    }
    // gain filters (filter.h): the first sample is copied, dt = reference_dt keeps the gain
    {
        gdf::GainFilter<double, 1> g(0.2, 0.1);
        CHECK(near(g.gain_for_dt(0.1), 0.2, 1e-12));
        CHECK(g.gain_for_dt(0.2) > 0.2);
        const double x0 = 4, x1 = 9;
        g.filter(0.1, &x0);
        CHECK(g.values[0] == 4);
        g.filter(0.1, &x1);
        CHECK(near(g.values[0], 9 * 0.2 + 0.8 * 4, 1e-12));
        gdf::ObservePredictFilter<double, 1> op(0.25, 0.1, 0.9, 0.1);
        const double half = 0.5, one = 1.0;
        op.correct(1, &half);
        CHECK(op.values[0] == 0.5);
        op.correct(1.0 / 30, &one);
        CHECK(op.values[0] > 0.5 && op.values[0] < 1.0);
        gdf::RotatedRectFilter rf(gdf::RotatedRect(Point2f(1, 2), gdf::Size2f(3, 4), -30));
        CHECK(near(rf.rrect.center.x, 1, 1e-6) && near(rf.rrect.size.height, 4, 1e-6) &&
              near(rf.rrect.angle, -30, 1e-4));
    }
    // objectTracking: two objects tracked over frames, a third appears, then all vanish
    {
        std::vector<gdf::CCObjectTrack> tracks;
        std::vector<gdf::CCObject> objs;
        objs.push_back(gdf::CCObject());  // background object 0
        objs.push_back(box_object(2, 2, 1, 0.5f, -10));
        objs.push_back(box_object(8, 1, 0.8f, 0.8f, -45));
        objs.push_back(box_object(30, 30, 0.01f, 0.01f, -45));  // below min_area: ignored
        gdf::object_tracking(objs, tracks, 0.05f);
        CHECK(tracks.size() == 2);
        const double s0 = tracks[0].score_filter.values[0];
        CHECK(near(s0, 0.5, 1e-12));
        for (int f = 1; f <= 5; ++f) {  // both move slowly: merged into their tracks
            objs[1].topview.shapes.world.box.center.x += 0.05f;
            objs[2].topview.shapes.world.box.center.y += 0.05f;
            gdf::object_tracking(objs, tracks, 0.05f);
            CHECK(tracks.size() == 2);
        }
        CHECK(tracks[0].score_filter.values[0] > s0);
        CHECK(tracks[0].age >= 5);
        CHECK(near(tracks[0].lastObject.topview.shapes.world.box.center.x, 2.25, 1e-4));
        objs.push_back(box_object(-5, 4, 1, 1, -80));
        gdf::object_tracking(objs, tracks, 0.05f);
        CHECK(tracks.size() == 3);
        std::vector<gdf::CCObject> empty(1);
        size_t n = tracks.size();
        for (int f = 0; f < 200 && n; ++f) {
            gdf::object_tracking(empty, tracks, 0.05f);
            CHECK(tracks.size() <= n);
            n = tracks.size();
        }
        CHECK(tracks.empty());
    }
    std::printf(fails ? "%d failures\n" : "ok\n", fails);
    return fails ? 1 : 0;
}
