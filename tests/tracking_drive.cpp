// Driver of gdf::object_tracking (include/gdf_objects.hpp) for tests/test_tracking_parity.py.
// Reads object sequences on stdin - per frame the objects of m_ccObjects (object 0 = background),
// each either its top-view world points (the box is CCObject::MinShapes of them, as
// createCCObjects builds topview.shapes.world, gpu_depthmap_fusion.cpp:2533-2537) or a box -
// runs objectTracking(min_area) frame after frame and prints, per frame, every object's box and
// every track's state (filtered box, score, age, last object's label).  Floats as C99 hex
// floats (exact).
//
//   input : min_area <a>\n frames <F>\n  then per frame: objects <N>\n and N lines
//           "p <label> <npts> x0 y0 x1 y1 ..."  or  "b <label> cx cy w h angle"
//   output: per frame "frame f" / "boxes N" + N lines / "tracks T" + T lines
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "gdf_objects.hpp"

static float rd() {
    char buf[64];
    if (std::scanf("%63s", buf) != 1) std::exit(2);
    return std::strtof(buf, nullptr);
}

int main() {
    char tag[32];
    if (std::scanf("%31s", tag) != 1) return 2;
    const float min_area = rd();
    int frames = 0;
    if (std::scanf("%31s %d", tag, &frames) != 2) return 2;
    std::vector<gdf::CCObjectTrack> tracks;
    for (int f = 0; f < frames; ++f) {
        int n = 0;
        if (std::scanf("%31s %d", tag, &n) != 2) return 2;
        std::vector<gdf::CCObject> objs((size_t)n);
        for (int o = 0; o < n; ++o) {
            char kind[4];
            unsigned label = 0;
            if (std::scanf("%3s %u", kind, &label) != 2) return 2;
            objs[o].label = label;
            if (kind[0] == 'p') {
                int np = 0;
                if (std::scanf("%d", &np) != 1) return 2;
                std::vector<gdf::Point2f>& pts = objs[o].topview.points2d.world;
                for (int i = 0; i < np; ++i) {
                    const float x = rd(), y = rd();
                    pts.push_back(gdf::Point2f(x, y));
                }
                objs[o].topview.shapes.world = gdf::CCObject::MinShapes(pts);
            } else {
                const float cx = rd(), cy = rd(), w = rd(), h = rd(), a = rd();
                objs[o].topview.shapes.world.box =
                    gdf::RotatedRect(gdf::Point2f(cx, cy), gdf::Size2f(w, h), a);
            }
        }
        gdf::object_tracking(objs, tracks, min_area);
        std::printf("frame %d\nboxes %d\n", f, n);
        for (const gdf::CCObject& o : objs) {
            const gdf::RotatedRect& r = o.topview.shapes.world.box;
            std::printf("%a %a %a %a %a\n", r.center.x, r.center.y, r.size.width, r.size.height,
                        r.angle);
        }
        std::printf("tracks %d\n", (int)tracks.size());
        for (const gdf::CCObjectTrack& t : tracks) {
            const gdf::RotatedRect& r = t.rrect_filter.rrect;
            std::printf("%a %a %a %a %a %a %a %u\n", r.center.x, r.center.y, r.size.width,
                        r.size.height, r.angle, t.score_filter.values[0], t.age,
                        t.lastObject.label);
        }
    }
    return 0;
}
