"""Independent Python restatement of the reference's object tracking - TEST INFRASTRUCTURE.

Follows src/gpu_depthmap_fusion.cpp:2579-2944 (CCObjectTrack, rolledRRect,
CCObjectTrackComparison, GPUDepthmapFusion::objectTracking) and the filters it uses,
include/gpu_depthmap_fusion/filter/filter.h (GainFilter, ObservePredictFilter),
const_global_velocity_filter.h, orientation_2d_filter.h, wrap_pi.h and rotated_rect_filter.h,
plus cv::RotatedRect::points / cv::norm (OpenCV 4.x core, absent here: restated from its
published definition).  It is written from the reference, not from include/gdf_objects.hpp, and
keeps the reference's C++ types: `float` members and locals are numpy float32 scalars (every f32
operation rounds), `double` ones Python floats, float-to-double promotions where C++ makes them
(`0.25 * float`, `float > 2.5`, `age += dt`).  tests/test_tracking_parity.py compares it with
gdf::object_tracking bit for bit.  The reference's diagnostic prints are not restated.
"""
import math

import numpy as np

f32 = np.float32
PI = math.pi


# ---- cv::RotatedRect / cv::Point2f / cv::norm ------------------------------------------------------
class RRect:
    """cv::RotatedRect: center (f32 x, y), size (f32 width, height), angle (f32 degrees)."""
    __slots__ = ("cx", "cy", "w", "h", "angle")

    def __init__(self, cx, cy, w, h, angle):
        self.cx, self.cy, self.w, self.h, self.angle = f32(cx), f32(cy), f32(w), f32(h), f32(angle)

    def area(self):  # Size2f::area: width * height in float
        return f32(self.w * self.h)

    def points(self):
        """cv::RotatedRect::points: _angle = angle*CV_PI/180 (double), b = (float)cos*0.5f,
        a = (float)sin*0.5f; corners 0/1 in float, 2/3 mirrored through the center."""
        ang = float(self.angle) * PI / 180.0
        b = f32(f32(math.cos(ang)) * f32(0.5))
        a = f32(f32(math.sin(ang)) * f32(0.5))
        p0x = f32(f32(self.cx - f32(a * self.h)) - f32(b * self.w))
        p0y = f32(f32(self.cy + f32(b * self.h)) - f32(a * self.w))
        p1x = f32(f32(self.cx + f32(a * self.h)) - f32(b * self.w))
        p1y = f32(f32(self.cy - f32(b * self.h)) - f32(a * self.w))
        two = f32(2.0)
        p2x, p2y = f32(two * self.cx - p0x), f32(two * self.cy - p0y)
        p3x, p3y = f32(two * self.cx - p1x), f32(two * self.cy - p1y)
        return [(p0x, p0y), (p1x, p1y), (p2x, p2y), (p3x, p3y)]


def cv_norm(x, y):
    """cv::norm(Point_<float>): sqrt((double)x*x + (double)y*y), a double."""
    x, y = float(x), float(y)
    return math.sqrt(x * x + y * y)


def rolled_rrect(r, roll):  # rolledRRect (fusion.cpp:2650-2664): angle + 90*roll in float
    ang = f32(r.angle + f32(90 * roll))
    if roll % 2 == 0:
        return RRect(r.cx, r.cy, r.w, r.h, ang)
    return RRect(r.cx, r.cy, r.h, r.w, ang)


# ---- filter.h --------------------------------------------------------------------------------------
class GainFilter:
    """GainFilter<double, N> (filter.h:17-92)."""

    def __init__(self, gain=0.5, reference_dt=1.0, n=1):
        self.gain, self.reference_dt = float(gain), float(reference_dt)
        self.has_values = False
        self.values = [0.0] * n  # (uninitialised in the reference until the first sample)

    def gain_for_dt(self, dt):
        if abs(self.gain) < 1e-9:
            return 0.0
        denom = (self.reference_dt / self.gain) + dt - self.reference_dt
        if abs(denom) < 1e-9:
            return 1.0
        return dt / denom

    def filter_dt(self, dt, new):
        if self.has_values:
            g = self.gain_for_dt(dt)
            self.values = [new[i] * g + (1 - g) * self.values[i] for i in range(len(self.values))]
        else:
            self.values = list(new)
            self.has_values = True


class ObservePredictFilter:
    """ObservePredictFilter<double, N> (filter.h:95-155)."""

    def __init__(self, pg=0.5, pg_dt=1.0, cg=0.5, cg_dt=1.0, n=1):
        self.prediction = GainFilter(pg, pg_dt, n)
        self.correction = GainFilter(cg, cg_dt, n)
        self.has_values = False
        self.values = [0.0] * n

    def _first(self, x):
        self.has_values = True
        self.values = list(x)
        self.correction.values = list(x)
        self.prediction.values = list(x)
        self.correction.has_values = self.prediction.has_values = True

    def correct(self, dt, observed):
        if self.has_values:
            self.correction.values = list(self.values)
            self.correction.filter_dt(dt, observed)
            self.values = list(self.correction.values)
        else:
            self._first(observed)

    def predict(self, dt, prediction):
        if self.has_values:
            self.prediction.values = list(self.values)
            self.prediction.filter_dt(dt, prediction)
            self.values = list(self.prediction.values)
        else:
            self._first(prediction)


class ConstGlobalVelocityFilter:
    """ConstGlobalVelocityFilter<double, N> (const_global_velocity_filter.h)."""

    def __init__(self, vpg, vpg_dt, vcg, vcg_dt, wpg, wpg_dt, wcg, wcg_dt, n):
        self.value_filter = ObservePredictFilter(vpg, vpg_dt, vcg, vcg_dt, n)
        self.velocity_filter = ObservePredictFilter(wpg, wpg_dt, wcg, wcg_dt, n)
        self.values = [0.0] * n
        self.velocity = [0.0] * n
        self.predicted_velocity = [0.0] * n
        self.last = [0.0] * n
        self.has_last = False
        self.n = n

    def observe(self, dt, obs):
        self.predict(dt)
        self.correct(dt, obs)

    def correct(self, dt, obs):
        if self.has_last and abs(dt) > 1e-6:
            ov = [(obs[i] - self.last[i]) / dt for i in range(self.n)]
            self.velocity_filter.correct(dt, ov)
            self.velocity = list(self.velocity_filter.values)
        self.value_filter.correct(dt, obs)
        self.values = list(self.value_filter.values)
        self.last = list(obs)
        self.has_last = True

    def predict(self, dt):
        if self.has_last:
            pred = [self.values[i] + self.velocity[i] * dt for i in range(self.n)]
            self.value_filter.predict(dt, pred)
            self.velocity_filter.predict(dt, self.predicted_velocity)
            self.values = list(self.value_filter.values)
            self.velocity = list(self.velocity_filter.values)


# ---- wrap_pi.h -------------------------------------------------------------------------------------
def wrap_to_2pi(rad):
    return math.fmod(rad, 2 * PI) + ((2 * PI) if rad < 0 else 0.0)


def wrap_to_pi(rad):
    return wrap_to_2pi(rad + PI) - PI


def wrap_to_pi_seq(before, now):
    before = wrap_to_pi(before)
    now = wrap_to_pi(now)
    diff = now - before
    if diff > PI:
        now -= 2 * PI
    if diff < -PI:
        now += 2 * PI
    return now


def angle_diff(before, now):
    return wrap_to_pi(wrap_to_pi_seq(before, now) - before)


class Orientation2DFilter:
    """Orientation2DFilter<double> (orientation_2d_filter.h): correct() unwraps the observed angle
    against the last measurement modulo rotation_wrap."""

    def __init__(self, vpg, vpg_dt, vcg, vcg_dt, wpg, wpg_dt, wcg, wcg_dt, wrap):
        self.filter = ConstGlobalVelocityFilter(vpg, vpg_dt, vcg, vcg_dt, wpg, wpg_dt, wcg, wcg_dt, 1)
        self.wrap = float(wrap)
        self.orientation = 0.0

    def correct(self, dt, observed):
        if self.filter.has_last:
            diff = angle_diff(self.filter.last[0], observed)
            if self.wrap != 0:
                diff = -self.wrap / 2 + math.fmod(diff + self.wrap / 2, self.wrap)
            unwrapped = self.filter.last[0] + diff
        else:
            unwrapped = observed
        self.filter.correct(dt, [unwrapped])
        self.orientation = self.filter.values[0]


class RotatedRectFilter:
    """rotated_rect_filter.h: position by a constant-velocity filter, angle by the 90-degree
    wrapped orientation filter, size by a gain filter; the filtered box is a float RotatedRect."""

    def __init__(self, rrect=None):
        ref_dt = 0.1
        self.orientation = Orientation2DFilter(1.0, ref_dt, 0.5, ref_dt, 1.0, ref_dt, 0.5, ref_dt, PI / 2)
        self.kinematic = ConstGlobalVelocityFilter(1, ref_dt, 0.3, ref_dt, 1.0, ref_dt, 0.0, ref_dt, 2)
        self.size = GainFilter(0.2, ref_dt, 2)
        self.rrect = RRect(0, 0, 0, 0, 0)
        if rrect is not None:
            self.filter(1, rrect)

    def filter(self, dt, r):
        pos = [float(r.cx), float(r.cy)]
        angle = float(r.angle) * PI / 180
        size = [float(r.w), float(r.h)]
        self.kinematic.observe(dt, pos)
        self.orientation.correct(dt, angle)
        self.size.filter_dt(dt, size)
        self.rrect = RRect(f32(self.kinematic.values[0]), f32(self.kinematic.values[1]),
                           f32(self.size.values[0]), f32(self.size.values[1]),
                           f32(self.orientation.orientation * 180 / PI))


# ---- CCObjectTrack / CCObjectTrackComparison / objectTracking (fusion.cpp:2579-2944) ----------------
class Track:
    def __init__(self, obj=None):
        if obj is None:  # CCObjectTrack(): score filter (0.5, 0.1, 0.9, 0.1)
            self.initialized = False
            self.rrect_filter = RotatedRectFilter()
            self.score = ObservePredictFilter(0.5, 0.1, 0.9, 0.1)
            self.last_label = None
        else:
            self.initialized = True
            self.rrect_filter = RotatedRectFilter(obj["box"])
            self.last_label = obj["label"]
            self.score = ObservePredictFilter(0.25, 0.1, 0.9, 0.1)
            self.score.correct(1, [0.5])
        self.age = f32(0)

    def is_dead(self):
        return (float(self.age) > 0.06) and (self.score.values[0] < 0.1)

    def is_acceptable(self, c):
        area = float(c.track_box.area())
        track_size = f32(c.track_box.w + c.track_box.h)
        object_size = f32(c.object_box.w + c.object_box.h)
        dt_track = f32(float(track_size) * 0.5)
        dt_obj = f32(float(object_size) * 0.5)
        if area > 0.5 and float(c.area_diff) > area * 0.5:
            return False
        if c.center_dist > f32(dt_track + dt_obj):
            return False
        if float(c.center_dist) > 2.5:
            return False
        if float(c.mean_box_point_dist) > 2.5:
            return False
        return True

    def advance(self, dt):
        self.age = f32(float(self.age) + dt)
        self.score.predict(dt, [0.0])

    def merge(self, dt, obj, comp):
        self.age = f32(self.age + f32(1))
        self.rrect_filter.filter(dt, rolled_rrect(obj["box"], comp.best_roll))
        self.last_label = obj["label"]
        self.score.correct(dt, [1.0])


class Comparison:
    def __init__(self, track, obj):
        tb, ob = track.rrect_filter.rrect, obj["box"]
        self.track_box, self.object_box = tb, ob
        dx, dy = f32(tb.cx - ob.cx), f32(tb.cy - ob.cy)
        self.center_dist = f32(cv_norm(dx, dy))
        pa, pb = tb.points(), ob.points()
        self.best_roll, self.mean_box_point_dist = 0, f32(0)
        for roll in range(4):
            dist = []
            for i in range(4):
                ex = f32(pa[i][0] - pb[(i + roll) % 4][0])
                ey = f32(pa[i][1] - pb[(i + roll) % 4][1])
                dist.append(f32(cv_norm(ex, ey)))
            s = f32(f32(f32(dist[0] + dist[1]) + dist[2]) + dist[3])
            mean = f32(0.25 * float(s))
            if roll == 0 or mean < self.mean_box_point_dist:
                self.best_roll = roll
                self.mean_box_point_dist = mean
        self.area_diff = f32(abs(f32(tb.area() - ob.area())))
        w_center, w_pts, w_area = f32(0.0), f32(0.1), f32(0.0)
        self.score = -f32(f32(f32(w_center * self.center_dist) + f32(w_pts * self.mean_box_point_dist))
                          + f32(w_area * self.area_diff))


def object_tracking(objects, tracks, min_area):
    """GPUDepthmapFusion::objectTracking(min_area) on `objects` (dicts with "box": RRect of the
    top view, "label") and the track list (modified in place)."""
    dt = 1.0 / 30.0
    n_obj, n_tr = len(objects), len(tracks)
    assigned = [0] * n_obj
    comps = {}
    min_area = f32(min_area)
    for o in range(n_obj):
        assigned[o] = -2
        if o == 0:
            continue
        if objects[o]["box"].area() < min_area:
            continue
        assigned[o] = -1
        best = f32(0)
        for t in range(n_tr):
            c = comps[(o, t)] = Comparison(tracks[t], objects[o])
            if not tracks[t].is_acceptable(c):
                continue
            if assigned[o] < 0 or c.score > best:
                best = c.score
                assigned[o] = t
    obj_per_track = [-1] * n_tr
    best_per_track = [f32(0)] * n_tr
    for o in range(1, n_obj):
        t = assigned[o]
        if t < 0:
            continue
        c = comps[(o, t)]
        if obj_per_track[t] == -1 or c.score > best_per_track[t]:
            obj_per_track[t] = o
            best_per_track[t] = c.score
    for o in range(1, n_obj):
        t = assigned[o]
        if t < 0 or obj_per_track[t] == o:
            continue
        assigned[o] = -1
    n_new = sum(1 for o in range(1, n_obj) if assigned[o] == -1)
    tracks.extend(Track() for _ in range(n_new))
    do_advance = [True] * (n_tr + n_new)
    nxt = n_tr
    for o in range(1, n_obj):
        t = assigned[o]
        if t == -2:
            continue
        if t == -1:
            tracks[nxt] = Track(objects[o])
            do_advance[nxt] = False
            nxt += 1
        else:
            tracks[t].merge(dt, objects[o], comps[(o, t)])
            do_advance[t] = False
    for t in range(n_tr + n_new):
        if do_advance[t]:
            tracks[t].advance(dt)
    tracks[:] = [t for t in tracks if not t.is_dead()]


def track_state(t):
    """What the parity test compares per track: the filtered box, the score, the age, the label
    of the last merged object (f32 / f64 values)."""
    r = t.rrect_filter.rrect
    return (r.cx, r.cy, r.w, r.h, r.angle, t.score.values[0], t.age, t.last_label)
