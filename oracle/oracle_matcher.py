"""TEST INFRASTRUCTURE ONLY — sequential restatement of Matcher::Track (matcher.cpp:301-405) over the CPU
tracker oracle (oracle_track.cpp via oracle.py).  Imported only by tests/.

Unlike the product (csrc/frontend.cpp, which batches FindMatches over features on the device), this walks
the features one at a time exactly as the reference loop does, so it also checks the batching.  Parity is
unpinned by reference fixtures (none exist for this path); the tracker primitives underneath
are pinned by known-answer tests (tests/test_oracle_track.py, tests/test_corners.py).

The map is a plain Python structure (`OracleMap`), independent of slamgpu's MapArrays growth helpers.
Defined orders (the reference's are implementation details), as in the product:
  * a feature's views (map<View*, Point2f>, matcher.cpp:43) are tried in creation order;
  * features whose point is no longer feature_usable() are all removed (matcher.cpp:325-328 erases while
    iterating);
  * Eigen's quaternion squaredNorm sums x^2 + y^2 + z^2 + w^2 in that order.
"""
from __future__ import annotations

import math

import numpy as np

import oracle

WINDOW, DEPTH = 13, 6                  # kWindowSize (matcher.cpp:27), MakePyramid(img, 6) (matcher.cpp:321)
MIN_MATCHES, MAX_VIEWS = 40, 4         # matcher.cpp:336/350, 398
INITIAL_DEPTH = 2000.0                 # matcher.cpp:376
NO_BASELINE, NO_OBSERVATIONS, MISMATCHED, BAD_LOCATION = 1, 2, 3, 0


class OracleMap:
    """What Matcher::Track reads and writes of LocalMap: poses, intrinsics, points, per-frame observations."""

    def __init__(self, k, q, t, frame_camera, X=None, flags=None, uncertainty=None):
        self.k = [list(map(float, k[7 * c:7 * c + 7])) for c in range(len(k) // 7)]
        self.q = [list(map(float, q[4 * f:4 * f + 4])) for f in range(len(frame_camera))]
        self.t = [list(map(float, t[3 * f:3 * f + 3])) for f in range(len(frame_camera))]
        self.frame_camera = [int(c) for c in frame_camera]
        n = 0 if X is None else len(X) // 4
        self.X = [list(map(float, X[4 * i:4 * i + 4])) for i in range(n)]
        self.flags = [int(f) for f in flags] if flags is not None else []
        self.uncertainty = [float(u) for u in uncertainty] if uncertainty is not None else []
        self.obs = {f: [] for f in range(len(frame_camera))}     # frame -> [(x, y, point)]
        self.keyframe = [0] * len(frame_camera)

    def add_point(self, X):                                      # LocalMap::AddPoint (localmap.cpp:103-109)
        self.X.append(list(X))
        self.flags.append((1 << NO_OBSERVATIONS) | (1 << NO_BASELINE))
        self.uncertainty.append(1e8)
        return len(self.X) - 1


def feature_usable(flags):                                       # localmap.h:249
    return not (flags & (1 << MISMATCHED)) and not (flags & (1 << BAD_LOCATION))


def pixel_to_plane(k, px, py):                                   # localmap.h:55-78
    xp, yp = px, py
    xp -= k[5]
    yp -= k[6]
    xp /= k[3]
    yp /= k[4]
    x0, y0 = xp, yp
    for _ in range(3):
        r2 = xp * xp + yp * yp
        distort = 1. / (1.0 + r2 * (k[0] + r2 * (k[1] + r2 * k[2])))
        xp = x0 * distort
        yp = y0 * distort
    return xp, yp


def unproject(q, t, plane, distance):                            # localmap.cpp:29-37 with Eigen semantics
    v = [plane[0] * distance, plane[1] * distance, distance]
    n2 = q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3]
    qi = [-q[0] / n2, -q[1] / n2, -q[2] / n2, q[3] / n2] if n2 > 0 else [0.0] * 4   # Quaternion::inverse
    uv = [qi[1] * v[2] - qi[2] * v[1], qi[2] * v[0] - qi[0] * v[2], qi[0] * v[1] - qi[1] * v[0]]
    uv = [a + a for a in uv]                                     # _transformVector: uv = 2 vec x v
    cx = [qi[1] * uv[2] - qi[2] * uv[1], qi[2] * uv[0] - qi[0] * uv[2], qi[0] * uv[1] - qi[1] * uv[0]]
    p = [(v[i] + qi[3] * uv[i]) + cx[i] + t[i] for i in range(3)]
    nrm = math.sqrt(p[0] * p[0] + p[1] * p[1] + p[2] * p[2] + 1.0 * 1.0)   # Vector4d::normalize
    return [p[0] / nrm, p[1] / nrm, p[2] / nrm, 1.0 / nrm]


class OracleMatcher:
    def __init__(self):
        self.features = {}        # point id -> {"point": idx, "matches": [(view_seq, x, y)]}
        self.views = []           # [{"seq", "frame", "pyr", "dims", "w", "h"}]
        self.next_fid = 0
        self.next_seq = 0
        self.last_stats = None

    def _view(self, seq):
        return next(v for v in self.views if v["seq"] == seq)

    def _track(self, from_view, from_pt, to_view, levels, to_pt):
        """TrackFeature (matcher.cpp:173-206) + the retry of FindMatches (247-251)."""
        out, acc, _ = oracle.track_fb(from_view["pyr"], to_view["pyr"], from_view["dims"], WINDOW,
                                      np.float32([from_pt]), np.float32([to_pt]), np.int32([levels]))
        return bool(acc[0]), (out[0, 0], out[0, 1])

    def _find_matches(self, m: OracleMap, view, matches):
        """FindMatches (matcher.cpp:210-271), one feature at a time in id order."""
        f_to = view["frame"]
        q, t, k = m.q[f_to], m.t[f_to], m.k[m.frame_camera[f_to]]
        for fid in sorted(self.features):
            if fid in matches:
                continue
            feat = self.features[fid]
            p = feat["point"]
            for seq, fx, fy in feat["matches"]:
                from_view = self._view(seq)
                to_pt = (np.float32(fx), np.float32(fy))
                levels = 6 if m.uncertainty[p] > 100 else 3
                if m.uncertainty[p] < 100:
                    uv, ok = oracle.project(np.array(q), np.array(t), np.array(k), np.array(m.X[p]))
                    if ok[0]:
                        to_pt = (np.float32(uv[0, 0]), np.float32(uv[0, 1]))
                if to_pt[0] < 0 or to_pt[1] < 0 or to_pt[0] >= view["w"] or to_pt[1] > view["h"]:
                    continue
                good, pt = self._track(from_view, (fx, fy), view, levels, to_pt)
                if not good:
                    continue          # (the retry with 6 levels is inside _track, as in TrackFB)
                matches[fid] = pt
                m.obs[f_to].append((float(pt[0]), float(pt[1]), p))
                break

    def Track(self, img, frame, m: OracleMap, update_frames=None):
        img = np.ascontiguousarray(img, dtype=np.uint8)
        h, w = img.shape[:2]
        pyr, dims = oracle.make_pyramid(img, DEPTH)
        view = {"seq": self.next_seq, "frame": frame, "pyr": pyr, "dims": dims, "w": w, "h": h}
        self.next_seq += 1
        for fid in [f for f, v in self.features.items() if not feature_usable(m.flags[v["point"]])]:
            del self.features[fid]
        matches = {}
        self._find_matches(m, view, matches)
        st = {"matches_first": len(matches)}
        if len(matches) < MIN_MATCHES and update_frames is not None and update_frames():
            self._find_matches(m, view, matches)
        st["matches"] = len(matches)
        st.update(keyframe=0, corners=0, added=0)
        if len(matches) >= MIN_MATCHES:
            st.update(features=len(self.features), views=len(self.views))
            self.last_stats = st
            return True
        m.keyframe[frame] = 1
        for fid, pt in matches.items():
            self.features[fid]["matches"].append((view["seq"], pt[0], pt[1]))
        self.views.append(view)
        mxy = np.float32([matches[f] for f in sorted(matches)]).reshape(-1, 2)
        corners, added = oracle.seed_features(img, mxy)
        st.update(keyframe=1, corners=len(corners), added=len(added))
        q, t, k = m.q[frame], m.t[frame], m.k[m.frame_camera[frame]]
        for px, py in added:
            plane = pixel_to_plane(k, float(px), float(py))
            X = unproject(q, t, plane, INITIAL_DEPTH)
            fid = self.next_fid
            self.next_fid += 1
            p = m.add_point(X)
            m.obs[frame].append((float(px), float(py), p))
            self.features[fid] = {"point": p, "matches": [(view["seq"], px, py)]}
        if len(self.views) > MAX_VIEWS:
            old = self.views.pop(0)
            for feat in self.features.values():
                feat["matches"] = [mt for mt in feat["matches"] if mt[0] != old["seq"]]
        st.update(features=len(self.features), views=len(self.views))
        self.last_stats = st
        return True
