"""Offline estimate: walk steps of the bunny's 4-wide tree built from the reference's
median-split BVH (BVH.cpp:30-99) vs from a binned-SAH BVH over the same triangles, for
random rays that pass the bunny's box (closest hit: every passing box is visited; shadow:
any-hit with early exit is not modelled, all passing boxes counted).
    python scripts/diag/bvh_sah_sim.py [NRAYS]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
OBJ = os.path.join(ROOT, "toypathtracer-games101-assignment7_amd", "models", "bunny_cornell.obj")


def load(path):
    v, f = [], []
    for line in open(path):
        p = line.split()
        if not p:
            continue
        if p[0] == "v":
            v.append([float(x) for x in p[1:4]])
        elif p[0] == "f":
            f.append([int(x.split("/")[0]) - 1 for x in p[1:4]])
    v = np.array(v, np.float32)
    return v[np.array(f)]  # T x 3 x 3


def build_median(tb, cen, idx):
    """reference: largest centroid extent axis, sort by centroid, split at the middle"""
    nodes = []  # (bmin, bmax, left, right, tri)

    def rec(ix):
        me = len(nodes)
        nodes.append(None)
        lo, hi = tb[ix, 0].min(0), tb[ix, 1].max(0)
        if len(ix) == 1:
            nodes[me] = (lo, hi, -1, -1, ix[0])
            return me
        c = cen[ix]
        ext = c.max(0) - c.min(0)
        d = int(np.argmax(ext))
        o = ix[np.argsort(c[:, d], kind="stable")]
        m = len(o) // 2
        l = rec(o[:m])
        r = rec(o[m:])
        nodes[me] = (lo, hi, l, r, -1)
        return me
    rec(idx)
    return nodes


def area(lo, hi):
    d = np.maximum(hi - lo, 0)
    return 2 * (d[..., 0] * d[..., 1] + d[..., 1] * d[..., 2] + d[..., 2] * d[..., 0])


def build_sah(tb, cen, idx, bins=32):
    nodes = []

    def rec(ix):
        me = len(nodes)
        nodes.append(None)
        lo, hi = tb[ix, 0].min(0), tb[ix, 1].max(0)
        if len(ix) == 1:
            nodes[me] = (lo, hi, -1, -1, ix[0])
            return me
        c = cen[ix]
        cl, ch = c.min(0), c.max(0)
        best = (np.inf, None)
        for d in range(3):
            if ch[d] <= cl[d]:
                continue
            b = np.minimum(((c[:, d] - cl[d]) / (ch[d] - cl[d]) * bins).astype(int), bins - 1)
            for s in range(1, bins):
                L = b < s
                nl = L.sum()
                if nl == 0 or nl == len(ix):
                    continue
                cost = area(tb[ix[L], 0].min(0), tb[ix[L], 1].max(0)) * nl + \
                    area(tb[ix[~L], 0].min(0), tb[ix[~L], 1].max(0)) * (len(ix) - nl)
                if cost < best[0]:
                    best = (cost, (d, L))
        if best[1] is None:
            o = ix[np.argsort(c[:, int(np.argmax(ch - cl))], kind="stable")]
            L = np.zeros(len(ix), bool)
            L[: len(ix) // 2] = True
            ix = o
        else:
            L = best[1][1]
        l = rec(ix[L])
        r = rec(ix[~L])
        nodes[me] = (lo, hi, l, r, -1)
        return me
    rec(idx)
    return nodes


def wide(nodes):
    """4-wide: a QNode lists its binary node's grandchildren (or a shallower leaf)"""
    q = []

    def ent(x, lv, out):
        n = nodes[x]
        if n[4] >= 0 or lv == 0:
            out.append(x)
        else:
            ent(n[3], lv - 1, out)
            ent(n[2], lv - 1, out)

    def rec(p):
        me = len(q)
        q.append(None)
        e = []
        ent(nodes[p][3], 1, e)
        ent(nodes[p][2], 1, e)
        kids = []
        for x in e:
            kids.append(("leaf", x) if nodes[x][4] >= 0 else ("node", rec(x)))
        q[me] = [(nodes[x][0], nodes[x][1], k) for x, k in zip(e, kids)]
        return me
    rec(0)
    return q


def slab(lo, hi, o, inv):
    a, b = (lo - o) * inv, (hi - o) * inv
    tmin = np.maximum(np.minimum(a, b).max(), 1.17549435e-38)
    tmax = min(np.maximum(a, b).min(), 3.40282347e38)
    return tmax > 0 and tmin <= tmax


def walk_steps(q, o, inv):
    steps, st = 0, [("node", 0)]
    while st:
        kind, x = st.pop()
        steps += 1
        if kind == "leaf":
            continue
        for lo, hi, k in q[x]:
            if slab(lo, hi, o, inv):
                st.append(k)
    return steps


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 3000
    tri = load(OBJ)
    tb = np.stack([tri.min(1), tri.max(1)], 1)
    cen = (tb[:, 0] + tb[:, 1]) * 0.5
    idx = np.arange(len(tri))
    med, sah = wide(build_median(tb, cen, idx)), wide(build_sah(tb, cen, idx))
    print("triangles %d, 4-wide nodes: median %d, SAH %d" % (len(tri), len(med), len(sah)))
    lo, hi = tb[:, 0].min(0), tb[:, 1].max(0)
    rng = np.random.default_rng(1)
    res = {"median": [], "sah": []}
    k = 0
    while k < n:
        o = rng.uniform([0, 0, 0], [556, 548, 559]).astype(np.float32)
        d = rng.normal(size=3).astype(np.float32)
        d /= np.linalg.norm(d)
        inv = (1.0 / d).astype(np.float32)
        if not slab(lo, hi, o, inv):
            continue
        k += 1
        res["median"].append(walk_steps(med, o, inv))
        res["sah"].append(walk_steps(sah, o, inv))
    for key, v in res.items():
        v = np.array(v)
        # a wave walks as long as its longest lane: mean of the max over groups of 19 lanes
        g = v[: len(v) // 19 * 19].reshape(-1, 19).max(1)
        print("%-6s steps per ray mean %.1f  p90 %.0f  max-of-19 mean %.1f" % (key, v.mean(), np.percentile(v, 90), g.mean()))


if __name__ == "__main__":
    main()
