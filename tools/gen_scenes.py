#!/usr/bin/env python3
"""Synthetic scenes for BASELINE configs 3-5, written in the
reference's JSON scene format (Raytracer.cpp:645-779; mesh items carry v, n and t,
`type` only on data[0], :606-616). Deterministic: seed 580.

  cornell10k   config 3: Cornell box — 5 tessellated walls + a tessellated block
               + a tessellated sphere = 10,000 triangles; walls Ks=0.1 Kt=0; the
               glossy block Ks=0.5 Kt=0.3; ambient + directional + point light.
  field100k    config 4: displaced grid (vertex jitter U(-0.01,0.01)) + a field of
               icospheres = 100,000+ triangles.
  field1m      config 5: the same construction at 1,000,000+ triangles.

usage: gen_scenes.py <out_dir> [cornell10k field100k field1m]
Writes <out_dir>/Assets/<scene>.json and its meshes; skips files already present
with the same generator version (a .stamp file).
"""
import json
import math
import os
import sys

import numpy as np

VERSION = "1"
SEED = 580


def fmt(x):
    return "%.6g" % float(x)


def write_mesh(path, verts, norms, tris):
    """verts/norms: (V,3) float32; tris: (T,3) int -> reference mesh JSON."""
    with open(path, "w") as f:
        f.write('{"data": [\n')
        for i, (a, b, c) in enumerate(tris):
            items = []
            for k, vi in (("v0", a), ("v1", b), ("v2", c)):
                v, n = verts[vi], norms[vi]
                items.append('"%s": {"v": [%s, %s, %s], "n": [%s, %s, %s], "t": [0, 0]}' % (
                    k, fmt(v[0]), fmt(v[1]), fmt(v[2]), fmt(n[0]), fmt(n[1]), fmt(n[2])))
            head = '"type": "polygon", ' if i == 0 else ""
            f.write("  {%s%s}%s\n" % (head, ", ".join(items), "," if i + 1 < len(tris) else ""))
        f.write("]}\n")


def grid(nx, nz, size_x, size_z, jitter, rng, height_fn=None):
    xs = np.linspace(-size_x / 2, size_x / 2, nx + 1)
    zs = np.linspace(-size_z / 2, size_z / 2, nz + 1)
    X, Z = np.meshgrid(xs, zs, indexing="xy")
    Y = height_fn(X, Z) if height_fn else np.zeros_like(X)
    V = np.stack([X, Y, Z], axis=-1).reshape(-1, 3)
    if jitter:
        V = V + rng.uniform(-jitter, jitter, size=V.shape)
    idx = np.arange((nx + 1) * (nz + 1)).reshape(nz + 1, nx + 1)
    a, b, c, d = idx[:-1, :-1], idx[:-1, 1:], idx[1:, 1:], idx[1:, :-1]
    # counter-clockwise seen from +y
    t1 = np.stack([a, d, c], axis=-1).reshape(-1, 3)
    t2 = np.stack([a, c, b], axis=-1).reshape(-1, 3)
    T = np.empty((t1.shape[0] * 2, 3), dtype=np.int64)
    T[0::2], T[1::2] = t1, t2
    return V.astype(np.float32), T


def vertex_normals(V, T):
    N = np.zeros_like(V, dtype=np.float64)
    fn = np.cross(V[T[:, 1]] - V[T[:, 0]], V[T[:, 2]] - V[T[:, 0]])
    for k in range(3):
        np.add.at(N, T[:, k], fn)
    N /= np.maximum(np.linalg.norm(N, axis=1, keepdims=True), 1e-12)
    return N.astype(np.float32)


def icosphere(level):
    t = (1.0 + 5 ** 0.5) / 2
    V = [(-1, t, 0), (1, t, 0), (-1, -t, 0), (1, -t, 0), (0, -1, t), (0, 1, t), (0, -1, -t), (0, 1, -t),
         (t, 0, -1), (t, 0, 1), (-t, 0, -1), (-t, 0, 1)]
    V = [np.array(v) / np.linalg.norm(v) for v in V]
    F = [(0, 11, 5), (0, 5, 1), (0, 1, 7), (0, 7, 10), (0, 10, 11), (1, 5, 9), (5, 11, 4), (11, 10, 2),
         (10, 7, 6), (7, 1, 8), (3, 9, 4), (3, 4, 2), (3, 2, 6), (3, 6, 8), (3, 8, 9), (4, 9, 5), (2, 4, 11),
         (6, 2, 10), (8, 6, 7), (9, 8, 1)]
    for _ in range(level):
        cache = {}

        def mid(i, j):
            key = (min(i, j), max(i, j))
            if key not in cache:
                m = V[i] + V[j]
                V.append(m / np.linalg.norm(m))
                cache[key] = len(V) - 1
            return cache[key]
        nf = []
        for a, b, c in F:
            ab, bc, ca = mid(a, b), mid(b, c), mid(c, a)
            nf += [(a, ab, ca), (b, bc, ab), (c, ca, bc), (ab, bc, ca)]
        F = nf
    V = np.array(V, dtype=np.float32)
    return V, np.array(F, dtype=np.int64)


def box(n):
    """Unit cube [-0.5,0.5]^3, each face an n x n grid (12 n^2 triangles), outward."""
    Vs, Ts, off = [], [], 0
    for axis in range(3):
        for sgn in (-1.0, 1.0):
            V, T = grid(n, n, 1.0, 1.0, 0.0, None)
            # grid lies in xz at y=0 with normal +y; rotate so normal = sgn * e_axis
            P = np.zeros_like(V)
            u, v = [(1, 2), (2, 0), (0, 1)][axis]
            P[:, axis] = 0.5 * sgn
            P[:, u] = V[:, 0]
            P[:, v] = V[:, 2]
            # orientation: make the face normal point outward
            fn = np.cross(P[T[0, 1]] - P[T[0, 0]], P[T[0, 2]] - P[T[0, 0]])
            if fn[axis] * sgn < 0:
                T = T[:, ::-1]
            Vs.append(P)
            Ts.append(T + off)
            off += len(P)
    V = np.concatenate(Vs).astype(np.float32)
    T = np.concatenate(Ts)
    return V, T


def mat(cs, ka, kd, ks, kt, n):
    return {"Cs": [float(x) for x in cs], "Ka": ka, "Kd": kd, "Ks": ks, "Kt": kt, "n": n}


def shape(sid, geo, material, S=(1, 1, 1), T=(0, 0, 0), R=None):
    """T is the desired world position of the local origin. ComputeModelMatrix
    (Raytracer.h) composes S*R*T (p' = S R (p + t)), so pass t = R^T S^-1 T to land
    the object at T (only Ry is used here)."""
    u = [t / s for t, s in zip(T, S)]
    th = math.radians((R or {}).get("Ry", 0.0))
    c, s_ = math.cos(th), math.sin(th)
    T = [round(c * u[0] - s_ * u[2], 6), round(u[1], 6), round(s_ * u[0] + c * u[2], 6)]
    tr = []
    if R:
        tr += [{k: v} for k, v in R.items()]
    tr += [{"S": list(S)}, {"T": list(T)}]
    return {"id": sid, "geometry": geo, "material": material, "transforms": tr}


def scene_json(shapes, lights, cam_from, cam_to, res):
    return {"scene": {"shapes": shapes, "lights": lights,
                      "camera": {"from": cam_from, "to": cam_to, "bounds": [0.1, 100, 1, -1, 1, -1],
                                 "resolution": res}}}


def gen_cornell10k(assets):
    rng = np.random.default_rng(SEED)
    # walls: 5 faces of a 10-unit box (open towards the camera), 10x10 grids -> 5*200 = 1000 tris
    Vw, Tw = [], []
    off = 0
    V, T = grid(10, 10, 10.0, 10.0, 0.0, rng)
    for (rot, trans, flip) in [
            (lambda p: p, (0, -5, 0), False),                         # floor, normal +y
            (lambda p: p * np.array([1, -1, 1]), (0, 5, 0), True),    # ceiling, normal -y
            (lambda p: p[:, [0, 2, 1]], (0, 0, -5), True),            # back wall, normal +z
            (lambda p: p[:, [1, 0, 2]], (-5, 0, 0), True),            # left wall, normal +x
            (lambda p: p[:, [1, 0, 2]] * np.array([-1, 1, 1]), (5, 0, 0), False)]:  # right wall, normal -x
        P = rot(V.astype(np.float64)) + np.array(trans)
        TT = T[:, ::-1] if flip else T
        Vw.append(P)
        Tw.append(TT + off)
        off += len(P)
    Vw = np.concatenate(Vw).astype(np.float32)
    Tw = np.concatenate(Tw)
    write_mesh(os.path.join(assets, "cornell_walls.json"), Vw, vertex_normals(Vw, Tw), Tw)
    # glossy block: 12*n^2 with n=16 -> 3072 tris
    Vb, Tb = box(16)
    write_mesh(os.path.join(assets, "cornell_block.json"), Vb, vertex_normals(Vb, Tb), Tb)
    # sphere: icosphere level 5 = 20480 -> too many; UV sphere with 5928 tris
    total_target = 10000 - len(Tw) - len(Tb)
    Vs, Ts = uv_sphere_exact(total_target)
    write_mesh(os.path.join(assets, "cornell_sphere.json"), Vs, vertex_normals(Vs, Ts), Ts)
    shapes = [
        shape("walls", "cornell_walls", mat((0.75, 0.75, 0.75), 0.3, 0.7, 0.1, 0.0, 20)),
        shape("block", "cornell_block", mat((0.9, 0.6, 0.3), 0.3, 0.6, 0.5, 0.3, 64),
              S=(2.5, 4.0, 2.5), T=(-2.0, -3.0, -1.5), R={"Ry": 25}),
        shape("ball", "cornell_sphere", mat((0.3, 0.5, 0.9), 0.3, 0.7, 0.2, 0.0, 120),
              S=(1.8, 1.8, 1.8), T=(2.2, -3.2, 1.0)),
    ]
    lights = [
        {"id": "amb", "type": "ambient", "color": [1, 1, 1], "intensity": 0.25},
        {"id": "sun", "type": "directional", "color": [1, 0.95, 0.9], "intensity": 0.6,
         "from": [3, 10, 8], "to": [0, 0, 0]},
        {"id": "lamp", "type": "point", "color": [1, 1, 1], "intensity": 0.5, "position": [0, 4.5, 1]},
    ]
    n = len(Tw) + len(Tb) + len(Ts)
    assert n == 10000, n
    return scene_json(shapes, lights, [0, 0, 12.5], [0, -0.3, 0], [1920, 1080]), n


def uv_sphere_exact(n_tris):
    """Unit UV sphere with exactly n_tris triangles (2*lon per inner band, lon per cap)."""
    best = None
    for n_lon in range(8, 400):
        # tris = 2*n_lon*(n_lat-2) + 2*n_lon  (two caps of n_lon each)
        if (n_tris - 2 * n_lon) % (2 * n_lon) == 0:
            n_lat = (n_tris - 2 * n_lon) // (2 * n_lon) + 2
            if n_lat >= 3 and abs(n_lat - n_lon / 2) < (abs(best[0] - best[1] / 2) if best else 1e9):
                best = (n_lat, n_lon)
    assert best, n_tris
    n_lat, n_lon = best
    V = [(0.0, 1.0, 0.0)]
    for i in range(1, n_lat):
        th = math.pi * i / n_lat
        for j in range(n_lon):
            ph = 2 * math.pi * j / n_lon
            V.append((math.sin(th) * math.cos(ph), math.cos(th), math.sin(th) * math.sin(ph)))
    V.append((0.0, -1.0, 0.0))
    V = np.array(V, dtype=np.float32)
    T = []
    ring = lambda i, j: 1 + (i - 1) * n_lon + (j % n_lon)
    for j in range(n_lon):
        T.append((0, ring(1, j + 1), ring(1, j)))
    for i in range(1, n_lat - 1):
        for j in range(n_lon):
            a, b, c, d = ring(i, j), ring(i, j + 1), ring(i + 1, j + 1), ring(i + 1, j)
            T += [(a, b, c), (a, c, d)]
    last = len(V) - 1
    for j in range(n_lon):
        T.append((last, ring(n_lat - 1, j), ring(n_lat - 1, j + 1)))
    T = np.array(T, dtype=np.int64)
    assert len(T) == n_tris, (len(T), n_tris)
    return V, T


def gen_field(assets, name, grid_nxz, n_spheres, ico_level):
    rng = np.random.default_rng(SEED)
    hf = lambda X, Z: 0.35 * np.sin(0.7 * X) * np.cos(0.5 * Z) + 0.15 * np.sin(2.3 * X + 1.7 * Z)
    V, T = grid(grid_nxz[0], grid_nxz[1], 24.0, 24.0, 0.01, rng, hf)
    write_mesh(os.path.join(assets, name + "_ground.json"), V, vertex_normals(V, T), T)
    Vi, Ti = icosphere(ico_level)
    Vi = (Vi + rng.uniform(-0.01, 0.01, size=Vi.shape)).astype(np.float32)
    write_mesh(os.path.join(assets, name + "_ico.json"), Vi, vertex_normals(Vi, Ti), Ti)
    shapes = [shape("ground", name + "_ground", mat((0.6, 0.65, 0.55), 0.3, 0.8, 0.2, 0.0, 30))]
    for k in range(n_spheres):
        x, z = rng.uniform(-8, 8), rng.uniform(-8, 4)
        r = rng.uniform(0.6, 1.4)
        glossy = k % 3 == 0
        shapes.append(shape("ico%d" % k, name + "_ico",
                            mat(rng.uniform(0.2, 1.0, 3).round(3), 0.3, 0.7, 0.5 if glossy else 0.1,
                                0.3 if glossy else 0.0, int(rng.integers(10, 200))),
                            S=(r, r, r), T=(round(x, 3), round(r + 0.3, 3), round(z, 3))))
    lights = [
        {"id": "amb", "type": "ambient", "color": [1, 1, 1], "intensity": 0.2},
        {"id": "sun", "type": "directional", "color": [1, 1, 0.95], "intensity": 0.8,
         "from": [4, 10, 6], "to": [0, 0, 0]},
    ]
    n = len(T) + n_spheres * len(Ti)
    assert n == {"field100k": 100000, "field1m": 1000000}[name], n
    return scene_json(shapes, lights, [0, 7, 13], [0, -1.5, -2], [3840, 2160]), n


SCENES = {
    "cornell10k": lambda a: gen_cornell10k(a),
    "field100k": lambda a: gen_field(a, "field100k", (200, 186), 5, 4),   # 74,400 + 5*5,120 = 100,000
    "field1m": lambda a: gen_field(a, "field1m", (800, 593), 10, 4),      # 948,800 + 10*5,120 = 1,000,000
}


def scene_files(name):
    """Every file under Assets/ that LoadSceneJSON reads for this scene."""
    if name == "cornell10k":
        return [name + ".json", "cornell_walls.json", "cornell_block.json", "cornell_sphere.json"]
    return [name + ".json", name + "_ground.json", name + "_ico.json"]


def ensure(out_dir, name):
    assets = os.path.join(out_dir, "Assets")
    os.makedirs(assets, exist_ok=True)
    stamp = os.path.join(assets, name + ".stamp")
    scene_path = os.path.join(assets, name + ".json")
    if os.path.exists(stamp) and open(stamp).read().strip() == VERSION and os.path.exists(scene_path):
        return json.load(open(stamp + ".json"))["triangles"]
    sc, n = SCENES[name](assets)
    with open(scene_path, "w") as f:
        json.dump(sc, f, indent=1)
    json.dump({"triangles": n}, open(stamp + ".json", "w"))
    open(stamp, "w").write(VERSION)
    return n


def main():
    out = sys.argv[1]
    names = sys.argv[2:] or list(SCENES)
    for n in names:
        print(n, ensure(out, n), "triangles", flush=True)


if __name__ == "__main__":
    main()
