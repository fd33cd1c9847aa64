"""Writes tests/golden/reference_kats.json: the known-answer vectors izpi's own Go
tests hold for the hot path, transcribed as data (inputs + expected outputs).

Sources (read-only reference, /root/reference/internal):
  hitable/bvh4_simd_test.go:67-157   RayAABB4 masks, 7 cases ("expected")
  hitable/bvh4_test.go:160-278       RayAABB4 with +Inf inverse directions, 3 cases
  hitable/triangle_test.go:15-134    NewTriangleWithUV fields; Triangle.Hit 4 cases
  grid/grid_test.go:9-77             spiral tile order 3x3, 4x4, 5x5
  material/dielectric_test.go:28-45  Beer-Lambert exp(-0.5*1) = 0.6065 +- 1e-3
  material/dielectric_test.go:47-84  calculatePathLength against mockSceneGeometry (its Hit
                                     always returns the exit point (0.5, 0.5, 1.5)): the hit
                                     point (0.5, 0.5, 0.5) is 1.0 from it, inside the
                                     [0.1, 10] bounds the test asserts; the exact 1.0 is
                                     Length(exit - p) by dielectric.go:141-150
  mat3/mat3_test.go:10-54            MatrixVectorMul of the identity and of NewTBN(t, b, n)
                                     for the XY, XZ and YZ planes, exact (cmp.Diff)
  fastrandom/fastrandom.go:41-47     LCG seed 12345 (dielectric_test.go:108): derived
                                     here by exact integer arithmetic.
Run: python tests/golden/make_golden.py
"""
import json
from pathlib import Path

F32_MAX = 3.4028234663852886e38
INF = "inf"


def lcg(seed, n):
    s, out, st = seed, [], []
    for _ in range(n):
        s = (1664525 * s + 1013904223) % 4294967296
        st.append(s)
        out.append(s / 4294967296.0)
    return out, st


def main():
    aabb = [
        # name, org, invdir, minX, minY, minZ, maxX, maxY, maxZ, tmax, expected
        ("All hits", [0, 0, 0], [1, 1, 1], [1, 2, 3, 4], [1, 2, 3, 4], [1, 2, 3, 4], [2, 3, 4, 5], [2, 3, 4, 5], [2, 3, 4, 5], 100, 0b1111),
        ("No hits - ray pointing away", [0, 0, 0], [-1, -1, -1], [1, 2, 3, 4], [1, 2, 3, 4], [1, 2, 3, 4], [2, 3, 4, 5], [2, 3, 4, 5], [2, 3, 4, 5], 100, 0),
        ("tMax cutoff", [0, 0, 0], [1, 1, 1], [1, 2, 10, 20], [1, 2, 10, 20], [1, 2, 10, 20], [2, 3, 11, 21], [2, 3, 11, 21], [2, 3, 11, 21], 5, 0b0011),
        ("origin inside AABB", [1.5, 1.5, 1.5], [1, 1, 1], [1, 5, 5, 5], [1, 5, 5, 5], [1, 5, 5, 5], [2, 6, 6, 6], [2, 6, 6, 6], [2, 6, 6, 6], 100, 0b1111),
        ("Negative direction components", [5, 5, 5], [-1, -1, -1], [1, 2, 3, 6], [1, 2, 3, 6], [1, 2, 3, 6], [2, 3, 4, 7], [2, 3, 4, 7], [2, 3, 4, 7], 10, 0b0111),
        ("Mixed directions", [0, 0, 0], [1, 1, -1], [1, 1, 1, 1], [1, 1, 1, 1], [-2, 1, -2, 1], [2, 2, 2, 2], [2, 2, 2, 2], [-1, 2, -1, 2], 100, 0b0101),
        ("Infinite ray direction", [0, 5, 5], [1, F32_MAX, F32_MAX], [1, 2, 3, 4], [4, 4, 6, 6], [4, 4, 6, 6], [2, 3, 4, 5], [6, 6, 7, 7], [6, 6, 7, 7], 100, 0b0011),
        # bvh4_test.go: +Inf inverse x/y, ray down -z; expectation: only box 0 / all / none
        ("TestRayAABB4_SIMD", [0, 0, 0], [INF, INF, -1], [-1, 10, -1, 10], [-1, -1, 10, 10], [-10, -10, -10, -10], [1, 12, 1, 12], [1, 1, 12, 12], [-2, -2, -2, -2], 100, 0b0001),
        ("TestRayAABB4_SIMD_AllHit", [0, 0, 0], [INF, INF, -1], [-2, -2, -2, -2], [-2, -2, -2, -2], [-10, -10, -10, -10], [2, 2, 2, 2], [2, 2, 2, 2], [-1, -1, -1, -1], 100, 0b1111),
        ("TestRayAABB4_SIMD_NoneHit", [0, 0, 0], [INF, INF, -1], [-2, -2, -2, -2], [-2, -2, -2, -2], [1, 1, 1, 1], [2, 2, 2, 2], [2, 2, 2, 2], [10, 10, 10, 10], 100, 0),
    ]
    tri_new = {
        "v0": [0, 0, 0], "v1": [-1, 0, 0], "v2": [0, 1, 0], "uv": [0, 0, 1, 0, 0, 1],
        "edge1": [-1, 0, 0], "edge2": [0, 1, 0], "normal": [0, 0, -1], "tangent": [-1, 0, 0], "bitangent": [0, 1, 0],
        "area": 0.5, "bb_min": [-1.0001, -0.0001, -0.0001], "bb_max": [0.0001, 1.0001, 0.0001],
    }
    tri_hit = [
        {"name": "parallel", "tri": [[1, 0, -1], [1, 1, -1], [0, 0, -1]], "ray": [[0, -1, 0], [0, 1, 0]], "hit": False},
        {"name": "perpendicular hit", "tri": [[.5, -.5, -10], [0, .5, -10], [-.5, -.5, -10]], "ray": [[0, 0, 1], [0, 0, -1]],
         "hit": True, "t": 11, "p": [0, 0, -10], "n": [0, 0, 1]},
        {"name": "perpendicular miss", "tri": [[.5, -.5, -10], [0, .5, -10], [-.5, -.5, -10]], "ray": [[-1, 0, 1], [-1, 0, -1]], "hit": False},
        {"name": "angled hit", "tri": [[.5, -.5, -20], [0, .5, -10], [-.5, -.5, -10]], "ray": [[0, 0, 1], [0, 0, -1]],
         "hit": True, "t": 13.5, "p": [0, 0, -12.5], "n": [0.8908708063747479, -0.44543540318737396, 0.0890870806374748]},
    ]
    spiral = {
        "3x3": [[1, 1], [1, 0], [2, 0], [2, 1], [2, 2], [1, 2], [0, 2], [0, 1], [0, 0]],
        "4x4": [[2, 2], [2, 1], [3, 1], [3, 2], [3, 3], [2, 3], [1, 3], [1, 2], [1, 1], [1, 0], [2, 0], [3, 0],
                [0, 3], [0, 2], [0, 1], [0, 0]],
        "5x5": [[2, 2], [2, 1], [3, 1], [3, 2], [3, 3], [2, 3], [1, 3], [1, 2], [1, 1], [1, 0], [2, 0], [3, 0],
                [4, 0], [4, 1], [4, 2], [4, 3], [4, 4], [3, 4], [2, 4], [1, 4], [0, 4], [0, 3], [0, 2], [0, 1], [0, 0]],
    }
    vals, states = lcg(12345, 4)
    out = {
        "ray_aabb4": [dict(zip(["name", "org", "invdir", "min_x", "min_y", "min_z", "max_x", "max_y", "max_z", "tmax", "expected"], c)) for c in aabb],
        "new_triangle_with_uv": tri_new,
        "triangle_hit": tri_hit,
        "spiral": spiral,
        "beer_lambert": {"peak": 0.5, "center": 480.0, "width": 60.0, "lambda": 480.0, "path": 1.0, "expected": 0.6065, "tol": 1e-3},
        "lcg_seed_12345": {"values": vals, "states": states},
        # mat3_test.go: (t, b, n) are the matrix's columns (NewTBN, mat3.go:19-31); the
        # identity case is Mat3{A11: 1, A22: 1, A33: 1}, i.e. columns x, y, z
        "mat3_tbn": [
            {"name": "Multiply by identity", "t": [1, 0, 0], "b": [0, 1, 0], "n": [0, 0, 1], "v": [1, 2, 3], "want": [1, 2, 3]},
            {"name": "TBN XY plane", "t": [-1, 0, 0], "b": [0, 1, 0], "n": [0, 0, -1], "v": [0, 0, 1], "want": [0, 0, -1]},
            {"name": "TBN XZ plane", "t": [-1, 0, 0], "b": [0, 0, 1], "n": [0, 1, 0], "v": [0, 0, 1], "want": [0, 1, 0]},
            {"name": "TBN YZ plane", "t": [0, 0, 1], "b": [0, 1, 0], "n": [-1, 0, 0], "v": [0, 0, 1], "want": [-1, 0, 0]},
        ],
        "path_length": {"hit_p": [0.5, 0.5, 0.5], "hit_n": [0.577, 0.577, 0.577], "ray_o": [0, 0, -2], "ray_d": [0, 0, 1],
                        "scattered_d": [0, 0, 1], "mock_exit": [0.5, 0.5, 1.5], "bounds": [0.1, 10.0], "expected": 1.0},
    }
    (Path(__file__).parent / "reference_kats.json").write_text(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
