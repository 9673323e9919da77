"""Reference sample cameras and the synthetic workload generator.

Parameter sets are the reference's fixtures /root/reference/samples/*.yaml
(copied verbatim to tests/golden/samples/), in factor order.  The synthetic
point cloud follows SURVEY.md §8(d): seed 20251205, x,y ~ U[-1,1),
z ~ U[0.5,4.0) (the distribution of examples/batch_processing.rs:305-325),
plus ~0.1% edge points that exercise every status branch.
"""
from __future__ import annotations

import numpy as np

from . import _lib

SEED = 20251205

# model id -> (params, (width, height)); samples/*.yaml
SAMPLES = {
    _lib.PINHOLE: ([461.629, 460.152, 362.680, 246.049], (752, 480)),
    _lib.RADTAN: ([461.629, 460.152, 362.680, 246.049,
                   -0.28340811, 0.07395907, 0.00019359, 1.76187114e-05, 0.0], (752, 480)),
    _lib.KANNALA_BRANDT: ([190.97847715128717, 190.9733070521226, 254.93170605935475,
                           256.8974428996504, 0.0034823894022493434, 0.0007150348452162257,
                           -0.0020532361418706202, 0.00020293673591811182], (512, 512)),
    _lib.DOUBLE_SPHERE: ([348.112754378549, 347.1109973814674, 365.8121721753254,
                          249.3555778487899, 0.5657413673629862, -0.24425190195168348],
                         (752, 480)),
    _lib.UCM: ([1313.83, 1313.27, 960.471, 546.981, 1.01674], (752, 480)),
    _lib.EUCM: ([1313.83, 1313.27, 960.471, 546.981, 1.01674, 0.5], (752, 480)),
    _lib.FOV: ([379.045, 379.008, 505.512, 509.969, 0.9259487501905697], (752, 480)),
}

MODEL_NAMES = {
    _lib.PINHOLE: "pinhole", _lib.RADTAN: "rad_tan", _lib.KANNALA_BRANDT: "kannala_brandt",
    _lib.DOUBLE_SPHERE: "double_sphere", _lib.UCM: "ucm", _lib.EUCM: "eucm", _lib.FOV: "fov",
}

EPS = 2.220446049250313e-16
EPS_SQRT = 1.4901161193847656e-08

# Points on every decision boundary the reference tests or implies.
EDGE_POINTS = np.array([
    [0.0, 0.0, 0.0], [0.1, 0.2, -1.0], [0.0, 0.0, 1e-9], [0.0, 0.0, 1.0],
    [0.0, 0.0, -0.0], [0.3, -0.2, EPS], [0.3, -0.2, EPS / 2], [0.3, -0.2, EPS_SQRT],
    [0.3, -0.2, np.nextafter(EPS_SQRT, 0.0)], [0.3, -0.2, np.nextafter(EPS_SQRT, 1.0)],
    [1e-17, 0.0, 1.0], [0.0, 1e-300, 2.0], [EPS, 0.0, 1.0], [-EPS, EPS, 1.0],
    [5.0, 5.0, 0.01], [-5.0, 3.0, -0.5], [1.0, 0.0, -1.0], [0.0, 1.0, 0.0],
    [1e3, -1e3, 1.0], [0.5, 0.0, 2.0], [-0.5, 0.0, 2.0], [0.0, 0.5, 2.0],
    [0.0, -0.5, 2.0], [0.1, 0.1, 3.0], [0.5, -0.3, 2.0], [0.1, 0.2, 1.0],
    [np.inf, 0.0, 1.0], [0.0, 0.0, np.inf], [np.nan, 0.0, 1.0], [0.0, 0.0, np.nan],
], dtype=np.float64)


def synthetic_points(n: int, seed: int = SEED, edge_fraction: float = 1e-3,
                     offset: int = 0) -> np.ndarray:
    """(n, 3) float64 AoS point cloud (host).  `offset` = shard start for ranks."""
    rng = np.random.Generator(np.random.Philox(key=seed + offset))
    pts = np.empty((n, 3), dtype=np.float64)
    pts[:, 0] = rng.uniform(-1.0, 1.0, n)
    pts[:, 1] = rng.uniform(-1.0, 1.0, n)
    pts[:, 2] = rng.uniform(0.5, 4.0, n)
    n_edge = int(n * edge_fraction)
    if n_edge:
        idx = rng.choice(n, size=n_edge, replace=False)
        pts[idx] = EDGE_POINTS[rng.integers(0, len(EDGE_POINTS), n_edge)]
    return pts


def synthetic_points_device(n: int, seed: int = SEED, offset: int = 0, layout: str = "aos"):
    """Same distribution generated directly in HBM (torch Philox on the GPU);
    used for the 10M-point bench so the inputs are resident before timing."""
    import torch
    g = torch.Generator(device="cuda")
    g.manual_seed(seed + offset)
    pts = torch.empty((3, n), dtype=torch.float64, device="cuda")
    pts[0].uniform_(-1.0, 1.0, generator=g)
    pts[1].uniform_(-1.0, 1.0, generator=g)
    pts[2].uniform_(0.5, 4.0, generator=g)
    n_edge = n // 1000
    if n_edge:
        idx = torch.randint(0, n, (n_edge,), device="cuda", generator=g)
        e = torch.as_tensor(EDGE_POINTS, device="cuda")
        pick = torch.randint(0, len(EDGE_POINTS), (n_edge,), device="cuda", generator=g)
        pts[:, idx] = e[pick].t()
    if layout == "soa":
        return pts.contiguous()
    return pts.t().contiguous()
