"""Two interchangeable backends with one signature, so the same known-answer
tests run against the CPU oracle (``-m "not gpu"``) and against libacm.so's
HIP kernels (``-m gpu``).

project(model, params, w, h, pts(N,3)) -> uv (N,2), status (N,), jac (P,N,2)
unproject(model, params, w, h, uv(N,2)) -> rays (N,3), status (N,)
"""
import numpy as np

MODEL_IDS = {"pinhole": 0, "rad_tan": 1, "kannala_brandt": 2, "double_sphere": 3, "ucm": 4,
             "eucm": 5, "fov": 6}
STATUS = {"Ok": 0, "ProjectionOutSideImage": 1, "PointIsOutSideImage": 2,
          "PointAtCameraCenter": 3, "NumericalError": 4}
NUM_PARAMS = {0: 4, 1: 9, 2: 8, 3: 6, 4: 5, 5: 6, 6: 5}


class OracleBackend:
    name = "oracle"

    def __init__(self):
        import oracle
        self.O = oracle

    def project(self, model, params, w, h, pts, want_jac=True):
        return self.O.project(model, params, w, h, pts, want_jac)

    def unproject(self, model, params, w, h, uv):
        return self.O.unproject(model, params, w, h, uv)


class GpuBackend:
    name = "gpu"

    def __init__(self):
        import torch
        import apex_camera_models as acm
        self.torch = torch
        self.acm = acm

    def _model(self, model, params, w, h):
        from apex_camera_models.camera import MODEL_CLASSES
        cls = {0: "pinhole", 1: "rad_tan", 2: "kannala_brandt", 3: "double_sphere", 4: "ucm",
               5: "eucm", 6: "fov"}[model]
        m = MODEL_CLASSES[cls]._from_params([float(p) for p in params],
                                            self.acm.Resolution(w, h))
        return m

    def project(self, model, params, w, h, pts, want_jac=True, layout="aos"):
        m = self._model(model, params, w, h)
        pts = np.ascontiguousarray(pts, dtype=np.float64).reshape(-1, 3)
        t = self.torch.as_tensor(pts if layout == "aos" else pts.T.copy(), device="cuda")
        uv, st, jac = m.project_batch(t, jacobian=want_jac, layout=layout)
        self.torch.cuda.synchronize()
        return (uv.cpu().numpy(), st.cpu().numpy(),
                jac.cpu().numpy() if jac is not None else None)

    def round_trip(self, model, params, w, h, pts, layout="aos"):
        """acm_project_unproject: (uv, status, rays (N,3), ray_status)"""
        m = self._model(model, params, w, h)
        pts = np.ascontiguousarray(pts, dtype=np.float64).reshape(-1, 3)
        t = self.torch.as_tensor(pts if layout == "aos" else pts.T.copy(), device="cuda")
        uv, st, rays, st2 = m.project_unproject_batch(t, layout=layout)
        self.torch.cuda.synchronize()
        r = rays.cpu().numpy()
        if layout == "soa":
            r = r.T.copy()
        return uv.cpu().numpy(), st.cpu().numpy(), r, st2.cpu().numpy()

    def unproject(self, model, params, w, h, uv, layout="aos", reference_newton=False):
        m = self._model(model, params, w, h)
        t = self.torch.as_tensor(np.ascontiguousarray(uv, dtype=np.float64).reshape(-1, 2),
                                 device="cuda")
        rays, st = m.unproject_batch(t, layout=layout, reference_newton=reference_newton)
        self.torch.cuda.synchronize()
        r = rays.cpu().numpy()
        if layout == "soa":
            r = r.T.copy()
        return r, st.cpu().numpy()


def parse_params(params):
    return [float(p) if not isinstance(p, str) else float(p) for p in params]


def rel_err(a, b, floor=0.0):
    """max |a-b| / max(|b|, floor) over finite entries; NaN positions must match."""
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    na, nb = np.isnan(a), np.isnan(b)
    assert np.array_equal(na, nb), "NaN pattern differs"
    m = ~nb
    if not m.any():
        return 0.0
    d = np.abs(a[m] - b[m])
    s = np.maximum(np.abs(b[m]), floor)
    with np.errstate(divide="ignore", invalid="ignore"):
        r = np.where(d == 0, 0.0, d / np.where(s == 0, np.inf, s))
    r = np.where((d != 0) & (s == 0), np.inf, r)
    return float(r.max())
