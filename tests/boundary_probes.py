"""Points placed on every status threshold of the hot path (VERDICT r01 item
2), and an independent binary64 emulation of the reference's status
decisions to check them against.

Each probe family puts a continuous parameter t (a depth z, a pixel u) at
the real-valued root of the threshold equation (found in 60-digit mpmath),
then takes the double nearest to it and its neighbours up to +-8 ulps: the
f64-evaluated condition flips somewhere in that window, so every decision is
exercised right where a different operation order, an FMA contraction or a
non-IEEE division / square root would flip it.

`emulate_status` restates each decision from the Rust source (file:line) in
mpmath at 53-bit precision, round-to-nearest per operation -- binary64
arithmetic for these normal-range values, written independently of
oracle/acm_oracle.c and of the HIP kernels.

Families (sample parameters of samples/*.yaml unless noted):
  UCM / DS / EUCM project   denom = 1e-3, and the z vs -w d (UCM, DS) /
                            z vs denom (a-1)/(2a-1) (EUCM) conditions
  DS / UCM / EUCM unproject r^2 = 1/(2a-1) (DS), 1 - r^2 = 1e-3 and
                            r^2 = (1-a)^2/(2a-1) (UCM), det = 1e-3 and
                            r^2 = (1/b)(2a-1) (EUCM)
  KB project                r = EPS (the axis test), z = 0 and z = EPS
  KB unproject              ru = 1e-6 (the Newton gate), ru = 0
  Pinhole / RadTan project  z = sqrt(EPS), u = w and v = h bounds
  RadTan unproject          a near-singular Newton Jacobian (k1 = -1/3:
                            det ~ 1e-16 at the first step)
"""
import mpmath
import numpy as np

EPS = 2.220446049250313e-16
EPS_SQRT = 1.4901161193847656e-08
PI_HALF = 1.5707963267948966  # f64 std::f64::consts::PI / 2.0

S_UCM = [1313.83, 1313.27, 960.471, 546.981, 1.01674]
S_EUCM = [1313.83, 1313.27, 960.471, 546.981, 1.01674, 0.5]
S_DS = [348.112754378549, 347.1109973814674, 365.8121721753254, 249.3555778487899,
        0.5657413673629862, -0.24425190195168348]
S_KB = [190.97847715128717, 190.9733070521226, 254.93170605935475, 256.8974428996504,
        0.0034823894022493434, 0.0007150348452162257, -0.0020532361418706202,
        0.00020293673591811182]
S_PIN = [461.629, 460.152, 362.680, 246.049]
S_RT_SING = [500.0, 500.0, 320.0, 240.0, -1.0 / 3.0, 0.0, 0.0, 0.0, 0.0]


def _ulps(t, k=8):
    t = float(t)
    out = [t]
    lo = hi = t
    for _ in range(k):
        lo = float(np.nextafter(lo, -np.inf))
        hi = float(np.nextafter(hi, np.inf))
        out += [lo, hi]
    return out


def _root(f, t0):
    with mpmath.workdps(60):
        return mpmath.findroot(f, mpmath.mpf(t0))


def probes():
    """[(model, params, (w, h), kind, points)] with kind 'project' (N,3) or
    'unproject' (N,2)."""
    mp = mpmath
    out = []
    # ---- UCM project: denom = a d + (1 - a) z = 1e-3 (ucm.rs:307-311), and
    # the condition z > -w d with w = (1 - a)/a for a > 0.5 (ucm.rs:154-161)
    a = mp.mpf(S_UCM[4])
    pts = []
    for r in (1e-4, 3e-4, 6e-4):
        z0 = _root(lambda z: a * mp.sqrt(2 * r * r + z * z) + (1 - a) * z - mp.mpf("1e-3"), 1e-3)
        pts += [[r, r, z] for z in _ulps(z0)]
        w = (1 - a) / a
        zc = _root(lambda z: z + w * mp.sqrt(2 * r * r + z * z), r)
        pts += [[r * 1e3, r * 1e3, z * 1e3] for z in _ulps(zc)]
    out.append((4, S_UCM, (752, 480), "project", np.array(pts)))
    # ---- DS project: denom = a d2 + (1 - a) g = 1e-3 (double_sphere.rs:367-376)
    # and z > -w2 d1 (:177-184)
    a, xi = mp.mpf(S_DS[4]), mp.mpf(S_DS[5])
    w1 = (1 - a) / a
    w2 = (w1 + xi) / mp.sqrt(2 * w1 * xi + xi * xi + 1)
    pts = []
    for r in (1e-4, 4e-4, 0.3):
        def den(z, r=r):
            d1 = mp.sqrt(2 * r * r + z * z)
            g = xi * d1 + z
            return a * mp.sqrt(2 * r * r + g * g) + (1 - a) * g - mp.mpf("1e-3")
        try:
            z0 = _root(den, 1e-3)
            pts += [[r, r, z] for z in _ulps(z0)]
        except (ValueError, ZeroDivisionError):
            pass
        zc = _root(lambda z: z + w2 * mp.sqrt(2 * r * r + z * z), -r)
        pts += [[r, r, z] for z in _ulps(zc)]
    out.append((3, S_DS, (752, 480), "project", np.array(pts)))
    # ---- EUCM project: denom = 1e-3 and z < denom (a-1)/(2a-1) (eucm.rs:167-177)
    a, b = mp.mpf(S_EUCM[4]), mp.mpf(S_EUCM[5])
    c = (a - 1) / (2 * a - 1)
    pts = []
    for r in (1e-4, 5e-4, 1.0):
        def den(z, r=r):
            return a * mp.sqrt(b * 2 * r * r + z * z) + (1 - a) * z
        try:
            z0 = _root(lambda z: den(z) - mp.mpf("1e-3"), 1e-3)
            pts += [[r, r, z] for z in _ulps(z0)]
        except (ValueError, ZeroDivisionError):
            pass
        zc = _root(lambda z: z - den(z) * c, 0.1 * r)
        pts += [[r, r, z] for z in _ulps(zc)]
    out.append((5, S_EUCM, (752, 480), "project", np.array(pts)))
    # ---- KB project: z < 0, z < EPS (kannala_brandt.rs:345-351), r < EPS (:375)
    pts = [[x, 0.0, 1.0] for x in _ulps(EPS)] + [[0.0, y, 2.0] for y in _ulps(EPS)]
    pts += [[0.3, -0.2, z] for z in _ulps(EPS)] + [[0.3, -0.2, z] for z in _ulps(0.0)]
    pts += [[x * 0.6, x * 0.8, 1.0] for x in _ulps(EPS)]
    out.append((2, S_KB, (512, 512), "project", np.array(pts)))
    # ---- Pinhole project: z < sqrt(EPS) (pinhole.rs:167), u >= w, v >= h (:173-179)
    fx, fy, cx, cy = S_PIN
    pts = [[0.1, 0.1, z] for z in _ulps(EPS_SQRT)]
    pts += [[x, 0.0, 2.0] for x in _ulps((752.0 - cx) / fx * 2.0)]
    pts += [[0.0, y, 2.0] for y in _ulps((480.0 - cy) / fy * 2.0)]
    pts += [[x, 0.0, 2.0] for x in _ulps(-cx / fx * 2.0)]
    out.append((0, S_PIN, (752, 480), "project", np.array(pts)))
    # ---- unprojections: pixel u along the x axis (v = cy)
    def pix(p, mx_target_sq, scale):
        """pixels u = cx + fx * m with (m * scale)^2 at the root"""
        m0 = mp.sqrt(mp.mpf(mx_target_sq)) / scale
        u0 = mp.mpf(p[2]) + mp.mpf(p[0]) * m0
        return [[u, p[3]] for u in _ulps(u0)]
    a = mp.mpf(S_DS[4])
    out.append((3, S_DS, (0, 0), "unproject", np.array(pix(S_DS, 1 / (2 * a - 1), 1))))
    a = mp.mpf(S_UCM[4])
    g = 1 - a
    pts = pix(S_UCM, mp.mpf("0.999"), abs(g)) + pix(S_UCM, g * g / (2 * a - 1), abs(g))
    out.append((4, S_UCM, (0, 0), "unproject", np.array(pts)))
    a, b = mp.mpf(S_EUCM[4]), mp.mpf(S_EUCM[5])
    g = 1 - a
    pts = pix(S_EUCM, mp.mpf("0.999") / ((a - g) * b), 1) + pix(S_EUCM, (2 * a - 1) / b, 1)
    out.append((5, S_EUCM, (0, 0), "unproject", np.array(pts)))
    # KB unproject: ru = 1e-6 (kannala_brandt.rs:474, :526-533), ru = 0
    fx, fy, cx, cy = S_KB[:4]
    pts = [[cx, cy]] + [[u, cy] for u in _ulps(cx + fx * 1e-6)] + \
        [[cx, v] for v in _ulps(cy - fy * 1e-6)]
    out.append((2, S_KB, (512, 512), "unproject", np.array(pts)))
    # RadTan unproject: near-singular Newton Jacobian (rad_tan.rs:476-497)
    fx, fy, cx, cy = S_RT_SING[:4]
    pts = [[cx + fx * m, cy + fy * n] for m in (1.0, 0.999999, 1.000001, 0.5, 0.99)
           for n in (0.0, 1e-9, -1e-6, 1e-3)]
    out.append((1, S_RT_SING, (2000, 2000), "unproject", np.array(pts)))
    return out


# ----------------------------------------------------------- f64 emulation
def _st_project(model, p, w, h, pt):
    from mpmath import mpf, sqrt
    x, y, z = (mpf(float(c)) for c in pt)
    P = [mpf(float(c)) for c in p]
    fx, fy, cx, cy = P[:4]
    one, two = mpf(1), mpf(2)
    pr = mpf("1e-3")
    if model in (0, 1):  # pinhole.rs:165-182, rad_tan.rs:302-348
        if z < mpf(EPS_SQRT):
            return 3
        xp, yp = x / z, y / z
        if model == 0:
            u, v = fx * x / z + cx, fy * y / z + cy  # pinhole.rs:170-171
        else:
            k1, k2, p1, p2, k3 = P[4:9]
            r2 = xp * xp + yp * yp
            r4 = r2 * r2
            r6 = r4 * r2
            rad = one + k1 * r2 + k2 * r4 + k3 * r6
            xd = xp * rad + two * p1 * xp * yp + p2 * (r2 + two * xp * xp)
            yd = yp * rad + p1 * (r2 + two * yp * yp) + two * p2 * xp * yp
            u, v = fx * xd + cx, fy * yd + cy
        if u < 0 or u >= mpf(w) or v < 0 or v >= mpf(h):
            return 1
        return 0
    if model == 2:  # kannala_brandt.rs:345-351 (the axis test only shapes values)
        if z < 0:
            return 2
        if z < mpf(EPS):
            return 3
        return 0
    if model == 3:  # double_sphere.rs:361-390, :177-184
        a, xi = P[4], P[5]
        rs = (x * x) + (y * y)
        d1 = sqrt(rs + (z * z))
        g = xi * d1 + z
        d2 = sqrt(rs + g * g)
        den = a * d2 + (one - a) * g
        w1 = a / (one - a) if a <= mpf(0.5) else (one - a) / a
        w2 = (w1 + xi) / sqrt(two * w1 * xi + xi * xi + one)
        return 2 if (den < pr or not (z > -w2 * d1)) else 0
    if model == 4:  # ucm.rs:297-316, :154-161
        a = P[4]
        d = sqrt(x * x + y * y + z * z)
        den = a * d + (one - a) * z
        ww = a / (one - a) if a <= mpf(0.5) else (one - a) / a
        return 2 if (den < pr or not (z > -ww * d)) else 0
    if model == 5:  # eucm.rs:328-347, :167-177
        a, b = P[4], P[5]
        d = sqrt(b * (x * x + y * y) + z * z)
        den = a * d + (one - a) * z
        cond = True
        if a > mpf(0.5):
            c = (a - one) / (two * a - one)
            cond = not (z < den * c)
        return 2 if (den < pr or not cond) else 0
    if model == 6:  # fov.rs:290-292
        return 3 if z < mpf(EPS_SQRT) else 0
    raise ValueError(model)


def _st_unproject(model, p, w, h, uv):
    from mpmath import mpf, sqrt
    u, v = mpf(float(uv[0])), mpf(float(uv[1]))
    P = [mpf(float(c)) for c in p]
    fx, fy, cx, cy = P[:4]
    one, two = mpf(1), mpf(2)
    pr = mpf("1e-3")
    if model == 3:  # double_sphere.rs:436-476, :200-209
        a, xi = P[4], P[5]
        mx, my = (u - cx) / fx, (v - cy) / fy
        rs = (mx * mx) + (my * my)
        cond = not (a > mpf(0.5) and rs > one / (two * a - one))
        if a != 0 and not cond:
            return 2
        mz = (one - a * a * rs) / (a * sqrt(one - (two * a - one) * rs) + (one - a))
        den = mz * mz + rs
        return 2 if den < pr else 0
    if model == 4:  # ucm.rs:337-367, :177-184
        a = P[4]
        g = one - a
        mx, my = (u - cx) / fx * g, (v - cy) / fy * g
        rs = mx * mx + my * my
        den = one - rs
        cond = rs <= g * g / (two * a - one) if a > mpf(0.5) else True
        return 2 if (den < pr or not cond) else 0
    if model == 5:  # eucm.rs:368-398, :194-200
        a, b = P[4], P[5]
        mx, my = (u - cx) / fx, (v - cy) / fy
        rs = mx * mx + my * my
        g = one - a
        det = one - (a - g) * b * rs
        cond = not (a > mpf(0.5) and rs > (one / b * (two * a - one)))
        return 2 if (det < pr or not cond) else 0
    if model == 2:  # kannala_brandt.rs:445-562
        if w > 0 and h > 0 and (u < 0 or u >= mpf(w) or v < 0 or v >= mpf(h)):
            return 2
        k1, k2, k3, k4 = P[4:8]
        mx, my = (u - cx) / fx, (v - cy) / fy
        ru = sqrt(mx * mx + my * my)
        ru = min(ru, mpf(PI_HALF))
        prec = mpf("1e-6")
        if not ru > prec:
            return 0 if ru == 0 else 4
        th = ru
        for i in range(10):
            t2 = th * th
            t4 = t2 * t2
            t6 = t4 * t2
            t8 = t4 * t4
            a1, a2, a3, a4 = k1 * t2, k2 * t4, k3 * t6, k4 * t8
            f = th * (one + a1 + a2 + a3 + a4) - ru
            fp = one + (3 * a1) + (5 * a2) + (7 * a3) + (9 * a4)
            if abs(fp) < mpf(EPS):
                return 4
            dl = f / fp
            th = th - dl
            if abs(dl) < prec:
                return 0
        return 4
    if model == 1:  # rad_tan.rs:401-524
        if u < 0 or u >= mpf(w) or v < 0 or v >= mpf(h):
            return 2
        k1, k2, p1, p2, k3 = P[4:9]
        tx, ty = (u - cx) / fx, (v - cy) / fy
        x, y = tx, ty
        e6 = mpf("1e-6")
        for it in range(100):
            r2 = x * x + y * y
            r4 = r2 * r2
            r6 = r4 * r2
            rad = one + k1 * r2 + k2 * r4 + k3 * r6
            xe = x * rad + two * p1 * x * y + p2 * (r2 + two * x * x)
            ye = y * rad + p1 * (r2 + two * y * y) + two * p2 * x * y
            ex, ey = xe - tx, ye - ty
            if sqrt(ex * ex + ey * ey) < e6:
                return 0
            if ex != ex or ey != ey:
                return 4
            drdx, drdy = two * x, two * y
            ddx = (k1 + two * k2 * r2 + 3 * k3 * r4) * drdx
            ddy = (k1 + two * k2 * r2 + 3 * k3 * r4) * drdy
            j00 = rad + x * ddx + two * p1 * y + p2 * (drdx + 4 * x)
            j01 = x * ddy + two * p1 * x + p2 * (drdy)
            j10 = y * ddx + p1 * (drdx) + two * p2 * y
            j11 = rad + y * ddy + p1 * (drdy + 4 * y) + two * p2 * x
            det = j00 * j11 - j10 * j01
            if det == 0:
                return 4
            i00, i01, i10, i11 = j11 / det, -j01 / det, -j10 / det, j00 / det
            dx = i00 * ex + i01 * ey
            dy = i10 * ex + i11 * ey
            x, y = x - dx, y - dy
            if sqrt(dx * dx + dy * dy) < e6:
                return 0
            if it == 99:
                return 4
        return 4
    raise ValueError(model)


def emulate_status(model, p, w, h, kind, pt):
    """The reference's status for one probe, in binary64 (mpmath, 53 bits)."""
    with mpmath.workprec(53):
        if kind == "project":
            return _st_project(model, p, w, h, pt)
        return _st_unproject(model, p, w, h, pt)
