"""Independent 50-digit mpmath restatement of the seven camera models,
written from the model equations (with the reference's documented quirks:
UCM unproject's `1 - r^2` denominator ucm.rs:354, EUCM's (1/beta)*(2a-1)
condition eucm.rs:196, the KB/RadTan Newton solvers).  Used only to pin the
f64 oracle: its values must agree with these to a few ulps, and its analytic
Jacobians with 50-digit numerical derivatives (mp.diff).
"""
import mpmath as mp

mp.mp.dps = 50


def project(model, p, pt):
    """Returns (u, v) as mpf, or None where the reference returns Err."""
    x, y, z = (mp.mpf(c) for c in pt)
    fx, fy, cx, cy = (mp.mpf(c) for c in p[:4])
    if model == 0:  # pinhole
        return fx * x / z + cx, fy * y / z + cy
    if model == 1:  # radtan
        k1, k2, p1, p2, k3 = (mp.mpf(c) for c in p[4:9])
        xp, yp = x / z, y / z
        r2 = xp * xp + yp * yp
        rad = 1 + k1 * r2 + k2 * r2 ** 2 + k3 * r2 ** 3
        xd = xp * rad + 2 * p1 * xp * yp + p2 * (r2 + 2 * xp * xp)
        yd = yp * rad + p1 * (r2 + 2 * yp * yp) + 2 * p2 * xp * yp
        return fx * xd + cx, fy * yd + cy
    if model == 2:  # KB
        k = [mp.mpf(c) for c in p[4:8]]
        r = mp.sqrt(x * x + y * y)
        th = mp.atan2(r, z)
        thd = th + k[0] * th ** 3 + k[1] * th ** 5 + k[2] * th ** 7 + k[3] * th ** 9
        if r == 0:
            return cx, cy
        return fx * thd * x / r + cx, fy * thd * y / r + cy
    if model == 3:  # DS
        a, xi = mp.mpf(p[4]), mp.mpf(p[5])
        d1 = mp.sqrt(x * x + y * y + z * z)
        g = xi * d1 + z
        d2 = mp.sqrt(x * x + y * y + g * g)
        den = a * d2 + (1 - a) * g
        return fx * x / den + cx, fy * y / den + cy
    if model == 4:  # UCM
        a = mp.mpf(p[4])
        d = mp.sqrt(x * x + y * y + z * z)
        den = a * d + (1 - a) * z
        return fx * x / den + cx, fy * y / den + cy
    if model == 5:  # EUCM
        a, b = mp.mpf(p[4]), mp.mpf(p[5])
        d = mp.sqrt(b * (x * x + y * y) + z * z)
        den = a * d + (1 - a) * z
        return fx * x / den + cx, fy * y / den + cy
    if model == 6:  # FOV
        w = mp.mpf(p[4])
        r = mp.sqrt(x * x + y * y)
        t = mp.tan(w / 2)
        if r * r < mp.mpf("1.4901161193847656e-08"):
            rd = 2 * t / w
        else:
            rd = mp.atan2(2 * t * r, z) / (r * w)
        return fx * x * rd + cx, fy * y * rd + cy
    raise ValueError(model)


def unproject(model, p, uv):
    """Closed-form / converged-Newton ray (normalised), mpf triple."""
    u, v = mp.mpf(uv[0]), mp.mpf(uv[1])
    fx, fy, cx, cy = (mp.mpf(c) for c in p[:4])
    mx, my = (u - cx) / fx, (v - cy) / fy

    def nrm(a, b, c):
        n = mp.sqrt(a * a + b * b + c * c)
        return a / n, b / n, c / n

    if model == 0:
        return nrm(mx, my, mp.mpf(1))
    if model == 1:  # invert the radtan distortion exactly (Newton to 1e-40)
        k1, k2, p1, p2, k3 = (mp.mpf(c) for c in p[4:9])
        x, y = mx, my
        for _ in range(200):
            r2 = x * x + y * y
            rad = 1 + k1 * r2 + k2 * r2 ** 2 + k3 * r2 ** 3
            ex = x * rad + 2 * p1 * x * y + p2 * (r2 + 2 * x * x) - mx
            ey = y * rad + p1 * (r2 + 2 * y * y) + 2 * p2 * x * y - my
            dr = k1 + 2 * k2 * r2 + 3 * k3 * r2 ** 2
            j00 = rad + 2 * x * x * dr + 2 * p1 * y + 6 * p2 * x
            j01 = 2 * x * y * dr + 2 * p1 * x + 2 * p2 * y
            j10 = 2 * x * y * dr + 2 * p1 * x + 2 * p2 * y
            j11 = rad + 2 * y * y * dr + 6 * p1 * y + 2 * p2 * x
            det = j00 * j11 - j01 * j10
            dx = (j11 * ex - j01 * ey) / det
            dy = (-j10 * ex + j00 * ey) / det
            x, y = x - dx, y - dy
            if abs(dx) + abs(dy) < mp.mpf("1e-45"):
                break
        return nrm(x, y, mp.mpf(1))
    if model == 2:  # KB: solve theta_d(theta) = ru exactly
        k = [mp.mpf(c) for c in p[4:8]]
        # kannala_brandt.rs:467 clamps ru to pi/2 and keeps mx/ru unnormalised
        ru = min(mp.sqrt(mx * mx + my * my), mp.pi / 2)
        if ru == 0:
            return (mp.mpf(0), mp.mpf(0), mp.mpf(1))
        th = mp.findroot(lambda t: t + k[0] * t ** 3 + k[1] * t ** 5 + k[2] * t ** 7
                         + k[3] * t ** 9 - ru, ru)
        return nrm(mp.sin(th) * mx / ru, mp.sin(th) * my / ru, mp.cos(th))
    if model == 3:
        a, xi = mp.mpf(p[4]), mp.mpf(p[5])
        r2 = mx * mx + my * my
        mz = (1 - a * a * r2) / (a * mp.sqrt(1 - (2 * a - 1) * r2) + 1 - a)
        c = (mz * xi + mp.sqrt(mz * mz + (1 - xi * xi) * r2)) / (mz * mz + r2)
        return nrm(c * mx, c * my, c * mz - xi)
    if model == 4:  # UCM, reference's 1 - r^2 denominator
        a = mp.mpf(p[4])
        g = 1 - a
        xi = a / g
        mx, my = mx * g, my * g
        r2 = mx * mx + my * my
        c = (xi + mp.sqrt(1 + (1 - xi * xi) * r2)) / (1 - r2)
        return nrm(c * mx, c * my, c - xi)
    if model == 5:
        a, b = mp.mpf(p[4]), mp.mpf(p[5])
        r2 = mx * mx + my * my
        mz = (1 - r2 * a * a * b) / ((1 - a) + a * mp.sqrt(1 - (2 * a - 1) * b * r2))
        return nrm(mx, my, mz)
    if model == 6:
        w = mp.mpf(p[4])
        rd = mp.sqrt(mx * mx + my * my)
        t2 = 2 * mp.tan(w / 2)
        ru = mp.sin(rd * w) / (rd * t2)
        return nrm(mx * ru / mp.cos(rd * w), my * ru / mp.cos(rd * w), mp.mpf(1))
    raise ValueError(model)


def jacobian(model, p, pt):
    """d(u,v)/d params by 50-digit numerical differentiation."""
    P = len(p)
    Ju, Jv = [], []
    for k in range(P):
        def fu(t, k=k):
            q = list(p)
            q[k] = t
            return project(model, q, pt)[0]

        def fv(t, k=k):
            q = list(p)
            q[k] = t
            return project(model, q, pt)[1]
        Ju.append(mp.diff(fu, mp.mpf(p[k])))
        Jv.append(mp.diff(fv, mp.mpf(p[k])))
    return Ju, Jv
