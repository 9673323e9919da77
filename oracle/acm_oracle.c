/*
 * acm_oracle.c -- CPU parity oracle (TEST INFRASTRUCTURE ONLY, see header).
 *
 * Operation-for-operation restatement of the reference Rust code.  Citations
 * are /root/reference paths (amin-abouee/apex-camera-models v0.4.1).
 * Build: oracle/Makefile (gcc -O2 -ffp-contract=off).  Parenthesisation below
 * reproduces Rust's left-to-right evaluation of every expression, e.g.
 * `a + b + c` is (a + b) + c and `2.0 * p1 * x * y` is ((2*p1)*x)*y.
 */
#include "acm_oracle.h"

#include <float.h>
#include <math.h>
#include <stdlib.h>
#include <string.h>

#define F64_EPS 2.220446049250313e-16       /* f64::EPSILON */
#define F64_EPS_SQRT 1.4901161193847656e-08 /* f64::EPSILON.sqrt() */

int oracle_num_params(int model) {
    switch (model) {
    case OR_PINHOLE: return 4;
    case OR_RADTAN: return 9;
    case OR_KB: return 8;
    case OR_DS: return 6;
    case OR_UCM: return 5;
    case OR_EUCM: return 6;
    case OR_FOV: return 5;
    default: return -1;
    }
}

/* nalgebra Vector3::normalize(): each component divided by
 * norm() = sqrt((x*x + y*y) + z*z) (nalgebra blas dotc, U3 special case). */
static void normalize3(double x, double y, double z, double out[3]) {
    double n = sqrt(x * x + y * y + z * z);
    out[0] = x / n;
    out[1] = y / n;
    out[2] = z / n;
}

static void set_nan2(double uv[2]) { uv[0] = NAN; uv[1] = NAN; }
static void set_nan3(double r[3]) { r[0] = NAN; r[1] = NAN; r[2] = NAN; }

/* ------------------------------------------------------------------ Pinhole */
/* src/camera/pinhole.rs:165-182 */
static int pinhole_project(const double *P, uint32_t w, uint32_t h,
                           const double *p, double *uv, double *J) {
    double fx = P[0], fy = P[1], cx = P[2], cy = P[3];
    double x = p[0], y = p[1], z = p[2];
    if (z < F64_EPS_SQRT) return OR_POINT_AT_CAMERA_CENTER;      /* :167-169 */
    double u = fx * x / z + cx;                                  /* :170 */
    double v = fy * y / z + cy;                                  /* :171 */
    if (u < 0.0 || u >= (double)w || v < 0.0 || v >= (double)h) /* :173-179 */
        return OR_PROJECTION_OUT_SIDE_IMAGE;
    uv[0] = u;
    uv[1] = v;
    if (J) { /* d(u,v)/d(fx,fy,cx,cy) */
        double *Ju = J, *Jv = J + 4;
        Ju[0] = x / z; Ju[1] = 0.0; Ju[2] = 1.0; Ju[3] = 0.0;
        Jv[0] = 0.0; Jv[1] = y / z; Jv[2] = 0.0; Jv[3] = 1.0;
    }
    return OR_OK;
}

/* src/camera/pinhole.rs:228-246 */
static int pinhole_unproject(const double *P, uint32_t w, uint32_t h,
                             const double *uv, double *ray) {
    double fx = P[0], fy = P[1], cx = P[2], cy = P[3];
    if (uv[0] < 0.0 || uv[0] >= (double)w || uv[1] < 0.0 || uv[1] >= (double)h)
        return OR_POINT_IS_OUT_SIDE_IMAGE;                       /* :229-236 */
    double mx = (uv[0] - cx) / fx;                               /* :238 */
    double my = (uv[1] - cy) / fy;
    double r2 = mx * mx + my * my;                               /* :241 */
    double norm = sqrt(1.0 + r2);                                /* :243 */
    double norm_inv = 1.0 / norm;
    ray[0] = mx * norm_inv;                                      /* :245 */
    ray[1] = my * norm_inv;
    ray[2] = norm_inv;
    return OR_OK;
}

/* ------------------------------------------------------------------- RadTan */
/* src/camera/rad_tan.rs:302-348; params fx fy cx cy k1 k2 p1 p2 k3 */
static int radtan_project(const double *P, uint32_t w, uint32_t h,
                          const double *p, double *uv, double *J) {
    double fx = P[0], fy = P[1], cx = P[2], cy = P[3];
    double k1 = P[4], k2 = P[5], p1 = P[6], p2 = P[7], k3 = P[8];
    if (p[2] < F64_EPS_SQRT) return OR_POINT_AT_CAMERA_CENTER;   /* :304-306 */
    double x = p[0], y = p[1], z = p[2];
    double xp = x / z, yp = y / z;                               /* :319-320 */
    double r2 = xp * xp + yp * yp;                               /* :322 powi(2) */
    double r4 = r2 * r2;
    double r6 = r4 * r2;
    double radial = 1.0 + k1 * r2 + k2 * r4 + k3 * r6;
    double xd = xp * radial + 2.0 * p1 * xp * yp + p2 * (r2 + 2.0 * xp * xp);
    double yd = yp * radial + p1 * (r2 + 2.0 * yp * yp) + 2.0 * p2 * xp * yp;
    double u = fx * xd + cx;                                     /* :336-337 */
    double v = fy * yd + cy;
    if (u < 0.0 || u >= (double)w || v < 0.0 || v >= (double)h) /* :339-345 */
        return OR_PROJECTION_OUT_SIDE_IMAGE;
    uv[0] = u;
    uv[1] = v;
    if (J) {
        double *Ju = J, *Jv = J + 9;
        double xpyp2 = 2.0 * xp * yp;
        Ju[0] = xd; Ju[1] = 0.0; Ju[2] = 1.0; Ju[3] = 0.0;
        Ju[4] = fx * xp * r2;
        Ju[5] = fx * xp * r4;
        Ju[6] = fx * xpyp2;
        Ju[7] = fx * (r2 + 2.0 * xp * xp);
        Ju[8] = fx * xp * r6;
        Jv[0] = 0.0; Jv[1] = yd; Jv[2] = 0.0; Jv[3] = 1.0;
        Jv[4] = fy * yp * r2;
        Jv[5] = fy * yp * r4;
        Jv[6] = fy * (r2 + 2.0 * yp * yp);
        Jv[7] = fy * xpyp2;
        Jv[8] = fy * yp * r6;
    }
    return OR_OK;
}

/* src/camera/rad_tan.rs:401-524 (Newton, <=100 iterations) */
static int radtan_unproject(const double *P, uint32_t w, uint32_t h,
                            const double *uvp, double *ray) {
    double fx = P[0], fy = P[1], cx = P[2], cy = P[3];
    double k1 = P[4], k2 = P[5], p1 = P[6], p2 = P[7], k3 = P[8];
    if (uvp[0] < 0.0 || uvp[0] >= (double)w || uvp[1] < 0.0 ||
        uvp[1] >= (double)h)
        return OR_POINT_IS_OUT_SIDE_IMAGE;                       /* :402-409 */
    double tx = (uvp[0] - cx) / fx;                              /* :425-426 */
    double ty = (uvp[1] - cy) / fy;
    double px = tx, py = ty;                                     /* :430 */
    const double EPS = 1e-6;
    const unsigned MAX_IT = 100;
    for (unsigned it = 0; it < MAX_IT; ++it) {                   /* :436 */
        double x = px, y = py;
        double r2 = x * x + y * y;
        double r4 = r2 * r2;
        double r6 = r4 * r2;
        double rad = 1.0 + k1 * r2 + k2 * r4 + k3 * r6;          /* :444 */
        double xe = x * rad + 2.0 * p1 * x * y + p2 * (r2 + 2.0 * x * x);
        double ye = y * rad + p1 * (r2 + 2.0 * y * y) + 2.0 * p2 * x * y;
        double ex = xe - tx, ey = ye - ty;                       /* :456 */
        if (sqrt(ex * ex + ey * ey) < EPS) break;                /* :459 */
        double drdx = 2.0 * x, drdy = 2.0 * y;                   /* :470-471 */
        double ddx = (k1 + 2.0 * k2 * r2 + 3.0 * k3 * r4) * drdx;
        double ddy = (k1 + 2.0 * k2 * r2 + 3.0 * k3 * r4) * drdy;
        double j00 = rad + x * ddx + 2.0 * p1 * y + p2 * (drdx + 4.0 * x);
        double j01 = x * ddy + 2.0 * p1 * x + p2 * (drdy);
        double j10 = y * ddx + p1 * (drdx) + 2.0 * p2 * y;
        double j11 = rad + y * ddy + p1 * (drdy + 4.0 * y) + 2.0 * p2 * x;
        /* nalgebra Matrix2::try_inverse (linalg/inverse.rs, 2x2 closed form) */
        double det = j00 * j11 - j10 * j01;
        if (det == 0.0) return OR_NUMERICAL_ERROR;               /* :512-517 */
        double i00 = j11 / det, i01 = -j01 / det;
        double i10 = -j10 / det, i11 = j00 / det;
        double dx = i00 * ex + i01 * ey;                         /* :497 gemv */
        double dy = i10 * ex + i11 * ey;
        px = px - dx;                                            /* :500 */
        py = py - dy;
        if (sqrt(dx * dx + dy * dy) < EPS) break;                /* :503 */
        if (it == MAX_IT - 1) return OR_NUMERICAL_ERROR;         /* :514-520 */
    }
    normalize3(px, py, 1.0, ray);                                /* :522-523 */
    return OR_OK;
}

/* ------------------------------------------------------------ Kannala-Brandt */
/* src/camera/kannala_brandt.rs:340-394; params fx fy cx cy k1 k2 k3 k4 */
static int kb_project(const double *P, const double *p, double *uv,
                      double *J) {
    double x = p[0], y = p[1], z = p[2];
    if (z < 0.0) return OR_POINT_IS_OUT_SIDE_IMAGE;              /* :345-347 */
    else if (z < F64_EPS) return OR_POINT_AT_CAMERA_CENTER;      /* :348-351 */
    double k1 = P[4], k2 = P[5], k3 = P[6], k4 = P[7];
    double fx = P[0], fy = P[1], cx = P[2], cy = P[3];
    double r_sq = x * x + y * y;                                 /* :363 */
    double r = sqrt(r_sq);
    double theta = atan2(r, z);                                  /* :365 */
    double theta2 = theta * theta;
    double theta3 = theta2 * theta;
    double theta5 = theta3 * theta2;
    double theta7 = theta5 * theta2;
    double theta9 = theta7 * theta2;
    double theta_d = theta + k1 * theta3 + k2 * theta5 + k3 * theta7 + k4 * theta9;
    double x_r, y_r;
    if (r < F64_EPS) { x_r = 0.0; y_r = 0.0; }                   /* :375-388 */
    else { x_r = x / r; y_r = y / r; }
    uv[0] = fx * theta_d * x_r + cx;                             /* :390 */
    uv[1] = fy * theta_d * y_r + cy;
    if (J) {
        double *Ju = J, *Jv = J + 8;
        double fxr = fx * x_r, fyr = fy * y_r;
        Ju[0] = theta_d * x_r; Ju[1] = 0.0; Ju[2] = 1.0; Ju[3] = 0.0;
        Ju[4] = fxr * theta3; Ju[5] = fxr * theta5;
        Ju[6] = fxr * theta7; Ju[7] = fxr * theta9;
        Jv[0] = 0.0; Jv[1] = theta_d * y_r; Jv[2] = 0.0; Jv[3] = 1.0;
        Jv[4] = fyr * theta3; Jv[5] = fyr * theta5;
        Jv[6] = fyr * theta7; Jv[7] = fyr * theta9;
    }
    return OR_OK;
}

/* src/camera/kannala_brandt.rs:445-562 (Newton, <=10 iterations) */
static int kb_unproject(const double *P, uint32_t w, uint32_t h,
                        const double *uvp, double *ray) {
    if (w > 0 && h > 0 &&
        (uvp[0] < 0.0 || uvp[0] >= (double)w || uvp[1] < 0.0 ||
         uvp[1] >= (double)h))
        return OR_POINT_IS_OUT_SIDE_IMAGE;                       /* :447-455 */
    double fx = P[0], fy = P[1], cx = P[2], cy = P[3];
    double mx = (uvp[0] - cx) / fx;                              /* :460 */
    double my = (uvp[1] - cy) / fy;
    double ru = sqrt(mx * mx + my * my);                         /* :463 */
    ru = fmin(ru, M_PI / 2.0);     /* :467 f64::min (NaN -> other operand) */
    double theta = ru;
    const double PRECISION = 1e-6;
    const int MAX_IT = 10;
    int converged = 1;
    if (ru > PRECISION) {                                        /* :474 */
        double k1 = P[4], k2 = P[5], k3 = P[6], k4 = P[7];
        for (int i = 0; i < MAX_IT; ++i) {
            double theta2 = theta * theta;
            double theta4 = theta2 * theta2;
            double theta6 = theta4 * theta2;
            double theta8 = theta4 * theta4;
            double k1t2 = k1 * theta2, k2t4 = k2 * theta4;
            double k3t6 = k3 * theta6, k4t8 = k4 * theta8;
            double f = theta * (1.0 + k1t2 + k2t4 + k3t6 + k4t8) - ru; /* :493 */
            double fp = 1.0 + (3.0 * k1t2) + (5.0 * k2t4) + (7.0 * k3t6) +
                        (9.0 * k4t8);                            /* :496-500 */
            if (fabs(fp) < F64_EPS) { converged = 0; break; }    /* :502-506 */
            double delta = f / fp;
            theta -= delta;
            if (fabs(delta) < PRECISION) break;                  /* :510-512 */
            if (i == MAX_IT - 1) converged = 0;                  /* :513-516 */
        }
    } else {
        if (ru > 0.0) converged = 0;                             /* :526-528 */
        else { theta = 0.0; converged = 1; }                     /* :529-533 */
    }
    if (!converged) return OR_NUMERICAL_ERROR;                   /* :536-540 */
    double xc, yc;
    if (fabs(ru) < F64_EPS) { xc = 0.0; yc = 0.0; }              /* :545-552 */
    else { xc = mx / ru; yc = my / ru; }
    double s = sin(theta), c = cos(theta);                       /* :557-558 */
    normalize3(s * xc, s * yc, c, ray);                          /* :560-561 */
    return OR_OK;
}

/* ------------------------------------------------------------- Double Sphere */
/* src/camera/double_sphere.rs:177-184 */
static int ds_check_projection_condition(double alpha, double xi, double z,
                                         double d1) {
    double w1 = alpha <= 0.5 ? alpha / (1.0 - alpha) : (1.0 - alpha) / alpha;
    double w2 = (w1 + xi) / sqrt(2.0 * w1 * xi + xi * xi + 1.0);
    return z > -w2 * d1;
}

/* src/camera/double_sphere.rs:361-390; params fx fy cx cy alpha xi */
static int ds_project(const double *P, const double *p, double *uv,
                      double *J) {
    const double PRECISION = 1e-3;
    double fx = P[0], fy = P[1], cx = P[2], cy = P[3];
    double alpha = P[4], xi = P[5];
    double x = p[0], y = p[1], z = p[2];
    double r_squared = (x * x) + (y * y);                        /* :368 */
    double d1 = sqrt(r_squared + (z * z));
    double gamma = xi * d1 + z;                                  /* :370 */
    double d2 = sqrt(r_squared + gamma * gamma);
    double denom = alpha * d2 + (1.0 - alpha) * gamma;           /* :373 */
    if (denom < PRECISION || !ds_check_projection_condition(alpha, xi, z, d1))
        return OR_POINT_IS_OUT_SIDE_IMAGE;                       /* :376-380 */
    double mx = x / denom, my = y / denom;                       /* :382-383 */
    uv[0] = fx * (mx) + cx;                                      /* :386 */
    uv[1] = fy * (my) + cy;
    if (J) {
        double *Ju = J, *Jv = J + 6;
        double tu = fx * mx / denom, tv = fy * my / denom; /* f*x/den^2 */
        double dden_dalpha = d2 - gamma;
        double dden_dxi = d1 * (alpha * gamma / d2 + (1.0 - alpha));
        Ju[0] = mx; Ju[1] = 0.0; Ju[2] = 1.0; Ju[3] = 0.0;
        Ju[4] = -tu * dden_dalpha; Ju[5] = -tu * dden_dxi;
        Jv[0] = 0.0; Jv[1] = my; Jv[2] = 0.0; Jv[3] = 1.0;
        Jv[4] = -tv * dden_dalpha; Jv[5] = -tv * dden_dxi;
    }
    return OR_OK;
}

/* src/camera/double_sphere.rs:436-476 (+ check_unprojection_condition :200-209) */
static int ds_unproject(const double *P, const double *uvp, double *ray) {
    const double PRECISION = 1e-3;
    double fx = P[0], fy = P[1], cx = P[2], cy = P[3];
    double alpha = P[4], xi = P[5];
    double gamma_ds = 1.0 - alpha;                               /* :448 */
    double mx = (uvp[0] - cx) / fx;
    double my = (uvp[1] - cy) / fy;
    double r_squared = (mx * mx) + (my * my);                    /* :451 */
    int cond = 1;                                                /* :200-209 */
    if (alpha > 0.5 && r_squared > 1.0 / (2.0 * alpha - 1.0)) cond = 0;
    if (alpha != 0.0 && !cond) return OR_POINT_IS_OUT_SIDE_IMAGE; /* :454 */
    double mz = (1.0 - alpha * alpha * r_squared) /
                (alpha * sqrt(1.0 - (2.0 * alpha - 1.0) * r_squared) + gamma_ds);
    double mz_squared = mz * mz;                                 /* :460 */
    double num = mz * xi + sqrt(mz_squared + (1.0 - xi * xi) * r_squared);
    double denom = mz_squared + r_squared;                       /* :463 */
    if (denom < PRECISION) return OR_POINT_IS_OUT_SIDE_IMAGE;    /* :466-468 */
    double coeff = num / denom;
    normalize3(coeff * mx, coeff * my, coeff * mz - xi, ray);    /* :473-475 */
    return OR_OK;
}

/* ---------------------------------------------------------------------- UCM */
/* src/camera/ucm.rs:154-161 */
static int ucm_check_proj_condition(double z, double d, double alpha) {
    double w = alpha <= 0.5 ? alpha / (1.0 - alpha) : (1.0 - alpha) / alpha;
    return z > -w * d;
}

/* src/camera/ucm.rs:297-316; params fx fy cx cy alpha */
static int ucm_project(const double *P, const double *p, double *uv,
                       double *J) {
    const double PRECISION = 1e-3;
    double fx = P[0], fy = P[1], cx = P[2], cy = P[3], alpha = P[4];
    double x = p[0], y = p[1], z = p[2];
    double d = sqrt(x * x + y * y + z * z);                      /* :304 */
    double denom = alpha * d + (1.0 - alpha) * z;                /* :305 */
    if (denom < PRECISION || !ucm_check_proj_condition(z, d, alpha))
        return OR_POINT_IS_OUT_SIDE_IMAGE;                       /* :308-310 */
    uv[0] = fx * (x / denom) + cx;                               /* :312-313 */
    uv[1] = fy * (y / denom) + cy;
    if (J) {
        double *Ju = J, *Jv = J + 5;
        double mx = x / denom, my = y / denom;
        double tu = fx * mx / denom, tv = fy * my / denom;
        double dden_dalpha = d - z;
        Ju[0] = mx; Ju[1] = 0.0; Ju[2] = 1.0; Ju[3] = 0.0;
        Ju[4] = -tu * dden_dalpha;
        Jv[0] = 0.0; Jv[1] = my; Jv[2] = 0.0; Jv[3] = 1.0;
        Jv[4] = -tv * dden_dalpha;
    }
    return OR_OK;
}

/* src/camera/ucm.rs:337-367 (+ check_unproj_condition :177-184).
 * Reproduces the reference's `denom = 1.0 - r_squared` (:354). */
static int ucm_unproject(const double *P, const double *uvp, double *ray) {
    const double PRECISION = 1e-3;
    double fx = P[0], fy = P[1], cx = P[2], cy = P[3], alpha = P[4];
    double gamma = 1.0 - alpha;                                  /* :347 */
    double xi = alpha / gamma;
    double mx = (uvp[0] - cx) / fx * gamma;                      /* :349 */
    double my = (uvp[1] - cy) / fy * gamma;
    double r_squared = mx * mx + my * my;                        /* :352 */
    double num = xi + sqrt(1.0 + (1.0 - xi * xi) * r_squared);
    double denom = 1.0 - r_squared;                              /* :354 */
    int cond = alpha > 0.5 ? (r_squared <= gamma * gamma / (2.0 * alpha - 1.0))
                           : 1;                                  /* :177-184 */
    if (denom < PRECISION || !cond) return OR_POINT_IS_OUT_SIDE_IMAGE;
    double coeff = num / denom;                                  /* :361 */
    normalize3(coeff * mx - 0.0, coeff * my - 0.0, coeff - xi, ray); /* :364-366 */
    return OR_OK;
}

/* --------------------------------------------------------------------- EUCM */
/* src/camera/eucm.rs:167-177 */
static int eucm_check_proj_condition(double z, double denom, double alpha) {
    int condition = 1;
    if (alpha > 0.5) {
        double c = (alpha - 1.0) / (2.0 * alpha - 1.0);
        if (z < denom * c) condition = 0;
    }
    return condition;
}

/* src/camera/eucm.rs:328-347; params fx fy cx cy alpha beta */
static int eucm_project(const double *P, const double *p, double *uv,
                        double *J) {
    const double PRECISION = 1e-3;
    double fx = P[0], fy = P[1], cx = P[2], cy = P[3];
    double alpha = P[4], beta = P[5];
    double x = p[0], y = p[1], z = p[2];
    double d = sqrt(beta * (x * x + y * y) + z * z);             /* :335 */
    double denom = alpha * d + (1.0 - alpha) * z;                /* :336 */
    if (denom < PRECISION || !eucm_check_proj_condition(z, denom, alpha))
        return OR_POINT_IS_OUT_SIDE_IMAGE;                       /* :339-341 */
    uv[0] = fx * (x / denom) + cx;                               /* :343-344 */
    uv[1] = fy * (y / denom) + cy;
    if (J) {
        double *Ju = J, *Jv = J + 6;
        double mx = x / denom, my = y / denom;
        double tu = fx * mx / denom, tv = fy * my / denom;
        double dden_dalpha = d - z;
        double dden_dbeta = alpha * (x * x + y * y) / (2.0 * d);
        Ju[0] = mx; Ju[1] = 0.0; Ju[2] = 1.0; Ju[3] = 0.0;
        Ju[4] = -tu * dden_dalpha; Ju[5] = -tu * dden_dbeta;
        Jv[0] = 0.0; Jv[1] = my; Jv[2] = 0.0; Jv[3] = 1.0;
        Jv[4] = -tv * dden_dalpha; Jv[5] = -tv * dden_dbeta;
    }
    return OR_OK;
}

/* src/camera/eucm.rs:368-398 (+ check_unproj_condition :194-200, whose
 * `1.0 / beta * (2.0 * alpha - 1.0)` is (1/beta)*(2a-1) by precedence). */
static int eucm_unproject(const double *P, const double *uvp, double *ray) {
    const double PRECISION = 1e-3;
    double fx = P[0], fy = P[1], cx = P[2], cy = P[3];
    double alpha = P[4], beta = P[5];
    double mx = (uvp[0] - cx) / fx;                              /* :380 */
    double my = (uvp[1] - cy) / fy;
    double r_squared = mx * mx + my * my;                        /* :383 */
    double gamma = 1.0 - alpha;
    double num = 1.0 - r_squared * alpha * alpha * beta;         /* :385 */
    double det = 1.0 - (alpha - gamma) * beta * r_squared;       /* :386 */
    double denom = gamma + alpha * sqrt(det);                    /* :387 */
    int cond = 1;
    if (alpha > 0.5 && r_squared > (1.0 / beta * (2.0 * alpha - 1.0))) cond = 0;
    if (det < PRECISION || !cond) return OR_POINT_IS_OUT_SIDE_IMAGE; /* :390 */
    double mz = num / denom;                                     /* :394 */
    double norm = sqrt(mx * mx + my * my + mz * mz);             /* :395 */
    ray[0] = mx / norm;
    ray[1] = my / norm;
    ray[2] = mz / norm;
    return OR_OK;
}

/* ---------------------------------------------------------------------- FOV */
/* src/camera/fov.rs:284-316; params fx fy cx cy w */
static int fov_project(const double *P, const double *p, double *uv,
                       double *J) {
    double fx = P[0], fy = P[1], cx = P[2], cy = P[3], wfov = P[4];
    double x = p[0], y = p[1], z = p[2];
    if (z < F64_EPS_SQRT) return OR_POINT_AT_CAMERA_CENTER;      /* :290-292 */
    double r2 = x * x + y * y;
    double r = sqrt(r2);
    double tan_w_half = tan(wfov / 2.0);                         /* :297 */
    double atan_wrd = atan2(2.0 * tan_w_half * r, z);            /* :298 */
    double rd, drd_dw;
    if (r2 < F64_EPS_SQRT) {                                     /* :302-305 */
        rd = 2.0 * tan_w_half / wfov;
        drd_dw = ((1.0 + tan_w_half * tan_w_half) * wfov - 2.0 * tan_w_half) /
                 (wfov * wfov);
    } else {
        rd = atan_wrd / (r * wfov);                              /* :306-308 */
        double a = 2.0 * tan_w_half * r;
        double datan_dw = z * r * (1.0 + tan_w_half * tan_w_half) / (a * a + z * z);
        drd_dw = datan_dw / (r * wfov) - atan_wrd / (r * wfov * wfov);
    }
    double mx = x * rd, my = y * rd;                             /* :310-311 */
    uv[0] = fx * mx + cx;                                        /* :313-314 */
    uv[1] = fy * my + cy;
    if (J) {
        double *Ju = J, *Jv = J + 5;
        Ju[0] = mx; Ju[1] = 0.0; Ju[2] = 1.0; Ju[3] = 0.0;
        Ju[4] = fx * x * drd_dw;
        Jv[0] = 0.0; Jv[1] = my; Jv[2] = 0.0; Jv[3] = 1.0;
        Jv[4] = fy * y * drd_dw;
    }
    return OR_OK;
}

/* src/camera/fov.rs:336-363 */
static int fov_unproject(const double *P, const double *uvp, double *ray) {
    double fx = P[0], fy = P[1], cx = P[2], cy = P[3], wfov = P[4];
    double tan_w_2 = tan(wfov / 2.0);                            /* :340 */
    double mul2tanwby2 = tan_w_2 * 2.0;
    double mx = (uvp[0] - cx) / fx;
    double my = (uvp[1] - cy) / fy;
    double r2 = mx * mx + my * my;
    double rd = sqrt(r2);
    double X, Y, Z;
    if (mul2tanwby2 > F64_EPS_SQRT && rd > F64_EPS_SQRT) {       /* :351 */
        double sin_rd_w = sin(rd * wfov);
        double cos_rd_w = cos(rd * wfov);
        double ru = sin_rd_w / (rd * mul2tanwby2);
        X = mx * ru / cos_rd_w;                                  /* :357 */
        Y = my * ru / cos_rd_w;
        Z = 1.0;
    } else {
        X = mx; Y = my; Z = 1.0;
    }
    normalize3(X, Y, Z, ray);                                    /* :362-363 */
    return OR_OK;
}

/* ------------------------------------------------------------- dispatchers */
int oracle_project_jacobian(int model, const double *params, uint32_t w,
                            uint32_t h, const double p[3], double uv[2],
                            double *J) {
    switch (model) {
    case OR_PINHOLE: return pinhole_project(params, w, h, p, uv, J);
    case OR_RADTAN: return radtan_project(params, w, h, p, uv, J);
    case OR_KB: return kb_project(params, p, uv, J);
    case OR_DS: return ds_project(params, p, uv, J);
    case OR_UCM: return ucm_project(params, p, uv, J);
    case OR_EUCM: return eucm_project(params, p, uv, J);
    case OR_FOV: return fov_project(params, p, uv, J);
    default: return -1;
    }
}

int oracle_project(int model, const double *params, uint32_t w, uint32_t h,
                   const double p[3], double uv[2]) {
    return oracle_project_jacobian(model, params, w, h, p, uv, NULL);
}

int oracle_unproject(int model, const double *params, uint32_t w, uint32_t h,
                     const double uv[2], double ray[3]) {
    switch (model) {
    case OR_PINHOLE: return pinhole_unproject(params, w, h, uv, ray);
    case OR_RADTAN: return radtan_unproject(params, w, h, uv, ray);
    case OR_KB: return kb_unproject(params, w, h, uv, ray);
    case OR_DS: return ds_unproject(params, uv, ray);
    case OR_UCM: return ucm_unproject(params, uv, ray);
    case OR_EUCM: return eucm_unproject(params, uv, ray);
    case OR_FOV: return fov_unproject(params, uv, ray);
    default: return -1;
    }
}

/* ------------------------------------------------------------ batch loops */
void oracle_project_batch(int model, const double *params, uint32_t w,
                          uint32_t h, size_t n, const double *xyz, double *uv,
                          uint8_t *status, double *jac) {
    int P = oracle_num_params(model);
    double J[18];
    for (size_t i = 0; i < n; ++i) {
        double o[2];
        int st = oracle_project_jacobian(model, params, w, h, xyz + 3 * i, o,
                                         jac ? J : NULL);
        status[i] = (uint8_t)st;
        if (st != OR_OK) set_nan2(o);
        uv[2 * i] = o[0];
        uv[2 * i + 1] = o[1];
        if (jac) {
            for (int k = 0; k < P; ++k) {
                jac[(size_t)k * 2 * n + 2 * i] = st == OR_OK ? J[k] : 0.0;
                jac[(size_t)k * 2 * n + 2 * i + 1] = st == OR_OK ? J[P + k] : 0.0;
            }
        }
    }
}

void oracle_unproject_batch(int model, const double *params, uint32_t w,
                            uint32_t h, size_t n, const double *uv,
                            double *xyz, uint8_t *status) {
    for (size_t i = 0; i < n; ++i) {
        double r[3];
        int st = oracle_unproject(model, params, w, h, uv + 2 * i, r);
        status[i] = (uint8_t)st;
        if (st != OR_OK) set_nan3(r);
        xyz[3 * i] = r[0];
        xyz[3 * i + 1] = r[1];
        xyz[3 * i + 2] = r[2];
    }
}

void oracle_residual_jacobian_batch(int model, const double *params,
                                    uint32_t w, uint32_t h, size_t n,
                                    const double *xyz, const double *uv_obs,
                                    int policy, double *res, double *jac,
                                    uint8_t *status) {
    int P = oracle_num_params(model);
    double J[18];
    for (size_t i = 0; i < n; ++i) {
        double o[2];
        int st = oracle_project_jacobian(model, params, w, h, xyz + 3 * i, o,
                                         jac ? J : NULL);
        if (status) status[i] = (uint8_t)st;
        if (st == OR_OK) {
            res[2 * i] = o[0] - uv_obs[2 * i];
            res[2 * i + 1] = o[1] - uv_obs[2 * i + 1];
        } else {
            double s = policy == 1 ? 1e6 : 0.0;
            res[2 * i] = s;
            res[2 * i + 1] = s;
        }
        if (jac) {
            for (int k = 0; k < P; ++k) {
                jac[(size_t)k * 2 * n + 2 * i] = st == OR_OK ? J[k] : 0.0;
                jac[(size_t)k * 2 * n + 2 * i + 1] = st == OR_OK ? J[P + k] : 0.0;
            }
        }
    }
}

void oracle_normal_equations(int model, const double *params, uint32_t w,
                             uint32_t h, size_t n, const double *xyz,
                             const double *uv_obs, int policy, double *JtJ,
                             double *Jtr, double *cost, uint64_t *n_valid) {
    int P = oracle_num_params(model);
    long double A[81], g[9], c = 0.0L;
    uint64_t nv = 0;
    memset(A, 0, sizeof(A));
    memset(g, 0, sizeof(g));
    double J[18];
    for (size_t i = 0; i < n; ++i) {
        double o[2], r0, r1;
        int st = oracle_project_jacobian(model, params, w, h, xyz + 3 * i, o, J);
        if (st == OR_OK) {
            r0 = o[0] - uv_obs[2 * i];
            r1 = o[1] - uv_obs[2 * i + 1];
            ++nv;
            for (int a = 0; a < P; ++a) {
                g[a] += (long double)J[a] * r0 + (long double)J[P + a] * r1;
                for (int b = 0; b < P; ++b)
                    A[a * P + b] += (long double)J[a] * J[b] +
                                    (long double)J[P + a] * J[P + b];
            }
        } else {
            r0 = r1 = policy == 1 ? 1e6 : 0.0;
        }
        c += (long double)r0 * r0 + (long double)r1 * r1;
    }
    for (int a = 0; a < P * P; ++a) JtJ[a] = (double)A[a];
    for (int a = 0; a < P; ++a) Jtr[a] = (double)g[a];
    *cost = (double)(0.5L * c);
    *n_valid = nv;
}

/* ---------------------------------------------------- reprojection error */
static int cmp_double(const void *a, const void *b) {
    double x = *(const double *)a, y = *(const double *)b;
    return (x > y) - (x < y);
}

/* src/util/error_metrics.rs:62-121 */
size_t oracle_reprojection_error(int model, const double *params, uint32_t w,
                                 uint32_t h, size_t n, const double *xyz,
                                 const double *uv, double out[6]) {
    double *errs = (double *)malloc((n ? n : 1) * sizeof(double));
    size_t m = 0;
    for (size_t i = 0; i < n; ++i) {                             /* :72-80 */
        double o[2];
        if (oracle_project(model, params, w, h, xyz + 3 * i, o) == OR_OK) {
            double du = o[0] - uv[2 * i], dv = o[1] - uv[2 * i + 1];
            errs[m++] = sqrt(du * du + dv * dv);                 /* :77 norm */
        }
    }
    if (m == 0) { free(errs); return 0; }                        /* :82-84 */
    double nn = (double)m;
    double sum = 0.0;                                            /* :88 */
    for (size_t i = 0; i < m; ++i) sum += errs[i];
    double mean = sum / nn;
    double var = 0.0;                                            /* :92 */
    for (size_t i = 0; i < m; ++i) { double d = errs[i] - mean; var += d * d; }
    var = var / nn;
    double stddev = sqrt(var);
    double ssq = 0.0;                                            /* :96 */
    for (size_t i = 0; i < m; ++i) ssq += errs[i] * errs[i];
    double rmse = sqrt(ssq / nn);
    double mn = INFINITY, mx = -INFINITY;                        /* :100-101 */
    for (size_t i = 0; i < m; ++i) {
        mn = fmin(mn, errs[i]);
        mx = fmax(mx, errs[i]);
    }
    qsort(errs, m, sizeof(double), cmp_double);                  /* :104-105 */
    double median = (m % 2 == 0) ? (errs[m / 2 - 1] + errs[m / 2]) / 2.0
                                 : errs[m / 2];                  /* :106-111 */
    out[0] = rmse; out[1] = mn; out[2] = mx;
    out[3] = mean; out[4] = stddev; out[5] = median;
    free(errs);
    return m;
}

/* ------------------------------------------------------------ sample_points */
/* src/util/point_sampling.rs:46-120 */
size_t oracle_sample_points(int model, const double *params, uint32_t w,
                            uint32_t h, size_t n_requested, size_t cap,
                            double *uv_out, double *xyz_out,
                            size_t *grid_total) {
    double width = (double)w, height = (double)h;                /* :50-51 */
    int ncx = (int)round(sqrt((double)n_requested * (width / height))); /* :53 */
    int ncy = (int)round(sqrt((double)n_requested * (height / width))); /* :54 */
    double cw = width / (double)ncx;                             /* :57 */
    double ch = height / (double)ncy;
    if (grid_total) *grid_total = (size_t)ncx * (size_t)ncy;
    size_t m = 0;
    for (int i = 0; i < ncy; ++i) {                              /* :66-73 */
        for (int j = 0; j < ncx; ++j) {
            double p2[2] = {((double)j + 0.5) * cw, ((double)i + 0.5) * ch};
            double r[3];
            if (oracle_unproject(model, params, w, h, p2, r) == OR_OK &&
                r[2] > 0.0) {                                    /* :91-103 */
                if (m < cap) {
                    uv_out[2 * m] = p2[0];
                    uv_out[2 * m + 1] = p2[1];
                    xyz_out[3 * m] = r[0];
                    xyz_out[3 * m + 1] = r[1];
                    xyz_out[3 * m + 2] = r[2];
                }
                ++m;
            }
        }
    }
    return m;
}

/* ------------------------------------------------------ FOV grid search */
/* src/camera/fov.rs:153-251, statement for statement: for each grid w the
 * points are visited in order and every finite error is added to a running
 * sum; the first w with the strictly smallest average wins. */
double oracle_fov_grid_search(const double *params, size_t n, const double *xyz,
                              const double *uv, double *error_sum,
                              double *valid_count) {
    const double fx = params[0], fy = params[1], cx = params[2], cy = params[3];
    double best_w = 1.0, best_error = INFINITY;
    for (int i = 10; i < 300; ++i) { /* :180 */
        const double w_test = (double)i / 100.0;
        double sum = 0.0;
        size_t cnt = 0;
        for (size_t k = 0; k < n; ++k) {
            const double x = xyz[3 * k], y = xyz[3 * k + 1], z = xyz[3 * k + 2];
            const double uo = uv[2 * k], vo = uv[2 * k + 1];
            const double r2 = x * x + y * y;                      /* :192 */
            const double r = sqrt(r2);
            const double tan_w_half = tan(w_test / 2.0);          /* :195 */
            const double atan_wrd = atan2(2.0 * tan_w_half * r, z);
            const double eps_sqrt = sqrt(DBL_EPSILON);            /* :198 */
            const double rd = r2 < eps_sqrt ? 2.0 * tan_w_half / w_test
                                            : atan_wrd / (r * w_test);
            const double mx = x * rd, my = y * rd;
            const double up = fx * mx + cx, vp = fy * my + cy;    /* :208-209 */
            const double du = up - uo, dv = vp - vo;
            const double e = sqrt(du * du + dv * dv);             /* :211-213 */
            if (isfinite(e)) { sum += e; ++cnt; }
        }
        error_sum[i - 10] = sum;
        valid_count[i - 10] = (double)cnt;
        if (cnt > 0) { /* :221-227 */
            const double avg = sum / (double)cnt;
            if (avg < best_error) { best_error = avg; best_w = w_test; }
        }
    }
    /* :166-171 rejects n < 2 before searching; the sums are still filled so
     * the GPU grid can be checked at n = 0 / 1 too. */
    return n < 2 ? -1.0 : best_w;
}

/* -------------------------------------------------------- linear estimation */
int oracle_linear_estimation_system(int model, const double *params, size_t n,
                                    const double *xyz, const double *uv,
                                    double *A, double *b) {
    double fx = params[0], fy = params[1], cx = params[2], cy = params[3];
    if (model == OR_KB) { /* src/camera/kannala_brandt.rs:164-272 */
        if (n < 4) return -1;
        memset(A, 0, sizeof(double) * 8 * n);
        memset(b, 0, sizeof(double) * 2 * n);
        for (size_t i = 0; i < n; ++i) {
            double X = xyz[3 * i], Y = xyz[3 * i + 1], Z = xyz[3 * i + 2];
            double u = uv[2 * i], v = uv[2 * i + 1];
            if (Z <= F64_EPS) continue;                          /* :195-197 */
            double r = sqrt(X * X + Y * Y);
            double theta = atan2(r, Z);
            double t2 = theta * theta, t3 = t2 * theta, t5 = t3 * t2;
            double t7 = t5 * t2, t9 = t7 * t2;
            double *a0 = A + 2 * i * 4, *a1 = A + (2 * i + 1) * 4;
            a0[0] = t3; a0[1] = t5; a0[2] = t7; a0[3] = t9;      /* :208-216 */
            a1[0] = t3; a1[1] = t5; a1[2] = t7; a1[3] = t9;
            double x_r = r < F64_EPS ? 0.0 : X / r;              /* :218-227 */
            double y_r = r < F64_EPS ? 0.0 : Y / r;
            if (fabs(fx * x_r) < F64_EPS && fabs(x_r) > F64_EPS) return -2;
            if (fabs(fy * y_r) < F64_EPS && fabs(y_r) > F64_EPS) return -2;
            if (fabs(x_r) > F64_EPS)                             /* :240-248 */
                b[2 * i] = (u - cx) / (fx * x_r) - theta;
            else
                b[2 * i] = fabs(u - cx) < F64_EPS ? -theta : 0.0;
            if (fabs(y_r) > F64_EPS)                             /* :250-259 */
                b[2 * i + 1] = (v - cy) / (fy * y_r) - theta;
            else
                b[2 * i + 1] = fabs(v - cy) < F64_EPS ? -theta : 0.0;
        }
        return 4;
    }
    if (model == OR_DS || model == OR_UCM || model == OR_EUCM) {
        /* double_sphere.rs:225-290, ucm.rs:200-258, eucm.rs:216-288 (the
         * three assemble the same 2N x 1 system) */
        if (model == OR_EUCM && n < 1) return -1;
        for (size_t i = 0; i < n; ++i) {
            double X = xyz[3 * i], Y = xyz[3 * i + 1], Z = xyz[3 * i + 2];
            double u = uv[2 * i], v = uv[2 * i + 1];
            double d = sqrt(X * X + Y * Y + Z * Z);
            double u_cx = u - cx, v_cy = v - cy;
            A[2 * i] = u_cx * (d - Z);
            A[2 * i + 1] = v_cy * (d - Z);
            b[2 * i] = (fx * X) - (u_cx * Z);
            b[2 * i + 1] = (fy * Y) - (v_cy * Z);
        }
        return 1;
    }
    if (model == OR_RADTAN) { /* src/camera/rad_tan.rs:153-234 */
        if (n < 3) return -1;
        for (size_t i = 0; i < n; ++i) {
            double X = xyz[3 * i], Y = xyz[3 * i + 1], Z = xyz[3 * i + 2];
            double u = uv[2 * i], v = uv[2 * i + 1];
            double xn = X / Z, yn = Y / Z;
            double r2 = xn * xn + yn * yn, r4 = r2 * r2, r6 = r4 * r2;
            double uu = fx * xn + cx, vu = fy * yn + cy;
            double *a0 = A + 2 * i * 3, *a1 = A + (2 * i + 1) * 3;
            a0[0] = fx * xn * r2; a0[1] = fx * xn * r4; a0[2] = fx * xn * r6;
            a1[0] = fy * yn * r2; a1[1] = fy * yn * r4; a1[2] = fy * yn * r6;
            b[2 * i] = u - uu;
            b[2 * i + 1] = v - vu;
        }
        return 3;
    }
    return -1;
}

/* ---------------------------------------------------------------- undistort */
/* Rust `f64 as i32`: saturating, NaN -> 0 */
static int rust_as_i32(double v) {
    if (v != v) return 0;
    if (v >= 2147483647.0) return 2147483647;
    if (v <= -2147483648.0) return (-2147483647 - 1);
    return (int)v;
}

/* src/util/undistort.rs:51-105 (interpolate_pixel).  Returns 1 and writes
 * rgb if the sample exists. */
static int interpolate_pixel(const uint8_t *img, uint32_t w, uint32_t h, double x,
                             double y, int bilinear, uint8_t rgb[3]) {
    if (!bilinear) {                                             /* :61-69 */
        int u = rust_as_i32(round(x)), v = rust_as_i32(round(y));
        if (u >= 0 && u < (int)w && v >= 0 && v < (int)h) {
            const uint8_t *p = img + ((size_t)v * w + (size_t)u) * 3;
            rgb[0] = p[0]; rgb[1] = p[1]; rgb[2] = p[2];
            return 1;
        }
        return 0;
    }
    double x0 = floor(x), y0 = floor(y);                         /* :71-74 */
    double x1 = x0 + 1.0, y1 = y0 + 1.0;
    if (x0 < 0.0 || x1 >= (double)w || y0 < 0.0 || y1 >= (double)h) return 0;
    uint32_t x0u = (uint32_t)x0, y0u = (uint32_t)y0, x1u = (uint32_t)x1, y1u = (uint32_t)y1;
    const uint8_t *p00 = img + ((size_t)y0u * w + x0u) * 3;
    const uint8_t *p10 = img + ((size_t)y0u * w + x1u) * 3;
    const uint8_t *p01 = img + ((size_t)y1u * w + x0u) * 3;
    const uint8_t *p11 = img + ((size_t)y1u * w + x1u) * 3;
    double wx = x - x0, wy = y - y0;                             /* :89-92 */
    double wx_inv = 1.0 - wx, wy_inv = 1.0 - wy;
    for (int c = 0; c < 3; ++c) {                                /* :95-101 */
        double val = (double)p00[c] * wx_inv * wy_inv + (double)p10[c] * wx * wy_inv +
                     (double)p01[c] * wx_inv * wy + (double)p11[c] * wx * wy;
        double r = round(val);
        r = r < 0.0 ? 0.0 : (r > 255.0 ? 255.0 : r);
        rgb[c] = (uint8_t)r;
    }
    return 1;
}

/* src/util/undistort.rs:14-49 (undistort_image).  img/out: row-major RGB8,
 * w x h = the model's resolution; target: fx fy cx cy. */
void oracle_undistort_image(int model, const double *params, uint32_t w, uint32_t h,
                            const double *target, int bilinear, const uint8_t *img,
                            uint8_t *out) {
    memset(out, 0, (size_t)w * h * 3);                           /* :31 */
    for (uint32_t v_out = 0; v_out < h; ++v_out) {
        for (uint32_t u_out = 0; u_out < w; ++u_out) {
            double x_norm = ((double)u_out - target[2]) / target[0]; /* :35 */
            double y_norm = ((double)v_out - target[3]) / target[1];
            double ray[3] = {x_norm, y_norm, 1.0};
            double uv[2];
            if (oracle_project(model, params, w, h, ray, uv) == OR_OK) {
                uint8_t rgb[3];
                if (interpolate_pixel(img, w, h, uv[0], uv[1], bilinear, rgb)) {
                    uint8_t *o = out + ((size_t)v_out * w + u_out) * 3;
                    o[0] = rgb[0]; o[1] = rgb[1]; o[2] = rgb[2];
                }
            }
        }
    }
}
