/*
 * acm_oracle.h -- CPU parity oracle for the batched camera-model hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in the product path (libacm.so, the
 * apex_camera_models package) may include, link or call this code.  Only
 * tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use it, as
 * the checker / the timed CPU restatement of the reference.
 *
 * This is a plain-C, operation-for-operation restatement of the reference's
 * single-threaded Rust per-point code (amin-abouee/apex-camera-models v0.4.1).
 * Every function cites the reference file:line it follows.  It is built with
 * -ffp-contract=off so every + and * rounds exactly like the Rust/nalgebra
 * code (Rust never contracts to FMA).  Transcendentals (atan2, sin, cos) come
 * from glibc libm, the same libm Rust's std uses on x86_64-linux-gnu.
 *
 * Parity pinning: the reference is Rust and no rustc/cargo exists in this
 * image, so the oracle is pinned by the reference's own known-answer tests
 * and fixtures (tests/golden/reference_kats.json, transcribed from the
 * reference test sources) plus an independent mpmath restatement
 * (tests/test_oracle_*.py).  The parameter Jacobians / factor residuals live
 * in the absent external crate apex-solver ^0.1.5 and are "parity unpinned"
 * against it; they are pinned against 50-digit mpmath derivatives instead.
 */
#ifndef ACM_ORACLE_H
#define ACM_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* model ids -- identical to include/acm.h */
enum {
    OR_PINHOLE = 0,
    OR_RADTAN = 1,
    OR_KB = 2,
    OR_DS = 3,
    OR_UCM = 4,
    OR_EUCM = 5,
    OR_FOV = 6
};

/* status codes -- mirror CameraModelError (src/camera/mod.rs:80-113) */
enum {
    OR_OK = 0,
    OR_PROJECTION_OUT_SIDE_IMAGE = 1,
    OR_POINT_IS_OUT_SIDE_IMAGE = 2,
    OR_POINT_AT_CAMERA_CENTER = 3,
    OR_NUMERICAL_ERROR = 4
};

int oracle_num_params(int model);

/* Per-point reference restatement.  params in factor order
 * (bin/camera_converter.rs:385-392 etc.).  Returns a status code. */
int oracle_project(int model, const double *params, uint32_t w, uint32_t h,
                   const double p[3], double uv[2]);
int oracle_unproject(int model, const double *params, uint32_t w, uint32_t h,
                     const double uv[2], double ray[3]);
/* project + analytic 2xP parameter Jacobian, J row-major [u-row | v-row]. */
int oracle_project_jacobian(int model, const double *params, uint32_t w,
                            uint32_t h, const double p[3], double uv[2],
                            double *J);

/* Batched loops over the per-point calls (the reference's caller loops).
 * xyz: nalgebra Matrix3xX column-major [x0 y0 z0 x1 ...]; uv: Matrix2xX.
 * jac: 2N x P column-major (nalgebra DMatrix) or NULL.
 * Invalid points: uv = NaN, J column entries = 0. */
void oracle_project_batch(int model, const double *params, uint32_t w,
                          uint32_t h, size_t n, const double *xyz, double *uv,
                          uint8_t *status, double *jac);
void oracle_unproject_batch(int model, const double *params, uint32_t w,
                            uint32_t h, size_t n, const double *uv,
                            double *xyz, uint8_t *status);
/* factor residual r = project(p) - obs (2N) and Jacobian (2N x P, col-major).
 * policy 0 = skip (r = 0, J = 0 on invalid points),
 * policy 1 = sentinel (r = (1e6, 1e6), J = 0). */
void oracle_residual_jacobian_batch(int model, const double *params,
                                    uint32_t w, uint32_t h, size_t n,
                                    const double *xyz, const double *uv_obs,
                                    int policy, double *res, double *jac,
                                    uint8_t *status);
/* Normal equations over the batch: JtJ (P x P full, row-major), Jtr (P),
 * cost = 0.5 * sum ||r||^2, n_valid.  Sums in point order (long double
 * accumulators so the checker is at least as accurate as the GPU). */
void oracle_normal_equations(int model, const double *params, uint32_t w,
                             uint32_t h, size_t n, const double *xyz,
                             const double *uv_obs, int policy, double *JtJ,
                             double *Jtr, double *cost, uint64_t *n_valid);

/* compute_reprojection_error (src/util/error_metrics.rs:62-121).
 * out = [rmse, min, max, mean, stddev, median]; returns number of valid
 * projections (0 -> the reference's ZeroProjectionPoints error). */
size_t oracle_reprojection_error(int model, const double *params, uint32_t w,
                                 uint32_t h, size_t n, const double *xyz,
                                 const double *uv, double out[6]);

/* sample_points (src/util/point_sampling.rs:46-120).  Writes up to
 * cap kept points (uv_out 2xM, xyz_out 3xM, both column-major) and returns M
 * (the number kept); *grid_total receives num_cells_x*num_cells_y. */
size_t oracle_sample_points(int model, const double *params, uint32_t w,
                            uint32_t h, size_t n_requested, size_t cap,
                            double *uv_out, double *xyz_out,
                            size_t *grid_total);

/* linear_estimation A (2N x k, row-major) and b (2N) assembly for
 * KB (k=4), DS/UCM/EUCM (k=1), RadTan (k=3).  Returns k, or <0 on the
 * reference's error paths (-1 InvalidParams, -2 NumericalError). */
int oracle_linear_estimation_system(int model, const double *params,
                                    size_t n, const double *xyz,
                                    const double *uv, double *A, double *b);

/* FOV linear_estimation (src/camera/fov.rs:153-251): the grid search over
 * w = i/100, i = 10..299.  Writes, per grid value, the serial error sum and
 * the finite-error count (both 290 long), and returns the w the reference
 * keeps (before its clamp / validate), or -1.0 if n < 2 (InvalidParams;
 * the sums are filled in either case). */
#define ORACLE_FOV_GRID 290
double oracle_fov_grid_search(const double *params, size_t n, const double *xyz,
                              const double *uv, double *error_sum,
                              double *valid_count);

/* undistort_image (src/util/undistort.rs:14-105): RGB8 row-major w x h,
 * target = [fx fy cx cy], bilinear 0 = Nearest, 1 = Bilinear. */
void oracle_undistort_image(int model, const double *params, uint32_t w,
                            uint32_t h, const double *target, int bilinear,
                            const uint8_t *img, uint8_t *out);

#ifdef __cplusplus
}
#endif
#endif
