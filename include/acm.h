/*
 * acm.h -- C-ABI of the MI355X-native batched camera-model engine (libacm.so).
 *
 * Drop-in boundary for the reference's one data-parallel hot path
 * (amin-abouee/apex-camera-models v0.4.1, a pure-Rust crate):
 *
 *   trait CameraModel::project    src/camera/mod.rs:256   (per point, Result)
 *   trait CameraModel::unproject  src/camera/mod.rs:271   (per point, Result)
 *   apex_solver::factors::*CameraParamsFactor  (residual 2N + Jacobian 2N x P,
 *       constructed at bin/camera_converter.rs:378,513,652,794,925,1058)
 *   util::compute_reprojection_error   src/util/error_metrics.rs:62-121
 *   util::sample_points                src/util/point_sampling.rs:46-120
 *
 * Every entry point is batched (a per-point FFI call would be latency bound),
 * takes plain pointers and sizes, never allocates on the hot path, and is
 * stream-ordered on the caller's HIP stream (`void *stream`, NULL = default
 * stream).  All point/ray/residual/Jacobian buffers are DEVICE pointers owned
 * by the caller (hipMalloc'd or from any allocator on the same HIP runtime).
 *
 * Memory layouts (all f64):
 *   points_3d  ACM_LAYOUT_AOS: nalgebra Matrix3xX column-major [x0 y0 z0 x1 ..]
 *              ACM_LAYOUT_SOA: three planes [x0..x(N-1) | y0.. | z0..]
 *   points_2d  nalgebra Matrix2xX column-major [u0 v0 u1 v1 ..]
 *   jacobian   nalgebra DMatrix 2N x P column-major: entry (2i+r, p) at
 *              jacobian[p*2N + 2i + r], r=0 for u, r=1 for v.  Parameter order
 *              is the factor's (camera_converter.rs:385-392, :520-529, ...).
 *   status     one uint8 per point, values acm_point_status below.
 *
 * Return codes: ACM_SUCCESS (0) or a negative acm_result.
 */
#ifndef ACM_H
#define ACM_H

#include <stddef.h>
#include <stdint.h>

#if defined(__GNUC__)
#define ACM_API __attribute__((visibility("default")))
#else
#define ACM_API
#endif

#ifdef __cplusplus
extern "C" {
#endif

/* Camera model ids.  Parameter vectors (factor order):
 *   PINHOLE  fx fy cx cy                       (src/camera/pinhole.rs)
 *   RADTAN   fx fy cx cy k1 k2 p1 p2 k3        (src/camera/rad_tan.rs)
 *   KB       fx fy cx cy k1 k2 k3 k4           (src/camera/kannala_brandt.rs)
 *   DS       fx fy cx cy alpha xi              (src/camera/double_sphere.rs)
 *   UCM      fx fy cx cy alpha                 (src/camera/ucm.rs)
 *   EUCM     fx fy cx cy alpha beta            (src/camera/eucm.rs)
 *   FOV      fx fy cx cy w                     (src/camera/fov.rs)          */
typedef enum acm_model {
    ACM_PINHOLE = 0,
    ACM_RADTAN = 1,
    ACM_KANNALA_BRANDT = 2,
    ACM_DOUBLE_SPHERE = 3,
    ACM_UCM = 4,
    ACM_EUCM = 5,
    ACM_FOV = 6
} acm_model;

/* Per-point status, mirroring the CameraModelError variants a projection or
 * unprojection can return (src/camera/mod.rs:80-113). */
typedef enum acm_point_status {
    ACM_STATUS_OK = 0,
    ACM_STATUS_PROJECTION_OUT_SIDE_IMAGE = 1, /* ProjectionOutSideImage */
    ACM_STATUS_POINT_IS_OUT_SIDE_IMAGE = 2,   /* PointIsOutSideImage */
    ACM_STATUS_POINT_AT_CAMERA_CENTER = 3,    /* PointAtCameraCenter */
    ACM_STATUS_NUMERICAL_ERROR = 4            /* NumericalError(_) */
} acm_point_status;

/* Function results.  The positive CameraModelError codes returned by
 * acm_validate_params mirror mod.rs:80-113 variant order + 1. */
typedef enum acm_result {
    ACM_SUCCESS = 0,
    ACM_ERR_INVALID_MODEL = -1,
    ACM_ERR_INVALID_PARAMS = -2, /* CameraModelError::InvalidParams */
    ACM_ERR_INVALID_ARGUMENT = -3,
    ACM_ERR_HIP = -4,
    ACM_ERR_WORKSPACE_TOO_SMALL = -5,
    ACM_ERR_NOT_SUPPORTED = -6,
    ACM_ERR_NUMERICAL = -7 /* CameraModelError::NumericalError */
} acm_result;

typedef enum acm_validation {
    ACM_VALID = 0,
    ACM_FOCAL_LENGTH_MUST_BE_POSITIVE = 4, /* FocalLengthMustBePositive */
    ACM_PRINCIPAL_POINT_MUST_BE_FINITE = 5, /* PrincipalPointMustBeFinite */
    ACM_INVALID_DISTORTION = 6             /* InvalidParams(alpha/xi/beta) */
} acm_validation;

enum { ACM_LAYOUT_AOS = 0, ACM_LAYOUT_SOA = 1 };

/* Per-call option OR-ed into acm_project's `layout`: reference-exact math for
 * Kannala-Brandt and FOV (IEEE sqrt / divisions and a correctly rounded
 * double-double atan2 instead of the fast polynomial / rsq forms, ~1e-16
 * apart).  Projections and Jacobians then equal the reference (Rust f64 +
 * glibc libm) bit for bit wherever glibc's atan2 is correctly rounded, i.e.
 * on all but ~0.2% of arguments, where the two differ by one ulp.  The other
 * five models are reference-exact without it (the flag is ignored). */
enum { ACM_EXACT_MATH = 0x100 };

/* Per-call option OR-ed into acm_unproject's `layout` (and passed in
 * acm_sample_points_ex's `flags`): the reference's own Newton loops for every
 * pixel (kannala_brandt.rs:474-511, rad_tan.rs:436-518) instead of the
 * certified fast ones, and FOV's IEEE unprojection (fov.rs:336-363) instead
 * of its reciprocal / polynomial form.  Statuses (and the sample_points kept
 * set) are identical either way; with the flag RadTan's rays equal the
 * reference's bit for bit (by default they agree within a few ulp).  A
 * per-call choice, so two callers on different threads can use different
 * numerics on the same library (the reference's CameraModel is Send + Sync,
 * mod.rs:241-340).  Replaces the process-wide ACM_TUNE_NEWTON_FAST knob. */
enum { ACM_REFERENCE_NEWTON = 0x200 };

/* Invalid-point policy of the factor evaluation (apex-solver source absent:
 * "skip" matches compute_reprojection_error skipping failed projections,
 * error_metrics.rs:76; "sentinel" is the (1e6,1e6) residual of the removed
 * in-tree factor, doc/COMPREHENSIVE_ANALYSIS.md:116-121).  J = 0 in both. */
enum { ACM_INVALID_SKIP = 0, ACM_INVALID_SENTINEL = 1 };

#define ACM_MAX_PARAMS 9

/* A camera: model id, resolution and the factor-order parameter vector.
 * Replaces the model structs (e.g. KannalaBrandtModel,
 * kannala_brandt.rs:65-72).  Passed by value into every kernel, so the
 * parameters live in SGPRs (uniform across the wave), not in HBM or LDS. */
typedef struct acm_camera {
    int32_t model;
    uint32_t width;
    uint32_t height;
    uint32_t num_params;
    double params[ACM_MAX_PARAMS];
} acm_camera;

/* Number of parameters of a model (Pinhole 4 .. RadTan 9), or -1. */
ACM_API int acm_num_params(int model);

/* Fill *cam.  Mirrors XModel::new(&DVector): wrong parameter count ->
 * ACM_ERR_INVALID_PARAMS (kannala_brandt.rs:122-128, pinhole.rs:60-66, ...).
 * Like the reference, Pinhole and RadTan also run validate_params here
 * (pinhole.rs:80, rad_tan.rs:135): a failure returns ACM_ERR_INVALID_PARAMS.*/
ACM_API int acm_camera_init(acm_camera *cam, int model, const double *params,
                            size_t num_params, uint32_t width, uint32_t height);

/* validate_params (mod.rs:362-371 + per-model rules, e.g.
 * double_sphere.rs:592-607).  Returns an acm_validation code. */
ACM_API int acm_validate_params(const acm_camera *cam);

/* Batched CameraModel::project (+ optional dense parameter Jacobian).
 * points_3d: 3N f64 (layout, optionally | ACM_EXACT_MATH), points_2d: 2N f64
 * out, status: N u8 out,
 * jacobian: 2N*P f64 out or NULL.  Failed points: uv = NaN, J = 0.
 * Replaces mod.rs:256 (per point) and the factor's Jacobian. */
ACM_API int acm_project(const acm_camera *cam, size_t n,
                        const double *points_3d, int layout, double *points_2d,
                        uint8_t *status, double *jacobian, void *stream);

/* The same projection evaluated in f32 (float buffers, same layouts; the
 * camera parameters are rounded to float).  For the f32-vs-f64 tolerance
 * sweep of BASELINE config 5; the reference itself is f64 only. */
ACM_API int acm_project_f32(const acm_camera *cam, size_t n,
                            const float *points_3d, int layout, float *points_2d,
                            uint8_t *status, float *jacobian, void *stream);

/* Batched CameraModel::unproject (mod.rs:271).  rays: 3N f64 out written in
 * `layout` (optionally | ACM_REFERENCE_NEWTON); failed points: ray = NaN. */
ACM_API int acm_unproject(const acm_camera *cam, size_t n,
                          const double *points_2d, double *rays, int layout,
                          uint8_t *status, void *stream);

/* Factor linearisation: residual r = project(p_i) - obs_i (2N) and the
 * 2N x P Jacobian (nullable) of *CameraParamsFactor
 * (camera_converter.rs:378 & co).  status nullable. */
/* Project -> unproject round trip (BASELINE config 4; the reference's
 * per-point loop of tests/projection_accuracy.rs over mod.rs:256 and :271)
 * in one pass: writes exactly what acm_project (no Jacobian) followed by
 * acm_unproject of its pixels writes -- points_2d (NaN where the projection
 * failed), status, rays (NaN where the unprojection failed) and ray_status
 * -- bit for bit, without reading the pixels back from memory.  layout as
 * acm_project / acm_unproject; with ACM_EXACT_MATH or ACM_REFERENCE_NEWTON
 * set it runs the two calls in order. (r04) */
ACM_API int acm_project_unproject(const acm_camera *cam, size_t n,
                                  const double *points_3d, int layout,
                                  double *points_2d, uint8_t *status,
                                  double *rays, uint8_t *ray_status,
                                  void *stream);
ACM_API int acm_residual_jacobian(const acm_camera *cam, size_t n,
                                  const double *points_3d, int layout,
                                  const double *points_2d_obs,
                                  int invalid_policy, double *residual,
                                  double *jacobian, uint8_t *status,
                                  void *stream);

/* Fused LM linearisation: JtJ (P x P, row-major, symmetric), Jtr (P),
 * cost = 0.5*sum ||r||^2 and n_valid, without materialising r or J.
 * result (device, f64): [JtJ (P*P) | Jtr (P) | cost | n_valid].
 * Deterministic: fixed per-block partials + an ordered final sum.  The
 * workspace (device) must hold acm_normal_equations_workspace_size bytes. */
ACM_API size_t acm_normal_equations_workspace_size(int model, size_t n);
ACM_API int acm_normal_equations(const acm_camera *cam, size_t n,
                                 const double *points_3d, int layout,
                                 const double *points_2d_obs,
                                 int invalid_policy, double *result,
                                 void *workspace, size_t workspace_bytes,
                                 void *stream);

/* compute_reprojection_error (error_metrics.rs:62-121) minus the median:
 * result (device, f64): [rmse, min, max, mean, stddev, n_valid, sum, sumsq]
 * errors (nullable, device, N f64): per-point ||proj - obs||, NaN if failed.
 * The stddev is sum((e - mean)^2) / n (the reference's two-pass form)
 * computed in the same single pass: per-lane shifted sums merged with
 * Chan's pairwise update (equal up to rounding). */
ACM_API size_t acm_reprojection_stats_workspace_size(size_t n);
ACM_API int acm_reprojection_stats(const acm_camera *cam, size_t n,
                                   const double *points_3d, int layout,
                                   const double *points_2d, double *result,
                                   double *errors, void *workspace,
                                   size_t workspace_bytes, void *stream);
/* compute_reprojection_error (error_metrics.rs:62-121) in full, one call:
 * result (device, 9 f64) = acm_reprojection_stats' 8 + [8] the median of the
 * valid errors (acm_median_valid's rule; NaN when n_valid = 0).  The
 * statistics pass also counts the median's first radix-select histogram
 * (per workgroup, merged afterwards), so the median reads the errors one
 * time fewer than acm_reprojection_stats + acm_median_valid, and n_valid
 * stays on the device in between.  errors: nullable device N f64 output
 * (NaN if failed); when NULL they live in the workspace. */
ACM_API size_t acm_reprojection_error_workspace_size(size_t n);
ACM_API int acm_reprojection_error(const acm_camera *cam, size_t n,
                                   const double *points_3d, int layout,
                                   const double *points_2d, double *result,
                                   double *errors, void *workspace,
                                   size_t workspace_bytes, void *stream);
/* Host-side merge of the results of disjoint shards (the multi-GPU form of
 * compute_reprojection_error, error_metrics.rs:86-111): parts = nparts x 8
 * host doubles, each an acm_reprojection_stats result, folded in order --
 * sums added, extrema combined, (n_valid, mean, n * stddev^2) merged by
 * Chan's pairwise update -- into result (8 host doubles, same layout).  One
 * all-gather of the 8 doubles per rank + this merge gives every rank the
 * same statistics bit for bit.  A point whose error is NaN (failed
 * projection or NaN observation) is never counted. */
ACM_API int acm_reprojection_stats_merge(size_t nparts, const double *parts, double *result);

/* The same 8-double result from an error vector already in HBM (errors:
 * device, N f64, NaN = invalid; e.g. a shard's acm_reprojection_stats
 * `errors` output): the per-shard leg of the multi-GPU statistics
 * (error_metrics.rs:86-111 over one shard) without copying the errors to the
 * host.  Same per-workgroup shifted sums + fixed-order Chan merge as
 * acm_reprojection_stats, so bit-reproducible run to run. */
ACM_API size_t acm_error_stats_workspace_size(size_t n);
ACM_API int acm_error_stats(size_t n, const double *errors, double *result,
                            void *workspace, size_t workspace_bytes, void *stream);

/* linear_estimation (kannala_brandt.rs:164-272, double_sphere.rs:225-290,
 * ucm.rs:200-258, eucm.rs:216-288, rad_tan.rs:153-234).  The 2N x k system
 * [A | b] is never materialised: acm_linear_system_qr reduces its rows on
 * the GPU into the (k+1)x(k+1) upper-triangular R factor of a tall-skinny QR
 * (r_factor: device, packed row-major upper triangle; error_flag: device int,
 * set on the reference's NumericalError path).  acm_linear_estimation then
 * solves R_A x = z on the host with nalgebra's SVD::solve(eps) semantics
 * (eps = f64::EPSILON for KB, 1e-10 otherwise), applies the model's clamps
 * and validation, and writes the estimate into cam->params (k = 4 KB,
 * 3 RadTan, 1 DS/UCM/EUCM; FOV: the grid search below). */
ACM_API int acm_linear_system_columns(int model);
ACM_API size_t acm_linear_system_qr_workspace_size(int model, size_t n);
ACM_API int acm_linear_system_qr(const acm_camera *cam, size_t n,
                                 const double *points_3d, int layout,
                                 const double *points_2d, double *r_factor,
                                 int *error_flag, void *workspace,
                                 size_t workspace_bytes, void *stream);
ACM_API size_t acm_linear_estimation_workspace_size(int model, size_t n);
/* convert_to_*'s opening (camera_converter.rs:371-375): the reprojection
 * error of *cam as given (initial_error; device, 9 f64 as
 * acm_reprojection_error) and then linear_estimation of *cam (updated in
 * place, return code as acm_linear_estimation) -- for the TSQR models in ONE
 * pass over the correspondences (k_tsqr also computes the errors, their
 * statistics and the median's first histogram).  The initial error is
 * written even when the estimation then fails (as the reference computes it
 * first); for FOV and too-few-point calls the two run one after the other. */
ACM_API size_t acm_linear_estimation_with_error_workspace_size(int model, size_t n);
ACM_API int acm_linear_estimation_with_error(acm_camera *cam, size_t n,
                                             const double *points_3d, int layout,
                                             const double *points_2d,
                                             double *initial_error, void *workspace,
                                             size_t workspace_bytes, void *stream);
/* (r05) The same, returning as soon as *cam is estimated: the initial
 * error's 8 statistics (acm_reprojection_stats' layout, n_valid at [5]) are
 * copied to initial_error_host (nullable, host, 8 f64) before the median
 * runs, the host solve overlaps the median, and the median itself lands in
 * initial_error[8] in stream order (read it after a later synchronisation of
 * `stream`; the workspace must stay allocated until then).  What
 * conversion.convert uses, so the LM's first evaluation queues behind the
 * median without a host round trip in between.  acm_linear_estimation_with_error
 * is this call followed by a synchronisation of `stream`. */
ACM_API int acm_linear_estimation_with_error_async(acm_camera *cam, size_t n,
                                                   const double *points_3d, int layout,
                                                   const double *points_2d,
                                                   double *initial_error,
                                                   double *initial_error_host, void *workspace,
                                                   size_t workspace_bytes, void *stream);
/* Multi-GPU linear_estimation: each rank runs acm_linear_system_qr on its
 * shard, the packed factors (host copies) are folded in rank order with
 * acm_linear_system_r_merge (Givens; R of the stacked rows), error flags
 * OR-ed, and acm_linear_estimation_solve finishes on every rank with the
 * global point count.  acm_linear_estimation = qr + solve on one GPU. */
ACM_API int acm_linear_system_r_merge(int model, double *r_inout,
                                      const double *r_other);
ACM_API int acm_linear_estimation_solve(acm_camera *cam, size_t n_total,
                                        const double *r_factor_host,
                                        int error_flag);
ACM_API int acm_linear_estimation(acm_camera *cam, size_t n,
                                  const double *points_3d, int layout,
                                  const double *points_2d, void *workspace,
                                  size_t workspace_bytes, void *stream);

/* FOV linear_estimation (fov.rs:153-251) is a grid search, not a linear
 * system: for w = i/100, i = 10..299 (ACM_FOV_GRID_SIZE values) the sum of
 * finite reprojection errors and their count over all points.
 * acm_fov_grid_errors writes grid_sums (device, 2 x 290 doubles: the 290
 * error sums, then the 290 counts); the sums are additive over shards of
 * the points, so a multi-GPU caller all-reduces them before
 * acm_fov_grid_select, which keeps the first w with the strictly smallest
 * mean (host array), applies the clamp to [0.01, 3] and validate_params,
 * and writes w into cam->params[4].  acm_linear_estimation runs both for
 * ACM_FOV (n < 2 -> ACM_ERR_INVALID_PARAMS, fov.rs:166-171). */
#define ACM_FOV_GRID_SIZE 290
ACM_API size_t acm_fov_grid_workspace_size(size_t n);
ACM_API int acm_fov_grid_errors(const acm_camera *cam, size_t n,
                                const double *points_3d, int layout,
                                const double *points_2d, double *grid_sums,
                                void *workspace, size_t workspace_bytes,
                                void *stream);
ACM_API int acm_fov_grid_select(acm_camera *cam, const double *grid_sums_host);

/* Bounded Levenberg-Marquardt over the fused normal equations: the
 * apex-solver call of camera_converter.rs:381-420.  Each evaluation runs
 * acm_normal_equations, then (if allreduce != NULL) hands the device result
 * vector [JtJ | Jtr | cost | n_valid] to the callback for a cross-rank sum
 * (e.g. RCCL all-reduce), copies it to the host and solves the damped
 * P x P system by Cholesky.  cam->params: initial value in, optimum out. */
typedef struct acm_lm_config {
    int32_t max_iterations;      /* 100 (camera_converter.rs:411) */
    int32_t invalid_policy;      /* ACM_INVALID_SKIP / _SENTINEL */
    double cost_tolerance;       /* 1e-6 relative cost decrease */
    double parameter_tolerance;  /* 1e-8 */
    double gradient_tolerance;   /* 1e-6 on |Jtr|_inf */
    double initial_damping;      /* mu0 (Marquardt-scaled), 1e-4 */
    uint32_t has_bounds;
    uint32_t reserved;
    double lower[ACM_MAX_PARAMS]; /* set_variable_bounds */
    double upper[ACM_MAX_PARAMS];
} acm_lm_config;

enum {
    ACM_LM_MAX_ITERATIONS = 0,
    ACM_LM_COST = 1,
    ACM_LM_PARAMETER = 2,
    ACM_LM_GRADIENT = 3,
    ACM_LM_FAILED = 4
};

typedef struct acm_lm_summary {
    int32_t iterations;
    int32_t termination; /* ACM_LM_* */
    int32_t evaluations;
    int32_t reserved;
    double initial_cost; /* 0.5 * sum ||r||^2 */
    double final_cost;
    double n_valid;
} acm_lm_summary;

typedef int (*acm_allreduce_fn)(void *ctx, double *device_buffer, size_t count,
                                void *stream);

/* (r06) Grid-sampled correspondences by cell (acm_sample_points_cells):
 * cell c = i * num_cells_x + j of the row-major grid whose centres are
 * ((j + 0.5) * width / num_cells_x, (i + 0.5) * height / num_cells_y)
 * (point_sampling.rs:56-78; width, height: the SAMPLED camera's
 * resolution).  A uint32 per point instead of the 16-B pixel: the cell
 * forms below recompute each pixel exactly as sample_points wrote it, so
 * their results are the pixel forms' bit for bit (with the default
 * ACM_TUNE_NE_WAVES / NE_UNROLL, which they always use). */
typedef struct acm_cell_grid {
    uint32_t num_cells_x, num_cells_y;
    uint32_t width, height;
} acm_cell_grid;
ACM_API int acm_normal_equations_cells(const acm_camera *cam, size_t n,
                                       const double *points_3d, int layout,
                                       const uint32_t *cells, const acm_cell_grid *grid,
                                       int invalid_policy, double *result, void *workspace,
                                       size_t workspace_bytes, void *stream);

ACM_API void acm_lm_default_config(acm_lm_config *cfg);
ACM_API size_t acm_lm_workspace_size(int model, size_t n);
ACM_API int acm_lm_optimize(acm_camera *cam, size_t n, const double *points_3d,
                            int layout, const double *points_2d,
                            const acm_lm_config *cfg, acm_allreduce_fn allreduce,
                            void *allreduce_ctx, acm_lm_summary *summary,
                            void *workspace, size_t workspace_bytes, void *stream);
/* (r06) acm_lm_optimize over cell-form observations (acm_cell_grid):
 * the same iterates, 12 B per point less read per evaluation.  Workspace:
 * acm_lm_workspace_size. */
ACM_API int acm_lm_optimize_cells(acm_camera *cam, size_t n, const double *points_3d,
                                  int layout, const uint32_t *cells,
                                  const acm_cell_grid *grid, const acm_lm_config *cfg,
                                  acm_allreduce_fn allreduce, void *allreduce_ctx,
                                  acm_lm_summary *summary, void *workspace,
                                  size_t workspace_bytes, void *stream);
/* (r06) The conversion's other two passes in the cell form, the same bits:
 * acm_reprojection_error over cell-form observations (workspace:
 * acm_reprojection_error_workspace_size), and
 * acm_linear_estimation_with_error_async whose fused pass reads the cells
 * (points_2d still required: the FOV grid search and the too-few-points
 * path read pixels; workspace: acm_linear_estimation_with_error_workspace_size). */
ACM_API int acm_reprojection_error_cells(const acm_camera *cam, size_t n,
                                         const double *points_3d, int layout,
                                         const uint32_t *cells, const acm_cell_grid *grid,
                                         double *result, double *errors, void *workspace,
                                         size_t workspace_bytes, void *stream);
ACM_API int acm_linear_estimation_with_error_cells_async(
    acm_camera *cam, size_t n, const double *points_3d, int layout, const double *points_2d,
    const uint32_t *cells, const acm_cell_grid *grid, double *initial_error,
    double *initial_error_host, void *workspace, size_t workspace_bytes, void *stream);

/* (r06) The sharded conversion's collectives.  One
 * process per GPU, each holding a shard of the correspondences; both
 * collectives are stream-ordered on device f64 buffers:
 *   allreduce -- in-place sum over the ranks (the acm_allreduce_fn of
 *                acm_lm_optimize / acm_median_valid_allreduce);
 *   allgather -- every rank's `count` values into recv (world x count, in
 *                rank order).
 * acm_rccl_init builds one over an RCCL communicator that libacm drives
 * itself (librccl.so.1: the copy already loaded in the process, e.g.
 * torch's, else ROCm's), so no Python runs per collective; rank 0 makes the
 * id (acm_rccl_unique_id), the caller broadcasts it (e.g. through
 * torch.distributed) and every rank calls acm_rccl_init with its own GPU
 * current -- one GPU per rank.  acm_rccl_destroy frees it.  Any other
 * transport can fill the struct with its own callbacks (the tests' gloo
 * ranks sharing one GPU do). */
typedef int (*acm_allgather_fn)(void *ctx, const double *send, double *recv,
                                size_t count, void *stream);
typedef struct acm_collective {
    acm_allreduce_fn allreduce;
    acm_allgather_fn allgather;
    void *ctx;
    int32_t rank;
    int32_t world;
} acm_collective;
#define ACM_RCCL_UNIQUE_ID_BYTES 128
ACM_API int acm_rccl_available(void);
ACM_API int acm_rccl_unique_id(uint8_t *id);
ACM_API int acm_rccl_init(const uint8_t *id, int32_t world, int32_t rank,
                          acm_collective *out);
ACM_API int acm_rccl_destroy(acm_collective *coll);

/* (r06) convert_to_*'s opening over the union of the ranks' shards
 * (camera_converter.rs:371-375; the multi-GPU form of
 * acm_linear_estimation_with_error_async): per shard the same fused pass
 * (R factor, error flag, the 8 statistics, the median's first histogram),
 * then ONE all-gather of a 32-double record per rank, the rank-ordered
 * Givens merge of the factors and Chan merge of the statistics on the host,
 * the exact median of the union (every histogram summed by coll->allreduce;
 * it lands in initial_error[8] in stream order, initial_error[0..7] hold the
 * union's statistics), and the solve (count checks on the union's size).
 * FOV: the statistics, then the grid sums all-reduced and
 * acm_fov_grid_select.  Every rank gets the same cam->params bit for bit;
 * with one rank (coll NULL, or world 1) the bits of the 1-GPU call.
 * initial_error_host: nullable, host, the union's 8 statistics.
 * cells / grid: nullable, the shard's observations also in the cell form
 * (acm_cell_grid): the fused pass then reads those (same bits); points_2d
 * is still required (the FOV grid search reads pixels). */
ACM_API size_t acm_linear_estimation_with_error_sharded_workspace_size(int model, size_t n,
                                                                       int32_t world);
ACM_API int acm_linear_estimation_with_error_sharded(acm_camera *cam, size_t n,
                                                     const double *points_3d, int layout,
                                                     const double *points_2d,
                                                     const uint32_t *cells,
                                                     const acm_cell_grid *grid,
                                                     double *initial_error,
                                                     double *initial_error_host,
                                                     const acm_collective *coll,
                                                     void *workspace, size_t workspace_bytes,
                                                     void *stream);
/* (r06) compute_reprojection_error (error_metrics.rs:62-121) over the union
 * of the ranks' shards: this shard's statistics pass (with the median's
 * first histogram), one all-gather of the records, Chan's merge, the
 * distributed exact median.  result: device, 9 f64 as acm_reprojection_error
 * (the union's), identical on every rank; errors: nullable device N f64.
 * cells / grid: nullable, the cell form of the observations (then
 * points_2d may be NULL). */
ACM_API size_t acm_reprojection_error_sharded_workspace_size(size_t n, int32_t world);
ACM_API int acm_reprojection_error_sharded(const acm_camera *cam, size_t n,
                                           const double *points_3d, int layout,
                                           const double *points_2d, const uint32_t *cells,
                                           const acm_cell_grid *grid, double *result,
                                           double *errors, const acm_collective *coll,
                                           void *workspace, size_t workspace_bytes,
                                           void *stream);

/* Exact median of the non-NaN values of `values` (the per-point errors of
 * acm_reprojection_stats), error_metrics.rs:103-111: the mean of ranks
 * m/2-1 and m/2 for even m, rank m/2 for odd m, m = n_valid (read from
 * device memory n_valid_device if non-NULL, e.g. result[5] of
 * acm_reprojection_stats, else the host value n_valid).  Values must be
 * >= 0 or NaN.  out: device f64.
 * acm_median_valid_allreduce is the multi-GPU form: `values` is this
 * rank's shard, n_valid the GLOBAL count, and after each of the 6
 * histogram passes the 2 x 2048-bin f64 histogram (device; both median
 * ranks, 11-bit digits) goes through the allreduce callback (a sum over
 * ranks), so every rank selects the same digits and returns the median of
 * the union.  Two passes read all n values; the candidates sharing the
 * selected 22-bit prefix are then compacted into the workspace (which is
 * sized for n of them) and the last four passes read only those. */
ACM_API size_t acm_median_workspace_size(size_t n);
ACM_API int acm_median_valid(size_t n, const double *values,
                             const double *n_valid_device, uint64_t n_valid,
                             double *out, void *workspace,
                             size_t workspace_bytes, void *stream);
ACM_API int acm_median_valid_allreduce(size_t n, const double *values,
                                       const double *n_valid_device,
                                       uint64_t n_valid, double *out,
                                       void *workspace, size_t workspace_bytes,
                                       acm_allreduce_fn allreduce,
                                       void *allreduce_ctx, void *stream);

/* util::sample_points (point_sampling.rs:46-120): a grid of
 * round(sqrt(n*w/h)) x round(sqrt(n*h/w)) cell centres (row-major, as the
 * reference loop), each unprojected; a cell is kept iff the unprojection
 * succeeds and ray.z > 0, in grid order (order-preserving compaction, so
 * indices match the reference's Vec::push order).
 * acm_sample_points_grid (host) gives the grid; the output buffers must hold
 * ncx*ncy points (points_2d_out 2*cap f64, points_3d_out 3*cap f64 AoS).
 * counts (device, 2 x uint64): [kept, ncx*ncy]. */
ACM_API int acm_sample_points_grid(uint32_t width, uint32_t height, size_t n_requested,
                                   uint32_t *num_cells_x, uint32_t *num_cells_y);
ACM_API size_t acm_sample_points_workspace_size(const acm_camera *cam, size_t n_requested);
ACM_API int acm_sample_points(const acm_camera *cam, size_t n_requested,
                              double *points_2d_out, double *points_3d_out,
                              uint64_t *counts, void *workspace,
                              size_t workspace_bytes, void *stream);
/* Same over the cell range [cell_begin, cell_end) of the row-major grid (a
 * multi-GPU shard: ranks take contiguous row ranges and concatenating their
 * outputs in rank order reproduces the serial order).  counts[1] = cells in
 * the range.  Workspace: acm_sample_points_workspace_size of the full grid
 * is always enough. */
ACM_API int acm_sample_points_range(const acm_camera *cam, size_t n_requested,
                                    size_t cell_begin, size_t cell_end,
                                    double *points_2d_out, double *points_3d_out,
                                    uint64_t *counts, void *workspace,
                                    size_t workspace_bytes, void *stream);
/* The host-certified keep regions acm_sample_points counts segments by
 * (inspection / tests; csrc/acm.hip kb_seg_cert): out = [on, all_lo, all_hi,
 * none_lo, none_hi] in the model's certificate variable (KB: ru =
 * min(sqrt(mx^2 + my^2), pi/2); others: r2 = mx^2 + my^2).  Every cell whose
 * variable lies in [all_lo, all_hi] is kept (Ok and z > 0), none in
 * [none_lo, none_hi]; on = 0: no certificate (every segment is counted cell
 * by cell).  Host only. */
ACM_API int acm_sample_points_certificate(const acm_camera *cam, double *out);
/* (r05) RadTan only: the host-certified disk of acm_unproject's fast Newton
 * loop (csrc/acm.hip radtan_newton_disk).  out = [S, fast]: for every (x, y)
 * with x^2 + y^2 <= S the distortion Jacobian has |det| >= 1/16 and
 * |j00| + |j11| + 2 |j01| <= 64, so the loop tests only s <= S per step
 * (S = 0: no disk, the per-step tests); fast = 1 when the certified fast
 * loop runs at all (its distortion bound holds).  Host only; [0, 0] for the
 * other models. */
ACM_API int acm_unproject_certificate(const acm_camera *cam, double *out);
/* (r04) KB only: how acm_sample_points forms the rays of cells inside the
 * certified kept interval.  out = [mode, M, ef, fit_err, all_lo, all_hi]:
 * mode 0 = the reference-iterate path for every cell, 1 / 2 = the root by
 * the fitted initial guess + 1 / 2 Newton steps, 3 = the ray polynomials;
 * M = the Newton error constant, ef = the bound on the distance between the
 * reference's final iterate and the root the certified rays use (modes 1-3
 * require ef <= 1e-11), fit_err = a bound on the ray polynomials' error
 * over the whole certified interval, incl. the device's evaluation rounding
 * (r05: Taylor remainders on 256 pieces, csrc/acm.hip kb_ray_poly_bound;
 * r04 sampled it on 16385 points; mode 3 requires <= 1e-13).  Zeros for
 * other models.  Host only. */
ACM_API int acm_sample_points_ray_fit(const acm_camera *cam, double *out);
/* (r05) KB only: the fitted polynomials themselves, for independent checks
 * of the bounds.  out = 2 * ACM_RAY_POLY_N + ACM_RAY_GUESS_N + 1 doubles:
 * [C_0 .. C_16 | S_0 .. S_16] (cos(theta*) and sin(theta*) / ru in powers of
 * r2; what acm_sample_points evaluates when ray_fit's mode is 3), [g_0 ..
 * g_8] (theta* / ru in powers of r2, the initial guess of modes 1 / 2) and
 * the bound on |ru g(r2) - theta*| over the certified interval.  Zeros when
 * no fit was made.  Host only. */
#define ACM_RAY_POLY_N 17
#define ACM_RAY_GUESS_N 9
ACM_API int acm_sample_points_ray_poly(const acm_camera *cam, double *out);

/* acm_sample_points_range with per-call options: flags = 0 or
 * ACM_REFERENCE_NEWTON.  (acm_sample_points / _range = flags 0.) */
ACM_API int acm_sample_points_ex(const acm_camera *cam, size_t n_requested,
                                 size_t cell_begin, size_t cell_end, int flags,
                                 double *points_2d_out, double *points_3d_out,
                                 uint64_t *counts, void *workspace,
                                 size_t workspace_bytes, void *stream);

/* (r06) acm_sample_points_ex also writing each kept point's grid cell
 * c = i * num_cells_x + j (cells_out: device uint32, cap entries; the
 * grid: acm_sample_points_grid of cam's resolution) -- the cell form of
 * the correspondences for acm_lm_optimize_cells.  Grids of more than
 * 2^32 - 1 cells: ACM_ERR_INVALID_ARGUMENT. */
ACM_API int acm_sample_points_cells(const acm_camera *cam, size_t n_requested,
                                    size_t cell_begin, size_t cell_end, int flags,
                                    double *points_2d_out, double *points_3d_out,
                                    uint32_t *cells_out, uint64_t *counts, void *workspace,
                                    size_t workspace_bytes, void *stream);

/* util::undistort_image (src/util/undistort.rs:14-105).  image/output:
 * device RGB8 row-major, cam->width x cam->height (the reference requires
 * the image to match the model resolution).  target_intrinsics: host
 * [fx fy cx cy] or NULL for the camera's own (:30).  Pixels whose ray fails
 * to project or whose sample falls outside the image are written 0. */
enum { ACM_INTERP_NEAREST = 0, ACM_INTERP_BILINEAR = 1 };
ACM_API int acm_undistort_image(const acm_camera *cam, const double *target_intrinsics,
                                int interpolation, const uint8_t *image,
                                uint8_t *output, void *stream);

/* Device-memory helpers so a host without HIP bindings (e.g. the Rust crate
 * through `extern "C"`) can own device buffers: thin wrappers over
 * hipMalloc / hipFree / hipMemcpyAsync / hipStreamSynchronize / hipSetDevice. */
ACM_API int acm_set_device(int device);
ACM_API int acm_device_malloc(void **ptr, size_t bytes);
ACM_API int acm_device_free(void *ptr);
ACM_API int acm_memcpy_htod(void *dst_device, const void *src_host, size_t bytes, void *stream);
ACM_API int acm_memcpy_dtoh(void *dst_host, const void *src_device, size_t bytes, void *stream);
ACM_API int acm_stream_synchronize(void *stream);

/* Process-wide kernel tuning knobs: performance only.  Every knob selects
 * among kernels that return the same results -- bit for bit, except that
 * ACM_TUNE_NE_WAVES / ACM_TUNE_NE_UNROLL / ACM_TUNE_FOV_UNROLL change the
 * summation order of the normal-equations / grid sums (deterministic for a
 * fixed setting, <= ~1e-15 relative apart).  Numerics are never a knob: they
 * are chosen per call (ACM_EXACT_MATH, ACM_REFERENCE_NEWTON).
 * ACM_TUNE_PROJECT_VARIANT: bit flags of acm_project's
 * direct kernel, 1 = non-temporal stores, 2 = persistent grid-stride launch,
 * 4 = non-temporal loads; -1 (default) = auto (non-temporal stores when the
 * outputs exceed 64 MiB; non-temporal loads only if ACM_TUNE_NT_LOADS = 1).  ACM_TUNE_RESIDUAL_NT: non-temporal stores in
 * acm_residual_jacobian (-1 auto, 0 off = default, 1 on).  ACM_TUNE_NE_WAVES:
 * minimum waves per SIMD the normal-equations kernel is compiled for
 * (0 = per-model default, 1, 3, 4).  ACM_TUNE_FOV_UNROLL: the FOV grid search's kernel
 * (-1 = auto (r03) = the point-lane form: lanes own points, every wave
 * walks the grid, sums by wave butterfly -- another summation order, counts
 * identical, sums within ~1e-15; 0 = per-point 64-B records in LDS, each
 * read whole one point ahead (the r03 record form, -1 until r03's point-lane
 * form); 1 / 2 / 4 = the round-2 LDS kernel with 1 / 2 / 4 points per lane
 * step).  acm_fov_grid_workspace_size grew by 2 x 290 doubles (r03).  ACM_TUNE_NE_UNROLL: points per lane step
 * of the normal-equations kernel (0 = per-model default, 1, 2; 3, 4, 5 = one
 * point per step with its loads issued 2, 3, 4 steps ahead; 4 and 5 are
 * Kannala-Brandt only, other models take 3).
 * ACM_TUNE_ALIGN_J: kernel of +Jacobian launches of acm_project /
 * acm_residual_jacobian: -1 = auto (default) = line-aligned store windows
 * through LDS, 0 = one point per lane with direct stores, 1 = aligned.
 * ACM_TUNE_NT_LOADS: non-temporal loads of the point / observation streams
 * in the normal-equations, reprojection-statistics and median kernels
 * (-1 = auto = on, 0, 1; 1 also turns them on in the direct project kernel).  ACM_TUNE_NT_LOADS_UNPROJECT: the same
 * for acm_unproject's pixel stream (-1 = auto = off, 0, 1).
 * ACM_TUNE_LM_HOST_RESULT: acm_lm_optimize without an all-reduce callback
 * has the normal-equations kernel write its results straight into pinned
 * host memory rather than device memory plus a copy: 0 = off, 1 = on with a
 * stream synchronisation, 2 = on with the host spinning on a completion
 * word the kernel publishes, 3 = as 2 with each evaluation queued ahead of
 * the host's decision and released by a host-written doorbell (AoS points,
 * default NE knobs; else 2); -1 = auto = 2.  Every mode takes the same
 * iterates.
 * ACM_TUNE_SAMPLE_FUSED: acm_sample_points' kernels.  -1 = auto (r03) = the
 * speculative segment path (4, below) for RadTan, else the segment two-pass path (certified per-segment counts, offsets by a scan,
 * then a write pass with known offsets); 0 = the round-1 two-pass count /
 * scan / recompute-and-write path (tiles of 16 x 256 cells); 1 / 2 / 3 = the
 * single pass with a decoupled look-back, tiles of 2 / 4 / 8 x 256 cells
 * (round 1 mapped 1 / 2 / 3 to 4 / 8 / 16 x 256; changed in round 2); 4 =
 * speculative segments (r03; auto for RadTan): one pass writes every
 * segment of 64 cells in place as if nothing before it was dropped, a scan
 * gives the true offsets and a repair pass rewrites only the segments after
 * the first drop.
 * Outputs are identical for every value.
 * ACM_TUNE_SAMPLE_CERT: the segment path's host-certified keep regions
 * (-1 = auto = on; 0 = every segment counted cell by cell).  Same outputs.
 * ACM_TUNE_SAMPLE_WRITE: the segment path's write pass, segments per wave
 * and their order (-1 = auto = 16 interleaved across the workgroup's four
 * waves, 4 for KB / UCM / EUCM / FOV; 1 = 64 contiguous, 2 = 16
 * interleaved, 3 = 4 interleaved, 4 = 16 contiguous, 5 = 16 interleaved
 * with non-temporal stores).  Same outputs.
 * ACM_TUNE_UNPROJECT_RCP: unprojections (acm_unproject, acm_sample_points*)
 * divide by fx, fy through the host's correctly rounded 1/fx, 1/fy and one
 * FMA correction, bit-identical to the division (-1 = auto = on, 0 = plain
 * IEEE divisions, 1 = on).
 * ACM_TUNE_SAMPLE_PATIENCE: polls the single-pass sample_points look-back
 * spends on a predecessor tile that has not published its count before the
 * waiting wave counts that tile's cells itself (-1 = auto = 512; 0 = at once,
 * which exercises that path; outputs are identical for every value).
 * ACM_TUNE_NEWTON_FAST (12): removed in round 3 (it changed RadTan's rays by a
 * few ulp process-wide); acm_set_tuning returns ACM_ERR_NOT_SUPPORTED.  Use
 * the per-call ACM_REFERENCE_NEWTON.
 * ACM_TUNE_UNPROJECT_PPT: acm_unproject's pixels per lane and AoS ray
 * stores (-1 = auto = 2 pixels per lane; for Pinhole, DS, UCM and EUCM each
 * wave's 64 AoS rays staged in LDS and written as 16-B pieces when rays is
 * 16-B aligned; 1 / 2 = pixels per lane with three 8-B stores per ray; 3 =
 * 1 pixel per lane, staged when rays is 16-B aligned).
 * Outputs are identical for every value.
 * ACM_TUNE_LM_DEVICE (16): removed in round 5.  Round 4 added it to run the
 * LM state machine on the device behind each evaluation; that loop measured
 * slower than the host loop (1.41 vs 1.33 ms at config 3) and never was the
 * default.  acm_set_tuning returns ACM_ERR_NOT_SUPPORTED; acm_lm_optimize
 * always runs the host loop.
 * ACM_TUNE_ROUND_TRIP (r05): acm_project_unproject's pixels per lane and
 * AoS ray stores: -1 = auto (the per-model default); else PPT (1, 2 or 4)
 * + 8 x stores (0 = the model's default, 1 = each wave's 64 rays staged in
 * LDS and written as 16-B pieces, 2 = three 8-B stores per ray).  Same
 * outputs for every value.
 * Defaults (the value acm_set_tuning returns as "previous" in a fresh
 * process; tests/test_capi.py checks every one): PROJECT_VARIANT -1,
 * RESIDUAL_NT 0, NE_WAVES 0, FOV_UNROLL -1, NE_UNROLL 0, ALIGN_J -1,
 * NT_LOADS -1, NT_LOADS_UNPROJECT -1, LM_HOST_RESULT -1, SAMPLE_FUSED -1,
 * UNPROJECT_RCP -1, SAMPLE_PATIENCE -1, UNPROJECT_PPT -1, SAMPLE_CERT -1,
 * SAMPLE_WRITE -1, ROUND_TRIP -1.
 * Every knob is an atomic: acm_set_tuning may race with any other call.
 * Returns the previous value or an error. */
enum {
    ACM_TUNE_PROJECT_VARIANT = 0,
    ACM_TUNE_RESIDUAL_NT = 1,
    ACM_TUNE_NE_WAVES = 2,
    ACM_TUNE_FOV_UNROLL = 3,
    ACM_TUNE_NE_UNROLL = 4,
    ACM_TUNE_ALIGN_J = 5,
    ACM_TUNE_NT_LOADS = 6,
    ACM_TUNE_NT_LOADS_UNPROJECT = 7,
    ACM_TUNE_LM_HOST_RESULT = 8,
    ACM_TUNE_SAMPLE_FUSED = 9,
    ACM_TUNE_UNPROJECT_RCP = 10,
    ACM_TUNE_SAMPLE_PATIENCE = 11,
    ACM_TUNE_NEWTON_FAST = 12,
    ACM_TUNE_UNPROJECT_PPT = 13,
    ACM_TUNE_SAMPLE_CERT = 14,
    ACM_TUNE_SAMPLE_WRITE = 15,
    ACM_TUNE_LM_DEVICE = 16,
    ACM_TUNE_ROUND_TRIP = 17
};
ACM_API int acm_set_tuning(int key, int value);

/* Diagnostics: last HIP error code / message of the calling thread. */
ACM_API int acm_last_hip_error(void);
ACM_API const char *acm_last_error(void);
ACM_API const char *acm_version(void);

#ifdef __cplusplus
}
#endif
#endif /* ACM_H */
