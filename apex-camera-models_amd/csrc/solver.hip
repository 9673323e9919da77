// solver.hip -- host-side drivers on top of the kernels: linear_estimation
// (TSQR factor from the GPU, k x k SVD solve on the host) and the
// Levenberg-Marquardt loop of the model conversion (normal equations from
// the fused GPU kernel, optional cross-rank all-reduce callback, P x P
// Cholesky on the host).
//
// Reference: bin/camera_converter.rs:355-1163 (convert_to_*: linear
// estimation then apex-solver LM with bounds and
// max_iterations=100, cost_tolerance=1e-6, parameter_tolerance=1e-8,
// gradient_tolerance=1e-6).  apex-solver 0.1.5's LM source is absent, so the
// LM here is a standard bounded Levenberg-Marquardt (Madsen/Nielsen damping
// update, Marquardt diagonal scaling, projection onto the bounds), with the
// reference's configuration; DESIGN.md documents the (unpinned) choice.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <string>
#include <vector>

#include "acm.h"
#include "lm_core.hpp"
#include "lm_doorbell.hpp"

namespace acm {
int set_error(int code, const std::string& msg);  // acm.hip (one last-error slot)
int lm_host_result();                              // acm.hip, ACM_TUNE_LM_HOST_RESULT
int normal_equations_impl(const acm_camera* cam, size_t n, const double* points_3d, int layout,
                          const double* points_2d_obs, int invalid_policy, double* result,
                          void* workspace, size_t workspace_bytes, void* stream,
                          unsigned long long* flag, unsigned long long seq,
                          unsigned int* ticket, const uint32_t* cells,
                          const acm_cell_grid* grid, const LmDoorbell* db);
bool ne_dev_ok(int layout);
int check_cell_grid(const acm_cell_grid* grid);
int linear_system_qr_error(const acm_camera* cam, size_t n, const double* points_3d, int layout,
                           const double* points_2d, double* r_factor, int* error_flag,
                           double* result, void* ws_qr, void* ws_err, void* stream,
                           double* host_out, hipEvent_t ready, int* hist_nb = nullptr,
                           const uint32_t* cells = nullptr, const acm_cell_grid* grid = nullptr);
}

namespace {

int sfail(int code, const std::string& m) { return acm::set_error(code, m); }

int hip_ok(hipError_t e) { return e == hipSuccess ? ACM_SUCCESS : ACM_ERR_HIP; }

// One-sided Jacobi SVD of a k x k matrix A (row-major), then
// x = V diag(1/s) U^T b with singular values <= eps treated as zero --
// the semantics of nalgebra's SVD::solve(b, eps).
void svd_solve(int k, const double* A, const double* b, double eps, double* x) {
    std::vector<double> W(A, A + k * k), V(k * k, 0.0);
    for (int i = 0; i < k; ++i) V[i * k + i] = 1.0;
    for (int sweep = 0; sweep < 60; ++sweep) {
        double off = 0.0;
        for (int p = 0; p < k; ++p)
            for (int q = p + 1; q < k; ++q) {
                double al = 0, be = 0, ga = 0;
                for (int i = 0; i < k; ++i) {
                    al += W[i * k + p] * W[i * k + p];
                    be += W[i * k + q] * W[i * k + q];
                    ga += W[i * k + p] * W[i * k + q];
                }
                if (ga == 0.0) continue;
                off = std::fmax(off, std::fabs(ga) / std::sqrt(al * be));
                const double zeta = (be - al) / (2.0 * ga);
                const double t = (zeta >= 0 ? 1.0 : -1.0) / (std::fabs(zeta) + std::sqrt(1.0 + zeta * zeta));
                const double c = 1.0 / std::sqrt(1.0 + t * t), s = c * t;
                for (int i = 0; i < k; ++i) {
                    const double wp = W[i * k + p], wq = W[i * k + q];
                    W[i * k + p] = c * wp - s * wq;
                    W[i * k + q] = s * wp + c * wq;
                    const double vp = V[i * k + p], vq = V[i * k + q];
                    V[i * k + p] = c * vp - s * vq;
                    V[i * k + q] = s * vp + c * vq;
                }
            }
        if (off < 1e-15) break;
    }
    for (int i = 0; i < k; ++i) x[i] = 0.0;
    for (int j = 0; j < k; ++j) {
        double sj = 0.0;
        for (int i = 0; i < k; ++i) sj += W[i * k + j] * W[i * k + j];
        sj = std::sqrt(sj);
        if (!(sj > eps)) continue;
        double utb = 0.0;  // u_j = W[:, j] / s_j
        for (int i = 0; i < k; ++i) utb += W[i * k + j] * b[i];
        const double coef = utb / (sj * sj);
        for (int i = 0; i < k; ++i) x[i] += V[i * k + j] * coef;
    }
}

int validate(const acm_camera* cam) {
    const int v = acm_validate_params(cam);
    if (v == ACM_VALID) return ACM_SUCCESS;
    return sfail(ACM_ERR_INVALID_PARAMS, "validate_params failed after linear estimation");
}

int fov_linear_estimation(acm_camera* cam, size_t n, const double* points_3d, int layout,
                          const double* points_2d, void* workspace, size_t workspace_bytes,
                          void* stream) {
    if (n < 2)  // fov.rs:166-171
        return sfail(ACM_ERR_INVALID_PARAMS,
                     "Need at least 2 point correspondences for linear estimation");
    const size_t g = acm_fov_grid_workspace_size(n);
    if (!workspace || workspace_bytes < g + 2 * ACM_FOV_GRID_SIZE * sizeof(double))
        return sfail(ACM_ERR_WORKSPACE_TOO_SMALL, "linear-estimation workspace too small");
    double* d_sums = (double*)((char*)workspace + g);
    int rc = acm_fov_grid_errors(cam, n, points_3d, layout, points_2d, d_sums, workspace, g,
                                 stream);
    if (rc) return rc;
    double sums[2 * ACM_FOV_GRID_SIZE];
    hipStream_t s = (hipStream_t)stream;
    if (hip_ok(hipMemcpyAsync(sums, d_sums, sizeof(sums), hipMemcpyDeviceToHost, s)) ||
        hip_ok(hipStreamSynchronize(s)))
        return sfail(ACM_ERR_HIP, "FOV grid search: device copy failed");
    return acm_fov_grid_select(cam, sums);
}

}  // namespace

extern "C" {

// fov.rs:176-249: first grid value with the strictly smallest mean error
// (best starts at w = 1.0, +inf), then the clamp and validate_params.
ACM_API int acm_fov_grid_select(acm_camera* cam, const double* grid_sums_host) {
    if (!cam || !grid_sums_host) return sfail(ACM_ERR_INVALID_ARGUMENT, "NULL argument");
    if (cam->model != ACM_FOV) return sfail(ACM_ERR_NOT_SUPPORTED, "grid search is FOV-only");
    double best_w = 1.0, best_error = INFINITY;
    for (int i = 0; i < ACM_FOV_GRID_SIZE; ++i) {
        const double cnt = grid_sums_host[ACM_FOV_GRID_SIZE + i];
        if (cnt > 0.0) {
            const double avg = grid_sums_host[i] / cnt;
            if (avg < best_error) {
                best_error = avg;
                best_w = (double)(i + 10) / 100.0;
            }
        }
    }
    if (best_w <= 2.220446049250313e-16) best_w = 0.01;  // :236-242
    else if (best_w > 3.0) best_w = 3.0;
    cam->params[4] = best_w;
    return validate(cam);
}

ACM_API size_t acm_linear_estimation_workspace_size(int model, size_t n) {
    if (model == ACM_FOV)
        return acm_fov_grid_workspace_size(n) + 2 * ACM_FOV_GRID_SIZE * sizeof(double);
    const size_t qr = acm_linear_system_qr_workspace_size(model, n);
    if (!qr) return 0;
    return qr + 32 * sizeof(double);
}

// linear_estimation (kannala_brandt.rs:164-272, double_sphere.rs:225-290,
// ucm.rs:200-258, eucm.rs:216-288, rad_tan.rs:153-234): updates cam->params.
static int count_check(int model, size_t n) {
    if (model == ACM_KANNALA_BRANDT && n < 4)  // kannala_brandt.rs:174-178
        return sfail(ACM_ERR_INVALID_PARAMS, "Not enough points for linear estimation (need at least 4)");
    if (model == ACM_RADTAN && n < 3)  // rad_tan.rs:152-156
        return sfail(ACM_ERR_INVALID_PARAMS, "Need at least 3 points for RadTan linear estimation");
    if (model == ACM_EUCM && n < 1)  // eucm.rs:228-232
        return sfail(ACM_ERR_INVALID_PARAMS, "Need at least 1 point for EUCM linear estimation");
    return ACM_SUCCESS;
}

// Givens fold of one packed upper-triangular (M x M) factor into another:
// the host twin of tri_merge in acm.hip.  qr([R_a; R_b]) = R of the
// stacked rows of both shards, so a multi-GPU caller merges the per-rank
// factors in rank order and every rank gets the same R.
ACM_API int acm_linear_system_r_merge(int model, double* r_inout, const double* r_other) {
    const int k = acm_linear_system_columns(model);
    if (k < 0) return sfail(ACM_ERR_NOT_SUPPORTED, "model has no linear_estimation");
    if (!r_inout || !r_other) return sfail(ACM_ERR_INVALID_ARGUMENT, "NULL factor");
    const int M = k + 1;
    auto at = [M](int r, int c) { return r * M - r * (r - 1) / 2 + (c - r); };
    for (int r0 = 0; r0 < M; ++r0) {
        double row[8];
        for (int c = 0; c < M; ++c) row[c] = c < r0 ? 0.0 : r_other[at(r0, c)];
        for (int j = 0; j < M; ++j) {
            const double b = row[j];
            if (b == 0.0) continue;
            const double a = r_inout[at(j, j)];
            const double r = std::sqrt(a * a + b * b);
            const double c = a / r, sn = b / r;
            r_inout[at(j, j)] = r;
            for (int l = j + 1; l < M; ++l) {
                const double Rl = r_inout[at(j, l)], rl = row[l];
                r_inout[at(j, l)] = c * Rl + sn * rl;
                row[l] = c * rl - sn * Rl;
            }
        }
    }
    return ACM_SUCCESS;
}

// The host half of linear_estimation: solve R_A x = z from the (k+1) x (k+1)
// factor of [A | b] with nalgebra's SVD::solve(eps) semantics, apply the
// model's clamps and validation (n_total: the global point count, for the
// reference's minimum-count checks).
ACM_API int acm_linear_estimation_solve(acm_camera* cam, size_t n_total,
                                        const double* r_factor_host, int error_flag) {
    if (!cam || !r_factor_host) return sfail(ACM_ERR_INVALID_ARGUMENT, "NULL argument");
    const int k = acm_linear_system_columns(cam->model);
    if (k < 0) return sfail(ACM_ERR_NOT_SUPPORTED, "model has no linear_estimation");
    int rc = count_check(cam->model, n_total);
    if (rc) return rc;
    if (error_flag) return sfail(ACM_ERR_NUMERICAL, "fx * x_r is zero in linear estimation");
    const int M = k + 1;
    const double* R = r_factor_host;
    // R = [[R_A, z], [0, rho]] (packed upper triangle, row-major)
    double RA[16] = {0}, z[4] = {0}, x[4] = {0};
    auto at = [M](int r, int c) { return r * M - r * (r - 1) / 2 + (c - r); };
    for (int r = 0; r < k; ++r) {
        for (int c = r; c < k; ++c) RA[r * k + c] = R[at(r, c)];
        z[r] = R[at(r, k)];
    }
    const double eps = cam->model == ACM_KANNALA_BRANDT ? 2.220446049250313e-16 : 1e-10;
    svd_solve(k, RA, z, eps, x);
    double* p = cam->params;
    switch (cam->model) {
    case ACM_KANNALA_BRANDT:  // :268-270
        for (int i = 0; i < 4; ++i) p[4 + i] = x[i];
        return validate(cam);
    case ACM_DOUBLE_SPHERE:  // :269-287
        p[4] = x[0];
        p[5] = 0.0;
        if (p[4] <= 0.0) p[4] = 0.01;
        else if (p[4] > 1.0) p[4] = 1.0;
        return validate(cam);
    case ACM_UCM:  // ucm.rs:245-255
        p[4] = x[0];
        if (p[4] <= 0.0) p[4] = 0.01;
        return validate(cam);
    case ACM_EUCM:  // eucm.rs:234-285
        p[5] = 1.0;
        p[4] = x[0];
        if (p[4] <= 0.0) p[4] = 0.01;
        else if (p[4] > 2.0) p[4] = 2.0;
        return validate(cam);
    case ACM_RADTAN:  // rad_tan.rs:209-214
        p[4] = x[0];
        p[5] = x[1];
        p[6] = 0.0;
        p[7] = 0.0;
        p[8] = x[2];
        return ACM_SUCCESS;
    default: return sfail(ACM_ERR_NOT_SUPPORTED, "unsupported model");
    }
}

ACM_API int acm_linear_estimation(acm_camera* cam, size_t n, const double* points_3d, int layout,
                                  const double* points_2d, void* workspace,
                                  size_t workspace_bytes, void* stream) {
    if (!cam) return sfail(ACM_ERR_INVALID_ARGUMENT, "camera is NULL");
    if (cam->model == ACM_FOV) return fov_linear_estimation(cam, n, points_3d, layout, points_2d,
                                                            workspace, workspace_bytes, stream);
    const int k = acm_linear_system_columns(cam->model);
    if (k < 0) return sfail(ACM_ERR_NOT_SUPPORTED, "model has no linear_estimation");
    int rc = count_check(cam->model, n);
    if (rc) return rc;
    const size_t need = acm_linear_estimation_workspace_size(cam->model, n);
    if (!workspace || workspace_bytes < need)
        return sfail(ACM_ERR_WORKSPACE_TOO_SMALL, "linear-estimation workspace too small");
    const int M = k + 1, S = M * (M + 1) / 2;
    const size_t qr = acm_linear_system_qr_workspace_size(cam->model, n);
    double* d_r = (double*)((char*)workspace + qr);
    int* d_err = (int*)(d_r + 16);
    rc = acm_linear_system_qr(cam, n, points_3d, layout, points_2d, d_r, d_err, workspace, qr,
                              stream);
    if (rc) return rc;
    // R (S <= 15 doubles) and the flag (at double 16) in one copy
    double R[17];
    hipStream_t s = (hipStream_t)stream;
    (void)S;
    if (hip_ok(hipMemcpyAsync(R, d_r, 17 * sizeof(double), hipMemcpyDeviceToHost, s)) ||
        hip_ok(hipStreamSynchronize(s)))
        return sfail(ACM_ERR_HIP, "linear estimation: device copy failed");
    int err = 0;
    std::memcpy(&err, &R[16], sizeof(int));
    return acm_linear_estimation_solve(cam, n, R, err);
}

// convert_to_*'s initial_error + linear_estimation (camera_converter.rs:
// 371-375, :507-511, ...) in one pass over the correspondences.  Workspace:
// [TSQR partials | R + flag (32 f64) | acm_reprojection_error's workspace].
static size_t lin_err_qr_bytes(int model, size_t n) {
    return (acm_linear_system_qr_workspace_size(model, n) + 255) / 256 * 256;
}

ACM_API size_t acm_linear_estimation_with_error_workspace_size(int model, size_t n) {
    const size_t le = acm_linear_estimation_workspace_size(model, n);
    if (!le) return 0;
    const size_t err = acm_reprojection_error_workspace_size(n);
    if (model == ACM_FOV) return std::max(le, err);
    return lin_err_qr_bytes(model, n) + 32 * sizeof(double) + err;
}

// One pinned host buffer (R + flag + the 8 statistics) and one event per host
// thread for the opening's early hand-off, freed when the thread exits.  The
// event is made on the device of the caller's stream (which need not be the
// current one: ADVICE r05), switching to it for the creation only; a stream
// on another device gets a new event.
namespace {
struct OpeningHost {
    double* p = nullptr;
    hipEvent_t ev = nullptr;
    int ev_dev = -1;
    bool ok(hipStream_t stream) {
        if (!p) {
            void* q = nullptr;
            if (hipHostMalloc(&q, 32 * sizeof(double), hipHostMallocPortable) != hipSuccess) {
                (void)hipGetLastError();
                return false;
            }
            p = (double*)q;
        }
        int cur = -1, dev = -1;
        if (hipGetDevice(&cur) != hipSuccess) {
            (void)hipGetLastError();
            return false;
        }
        dev = cur;
        if (stream) {
            hipDevice_t d = 0;
            if (hipStreamGetDevice(stream, &d) != hipSuccess) {
                (void)hipGetLastError();
                return false;
            }
            dev = (int)d;
        }
        if (ev && ev_dev != dev) {
            if (hipEventDestroy(ev) != hipSuccess) (void)hipGetLastError();
            ev = nullptr;
        }
        if (!ev) {
            if (dev != cur && hipSetDevice(dev) != hipSuccess) {
                (void)hipGetLastError();
                return false;
            }
            const bool made = hipEventCreateWithFlags(&ev, hipEventDisableTiming) == hipSuccess;
            if (!made) {
                (void)hipGetLastError();
                ev = nullptr;
            }
            if (dev != cur && hipSetDevice(cur) != hipSuccess) (void)hipGetLastError();
            if (!made) return false;
            ev_dev = dev;
        }
        return true;
    }
    ~OpeningHost() {
        if (ev && hipEventDestroy(ev) != hipSuccess) (void)hipGetLastError();
        if (p && hipHostFree(p) != hipSuccess) (void)hipGetLastError();
    }
};
}  // namespace

static int linear_estimation_with_error_async(acm_camera* cam, size_t n, const double* points_3d,
                                              int layout, const double* points_2d,
                                              const uint32_t* cells, const acm_cell_grid* grid,
                                              double* initial_error, double* initial_error_host,
                                              void* workspace, size_t workspace_bytes,
                                              void* stream) {
    if (!cam) return sfail(ACM_ERR_INVALID_ARGUMENT, "camera is NULL");
    if (!initial_error) return sfail(ACM_ERR_INVALID_ARGUMENT, "NULL buffer");
    const size_t need = acm_linear_estimation_with_error_workspace_size(cam->model, n);
    if (!need) return sfail(ACM_ERR_NOT_SUPPORTED, "model has no linear_estimation");
    if (!workspace || workspace_bytes < need)
        return sfail(ACM_ERR_WORKSPACE_TOO_SMALL, "linear-estimation workspace too small");
    hipStream_t s = (hipStream_t)stream;
    const int k = acm_linear_system_columns(cam->model);
    // the reference computes initial_error first: it is written whatever the
    // estimation then does (FOV, or too few points: the two calls in order)
    if (k < 0 || count_check(cam->model, n) != ACM_SUCCESS) {
        int rc = acm_reprojection_error(cam, n, points_3d, layout, points_2d, initial_error,
                                        nullptr, workspace,
                                        acm_reprojection_error_workspace_size(n), stream);
        if (rc) return rc;
        if (initial_error_host &&
            (hip_ok(hipMemcpyAsync(initial_error_host, initial_error, 8 * sizeof(double),
                                   hipMemcpyDeviceToHost, s)) ||
             hip_ok(hipStreamSynchronize(s))))
            return sfail(ACM_ERR_HIP, "linear estimation: device copy failed");
        return acm_linear_estimation(cam, n, points_3d, layout, points_2d, workspace,
                                     workspace_bytes, stream);
    }
    static thread_local OpeningHost host;
    if (!host.ok(s)) return sfail(ACM_ERR_HIP, "linear estimation: pinned buffer or event");
    const size_t qr = lin_err_qr_bytes(cam->model, n);
    double* d_r = (double*)((char*)workspace + qr);
    int* d_err = (int*)(d_r + 16);
    void* ws_err = (char*)workspace + qr + 32 * sizeof(double);
    // R (<= 15 doubles), the flag (at double 16) and the statistics reach the
    // host before the median runs (r05): the solve below overlaps it, and the
    // median's result lands in initial_error[8] in stream order
    int rc = acm::linear_system_qr_error(cam, n, points_3d, layout, points_2d, d_r, d_err,
                                         initial_error, workspace, ws_err, stream, host.p,
                                         host.ev, nullptr, cells, grid);
    if (rc) return rc;
    if (hip_ok(hipEventSynchronize(host.ev)))
        return sfail(ACM_ERR_HIP, "linear estimation: device copy failed");
    double R[17];
    std::memcpy(R, host.p, sizeof(R));
    if (initial_error_host) std::memcpy(initial_error_host, host.p + 17, 8 * sizeof(double));
    int err = 0;
    std::memcpy(&err, &R[16], sizeof(int));
    return acm_linear_estimation_solve(cam, n, R, err);
}

ACM_API int acm_linear_estimation_with_error_async(acm_camera* cam, size_t n,
                                                   const double* points_3d, int layout,
                                                   const double* points_2d, double* initial_error,
                                                   double* initial_error_host, void* workspace,
                                                   size_t workspace_bytes, void* stream) {
    return linear_estimation_with_error_async(cam, n, points_3d, layout, points_2d, nullptr,
                                              nullptr, initial_error, initial_error_host,
                                              workspace, workspace_bytes, stream);
}

// (r06) the same with the fused pass reading the cell form of the
// observations (acm_cell_grid); points_2d is still required, for the FOV
// grid search and the too-few-points path, which read the pixels
ACM_API int acm_linear_estimation_with_error_cells_async(
    acm_camera* cam, size_t n, const double* points_3d, int layout, const double* points_2d,
    const uint32_t* cells, const acm_cell_grid* grid, double* initial_error,
    double* initial_error_host, void* workspace, size_t workspace_bytes, void* stream) {
    int rc = acm::check_cell_grid(grid);
    if (rc) return rc;
    if (n && (!cells || !points_2d)) return sfail(ACM_ERR_INVALID_ARGUMENT, "NULL buffer");
    static const uint32_t none = 0;
    return linear_estimation_with_error_async(cam, n, points_3d, layout, points_2d,
                                              cells ? cells : &none, grid, initial_error,
                                              initial_error_host, workspace, workspace_bytes,
                                              stream);
}

ACM_API int acm_linear_estimation_with_error(acm_camera* cam, size_t n, const double* points_3d,
                                             int layout, const double* points_2d,
                                             double* initial_error, void* workspace,
                                             size_t workspace_bytes, void* stream) {
    const int rc = acm_linear_estimation_with_error_async(cam, n, points_3d, layout, points_2d,
                                                          initial_error, nullptr, workspace,
                                                          workspace_bytes, stream);
    // as before r05: everything, the median included, is done on return
    if (hip_ok(hipStreamSynchronize((hipStream_t)stream)))
        return sfail(ACM_ERR_HIP, "linear estimation: stream synchronize failed");
    return rc;
}

// (r06) after the all-reduce: the R summed results into the pinned buffer,
// then the completion word with a system-scope release (one lane: R <= 92)
__global__ void k_lm_copy_publish(const double* __restrict__ src, double* __restrict__ dst,
                                  int count, unsigned long long* __restrict__ flag,
                                  unsigned long long seq) {
    if (threadIdx.x == 0) {
        for (int t = 0; t < count; ++t) dst[t] = src[t];
        __threadfence_system();
        __hip_atomic_store(flag, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

ACM_API void acm_lm_default_config(acm_lm_config* cfg) {
    if (!cfg) return;
    std::memset(cfg, 0, sizeof(*cfg));
    cfg->max_iterations = 100;  // camera_converter.rs:410-415
    cfg->cost_tolerance = 1e-6;
    cfg->parameter_tolerance = 1e-8;
    cfg->gradient_tolerance = 1e-6;
    cfg->initial_damping = 1e-4;
    cfg->invalid_policy = ACM_INVALID_SKIP;
    cfg->has_bounds = 0;
    for (int i = 0; i < ACM_MAX_PARAMS; ++i) {
        cfg->lower[i] = -INFINITY;
        cfg->upper[i] = INFINITY;
    }
}

// LM workspace: the normal equations' partials | the results (R doubles + 8
// spare, one of them the finish kernel's ticket) | (r06) the pre-queued
// evaluation's camera (12 doubles).
constexpr int kLmDevCamDoubles = (int)((sizeof(acm_camera) + 7) / 8);
ACM_API size_t acm_lm_workspace_size(int model, size_t n) {
    const int P = acm_num_params(model);
    if (P < 0) return 0;
    return acm_normal_equations_workspace_size(model, n) +
           (size_t)(P * P + P + 2 + 8 + kLmDevCamDoubles) * 8;
}

static void lm_summarize(const acm::lm::State& st, acm_camera* cam, int P,
                         acm_lm_summary* summary) {
    for (int i = 0; i < P; ++i) cam->params[i] = st.x[i];
    acm_lm_summary sum;
    std::memset(&sum, 0, sizeof(sum));
    sum.iterations = st.it;
    sum.termination = st.term;
    sum.evaluations = st.evals;
    sum.initial_cost = st.initial_cost;
    sum.final_cost = st.F;
    sum.n_valid = st.nv;
    if (summary) *summary = sum;
}

// (r06) The LM host loop with pre-queued evaluations (ACM_TUNE_LM_HOST_RESULT
// 3; lm_doorbell.hpp).  The same evaluations in the same order as the
// launch-per-evaluation loop, from the same kernel body: the same iterates.
static int lm_doorbell_loop(acm_camera* cam, size_t n, const double* points_3d, int layout,
                            const double* points_2d, const uint32_t* cells,
                            const acm_cell_grid* grid, const acm_lm_config* cfg,
                            acm::lm::State& st, int P, double* pinned, unsigned long long& seq,
                            double* d_res, void* workspace, size_t ne_ws,
                            acm_lm_summary* summary, hipStream_t s) {
    using acm::kLmCancel;
    using acm::LmMailbox;
    struct Mailbox {
        LmMailbox* p = nullptr;
        ~Mailbox() {
            if (p && hipHostFree(p) != hipSuccess) (void)hipGetLastError();
        }
    };
    static thread_local Mailbox tl_mb;
    if (!tl_mb.p) {
        void* q = nullptr;
        if (hipHostMalloc(&q, 4096, hipHostMallocMapped | hipHostMallocPortable |
                                        hipHostMallocCoherent) != hipSuccess) {
            (void)hipGetLastError();
            return sfail(ACM_ERR_HIP, "LM: mailbox allocation failed");
        }
        tl_mb.p = (LmMailbox*)q;
        std::memset(q, 0, 4096);
    }
    LmMailbox* mb = tl_mb.p;
    int dev = 0, khz = 0;
    if (hip_ok(hipGetDevice(&dev)) ||
        hip_ok(hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev)) || khz <= 0)
        return sfail(ACM_ERR_HIP, "LM: wall clock rate unavailable");
    const int R = P * P + P + 2;
    auto* flag = reinterpret_cast<unsigned long long*>(pinned + 127);
    auto* ticket = reinterpret_cast<unsigned int*>(d_res + R);
    // the spare words after the results: [ticket | device flag | ... |
    // camera at +8]
    acm::LmDoorbell db;
    db.mb = mb;
    db.flag = reinterpret_cast<unsigned long long*>(d_res + R + 1);
    db.cam = reinterpret_cast<acm_camera*>(d_res + R + 8);
    // a doorbell not rung within 10 s ends its wait (the evaluation is then
    // reported as failed): the queued kernels always drain
    db.timeout = 10000ull * (unsigned long long)khz;
    if (hip_ok(hipMemsetAsync(d_res + R, 0, 2 * sizeof(double), s)))
        return sfail(ACM_ERR_HIP, "LM: ticket reset failed");
    auto* ack = &mb->ack;
    // queue evaluation `q`: the normal equations behind the doorbell, then
    // their epilogue (results into the pinned buffer, completion word = q)
    auto enqueue = [&](unsigned long long q) -> int {
        db.seq = q;
        return acm::normal_equations_impl(cam, n, points_3d, layout, points_2d,
                                          cfg->invalid_policy, pinned, workspace, ne_ws, s, flag,
                                          q, ticket, cells, grid, &db);
    };
    auto ring = [&](unsigned long long q, const double* x) {
        acm_camera c = *cam;
        for (int i = 0; i < P; ++i) c.params[i] = x[i];
        std::memcpy(&mb->cam, &c, sizeof(c));
        __atomic_store_n(&mb->seq, q, __ATOMIC_RELEASE);
    };
    // spin on evaluation q's completion word (as the mode-2 loop)
    auto wait = [&](unsigned long long q) -> int {
        for (unsigned spin = 1;; ++spin) {
            if (__atomic_load_n(flag, __ATOMIC_ACQUIRE) == q) break;
            if ((spin & 255) == 0) {
                const hipError_t e = hipStreamQuery(s);
                if (e == hipSuccess) {
                    if (__atomic_load_n(flag, __ATOMIC_ACQUIRE) == q) break;
                    return sfail(ACM_ERR_HIP, "LM: completion word not published");
                }
                if (e != hipErrorNotReady) return sfail(ACM_ERR_HIP, "LM: stream failed");
            }
            __builtin_ia32_pause();
        }
        return ACM_SUCCESS;
    };
    // a queued evaluation the loop no longer wants: cancel it and let the
    // queue drain before returning (its epilogue still publishes q)
    auto cancel = [&](unsigned long long q) {
        __atomic_store_n(&mb->seq, q | kLmCancel, __ATOMIC_RELEASE);
        (void)wait(q);
    };
    // on an error: cancel q (perhaps only partly queued) and drain the stream
    auto abandon = [&](unsigned long long q) {
        __atomic_store_n(&mb->seq, q | kLmCancel, __ATOMIC_RELEASE);
        if (hipStreamSynchronize(s) != hipSuccess) (void)hipGetLastError();
    };
    std::vector<double> res(R);
    unsigned long long cur = ++seq;
    int rc = enqueue(cur);
    if (rc) {
        abandon(cur);
        return rc;
    }
    ring(cur, st.xn);
    int r = acm::lm::NEED_EVAL;
    while (r == acm::lm::NEED_EVAL) {
        const unsigned long long next = ++seq;
        if ((rc = enqueue(next))) {
            (void)wait(cur);
            abandon(next);
            return rc;
        }
        if ((rc = wait(cur))) {
            abandon(next);
            return rc;
        }
        if (__atomic_load_n(ack, __ATOMIC_ACQUIRE) != cur) {
            cancel(next);
            return sfail(ACM_ERR_HIP, "LM: evaluation not served (doorbell timed out)");
        }
        std::memcpy(res.data(), pinned, R * sizeof(double));
        r = acm::lm::consume(st, *cfg, res.data(), P);
        if (r != acm::lm::NEED_EVAL) {
            cancel(next);
            break;
        }
        ring(next, st.xn);
        cur = next;
    }
    lm_summarize(st, cam, P, summary);
    return ACM_SUCCESS;
}

static int lm_optimize(acm_camera* cam, size_t n, const double* points_3d, int layout,
                       const double* points_2d, const uint32_t* cells, const acm_cell_grid* grid,
                       const acm_lm_config* cfg, acm_allreduce_fn allreduce, void* allreduce_ctx,
                       acm_lm_summary* summary, void* workspace, size_t workspace_bytes,
                       void* stream) {
    if (!cam || !cfg) return sfail(ACM_ERR_INVALID_ARGUMENT, "NULL argument");
    const int P = acm_num_params(cam->model);
    if (P < 0) return sfail(ACM_ERR_INVALID_MODEL, "unknown camera model id");
    const size_t need = acm_lm_workspace_size(cam->model, n);
    if (!workspace || workspace_bytes < need)
        return sfail(ACM_ERR_WORKSPACE_TOO_SMALL, "LM workspace too small");
    const size_t ne_ws = acm_normal_equations_workspace_size(cam->model, n);
    double* d_res = (double*)((char*)workspace + ne_ws);
    const int R = P * P + P + 2;
    hipStream_t s = (hipStream_t)stream;
    // Without an all-reduce the epilogue kernel writes the R results straight
    // into pinned, device-mapped host memory: no device-to-host copy launch
    // per evaluation.  One buffer per host thread (calls on different threads
    // never share it), owned by a thread_local that frees it when the thread
    // exits.  In mode 2 the kernel also publishes a sequence number in the
    // buffer's last word, and the host spins on that word instead of
    // synchronising the stream.
    struct PinnedResults {
        double* p = nullptr;
        unsigned long long seq = 0;
        ~PinnedResults() {
            if (p && hipHostFree(p) != hipSuccess) (void)hipGetLastError();
        }
    };
    static thread_local PinnedResults tl;
    double*& pinned = tl.p;
    unsigned long long& seq = tl.seq;
    // (r06) With an all-reduce the epilogue writes device memory, the
    // callback sums it in place on the stream (RCCL), and in mode 2 one
    // single-lane kernel then copies the sums into the pinned buffer and
    // publishes the completion word: the host spins as without an
    // all-reduce, instead of a pageable copy and a stream synchronisation.
    const int knob = acm::lm_host_result();
    if (knob && !pinned) {
        void* p = nullptr;
        if (hipHostMalloc(&p, 128 * sizeof(double),
                          hipHostMallocMapped | hipHostMallocPortable |
                              hipHostMallocCoherent) == hipSuccess)
            pinned = (double*)p;
        else
            (void)hipGetLastError();
    }
    int host_mode = pinned ? knob : 0;
    // (r06) 3: the pre-queued evaluations (lm_doorbell_loop) where the
    // normal equations support them, else the mode-2 loop
    const bool doorbell = host_mode == 3 && !allreduce && acm::ne_dev_ok(layout);
    if (host_mode == 3) host_mode = 2;
    double* res_out = d_res;
    unsigned long long* flag = nullptr;
    // the finish kernel's ticket (mode 2 without an all-reduce): one of
    // d_res's spare words, zeroed here and re-armed by the last workgroup of
    // every evaluation
    unsigned int* ticket = nullptr;
    if (host_mode == 2) flag = reinterpret_cast<unsigned long long*>(pinned + 127);
    if (host_mode && !allreduce) {
        res_out = pinned;
        if (host_mode == 2) {
            ticket = reinterpret_cast<unsigned int*>(d_res + R);
            if (hip_ok(hipMemsetAsync(ticket, 0, sizeof(unsigned int), s)))
                return sfail(ACM_ERR_HIP, "LM: ticket reset failed");
        }
    }
    // evaluate [JtJ | Jtr | 0.5 r.r | n_valid] at parameter vector x (the
    // host loop)
    auto eval = [&](const double* x, double* out) -> int {
        acm_camera c = *cam;
        for (int i = 0; i < P; ++i) c.params[i] = x[i];
        const unsigned long long want = flag ? ++seq : 0;
        int rc = acm::normal_equations_impl(&c, n, points_3d, layout, points_2d,
                                            cfg->invalid_policy, res_out, workspace, ne_ws, stream,
                                            allreduce ? nullptr : flag, want, ticket, cells, grid,
                                            nullptr);
        if (rc) return rc;
        if (allreduce) {
            rc = allreduce(allreduce_ctx, d_res, (size_t)R, stream);
            if (rc) return sfail(ACM_ERR_HIP, "all-reduce callback failed");
            if (flag) {
                hipLaunchKernelGGL(k_lm_copy_publish, dim3(1), dim3(64), 0, s, d_res, pinned, R,
                                   flag, want);
                if (hip_ok(hipGetLastError())) return sfail(ACM_ERR_HIP, "LM: publish launch");
            } else if (host_mode == 1 &&
                       hip_ok(hipMemcpyAsync(pinned, d_res, R * sizeof(double),
                                             hipMemcpyDeviceToHost, s))) {
                return sfail(ACM_ERR_HIP, "LM: device copy failed");
            }
        }
        if (flag) {
            // spin on the completion word; every 256 polls ask the stream, so
            // a failed launch surfaces as an error instead of a hang
            for (unsigned spin = 1;; ++spin) {
                if (__atomic_load_n(flag, __ATOMIC_ACQUIRE) == want) break;
                if ((spin & 255) == 0) {
                    const hipError_t q = hipStreamQuery(s);
                    if (q == hipSuccess) {
                        if (__atomic_load_n(flag, __ATOMIC_ACQUIRE) == want) break;
                        return sfail(ACM_ERR_HIP, "LM: completion word not published");
                    }
                    if (q != hipErrorNotReady) return sfail(ACM_ERR_HIP, "LM: stream failed");
                }
                __builtin_ia32_pause();
            }
            std::memcpy(out, pinned, R * sizeof(double));
        } else if (host_mode == 1) {
            if (hip_ok(hipStreamSynchronize(s))) return sfail(ACM_ERR_HIP, "LM: stream failed");
            std::memcpy(out, pinned, R * sizeof(double));
        } else if (hip_ok(hipMemcpyAsync(out, d_res, R * sizeof(double), hipMemcpyDeviceToHost,
                                         s)) ||
                   hip_ok(hipStreamSynchronize(s))) {
            return sfail(ACM_ERR_HIP, "LM: device copy failed");
        }
        return ACM_SUCCESS;
    };

    acm::lm::State st;
    acm::lm::start(st, *cfg, P, cam->params);
    if (doorbell) {
        return lm_doorbell_loop(cam, n, points_3d, layout, points_2d, cells, grid, cfg, st, P,
                                pinned, seq, d_res, workspace, ne_ws, summary, s);
    }
    // the host loop: one normal-equations evaluation per state-machine step
    // (lm_core.hpp).  A device-resident form of this loop (r04: the state
    // machine in a one-wave kernel behind each evaluation, the host queueing
    // evaluations ahead) measured slower -- 1.41 vs 1.33 ms at config 3 --
    // and was removed in r05 (history: git show 5cd4fce:apex-camera-models_amd/csrc/solver.hip).
    std::vector<double> res(R);
    int r = acm::lm::NEED_EVAL;
    while (r == acm::lm::NEED_EVAL) {
        int rc = eval(st.xn, res.data());
        if (rc) return rc;
        r = acm::lm::consume(st, *cfg, res.data(), P);
    }
    lm_summarize(st, cam, P, summary);
    return ACM_SUCCESS;
}

ACM_API int acm_lm_optimize(acm_camera* cam, size_t n, const double* points_3d, int layout,
                            const double* points_2d, const acm_lm_config* cfg,
                            acm_allreduce_fn allreduce, void* allreduce_ctx,
                            acm_lm_summary* summary, void* workspace, size_t workspace_bytes,
                            void* stream) {
    return lm_optimize(cam, n, points_3d, layout, points_2d, nullptr, nullptr, cfg, allreduce,
                       allreduce_ctx, summary, workspace, workspace_bytes, stream);
}

// (r06) the same LM over grid-sampled correspondences given by their cells
// (acm_normal_equations_cells): identical iterates, 28 instead of 40 B per
// point read by every evaluation
ACM_API int acm_lm_optimize_cells(acm_camera* cam, size_t n, const double* points_3d, int layout,
                                  const uint32_t* cells, const acm_cell_grid* grid,
                                  const acm_lm_config* cfg, acm_allreduce_fn allreduce,
                                  void* allreduce_ctx, acm_lm_summary* summary, void* workspace,
                                  size_t workspace_bytes, void* stream) {
    int rc = acm::check_cell_grid(grid);
    if (rc) return rc;
    if (n && !cells) return sfail(ACM_ERR_INVALID_ARGUMENT, "NULL cells");
    static const uint32_t none = 0;
    return lm_optimize(cam, n, points_3d, layout, nullptr, cells ? cells : &none, grid, cfg,
                       allreduce, allreduce_ctx, summary, workspace, workspace_bytes, stream);
}

}  // extern "C"
