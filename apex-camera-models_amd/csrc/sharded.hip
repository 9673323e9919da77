// sharded.hip -- the multi-GPU conversion path (r06):
// every rank holds a shard of the correspondences, and the conversion runs
// over their union with stream-ordered collectives and no Python in the loop.
//
//   * acm_linear_estimation_with_error_sharded -- convert_to_*'s opening
//     (camera_converter.rs:371-375): per shard the fused k_tsqr<+initial
//     error> pass (R factor, error flag, the 8 statistics, the median's
//     first histogram) as on one GPU, then ONE all-gather of a 32-double
//     record per rank [R | flag | n | statistics], the Givens merge of the
//     factors and Chan's merge of the statistics in rank order on the host,
//     and the exact median of the union (error_metrics.rs:103-111) with its
//     first histogram merged from the fused pass and every histogram summed
//     over the ranks.  The host solve overlaps the median, as on one GPU.
//   * acm_reprojection_error_sharded -- compute_reprojection_error
//     (error_metrics.rs:62-121) over the union, the same way.
//   * acm_rccl_* -- an acm_collective over an RCCL communicator that libacm
//     drives itself (librccl loaded at run time), so the LM's all-reduce per
//     evaluation and the median's histogram all-reduces are RCCL calls on the
//     caller's stream with no host round trip of their own.
//
// With one rank every merge is the identity (a single part passes through
// unchanged), so the sharded path at world 1 returns the bits of the 1-GPU
// path (tests/test_gpu_sharded.py).
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>  // types and prototypes only: the library is dlopen-ed

#include <algorithm>
#include <cmath>
#include <cstring>
#include <string>
#include <vector>

#include "acm.h"

namespace acm {
int set_error(int code, const std::string& msg);  // acm.hip
int linear_system_qr_error(const acm_camera* cam, size_t n, const double* points_3d, int layout,
                           const double* points_2d, double* r_factor, int* error_flag,
                           double* result, void* ws_qr, void* ws_err, void* stream,
                           double* host_out, hipEvent_t ready, int* hist_nb,
                           const uint32_t* cells, const acm_cell_grid* grid);
size_t reproj_error_hist_off(size_t n);
size_t reproj_error_median_off(size_t n);
int reprojection_stats_hist(const acm_camera* cam, size_t n, const double* points_3d, int layout,
                            const double* points_2d, double* result, double* errors,
                            void* workspace, void* stream, int* hist_nb,
                            const uint32_t* cells, const acm_cell_grid* grid);
int check_cell_grid(const acm_cell_grid* grid);
int median_union(size_t n, const double* values, uint64_t n_valid_global, double* out,
                 void* median_ws, acm_allreduce_fn allreduce, void* allreduce_ctx, void* stream,
                 const unsigned int* hparts, int hist_nb);
}  // namespace acm

namespace {

int sfail(int code, const std::string& m) { return acm::set_error(code, m); }

constexpr int kRec = 32;  // doubles per rank in the opening's all-gather
// record layout: [0..16] R factor (packed upper triangle, <= 15) + the error
// flag's int bits in [16] (as acm_linear_system_qr leaves them), [17] n,
// [18..25] the shard's acm_reprojection_stats result
constexpr int kRecN = 17, kRecStats = 18;

size_t up256(size_t b) { return (b + 255) / 256 * 256; }

// ------------------------------------------------------------------ RCCL
struct RcclApi {
    decltype(&ncclGetUniqueId) get_id = nullptr;
    decltype(&ncclCommInitRank) init = nullptr;
    decltype(&ncclAllReduce) allreduce = nullptr;
    decltype(&ncclAllGather) allgather = nullptr;
    decltype(&ncclCommDestroy) destroy = nullptr;
    decltype(&ncclGetErrorString) errstr = nullptr;
    bool ok = false;
};

// The process's RCCL: the copy already loaded (torch's, whose soname is
// librccl.so.1) if there is one -- one RCCL per process -- else ROCm's.
const RcclApi* rccl() {
    static const RcclApi api = [] {
        RcclApi a;
        void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_NOLOAD);
        if (!h) h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
        if (!h) h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
        if (!h) return a;
        a.get_id = (decltype(a.get_id))dlsym(h, "ncclGetUniqueId");
        a.init = (decltype(a.init))dlsym(h, "ncclCommInitRank");
        a.allreduce = (decltype(a.allreduce))dlsym(h, "ncclAllReduce");
        a.allgather = (decltype(a.allgather))dlsym(h, "ncclAllGather");
        a.destroy = (decltype(a.destroy))dlsym(h, "ncclCommDestroy");
        a.errstr = (decltype(a.errstr))dlsym(h, "ncclGetErrorString");
        a.ok = a.get_id && a.init && a.allreduce && a.allgather && a.destroy && a.errstr;
        return a;
    }();
    return api.ok ? &api : nullptr;
}

struct RcclCtx {
    ncclComm_t comm = nullptr;
};

int rccl_allreduce_cb(void* ctx, double* buf, size_t count, void* stream) {
    const RcclApi* r = rccl();
    auto* c = (RcclCtx*)ctx;
    if (!r || !c || !c->comm) return -1;
    return r->allreduce(buf, buf, count, ncclDouble, ncclSum, c->comm, (hipStream_t)stream) ==
                   ncclSuccess
               ? 0
               : -1;
}

int rccl_allgather_cb(void* ctx, const double* send, double* recv, size_t count, void* stream) {
    const RcclApi* r = rccl();
    auto* c = (RcclCtx*)ctx;
    if (!r || !c || !c->comm) return -1;
    return r->allgather(send, recv, count, ncclDouble, c->comm, (hipStream_t)stream) == ncclSuccess
               ? 0
               : -1;
}

// ------------------------------------------------- host side of a stage
// Pinned memory for the gathered records and one event per host thread,
// made on the device of the caller's stream (switching to it only to create
// the event); grown on demand, freed when the thread exits.
struct ShardHost {
    double* p = nullptr;
    size_t cap = 0;
    hipEvent_t ev = nullptr;
    int ev_dev = -1;
    bool ok(hipStream_t stream, size_t doubles) {
        if (cap < doubles) {
            if (p && hipHostFree(p) != hipSuccess) (void)hipGetLastError();
            p = nullptr;
            cap = 0;
            void* q = nullptr;
            if (hipHostMalloc(&q, doubles * sizeof(double), hipHostMallocPortable) != hipSuccess) {
                (void)hipGetLastError();
                return false;
            }
            p = (double*)q;
            cap = doubles;
        }
        int cur = -1;
        if (hipGetDevice(&cur) != hipSuccess) {
            (void)hipGetLastError();
            return false;
        }
        int dev = cur;
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
            if (!made) (void)hipGetLastError();
            if (dev != cur && hipSetDevice(cur) != hipSuccess) (void)hipGetLastError();
            if (!made) {
                ev = nullptr;
                return false;
            }
            ev_dev = dev;
        }
        return true;
    }
    ~ShardHost() {
        if (ev && hipEventDestroy(ev) != hipSuccess) (void)hipGetLastError();
        if (p && hipHostFree(p) != hipSuccess) (void)hipGetLastError();
    }
};

struct Eight {
    double v[8];
};

// one shard's record: the R factor and flag (17 doubles as written by
// k_tsqr_final / the flag), n, and the 8 statistics
__global__ void k_shard_record(const double* __restrict__ r17, const double* __restrict__ stats,
                               double n, double* __restrict__ rec) {
    const int t = threadIdx.x;
    if (t < kRec) {
        double v = 0.0;
        if (t < kRecN && r17) v = r17[t];
        else if (t == kRecN) v = n;
        else if (t >= kRecStats && t < kRecStats + 8) v = stats[t - kRecStats];
        rec[t] = v;
    }
}

// the merged statistics, written in stream order from the kernel argument
// (no pinned source that a later call could overwrite before the copy runs)
__global__ void k_store8(Eight e, double* __restrict__ dst) {
    if (threadIdx.x < 8) dst[threadIdx.x] = e.v[threadIdx.x];
}

int hip_fail(const char* what) {
    const hipError_t e = hipGetLastError();
    return sfail(ACM_ERR_HIP, std::string(what) + ": " + hipGetErrorString(e));
}

// All-gather `rec` (kRec doubles) into `gath` (world x kRec) and bring the
// gathered records to the host (host.p).  world 1 without callbacks: the
// record itself.
int gather_records(const acm_collective* coll, int world, const double* rec, double* gath,
                   ShardHost& host, hipStream_t s) {
    const double* src = rec;
    if (coll && coll->allgather) {
        if (coll->allgather(coll->ctx, rec, gath, kRec, s) != 0)
            return sfail(ACM_ERR_HIP, "sharded: all-gather callback failed");
        src = gath;
    } else if (world != 1) {
        return sfail(ACM_ERR_INVALID_ARGUMENT, "sharded: world > 1 needs an all-gather");
    }
    if (hipMemcpyAsync(host.p, src, (size_t)world * kRec * sizeof(double), hipMemcpyDeviceToHost,
                       s) != hipSuccess ||
        hipEventRecord(host.ev, s) != hipSuccess || hipEventSynchronize(host.ev) != hipSuccess)
        return hip_fail("sharded: gathered records");
    return ACM_SUCCESS;
}

// Rank-ordered merge of the statistics in the gathered records; a single
// contributing part passes through bit for bit (world 1 = the 1-GPU result).
void merge_stats(const double* recs, int world, double* g8) {
    std::vector<double> parts((size_t)world * 8);
    int contributing = 0, last = 0;
    for (int r = 0; r < world; ++r) {
        std::memcpy(&parts[(size_t)r * 8], recs + (size_t)r * kRec + kRecStats, 8 * sizeof(double));
        if (parts[(size_t)r * 8 + 5] > 0.0) {
            ++contributing;
            last = r;
        }
    }
    if (contributing == 1) {
        std::memcpy(g8, &parts[(size_t)last * 8], 8 * sizeof(double));
        return;
    }
    acm_reprojection_stats_merge((size_t)world, parts.data(), g8);
}

int check_coll(const acm_collective* coll, int* world) {
    *world = coll ? coll->world : 1;
    if (*world < 1 || (coll && (coll->rank < 0 || coll->rank >= coll->world)))
        return sfail(ACM_ERR_INVALID_ARGUMENT, "sharded: bad rank / world");
    if (*world > 1 && (!coll->allreduce || !coll->allgather))
        return sfail(ACM_ERR_INVALID_ARGUMENT, "sharded: world > 1 needs both collectives");
    return ACM_SUCCESS;
}

// The distributed statistics + median stage shared by both entry points:
// `result` (device) holds this shard's 8 statistics; on return it holds the
// union's, result[8] gets the union's median in stream order, and g8 (host)
// the merged statistics.  rec / gath: device scratch; n_total_out: the
// union's point count.
int union_stats_and_median(const acm_collective* coll, int world, size_t n,
                           const double* r17, double* result, const double* errs, void* mws,
                           const unsigned int* hparts, int hist_nb, double* rec, double* gath,
                           ShardHost& host, hipStream_t s, double* g8, double* recs_out,
                           size_t* n_total_out) {
    hipLaunchKernelGGL(k_shard_record, dim3(1), dim3(64), 0, s, r17, result, (double)n, rec);
    if (hipGetLastError() != hipSuccess) return hip_fail("sharded: record");
    int rc = gather_records(coll, world, rec, gath, host, s);
    if (rc) return rc;
    std::memcpy(recs_out, host.p, (size_t)world * kRec * sizeof(double));
    merge_stats(recs_out, world, g8);
    size_t n_total = 0;
    for (int r = 0; r < world; ++r) n_total += (size_t)recs_out[(size_t)r * kRec + kRecN];
    *n_total_out = n_total;
    Eight e;
    std::memcpy(e.v, g8, sizeof(e.v));
    hipLaunchKernelGGL(k_store8, dim3(1), dim3(64), 0, s, e, result);
    if (hipGetLastError() != hipSuccess) return hip_fail("sharded: statistics store");
    const double nv = g8[5];
    const uint64_t n_valid = nv > 0.0 ? (uint64_t)nv : 0;
    return acm::median_union(n, errs, n_valid, result + 8, mws, coll ? coll->allreduce : nullptr,
                             coll ? coll->ctx : nullptr, s, hparts, hist_nb);
}

int count_check_total(int model, size_t n_total) {
    if (model == ACM_KANNALA_BRANDT && n_total < 4)  // kannala_brandt.rs:174-178
        return sfail(ACM_ERR_INVALID_PARAMS,
                     "Not enough points for linear estimation (need at least 4)");
    if (model == ACM_RADTAN && n_total < 3)  // rad_tan.rs:152-156
        return sfail(ACM_ERR_INVALID_PARAMS, "Need at least 3 points for RadTan linear estimation");
    if (model == ACM_EUCM && n_total < 1)  // eucm.rs:228-232
        return sfail(ACM_ERR_INVALID_PARAMS, "Need at least 1 point for EUCM linear estimation");
    if (model == ACM_FOV && n_total < 2)  // fov.rs:166-171
        return sfail(ACM_ERR_INVALID_PARAMS,
                     "Need at least 2 point correspondences for linear estimation");
    return ACM_SUCCESS;
}

// workspace layout of the sharded opening
struct OpenLayout {
    size_t qr, r, err, fov, rec, gath, total;
};
OpenLayout open_layout(int model, size_t n, int world) {
    OpenLayout L{};
    const int k = acm_linear_system_columns(model);
    const size_t qr = k >= 0 ? up256(acm_linear_system_qr_workspace_size(model, n)) : 0;
    L.qr = 0;
    L.r = qr;
    L.err = L.r + 256;
    const size_t fov = model == ACM_FOV ? up256(acm_fov_grid_workspace_size(n)) +
                                              up256(2 * ACM_FOV_GRID_SIZE * sizeof(double))
                                        : 0;
    L.fov = L.err + up256(acm_reprojection_error_workspace_size(n));
    L.rec = L.fov + fov;
    L.gath = L.rec + 256;
    L.total = L.gath + up256((size_t)world * kRec * sizeof(double));
    return L;
}

size_t reproj_layout(size_t n, int world, size_t* rec, size_t* gath) {
    *rec = up256(acm_reprojection_error_workspace_size(n));
    *gath = *rec + 256;
    return *gath + up256((size_t)world * kRec * sizeof(double));
}

}  // namespace

extern "C" {

ACM_API int acm_rccl_available(void) { return rccl() ? 1 : 0; }

ACM_API int acm_rccl_unique_id(uint8_t* id) {
    if (!id) return sfail(ACM_ERR_INVALID_ARGUMENT, "NULL id");
    const RcclApi* r = rccl();
    if (!r) return sfail(ACM_ERR_NOT_SUPPORTED, "librccl.so.1 not loadable");
    ncclUniqueId u;
    const ncclResult_t e = r->get_id(&u);
    if (e != ncclSuccess) return sfail(ACM_ERR_HIP, std::string("ncclGetUniqueId: ") + r->errstr(e));
    std::memcpy(id, u.internal, ACM_RCCL_UNIQUE_ID_BYTES);
    return ACM_SUCCESS;
}

ACM_API int acm_rccl_init(const uint8_t* id, int32_t world, int32_t rank, acm_collective* out) {
    if (!id || !out) return sfail(ACM_ERR_INVALID_ARGUMENT, "NULL argument");
    if (world < 1 || rank < 0 || rank >= world)
        return sfail(ACM_ERR_INVALID_ARGUMENT, "bad rank / world");
    const RcclApi* r = rccl();
    if (!r) return sfail(ACM_ERR_NOT_SUPPORTED, "librccl.so.1 not loadable");
    ncclUniqueId u;
    std::memcpy(u.internal, id, ACM_RCCL_UNIQUE_ID_BYTES);
    auto* c = new RcclCtx;
    const ncclResult_t e = r->init(&c->comm, world, u, rank);
    if (e != ncclSuccess) {
        delete c;
        return sfail(ACM_ERR_HIP, std::string("ncclCommInitRank: ") + r->errstr(e));
    }
    std::memset(out, 0, sizeof(*out));
    out->allreduce = rccl_allreduce_cb;
    out->allgather = rccl_allgather_cb;
    out->ctx = c;
    out->rank = rank;
    out->world = world;
    return ACM_SUCCESS;
}

ACM_API int acm_rccl_destroy(acm_collective* coll) {
    if (!coll) return sfail(ACM_ERR_INVALID_ARGUMENT, "NULL collective");
    if (coll->allreduce != rccl_allreduce_cb || !coll->ctx)
        return sfail(ACM_ERR_INVALID_ARGUMENT, "not an acm_rccl_init collective");
    auto* c = (RcclCtx*)coll->ctx;
    int rc = ACM_SUCCESS;
    const RcclApi* r = rccl();
    if (r && c->comm && r->destroy(c->comm) != ncclSuccess)
        rc = sfail(ACM_ERR_HIP, "ncclCommDestroy failed");
    delete c;
    std::memset(coll, 0, sizeof(*coll));
    return rc;
}

ACM_API size_t acm_linear_estimation_with_error_sharded_workspace_size(int model, size_t n,
                                                                       int32_t world) {
    if (acm_num_params(model) < 0 || world < 1) return 0;
    if (acm_linear_system_columns(model) < 0 && model != ACM_FOV) return 0;
    return open_layout(model, n, world).total;
}

ACM_API int acm_linear_estimation_with_error_sharded(acm_camera* cam, size_t n,
                                                     const double* points_3d, int layout,
                                                     const double* points_2d,
                                                     const uint32_t* cells,
                                                     const acm_cell_grid* grid,
                                                     double* initial_error,
                                                     double* initial_error_host,
                                                     const acm_collective* coll, void* workspace,
                                                     size_t workspace_bytes, void* stream) {
    if (!cam) return sfail(ACM_ERR_INVALID_ARGUMENT, "camera is NULL");
    if (!initial_error || !workspace || (n && (!points_3d || !points_2d)))
        return sfail(ACM_ERR_INVALID_ARGUMENT, "NULL buffer");
    int world = 1;
    int rc = check_coll(coll, &world);
    if (rc) return rc;
    static const uint32_t none = 0;
    if (cells || grid) {  // the cell form of the observations (r06)
        if ((rc = acm::check_cell_grid(grid))) return rc;
        if (n && !cells) return sfail(ACM_ERR_INVALID_ARGUMENT, "NULL buffer");
        if (!cells) cells = &none;
    }
    const size_t need = acm_linear_estimation_with_error_sharded_workspace_size(cam->model, n, world);
    if (!need) return sfail(ACM_ERR_NOT_SUPPORTED, "model has no linear_estimation");
    if (workspace_bytes < need)
        return sfail(ACM_ERR_WORKSPACE_TOO_SMALL, "sharded linear-estimation workspace too small");
    hipStream_t s = (hipStream_t)stream;
    static thread_local ShardHost host;
    if (!host.ok(s, (size_t)world * kRec + 2 * ACM_FOV_GRID_SIZE))
        return sfail(ACM_ERR_HIP, "sharded: pinned buffer or event");
    const OpenLayout Lo = open_layout(cam->model, n, world);
    char* ws = (char*)workspace;
    double* d_r = (double*)(ws + Lo.r);
    void* ws_err = ws + Lo.err;
    double* errs = (double*)ws_err;  // the errors lead acm_reprojection_error's workspace
    void* mws = (char*)ws_err + acm::reproj_error_median_off(n);
    const unsigned int* hparts = (const unsigned int*)((char*)ws_err + acm::reproj_error_hist_off(n));
    double* rec = (double*)(ws + Lo.rec);
    double* gath = (double*)(ws + Lo.gath);
    const int k = acm_linear_system_columns(cam->model);
    int nb = 1;
    // this shard: the fused pass (TSQR models), or the statistics pass (FOV)
    if (k >= 0)
        rc = acm::linear_system_qr_error(cam, n, points_3d, layout, points_2d, d_r, (int*)(d_r + 16),
                                         initial_error, ws + Lo.qr, ws_err, stream, nullptr,
                                         nullptr, &nb, cells, grid);
    else
        rc = acm::reprojection_stats_hist(cam, n, points_3d, layout, points_2d, initial_error,
                                          nullptr, ws_err, stream, &nb, cells, grid);
    if (rc) return rc;
    std::vector<double> recs((size_t)world * kRec);
    double g8[8];
    size_t n_total = 0;
    rc = union_stats_and_median(coll, world, n, k >= 0 ? d_r : nullptr, initial_error, errs, mws,
                                hparts, nb, rec, gath, host, s, g8, recs.data(), &n_total);
    if (rc) return rc;
    if (initial_error_host) std::memcpy(initial_error_host, g8, sizeof(g8));
    // the reference computes the initial error first, then linear_estimation
    // raises on too few points (of the union)
    if ((rc = count_check_total(cam->model, n_total))) return rc;
    if (k < 0) {  // FOV: the grid sums are additive over shards (fov.rs:176-249)
        double* d_sums = (double*)(ws + Lo.fov + up256(acm_fov_grid_workspace_size(n)));
        if (n) {
            rc = acm_fov_grid_errors(cam, n, points_3d, layout, points_2d, d_sums, ws + Lo.fov,
                                     acm_fov_grid_workspace_size(n), stream);
            if (rc) return rc;
        } else if (hipMemsetAsync(d_sums, 0, 2 * ACM_FOV_GRID_SIZE * sizeof(double), s) !=
                   hipSuccess) {
            return hip_fail("sharded: FOV sums");
        }
        if (coll && coll->allreduce &&
            coll->allreduce(coll->ctx, d_sums, 2 * ACM_FOV_GRID_SIZE, stream) != 0)
            return sfail(ACM_ERR_HIP, "sharded: all-reduce callback failed");
        if (hipMemcpyAsync(host.p, d_sums, 2 * ACM_FOV_GRID_SIZE * sizeof(double),
                           hipMemcpyDeviceToHost, s) != hipSuccess ||
            hipEventRecord(host.ev, s) != hipSuccess || hipEventSynchronize(host.ev) != hipSuccess)
            return hip_fail("sharded: FOV sums copy");
        return acm_fov_grid_select(cam, host.p);
    }
    // R of the stacked rows: the factors folded in rank order (Givens), the
    // flags OR-ed; the host solve overlaps the median on the stream
    const int M = k + 1, S = M * (M + 1) / 2;
    double R[16] = {0};
    int err = 0;
    for (int r = 0; r < world; ++r) {
        const double* p = &recs[(size_t)r * kRec];
        int f = 0;
        std::memcpy(&f, p + 16, sizeof(int));
        err |= f;
        if (r == 0) std::memcpy(R, p, S * sizeof(double));
        else if ((rc = acm_linear_system_r_merge(cam->model, R, p))) return rc;
    }
    return acm_linear_estimation_solve(cam, n_total, R, err);
}

ACM_API size_t acm_reprojection_error_sharded_workspace_size(size_t n, int32_t world) {
    if (world < 1) return 0;
    size_t rec, gath;
    return reproj_layout(n, world, &rec, &gath);
}

ACM_API int acm_reprojection_error_sharded(const acm_camera* cam, size_t n,
                                           const double* points_3d, int layout,
                                           const double* points_2d, const uint32_t* cells,
                                           const acm_cell_grid* grid, double* result,
                                           double* errors, const acm_collective* coll,
                                           void* workspace, size_t workspace_bytes,
                                           void* stream) {
    if (!cam) return sfail(ACM_ERR_INVALID_ARGUMENT, "camera is NULL");
    if (!result || !workspace || (n && (!points_3d || !(points_2d || cells))))
        return sfail(ACM_ERR_INVALID_ARGUMENT, "NULL buffer");
    int world = 1;
    int rc = check_coll(coll, &world);
    if (rc) return rc;
    static const uint32_t none = 0;
    if (cells || grid) {
        if ((rc = acm::check_cell_grid(grid))) return rc;
        if (!cells) cells = &none;
    }
    size_t off_rec, off_gath;
    if (workspace_bytes < reproj_layout(n, world, &off_rec, &off_gath))
        return sfail(ACM_ERR_WORKSPACE_TOO_SMALL, "sharded reprojection-error workspace too small");
    hipStream_t s = (hipStream_t)stream;
    static thread_local ShardHost host;
    if (!host.ok(s, (size_t)world * kRec)) return sfail(ACM_ERR_HIP, "sharded: pinned buffer or event");
    char* ws = (char*)workspace;
    int nb = 1;
    rc = acm::reprojection_stats_hist(cam, n, points_3d, layout, points_2d, result, errors, ws,
                                      stream, &nb, cells, grid);
    if (rc) return rc;
    const double* errs = errors ? errors : (const double*)ws;
    void* mws = ws + acm::reproj_error_median_off(n);
    const unsigned int* hparts = (const unsigned int*)(ws + acm::reproj_error_hist_off(n));
    std::vector<double> recs((size_t)world * kRec);
    double g8[8];
    size_t n_total = 0;
    return union_stats_and_median(coll, world, n, nullptr, result, errs, mws, hparts, nb,
                                  (double*)(ws + off_rec), (double*)(ws + off_gath), host, s, g8,
                                  recs.data(), &n_total);
}

}  // extern "C"
