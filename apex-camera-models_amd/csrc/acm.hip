// acm.hip -- MI355X (gfx950) kernels and the C-ABI of libacm.so.
//
// The hot path of the reference (per-point CameraModel::project/unproject and
// the apex-solver *CameraParamsFactor linearisation, see include/acm.h) is a
// pure streaming map: every point is independent and touches 41-185 bytes of
// HBM for ~100-400 f64 operations.  It is bound by HBM bandwidth, so the
// kernels are built around the memory system, not MFMA:
//   * one point per lane, 256-lane workgroups, one launch covers the batch
//     (10M points -> 39k workgroups, far more than the 256 CUs x 8 slots);
//   * inputs read once, outputs written once, every store 16 B per lane and
//     contiguous across the wave (uv pairs, the (du,dv) pair of each column
//     of the 2N x P column-major Jacobian), status bytes contiguous;
//   * camera parameters arrive by value in the kernel arguments -> SGPRs;
//   * the reductions (normal equations, residual norms) keep per-lane sums
//     in registers, reduce with wave64 shuffles, then across the 4 waves of
//     a workgroup in LDS, and finish with a fixed-order second pass, so the
//     result is bit-reproducible run to run.
#include <hip/hip_runtime.h>

#include <atomic>

#include <cmath>
#include <cstdio>
#include <algorithm>
#include <array>
#include <cstring>
#include <map>
#include <mutex>
#include <string>
#include <type_traits>

#include "acm.h"
#include "camera_models.hpp"
#include "lm_doorbell.hpp"

namespace acm {

static thread_local std::string g_last_error;
static thread_local int g_last_hip_error = 0;

static int fail(int code, const std::string& msg) {
    g_last_error = msg;
    return code;
}

int set_error(int code, const std::string& msg) { return fail(code, msg); }

static int check_launch(const char* what) {
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        g_last_hip_error = (int)e;
        return fail(ACM_ERR_HIP, std::string(what) + ": " + hipGetErrorString(e));
    }
    return ACM_SUCCESS;
}

template <template <class> class M>
struct Tag {
    template <class T>
    using type = M<T>;
};

// sample_points' write kernels on a KB camera whose certified rays come from
// the host's ray polynomials (kb_fit_ray): a tag of its own, so those
// kernels hold only the polynomials' coefficients (the Newton form's
// initial guess and sin / cos coefficients beside them spilled SGPRs)
struct TagKbPoly : Tag<KannalaBrandt> {};
template <class TagT>
struct SampleTag {
    using count = TagT;  // the count kernels' tag
    static constexpr bool kb = std::is_same<TagT, Tag<KannalaBrandt>>::value;
    static constexpr bool poly = false;
};
template <>
struct SampleTag<TagKbPoly> {
    using count = Tag<KannalaBrandt>;
    static constexpr bool kb = true;
    static constexpr bool poly = true;
};

template <class F>
static int dispatch_model(int model, F&& f) {
    switch (model) {
    case ACM_PINHOLE: return f(Tag<Pinhole>{});
    case ACM_RADTAN: return f(Tag<RadTan>{});
    case ACM_KANNALA_BRANDT: return f(Tag<KannalaBrandt>{});
    case ACM_DOUBLE_SPHERE: return f(Tag<DoubleSphere>{});
    case ACM_UCM: return f(Tag<Ucm>{});
    case ACM_EUCM: return f(Tag<Eucm>{});
    case ACM_FOV: return f(Tag<Fov>{});
    default: return fail(ACM_ERR_INVALID_MODEL, "unknown camera model id");
    }
}

// Uniform subexpressions of the unprojections, in the reference's operation
// order (IEEE results: the host and a lane compute the same bits).
template <class T>
__host__ __device__ inline void unproject_consts(int model, const T* p, T* uk) {
    uk[0] = uk[1] = uk[2] = uk[3] = T(0);
    if (model == ACM_KANNALA_BRANDT) {
        // uk[0]: 1 enables the certified fast Newton of
        // KannalaBrandt::unproject, NaN disables it.  Its error bound assumes
        // the polynomial's terms stay small on theta in [0, 2]:
        // sum |k_i| 4^i <= 63 (other cameras take the reference loop).
        const T b = T(4) * fabs(p[4]) + T(16) * fabs(p[5]) + T(64) * fabs(p[6]) +
                    T(256) * fabs(p[7]);
        uk[0] = b <= T(63) ? T(1) : T(NAN);
        // uk[1]: the status of a NaN pixel -- the reference loop
        // (kannala_brandt.rs:474-511) on ru = min(NaN, pi/2) = pi/2, in its
        // own operation order (this file is built -ffp-contract=off)
        {
            const T k1 = p[4], k2 = p[5], k3 = p[6], k4 = p[7];
            const T ru = T(kPi / 2.0);
            T theta = ru;
            bool conv = true;
            for (int i = 0; i < 10; ++i) {
                T t2 = theta * theta, t4 = t2 * t2, t6 = t4 * t2, t8 = t4 * t4;
                T a = k1 * t2, bb = k2 * t4, cc = k3 * t6, d = k4 * t8;
                T f = theta * (T(1) + a + bb + cc + d) - ru;
                T fp = T(1) + (T(3) * a) + (T(5) * bb) + (T(7) * cc) + (T(9) * d);
                if (fabs(fp) < T(kEps)) { conv = false; break; }
                T delta = f / fp;
                theta -= delta;
                if (fabs(delta) < T(1e-6)) break;
                if (i == 9) conv = false;
            }
            uk[1] = conv ? T(ST_OK) : T(ST_NUMERICAL_ERROR);
        }
    } else if (model == ACM_RADTAN) {
        // uk[0]: the certified fast Newton of RadTan::unproject (1) or not
        // (NaN); its error bound assumes |rad| <= 16 for |x|, |y| <= 2.
        const T b = T(8) * fabs(p[4]) + T(64) * fabs(p[5]) + T(512) * fabs(p[8]) +
                    T(16) * (fabs(p[6]) + fabs(p[7]));
        uk[0] = b <= T(15) ? T(1) : T(NAN);
    } else if (model == ACM_FOV) {
        // Fov::unproject's fast form: uk[0] = 1 (NaN: off), uk[1] =
        // 1 / (2 tan(w / 2)) (p[8] = tan(w / 2), set by prep on the host)
        uk[0] = T(1);
        uk[1] = T(1) / (T(2) * p[8]);
    } else if (model == ACM_DOUBLE_SPHERE) {
        uk[0] = T(1) / (T(2) * p[4] - T(1));  // double_sphere.rs:205
        // (r05) the projection condition's w2 (double_sphere.rs:177-184), a
        // camera constant the reference evaluates per point: the same IEEE
        // operations, so the same bits, once per camera
        const T alpha = p[4], xi = p[5];
        const T w1 = alpha <= T(0.5) ? alpha / (T(1) - alpha) : (T(1) - alpha) / alpha;
        uk[1] = (w1 + xi) / sqrt(T(2) * w1 * xi + xi * xi + T(1));
    } else if (model == ACM_UCM) {
        const T gamma = T(1) - p[4];
        uk[0] = p[4] / gamma;                          // xi, ucm.rs:343
        uk[1] = gamma * gamma / (T(2) * p[4] - T(1));  // ucm.rs:180
        // (r05) the projection condition's w (ucm.rs:154-161), per camera
        uk[2] = p[4] <= T(0.5) ? p[4] / (T(1) - p[4]) : (T(1) - p[4]) / p[4];
    } else if (model == ACM_EUCM) {
        uk[0] = T(1) / p[5] * (T(2) * p[4] - T(1));  // eucm.rs:196 (precedence quirk)
        // (r05) the projection condition's (alpha - 1) / (2 alpha - 1)
        // (eucm.rs:167-177, used when alpha > 0.5), per camera
        uk[1] = (p[4] - T(1)) / (T(2) * p[4] - T(1));
    }
}

// The unprojection kernels' camera argument: acm_camera plus the host-side
// constants of Cam (prep): RN(1 / fx), RN(1 / fy) and unproject_consts.
struct CamArg : acm_camera {
    double ifx, ify;
    double uk[4];
    double kc[12];  // KB sample_points: certified kept interval + initial guess (Cam::kc)
    double rp[2 * kRayPolyN];  // KB sample_points: certified-ray polynomials (Cam::rp)
};

template <class T>
__device__ __forceinline__ Cam<T> make_cam(const acm_camera& c) {
    Cam<T> k;
#pragma unroll
    for (int i = 0; i < 9; ++i) k.p[i] = (T)c.params[i];
    k.w = (T)(double)c.width;
    k.h = (T)(double)c.height;
    k.wi = c.width;
    k.hi = c.height;
    k.ifx = k.ify = T(0);  // divide
    unproject_consts<T>(c.model, k.p, k.uk);
#pragma unroll
    for (int i = 0; i < 12; ++i) k.kc[i] = T(0);
    k.kc[0] = T(INFINITY);  // no certified interval (sample_points only)
#pragma unroll
    for (int i = 0; i < 2 * kRayPolyN; ++i) k.rp[i] = T(0);
    k.rpl = nullptr;
    return k;
}

template <class T>
__device__ __forceinline__ Cam<T> make_cam(const CamArg& c) {
    static_assert(sizeof(T) == 8, "the unprojection kernels run in double");
    Cam<T> k;
#pragma unroll
    for (int i = 0; i < 9; ++i) k.p[i] = c.params[i];
    k.w = (double)c.width;
    k.h = (double)c.height;
    k.wi = c.width;
    k.hi = c.height;
    k.ifx = c.ifx;
    k.ify = c.ify;
#pragma unroll
    for (int i = 0; i < 4; ++i) k.uk[i] = c.uk[i];
#pragma unroll
    for (int i = 0; i < 12; ++i) k.kc[i] = c.kc[i];
#pragma unroll
    for (int i = 0; i < 2 * kRayPolyN; ++i) k.rp[i] = c.rp[i];
    k.rpl = nullptr;
    return k;
}

// The sample_points kernels' camera: make_cam, plus (TagKbPoly) the ray
// polynomials staged in LDS as (C_i, S_i) pairs for ray_certified<true>.
// Every thread of the workgroup must call it (it synchronises).
template <class TagT>
__device__ __forceinline__ Cam<double> sample_cam(const CamArg& cam) {
    Cam<double> c = make_cam<double>(cam);
    if constexpr (SampleTag<TagT>::poly) {
        __shared__ RayPolyPair s_rp[kRayPolyN];
        if (threadIdx.x < kRayPolyN)
            s_rp[threadIdx.x] = RayPolyPair{cam.rp[threadIdx.x], cam.rp[kRayPolyN + threadIdx.x]};
        __syncthreads();
        c.rpl = (lds_ray_poly*)s_rp;
    }
    return c;
}

// NTL: non-temporal loads (read-once streams; the read probe measured 6.9 vs
// 6.3 TB/s for a 400 MB sweep, profiles/r01_hbm_ceiling.log)
template <bool NTL>
__device__ __forceinline__ double ld1(const double* p) {
    if (NTL) return __builtin_nontemporal_load(p);
    return *p;
}

template <bool NTL>
__device__ __forceinline__ double2 ld2(const double* p) {
    typedef double d2v __attribute__((ext_vector_type(2)));
    if (NTL) {
        const d2v v = __builtin_nontemporal_load(reinterpret_cast<const d2v*>(p));
        return make_double2(v.x, v.y);
    }
    return *reinterpret_cast<const double2*>(p);
}

template <int LAYOUT, bool NTL = false>
__device__ __forceinline__ void load_point(const double* __restrict__ pts, size_t n, size_t i,
                                           double& x, double& y, double& z) {
    if (LAYOUT == ACM_LAYOUT_AOS) {
        x = ld1<NTL>(pts + 3 * i);
        y = ld1<NTL>(pts + 3 * i + 1);
        z = ld1<NTL>(pts + 3 * i + 2);
    } else {
        x = ld1<NTL>(pts + i);
        y = ld1<NTL>(pts + n + i);
        z = ld1<NTL>(pts + 2 * n + i);
    }
}

constexpr int kBlock = 256;

// ------------------------------------------------------------ project (+J)
typedef double dbl2 __attribute__((ext_vector_type(2)));

template <bool NT>
__device__ __forceinline__ void st2(double* p, double a, double b) {
    dbl2 v = {a, b};
    if (NT) __builtin_nontemporal_store(v, reinterpret_cast<dbl2*>(p));
    else *reinterpret_cast<dbl2*>(p) = v;
}

template <bool NT>
__device__ __forceinline__ void st1(uint8_t* p, uint8_t v) {
    if (NT) __builtin_nontemporal_store(v, p);
    else *p = v;
}

// Tuning variants of the direct project kernel (bit flags, see acm_set_tuning):
//   kVarNT     non-temporal stores for the write-once outputs
//   kVarGrid   persistent grid-stride launch (8 workgroups per CU)
//   kVarNTL    non-temporal loads of the point stream
// Default (-1, "auto"): non-temporal stores once the outputs exceed
// kNtThresholdBytes (0.252 vs 0.312 ms for 10M-point KB project+J,
// profiles/r01_sweep_project.log), plain loads (nt loads measured 20%
// slower beside the store stream, profiles/r01_diag_ntl.log).  (+J launches
// go to k_project_al unless ACM_TUNE_ALIGN_J = 0.)  A two-points-per-lane
// variant measured no gain and was dropped.
enum { kVarNT = 1, kVarGrid = 2, kVarNTL = 4 };
static std::atomic<int> g_project_variant{-1};
// Residual+J: plain stores by default.  Unlike project+J, non-temporal stores
// measured slower here (DS, 9.3M points: 0.273 ms plain vs 0.310 ms nt,
// profiles/r01_configs.log); -1 = auto (nt above kNtThresholdBytes), 1 = on.
static std::atomic<int> g_residual_nt{0};
// Normal equations: minimum waves per SIMD for the register allocator (1, 3,
// 4) and points per lane step (1, 2, 4); 0 = the per-model default below.
static std::atomic<int> g_ne_waves{0};
static std::atomic<int> g_ne_unroll{0};
// +J launches: -1 = auto = k_project_al (line-aligned store windows; as fast
// as k_project for N a multiple of 8 and 30-45% faster otherwise,
// profiles/r01_diag_align.log), 0 = k_project / k_residual, 1 = k_project_al.
static std::atomic<int> g_align_j{-1};
// Non-temporal loads of the read-once point / observation streams in
// k_normal_eq: -1 = auto (on), 0 = off, 1 = on (5-11% faster, read probe
// 6.9 vs 6.3 TB/s; profiles/r01_ne_sweep.log, r01_hbm_ceiling.log).
static std::atomic<int> g_nt_loads{-1};
// Non-temporal loads of the pixel stream in k_unproject (-1 auto = off, 0,
// 1): beside the non-temporal ray stores they measured 2-25% slower for
// every model (profiles/r01_diag_ntl.log).
static std::atomic<int> g_nt_loads_unproject{-1};
// FOV grid search kernel: -1 = the point-lane form (default), 0 = the
// per-point LDS record form, 1 / 2 / 4 = the LDS form with that many points
// per lane step.
static std::atomic<int> g_fov_unroll{-1};
// sample_points (include/acm.h ACM_TUNE_SAMPLE_FUSED): -1 = auto = the
// segment two-pass path (certified counts, scan, write) -- the speculative
// segment path (4) for RadTan; 0 = the round-1 two-pass count / scan /
// write path; 1 / 2 / 3 = single pass with a decoupled look-back, tiles of
// 2 / 4 / 8 x 256 cells; 4 = speculative segments.
static std::atomic<int> g_sample_fused{-1};
// sample_points look-back: polls of an unpublished predecessor's status word
// before the waiting wave counts that tile's cells itself (-1 = auto =
// kLbPatience; 0 = at once, which exercises the fallback in tests).
static std::atomic<int> g_sample_patience{-1};
// Unprojections: (u - cx) / fx and (v - cy) / fy from the host's RN(1 / fx),
// RN(1 / fy) (div_by_f, bit-identical) instead of two IEEE divisions per
// point: -1 = auto = on, 0 = off, 1 = on.
static std::atomic<int> g_unproject_rcp{-1};
static std::atomic<int> g_unproject_ppt{-1};
// acm_project_unproject's points per lane and AoS ray stores (include/acm.h
// ACM_TUNE_ROUND_TRIP): -1 = auto; else PPT (1, 2, 4) + 8 x stores (0 =
// the model's default, 1 = LDS-staged, 2 = three 8-B stores per ray).
static std::atomic<int> g_round_trip{-1};
// acm_lm_optimize without an all-reduce: the normal-equations epilogue writes
// its P*P + P + 2 results straight into pinned host memory instead of device
// memory + a device-to-host copy.  0 = off (copy + stream synchronise), 1 =
// pinned results + stream synchronise, 2 = pinned results + the host spins
// on a completion word the epilogue publishes; -1 = auto = 2.
static std::atomic<int> g_lm_host_result{-1};
int lm_host_result() {
    const int v = g_lm_host_result.load(std::memory_order_relaxed);
    return v < 0 ? 2 : v;
}
// Outputs above this many bytes are stored non-temporally.  Measured at 10M
// points (profiles/r01_diag_ntl.log): project without J (170 MB out) 0.056 ms
// nt vs 0.072 plain; a consumer that re-reads a smaller output soon after
// still finds it in the 256 MiB Infinity Cache with plain stores.
constexpr size_t kNtThresholdBytes = 64ull << 20;

template <class TagT, int LAYOUT, bool WJ, bool NT, bool EXACT = false>
__device__ __forceinline__ void project_point(const Cam<double>& c, size_t n, size_t i, double x,
                                              double y, double z, double* __restrict__ uv,
                                              uint8_t* __restrict__ status,
                                              double* __restrict__ jac) {
    using M = typename TagT::template type<double>;
    constexpr int P = M::P;
    double u, v, ju[P], jv[P];
    const uint8_t st = M::template project<WJ, false, EXACT>(c, x, y, z, u, v, ju, jv);
    const bool ok = st == ST_OK;
    st2<NT>(uv + 2 * i, ok ? u : __builtin_nan(""), ok ? v : __builtin_nan(""));
    st1<NT>(status + i, st);
    if (WJ) {
        const size_t col = 2 * n;
#pragma unroll
        for (int p = 0; p < P; ++p) st2<NT>(jac + p * col + 2 * i, ok ? ju[p] : 0.0, ok ? jv[p] : 0.0);
    }
}

// The per-point projection kernels take CamArg (r05): the per-camera
// constants of unproject_consts that a projection reads (DS w2, UCM w,
// EUCM's (alpha - 1) / (2 alpha - 1)) come from the host, computed once with
// the same IEEE operations, instead of once per lane by make_cam(acm_camera)
// -- with one point per lane that was once per point (equal speed, measured:
// profiles/r05aa_residual_camarg.log).
template <class TagT, int LAYOUT, bool WJ, int VAR>
__global__ __launch_bounds__(kBlock) void k_project(CamArg cam, size_t n,
                                                    const double* __restrict__ pts,
                                                    double* __restrict__ uv,
                                                    uint8_t* __restrict__ status,
                                                    double* __restrict__ jac) {
    constexpr bool NT = (VAR & kVarNT) != 0;
    constexpr bool NTL = (VAR & kVarNTL) != 0;
    const Cam<double> c = make_cam<double>(cam);
    if (VAR & kVarGrid) {
        const size_t stride = (size_t)gridDim.x * kBlock;
        for (size_t i = (size_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += stride) {
            double x, y, z;
            load_point<LAYOUT, NTL>(pts, n, i, x, y, z);
            project_point<TagT, LAYOUT, WJ, NT>(c, n, i, x, y, z, uv, status, jac);
        }
    } else {
        const size_t i = (size_t)blockIdx.x * kBlock + threadIdx.x;
        if (i >= n) return;
        double x, y, z;
        load_point<LAYOUT, NTL>(pts, n, i, x, y, z);
        project_point<TagT, LAYOUT, WJ, NT>(c, n, i, x, y, z, uv, status, jac);
    }
}

// ACM_EXACT_MATH projections of KB / FOV (camera_models.hpp EXACT: IEEE
// sqrt / divisions and the double-double atan2): one point per lane, direct
// stores.  Not a throughput path (the double-double atan2 costs ~10x the
// polynomial); the other models are exact in every kernel.
template <class TagT, int LAYOUT, bool WJ>
__global__ __launch_bounds__(kBlock) void k_project_exact(CamArg cam, size_t n,
                                                          const double* __restrict__ pts,
                                                          double* __restrict__ uv,
                                                          uint8_t* __restrict__ status,
                                                          double* __restrict__ jac) {
    const Cam<double> c = make_cam<double>(cam);
    const size_t i = (size_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    double x, y, z;
    load_point<LAYOUT>(pts, n, i, x, y, z);
    project_point<TagT, LAYOUT, WJ, false, true>(c, n, i, x, y, z, uv, status, jac);
}

// ------------------------------------------------ project (+J), f32 sweep
// The same model code evaluated in float (BASELINE config 5's f32 vs f64
// tolerance sweep): float in / float out, 12 + 8 + 1 + 8P bytes per point.
typedef float flt2 __attribute__((ext_vector_type(2)));

template <class TagT, int LAYOUT, bool WJ, bool NT>
__global__ __launch_bounds__(kBlock) void k_project_f32(acm_camera cam, size_t n,
                                                        const float* __restrict__ pts,
                                                        float* __restrict__ uv,
                                                        uint8_t* __restrict__ status,
                                                        float* __restrict__ jac) {
    using M = typename TagT::template type<float>;
    constexpr int P = M::P;
    const size_t i = (size_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    const Cam<float> c = make_cam<float>(cam);
    float x, y, z;
    if (LAYOUT == ACM_LAYOUT_AOS) {
        x = pts[3 * i]; y = pts[3 * i + 1]; z = pts[3 * i + 2];
    } else {
        x = pts[i]; y = pts[n + i]; z = pts[2 * n + i];
    }
    float u, v, ju[P], jv[P];
    const uint8_t st = M::template project<WJ>(c, x, y, z, u, v, ju, jv);
    const bool ok = st == ST_OK;
    auto put = [&](float* p, float a, float b) {
        flt2 val = {a, b};
        if (NT) __builtin_nontemporal_store(val, reinterpret_cast<flt2*>(p));
        else *reinterpret_cast<flt2*>(p) = val;
    };
    put(uv + 2 * i, ok ? u : __builtin_nanf(""), ok ? v : __builtin_nanf(""));
    status[i] = st;
    if (WJ) {
        const size_t col = 2 * n;
#pragma unroll
        for (int p = 0; p < P; ++p) put(jac + p * col + 2 * i, ok ? ju[p] : 0.0f, ok ? jv[p] : 0.0f);
    }
}

// ------------------------------------------ line-aligned Jacobian stores
// Column c of the 2N x P column-major Jacobian starts at byte 16*c*N.  Unless
// N is a multiple of 8, every wave's 1 KiB slice of a column straddles two
// 128-B lines that other workgroups (on other XCDs) complete at another
// time, and those partial-line writes cost HBM efficiency: the same traffic
// runs at 4.6-5.1 TB/s with 16/32-B-misaligned columns vs 6.7-7.2 TB/s
// aligned (tools/diag_align.py, profiles/r01_diag_align.log; the real kernel
// and a zero-compute mimic alike).  k_project_al makes every store window
// line-aligned whatever N and the buffer offsets are: workgroup b owns
// points [248b, 248b + 248) (lanes 0..247) and lanes 248..255 also project
// the 8 points before them.  A stream whose elements sit s (0..7) 16-B
// elements off the line grid is written by lane t as element 248b - s + t,
// so each 128-B line of it is written whole by one workgroup; the value
// comes from lane t - s, or from lead-in lane 256 - s + t for t < s, through
// LDS.  Streams already on the grid (s = 0) are stored straight from
// registers.  BASE_AL: uv / residual and J column 0 are on the grid (the
// buffers start on a 128-B line, as every torch / hipMalloc buffer does), so
// only columns 1..P-1 go through LDS (KB: 18.7 KB per workgroup, 8 per CU).
// The lead-in costs 3% extra math and 8 x 24 B of re-read per workgroup.
// Results are bit-identical to k_project / k_residual (same per-point code).
// Every model's J rows are u [a, 0, 1, 0, du..], v [0, b, 0, 1, dv..]
// (camera_models.hpp), so LDS holds a, b, validity and the D distortion
// pairs, not all 2P values.
// Each workgroup owns 256 points (lanes 0..7 also project one lead-in point
// each): window chunks of 256 keep each wave's 1 KiB column slices on the
// same 1 KiB grid as k_project (248-point windows measured 15% slower,
// profiles/r01_diag_align.log).
constexpr int kAlLead = 8;
constexpr int kAlOwn = kBlock;

__device__ __forceinline__ unsigned misalign16(const void* p, size_t elem_offset) {
    return (unsigned)(((reinterpret_cast<uintptr_t>(p) >> 4) + elem_offset) & 7u);
}

template <class TagT, int LAYOUT, bool RESID, bool BASE_AL>
__global__ __launch_bounds__(kBlock) void k_project_al(CamArg cam, size_t n,
                                                       const double* __restrict__ pts,
                                                       const double* __restrict__ obs,
                                                       int policy, double* __restrict__ out2,
                                                       uint8_t* __restrict__ status,
                                                       double* __restrict__ jac) {
    using M = typename TagT::template type<double>;
    constexpr int P = M::P;
    constexpr int D = P - 4;
    constexpr int S = kAlOwn + kAlLead;          // LDS slots: own points, then the lead-in
    constexpr int NW = BASE_AL ? 1 : S;       // s_uv / s_a only when they can be shifted
    __shared__ double2 s_uv[NW];
    __shared__ double s_a[NW];
    __shared__ double s_b[S];
    __shared__ double2 s_d[D > 0 ? D : 1][S];
    __shared__ uint8_t s_ok[S];
    const Cam<double> c = make_cam<double>(cam);
    const int t = threadIdx.x;
    const size_t base = (size_t)blockIdx.x * kAlOwn;
    auto eval = [&](size_t p, bool have, int slot, bool own) {
        double x = 0.0, y = 0.0, z = 1.0;
        // plain loads: non-temporal ones measured 25% slower here (the
        // lead-in re-read and the nt store stream, profiles/r01_ne_sweep.log)
        if (have) load_point<LAYOUT>(pts, n, p, x, y, z);
        double u, v, ju[P], jv[P];
        const uint8_t st = M::template project<true>(c, x, y, z, u, v, ju, jv);
        const bool ok = have && st == ST_OK;
        double2 w;
        if (RESID) {
            // the observations non-temporal (r05): DS at 9.29M 0.247 ->
            // 0.208 ms, KB -10% (profiles/r05aa_residual_obs_ntl.log); making
            // the point loads non-temporal too undoes most of it
            double2 o = make_double2(0.0, 0.0);
            if (have) o = ld2<true>(obs + 2 * p);
            const double sent = policy == ACM_INVALID_SENTINEL ? 1e6 : 0.0;
            w = make_double2(ok ? u - o.x : sent, ok ? v - o.y : sent);
        } else {
            w = make_double2(ok ? u : __builtin_nan(""), ok ? v : __builtin_nan(""));
        }
        const double a0 = ok ? ju[0] : 0.0;
        if (BASE_AL) {
            if (own && have) {
                st2<true>(out2 + 2 * p, w.x, w.y);
                st2<true>(jac + 2 * p, a0, 0.0);
            }
        } else {
            s_uv[slot] = w;
            s_a[slot] = a0;
        }
        s_b[slot] = ok ? jv[1] : 0.0;
        s_ok[slot] = ok;
#pragma unroll
        for (int k = 0; k < D; ++k)
            s_d[k][slot] = make_double2(ok ? ju[4 + k] : 0.0, ok ? jv[4 + k] : 0.0);
        if (status && own && have) st1<true>(status + p, st);
    };
    // lead-in point k (0..7) = base - 8 + k, in slot kAlOwn + k
    eval(base + t, base + t < n, t, true);
    if (t < kAlLead) eval(base + t - kAlLead, base >= (size_t)kAlLead, kAlOwn + t, false);
    __syncthreads();
    // element base - sh + t of a stream sitting sh elements off the line grid:
    // own point base + t - sh (slot t - sh) or lead-in slot S - sh + t
    size_t e;
    int j;
    auto elem = [&](unsigned sh) {
        j = t >= (int)sh ? t - (int)sh : S - (int)sh + t;
        e = base + t - sh;
        return base + t >= sh && e < n;
    };
    if (!BASE_AL && elem(misalign16(out2, 0))) st2<true>(out2 + 2 * e, s_uv[j].x, s_uv[j].y);
#pragma unroll
    for (int col = BASE_AL ? 1 : 0; col < P; ++col) {
        if (!elem(misalign16(jac, (size_t)col * n))) continue;
        double va, vb;
        if (col == 0) { va = s_a[j]; vb = 0.0; }
        else if (col == 1) { va = 0.0; vb = s_b[j]; }
        else if (col == 2) { va = s_ok[j] ? 1.0 : 0.0; vb = 0.0; }
        else if (col == 3) { va = 0.0; vb = s_ok[j] ? 1.0 : 0.0; }
        else { va = s_d[col - 4][j].x; vb = s_d[col - 4][j].y; }
        st2<true>(jac + (size_t)col * 2 * n + 2 * e, va, vb);
    }
}

// uv / residual and J column 0 on the 128-B grid (k_project_al<.., BASE_AL>)
static bool al_base_aligned(const void* out2, const double* jac) {
    return (reinterpret_cast<uintptr_t>(out2) & 127u) == 0 &&
           (reinterpret_cast<uintptr_t>(jac) & 127u) == 0;
}

// workgroups so that the last window [B*kAlOwn - s, ...) reaches n for every s <= 7
static unsigned al_blocks(size_t n) { return (unsigned)((n + kAlLead - 1 + kAlOwn) / kAlOwn); }

template <class TagT, int LAY, bool RESID>
static void launch_al(hipStream_t s, const CamArg& cam, size_t n, const double* pts,
                      const double* obs, int policy, double* out2, uint8_t* status,
                      double* jac) {
    auto kern = al_base_aligned(out2, jac) ? k_project_al<TagT, LAY, RESID, true>
                                           : k_project_al<TagT, LAY, RESID, false>;
    hipLaunchKernelGGL(kern, dim3(al_blocks(n)), dim3(kBlock), 0, s, cam, n, pts, obs, policy,
                       out2, status, jac);
}

// --------------------------------------------------------------- unproject
template <bool NT>
__device__ __forceinline__ void st1d(double* p, double v) {
    if (NT) __builtin_nontemporal_store(v, p);
    else *p = v;
}

// PPT pixels per lane: a workgroup owns PPT x 256 consecutive pixels, round
// r of lane t is pixel 256 r + t (every load and store instruction stays
// fully coalesced) and all PPT loads are issued before the first
// unprojection.  With one pixel per lane a 10M-pixel launch is 39K
// workgroups that each move only 10.5 KB: the closed-form models ran at the
// workgroup dispatch rate (~1.8 ns per workgroup, 5.7 TB/s for Pinhole).
// STG (AoS, rays 16-B aligned): a wave's 64 rays are 1536 contiguous bytes;
// they are staged in LDS and written as 96 16-B pieces (two store
// instructions per wave, every lane's address 16 B after its neighbour's)
// instead of three 8-B stores per lane at a 24-B stride.
template <class TagT, int LAYOUT, bool NT, bool NTL, int PPT, bool STG>
__global__ __launch_bounds__(kBlock) void k_unproject(CamArg cam, size_t n,
                                                      const double* __restrict__ uv,
                                                      double* __restrict__ rays,
                                                      uint8_t* __restrict__ status) {
    using M = typename TagT::template type<double>;
    const size_t i0 = (size_t)blockIdx.x * (kBlock * PPT) + threadIdx.x;
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const Cam<double> c = make_cam<double>(cam);
    __shared__ double s_ray[STG ? kBlock / 64 : 1][STG ? 64 * 3 : 1];
    double2 q[PPT];
#pragma unroll
    for (int r = 0; r < PPT; ++r) {
        const size_t i = i0 + (size_t)r * kBlock;
        q[r] = i < n ? ld2<NTL>(uv + 2 * i) : double2{0.0, 0.0};
    }
#pragma unroll
    for (int r = 0; r < PPT; ++r) {
        const size_t i = i0 + (size_t)r * kBlock;
        const size_t wfirst = i - (size_t)lane;  // the wave's first pixel this round
        if (wfirst >= n) break;                  // wave-uniform
        double X = 0.0, Y = 0.0, Z = 0.0;
        uint8_t st = ST_OK;
        if (i < n) {
            st = M::unproject(c, q[r].x, q[r].y, X, Y, Z);
            if (st != ST_OK) X = Y = Z = __builtin_nan("");
        }
        if (LAYOUT == ACM_LAYOUT_AOS) {
            if (STG && wfirst + 64 <= n) {  // whole wave in range
                double* sr = s_ray[STG ? wid : 0];
                sr[3 * lane] = X;
                sr[3 * lane + 1] = Y;
                sr[3 * lane + 2] = Z;
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                double* dst = rays + 3 * wfirst;
                st2<NT>(dst + 2 * lane, sr[2 * lane], sr[2 * lane + 1]);
                if (lane < 32) st2<NT>(dst + 128 + 2 * lane, sr[128 + 2 * lane], sr[129 + 2 * lane]);
                __builtin_amdgcn_wave_barrier();  // the next round rewrites sr
            } else if (i < n) {
                st1d<NT>(rays + 3 * i, X);
                st1d<NT>(rays + 3 * i + 1, Y);
                st1d<NT>(rays + 3 * i + 2, Z);
            }
        } else if (i < n) {
            st1d<NT>(rays + i, X);
            st1d<NT>(rays + n + i, Y);
            st1d<NT>(rays + 2 * n + i, Z);
        }
        if (i < n) st1<NT>(status + i, st);
    }
}

// Project -> unproject round trip in one pass (r04; BASELINE config 4, the
// reference's per-point loop of tests/projection_accuracy.rs over mod.rs:256
// and :271): each lane projects its points, stores the pixels and statuses
// exactly as k_project does (NaN pixels for failed projections), then
// unprojects those same pixel values from registers and stores rays and
// statuses exactly as k_unproject does -- the bits of acm_project followed by
// acm_unproject, without reading the 16 B per point of pixels back.
template <class TagT, int LAYOUT, bool NT, int PPT, bool STG>
__global__ __launch_bounds__(kBlock) void k_round_trip(CamArg cam, size_t n,
                                                       const double* __restrict__ pts,
                                                       double* __restrict__ uv,
                                                       uint8_t* __restrict__ pstatus,
                                                       double* __restrict__ rays,
                                                       uint8_t* __restrict__ rstatus) {
    using M = typename TagT::template type<double>;
    const size_t i0 = (size_t)blockIdx.x * (kBlock * PPT) + threadIdx.x;
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const Cam<double> c = make_cam<double>(cam);
    __shared__ double s_ray[STG ? kBlock / 64 : 1][STG ? 64 * 3 : 1];
    double px[PPT], py[PPT], pz[PPT];
#pragma unroll
    for (int r = 0; r < PPT; ++r) {
        const size_t i = i0 + (size_t)r * kBlock;
        px[r] = py[r] = 0.0;
        pz[r] = 1.0;
        if (i < n) load_point<LAYOUT>(pts, n, i, px[r], py[r], pz[r]);
    }
#pragma unroll
    for (int r = 0; r < PPT; ++r) {
        const size_t i = i0 + (size_t)r * kBlock;
        const size_t wfirst = i - (size_t)lane;
        if (wfirst >= n) break;  // wave-uniform
        double X = 0.0, Y = 0.0, Z = 0.0;
        uint8_t st = ST_OK;
        if (i < n) {
            double u, v;
            const uint8_t sp = M::template project<false>(c, px[r], py[r], pz[r], u, v, nullptr,
                                                          nullptr);
            if (sp != ST_OK) u = v = __builtin_nan("");
            st2<NT>(uv + 2 * i, u, v);
#ifndef ACM_AB_RT_NO_STATUS  // timing-only A/B build: the cost of the byte stores
            st1<NT>(pstatus + i, sp);
#endif
            // RadTan: the pixel is one its own project() kept (same bounds
            // test) or NaN, so the unprojection's bounds test is known false
            if constexpr (std::is_same<M, RadTan<double>>::value)
                st = M::template unproject<true>(c, u, v, X, Y, Z);
            else
                st = M::unproject(c, u, v, X, Y, Z);
            if (st != ST_OK) X = Y = Z = __builtin_nan("");
        }
        if (LAYOUT == ACM_LAYOUT_AOS) {
            if (STG && wfirst + 64 <= n) {  // whole wave in range
                double* sr = s_ray[STG ? wid : 0];
                sr[3 * lane] = X;
                sr[3 * lane + 1] = Y;
                sr[3 * lane + 2] = Z;
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                double* dst = rays + 3 * wfirst;
                st2<NT>(dst + 2 * lane, sr[2 * lane], sr[2 * lane + 1]);
                if (lane < 32) st2<NT>(dst + 128 + 2 * lane, sr[128 + 2 * lane], sr[129 + 2 * lane]);
                __builtin_amdgcn_wave_barrier();
            } else if (i < n) {
                st1d<NT>(rays + 3 * i, X);
                st1d<NT>(rays + 3 * i + 1, Y);
                st1d<NT>(rays + 3 * i + 2, Z);
            }
        } else if (i < n) {
            st1d<NT>(rays + i, X);
            st1d<NT>(rays + n + i, Y);
            st1d<NT>(rays + 2 * n + i, Z);
        }
#ifndef ACM_AB_RT_NO_STATUS
        if (i < n) st1<NT>(rstatus + i, st);
#endif
    }
}

// LDS-staged AoS ray stores by default for the models whose unprojection is
// memory-bound (Pinhole, DS, UCM, EUCM, FOV: 6.0-6.4 -> 6.4-7.2 TB/s at 10M
// pixels); the VALU-bound ones (KB, RadTan) lose 4-6% to the extra LDS and
// wave-barrier work (profiles/r02e_unproject_ppt.log).
template <class TagT> struct UnprojectStaged { static constexpr bool on = true; };
template <> struct UnprojectStaged<Tag<KannalaBrandt>> { static constexpr bool on = false; };
template <> struct UnprojectStaged<Tag<RadTan>> { static constexpr bool on = false; };

// acm_project_unproject's defaults per model: points per lane and whether
// the AoS rays go out LDS-staged (ACM_TUNE_ROUND_TRIP overrides both).
// From the r05 A/B at config 4's 50M points (tools/probes.py round_trip,
// profiles/r05d_round_trip_ab.log, best of 3 interleaved blocks): one point
// per lane for Pinhole / UCM / EUCM (0.565 -> 0.553 ms) and for KB, whose
// rays are now staged too (its VALU work fell with the SGPR-spill fix:
// 0.608 -> 0.587); RadTan keeps two, direct stores (every setting within
// 1.5%).  DS: four per lane until its projection's per-point camera
// constants moved to the host (r05), then two (0.590 -> 0.577 ms,
// profiles/r05u_ds_ppt.log).
template <class TagT> struct RoundTripDefault {
    static constexpr int ppt = 1;
    static constexpr bool staged = true;
};
template <> struct RoundTripDefault<Tag<DoubleSphere>> {
    static constexpr int ppt = 2;
    static constexpr bool staged = true;
};
template <> struct RoundTripDefault<Tag<RadTan>> {
    static constexpr int ppt = 2;
    static constexpr bool staged = false;
};
template <> struct RoundTripDefault<Tag<Fov>> {  // not measured: as acm_unproject
    static constexpr int ppt = 2;
    static constexpr bool staged = true;
};


// -------------------------------------------------- residual + Jacobian
template <class TagT, int LAYOUT, bool WJ, bool NT>
__global__ __launch_bounds__(kBlock) void k_residual(CamArg cam, size_t n,
                                                     const double* __restrict__ pts,
                                                     const double* __restrict__ obs,
                                                     int policy, double* __restrict__ res,
                                                     double* __restrict__ jac,
                                                     uint8_t* __restrict__ status) {
    using M = typename TagT::template type<double>;
    constexpr int P = M::P;
    const size_t i = (size_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    const Cam<double> c = make_cam<double>(cam);
    double x, y, z;
    load_point<LAYOUT>(pts, n, i, x, y, z);
    // non-temporal (r05): the residual alone at 9.29M 0.091 -> 0.084 ms
    // (profiles/r05ab_residual_noj.log)
    const double2 o = ld2<true>(obs + 2 * i);
    double u, v, ju[P], jv[P];
    const uint8_t st = M::template project<WJ>(c, x, y, z, u, v, ju, jv);
    const bool ok = st == ST_OK;
    const double sent = policy == ACM_INVALID_SENTINEL ? 1e6 : 0.0;
    st2<NT>(res + 2 * i, ok ? u - o.x : sent, ok ? v - o.y : sent);
    if (status) st1<NT>(status + i, st);
    if (WJ) {
        const size_t col = 2 * n;
#pragma unroll
        for (int p = 0; p < P; ++p) st2<NT>(jac + p * col + 2 * i, ok ? ju[p] : 0.0, ok ? jv[p] : 0.0);
    }
}

// -------------------------------------------------- wave / block reduction
__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
    return v;
}

// Reduce K per-lane values across the workgroup into out[0..K) (LDS staged).
// (r04) Wave reduce-scatter instead of K butterflies: KP - 1 + (6 - m)
// shuffles per lane instead of 6 K (DS: 34 vs 150, KB: 63 vs 240) at the end
// of every normal-equations workgroup; KB's call 0.084 -> 0.076 ms, DS at
// 9.29M 0.068 -> 0.065 ms (profiles/r04w_ne_reduce_scatter_ab.log).  Another
// summation order, fixed, so still bit-reproducible.
constexpr int pow2_at_least(int k) { return k <= 1 ? 1 : 2 * pow2_at_least((k + 1) / 2); }
constexpr int log2_exact(int k) { return k <= 1 ? 0 : 1 + log2_exact(k / 2); }
// out[k * ostride], k < K (the normal equations' partials are column-major:
// sum k of workgroup b at parts[k * nb + b], so k_ne_finish_cols reads each
// column coalesced)
template <int K>
__device__ __forceinline__ void block_sum_store(const double (&acc)[K], double* __restrict__ out,
                                                size_t ostride) {
    __shared__ double sm[kBlock / 64][K];
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    // wave reduce-scatter: with KP = 2^m >= K values per lane, each xor step
    // hands half of a lane's remaining values to its partner and adds the
    // half it keeps (KP - 1 shuffles in all instead of 6 K); lane l ends
    // with value l >> (6 - m) summed over 2^m lanes, and 6 - m plain xor
    // steps over the low lane bits finish the wave sum
    constexpr int KP = pow2_at_least(K) < 64 ? pow2_at_least(K) : 64;
    static_assert(K <= 64, "reduce-scatter over one wave");
    constexpr int m = log2_exact(KP);
    double v[KP];
#pragma unroll
    for (int k = 0; k < KP; ++k) v[k] = k < K ? acc[k] : 0.0;
#pragma unroll
    for (int st = 0; st < m; ++st) {
        const int h = KP >> (st + 1), o = 32 >> st;
        const bool up = (lane & o) != 0;
#pragma unroll
        for (int j = 0; j < h; ++j) {
            const double send = up ? v[j] : v[j + h];
            const double keep = up ? v[j + h] : v[j];
            v[j] = keep + __shfl_xor(send, o, 64);
        }
    }
    double t = v[0];
#pragma unroll
    for (int o = (32 >> m); o > 0; o >>= 1) t += __shfl_xor(t, o, 64);
    const int idx = lane >> (6 - m);
    if ((lane & ((1 << (6 - m)) - 1)) == 0 && idx < K) sm[wid][idx] = t;
    __syncthreads();
    for (int k = threadIdx.x; k < K; k += kBlock) {
        double s = 0.0;
#pragma unroll
        for (int w = 0; w < kBlock / 64; ++w) s += sm[w][k];
        out[(size_t)k * ostride] = s;
    }
}

// ---------------------------------------------------- normal equations
// Every model's Jacobian rows have the same structure (camera_models.hpp):
//   u-row [a, 0, 1, 0, du_0 .. du_{D-1}],  v-row [0, b, 0, 1, dv_0 .. dv_{D-1}]
// with D = P - 4 distortion parameters.  J^T J therefore has structural
// zeros ((fx,fy), (fx,cy), (fy,cx), (cx,cy)), (cx,cx) = (cy,cy) = n_valid,
// and J^T r has r0 / r1 sums for cx / cy.  Accumulating only the non-trivial
// sums (10 + 5D + D(D+1)/2 doubles per lane instead of P(P+1)/2 + P + 2)
// cuts both the FMAs and the accumulator registers; for finite values the
// sums are bit-identical to the dense ones (the dropped terms are exact 0).
// acc layout:
//   [0]        sum a^2        [1] sum a        [2, 2+D)      sum a du_k
//   [2+D]      sum b^2        [3+D] sum b      [4+D, 4+2D)   sum b dv_k
//   [4+2D, 4+3D) sum du_k     [4+3D, 4+4D)     sum dv_k
//   [4+4D, 4+4D+DD) sum du_j du_k + dv_j dv_k (j <= k, DD = D(D+1)/2)
//   then Jtr: sum a r0, sum b r1, sum r0, sum r1, sum du_k r0 + dv_k r1 (D)
//   then sum r.r, n_valid
template <int P>
struct NE {
    static constexpr int D = P - 4;
    static constexpr int DD = D * (D + 1) / 2;
    static constexpr int A_DU = 2, B2 = 2 + D, B1 = 3 + D, B_DV = 4 + D;
    static constexpr int DU = 4 + 2 * D, DV = 4 + 3 * D, DDB = 4 + 4 * D;
    static constexpr int G = DDB + DD;  // Jtr block
    static constexpr int K = G + 4 + D + 2;
};

// Per-model (waves, points per lane step) of k_normal_eq: the fastest cell of
// the interleaved {1,3,4} x {1, 2, 3 = one point two steps ahead} sweep with
// nt loads (tools/bench_configs.py --configs 3ne, profiles/r01s7_ne_sweep.log,
// 10M points).  All cells give the same sums up to summation order.
template <class TagT> struct NeDefault { static constexpr int W = 3, U = 1; };
template <> struct NeDefault<Tag<RadTan>> { static constexpr int W = 3, U = 2; };
template <> struct NeDefault<Tag<KannalaBrandt>> { static constexpr int W = 1, U = 3; };
template <> struct NeDefault<Tag<DoubleSphere>> { static constexpr int W = 1, U = 3; };
template <> struct NeDefault<Tag<Ucm>> { static constexpr int W = 3, U = 2; };
template <> struct NeDefault<Tag<Eucm>> { static constexpr int W = 3, U = 3; };
template <> struct NeDefault<Tag<Fov>> { static constexpr int W = 3, U = 3; };

constexpr int kNeMaxBlocks = 2048;  // reprojection stats / median partials
constexpr int kNqMaxBlocks = 2048;  // normal equations: 8 workgroups per CU

static int ne_blocks(size_t n) {
    size_t b = (n + kBlock - 1) / kBlock;
    if (b > (size_t)kNeMaxBlocks) b = kNeMaxBlocks;
    if (b == 0) b = 1;
    return (int)b;
}

static int nq_blocks(size_t n) {
    size_t b = (n + kBlock - 1) / kBlock;
    if (b > (size_t)kNqMaxBlocks) b = kNqMaxBlocks;
    if (b == 0) b = 1;
    return (int)b;
}

// Workgroups of `kernel` (kBlock lanes) that are resident on the whole
// device at once: occupancy per CU x CU count, cached per (kernel, device).
// Grid-stride reductions launch at most this many, so every workgroup starts
// in the first wave of dispatch -- a grid larger than the resident capacity
// leaves a second, partial round running alone at the end (a 2048-block
// launch of a 7-waves/SIMD kernel is 1.14 rounds).
static int resident_blocks(const void* kernel) {
    static std::mutex mu;
    static std::map<std::pair<const void*, int>, int> cache;
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return kNqMaxBlocks;
    std::lock_guard<std::mutex> lock(mu);
    auto it = cache.find({kernel, dev});
    if (it != cache.end()) return it->second;
    int per_cu = 0, cus = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kernel, kBlock, 0) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        per_cu <= 0 || cus <= 0) {
        (void)hipGetLastError();
        return kNqMaxBlocks;
    }
    const int r = per_cu * cus;
    cache[{kernel, dev}] = r;
    return r;
}

// Compute units of the current device (cached per device).
static int cu_count() {
    static std::mutex mu;
    static std::map<int, int> cache;
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return 256;
    std::lock_guard<std::mutex> lock(mu);
    auto it = cache.find(dev);
    if (it != cache.end()) return it->second;
    int cus = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        cus <= 0) {
        (void)hipGetLastError();
        return 256;
    }
    cache[dev] = cus;
    return cus;
}

// Per-lane running sums of the fused normal equations (k_normal_eq): NE<P>'s layout for every model but KB, whose 37 sums
// are built from powers of theta (below) and expanded to NE<8> at store().
// FAST projection (reciprocal instead of per-point divisions) and fused
// multiply-adds: the sums are held to 1e-10, not to the reference's
// operation order, and the validity mask stays exact (camera_models.hpp).
template <class TagT>
struct NeAccum {
    using M = typename TagT::template type<double>;
    static constexpr int P = M::P;
    using L = NE<P>;
    static constexpr int D = L::D;
    static constexpr int K = L::K;
    static constexpr bool kKB = std::is_same<TagT, Tag<KannalaBrandt>>::value;
    static constexpr int KA = kKB ? 37 : K;
    double acc[KA];

    __device__ __forceinline__ void init() {
#pragma unroll
        for (int k = 0; k < KA; ++k) acc[k] = 0.0;
    }

    __device__ __forceinline__ void add(const Cam<double>& c, double px, double py, double pz,
                                        double2 po, double sent2) {
        if constexpr (kKB) {
            // KB sums (37): [0] a^2 [1] a [2] b^2 [3] b, [4+k] a fxr T_k,
            // [8+k] b fyr T_k, [12+k] fxr T_k, [16+k] fyr T_k (T_k =
            // theta^(2k+3), k < 4), [20+m] (fxr^2 + fyr^2) theta^(6+2m)
            // (m < 7: every du_j du_k + dv_j dv_k with j + k = m), [27] a r0
            // [28] b r1 [29] r0 [30] r1, [31+k] (fxr r0 + fyr r1) T_k,
            // [35] r.r (or the sentinel), [36] n_valid
            double u, v, a, b, fxr, fyr, t2, t3;
            const uint8_t st = M::project_ne(c, px, py, pz, u, v, a, b, fxr, fyr, t2, t3);
            if (st == ST_OK) {
                const double r0 = u - po.x, r1 = v - po.y;
                acc[0] = fma(a, a, acc[0]);
                acc[1] += a;
                acc[2] = fma(b, b, acc[2]);
                acc[3] += b;
                const double afx = a * fxr, bfy = b * fyr, g = fma(fxr, r0, fyr * r1);
                double T = t3;
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    acc[4 + k] = fma(afx, T, acc[4 + k]);
                    acc[8 + k] = fma(bfy, T, acc[8 + k]);
                    acc[12 + k] = fma(fxr, T, acc[12 + k]);
                    acc[16 + k] = fma(fyr, T, acc[16 + k]);
                    acc[31 + k] = fma(g, T, acc[31 + k]);
                    T *= t2;
                }
                double q = fma(fxr, fxr, fyr * fyr) * (t3 * t3);
#pragma unroll
                for (int m = 0; m < 7; ++m) {
                    acc[20 + m] += q;
                    q *= t2;
                }
                acc[27] = fma(a, r0, acc[27]);
                acc[28] = fma(b, r1, acc[28]);
                acc[29] += r0;
                acc[30] += r1;
                acc[35] = fma(r0, r0, fma(r1, r1, acc[35]));
                acc[36] += 1.0;
            } else {
                acc[35] += sent2;
            }
        } else {
            double u, v, ju[P], jv[P];
            const uint8_t st = M::template project<true, true>(c, px, py, pz, u, v, ju, jv);
            if (st == ST_OK) {
                const double r0 = u - po.x, r1 = v - po.y;
                const double a = ju[0], b = jv[1];
                acc[0] = fma(a, a, acc[0]);
                acc[1] += a;
                acc[L::B2] = fma(b, b, acc[L::B2]);
                acc[L::B1] += b;
#pragma unroll
                for (int k = 0; k < D; ++k) {
                    acc[L::A_DU + k] = fma(a, ju[4 + k], acc[L::A_DU + k]);
                    acc[L::B_DV + k] = fma(b, jv[4 + k], acc[L::B_DV + k]);
                    acc[L::DU + k] += ju[4 + k];
                    acc[L::DV + k] += jv[4 + k];
                }
                int t = L::DDB;
#pragma unroll
                for (int j = 0; j < D; ++j) {
#pragma unroll
                    for (int k = j; k < D; ++k, ++t)
                        acc[t] = fma(ju[4 + j], ju[4 + k], fma(jv[4 + j], jv[4 + k], acc[t]));
                }
                acc[L::G + 0] = fma(a, r0, acc[L::G + 0]);
                acc[L::G + 1] = fma(b, r1, acc[L::G + 1]);
                acc[L::G + 2] += r0;
                acc[L::G + 3] += r1;
#pragma unroll
                for (int k = 0; k < D; ++k)
                    acc[L::G + 4 + k] = fma(ju[4 + k], r0, fma(jv[4 + k], r1, acc[L::G + 4 + k]));
                acc[K - 2] = fma(r0, r0, fma(r1, r1, acc[K - 2]));
                acc[K - 1] += 1.0;
            } else {
                acc[K - 2] += sent2;
            }
        }
    }

    // workgroup sum of the lanes' sums -> out[0..K) in NE<P>'s layout
    __device__ __forceinline__ void store(double* __restrict__ out, size_t ostride) const {
        if constexpr (kKB) {  // expand the 37 KB sums into the NE<8> layout
            static_assert(K == 40, "NE<8>");
            double full[K];
            full[0] = acc[0];
            full[1] = acc[1];
            full[L::B2] = acc[2];
            full[L::B1] = acc[3];
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                full[L::A_DU + k] = acc[4 + k];
                full[L::B_DV + k] = acc[8 + k];
                full[L::DU + k] = acc[12 + k];
                full[L::DV + k] = acc[16 + k];
                full[L::G + 4 + k] = acc[31 + k];
            }
            int t = L::DDB;
#pragma unroll
            for (int j = 0; j < 4; ++j)
#pragma unroll
                for (int k = j; k < 4; ++k, ++t) full[t] = acc[20 + j + k];
            full[L::G + 0] = acc[27];
            full[L::G + 1] = acc[28];
            full[L::G + 2] = acc[29];
            full[L::G + 3] = acc[30];
            full[K - 2] = acc[35];
            full[K - 1] = acc[36];
            block_sum_store<K>(full, out, ostride);
        } else {
            block_sum_store<K>(acc, out, ostride);
        }
    }
};

// Observation streams of k_normal_eq (r06).  ObsPixels: the caller's 2 x N
// pixels (16 B per point).  ObsCells: grid-sampled correspondences given by
// their cell index (4 B per point; acm_sample_points_cells): the pixel is
// the cell centre, recomputed exactly as sample_points wrote it --
// ((j + 0.5) * cw, (i + 0.5) * ch), point_sampling.rs:66-70 -- so the sums
// are the pixel form's bit for bit with 12 B per point fewer to read.
struct ObsPixels {
    const double* p;
    using raw = double2;
    template <bool NTL>
    __device__ __forceinline__ raw load(size_t i) const { return ld2<NTL>(p + 2 * i); }
    __device__ __forceinline__ double2 get(raw r) const { return r; }
    __device__ __forceinline__ static raw zero() { return make_double2(0.0, 0.0); }
};
struct ObsCells {
    const uint32_t* p;
    uint32_t ncx;
    double inv_ncx, cw, ch;  // RN(1 / ncx); width / ncx, height / ncy
    using raw = uint32_t;
    template <bool NTL>
    __device__ __forceinline__ raw load(size_t i) const {
        if (NTL) return __builtin_nontemporal_load(p + i);
        return p[i];
    }
    // c = i ncx + j: the f64 quotient is within 2^-52 (relative) of c / ncx
    // (c, ncx < 2^32), so its truncation is i, or i - 1 when c / ncx is an
    // integer approached from below -- one correction
    __device__ __forceinline__ double2 get(uint32_t c) const {
        uint32_t i = (uint32_t)((double)c * inv_ncx);
        uint32_t j = c - i * ncx;
        if (j >= ncx) {
            ++i;
            j -= ncx;
        }
        return make_double2(((double)j + 0.5) * cw, ((double)i + 0.5) * ch);
    }
    __device__ __forceinline__ static raw zero() { return 0u; }
};

// WAVES: minimum waves per SIMD the register allocator must allow
// (amdgpu_waves_per_eu).  1 leaves it free (KB lands at 176 VGPRs = 2 waves);
// 3 fits KB in 168 without spills; 4 forces 128 with scratch spills for KB and
// RadTan.  Selected per launch by ACM_TUNE_NE_WAVES (results identical).
template <class TagT, int LAYOUT, int U, bool NTL, class OBS>
__device__ __forceinline__ void normal_eq_body(const acm_camera& cam, size_t n,
                                               const double* __restrict__ pts, OBS obs,
                                               int policy, double* __restrict__ parts) {
    using ORaw = typename OBS::raw;
    using Acc = NeAccum<TagT>;
    constexpr int K = Acc::K;
    const Cam<double> c = make_cam<double>(cam);
    Acc sums;
    sums.init();
    const double sent2 = policy == ACM_INVALID_SENTINEL ? 2e12 : 0.0;
    const size_t stride = (size_t)gridDim.x * kBlock;
    size_t i = (size_t)blockIdx.x * kBlock + threadIdx.x;
    // Software pipeline: the next U points' 40 bytes each are in flight while
    // the current U are projected and accumulated (U points per lane step,
    // ACM_TUNE_NE_UNROLL).  Not for the largest accumulator sets (KB,
    // RadTan), where the extra registers cost a wave of occupancy.
    constexpr bool kPrefetch = K <= 40;
    auto accumulate = [&](double px, double py, double pz, ORaw po) {
        sums.add(c, px, py, pz, obs.get(po), sent2);
    };
    if constexpr (U >= 3) {
        // one point per lane step, loads issued A = U - 1 steps ahead (A
        // times the bytes in flight of U = 1 for 5(A-1) more registers).  The
        // A slots are unrolled, not rotated through register moves: a move of
        // a register with a load in flight makes the compiler wait for every
        // load (vmcnt(0)) at the top of each step, which left one step of
        // latency hiding whatever A was; with static slots each wait is the
        // counted vmcnt of the slot's own load.
        constexpr int A = U - 1;
        double xs[A], ys[A], zs[A];
        ORaw os[A];
        // branch-free loads (past the end: point n - 1 again, never
        // accumulated): with loads under exec branches the compiler cannot
        // count them and waits vmcnt(0)
        auto load_slot = [&](int q, size_t iq) {
            const size_t ic = iq < n ? iq : n - 1;
            load_point<LAYOUT, NTL>(pts, n, ic, xs[q], ys[q], zs[q]);
            os[q] = obs.template load<NTL>(ic);
        };
        if (n) {  // (n = 0: nothing to load, the loop below does not run)
#pragma unroll
            for (int q = 0; q < A; ++q) load_slot(q, i + (size_t)q * stride);
        }
        for (; i < n; i += (size_t)A * stride) {
#pragma unroll
            for (int q = 0; q < A; ++q) {
                const size_t iq = i + (size_t)q * stride;
                if (iq < n) accumulate(xs[q], ys[q], zs[q], os[q]);
                load_slot(q, iq + (size_t)A * stride);
            }
        }
    } else if constexpr (U == 1) {
        double x = 0, y = 0, z = 1;
        ORaw o = OBS::zero();
        if (kPrefetch && i < n) {
            load_point<LAYOUT, NTL>(pts, n, i, x, y, z);
            o = obs.template load<NTL>(i);
        }
        for (; i < n; i += stride) {
            const size_t inext = i + stride;
            double xn = 0, yn = 0, zn = 1;
            ORaw on = OBS::zero();
            if (kPrefetch) {
                if (inext < n) {
                    load_point<LAYOUT, NTL>(pts, n, inext, xn, yn, zn);
                    on = obs.template load<NTL>(inext);
                }
            } else {
                load_point<LAYOUT, NTL>(pts, n, i, x, y, z);
                o = obs.template load<NTL>(i);
            }
            accumulate(x, y, z, o);
            if (kPrefetch) { x = xn; y = yn; z = zn; o = on; }
        }
    } else {
        // each wave streams contiguous chunks of U x 64 points (loads in
        // flight a grid stride apart cost DRAM locality, tools/hbm_ceiling.py)
        double x[U], y[U], z[U], xn[U], yn[U], zn[U];
        ORaw o[U], on[U];
        const int lane = threadIdx.x & 63;
        const size_t nw = (size_t)gridDim.x * (kBlock / 64);
        constexpr size_t C = (size_t)U * 64;
        auto load = [&](size_t base, double (&xs)[U], double (&ys)[U], double (&zs)[U],
                        ORaw (&os)[U]) {
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const size_t j = base + (size_t)u * 64 + lane;
                xs[u] = 0.0; ys[u] = 0.0; zs[u] = 1.0;
                os[u] = OBS::zero();
                if (j < n) {
                    load_point<LAYOUT, NTL>(pts, n, j, xs[u], ys[u], zs[u]);
                    os[u] = obs.template load<NTL>(j);
                }
            }
        };
        size_t b0 = ((size_t)blockIdx.x * (kBlock / 64) + (threadIdx.x >> 6)) * C;
        if (kPrefetch) load(b0, x, y, z, o);
        for (; b0 < n; b0 += nw * C) {
            if (kPrefetch) load(b0 + nw * C, xn, yn, zn, on);
            else load(b0, x, y, z, o);
#pragma unroll
            for (int u = 0; u < U; ++u)
                if (b0 + (size_t)u * 64 + lane < n) accumulate(x[u], y[u], z[u], o[u]);
            if (kPrefetch) {
#pragma unroll
                for (int u = 0; u < U; ++u) { x[u] = xn[u]; y[u] = yn[u]; z[u] = zn[u]; o[u] = on[u]; }
            }
        }
    }
    sums.store(parts + blockIdx.x, gridDim.x);
}
template <class TagT, int LAYOUT, int WAVES, int U, bool NTL, class OBS = ObsPixels>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(WAVES))) void k_normal_eq(acm_camera cam, size_t n,
                                                      const double* __restrict__ pts,
                                                      OBS obs, int policy,
                                                      double* __restrict__ parts) {
    normal_eq_body<TagT, LAYOUT, U, NTL, OBS>(cam, n, pts, obs, policy, parts);
}
// (r06) The LM's pre-queued evaluation (solver.hip, ACM_TUNE_LM_HOST_RESULT
// 3): queued while the previous evaluation runs, it waits for the host's
// doorbell (lm_doorbell.hpp) and reads the camera the doorbell delivered.
// The same body, so the same sums; a cancelled evaluation computes nothing.
template <class TagT, int LAYOUT, int WAVES, int U, bool NTL, class OBS = ObsPixels>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(WAVES))) void k_normal_eq_dev(
        LmDoorbell db, size_t n, const double* __restrict__ pts, OBS obs, int policy,
        double* __restrict__ parts) {
    if (!lm_doorbell_wait(db)) return;
    const acm_camera cam = lm_doorbell_camera(db.cam);
    normal_eq_body<TagT, LAYOUT, U, NTL, OBS>(cam, n, pts, obs, policy, parts);
}

// Epilogue of k_normal_eq: sum the per-workgroup partials (nb x K,
// row-major) and expand the structured sums -> [JtJ full (P*P) | Jtr (P) |
// 0.5*rr | n_valid].  Spread over the chip (r03): workgroup k < K sums
// column k -- lane l takes rows l, l + 256, ... in order, then the wave
// butterfly and the four waves in order, a fixed order so the result is
// bit-reproducible -- and writes every output entry that is that sum (JtJ
// is symmetric: up to two entries per sum; n_valid fills (cx, cx), (cy, cy)
// and the last slot); workgroup K writes the structural zeros.  The
// round-2 epilogue, one 1024-lane workgroup reading all nb x K partials,
// took 6.5-7 us per evaluation (profiles/r03z_fp64_kernel_stats.csv); this
// one cut the KB call 81.7 -> 78.7 us and DS's 74.8 -> 71.7 us
// (profiles/r03u_ne_finish_ab_*.log).
// ne_out_src(t): the sum output entry t comes from (-1: a structural zero)
template <int P>
__device__ __forceinline__ int ne_out_src(int t) {
    using L = NE<P>;
    constexpr int D = L::D, K = L::K;
    if (t < P * P) {
        const int r = t / P, c = t % P;
        const int i = r < c ? r : c, j = r < c ? c : r;
        if (j >= 4) {
            const int kj = j - 4;
            if (i == 0) return L::A_DU + kj;
            if (i == 1) return L::B_DV + kj;
            if (i == 2) return L::DU + kj;
            if (i == 3) return L::DV + kj;
            const int ki = i - 4;  // upper triangle, row-major from (ki, ki)
            return L::DDB + ki * D - ki * (ki - 1) / 2 + (kj - ki);
        }
        if (i == 0 && j == 0) return 0;
        if (i == 0 && j == 2) return 1;
        if (i == 1 && j == 1) return L::B2;
        if (i == 1 && j == 3) return L::B1;
        if (i == j) return K - 1;  // (2, 2), (3, 3): n_valid
        return -1;
    }
    if (t < P * P + P) return L::G + (t - P * P);
    if (t == P * P + P) return K - 2;  // 0.5 * r.r
    return K - 1;                      // n_valid
}

// SYS (the LM's host-polled path): each workgroup's results are made
// visible at system scope before it ends; then the workgroups take a ticket
// and the last one releases the host's completion word (flag = seq) and
// re-arms the ticket (ticket == nullptr: a k_ne_publish follows instead).
template <int P, bool SYS>
__global__ __launch_bounds__(kBlock) void k_ne_finish_cols(const double* __restrict__ parts, int nb,
                                                           double* __restrict__ out,
                                                           unsigned int* __restrict__ ticket,
                                                           unsigned long long* __restrict__ flag,
                                                           unsigned long long seq) {
    using L = NE<P>;
    constexpr int K = L::K, NOUT = P * P + P + 2;
    const int k = blockIdx.x;
    __shared__ double sm[kBlock / 64];
    __shared__ double s_sum;
    if (k < K) {
        double a = 0.0;
        for (int b = threadIdx.x; b < nb; b += kBlock) a += parts[(size_t)k * nb + b];
        a = wave_sum(a);
        if ((threadIdx.x & 63) == 0) sm[threadIdx.x >> 6] = a;
        __syncthreads();
        if (threadIdx.x == 0) {
            double t = 0.0;
            for (int w = 0; w < kBlock / 64; ++w) t += sm[w];
            s_sum = t;
        }
        __syncthreads();
        const double S = s_sum;
        for (int t = threadIdx.x; t < NOUT; t += kBlock)
            if (ne_out_src<P>(t) == k) out[t] = t == P * P + P ? 0.5 * S : S;
    } else {
        for (int t = threadIdx.x; t < NOUT; t += kBlock)
            if (ne_out_src<P>(t) < 0) out[t] = 0.0;
    }
    if (SYS) {
        __threadfence_system();
        if (ticket) {  // the last workgroup releases the host's completion word
            __syncthreads();
            if (threadIdx.x == 0) {
                const unsigned t = __hip_atomic_fetch_add(ticket, 1u, __ATOMIC_ACQ_REL,
                                                          __HIP_MEMORY_SCOPE_AGENT);
                if (t == gridDim.x - 1) {
                    __hip_atomic_store(ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    __hip_atomic_store(flag, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
                }
            }
        }
    }
}

// The LM's host-polled path after k_ne_finish_cols: every result is out
// (stream order), publish `seq` with a system-scope release.
__global__ void k_ne_publish(unsigned long long* __restrict__ flag, unsigned long long seq) {
    __threadfence_system();
    __hip_atomic_store(flag, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// ----------------------------------------------------- reprojection stats
// One streaming pass.  The variance is not a second pass over the errors
// (error_metrics.rs:92 sums (e - mean)^2 after the mean): each lane keeps
// shifted sums S = sum (e - K), Q = sum (e - K)^2 about its first valid error
// K, i.e. (count, mean, M2) of its own errors without cancellation (K is a
// sample of the same distribution), and the lanes / waves / workgroups are
// merged in a fixed order with Chan's pairwise update
//   M2 = M2_a + M2_b + d^2 n_a n_b / n,   d = mean_b - mean_a,
// which equals the two-pass sum of squared deviations up to rounding (the
// reference's own sums are in a different order anyway).  This drops the
// 8 B/point re-read of the errors and three small launches.
struct Mv {
    double n, m, M2;
};

__device__ __forceinline__ Mv mv_merge(const Mv& a, const Mv& b) {
    if (a.n == 0.0) return b;
    if (b.n == 0.0) return a;
    const double n = a.n + b.n;
    const double d = b.m - a.m;
    return Mv{n, a.m + d * (b.n / n), a.M2 + b.M2 + d * d * (a.n * (b.n / n))};
}

__device__ __forceinline__ Mv mv_wave(Mv a) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        const Mv b{__shfl_xor(a.n, off, 64), __shfl_xor(a.m, off, 64), __shfl_xor(a.M2, off, 64)};
        a = mv_merge(a, b);
    }
    return a;
}

constexpr int kReprojW = 7;  // per-workgroup [sum e, sum e^2, min, max, count, mean, M2]

// [sum, sumsq, min, max, count] + (count, mean, M2) of a wave -> lane 0's
// values -> sm[wid]; then lane 0 of the workgroup merges the waves in order
__device__ __forceinline__ void reproj_block_store(double s, double ss, double mn, double mx,
                                                   Mv v, double* __restrict__ out) {
    __shared__ double sm[kBlock / 64][kReprojW];
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    s = wave_sum(s);
    ss = wave_sum(ss);
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        mn = fmin(mn, __shfl_xor(mn, off, 64));
        mx = fmax(mx, __shfl_xor(mx, off, 64));
    }
    v = mv_wave(v);
    if (lane == 0) {
        sm[wid][0] = s; sm[wid][1] = ss; sm[wid][2] = mn; sm[wid][3] = mx;
        sm[wid][4] = v.n; sm[wid][5] = v.m; sm[wid][6] = v.M2;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        double a = 0, b = 0, m0 = INFINITY, m1 = -INFINITY;
        Mv t{0.0, 0.0, 0.0};
        for (int w = 0; w < kBlock / 64; ++w) {
            a += sm[w][0]; b += sm[w][1]; m0 = fmin(m0, sm[w][2]); m1 = fmax(m1, sm[w][3]);
            t = mv_merge(t, Mv{sm[w][4], sm[w][5], sm[w][6]});
        }
        out[0] = a; out[1] = b; out[2] = m0; out[3] = m1; out[4] = t.n; out[5] = t.m;
        out[6] = t.M2;
    }
}

// The median's radix digits (see "median" below): 11 bits, 2048 bins.
constexpr int kSelBits = 11, kSelBins = 1 << kSelBits;

// One LDS histogram increment per lane with pred, aggregated across the wave
// when AGG: lanes holding the same digit add their count with one atomic
// (pass 0's digits are the exponent: a wave's 64 values share a handful of
// them, and 64 same-address LDS atomics would serialise).
template <bool AGG>
__device__ __forceinline__ void sel_count(unsigned int* h, bool pred, unsigned d) {
    if (!AGG) {
        if (pred) atomicAdd(&h[d], 1u);
        return;
    }
    unsigned long long act = __ballot(pred);
    const int lane = threadIdx.x & 63;
    while (act) {
        const int leader = __ffsll((long long)act) - 1;
        const unsigned dl = (unsigned)__shfl((int)d, leader, 64);
        const unsigned long long same = __ballot(pred && d == dl) & act;
        if (lane == leader) atomicAdd(&h[dl], (unsigned)__popcll(same));
        act &= ~same;
    }
}

// e_i = ||proj(p_i) - uv_i|| (NaN if the projection fails); per-workgroup
// partials (kReprojW doubles).  NTS: non-temporal error stores.  Software
// pipelined like k_normal_eq (r04): one point per lane step, the loads of the
// next kReprojA = 6 steps in flight in static slots, branch-free (past the
// end: point n - 1 again, never used).  compute_reprojection_error at 92.9M
// (profiles/r04m_*, r04n_*, same box, interleaved): 2 slots 1.271 ms, 4
// slots 1.198 / 1.203, 6 slots 1.179, 8 slots 1.179 (126 VGPRs); each
// workgroup streaming one contiguous range instead of the grid stride
// 1.251 (2 slots) / 1.269 (4 slots); plain instead of non-temporal error
// stores 1.287.  The round-3 form (2 points per lane per chunk, no
// prefetch) ran the pass at 4.96 TB/s (profiles/r04j_convert_kernel_stats.csv).
// HIST (acm_reprojection_error): the median's first radix-select histogram
// (the 11-bit digit of bits 53..63 of every error, NaN included, exactly
// k_sel_hist's pass 0) is counted here in LDS and written per workgroup to
// hparts (2048 u32), which saves the median one full read of the errors.
constexpr int kReprojA = 6;

// One lane's reprojection statistics: [sum, sumsq, min, max, count] and the
// shifted sums about its first valid error (see the comment above Mv).
struct ReprojAcc {
    double s = 0.0, ss = 0.0, mn = INFINITY, mx = -INFINITY, cnt = 0.0;
    double K = 0.0, S = 0.0, Q = 0.0;
    // One validity rule for the statistics and the median: an Ok projection
    // whose error is NaN (a NaN observation) is not a valid error --
    // acm_median_valid skips NaN too.  (The reference would sum the NaN and
    // then panic in its median sort, error_metrics.rs:104-108
    // partial_cmp().unwrap().)
    __device__ __forceinline__ void add(double e) {
        if (e == e) {
            s += e;
            ss += e * e;
            mn = fmin(mn, e);
            mx = fmax(mx, e);
            K = cnt == 0.0 ? e : K;
            const double d = e - K;
            S += d;
            Q += d * d;
            cnt += 1.0;
        }
    }
    // workgroup partials (kReprojW doubles); every lane of the workgroup calls it
    __device__ __forceinline__ void store(double* __restrict__ out) const {
        const double mloc = cnt > 0.0 ? S / cnt : 0.0;
        const Mv v{cnt, K + mloc, cnt > 0.0 ? Q - S * mloc : 0.0};
        reproj_block_store(s, ss, mn, mx, v, out);
    }
};

// e = ||proj(p) - o||, NaN if the projection fails (error_metrics.rs:70-84)
template <class M>
__device__ __forceinline__ double reproj_error(const Cam<double>& c, double x, double y, double z,
                                               double2 o) {
    double u, v;
    const uint8_t st = M::template project<false>(c, x, y, z, u, v, nullptr, nullptr);
    if (st != ST_OK) return __builtin_nan("");
    const double du = u - o.x, dv = v - o.y;
    return sqrt_rn(du * du + dv * dv);
}

// the median's pass-0 digit of an error (bits 53..63, k_sel_hist's pass 0)
__device__ __forceinline__ unsigned sel_digit0(double e) {
    return (unsigned)(((unsigned long long)__double_as_longlong(e) >> 53) & (kSelBins - 1));
}

template <class TagT, int LAYOUT, bool NTL, bool NTS, bool HIST, class OBS = ObsPixels>
__global__ __launch_bounds__(kBlock) void k_reproj_pass1(acm_camera cam, size_t n,
                                                         const double* __restrict__ pts,
                                                         OBS obs,
                                                         double* __restrict__ errs,
                                                         double* __restrict__ parts,
                                                         unsigned int* __restrict__ hparts) {
    using M = typename TagT::template type<double>;
    constexpr int HB = kSelBins;
    __shared__ unsigned int h[HIST ? HB : 1];
    if constexpr (HIST) {
        for (int j = threadIdx.x; j < HB; j += kBlock) h[j] = 0;
        __syncthreads();
    }
    const Cam<double> c = make_cam<double>(cam);
    ReprojAcc acc;
    const size_t stride = (size_t)gridDim.x * kBlock;
    size_t i = (size_t)blockIdx.x * kBlock + threadIdx.x;
    constexpr int A = kReprojA;
    double xs[A], ys[A], zs[A];
    typename OBS::raw os[A];
    auto load_slot = [&](int q, size_t iq) {
        const size_t ic = iq < n ? iq : n - 1;
        load_point<LAYOUT, NTL>(pts, n, ic, xs[q], ys[q], zs[q]);
        os[q] = obs.template load<NTL>(ic);
    };
    if (n) {
#pragma unroll
        for (int q = 0; q < A; ++q) load_slot(q, i + (size_t)q * stride);
    }
    for (; i < n; i += (size_t)A * stride) {
#pragma unroll
        for (int q = 0; q < A; ++q) {
            const size_t iq = i + (size_t)q * stride;
            const bool in = iq < n;
            double e = __builtin_nan("");
            if (in) {
                e = reproj_error<M>(c, xs[q], ys[q], zs[q], obs.get(os[q]));
                acc.add(e);
                if (NTS) __builtin_nontemporal_store(e, errs + iq);
                else errs[iq] = e;
            }
            if constexpr (HIST) sel_count<true>(h, in, sel_digit0(e));
            load_slot(q, iq + (size_t)A * stride);
        }
    }
    acc.store(parts + (size_t)blockIdx.x * kReprojW);
    if constexpr (HIST) {
        __syncthreads();
        unsigned int* hp = hparts + (size_t)blockIdx.x * HB;
        for (int j = threadIdx.x; j < HB; j += kBlock) hp[j] = h[j];
    }
}

// The same per-workgroup partials from a given error vector (NaN = invalid):
// the statistics of a shard whose errors already sit in HBM
// (acm_error_stats, distributed.combine_reprojection_stats).
__global__ __launch_bounds__(kBlock) void k_errstats_pass1(size_t n,
                                                           const double* __restrict__ errs,
                                                           double* __restrict__ parts) {
    double s = 0.0, ss = 0.0, mn = INFINITY, mx = -INFINITY, cnt = 0.0;
    double K = 0.0, S = 0.0, Q = 0.0;
    const size_t stride = (size_t)gridDim.x * kBlock;
    for (size_t i = (size_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += stride) {
        const double e = errs[i];
        if (e == e) {
            s += e;
            ss += e * e;
            mn = fmin(mn, e);
            mx = fmax(mx, e);
            K = cnt == 0.0 ? e : K;
            const double d = e - K;
            S += d;
            Q += d * d;
            cnt += 1.0;
        }
    }
    const double mloc = cnt > 0.0 ? S / cnt : 0.0;
    const Mv v{cnt, K + mloc, cnt > 0.0 ? Q - S * mloc : 0.0};
    reproj_block_store(s, ss, mn, mx, v, parts + (size_t)blockIdx.x * kReprojW);
}

// The median's selection state and workspace (acm_median_workspace_size):
// [SelState x 2 | hist 2 x kSelBins f64 | candidate count u64 (+ 8 B) |
// candidates].  Defined with the median below.
struct SelState;
struct SelWs {
    SelState* st;
    double* hist;
    unsigned long long* count;
    double* cbuf;
};
__device__ void sel_init_wg(const SelWs& w, unsigned long long m);

// Fixed-order finish of the statistics partials, one workgroup:
// tot = [sum, sumsq, min, max, count, mean, M2], then (r05: one launch
// instead of two) result = [rmse, min, max, mean, stddev, n_valid, sum,
// sumsq]; with sel.st != nullptr also the median's initial state for
// n_valid = count (what k_sel_init would do after it, a third launch).
__global__ __launch_bounds__(kBlock) void k_reproj_finish(const double* __restrict__ parts,
                                                          int nb, double* __restrict__ tot,
                                                          double* __restrict__ out, SelWs sel) {
    double s = 0, ss = 0, mn = INFINITY, mx = -INFINITY;
    Mv v{0.0, 0.0, 0.0};
    for (int b = threadIdx.x; b < nb; b += kBlock) {
        const double* p = parts + (size_t)b * kReprojW;
        s += p[0]; ss += p[1]; mn = fmin(mn, p[2]); mx = fmax(mx, p[3]);
        v = mv_merge(v, Mv{p[4], p[5], p[6]});
    }
    reproj_block_store(s, ss, mn, mx, v, tot);  // thread 0 writes tot
    __shared__ double s_nn;
    if (threadIdx.x == 0) {  // its own writes: no fence needed
        const double nn = tot[4];
        const double mean = tot[0] / nn;  // error_metrics.rs:88-89: sum / n
        out[0] = sqrt(tot[1] / nn);
        out[1] = tot[2];
        out[2] = tot[3];
        out[3] = mean;
        out[4] = sqrt(fmax(tot[6], 0.0) / nn);
        out[5] = nn;
        out[6] = tot[0];
        out[7] = tot[1];
        s_nn = nn;
    }
    if (sel.st) {
        __syncthreads();
        sel_init_wg(sel, (unsigned long long)s_nn);
    }
}

// ------------------------------------------------------------ sample_points
// point_sampling.rs:56-103.  Cell c = i*ncx + j (row-major like the
// reference's nested loop).  Two passes with the unprojection recomputed in
// the second (cheaper than a 40 B/cell scratch round trip through HBM):
//   1. per-workgroup keep counts, 2. exclusive scan of the counts (one
//   workgroup), 3. keep -> rank inside the workgroup (wave ballot + LDS
//   prefix over the 4 waves) -> ordered scatter.
struct Grid {
    uint32_t ncx, ncy;
    double cw, ch;
    size_t cell0;  // first cell of this launch (row-range shards, see acm_sample_points_range)
    int patience;  // look-back polls before counting a predecessor's cells itself
};

// 64-bit value known to be wave-uniform, moved to SGPRs (so arithmetic on
// it runs on the scalar unit).
__device__ __forceinline__ uint64_t uniform64(uint64_t x) {
    return ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(x >> 32)) << 32) |
           (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)x);
}

// Row/column of a cell, advanced incrementally.  init() divides the
// workgroup-uniform first cell of a tile once, on the scalar unit, and each
// lane adds its offset (< kBlock) with a wrap; each step of kBlock cells is
// an add and (for ncx >= kBlock) at most one wrap.  A per-lane 64-bit
// division and remainder is a ~60-instruction VALU sequence: done per lane
// at the start of every tile's compute and store passes it cost ~30 VALU
// instructions per 64 cells.
struct CellWalk {
    uint32_t i, j;
    __device__ __forceinline__ void init(const Grid& g, uint64_t base, uint32_t off) {
        const uint64_t cb = uniform64(base + g.cell0);
        const uint64_t i0 = cb / g.ncx;
        i = (uint32_t)i0;
        j = (uint32_t)(cb - i0 * g.ncx) + off;
        while (j >= g.ncx) { j -= g.ncx; ++i; }
    }
    __device__ __forceinline__ void step(const Grid& g) { step_by<kBlock>(g); }
    template <uint32_t S>
    __device__ __forceinline__ void step_by(const Grid& g) {
        j += S;
        while (j >= g.ncx) { j -= g.ncx; ++i; }
    }
};

template <class TagT>
__device__ __forceinline__ bool sample_cell(const Cam<double>& c, const Grid& g, const CellWalk& w,
                                            double& u, double& v, double& X, double& Y,
                                            double& Z) {
    using M = typename TagT::template type<double>;
    u = ((double)w.j + 0.5) * g.cw;  // :69
    v = ((double)w.i + 0.5) * g.ch;  // :70
    if constexpr (SampleTag<TagT>::kb) {
        // the keep decision taken exactly on the reference's theta, not read
        // off the polynomial-cos ray (KannalaBrandt::unproject_k)
        bool keep;
        const uint8_t st =
                M::template unproject_k<true, SampleTag<TagT>::poly>(c, u, v, X, Y, Z, keep);
        return st == ST_OK && keep;  // :91-94
    } else {
        const uint8_t st = M::unproject(c, u, v, X, Y, Z);
        return st == ST_OK && Z > 0.0;  // :91-94
    }
}

// The count pass only needs keep = (status Ok && Z > 0).  For Pinhole that
// is decidable without the ray: its only status is the image bounds
// (pinhole.rs:229-235) and Z = 1 / sqrt(1 + r2) (:240-245) is > 0 exactly
// when 1 + r2 is finite (sqrt >= 1 then; inf gives Z = 0, NaN fails), with
// mx, my the same correctly rounded quotients -- so the pass skips the
// square root, the division and the ray.
template <class TagT>
__device__ __forceinline__ bool sample_keep(const Cam<double>& c, const Grid& g,
                                            const CellWalk& w) {
    double u, v, X, Y, Z;
    return sample_cell<TagT>(c, g, w, u, v, X, Y, Z);
}
template <>
__device__ __forceinline__ bool sample_keep<Tag<Pinhole>>(const Cam<double>& c, const Grid& g,
                                                          const CellWalk& w) {
    const double u = ((double)w.j + 0.5) * g.cw;  // :69
    const double v = ((double)w.i + 0.5) * g.ch;  // :70
    const bool out = u < 0.0 || u >= c.w || v < 0.0 || v >= c.h;
    const double mx = div_by_f(u - c.p[2], c.p[0], c.ifx);
    const double my = div_by_f(v - c.p[3], c.p[1], c.ify);
    const double r2 = mx * mx + my * my;
    return !out && 1.0 + r2 < INFINITY;
}

// Each workgroup owns kSampleCells consecutive cells (kSampleR rounds of 256):
// few enough workgroups that the scan of their counts is a handful of
// coalesced tiles, and round r of lane t is cell base + 256 r + t, so the
// write pass emits kept points in cell order.
constexpr int kSampleR = 16;
constexpr size_t kSampleCells = (size_t)kBlock * kSampleR;

template <class TagT>
__global__ __launch_bounds__(kBlock) void k_sample_count(CamArg cam, Grid g, size_t cells,
                                                         uint64_t* __restrict__ counts) {
    const Cam<double> c = sample_cam<TagT>(cam);
    const size_t base = (size_t)blockIdx.x * kSampleCells;
    uint32_t mine = 0;
    CellWalk cw;
    cw.init(g, base, threadIdx.x);
    for (int r = 0; r < kSampleR; ++r, cw.step(g)) {
        const size_t cell = base + (size_t)r * kBlock + threadIdx.x;
        if (cell < cells) mine += sample_keep<TagT>(c, g, cw) ? 1u : 0u;
    }
    __shared__ uint32_t sm[kBlock / 64];
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) mine += __shfl_xor(mine, off, 64);
    if ((threadIdx.x & 63) == 0) sm[threadIdx.x >> 6] = mine;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint64_t t = 0;
        for (int w = 0; w < kBlock / 64; ++w) t += sm[w];
        counts[blockIdx.x] = t;
    }
}

// Exclusive scan of nb workgroup counts by one workgroup of 1024 lanes, in
// coalesced tiles of 1024 (wave shuffle scan + a 16-entry LDS scan per tile).
__global__ __launch_bounds__(1024) void k_scan_counts(const uint64_t* __restrict__ counts,
                                                      size_t nb, uint64_t* __restrict__ offsets,
                                                      uint64_t* __restrict__ out_counts,
                                                      uint64_t cells) {
    __shared__ uint64_t wsum[16];
    const int t = threadIdx.x, lane = t & 63, wid = t >> 6;
    uint64_t carry = 0;
    for (size_t tile = 0; tile < nb; tile += 1024) {
        const size_t b = tile + t;
        const uint64_t c = b < nb ? counts[b] : 0;
        uint64_t x = c;  // inclusive wave scan
#pragma unroll
        for (int off = 1; off < 64; off <<= 1) {
            const uint64_t y = __shfl_up(x, off, 64);
            if (lane >= off) x += y;
        }
        if (lane == 63) wsum[wid] = x;
        __syncthreads();
        uint64_t before = 0, total = 0;
        for (int w = 0; w < 16; ++w) {
            if (w < wid) before += wsum[w];
            total += wsum[w];
        }
        if (b < nb) offsets[b] = carry + before + x - c;
        carry += total;
        __syncthreads();
    }
    if (t == 0) {
        out_counts[0] = carry;
        out_counts[1] = cells;
    }
}

template <class TagT>
__global__ __launch_bounds__(kBlock) void k_sample_write(CamArg cam, Grid g, size_t cells,
                                                         const uint64_t* __restrict__ offsets,
                                                         double* __restrict__ uv_out,
                                                         double* __restrict__ xyz_out) {
    const Cam<double> c = sample_cam<TagT>(cam);
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    __shared__ uint32_t sm[kBlock / 64];
    const size_t base = (size_t)blockIdx.x * kSampleCells;
    uint64_t run = offsets[blockIdx.x];
    CellWalk cw;
    cw.init(g, base, threadIdx.x);
    for (int r = 0; r < kSampleR; ++r, cw.step(g)) {
        const size_t cell = base + (size_t)r * kBlock + threadIdx.x;
        bool keep = false;
        double u = 0, v = 0, X = 0, Y = 0, Z = 0;
        if (cell < cells) keep = sample_cell<TagT>(c, g, cw, u, v, X, Y, Z);
        const uint64_t m = __ballot(keep);
        if (lane == 0) sm[wid] = (uint32_t)__popcll(m);
        __syncthreads();
        uint64_t wbase = run, tot = 0;
        for (int w = 0; w < kBlock / 64; ++w) {
            if (w < wid) wbase += sm[w];
            tot += sm[w];
        }
        const uint64_t below = lane ? (m & ((~0ull) >> (64 - lane))) : 0ull;
        if (keep) {
            const size_t k = wbase + (uint64_t)__popcll(below);
            st2<false>(uv_out + 2 * k, u, v);
            xyz_out[3 * k] = X;
            xyz_out[3 * k + 1] = Y;
            xyz_out[3 * k + 2] = Z;
        }
        run += tot;
        __syncthreads();  // sm is rewritten next round
    }
}

// ------------------------------------------- segment two-pass (r03, default)
// The grid is cut into segments of 64 consecutive cells (one wave, one cell
// per lane).  Pass 1 (k_seg_count) gives every segment its kept count; pass 2
// scans the per-workgroup sums (k_scan_counts); pass 3 (k_seg_write)
// recomputes each segment and writes its kept points at known offsets.  No
// look-back and no cross-wave synchronisation in the write pass: a wave owns
// whole segments, compacts its kept rays in 1.5 KiB of its own LDS and writes
// them as 16-B pieces.  Segments with nothing kept are skipped outright.
//
// The count pass mostly needs no unprojection at all: every model's keep
// decision depends on the cell only through r2 = mx^2 + my^2 (KB through
// ru = min(sqrt(r2), pi/2)), so a segment whose r2 interval lies inside a
// region certified on the host (seg_cert) is counted from its geometry --
// ALL cells kept or NONE.  Only segments that straddle the boundary of the
// kept region (a thin ring: ~1-3% of the segments) run the per-cell keep.
constexpr int kSegCells = 64;
constexpr int kSegPerBlock = kBlock;  // segments per count / write workgroup
constexpr size_t kSegBlockCells = (size_t)kSegCells * kSegPerBlock;

enum : int { SEG_UNKNOWN = 0, SEG_ALL = 1, SEG_NONE = 2 };

// Keep certificates.  KB: host-certified regions in ru = min(sqrt(r2), pi/2)
// (kb_seg_cert): every cell whose ru lies in [all_lo, all_hi] is kept, none
// in [none_lo, none_hi].  Pinhole, FOV, DS, UCM, EUCM: on = 1 and the
// segment's r2 interval is pushed through the model's closed form in
// interval arithmetic on the device (seg_keep_iv).  RadTan, or on = 0
// (ACM_TUNE_SAMPLE_CERT = 0): every segment is decided cell by cell.
struct SegCert {
    int on;
    int ig_ok;  // KB: ig[] fits theta*(ru) on [0, all_hi] for ray_certified: its Newton steps (1, 2) or 0
    int rp_ok;  // KB: rp[] holds ray_certified's polynomials (kb_fit_ray)
    double all_lo, all_hi, none_lo, none_hi;
    double ig[9];  // KB: theta*(ru) ~= ru * sum ig[i] ru^(2i)
    double rp[2 * kRayPolyN];  // KB: cos theta*, sin theta* / ru ~= sum rp[i] r2^i, sum rp[N + i] r2^i
    // KB: M = cmax / (2 dmin) of the Newton analysis, ef = the bound on
    // |theta_ref - theta*| (the reference's final iterate vs the root, which
    // the certified rays use), and the bound on the ray polynomials' error
    // (kb_ray_poly_bound)
    double M, ef, rp_err, ig_err;  // ig_err: the bound on the initial guess (kb_guess_bound)
};

// Rigorous bounds of r2 = mx^2 + my^2 over the cells [c0, c1] (inclusive,
// launch-local) as the kernels compute them (mx = RN(RN(u - cx) / fx)
// etc.), widened far beyond their few-ulp rounding; false when any cell may
// lie outside the image (the unprojections' bounds test).
__device__ __forceinline__ bool seg_r2_bounds(const Cam<double>& c, const Grid& g, uint64_t c0,
                                              uint64_t c1, double& lo, double& hi) {
    const uint64_t a = c0 + g.cell0, b = c1 + g.cell0;
    const uint64_t i0 = a / g.ncx, i1 = b / g.ncx;
    uint64_t j0 = a - i0 * g.ncx, j1 = b - i1 * g.ncx;
    if (i0 != i1) {  // several rows: every column may occur
        j0 = 0;
        j1 = g.ncx - 1;
    }
    const double ulo = ((double)j0 + 0.5) * g.cw, uhi = ((double)j1 + 0.5) * g.cw;
    const double vlo = ((double)i0 + 0.5) * g.ch, vhi = ((double)i1 + 0.5) * g.ch;
    const bool inb = ulo >= 0.0 && vlo >= 0.0 && uhi < c.w * (1.0 - 0x1p-40) &&
                     vhi < c.h * (1.0 - 0x1p-40);
    // |m| over an interval of u (m monotone in u): [0 if the interval
    // straddles cx, else min |end|] .. max |end|, plus rounding slack
    auto mrange = [](double l, double h, double cc, double f, double& mlo, double& mhi) {
        const double e0 = (l - cc) / f, e1 = (h - cc) / f;
        const double slack = (fabs(l) + fabs(h) + fabs(cc)) * 0x1p-44 / fabs(f) + 0x1p-1000;
        const double a0 = fabs(e0), a1 = fabs(e1);
        const bool straddle = (e0 <= 0.0) != (e1 <= 0.0);
        mlo = fmax((straddle ? 0.0 : fmin(a0, a1)) * (1.0 - 0x1p-40) - slack, 0.0);
        mhi = fmax(a0, a1) * (1.0 + 0x1p-40) + slack;
    };
    double xlo, xhi, ylo, yhi;
    mrange(ulo, uhi, c.p[2], c.p[0], xlo, xhi);
    mrange(vlo, vhi, c.p[3], c.p[1], ylo, yhi);
    lo = (xlo * xlo + ylo * ylo) * (1.0 - 0x1p-40);
    hi = (xhi * xhi + yhi * yhi) * (1.0 + 0x1p-40);
    return inb && lo == lo && hi == hi;
}

// Interval arithmetic for the segment certificates: every operation returns
// an enclosure of its exact result widened by 2^-40 of the operands'
// magnitude (plus 2^-1000 absolute).  That covers the operation's own
// rounding and, by induction, the few-ulp rounding of the same expression
// evaluated per cell in double: every double the kernels compute for a cell
// whose r2 lies in the input interval lies inside the result.  A NaN
// anywhere (sqrt of a possibly negative value, 0 in a divisor) is reported
// as `nan` and the segment is left to the cells.
struct Iv {
    double lo, hi;
    bool nan;
};
__device__ __forceinline__ Iv iv_mk(double lo, double hi, double mag, bool nan) {
    const double e = mag * 0x1p-40 + 0x1p-1000;
    return Iv{lo - e, hi + e, nan || !(lo == lo) || !(hi == hi)};
}
__device__ __forceinline__ Iv iv_c(double x) { return Iv{x, x, !(x == x)}; }
__device__ __forceinline__ Iv operator+(Iv a, Iv b) {
    return iv_mk(a.lo + b.lo, a.hi + b.hi, fmax(fabs(a.lo), fabs(a.hi)) + fmax(fabs(b.lo), fabs(b.hi)),
                 a.nan || b.nan);
}
__device__ __forceinline__ Iv operator-(Iv a, Iv b) {
    return iv_mk(a.lo - b.hi, a.hi - b.lo, fmax(fabs(a.lo), fabs(a.hi)) + fmax(fabs(b.lo), fabs(b.hi)),
                 a.nan || b.nan);
}
__device__ __forceinline__ Iv operator*(Iv a, Iv b) {
    const double p0 = a.lo * b.lo, p1 = a.lo * b.hi, p2 = a.hi * b.lo, p3 = a.hi * b.hi;
    const double lo = fmin(fmin(p0, p1), fmin(p2, p3)), hi = fmax(fmax(p0, p1), fmax(p2, p3));
    return iv_mk(lo, hi, fmax(fabs(lo), fabs(hi)), a.nan || b.nan);
}
__device__ __forceinline__ Iv operator/(Iv a, Iv b) {
    if (!(b.lo > 0.0 || b.hi < 0.0)) return Iv{-INFINITY, INFINITY, true};
    const double p0 = a.lo / b.lo, p1 = a.lo / b.hi, p2 = a.hi / b.lo, p3 = a.hi / b.hi;
    const double lo = fmin(fmin(p0, p1), fmin(p2, p3)), hi = fmax(fmax(p0, p1), fmax(p2, p3));
    return iv_mk(lo, hi, fmax(fabs(lo), fabs(hi)), a.nan || b.nan);
}
__device__ __forceinline__ Iv iv_sqrt(Iv a) {
    if (!(a.lo >= 0.0)) return Iv{0.0, sqrt(fmax(a.hi, 0.0)) * 2.0 + 1.0, true};
    const double lo = sqrt(a.lo), hi = sqrt(a.hi);
    return iv_mk(lo, hi, hi, a.nan);
}
__device__ __forceinline__ Iv iv_sq(Iv a) {  // a * a, >= 0
    const double m = fmax(fabs(a.lo), fabs(a.hi));
    const double n = (a.lo <= 0.0 && a.hi >= 0.0) ? 0.0 : fmin(fabs(a.lo), fabs(a.hi));
    return iv_mk(n * n, m * m, m * m, a.nan);
}

// keep = status Ok && z > 0 && |p| finite, from the r2 interval of a segment.
// The closed forms follow the unprojections in camera_models.hpp operation
// by operation (double_sphere.rs:436-476, ucm.rs:337-367, eucm.rs:368-398).
__device__ __forceinline__ int seg_from(bool fail_all, bool fail_none, Iv z, Iv n2) {
    if (fail_all || (!z.nan && z.hi < 0.0)) return SEG_NONE;
    if (fail_none && !z.nan && !n2.nan && z.lo > 0.0 && n2.hi < 1e300) return SEG_ALL;
    return SEG_UNKNOWN;
}

template <class TagT>
__device__ __forceinline__ int seg_keep_iv(const Cam<double>& c, const SegCert& k, double r2lo,
                                           double r2hi) {
    return SEG_UNKNOWN;  // RadTan: Newton in (x, y), not a function of r2 alone
}
template <>
__device__ __forceinline__ int seg_keep_iv<Tag<KannalaBrandt>>(const Cam<double>& c,
                                                               const SegCert& k, double lo,
                                                               double hi) {
    // the host certificate, in ru = min(sqrt(r2), pi/2) (:462-467)
    constexpr double kHalfPi = kPi / 2.0;
    const double qlo = fmin(sqrt(lo) * (1.0 - 0x1p-40), kHalfPi);
    const double qhi = fmin(sqrt(hi) * (1.0 + 0x1p-40), kHalfPi);
    if (qlo >= k.all_lo && qhi <= k.all_hi) return SEG_ALL;
    if (qlo >= k.none_lo && qhi <= k.none_hi) return SEG_NONE;
    return SEG_UNKNOWN;
}
template <>
__device__ __forceinline__ int seg_keep_iv<Tag<Pinhole>>(const Cam<double>& c, const SegCert& k,
                                                         double lo, double hi) {
    // pinhole.rs:228-246: in the image (checked by the caller) and Z =
    // 1 / sqrt(1 + r2) > 0, i.e. 1 + r2 finite
    return hi < 1e300 ? SEG_ALL : SEG_UNKNOWN;
}
template <>
__device__ __forceinline__ int seg_keep_iv<Tag<Fov>>(const Cam<double>& c, const SegCert& k,
                                                     double lo, double hi) {
    // fov.rs:336-363: always Ok, z = 1 / |p| > 0 while |p| is finite, and
    // p = (m * sin(rd w) / (rd 2 tan(w/2))) / cos(rd w) stays finite while
    // rd w <= 0.99 pi/2 (cos(rd w) >= 0.0157) and r2 is moderate
    const double wf = c.p[4];
    if (!(wf > 0.0 && wf < INFINITY) || !(c.p[8] > 0.0)) return SEG_UNKNOWN;
    const double lim = 0.99 * (kPi / 2.0) / wf;
    return hi < lim * lim * (1.0 - 0x1p-30) && hi < 1e100 ? SEG_ALL : SEG_UNKNOWN;
}
template <>
__device__ __forceinline__ int seg_keep_iv<Tag<DoubleSphere>>(const Cam<double>& c,
                                                              const SegCert& k, double lo,
                                                              double hi) {
    const double alpha = c.p[4], xi = c.p[5];
    const Iv r2{lo, hi, false};
    // reject = alpha != 0 && alpha > 0.5 && r2 > 1 / (2 alpha - 1) (uk[0])
    const bool rej_on = alpha != 0.0 && alpha > 0.5;
    const bool rej_all = rej_on && lo > c.uk[0], rej_none = !rej_on || hi <= c.uk[0];
    const Iv a = iv_c(alpha), one = iv_c(1.0);
    const Iv mz = (one - a * a * r2) / (a * iv_sqrt(one - (iv_c(2.0) * a - one) * r2) +
                                        iv_c(1.0 - alpha));
    const Iv mz2 = iv_sq(mz);
    const Iv num = mz * iv_c(xi) + iv_sqrt(mz2 + (one - iv_c(xi) * iv_c(xi)) * r2);
    const Iv den = mz2 + r2;
    const Iv coeff = num / den;
    const Iv pz = coeff * mz - iv_c(xi);
    const Iv n2 = iv_sq(coeff) * r2 + iv_sq(pz);
    const bool den_fail_all = !den.nan && den.hi < 1e-3, den_fail_none = !den.nan && den.lo >= 1e-3;
    return seg_from(rej_all || den_fail_all, rej_none && den_fail_none, pz, n2);
}
template <>
__device__ __forceinline__ int seg_keep_iv<Tag<Ucm>>(const Cam<double>& c, const SegCert& k,
                                                     double lo, double hi) {
    const double alpha = c.p[4], xi = c.uk[0], gamma = 1.0 - alpha;
    // mx, my are scaled by gamma (ucm.rs:346-347): r2 = gamma^2 (mx0^2 + my0^2)
    const Iv r2 = iv_c(gamma * gamma) * Iv{lo, hi, false};
    const Iv one = iv_c(1.0);
    const Iv num = iv_c(xi) + iv_sqrt(one + (one - iv_c(xi) * iv_c(xi)) * r2);
    const Iv den = one - r2;  // the reference's 1 - r^2 (:354)
    const bool cond_on = alpha > 0.5;
    const bool cond_all_fail = cond_on && !r2.nan && r2.lo > c.uk[1] * (1.0 + 0x1p-30);
    const bool cond_none_fail = !cond_on || (!r2.nan && r2.hi <= c.uk[1] * (1.0 - 0x1p-30));
    const Iv coeff = num / den;
    const Iv pz = coeff - iv_c(xi);
    const Iv n2 = iv_sq(coeff) * r2 + iv_sq(pz);
    const bool den_fail_all = !den.nan && den.hi < 1e-3, den_fail_none = !den.nan && den.lo >= 1e-3;
    return seg_from(cond_all_fail || den_fail_all, cond_none_fail && den_fail_none, pz, n2);
}
template <>
__device__ __forceinline__ int seg_keep_iv<Tag<Eucm>>(const Cam<double>& c, const SegCert& k,
                                                      double lo, double hi) {
    const double alpha = c.p[4], beta = c.p[5];
    const Iv r2{lo, hi, false};
    const Iv one = iv_c(1.0), a = iv_c(alpha), b = iv_c(beta);
    const Iv num = one - r2 * a * a * b;
    const Iv det = one - (a - iv_c(1.0 - alpha)) * b * r2;
    const Iv den = iv_c(1.0 - alpha) + a * iv_sqrt(det);
    // cond = !(alpha > 0.5 && r2 > uk[0]) (eucm.rs:196, precedence quirk kept)
    const bool cond_on = alpha > 0.5;
    const bool cond_all_fail = cond_on && lo > c.uk[0], cond_none_fail = !cond_on || hi <= c.uk[0];
    const Iv mz = num / den;
    const Iv n2 = r2 + iv_sq(mz);
    const bool det_fail_all = !det.nan && det.hi < 1e-3, det_fail_none = !det.nan && det.lo >= 1e-3;
    return seg_from(cond_all_fail || det_fail_all, cond_none_fail && det_fail_none, mz, n2);
}

template <class TagT>
__device__ __forceinline__ int seg_classify(const Cam<double>& c, const Grid& g, const SegCert& k,
                                            uint64_t c0, uint64_t c1) {
    if (!k.on) return SEG_UNKNOWN;
    double lo, hi;
    if (!seg_r2_bounds(c, g, c0, c1, lo, hi)) return SEG_UNKNOWN;
    return seg_keep_iv<TagT>(c, k, lo, hi);
}

template <class TagT>
__global__ __launch_bounds__(kBlock) void k_seg_count(CamArg cam, Grid g, size_t cells, SegCert cert,
                                                      uint32_t* __restrict__ seg_cnt,
                                                      uint64_t* __restrict__ blk_sum) {
    const Cam<double> c = make_cam<double>(cam);
    const int lane = threadIdx.x & 63;
    const uint64_t nseg = (cells + kSegCells - 1) / kSegCells;
    const uint64_t seg = (uint64_t)blockIdx.x * kSegPerBlock + threadIdx.x;
    const uint64_t wseg0 = seg - lane;  // the wave's first segment
    uint32_t cnt = 0;
    int cls = SEG_NONE;
    if (seg < nseg) {
        const uint64_t c0 = seg * kSegCells;
        const uint64_t c1 = c0 + kSegCells <= cells ? c0 + kSegCells - 1 : cells - 1;
        cls = seg_classify<TagT>(c, g, cert, c0, c1);
        if (cls == SEG_ALL) cnt = (uint32_t)(c1 - c0 + 1);
    }
    // segments the geometry cannot decide: the whole wave counts their cells
    uint64_t unk = __ballot(cls == SEG_UNKNOWN);
    while (unk) {
        const int k = __builtin_amdgcn_readfirstlane(__ffsll((long long)unk) - 1);
        unk &= unk - 1;
        const uint64_t base = (wseg0 + (uint64_t)k) * kSegCells;
        CellWalk cw;
        cw.init(g, base, lane);
        const bool keep = base + lane < cells && sample_keep<TagT>(c, g, cw);
        const uint32_t kc = (uint32_t)__popcll(__ballot(keep));
        if (lane == k) cnt = kc;
    }
    if (seg < nseg) seg_cnt[seg] = cnt;
    __shared__ uint32_t sm[kBlock / 64];
    uint32_t t = cnt;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) t += __shfl_xor(t, off, 64);
    if (lane == 0) sm[threadIdx.x >> 6] = t;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint64_t tot = 0;
        for (int w = 0; w < kBlock / 64; ++w) tot += sm[w];
        blk_sum[blockIdx.x] = tot;
    }
}

// Write pass.  Workgroup b covers kSegBlockW = 4 * SPW segments; its 256
// lanes first turn the counts of the whole count block the segments sit in
// (256 segments, 1 KiB) into exclusive offsets in LDS (wave scan + the 4
// wave totals + the scanned block offset), then each wave writes SPW of the
// segments -- interleaved (ILV: wave w takes segments w, w + 4, ..., so the
// four waves of a workgroup write adjacent runs at the same time) or
// contiguous.  Per segment: the 64 cells are unprojected, the kept lanes
// ballot their rank, each writes its 16-B pixel at offset + rank, and the
// compacted rays (3 * kept doubles, staged in the wave's 1.5 KiB of LDS) go
// out as 16-B pieces.  A segment whose count is 0 is skipped.
//
// FIX (the repair pass of the speculative path, k_seg_spec): the segments
// were already written at their speculative offsets (64 x segment); rewrite
// only those whose true offset differs and that keep something -- none at
// all when nothing was dropped (total == cells).
template <class TagT, int SPW, bool ILV, bool NT = false, bool FIX = false>
// (r04) at least 6 waves per SIMD: the KB form (polynomial rays) drops from
// 88 to 80 VGPRs without spills and writes 1e8 cells 3.5% faster (0.763 vs
// 0.790 ms interleaved; 8 waves spill and gain 1.5%; the other models
// already fit; profiles/r04t_seg_write_waves_ab.log)
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(6))) void k_seg_write(CamArg cam, Grid g, size_t cells,
                                                      const uint32_t* __restrict__ seg_cnt,
                                                      const uint64_t* __restrict__ blk_off,
                                                      double* __restrict__ uv_out,
                                                      double* __restrict__ xyz_out,
                                                      const uint64_t* __restrict__ total,
                                                      uint32_t* __restrict__ cells_out) {
    static_assert(kSegPerBlock % (4 * SPW) == 0, "write workgroups tile the count blocks");
    if constexpr (FIX) {
        if (total[0] == (uint64_t)cells) return;  // every cell kept: all in place
        // segments before this workgroup's count block all full: its
        // segments' speculative offsets are right up to its first partial one
        // -- the scan below decides per segment
    }
    const Cam<double> c = sample_cam<TagT>(cam);
    const int lane = threadIdx.x & 63;
    const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint64_t nseg = (cells + kSegCells - 1) / kSegCells;
    const uint64_t wseg0 = (uint64_t)blockIdx.x * (4 * SPW);    // this workgroup's first segment
    const uint64_t cb = wseg0 / kSegPerBlock;                     // its count block
    __shared__ uint64_t s_off[kSegPerBlock];
    __shared__ uint32_t s_cnt[kSegPerBlock];
    __shared__ uint32_t s_wsum[kBlock / 64];
    __shared__ double s_ray[kBlock / 64][64 * 3];
    {
        const uint64_t sg = cb * kSegPerBlock + threadIdx.x;
        const uint32_t cnt = sg < nseg ? seg_cnt[sg] : 0u;
        uint32_t x = cnt;
#pragma unroll
        for (int off = 1; off < 64; off <<= 1) {
            const uint32_t y = __shfl_up(x, off, 64);
            if (lane >= off) x += y;
        }
        if (lane == 63) s_wsum[wid] = x;
        __syncthreads();
        uint64_t o = blk_off[cb];
        for (int w = 0; w < wid; ++w) o += s_wsum[w];
        s_off[threadIdx.x] = o + (x - cnt);
        s_cnt[threadIdx.x] = cnt;
        __syncthreads();
    }
    const uint64_t below = lane ? ((~0ull) >> (64 - lane)) : 0ull;
    double* lx = s_ray[wid];
    // the wave's cells, walked incrementally (one scalar division per wave:
    // a 64-bit division per segment cost more SALU time than Pinhole's math)
    constexpr uint32_t kStep = ILV ? 4 * kSegCells : kSegCells;
    const int li0 = (int)(wseg0 - cb * kSegPerBlock) + (ILV ? wid : SPW * wid);
    CellWalk cw;
    cw.init(g, (cb * kSegPerBlock + (uint64_t)li0) * kSegCells, lane);
#pragma unroll 1
    for (int k = 0; k < SPW; ++k, cw.template step_by<kStep>(g)) {
        const int li = li0 + (ILV ? 4 * k : k);
        const uint64_t sg = cb * kSegPerBlock + (uint64_t)li;
        if (sg >= nseg) break;
        const uint32_t sc = __builtin_amdgcn_readfirstlane(s_cnt[li]);
        if (sc == 0) continue;  // nothing kept here (certified or counted)
        const uint64_t off = uniform64(s_off[li]);
        if (FIX && off == sg * kSegCells) continue;  // already in place
        const uint64_t cell = sg * kSegCells + lane;
        double u = 0.0, v = 0.0, X = 0.0, Y = 0.0, Z = 0.0;
        bool keep = false;
        if (cell < cells) keep = sample_cell<TagT>(c, g, cw, u, v, X, Y, Z);
        const uint64_t m = __ballot(keep);
        const uint32_t rank = (uint32_t)__popcll(m & below);
        if (keep) {
            st2<NT>(uv_out + 2 * (off + rank), u, v);  // 16 B per lane, one run per wave
            if (cells_out) cells_out[off + rank] = cw.i * g.ncx + cw.j;  // (r06) the cell form
            double* d = lx + 3 * rank;
            d[0] = X;
            d[1] = Y;
            d[2] = Z;
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        // the kept rays: 3 * kc consecutive doubles of xyz_out, as 16-B pieces
        // on the 16-B grid (+ a single leading / trailing double)
        const uint32_t kc = (uint32_t)__popcll(m);
        double* dst = xyz_out + 3 * off;
        const uint32_t nd = 3 * kc;
        const uint32_t h = (uint32_t)((reinterpret_cast<uintptr_t>(dst) >> 3) & 1u);
        const uint32_t np = (nd - h) >> 1;
        for (uint32_t p = lane; p < np; p += 64) {
            const uint32_t dd = h + 2 * p;
            st2<NT>(dst + dd, lx[dd], lx[dd + 1]);
        }
        if (lane == 0 && h) dst[0] = lx[0];
        if (lane == 63 && ((nd - h) & 1u)) dst[nd - 1] = lx[nd - 1];
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
}

// Speculative segment path (ACM_TUNE_SAMPLE_FUSED = 4; auto for RadTan,
// which has no keep certificate, so a count pass would run its Newton loop
// for every cell).  One pass unprojects every segment once and writes its
// kept points compacted within the segment's own speculative range [64 s,
// 64 s + count) -- the final place whenever no cell before it was dropped
// (the output buffers hold every cell of the range, acm.h) -- and records
// the per-segment and per-count-block counts.  k_scan_counts then gives the
// true offsets and the total, and k_seg_write<FIX> recomputes and rewrites
// only the segments whose true offset differs.  Grids that keep every cell
// (RadTan's sample camera) cost one unprojection pass plus two tiny
// launches; a grid whose first drop comes early pays the write pass again
// over the segments after it.  Outputs are bit-identical to every other
// path (the same per-cell function, the same order).
template <class TagT>
__global__ __launch_bounds__(kBlock) void k_seg_spec(CamArg cam, Grid g, size_t cells,
                                                     uint32_t* __restrict__ seg_cnt,
                                                     uint64_t* __restrict__ blk_sum,
                                                     double* __restrict__ uv_out,
                                                     double* __restrict__ xyz_out,
                                                     uint32_t* __restrict__ cells_out) {
    // one workgroup per count block (256 segments), wave w takes segments
    // w, w + 4, ... so the four waves write adjacent runs at the same time
    constexpr int SPW = kSegPerBlock / 4;
    const Cam<double> c = sample_cam<TagT>(cam);
    const int lane = threadIdx.x & 63;
    const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint64_t nseg = (cells + kSegCells - 1) / kSegCells;
    const uint64_t seg0 = (uint64_t)blockIdx.x * kSegPerBlock;
    __shared__ double s_ray[kBlock / 64][64 * 3];
    __shared__ uint32_t s_wsum[kBlock / 64];
    const uint64_t below = lane ? ((~0ull) >> (64 - lane)) : 0ull;
    double* lx = s_ray[wid];
    constexpr uint32_t kStep = 4 * kSegCells;
    CellWalk cw;
    cw.init(g, (seg0 + (uint64_t)wid) * kSegCells, lane);
    uint32_t wsum = 0;
#pragma unroll 1
    for (int k = 0; k < SPW; ++k, cw.template step_by<kStep>(g)) {
        const uint64_t sg = seg0 + (uint64_t)(wid + 4 * k);
        if (sg >= nseg) break;
        const uint64_t cell = sg * kSegCells + lane;
        double u = 0.0, v = 0.0, X = 0.0, Y = 0.0, Z = 0.0;
        bool keep = false;
        if (cell < cells) keep = sample_cell<TagT>(c, g, cw, u, v, X, Y, Z);
        const uint64_t m = __ballot(keep);
        const uint32_t kc = (uint32_t)__popcll(m);
        if (lane == 0) seg_cnt[sg] = kc;
        wsum += kc;
        if (kc == 0) continue;
        const uint64_t off = sg * kSegCells;
        const uint32_t rank = (uint32_t)__popcll(m & below);
        if (keep) {
            st2<false>(uv_out + 2 * (off + rank), u, v);
            if (cells_out) cells_out[off + rank] = cw.i * g.ncx + cw.j;
            double* d = lx + 3 * rank;
            d[0] = X;
            d[1] = Y;
            d[2] = Z;
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        // 3 * 64 * sg doubles: the rays start on the 16-B grid when xyz_out
        // does
        double* dst = xyz_out + 3 * off;
        const uint32_t nd = 3 * kc;
        const uint32_t h = (uint32_t)((reinterpret_cast<uintptr_t>(dst) >> 3) & 1u);
        const uint32_t np = (nd - h) >> 1;
        for (uint32_t p = lane; p < np; p += 64) {
            const uint32_t dd = h + 2 * p;
            st2<false>(dst + dd, lx[dd], lx[dd + 1]);
        }
        if (lane == 0 && h) dst[0] = lx[0];
        if (lane == 63 && ((nd - h) & 1u)) dst[nd - 1] = lx[nd - 1];
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
    if (lane == 0) s_wsum[wid] = wsum;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint64_t t = 0;
        for (int w = 0; w < kBlock / 64; ++w) t += s_wsum[w];
        blk_sum[blockIdx.x] = t;
    }
}

// Single pass (ACM_TUNE_SAMPLE_FUSED >= 1): workgroup b owns tile b of
// kFusedR x 256 cells, unprojects them once keeping the rays in registers,
// publishes its kept count, and finds its output offset by a decoupled
// look-back over the tiles before it (one status word per tile: flag in bits
// 62-63 -- 1 = count of this tile only, 2 = inclusive prefix -- and the count
// below).  Wave 0 inspects 64 predecessors per load.  No ticket atomic: the
// 48.8K same-address returning atomics of a 1e8-cell grid alone took 0.37 ms
// (profiles/r02_diag_sample_phases.log), and the look-back does not need them
// for progress -- a predecessor that has not published after kLbPatience
// polls (one that is not resident: the dispatch order is not guaranteed) has
// its count computed by the waiting wave itself (tile_keep_count), so no
// workgroup ever waits on one that has not started.  The kept points come out
// in cell order exactly as from the two-pass path.
constexpr int kFusedRMin = 2;  // smallest tile (rounds of 256 cells) any setting uses
// Tiles of R rounds of 256 cells: fewer, larger tiles mean fewer look-backs,
// but each round's rays take 6 KiB of LDS per workgroup, so larger tiles cost
// occupancy (R = 4: 25 KB, 6 workgroups per CU).  ACM_TUNE_SAMPLE_FUSED
// 1 / 2 / 3 selects R = 2 / 4 / 8.  (Round 2's default; the segment two-pass
// path above replaced it in round 3.)
constexpr size_t kFusedCells = (size_t)kBlock * kFusedRMin;
constexpr uint64_t kLbAgg = 1ull << 62, kLbIncl = 2ull << 62, kLbVal = (1ull << 62) - 1;
constexpr int kLbPatience = 512;  // polls (s_sleep between) before computing a count itself


template <class TagT, int kFusedR>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(kFusedR >= 8 ? 3 : 6))) void k_sample_fused(CamArg cam, Grid g, size_t cells,
                                                         uint64_t* __restrict__ status,
                                                         double* __restrict__ uv_out,
                                                         double* __restrict__ xyz_out,
                                                         uint64_t* __restrict__ out_counts) {
    const Cam<double> c = sample_cam<TagT>(cam);
    const int lane = threadIdx.x & 63;
    const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // wave-uniform
    __shared__ uint64_t s_excl;
    __shared__ uint32_t sm[kFusedR][kBlock / 64];
    // The rays live in LDS, not in registers: each round's kept rays of a
    // wave, already compacted (rank order), 1.5 KiB per wave and round.  The
    // registers then hold only one unprojection's working set, which is what
    // bounds occupancy during the VALU-heavy phase (rays in VGPRs: 87-119
    // VGPRs = 4-5 waves/SIMD).
    __shared__ double s_ray[kFusedR][kBlock / 64][64 * 3];
    __shared__ uint64_t s_mask[kFusedR][kBlock / 64];  // each wave's kept-lane ballots
    // look-back state that survives the workgroup-wide fallback rounds
    __shared__ uint64_t s_lb_top, s_lb_excl, s_lb_helped, s_lb_help;
    __shared__ uint64_t s_lb_val[64];
    __shared__ int s_lb_state;
    const uint64_t tile = blockIdx.x;
    constexpr size_t kTile = (size_t)kBlock * kFusedR;
    const size_t base = (size_t)tile * kTile;
    const uint64_t below = lane ? ((~0ull) >> (64 - lane)) : 0ull;
    if (threadIdx.x == 0) {
        s_lb_top = tile - 1;  // lane l of wave 0 inspects tile top - l
        s_lb_excl = 0;
        s_lb_helped = 0;
        s_lb_state = tile == 0 ? 1 : 0;
    }
    // One compute block serves this tile and, on the rare fallback path, a
    // predecessor whose count the look-back could not get (a second inlined
    // unprojection beside the live rays cost 50 VGPRs).  `work` is the tile
    // whose rays and counts the registers / sm hold.
    uint64_t work = tile;
    uint64_t agg = 0;
    bool published = false;
    for (;;) {
        const size_t wbase0 = (size_t)work * kTile;
        CellWalk cw;
        cw.init(g, wbase0, threadIdx.x);
#pragma unroll 1
        for (int r = 0; r < kFusedR; ++r, cw.step(g)) {
            const size_t cell = wbase0 + (size_t)r * kBlock + threadIdx.x;
            bool keep = false;
            double u, v, X = 0.0, Y = 0.0, Z = 0.0;
            if (cell < cells) keep = sample_cell<TagT>(c, g, cw, u, v, X, Y, Z);
            const uint64_t mr = __ballot(keep);
            if (lane == 0) {
                sm[r][wid] = (uint32_t)__popcll(mr);
                s_mask[r][wid] = mr;
            }
            if (keep) {  // compacted: slot = rank among the wave's kept lanes
                double* d = s_ray[r][wid] + 3 * __popcll(mr & below);
                d[0] = X;
                d[1] = Y;
                d[2] = Z;
            }
        }
        __syncthreads();
        uint64_t cnt = 0;
        for (int r = 0; r < kFusedR; ++r)
            for (int w = 0; w < kBlock / 64; ++w) cnt += sm[r][w];
        if (work == tile) {
            agg = cnt;
            if (!published && threadIdx.x == 0)
                __hip_atomic_store(status + tile, (tile == 0 ? kLbIncl : kLbAgg) | agg,
                                   __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            published = true;
        } else if (threadIdx.x == 0) {  // a helped predecessor: its count joins the window
            const uint64_t l = s_lb_help;
            s_lb_val[l] = kLbAgg | cnt;
            s_lb_helped |= 1ull << l;
        }
        __syncthreads();
        // Decoupled look-back by wave 0.  A predecessor that has not
        // published after g.patience polls is counted here by the whole
        // workgroup (next pass of the loop); then this tile is recomputed.
        if (wid == 0 && __builtin_amdgcn_readfirstlane(s_lb_state) == 0) {
            int64_t top = (int64_t)s_lb_top;
            uint64_t excl = s_lb_excl, helped = s_lb_helped;
            const uint64_t help_w = ((helped >> lane) & 1ull) ? s_lb_val[lane] : 0;
            for (int polls = 0;;) {
                const int64_t idx = top - lane;
                uint64_t w = idx >= 0 ? __hip_atomic_load(status + idx, __ATOMIC_RELAXED,
                                                          __HIP_MEMORY_SCOPE_AGENT)
                                      : kLbIncl;  // before tile 0: prefix 0
                if (((helped >> lane) & 1ull) && (w >> 62) == 0) w = help_w;
                const uint64_t incl = __ballot((w >> 62) == 2);
                const uint64_t none = __ballot((w >> 62) == 0);
                const int stop = incl ? __ffsll((long long)incl) - 1 : 64;
                const uint64_t need = stop == 63 || stop == 64 ? ~0ull : ((2ull << stop) - 1);
                if (none & need) {  // a nearer tile has not published yet
                    if (++polls < g.patience) {
                        __builtin_amdgcn_s_sleep(2);
                        continue;
                    }
                    if (lane == 0) {  // not resident (or very late): count it here
                        s_lb_top = (uint64_t)top;
                        s_lb_excl = excl;
                        // the helped set belongs to THIS window: after the
                        // look-back moved on (top -= 64) the register copy is
                        // 0 and the old window's entries must not survive
                        s_lb_helped = helped;
                        s_lb_help = (uint64_t)(__ffsll((long long)(none & need)) - 1);
                        s_lb_state = 2;
                    }
                    break;
                }
                uint64_t v = lane <= stop ? (w & kLbVal) : 0;
#pragma unroll
                for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
                excl += v;
                if (stop < 64) {
                    if (lane == 0) {
                        __hip_atomic_store(status + tile, kLbIncl | (excl + agg),
                                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        s_lb_excl = excl;
                        s_lb_state = 1;
                    }
                    break;
                }
                top -= 64;
                helped = 0;
                polls = 0;
            }
        }
        __syncthreads();
        const int state = __builtin_amdgcn_readfirstlane(s_lb_state);
        if (state == 1 && work == tile) break;  // prefix known, own rays in registers
        if (state == 2) {
            work = s_lb_top - s_lb_help;
            __syncthreads();  // everyone has read the request before it is reset
            if (threadIdx.x == 0) s_lb_state = 0;
        } else {
            work = tile;  // prefix known: recompute this tile's rays
        }
    }
    if (threadIdx.x == 0) {
        s_excl = s_lb_excl;
        if (base + kTile >= cells) {  // last tile: the kept total
            out_counts[0] = s_lb_excl + agg;
            out_counts[1] = cells;
        }
    }
    __syncthreads();
    uint64_t run = s_excl;
    CellWalk cw;
    cw.init(g, base, threadIdx.x);
#pragma unroll 1
    for (int r = 0; r < kFusedR; ++r, cw.step(g)) {
        uint64_t wbase = run, tot = 0;
        for (int w = 0; w < kBlock / 64; ++w) {
            if (w < wid) wbase += sm[r][w];
            tot += sm[r][w];
        }
        const uint64_t mr = s_mask[r][wid];
        const uint32_t rank = (uint32_t)__popcll(mr & below);
        const uint32_t cnt = (uint32_t)__popcll(mr);
        if ((mr >> lane) & 1ull) {
            // the same u, v as sample_cell (point_sampling.rs:69-70): 16 B per
            // lane, consecutive kept points -> one contiguous run per wave
            st2<false>(uv_out + 2 * (wbase + rank), ((double)cw.j + 0.5) * g.cw,
                       ((double)cw.i + 0.5) * g.ch);
        }
        // The wave's kept rays of this round are 3*cnt consecutive doubles of
        // xyz_out, already compacted in LDS: written as 16-B pieces on the
        // 16-B grid (plus a single leading / trailing double) instead of
        // three 8-B stores per lane at a 24-B stride.
        if (cnt) {
            const double* lx = s_ray[r][wid];
            double* dst = xyz_out + 3 * wbase;
            const uint32_t nd = 3 * cnt;
            const uint32_t h = (uint32_t)((reinterpret_cast<uintptr_t>(dst) >> 3) & 1u);
            const uint32_t np = (nd - h) >> 1;
            for (uint32_t p = lane; p < np; p += 64) {
                const uint32_t d = h + 2 * p;
                st2<false>(dst + d, lx[d], lx[d + 1]);
            }
            if (lane == 0 && h) dst[0] = lx[0];
            if (lane == 63 && ((nd - h) & 1u)) dst[nd - 1] = lx[nd - 1];
        }
        run += tot;
    }
}

// ----------------------------------------------------------------- median
// Exact median of the valid (non-NaN, >= 0) errors, error_metrics.rs:104-111,
// without a full sort: MSB-first radix select on the f64 bit patterns (for
// non-negative doubles the unsigned bit order is the numeric order; the NaN
// markers 0x7ff8.. sort above +inf so they never reach a rank < n_valid).
// The selection state (prefix, mask, remaining rank) of both median ranks
// lives on device, so the passes need no host round trip.
struct SelState {
    unsigned long long prefix, mask, k;
};

// Exact radix select on the f64 bit patterns (values are >= 0 or NaN, so the
// unsigned order of the bits is the numeric order and NaNs sort last).  Both
// median ranks, (m-1)/2 (state a) and m/2 (state b), are selected in the
// same passes: each pass reads the values once and builds one 2048-bin
// histogram per state (11-bit digits: 6 passes over the values instead of
// 2 x 8 with 8-bit digits).  Histogram counts are kept as f64 (exact below
// 2^53, and integer sums are order-independent) so a multi-GPU caller can
// all-reduce them in place with the same f64 callback the LM uses.
// digit p covers bits [shift, shift + width): 53..63, 42..52, 31..41, 20..30, 9..19, 0..8
__host__ __device__ constexpr int sel_shift(int pass) { return pass < 5 ? 53 - 11 * pass : 0; }
__host__ __device__ constexpr int sel_width(int pass) { return pass < 5 ? 11 : 9; }
constexpr int kSelPasses = 6;
constexpr int kSelU = 8;  // values in flight per lane in the streaming passes

// The streaming selection kernels run one 1024-lane workgroup per CU: 16
// waves x kSelU loads in flight per CU, and only #CU workgroups flushing
// histogram bins / claiming candidate slots with global atomics (thousands
// of same-address atomics from 1024 small workgroups serialised: 0.47 ms of
// a 0.67 ms median, profiles/r01_diag_median.log).
constexpr int kSelBlock = 1024;
constexpr int kSelWaves = kSelBlock / 64;

// n_dev != nullptr: the value count lives in device memory (the compacted
// candidate buffer of the later passes).
template <bool AGG, bool NTL>
__global__ __launch_bounds__(kSelBlock) void k_sel_hist(size_t n, const unsigned long long* n_dev,
                                                        const double* __restrict__ vals,
                                                        const SelState* __restrict__ st,
                                                        int pass, double* __restrict__ hist) {
    __shared__ unsigned int h[2][kSelBins];
    for (int j = threadIdx.x; j < 2 * kSelBins; j += kSelBlock) (&h[0][0])[j] = 0;
    __syncthreads();
    if (n_dev) n = (size_t)*n_dev;
    const unsigned long long pa = st[0].prefix, ma = st[0].mask;
    const unsigned long long pb = st[1].prefix, mb = st[1].mask;
    const bool same = pa == pb && ma == mb;  // one histogram serves both states
    const int shift = sel_shift(pass);
    const unsigned long long dmask = (1ull << sel_width(pass)) - 1;
    // each wave streams contiguous chunks of kSelU x 64 values (a lane's
    // kSelU loads are 512 B apart, not a grid stride apart: the read probe
    // lost 25% with stride-separated loads in flight); whole waves iterate
    // together, as the AGG ballots need every lane
    const int lane = threadIdx.x & 63;
    const size_t nw = (size_t)gridDim.x * kSelWaves;
    constexpr size_t C = (size_t)kSelU * 64;
    for (size_t b0 = ((size_t)blockIdx.x * kSelWaves + (threadIdx.x >> 6)) * C; b0 < n;
         b0 += nw * C) {
        unsigned long long bits[kSelU];
#pragma unroll
        for (int u = 0; u < kSelU; ++u) {
            const size_t i = b0 + u * 64 + lane;
            bits[u] = i < n ? (unsigned long long)__double_as_longlong(ld1<NTL>(vals + i)) : ~0ull;
        }
#pragma unroll
        for (int u = 0; u < kSelU; ++u) {
            const bool in = b0 + u * 64 + lane < n;
            const unsigned d = (unsigned)((bits[u] >> shift) & dmask);
            sel_count<AGG>(h[0], in && (bits[u] & ma) == pa, d);
            if (!same) sel_count<AGG>(h[1], in && (bits[u] & mb) == pb, d);
        }
    }
    __syncthreads();
    for (int j = threadIdx.x; j < kSelBins; j += kSelBlock) {
        const unsigned c0 = h[0][j];
        const unsigned c1 = same ? c0 : h[1][j];
        if (c0) atomicAdd(&hist[j], (double)c0);
        if (c1) atomicAdd(&hist[kSelBins + j], (double)c1);
    }
}

// Pass 0's histogram from the per-workgroup counts of k_reproj_pass1<HIST>
// (nb x 2048 u32): grid (kSelBins / kBlock, kSelMergeG); each lane sums one
// bin over every kSelMergeG-th workgroup, then one f64 atomic per non-zero
// bin and group into both states' halves (k_sel_init zeroed them; integer
// sums, so the order of the atomics does not matter).
constexpr int kSelMergeG = 64;
__global__ __launch_bounds__(kBlock) void k_sel_hist_merge(const unsigned int* __restrict__ hparts,
                                                           int nb, double* __restrict__ hist) {
    const int j = blockIdx.x * kBlock + threadIdx.x;
    unsigned long long c = 0;
    for (int b = blockIdx.y; b < nb; b += kSelMergeG) c += hparts[(size_t)b * kSelBins + j];
    if (c) {
        atomicAdd(&hist[j], (double)c);
        atomicAdd(&hist[kSelBins + j], (double)c);
    }
}

// Candidates of either state (values matching its prefix after the first
// passes) appended to a compact buffer; later passes read only those.  Each
// workgroup stages its candidates in LDS and claims one slot range with a
// single global atomic (overflow beyond the LDS stage goes straight out,
// one atomic per wave).  The buffer order depends on scheduling, the
// selected ranks do not.
constexpr int kSelStage = 4096;
template <bool NTL>
__global__ __launch_bounds__(kSelBlock) void k_sel_compact(size_t n, const double* __restrict__ vals,
                                                           const SelState* __restrict__ st,
                                                           double* __restrict__ cbuf,
                                                           unsigned long long* __restrict__ count) {
    __shared__ double stage[kSelStage];
    __shared__ unsigned int staged, filled;
    __shared__ unsigned long long gbase;
    if (threadIdx.x == 0) staged = filled = 0;
    __syncthreads();
    const unsigned long long pa = st[0].prefix, ma = st[0].mask;
    const unsigned long long pb = st[1].prefix, mb = st[1].mask;
    const int lane = threadIdx.x & 63;
    const unsigned long long below = (1ull << lane) - 1;
    const size_t nw = (size_t)gridDim.x * kSelWaves;
    constexpr size_t C = (size_t)kSelU * 64;
    for (size_t b0 = ((size_t)blockIdx.x * kSelWaves + (threadIdx.x >> 6)) * C; b0 < n;
         b0 += nw * C) {
        double v[kSelU];
#pragma unroll
        for (int u = 0; u < kSelU; ++u) {
            const size_t i = b0 + u * 64 + lane;
            v[u] = i < n ? ld1<NTL>(vals + i) : 0.0;
        }
        unsigned long long m[kSelU];
        unsigned total = 0;
#pragma unroll
        for (int u = 0; u < kSelU; ++u) {
            const bool in = b0 + u * 64 + lane < n;
            const unsigned long long bits = (unsigned long long)__double_as_longlong(v[u]);
            m[u] = __ballot(in && ((bits & ma) == pa || (bits & mb) == pb));
            total += (unsigned)__popcll(m[u]);
        }
        if (!total) continue;
        unsigned pos = 0;
        if (lane == 0) pos = atomicAdd(&staged, total);
        pos = (unsigned)__shfl((int)pos, 0, 64);
        if (pos + total <= (unsigned)kSelStage) {
            if (lane == 0) atomicMax(&filled, pos + total);
#pragma unroll
            for (int u = 0; u < kSelU; ++u) {
                if ((m[u] >> lane) & 1ull) stage[pos + __popcll(m[u] & below)] = v[u];
                pos += (unsigned)__popcll(m[u]);
            }
        } else {  // stage full: this wave's candidates go straight to global
            unsigned long long base = 0;
            if (lane == 0) base = atomicAdd(count, (unsigned long long)total);
            base = __shfl((long long)base, 0, 64);
#pragma unroll
            for (int u = 0; u < kSelU; ++u) {
                if ((m[u] >> lane) & 1ull) cbuf[base + __popcll(m[u] & below)] = v[u];
                base += (unsigned long long)__popcll(m[u]);
            }
        }
    }
    __syncthreads();
    // claims are handed out in order, so the claims that fit the stage are
    // exactly the prefix [0, filled): later (overflowing) claims went global
    const unsigned k = filled;
    if (threadIdx.x == 0 && k) gbase = atomicAdd(count, (unsigned long long)k);
    __syncthreads();
    for (unsigned j = threadIdx.x; j < k; j += kSelBlock) cbuf[gbase + j] = stage[j];
}

// Picks this pass's digit for both states from the (all-reduced) histograms
// and clears them for the next pass.  One workgroup of NT lanes: each lane
// owns kSelBins / NT consecutive bins, a block-wide inclusive scan finds the
// bin where the running count passes k.
template <int NT>
__device__ __forceinline__ void sel_pick_wg(SelState* st, int pass, double* hist) {
    constexpr int PER = kSelBins / NT;
    __shared__ unsigned long long scan[NT];
    __shared__ int found;
    const int t = threadIdx.x;
    const int shift = sel_shift(pass);
    const unsigned long long dmask = (1ull << sel_width(pass)) - 1;
    for (int w = 0; w < 2; ++w) {
        double* hw = hist + w * kSelBins;
        unsigned long long mine = 0;
#pragma unroll
        for (int j = 0; j < PER; ++j) mine += (unsigned long long)hw[t * PER + j];
        scan[t] = mine;
        if (t == 0) found = NT - 1;
        __syncthreads();
        for (int off = 1; off < NT; off <<= 1) {  // Hillis-Steele inclusive scan
            const unsigned long long v = t >= off ? scan[t - off] : 0;
            __syncthreads();
            scan[t] += v;
            __syncthreads();
        }
        const unsigned long long k = st[w].k;
        const unsigned long long before = t ? scan[t - 1] : 0;
        if (before <= k && k < scan[t]) found = t;  // exactly one lane, unless k >= total
        __syncthreads();
        if (t == found) {
            unsigned long long run = t ? scan[t - 1] : 0;
            int b = t * PER + PER - 1;
            for (int j = 0; j < PER; ++j) {
                const unsigned long long c = (unsigned long long)hw[t * PER + j];
                if (run + c > k) { b = t * PER + j; break; }
                run += c;
            }
            st[w].k = k - run;
            st[w].prefix |= (unsigned long long)b << shift;
            st[w].mask |= dmask << shift;
        }
        __syncthreads();
    }
    for (int j = t; j < 2 * kSelBins; j += NT) hist[j] = 0.0;
}

__global__ __launch_bounds__(kBlock) void k_sel_pick(SelState* __restrict__ st, int pass,
                                                     double* __restrict__ hist) {
    sel_pick_wg<kBlock>(st, pass, hist);
}

// state a: rank (m - 1) / 2, state b: rank m / 2 (equal for odd m); zero
// histograms and candidate count.  Every lane of one workgroup.
__device__ void sel_init_wg(const SelWs& w, unsigned long long m) {
    if (threadIdx.x == 0) {
        *w.count = 0;
        w.st[0].k = m ? (m - 1) / 2 : 0;
        w.st[1].k = m / 2;
        w.st[0].prefix = w.st[1].prefix = 0;
        w.st[0].mask = w.st[1].mask = 0;
    }
    for (int j = threadIdx.x; j < 2 * kSelBins; j += blockDim.x) w.hist[j] = 0.0;
}

__global__ void k_sel_init(SelWs w, const double* __restrict__ nvalid_src,
                           unsigned long long nvalid_fixed) {
    sel_init_wg(w, nvalid_src ? (unsigned long long)nvalid_src[0] : nvalid_fixed);
}

__device__ void sel_finish_one(const SelState* a, const SelState* b, unsigned long long m,
                               double* out) {
    const double va = __longlong_as_double((long long)a->prefix);
    const double vb = __longlong_as_double((long long)b->prefix);
    if (m == 0) out[0] = __builtin_nan("");
    else out[0] = (m % 2 == 0) ? (va + vb) / 2.0 : vb;
}

__global__ void k_sel_finish(const SelState* __restrict__ a, const SelState* __restrict__ b,
                             const double* __restrict__ nvalid_src,
                             unsigned long long nvalid_fixed, double* __restrict__ out) {
    if (threadIdx.x != 0) return;
    sel_finish_one(a, b, nvalid_src ? (unsigned long long)nvalid_src[0] : nvalid_fixed, out);
}

// ------------------------------------------------------ linear estimation
// The reference assembles A (2N x k) and b (2N) per point and solves with
// nalgebra's SVD (kannala_brandt.rs:164-272, double_sphere.rs:225-290,
// ucm.rs:200-258, eucm.rs:216-288, rad_tan.rs:153-234).  At 1e8
// correspondences A alone is 1.6-6.4 GB, so here it is never written: a
// tall-skinny QR (TSQR) folds each row of [A | b] into a per-lane upper-
// triangular R ((k+1) x (k+1), Givens rotations), lanes merge their R's
// through wave shuffles, waves through LDS, workgroups in a fixed-order
// second pass.  A = QR gives the same singular values and least-squares
// solution as the SVD of A (x = R_A^+ Q^T b), numerically stable (no normal
// equations), and the reduction order is fixed -> bit-reproducible.
template <int M>
struct Tri {
    static constexpr int S = M * (M + 1) / 2;
    static __device__ __host__ constexpr int at(int r, int c) { return r * M - r * (r - 1) / 2 + (c - r); }
};

// fold one row (length M, entries before `first` are zero) into R
template <int M>
__device__ __forceinline__ void tri_add_row(double (&R)[Tri<M>::S], double (&row)[M]) {
#pragma unroll
    for (int j = 0; j < M; ++j) {
        const double b = row[j];
        if (b != 0.0) {
            const double a = R[Tri<M>::at(j, j)];
            const double r = sqrt_rn(a * a + b * b);
            const double c = a / r, s = b / r;
            R[Tri<M>::at(j, j)] = r;
#pragma unroll
            for (int l = j + 1; l < M; ++l) {
                const double Rl = R[Tri<M>::at(j, l)], rl = row[l];
                R[Tri<M>::at(j, l)] = c * Rl + s * rl;
                row[l] = c * rl - s * Rl;
            }
        }
    }
}

// fold NR rows at once into R with one Householder reflection per column
// (r04): the stacked [R; rows] has, in column j, R's diagonal x0 above the
// rows' entries; the reflector that zeroes the rows' column j costs one
// square root and one division for all NR rows, where tri_add_row's Givens
// rotations take one of each per row and column.  Backward stable like the
// rotations; the diagonal is kept >= 0 (a row of R may be negated: R^T R and
// the solve of [A | b] are unchanged), as tri_add_row's is.
template <int M, int NR>
__device__ __forceinline__ void tri_add_rows(double (&R)[Tri<M>::S], double (&rows)[NR][M]) {
#pragma unroll
    for (int j = 0; j < M; ++j) {
        double sig = 0.0;
#pragma unroll
        for (int i = 0; i < NR; ++i) sig += rows[i][j] * rows[i][j];
        if (sig != 0.0) {
            const double x0 = R[Tri<M>::at(j, j)];
            const double nrm = sqrt_rn(x0 * x0 + sig);
            const double v0 = x0 >= 0.0 ? x0 + nrm : x0 - nrm;  // no cancellation
            const double beta = 2.0 / (v0 * v0 + sig);
            // new diagonal -sign(x0) nrm, flipped to +nrm with its row
            const double flip = x0 >= 0.0 ? -1.0 : 1.0;
            R[Tri<M>::at(j, j)] = nrm;
#pragma unroll
            for (int l = j + 1; l < M; ++l) {
                double d = v0 * R[Tri<M>::at(j, l)];
#pragma unroll
                for (int i = 0; i < NR; ++i) d += rows[i][j] * rows[i][l];
                const double t = beta * d;
                R[Tri<M>::at(j, l)] = flip * (R[Tri<M>::at(j, l)] - t * v0);
#pragma unroll
                for (int i = 0; i < NR; ++i) rows[i][l] -= t * rows[i][j];
            }
        }
    }
}

template <int M>
__device__ __forceinline__ void tri_merge(double (&R)[Tri<M>::S], const double (&O)[Tri<M>::S]) {
#pragma unroll
    for (int r = 0; r < M; ++r) {
        double row[M];
#pragma unroll
        for (int c = 0; c < M; ++c) row[c] = c < r ? 0.0 : O[Tri<M>::at(r, c)];
        tri_add_row<M>(R, row);
    }
}

// Rows of [A | b] for point i (2 rows), per model; returns false to skip
// the point, sets *err on the reference's NumericalError path.
template <int MODEL>
struct LinRows;

template <>
struct LinRows<ACM_KANNALA_BRANDT> {  // kannala_brandt.rs:184-259, k = 4
    static constexpr int K = 4;
    __device__ static bool rows(const Cam<double>& c, double X, double Y, double Z, double u,
                                double v, double (&r0)[K + 1], double (&r1)[K + 1], int& err) {
        const double fx = c.p[0], fy = c.p[1], cx = c.p[2], cy = c.p[3];
        if (Z <= kEps) return false;  // :195-197
        const double r = sqrt_rn(X * X + Y * Y);
        const double theta = atan2(r, Z);
        const double t2 = theta * theta, t3 = t2 * theta, t5 = t3 * t2, t7 = t5 * t2, t9 = t7 * t2;
        r0[0] = r1[0] = t3; r0[1] = r1[1] = t5; r0[2] = r1[2] = t7; r0[3] = r1[3] = t9;
        const double x_r = r < kEps ? 0.0 : X / r;
        const double y_r = r < kEps ? 0.0 : Y / r;
        if ((fabs(fx * x_r) < kEps && fabs(x_r) > kEps) || (fabs(fy * y_r) < kEps && fabs(y_r) > kEps))
            err = 1;  // :229-238
        r0[K] = fabs(x_r) > kEps ? (u - cx) / (fx * x_r) - theta : (fabs(u - cx) < kEps ? -theta : 0.0);
        r1[K] = fabs(y_r) > kEps ? (v - cy) / (fy * y_r) - theta : (fabs(v - cy) < kEps ? -theta : 0.0);
        return true;
    }
};

struct LinRowsAlpha {  // double_sphere.rs:242-258 (= ucm.rs, eucm.rs), k = 1
    static constexpr int K = 1;
    __device__ static bool rows(const Cam<double>& c, double X, double Y, double Z, double u,
                                double v, double (&r0)[K + 1], double (&r1)[K + 1], int&) {
        const double fx = c.p[0], fy = c.p[1], cx = c.p[2], cy = c.p[3];
        const double d = sqrt_rn(X * X + Y * Y + Z * Z);
        const double u_cx = u - cx, v_cy = v - cy;
        r0[0] = u_cx * (d - Z);
        r1[0] = v_cy * (d - Z);
        r0[1] = (fx * X) - (u_cx * Z);
        r1[1] = (fy * Y) - (v_cy * Z);
        return true;
    }
};
template <> struct LinRows<ACM_DOUBLE_SPHERE> : LinRowsAlpha {};
template <> struct LinRows<ACM_UCM> : LinRowsAlpha {};
template <> struct LinRows<ACM_EUCM> : LinRowsAlpha {};

template <>
struct LinRows<ACM_RADTAN> {  // rad_tan.rs:168-198, k = 3
    static constexpr int K = 3;
    __device__ static bool rows(const Cam<double>& c, double X, double Y, double Z, double u,
                                double v, double (&r0)[K + 1], double (&r1)[K + 1], int&) {
        const double fx = c.p[0], fy = c.p[1], cx = c.p[2], cy = c.p[3];
        const double xn = X / Z, yn = Y / Z;
        const double r2 = xn * xn + yn * yn, r4 = r2 * r2, r6 = r4 * r2;
        r0[0] = fx * xn * r2; r0[1] = fx * xn * r4; r0[2] = fx * xn * r6;
        r1[0] = fy * yn * r2; r1[1] = fy * yn * r4; r1[2] = fy * yn * r6;
        r0[3] = u - (fx * xn + cx);
        r1[3] = v - (fy * yn + cy);
        return true;
    }
};

constexpr int kTsqrMaxBlocks = 2048;
// non-temporal loads of the read-once point / observation streams in k_tsqr
#ifndef ACM_TSQR_NTL
#define ACM_TSQR_NTL 1
#endif
constexpr bool kTsqrNtl = ACM_TSQR_NTL != 0;
// Householder batches per round of load slots (k_tsqr): the loads of this
// many batches are in flight at once (2 vs 1 at 92.9M, same box: the fused
// opening 1.157 -> 1.144 ms, TSQR alone 0.583 -> 0.580 ms,
// profiles/r05p_tsqr_rounds_ab.log; bit-identical, the fold order is the same)
#ifndef ACM_TSQR_ROUNDS
#define ACM_TSQR_ROUNDS 2
#endif
constexpr int kTsqrRounds = ACM_TSQR_ROUNDS;
template <int M> constexpr int kTsqrB = M <= 3 ? 4 : 2;

// TagR != void (acm_linear_estimation_with_error, r04): the same pass also
// computes the reprojection error of the camera as given -- the reference's
// initial_error, computed just before linear_estimation on the same
// correspondences (camera_converter.rs:371-375) -- so the 40 B per point are
// read once for both: per-point errors (errs), k_reproj_pass1's statistics
// partials (rparts) and the median's pass-0 histogram (hparts).
template <int MODEL, int LAYOUT, class TagR = void, bool NTS = false, bool NTL = false, class OBS = ObsPixels>
__global__ __launch_bounds__(kBlock) void k_tsqr(acm_camera cam, size_t n,
                                                 const double* __restrict__ pts,
                                                 OBS obs,
                                                 double* __restrict__ parts,
                                                 int* __restrict__ err_flag,
                                                 double* __restrict__ errs,
                                                 double* __restrict__ rparts,
                                                 unsigned int* __restrict__ hparts) {
    using RW = LinRows<MODEL>;
    constexpr int M = RW::K + 1;
    constexpr int S = Tri<M>::S;
    constexpr bool REPROJ = !std::is_void<TagR>::value;
    __shared__ unsigned int h[REPROJ ? kSelBins : 1];
    if constexpr (REPROJ) {
        for (int j = threadIdx.x; j < kSelBins; j += kBlock) h[j] = 0;
        __syncthreads();
    }
    ReprojAcc acc;
    const Cam<double> c = make_cam<double>(cam);
    double R[S];
#pragma unroll
    for (int q = 0; q < S; ++q) R[q] = 0.0;
    int err = 0;
    const size_t stride = (size_t)gridDim.x * kBlock;
    // kTsqrB<M> points per lane step, their 2 kTsqrB rows folded in with one
    // Householder reflection per column.  Software pipelined (r05) like
    // k_normal_eq / k_reproj_pass1: B static slots, each slot's next point
    // loaded as soon as the slot's current one is consumed, so the next
    // step's B points are in flight while this step's Householder runs
    // (branch-free loads; past the end: point n - 1 again, never used).
    // The r04 form loaded B points, then computed, with no loads in flight
    // across the step: 1.00 ms at 92.9M for the fused opening, whose
    // traffic's ceiling is ~0.80 ms (profiles/r05m_reproj_ceiling.log).
    constexpr int B = kTsqrB<M>;
    constexpr int A = B * kTsqrRounds;  // load slots: kTsqrRounds batches in flight
    double xs[A], ys[A], zs[A];
    typename OBS::raw os[A];
    auto load_slot = [&](int q, size_t iq) {
        const size_t ic = iq < n ? iq : n - 1;
        load_point<LAYOUT, NTL>(pts, n, ic, xs[q], ys[q], zs[q]);
        os[q] = obs.template load<NTL>(ic);
    };
    size_t i = (size_t)blockIdx.x * kBlock + threadIdx.x;
    if (n) {
#pragma unroll
        for (int q = 0; q < A; ++q) load_slot(q, i + (size_t)q * stride);
    }
    for (; i < n; i += (size_t)A * stride) {
#pragma unroll
      for (int g = 0; g < kTsqrRounds; ++g) {
        double rows[2 * B][M];
#pragma unroll
        for (int bb = 0; bb < B; ++bb) {
            const int b = g * B + bb;  // slot
            const size_t ib = i + (size_t)b * stride;
            const bool in = ib < n;
            const double2 ob = obs.get(os[b]);
            if constexpr (REPROJ) {
                using MR = typename TagR::template type<double>;
                double e = __builtin_nan("");
                if (in) {
                    e = reproj_error<MR>(c, xs[b], ys[b], zs[b], ob);
                    acc.add(e);
                    if (NTS) __builtin_nontemporal_store(e, errs + ib);
                    else errs[ib] = e;
                }
                sel_count<true>(h, in, sel_digit0(e));
            }
            int e = 0;
            const bool ok = in && RW::rows(c, xs[b], ys[b], zs[b], ob.x, ob.y, rows[2 * bb],
                                           rows[2 * bb + 1], e);
            if (in) err |= e;
            if (!ok) {
#pragma unroll
                for (int q = 0; q < M; ++q) rows[2 * bb][q] = rows[2 * bb + 1][q] = 0.0;
            }
            load_slot(b, ib + (size_t)A * stride);
        }
        tri_add_rows<M, 2 * B>(R, rows);
      }
    }
    // wave merge (fixed butterfly order)
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        double O[S];
#pragma unroll
        for (int q = 0; q < S; ++q) O[q] = __shfl_down(R[q], off, 64);
        if ((threadIdx.x & 63) < off) tri_merge<M>(R, O);
    }
    __shared__ double sm[kBlock / 64][S];
    __shared__ int serr;
    if (threadIdx.x == 0) serr = 0;
    __syncthreads();
    if (err) atomicOr(&serr, 1);
    if ((threadIdx.x & 63) == 0) {
#pragma unroll
        for (int q = 0; q < S; ++q) sm[threadIdx.x >> 6][q] = R[q];
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int w = 1; w < kBlock / 64; ++w) {
            double O[S];
#pragma unroll
            for (int q = 0; q < S; ++q) O[q] = sm[w][q];
            tri_merge<M>(R, O);
        }
#pragma unroll
        for (int q = 0; q < S; ++q) parts[(size_t)blockIdx.x * S + q] = R[q];
        if (serr) atomicOr(err_flag, 1);
    }
    if constexpr (REPROJ) {
        acc.store(rparts + (size_t)blockIdx.x * kReprojW);
        __syncthreads();
        unsigned int* hp = hparts + (size_t)blockIdx.x * kSelBins;
        for (int j = threadIdx.x; j < kSelBins; j += kBlock) hp[j] = h[j];
    }
}

// fixed-order merge of the per-workgroup R factors: 256 lanes take strided
// blocks, then the same butterfly + LDS order as above
template <int M>
__global__ __launch_bounds__(kBlock) void k_tsqr_final(const double* __restrict__ parts, int nb,
                                                       double* __restrict__ out) {
    constexpr int S = Tri<M>::S;
    double R[S];
#pragma unroll
    for (int q = 0; q < S; ++q) R[q] = 0.0;
    for (int b = threadIdx.x; b < nb; b += kBlock) {
        double O[S];
#pragma unroll
        for (int q = 0; q < S; ++q) O[q] = parts[(size_t)b * S + q];
        tri_merge<M>(R, O);
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        double O[S];
#pragma unroll
        for (int q = 0; q < S; ++q) O[q] = __shfl_down(R[q], off, 64);
        if ((threadIdx.x & 63) < off) tri_merge<M>(R, O);
    }
    __shared__ double sm[kBlock / 64][S];
    if ((threadIdx.x & 63) == 0) {
#pragma unroll
        for (int q = 0; q < S; ++q) sm[threadIdx.x >> 6][q] = R[q];
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int w = 1; w < kBlock / 64; ++w) {
            double O[S];
#pragma unroll
            for (int q = 0; q < S; ++q) O[q] = sm[w][q];
            tri_merge<M>(R, O);
        }
#pragma unroll
        for (int q = 0; q < S; ++q) out[q] = R[q];
    }
}

// ------------------------------------------------------- FOV grid search
// fov.rs:153-251: FOV's linear_estimation is a grid search -- for each
// w = i/100 (i = 10..299) the mean reprojection error of a simplified FOV
// projection over all points.  Here each lane owns ONE grid value (290 lanes
// of a 320-lane workgroup) and walks a contiguous chunk of points staged in
// LDS (every lane reads the same point: broadcast, no bank conflicts), so
// its running sum follows the reference's serial point order within the
// chunk and no cross-lane reduction is needed.  The per-w constants come
// from a host-built table (w, 2 tan(w/2), 2 tan(w/2)/w) so tan is glibc's.
// Compute-bound: one f64 atan (degree-20 polynomial) + rsq-based sqrt per
// (point, w); every per-point quantity (r / z, z / r, 1 / r, fx x, cx - u,
// ...) is computed once in LDS and shared by the 290 grid lanes.
constexpr int kFovGrid = ACM_FOV_GRID_SIZE;
constexpr int kFovBlock = 320;
constexpr int kFovMaxBlocks = 2048;

// The general (z <= 0, r == 0, non-finite) form with OCML atan2, out of line:
// it is rare and uniform per point, and inlined its registers cost the grid
// kernel a wave of occupancy.
__device__ __noinline__ double fov_rd_general(double tw2, double r, double z, double w,
                                              double r2, double rd0) {
    const double atan_wrd = atan2(tw2 * r, z);             // fov.rs:196
    return r2 < kEpsSqrt ? rd0 : atan_wrd / (r * w);       // :200-205
}

// U: points evaluated per step of a lane (independent chains the scheduler
// can interleave; the sum still adds them in point order).
template <int LAYOUT, int U>
__global__ __launch_bounds__(kFovBlock) void k_fov_grid(acm_camera cam, size_t n, size_t chunk,
                                                        const double* __restrict__ pts,
                                                        const double* __restrict__ obs,
                                                        const double* __restrict__ table,
                                                        double* __restrict__ parts) {
    __shared__ double sx[kFovBlock], sy[kFovBlock], sz[kFovBlock], su[kFovBlock],
        sv[kFovBlock], sr2[kFovBlock], sr[kFovBlock], stz[kFovBlock], szt[kFovBlock],
        sir[kFovBlock], sax[kFovBlock], say[kFovBlock], sbx[kFovBlock], sby[kFovBlock];
    __shared__ unsigned char smode[kFovBlock];
    const int t = threadIdx.x;
    const bool active = t < kFovGrid;
    const double fx = cam.params[0], fy = cam.params[1], cx = cam.params[2], cy = cam.params[3];
    double w = 1.0, tw2 = 0.0, rd0 = 0.0;
    if (active) {
        w = table[3 * t];
        tw2 = table[3 * t + 1];
        rd0 = table[3 * t + 2];
    }
    const double iw = 1.0 / w, itw2 = 1.0 / tw2;
    const size_t b0 = (size_t)blockIdx.x * chunk;
    const size_t b1 = b0 + chunk < n ? b0 + chunk : n;
    double sum = 0.0, cnt = 0.0;
    for (size_t base = b0; base < b1; base += kFovBlock) {
        __syncthreads();
        const size_t i = base + t;
        if (i < b1) {
            double x, y, z;
            load_point<LAYOUT>(pts, n, i, x, y, z);
            const double r2 = x * x + y * y;  // :192-193
            const double r = sqrt_rn(r2);
            const double u0 = obs[2 * i], v0 = obs[2 * i + 1];
            sx[t] = x; sy[t] = y; sz[t] = z;
            su[t] = u0; sv[t] = v0;
            sr2[t] = r2; sr[t] = r;
            // mode 0: z > 0, r > 0, both finite -- atan2(2 tan(w/2) r, z) =
            // atan(2 tan(w/2) r / z) from per-point r/z, z/r, 1/r shared by
            // every grid lane; 1: r2 < sqrt(EPS) (rd = rd0, :200-205);
            // 2: anything else (OCML atan2, fov_rd_general)
            const bool fast = z > 0.0 && r > 0.0 && z < INFINITY && r < INFINITY;
            smode[t] = r2 < kEpsSqrt ? 1 : (fast ? 0 : 2);
            stz[t] = fast ? r / z : 0.0;
            szt[t] = fast ? z / r : 0.0;
            sir[t] = fast ? 1.0 / r : 0.0;
            // the error terms as fma(fx x, rd, cx - u) / fma(fy y, rd, cy - v):
            // the reference's (fx (x rd) + cx) - u up to the last bit (the
            // grid sums are held to 1e-12, not to the serial order)
            sax[t] = fx * x; say[t] = fy * y;
            sbx[t] = cx - u0; sby[t] = cy - v0;
        }
        __syncthreads();
        const int m = (int)(b1 - base < (size_t)kFovBlock ? b1 - base : (size_t)kFovBlock);
        auto eval = [&](int k) -> double {
            const int md = smode[k];  // uniform: every lane reads point k
            double du, dv;
            if (md != 2) {
                double rd;
                if (md == 0) {
                    // a = 2 tan(w/2) r / z; atan(a) = pi/2 - atan(1/a) above 1
                    const double a = tw2 * stz[k];
                    const bool big = a > 1.0;
                    const double at = atan01(big ? itw2 * szt[k] : a);
                    const double atan_wrd = big ? 1.5707963267948966 - at : at;  // :196
                    rd = atan_wrd * sir[k] * iw;                                  // :205
                } else {
                    rd = rd0;  // :200-203
                }
                du = fma(sax[k], rd, sbx[k]);
                dv = fma(say[k], rd, sby[k]);
            } else {
                const double rd = fov_rd_general(tw2, sr[k], sz[k], w, sr2[k], rd0);
                const double mx = sx[k] * rd, my = sy[k] * rd;
                du = (fx * mx + cx) - su[k];
                dv = (fy * my + cy) - sv[k];
            }
            // sqrt(du^2 + dv^2) (:211-213) from rsq + Newton (~1 ulp) on the
            // normal range, the IEEE sqrt elsewhere (0, huge, NaN)
            const double d2 = fma(du, du, dv * dv);
            return nr_range(d2) ? d2 * rsq_nr(d2) : sqrt(d2);
        };
        if (active) {
            int k = 0;
            for (; k + U <= m; k += U) {
                double e[U];
#pragma unroll
                for (int j = 0; j < U; ++j) e[j] = eval(k + j);
#pragma unroll
                for (int j = 0; j < U; ++j)
                    if (isfinite(e[j])) { sum += e[j]; cnt += 1.0; }
            }
            for (; k < m; ++k) {
                const double e = eval(k);
                if (isfinite(e)) { sum += e; cnt += 1.0; }
            }
        }
    }
    if (active) {
        parts[(size_t)blockIdx.x * (2 * kFovGrid) + t] = sum;
        parts[(size_t)blockIdx.x * (2 * kFovGrid) + kFovGrid + t] = cnt;
    }
}

// Record form (r03, default): the same staging and evaluation, but each
// point's terms sit in LDS as one 64-B record (AoS) that a lane reads whole
// -- four 16-B broadcast reads -- one point ahead, alternating between two
// register slots (no register copies, whose pending loads the compiler would
// wait for).  The LDS form above reads the 8 values of a point inside the
// evaluation, each read followed by its own lgkmcnt wait: ~4 LDS round trips
// per (point, w) evaluation (VALU busy 0.59-0.72,
// profiles/r03_fp64_kernels.md).  (Records in global memory read by
// wave-uniform scalar loads measured 10.3 vs 8.7 ms: a scalar load from L2
// outlasts one evaluation, and the 16 + 16 record SGPRs beside the 42 atan
// coefficients spilled.)  Same per-point values and evaluation, so the sums
// are bit-identical to the LDS form.
// rec: r / z, z / r, 1 / r, fx x, fy y, cx - u, cy - v, mode (0: z > 0,
// r > 0, both finite; 1: r2 < sqrt(EPS); 2: the general form, whose x, y, z,
// u, v the evaluation reads back from the inputs).
constexpr int kFovRec = 8;

template <int LAYOUT>
__global__ __launch_bounds__(kFovBlock) void k_fov_grid_rec(acm_camera cam, size_t n, size_t chunk,
                                                            const double* __restrict__ pts,
                                                            const double* __restrict__ obs,
                                                            const double* __restrict__ table,
                                                            double* __restrict__ parts) {
    __shared__ __attribute__((aligned(16))) double srec[kFovBlock][kFovRec];
    const int t = threadIdx.x;
    const bool active = t < kFovGrid;
    const double fx = cam.params[0], fy = cam.params[1], cx = cam.params[2], cy = cam.params[3];
    double w = 1.0, tw2 = 0.0, rd0 = 0.0;
    if (active) {
        w = table[3 * t];
        tw2 = table[3 * t + 1];
        rd0 = table[3 * t + 2];
    }
    const double iw = 1.0 / w, itw2 = 1.0 / tw2;
    const size_t b0 = (size_t)blockIdx.x * chunk;
    const size_t b1 = b0 + chunk < n ? b0 + chunk : n;
    double sum = 0.0, cnt = 0.0;
    struct Rec { double q[kFovRec]; };
    auto ldrec = [&](int k) {
        Rec r;
        const double2* p = reinterpret_cast<const double2*>(&srec[k][0]);
#pragma unroll
        for (int j = 0; j < kFovRec / 2; ++j) {
            const double2 v = p[j];
            r.q[2 * j] = v.x;
            r.q[2 * j + 1] = v.y;
        }
        return r;
    };
    // the evaluation of k_fov_grid, operand for operand, on point i's record
    auto eval = [&](const Rec& r, size_t i) -> double {
        const double* q = r.q;
        const double md = q[7];
        double du, dv;
        if (md != 2.0) {
            double rd;
            if (md == 0.0) {
                const double a = tw2 * q[0];
                const bool big = a > 1.0;
                const double at = atan01(big ? itw2 * q[1] : a);
                const double atan_wrd = big ? 1.5707963267948966 - at : at;  // :196
                rd = atan_wrd * q[2] * iw;                                    // :205
            } else {
                rd = rd0;  // :200-203
            }
            du = fma(q[3], rd, q[5]);
            dv = fma(q[4], rd, q[6]);
        } else {
            double x, y, z;
            load_point<LAYOUT>(pts, n, i, x, y, z);
            const double r2 = x * x + y * y, rr = sqrt_rn(r2);
            const double rd = fov_rd_general(tw2, rr, z, w, r2, rd0);
            const double mx = x * rd, my = y * rd;
            du = (fx * mx + cx) - obs[2 * i];
            dv = (fy * my + cy) - obs[2 * i + 1];
        }
        const double d2 = fma(du, du, dv * dv);
        return nr_range(d2) ? d2 * rsq_nr(d2) : sqrt(d2);
    };
    auto add = [&](double e) {
        if (isfinite(e)) { sum += e; cnt += 1.0; }
    };
    for (size_t base = b0; base < b1; base += kFovBlock) {
        __syncthreads();
        const size_t i = base + t;
        if (i < b1) {
            double x, y, z;
            load_point<LAYOUT>(pts, n, i, x, y, z);
            const double r2 = x * x + y * y;  // :192-193
            const double r = sqrt_rn(r2);
            const double u0 = obs[2 * i], v0 = obs[2 * i + 1];
            const bool fast = z > 0.0 && r > 0.0 && z < INFINITY && r < INFINITY;
            double2* o = reinterpret_cast<double2*>(&srec[t][0]);
            o[0] = make_double2(fast ? r / z : 0.0, fast ? z / r : 0.0);
            o[1] = make_double2(fast ? 1.0 / r : 0.0, fx * x);
            o[2] = make_double2(fy * y, cx - u0);
            o[3] = make_double2(cy - v0, r2 < kEpsSqrt ? 1.0 : (fast ? 0.0 : 2.0));
        }
        __syncthreads();
        const int m = (int)(b1 - base < (size_t)kFovBlock ? b1 - base : (size_t)kFovBlock);
        if (active) {
            Rec A = ldrec(0);
            int k = 0;
            for (; k + 2 <= m; k += 2) {
                const Rec B = ldrec(k + 1);
                add(eval(A, base + k));
                A = ldrec(k + 2 < m ? k + 2 : k + 1);
                add(eval(B, base + k + 1));
            }
            if (k < m) add(eval(A, base + k));
        }
    }
    if (active) {
        parts[(size_t)blockIdx.x * (2 * kFovGrid) + t] = sum;
        parts[(size_t)blockIdx.x * (2 * kFovGrid) + kFovGrid + t] = cnt;
    }
}

// Point-lane form (r03, default): the transpose of the two forms above.  A
// lane owns P points of a 64 P-point group (their terms in registers, no LDS
// in the loop) and every wave walks the 290 grid values with the per-w
// constants as wave-uniform scalar loads; per grid value the wave's P x 64
// errors are summed lane-serially, then by the xor butterfly (the same bits
// in every lane), and the finite count is a ballot popcount.  Lane l of a
// wave keeps the running totals of grid values l, l + 64, ... in registers.
// Every lane is busy (the grid-lane forms run 290 of 320 lanes), the P
// evaluations of a lane are independent chains, and NW grid values are
// evaluated per step so that their butterflies' shuffles overlap.  The terms are those of the
// forms above, bit for bit; only the summation order differs (the grid sums
// are held to 1e-12 of the serial reference, counts exact).  Groups are split
// evenly over all waves of a grid sized to the resident workgroups.
// table: w, 2 tan(w/2), 2 tan(w/2) / w (3 per grid value), then 1 / w and
// 1 / (2 tan(w/2)) (2 per grid value; the host's IEEE divisions, the same
// bits as the device's).
constexpr int kFovPlBlock = 256;
// 3 points per lane, 2 grid values per step (5.36 ms on 9.3M correspondences;
// P = 2 / 4 and 1 / 4 values per step 5.6-5.9 ms: profiles/r03fov_*.log)
constexpr int kFovPlP = 3, kFovPlNW = 2;

template <int LAYOUT, int P, int NW>
__global__ __launch_bounds__(kFovPlBlock) void k_fov_grid_pl(acm_camera cam, size_t n,
                                                             const double* __restrict__ pts,
                                                             const double* __restrict__ obs,
                                                             const double* __restrict__ table,
                                                             double* __restrict__ parts) {
    constexpr int kWaves = kFovPlBlock / 64, kGroup = 64 * P, kWB = (kFovGrid + 63) / 64;
    __shared__ double s_sum[kWaves][kFovGrid], s_cnt[kWaves][kFovGrid];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const double fx = cam.params[0], fy = cam.params[1], cx = cam.params[2], cy = cam.params[3];
    const size_t groups = (n + kGroup - 1) / kGroup;
    const size_t nw = (size_t)gridDim.x * kWaves, gw = (size_t)blockIdx.x * kWaves + wv;
    const size_t g0 = groups * gw / nw, g1 = groups * (gw + 1) / nw;
    double acc[kWB];
    uint32_t accn[kWB];
#pragma unroll
    for (int b = 0; b < kWB; ++b) {
        acc[b] = 0.0;
        accn[b] = 0;
    }
    for (size_t g = g0; g < g1; ++g) {
        // Per point: r / z, z / r, 1 / r, fx x, fy y, cx - u, cy - v and fl.
        // Branch-free evaluation rd = fma(rd0, fl, atan * (1 / r) / w):
        // z > 0, r > 0, both finite -> fl = 0 (the atan form); r2 < sqrt(EPS)
        // -> 1 / r = 0, fl = 1 (rd = rd0, :200-203); anything else -> the
        // general form (OCML atan2, x, y, z, u, v read back) on a slow path
        // taken by the groups that hold such a point; past the end -> cx - u
        // = NaN, so the error is not finite and is not counted.
        double rz[P], zr[P], ir[P], ax[P], ay[P], bx[P], by[P], fl[P];
        bool gen = false;
#pragma unroll
        for (int j = 0; j < P; ++j) {
            const size_t i = g * kGroup + (size_t)j * 64 + lane;
            rz[j] = zr[j] = ir[j] = ax[j] = ay[j] = by[j] = fl[j] = 0.0;
            bx[j] = __builtin_nan("");
            if (i < n) {
                double x, y, z;
                load_point<LAYOUT>(pts, n, i, x, y, z);
                const double r2 = x * x + y * y;  // fov.rs:192-193
                const double r = sqrt_rn(r2);
                const double u0 = obs[2 * i], v0 = obs[2 * i + 1];
                const bool fast = z > 0.0 && r > 0.0 && z < INFINITY && r < INFINITY;
                const bool small = r2 < kEpsSqrt;
                rz[j] = fast ? r / z : 0.0;
                zr[j] = fast ? z / r : 0.0;
                ir[j] = fast && !small ? 1.0 / r : 0.0;
                fl[j] = small ? 1.0 : 0.0;
                ax[j] = fx * x; ay[j] = fy * y;
                bx[j] = cx - u0; by[j] = cy - v0;
                gen = gen || (!small && !fast);
            }
        }
        // one grid value k: the wave's P x 64 errors summed lane-serially
        // (s) and the finite count (c, wave-uniform)
        auto eval_w = [&](auto gen_c, int k, double& s, uint32_t& c) {
            constexpr bool GEN = decltype(gen_c)::value;
            const double w = table[3 * k], tw2 = table[3 * k + 1], rd0 = table[3 * k + 2];
            const double iw = table[3 * kFovGrid + 2 * k];
            const double itw2 = table[3 * kFovGrid + 2 * k + 1];
            double d2[P], e[P];
            bool slow = false;
#pragma unroll
            for (int j = 0; j < P; ++j) {
                // the evaluation of k_fov_grid, operand for operand
                const double a = tw2 * rz[j];
                const bool big = a > 1.0;
                const double at = atan01(big ? itw2 * zr[j] : a);
                const double atan_wrd = big ? 1.5707963267948966 - at : at;  // :196
                const double rd = fma(rd0, fl[j], atan_wrd * ir[j] * iw);    // :205
                const double du = fma(ax[j], rd, bx[j]), dv = fma(ay[j], rd, by[j]);
                d2[j] = fma(du, du, dv * dv);
                e[j] = d2[j] * rsq_nr(d2[j]);  // :211-213
                slow = slow || !nr_range(d2[j]);
            }
            if (GEN) {
#pragma unroll
                for (int j = 0; j < P; ++j) {
                    const size_t i = g * kGroup + (size_t)j * 64 + lane;
                    if (i < n && fl[j] == 0.0 && ir[j] == 0.0) {
                        double x, y, z;
                        load_point<LAYOUT>(pts, n, i, x, y, z);
                        const double r2 = x * x + y * y, rr = sqrt_rn(r2);
                        const double rdg = fov_rd_general(tw2, rr, z, w, r2, rd0);
                        const double du = (fx * (x * rdg) + cx) - obs[2 * i];
                        const double dv = (fy * (y * rdg) + cy) - obs[2 * i + 1];
                        d2[j] = fma(du, du, dv * dv);
                        e[j] = d2[j] * rsq_nr(d2[j]);
                        slow = slow || !nr_range(d2[j]);
                    }
                }
            }
            if (slow) {  // 0, huge or NaN: the IEEE sqrt
#pragma unroll
                for (int j = 0; j < P; ++j)
                    if (!nr_range(d2[j])) e[j] = sqrt(d2[j]);
            }
            s = 0.0;
            c = 0;
#pragma unroll
            for (int j = 0; j < P; ++j) {
                const bool f = isfinite(e[j]);
                s += f ? e[j] : 0.0;
                c += (uint32_t)__popcll(__ballot(f));
            }
        };
        auto walk = [&](auto gen_c) {
#pragma unroll
            for (int b = 0; b < kWB; ++b) {
                const int wl_end = kFovGrid - b * 64 < 64 ? kFovGrid - b * 64 : 64;
                // NW grid values per step, their butterflies interleaved
                static_assert(64 % NW == 0, "grid values in steps of NW");
                for (int wl = 0; wl < wl_end; wl += NW) {
                    double sv[NW];
                    uint32_t cv[NW];
#pragma unroll
                    for (int v = 0; v < NW; ++v) {
                        sv[v] = 0.0;
                        cv[v] = 0;
                        if (wl_end % NW == 0 || wl + v < wl_end)
                            eval_w(gen_c, b * 64 + wl + v, sv[v], cv[v]);
                    }
#pragma unroll
                    for (int off = 32; off > 0; off >>= 1) {
                        double t[NW];
#pragma unroll
                        for (int v = 0; v < NW; ++v) t[v] = __shfl_xor(sv[v], off, 64);
#pragma unroll
                        for (int v = 0; v < NW; ++v) sv[v] += t[v];
                    }
#pragma unroll
                    for (int v = 0; v < NW; ++v)
                        if (lane == wl + v) {
                            acc[b] += sv[v];
                            accn[b] += cv[v];
                        }
                }
            }
        };
        if (__ballot(gen)) walk(std::true_type{});
        else walk(std::false_type{});
    }
#pragma unroll
    for (int b = 0; b < kWB; ++b) {
        const int k = b * 64 + lane;
        if (k < kFovGrid) {
            s_sum[wv][k] = acc[b];
            s_cnt[wv][k] = (double)accn[b];
        }
    }
    __syncthreads();
    for (int k = threadIdx.x; k < kFovGrid; k += kFovPlBlock) {
        double s = s_sum[0][k], c = s_cnt[0][k];
#pragma unroll
        for (int v = 1; v < kWaves; ++v) {
            s += s_sum[v][k];
            c += s_cnt[v][k];
        }
        parts[(size_t)blockIdx.x * (2 * kFovGrid) + k] = s;
        parts[(size_t)blockIdx.x * (2 * kFovGrid) + kFovGrid + k] = c;
    }
}

// Chunk sums combined in block order (deterministic), one lane per column.
// One workgroup per column: lane l sums chunks l, l + 256, ... and the lanes
// combine in a fixed tree order (deterministic; a lane per column walking all
// chunks serially was latency-bound: 0.53 ms).
__global__ __launch_bounds__(kBlock) void k_fov_finish(const double* __restrict__ parts, int nb,
                                                       double* __restrict__ out) {
    const int c = blockIdx.x;
    double s = 0.0;
    for (int b = threadIdx.x; b < nb; b += kBlock) s += parts[(size_t)b * (2 * kFovGrid) + c];
    __shared__ double sm[kBlock / 64];
    s = wave_sum(s);
    if ((threadIdx.x & 63) == 0) sm[threadIdx.x >> 6] = s;
    __syncthreads();
    if (threadIdx.x == 0) {
        double t = 0.0;
        for (int w = 0; w < kBlock / 64; ++w) t += sm[w];
        out[c] = t;
    }
}

// ---------------------------------------------------------- undistort_image
// undistort.rs:14-105: per output pixel, the ray ((u-cx')/fx', (v-cy')/fy', 1)
// of the target intrinsics is projected through the camera model and the
// input RGB8 image is sampled there (nearest or bilinear, the reference's
// rounding/clamping); failed projections / out-of-image samples stay black.
// 64 x 4 workgroups: a wave covers 64 consecutive output pixels of a row.
__device__ __forceinline__ int rust_as_i32(double v) {
    if (v != v) return 0;  // Rust `as` casts saturate and map NaN to 0
    if (v >= 2147483647.0) return 2147483647;
    if (v <= -2147483648.0) return (-2147483647 - 1);
    return (int)v;
}

template <class TagT, bool BILINEAR>
__global__ __launch_bounds__(kBlock) void k_undistort(acm_camera cam, double tfx, double tfy,
                                                      double tcx, double tcy,
                                                      const uint8_t* __restrict__ img,
                                                      uint8_t* __restrict__ out) {
    using M = typename TagT::template type<double>;
    const uint32_t w = cam.width, h = cam.height;
    const uint32_t u_out = blockIdx.x * 64 + (threadIdx.x & 63);
    const uint32_t v_out = blockIdx.y * (kBlock / 64) + (threadIdx.x >> 6);
    if (u_out >= w || v_out >= h) return;
    const Cam<double> c = make_cam<double>(cam);
    const double x_norm = ((double)u_out - tcx) / tfx;  // :35-36
    const double y_norm = ((double)v_out - tcy) / tfy;
    double su, sv;
    // EXACT: the source coordinate is quantised by round() / floor() below,
    // so it takes the reference-exact projection (IEEE sqrt / divisions and
    // the correctly rounded atan2 for KB / FOV; camera_models.hpp)
    const uint8_t st =
        M::template project<false, false, true>(c, x_norm, y_norm, 1.0, su, sv, nullptr, nullptr);
    uint8_t r = 0, g = 0, b = 0;
    if (st == ST_OK) {
        if (!BILINEAR) {  // :61-69
            const int u = rust_as_i32(round(su)), v = rust_as_i32(round(sv));
            if (u >= 0 && u < (int)w && v >= 0 && v < (int)h) {
                const uint8_t* p = img + ((size_t)v * w + (size_t)u) * 3;
                r = p[0]; g = p[1]; b = p[2];
            }
        } else {  // :71-103
            const double x0 = floor(su), y0 = floor(sv);
            const double x1 = x0 + 1.0, y1 = y0 + 1.0;
            if (!(x0 < 0.0 || x1 >= (double)w || y0 < 0.0 || y1 >= (double)h)) {
                const uint32_t x0u = (uint32_t)x0, y0u = (uint32_t)y0;
                const uint32_t x1u = (uint32_t)x1, y1u = (uint32_t)y1;
                const uint8_t* p00 = img + ((size_t)y0u * w + x0u) * 3;
                const uint8_t* p10 = img + ((size_t)y0u * w + x1u) * 3;
                const uint8_t* p01 = img + ((size_t)y1u * w + x0u) * 3;
                const uint8_t* p11 = img + ((size_t)y1u * w + x1u) * 3;
                const double wx = su - x0, wy = sv - y0;
                const double wx_inv = 1.0 - wx, wy_inv = 1.0 - wy;
                uint8_t res[3];
#pragma unroll
                for (int ch = 0; ch < 3; ++ch) {
                    const double val = (double)p00[ch] * wx_inv * wy_inv +
                                       (double)p10[ch] * wx * wy_inv +
                                       (double)p01[ch] * wx_inv * wy + (double)p11[ch] * wx * wy;
                    double q = round(val);
                    q = q < 0.0 ? 0.0 : (q > 255.0 ? 255.0 : q);
                    res[ch] = (uint8_t)q;
                }
                r = res[0]; g = res[1]; b = res[2];
            }
        }
    }
    uint8_t* o = out + ((size_t)v_out * w + u_out) * 3;
    o[0] = r;
    o[1] = g;
    o[2] = b;
}

static unsigned grid_for(size_t n) { return (unsigned)((n + kBlock - 1) / kBlock); }

// Host-side per-camera constants folded into unused parameter slots before a
// launch.  FOV: params[8] = tan(w / 2) (fov.rs:297, :340), evaluated once by
// the host libm (the same glibc tan the reference's f64::tan calls) instead
// of once per lane by OCML.
// Unprojection launches also carry RN(1 / fx), RN(1 / fy) (0 outside the
// range div_by_f is exact in) and the model's uniform subexpressions.
// reference_newton (ACM_REFERENCE_NEWTON, per call): the reference's own
// Newton loops for every pixel (KB, RadTan) and FOV's IEEE unprojection.
// RadTan::newton_fast's certified disk (r05): the largest S (from a fixed
// schedule, S <= 4) such that for every (x, y) with x^2 + y^2 <= S (1 + 1e-6)
// the distortion Jacobian (rad_tan.rs:470-491) has det >= 1/16 (1 + 1e-6)
// and |j00| + |j11| + 2 |j01| <= 64 (1 - 1e-6) -- the two conditions the fast
// loop's error analysis needs, checked per step until r05 -- and |x|, |y| <=
// 2 (implied by S <= 4).  Then one test of the iterate's own s = x^2 + y^2
// replaces the per-step |x|, |y|, det and row-sum tests (~6 of the step's 77
// VALU instructions).  Rigorous: the square around the disk is cut into
// 128 x 128 cells and on every cell that meets the disk the Jacobian's
// entries are enclosed by interval arithmetic (each bound widened by 4 ulp
// of its magnitude, which covers the rounding of the host's own evaluation):
//   rad = 1 + k1 s + k2 s^2 + k3 s^3, w = 2 (k1 + 2 k2 s + 3 k3 s^2),
//   j00 = rad + x^2 w + 2 p1 y + 6 p2 x, j11 = rad + y^2 w + 6 p1 y + 2 p2 x,
//   j01 = xy w + 2 p1 x + 2 p2 y (= j10), det = j00 j11 - j01^2.
// 0 when no S qualifies: the loop keeps the per-step tests.  Memoised per
// distortion vector (~1 ms of host time per schedule step).
namespace hiv {  // host intervals (radtan_disk_ok)
struct Iv {
    double lo, hi;
};
inline Iv iv_w(double lo, double hi) {  // widen by 4 ulp of the magnitude
    const double e = 4 * 0x1p-52;
    return {lo - e * std::fabs(lo) - 1e-300, hi + e * std::fabs(hi) + 1e-300};
}
inline Iv operator+(Iv a, Iv b) { return iv_w(a.lo + b.lo, a.hi + b.hi); }
inline Iv operator-(Iv a, Iv b) { return iv_w(a.lo - b.hi, a.hi - b.lo); }
inline Iv operator*(Iv a, Iv b) {
    const double p[4] = {a.lo * b.lo, a.lo * b.hi, a.hi * b.lo, a.hi * b.hi};
    return iv_w(std::fmin(std::fmin(p[0], p[1]), std::fmin(p[2], p[3])),
                std::fmax(std::fmax(p[0], p[1]), std::fmax(p[2], p[3])));
}
inline Iv operator*(double c, Iv a) { return Iv{c, c} * a; }
inline Iv iv_sq(Iv a) {
    const double l = std::fabs(a.lo), h = std::fabs(a.hi);
    const double mx = std::fmax(l, h) * std::fmax(l, h);
    const double mn = (a.lo <= 0.0 && a.hi >= 0.0) ? 0.0 : std::fmin(l, h) * std::fmin(l, h);
    return iv_w(mn, mx);
}
inline double iv_mag(Iv a) { return std::fmax(std::fabs(a.lo), std::fabs(a.hi)); }
}  // namespace hiv

static bool radtan_disk_ok(const double* p, double S) {
    using hiv::Iv;
    using hiv::iv_sq;
    using hiv::iv_mag;
    const double k1 = p[4], k2 = p[5], p1 = p[6], p2 = p[7], k3 = p[8];
    const double r = std::sqrt(S * (1.0 + 1e-6)) * (1.0 + 1e-12);
    constexpr int G = 128;
    const double h = 2.0 * r / G;
    for (int i = 0; i < G; ++i) {
        const Iv X{-r + h * i, -r + h * (i + 1)};
        const double dx = X.lo > 0 ? X.lo : (X.hi < 0 ? -X.hi : 0.0);
        for (int j = 0; j < G; ++j) {
            const Iv Y{-r + h * j, -r + h * (j + 1)};
            const double dy = Y.lo > 0 ? Y.lo : (Y.hi < 0 ? -Y.hi : 0.0);
            if (dx * dx + dy * dy > r * r) continue;  // the cell misses the disk
            const Iv X2 = iv_sq(X), Y2 = iv_sq(Y), XY = X * Y;
            const Iv s = X2 + Y2, s2 = iv_sq(s);
            const Iv rad = Iv{1, 1} + k1 * s + k2 * s2 + k3 * (s * s2);
            const Iv w = 2.0 * (Iv{k1, k1} + (2 * k2) * s + (3 * k3) * s2);
            const Iv j00 = rad + X2 * w + (2 * p1) * Y + (6 * p2) * X;
            const Iv j11 = rad + Y2 * w + (6 * p1) * Y + (2 * p2) * X;
            const Iv j01 = XY * w + (2 * p1) * X + (2 * p2) * Y;
            const Iv det = j00 * j11 - iv_sq(j01);
            const double sj = iv_mag(j00) + iv_mag(j11) + 2 * iv_mag(j01);
            if (!(det.lo >= 0.0625 * (1.0 + 1e-6)) || !(sj <= 64.0 * (1.0 - 1e-6))) return false;
        }
    }
    return true;
}

static double radtan_newton_disk_uncached(const double* p) {
    for (int i = 4; i < 9; ++i)
        if (!std::isfinite(p[i])) return 0.0;
    for (double S : {4.0, 3.0, 2.5, 2.0, 1.6, 1.3, 1.0, 0.8, 0.6, 0.4, 0.25})
        if (radtan_disk_ok(p, S)) return S;
    return 0.0;
}

static double radtan_newton_disk(const double* p) {
    // a non-finite distortion never gets a disk, and never reaches the memo:
    // a NaN key would break std::map's ordering
    for (int i = 4; i < 9; ++i)
        if (!std::isfinite(p[i])) return 0.0;
    static std::mutex mu;
    // keyed on the bit patterns, so -0.0 and 0.0 are distinct cameras too
    static std::map<std::array<uint64_t, 5>, double> memo;
    std::array<uint64_t, 5> key;
    std::memcpy(key.data(), p + 4, sizeof(key));
    {
        std::lock_guard<std::mutex> lock(mu);
        auto it = memo.find(key);
        if (it != memo.end()) return it->second;
    }
    const double S = radtan_newton_disk_uncached(p);
    std::lock_guard<std::mutex> lock(mu);
    if (memo.size() > 256) memo.clear();
    memo[key] = S;
    return S;
}

// unprojects: the launch's kernels unproject (acm_unproject, the round trip,
// sample_points, the certificate query).  Only those pay for RadTan's
// certified disk; every other launch (projection, residuals, the normal
// equations inside each LM evaluation, statistics, TSQR, undistort) leaves
// uk[1] = 0 (an LM over RadTan changes the distortion at every
// step, so the memo missed and each evaluation paid ~ms of host time).
static CamArg prep(acm_camera c, bool reference_newton = false, bool unprojects = false) {
    if (c.model == ACM_FOV) c.params[8] = std::tan(c.params[4] / 2.0);
    CamArg a;
    static_cast<acm_camera&>(a) = c;
    auto recip = [](double f) {
        const double af = std::fabs(f);
        return af >= 0x1p-500 && af <= 0x1p500 ? 1.0 / f : 0.0;
    };
    const bool rcp = g_unproject_rcp != 0;
    a.ifx = rcp ? recip(c.params[0]) : 0.0;
    a.ify = rcp ? recip(c.params[1]) : 0.0;
    unproject_consts<double>(c.model, c.params, a.uk);
#ifndef ACM_AB_NO_RADTAN_DISK  // A/B build: the per-step tests of r04
    if (c.model == ACM_RADTAN && unprojects) a.uk[1] = radtan_newton_disk(c.params);
#endif
    if (reference_newton &&
        (c.model == ACM_KANNALA_BRANDT || c.model == ACM_RADTAN || c.model == ACM_FOV))
        a.uk[0] = NAN;  // fast Newton loops / FOV fast unprojection off
    for (int i = 0; i < 12; ++i) a.kc[i] = 0.0;
    a.kc[0] = INFINITY;  // no certified interval (set by acm_sample_points_ex for KB)
    for (int i = 0; i < 2 * kRayPolyN; ++i) a.rp[i] = 0.0;
    return a;
}

// ---------------------------------------- sample_points keep certificates
// KB (kannala_brandt.rs:462-561, point_sampling.rs:91-94): a cell is kept iff
// the reference's Newton loop (theta_0 = ru, theta -= f / f', break when
// |delta| < 1e-6, NumericalError when |f'| < EPS or after 10 steps) ends Ok
// and cos(theta) > 0, i.e. |theta| <= kHalfPiDown.  Everything depends on the
// cell only through ru = min(sqrt(r2), pi/2).  On theta in [-tmax, tmax] bound
// D = f' from below (dmin > 0) and |f''| from above (cmax) by dense sampling
// plus a Lipschitz margin; then for every ru in (0, R], with theta* the
// unique root (f' > 0), the Newton error e_k = |theta_k - theta*| obeys
//   e_0 <= E0 = max |f(ru)| / dmin,   e_{k+1} <= M e_k^2 + eta,
// M = cmax / (2 dmin), eta a generous bound on one step's rounding
// (|f| and |f'| are sums of <= 6 terms of size <= 1 + sum |k_i| tmax^2i).
// If M E0 <= 1/2 the iterates stay within E0 of theta* (in [-tmax, tmax]), f'
// stays >= dmin >> EPS, and the bound sequence shows a step with |delta| <=
// e_k + e_{k+1} + eta < 1e-6 within 10 steps: the reference returns Ok, with
// a final theta within ef = M (1.01e-6)^2 + 2 eta of theta*.  theta* rises
// with ru (theta_d(theta*) = ru, theta_d increasing), so
//   ru in [1e-6 (1 + 1e-6), min(R, theta_d(kHalfPiDown - ef - 1e-9))] -> kept,
//   ru in [theta_d(kHalfPiDown + ef + 1e-9), R]                  -> dropped.
// (ru <= 1e-6 is NumericalError or the ru = 0 special case: never certified.)
// kb_seg_cert_on does this for ru in (0, R], R <= pi/2 the largest bound for
// which the iterates provably stay in [-tmax, tmax] (pi/2 + 2 E0 <= tmax
// above becomes R + 2 E0(R) <= tmax).
static SegCert kb_seg_cert_on(const double* p, double tmax) {
    SegCert s{};
    s.all_lo = s.none_lo = INFINITY;
    s.all_hi = s.none_hi = -INFINITY;
    const double k1 = p[4], k2 = p[5], k3 = p[6], k4 = p[7];
    const double a1 = std::fabs(k1), a2 = std::fabs(k2), a3 = std::fabs(k3), a4 = std::fabs(k4);
    auto D = [&](double t2) { return 1.0 + t2 * (3 * k1 + t2 * (5 * k2 + t2 * (7 * k3 + t2 * 9 * k4))); };
    auto F2 = [&](double t) {  // f''(theta)
        const double t2 = t * t;
        return t * (6 * k1 + t2 * (20 * k2 + t2 * (42 * k3 + t2 * 72 * k4)));
    };
    auto thd = [&](double t) {  // theta_d(theta)
        const double t2 = t * t;
        return t * (1.0 + t2 * (k1 + t2 * (k2 + t2 * (k3 + t2 * k4))));
    };
    const double T2 = tmax * tmax;
    constexpr int G = 16384;
    double dmin = INFINITY, cmax = 0.0;
    for (int i = 0; i <= G; ++i) {
        dmin = std::fmin(dmin, D(T2 * i / G));                // theta^2 in [0, tmax^2]
        cmax = std::fmax(cmax, std::fabs(F2(tmax * i / G)));  // |f''| is odd: [0, tmax]
    }
    // Lipschitz margins of the sampling: |dD/dt2| and the third derivative of f
    const double LD = 3 * a1 + 10 * a2 * T2 + 21 * a3 * T2 * T2 + 36 * a4 * T2 * T2 * T2;
    const double LC = 6 * a1 + 60 * a2 * T2 + 210 * a3 * T2 * T2 + 504 * a4 * T2 * T2 * T2;
    dmin -= 1.01 * LD * (T2 / G) / 2 + 1e-12;
    cmax += 1.01 * LC * (tmax / G) / 2 + 1e-12;
    if (!(dmin > 1e-3) || !std::isfinite(cmax)) return s;
    constexpr double kHalfPi = kPi / 2.0;
    const double kb = 1.0 + a1 * T2 + a2 * T2 * T2 + a3 * T2 * T2 * T2 + a4 * T2 * T2 * T2 * T2;
    const double M = cmax / (2.0 * dmin);
    const double eta = (2.0 * kb + 2.0) * 64 * 0x1p-53 / dmin + 1e-14;
    // E0(R) = max over ru <= R of |f(ru)| / dmin (|f(ru)| rises with ru)
    auto E0 = [&](double R) {
        const double R2 = R * R;
        return R * R2 * (a1 + R2 * (a2 + R2 * (a3 + R2 * a4))) / dmin + 1e-12;
    };
    // the largest ru bound R (<= pi/2) the Newton analysis covers
    double R = kHalfPi;
    while (R > 0.05 && !(M * E0(R) <= 0.5 && R + 2.0 * E0(R) <= tmax * (1 - 1e-9) &&
                         thd(tmax) > R * (1 + 1e-9)))
        R *= 0.98;
    if (!(R > 0.05) || !(eta < 1e-9)) return s;
    bool breaks = false;
    double e = E0(R);
    for (int k = 0; k < 10 && !breaks; ++k) {  // a step with |delta| < 1e-6 by step 9
        const double en = M * e * e + eta;
        if (e + en + eta < 1e-6 * (1.0 - 1e-3)) breaks = true;
        e = en;
    }
    if (!breaks) return s;
    const double ef = M * 1.01e-6 * 1.01e-6 + 2.0 * eta;
    const double m = ef + 1e-9;
    constexpr double kHpd = KannalaBrandt<double>::kHalfPiDown;
    s.on = 1;
    s.M = M;
    s.ef = ef;
    s.ig[0] = M;  // passed to kb_fit_initial_guess (overwritten by the fit)
    s.all_lo = 1e-6 * (1.0 + 1e-6);
    s.all_hi = R;
    if (kHpd - m <= tmax && thd(kHpd - m) < R)  // theta* reaches pi/2 below R
        s.all_hi = thd(kHpd - m) * (1.0 - 1e-12);
    if (kHpd + m <= tmax) {
        const double rn = thd(kHpd + m) * (1.0 + 1e-12);
        if (rn <= R) {
            s.none_lo = rn;
            s.none_hi = R;
        }
    }
    return s;
}

// Any camera for which a check fails gets no certificate: every segment is
// then counted cell by cell.  The theta range the bounds cover is tried at a
// few sizes (a strongly distorted camera's f' may vanish near theta = 2 but
// not below pi/2); the certificate covering the most is kept.
// KB: theta*(ru) ~= ru g(ru^2), g the degree-8 interpolant of theta*(ru)/ru
// in s = ru^2 at Chebyshev nodes on [0, all_hi^2] (theta* solved in long
// double).  Its error e0 over the whole interval (kb_guess_bound, r05: a
// bound; r04 sampled 4001 points) decides ray_certified's Newton steps: one
// when M e0^2 <= 1e-17 (M as in kb_seg_cert_on), two when M^3 e0^4 <= 1e-13
// and e0 <= 1e-5, else the fit is not used (ig_ok = 0).
// Certified rays are the root's, the reference returns its last iterate:
// they differ by up to ef = M (1.01e-6)^2 + 2 eta (kb_seg_cert_on), so the
// rays are used only while ef <= 1e-11, a tenth of the 1e-10 bar (ADVICE
// r03); otherwise every cell takes the reference-iterate path.
static double kb_guess_bound(const double* p, const double* ig, long double Th);
static void kb_fit_initial_guess(const double* p, double M, SegCert& s) {
    s.ig_ok = 0;
    const long double k1 = p[4], k2 = p[5], k3 = p[6], k4 = p[7];
    auto root = [&](long double ru) {
        long double t = ru;
        for (int i = 0; i < 80; ++i) {
            const long double t2 = t * t;
            const long double f = t * (1 + t2 * (k1 + t2 * (k2 + t2 * (k3 + t2 * k4)))) - ru;
            const long double fp = 1 + t2 * (3 * k1 + t2 * (5 * k2 + t2 * (7 * k3 + t2 * 9 * k4)));
            const long double d = f / fp;
            t -= d;
            if (std::fabs((double)d) < 1e-19) break;
        }
        return t;
    };
    const double R = s.all_hi;
    if (!(R > 1e-3)) return;
    constexpr int N = 9;
    long double A[N][N + 1];
    const long double S = (long double)R * R;
    for (int j = 0; j < N; ++j) {
        const long double sj = S * (1 + std::cos(kPi * (j + 0.5) / N)) / 2;
        const long double ru = std::sqrt(sj);
        const long double gj = ru > 0 ? root(ru) / ru : 1;
        long double pw = 1;
        for (int i = 0; i < N; ++i, pw *= sj) A[j][i] = pw;
        A[j][N] = gj;
    }
    for (int c = 0; c < N; ++c) {  // Gauss-Jordan with partial pivoting
        int piv = c;
        for (int r = c + 1; r < N; ++r)
            if (std::fabs((double)A[r][c]) > std::fabs((double)A[piv][c])) piv = r;
        for (int k = 0; k <= N; ++k) std::swap(A[c][k], A[piv][k]);
        if (A[c][c] == 0) return;
        for (int r = 0; r < N; ++r) {
            if (r == c) continue;
            const long double f = A[r][c] / A[c][c];
            for (int k = c; k <= N; ++k) A[r][k] -= f * A[c][k];
        }
    }
    for (int i = 0; i < N; ++i) s.ig[i] = (double)(A[i][N] / A[i][i]);
    // a bound over the interval (r05; r04 sampled 4001 points)
    const double e0 = kb_guess_bound(p, s.ig, root((long double)R) * (1 + 1e-12L));
    s.ig_err = e0;
    s.ig_ok = M * e0 * e0 <= 1e-17 ? 1 : (e0 <= 1e-5 && M * M * M * e0 * e0 * e0 * e0 <= 1e-13 ? 2 : 0);
    if (!(s.ef <= 1e-11)) s.ig_ok = 0;
}

// A bound on the ray polynomials' error (r05; replaces
// a check on 16385 sample points).  The cells use the polynomials for s =
// r2 in [0, Sm], Sm = all_hi^2, i.e. for theta = theta*(sqrt(s)) in [0, Th],
// Th = theta*(all_hi).  In theta the errors are explicit functions, with no
// root to solve:
//   F1(theta) = C(s(theta)) - cos(theta),
//   F2(theta) = theta_d(theta) S(s(theta)) - sin(theta)   (= ru (S - S*)),
// s(theta) = theta_d(theta)^2, theta_d(theta) = theta (1 + k1 theta^2 + ...
// + k4 theta^8), C and S the fitted polynomials with their double
// coefficients.  [0, Th] is cut into kRayBoundCells pieces [m - r, m + r];
// on each, Taylor's theorem gives
//   |F(m + t)| <= sum_{k < J} |F_k| r^k + B_J r^J,
// F_k the Taylor coefficients at m, computed exactly up to rounding by
// truncated power-series (jet) arithmetic in long double, and B_J a bound on
// the J-th Taylor coefficient anywhere on the piece: the J-th coefficient of
// the majorant -- the same composition with every coefficient (p_i, k_i)
// replaced by its absolute value, taken at a = m + r -- plus 1 / J! for
// cos / sin.  (A polynomial in theta whose coefficients dominate another's
// in absolute value dominates every Taylor coefficient of it at any |xi| <=
// a; sums, products and compositions of such majorants are majorants.)  The
// jets' own rounding is covered by 2^-53 times the majorant's coefficient
// (>= 1000 long-double operations' worth of 2^-64 each).  To that the bound
// adds the device's evaluation error: Horner with FMAs in double over
// kRayPolyN terms, gamma_N |P|(Sm), plus one rounding of X = mx S.
namespace {
constexpr int kRayBoundCells = 256;
constexpr int kRayJ = 8;  // Taylor order of the remainder term
struct Jet {
    long double c[kRayJ + 1];
};
Jet jet_const(long double v) {
    Jet r{};
    r.c[0] = v;
    return r;
}
Jet jet_mul(const Jet& a, const Jet& b) {
    Jet r{};
    for (int i = 0; i <= kRayJ; ++i)
        for (int j = 0; i + j <= kRayJ; ++j) r.c[i + j] += a.c[i] * b.c[j];
    return r;
}
Jet jet_fma(const Jet& a, const Jet& b, long double c0) {  // a * b + c0
    Jet r = jet_mul(a, b);
    r.c[0] += c0;
    return r;
}
// theta_d and s = theta_d^2 as jets of theta = x + t (ABS: |k_i|, the majorant)
void jet_thd_s(const double* p, long double x, bool abs_, Jet& thd, Jet& s) {
    Jet th = jet_const(x);
    th.c[1] = 1;
    const Jet t2 = jet_mul(th, th);
    auto k = [&](int i) { return abs_ ? std::fabs((long double)p[i]) : (long double)p[i]; };
    Jet q = jet_const(k(7));
    q = jet_fma(q, t2, k(6));
    q = jet_fma(q, t2, k(5));
    q = jet_fma(q, t2, k(4));
    q = jet_fma(q, t2, 1.0L);
    thd = jet_mul(th, q);
    s = jet_mul(thd, thd);
}
Jet jet_poly(const double* c, const Jet& s, bool abs_, int n = kRayPolyN) {  // sum c_i s^i
    auto k = [&](int i) { return abs_ ? std::fabs((long double)c[i]) : (long double)c[i]; };
    Jet r = jet_const(k(n - 1));
    for (int i = n - 2; i >= 0; --i) r = jet_fma(r, s, k(i));
    return r;
}
}  // namespace

// The same bound for kb_fit_initial_guess's theta_0 = ru g(ru^2) (modes 1 /
// 2): F(theta) = theta_d(theta) g(s(theta)) - theta on [0, Th] (the initial
// error e0 against the root the Newton steps solve for), plus the device's
// evaluation of it (ru from rsq, s0 = RN(ru^2), Horner with FMAs over the 9
// coefficients, one rounding of ru g).
static double kb_guess_bound(const double* p, const double* ig, long double Th) {
    constexpr int NG = 9;
    const long double r = Th / (2 * kRayBoundCells);
    long double worst = 0;
    for (int cell = 0; cell < kRayBoundCells; ++cell) {
        const long double m = (2 * cell + 1) * r;
        Jet thd, s, thda, sa;
        jet_thd_s(p, m, false, thd, s);
        jet_thd_s(p, m + r, true, thda, sa);
        const Jet G = jet_mul(thd, jet_poly(ig, s, false, NG));
        const Jet Ga = jet_mul(thda, jet_poly(ig, sa, true, NG));
        long double rk = 1, b = 0;
        for (int k = 0; k < kRayJ; ++k) {
            const long double id = k == 0 ? m : (k == 1 ? 1.0L : 0.0L);  // theta's coefficients
            b += (std::fabs(G.c[k] - id) + 0x1p-53L * (Ga.c[k] + id)) * rk;
            rk *= r;
        }
        b += Ga.c[kRayJ] * rk;
        worst = std::fmax(worst, b);
    }
    Jet thd, s;
    jet_thd_s(p, Th, true, thd, s);
    const long double R = thd.c[0], Sm = s.c[0];
    Jet sj = jet_const(Sm);
    sj.c[1] = 1;
    const Jet Gm = jet_poly(ig, sj, true, NG);  // |g|(Sm), |g|'(Sm)
    const long double u = 0x1p-53L, gam = NG * u / (1 - NG * u);
    const long double dev = R * (gam * Gm.c[0] + Gm.c[1] * 4 * u * Sm + 4 * u * Gm.c[0]) + 2 * u * Th;
    return (double)(worst + dev) * (1 + 0x1p-40);
}

// max over [0, Th] of |F1| and |F2| (+ the device's evaluation error): a
// bound, not a sample; rp: [C_0..C_{N-1} | S_0..S_{N-1}]
static double kb_ray_poly_bound(const double* p, const double* rp, long double Th) {
    constexpr int N = kRayPolyN;
    long double jf = 1;  // J!
    for (int k = 2; k <= kRayJ; ++k) jf *= k;
    const long double r = Th / (2 * kRayBoundCells);
    long double worst = 0;
    for (int cell = 0; cell < kRayBoundCells; ++cell) {
        const long double m = (2 * cell + 1) * r;
        Jet thd, s;
        jet_thd_s(p, m, false, thd, s);
        const Jet Cj = jet_poly(rp, s, false);
        const Jet Sj = jet_mul(thd, jet_poly(rp + N, s, false));
        Jet thda, sa;
        jet_thd_s(p, m + r, true, thda, sa);
        const Jet Ca = jet_poly(rp, sa, true);
        const Jet Sa = jet_mul(thda, jet_poly(rp + N, sa, true));
        const long double cm = std::cos(m), sm = std::sin(m);
        // Taylor coefficients of cos / sin at m: derivatives cycle
        const long double dc[4] = {cm, -sm, -cm, sm}, ds[4] = {sm, cm, -sm, -cm};
        long double kf = 1, rk = 1, b1 = 0, b2 = 0;
        for (int k = 0; k < kRayJ; ++k) {
            if (k > 1) kf *= k;
            const long double f1 = Cj.c[k] - dc[k & 3] / kf;
            const long double f2 = Sj.c[k] - ds[k & 3] / kf;
            // rounding of the jets: 2^-53 of the majorant's coefficient
            b1 += (std::fabs(f1) + 0x1p-53L * (Ca.c[k] + 1 / kf)) * rk;
            b2 += (std::fabs(f2) + 0x1p-53L * (Sa.c[k] + 1 / kf)) * rk;
            rk *= r;
        }
        b1 += (Ca.c[kRayJ] + 1 / jf) * rk;
        b2 += (Sa.c[kRayJ] + 1 / jf) * rk;
        worst = std::fmax(worst, std::fmax(b1, b2));
    }
    // the device: Horner with FMAs over N terms in double, gamma_N |P|(Sm);
    // X = mx S rounds once more (|X| <= 1)
    Jet thd, s;
    jet_thd_s(p, Th, true, thd, s);
    const long double PC = jet_poly(rp, s, true).c[0];
    const long double PS = jet_mul(thd, jet_poly(rp + N, s, true)).c[0];
    const long double u = 0x1p-53L, gam = N * u / (1 - N * u);
    const long double dev = gam * std::fmax(PC, PS) + 2 * u;
    return (double)(worst + dev) * (1 + 0x1p-40);
}

// KB's certified-cell rays as polynomials in s = ru^2 on [0, all_hi^2]:
// C(s) = cos(theta*(ru)), S(s) = sin(theta*(ru)) / ru (S(0) = 1: theta*'(0)
// = 1).  Both are analytic in s (theta*(ru) / ru is an even analytic
// function of ru), so degree 16 interpolants at Chebyshev nodes, solved in
// long double (backward-stable elimination: the computed polynomials match
// the node values to ~1e-18, and the Chebyshev nodes keep them as close in
// between), reach rounding level.  The error is BOUNDED (kb_ray_poly_bound,
// r05): it must be <= 1e-13, and with the root-vs-reference distance ef, ef
// + error <= 1e-11 (the rays are held to 1e-10), or rp_ok stays 0 and
// ray_certified keeps its Newton form (which the ef gate of
// kb_fit_initial_guess covers in turn).
static void kb_fit_ray(const double* p, SegCert& s) {
    s.rp_ok = 0;
    const long double k1 = p[4], k2 = p[5], k3 = p[6], k4 = p[7];
    auto root = [&](long double ru) {
        long double t = ru;
        for (int i = 0; i < 80; ++i) {
            const long double t2 = t * t;
            const long double f = t * (1 + t2 * (k1 + t2 * (k2 + t2 * (k3 + t2 * k4)))) - ru;
            const long double fp = 1 + t2 * (3 * k1 + t2 * (5 * k2 + t2 * (7 * k3 + t2 * 9 * k4)));
            const long double d = f / fp;
            t -= d;
            if (std::fabs((double)d) < 1e-19) break;
        }
        return t;
    };
    auto cs = [&](long double sv, long double& C, long double& S) {
        const long double ru = std::sqrt(sv);
        const long double t = ru > 0 ? root(ru) : 0;
        C = std::cos(t);
        S = ru > 0 ? std::sin(t) / ru : 1;
    };
    const double R = s.all_hi;
    if (!(R > 1e-3) || !(R < 1.5707963267948966)) return;
    constexpr int N = kRayPolyN;
    const long double Sm = (long double)R * R;
    for (int which = 0; which < 2; ++which) {
        long double A[N][N + 1];
        for (int j = 0; j < N; ++j) {
            const long double sj = Sm * (1 + std::cos(kPi * (j + 0.5) / N)) / 2;
            long double C, S;
            cs(sj, C, S);
            long double pw = 1;
            for (int i = 0; i < N; ++i, pw *= sj) A[j][i] = pw;
            A[j][N] = which ? S : C;
        }
        for (int c = 0; c < N; ++c) {  // Gauss-Jordan with partial pivoting
            int piv = c;
            for (int r = c + 1; r < N; ++r)
                if (std::fabs((double)A[r][c]) > std::fabs((double)A[piv][c])) piv = r;
            for (int k = 0; k <= N; ++k) std::swap(A[c][k], A[piv][k]);
            if (A[c][c] == 0) return;
            for (int r = 0; r < N; ++r) {
                if (r == c) continue;
                const long double f = A[r][c] / A[c][c];
                for (int k = c; k <= N; ++k) A[r][k] -= f * A[c][k];
            }
        }
        for (int i = 0; i < N; ++i) s.rp[which * N + i] = (double)(A[i][N] / A[i][i]);
    }
    // theta*(all_hi), rounded up: the bound covers every cell's theta*
    const long double Th = root((long double)R) * (1 + 1e-12L);
    const double err = kb_ray_poly_bound(p, s.rp, Th);
    s.rp_err = err;
    s.rp_ok = std::isfinite(err) && err <= 1e-13 && s.ef + err <= 1e-11;
}

static SegCert kb_seg_cert(const double* p) {
    SegCert best{};
    best.all_lo = best.none_lo = INFINITY;
    best.all_hi = best.none_hi = -INFINITY;
    if (!(std::isfinite(p[4]) && std::isfinite(p[5]) && std::isfinite(p[6]) && std::isfinite(p[7])))
        return best;
    double cover = 0.0;
    for (double tmax : {1.99, 1.9, 1.8, 1.7, 1.62}) {
        const SegCert s = kb_seg_cert_on(p, tmax);
        if (!s.on) continue;
        const double c = std::fmax(s.all_hi, s.none_hi);
        if (c > cover) {
            cover = c;
            best = s;
        }
    }
    if (best.on && best.all_hi > best.all_lo) {
        kb_fit_initial_guess(p, best.ig[0], best);
        kb_fit_ray(p, best);
    }
    return best;
}

// kb_seg_cert costs ~1 ms of host time: memoised per distortion vector
// (thread-safe; a handful of cameras in practice)
static SegCert kb_seg_cert_cached(const double* p) {
    static std::mutex mu;
    static std::map<std::array<double, 4>, SegCert> memo;
    const std::array<double, 4> key{p[4], p[5], p[6], p[7]};
    {
        std::lock_guard<std::mutex> lock(mu);
        auto it = memo.find(key);
        if (it != memo.end()) return it->second;
    }
    const SegCert c = kb_seg_cert(p);
    std::lock_guard<std::mutex> lock(mu);
    if (memo.size() > 256) memo.clear();
    memo[key] = c;
    return c;
}

// ACM_TUNE_SAMPLE_CERT: -1 auto = on, 0 = off (every segment counted cell by cell)
static std::atomic<int> g_sample_cert{-1};
// ACM_TUNE_SAMPLE_WRITE: the segment write pass's layout (see its launch)
static std::atomic<int> g_sample_write{-1};

static SegCert seg_cert(const acm_camera& cam) {
    SegCert s{};
    s.all_lo = s.none_lo = INFINITY;
    s.all_hi = s.none_hi = -INFINITY;
    if (g_sample_cert == 0) return s;
    if (cam.model == ACM_KANNALA_BRANDT) return kb_seg_cert_cached(cam.params);
    // the closed-form models (and Pinhole, FOV) are certified per segment on
    // the device (seg_keep_iv); RadTan's Newton runs in (x, y): no certificate
    if (cam.model != ACM_RADTAN) s.on = 1;
    return s;
}

static int check_cam(const acm_camera* cam) {
    if (!cam) return fail(ACM_ERR_INVALID_ARGUMENT, "camera is NULL");
    const int p = acm_num_params(cam->model);
    if (p < 0) return fail(ACM_ERR_INVALID_MODEL, "unknown camera model id");
    if ((int)cam->num_params != p)
        return fail(ACM_ERR_INVALID_PARAMS, "camera num_params does not match the model");
    return ACM_SUCCESS;
}

static int check_layout(int layout) {
    if (layout != ACM_LAYOUT_AOS && layout != ACM_LAYOUT_SOA)
        return fail(ACM_ERR_INVALID_ARGUMENT, "layout must be ACM_LAYOUT_AOS or ACM_LAYOUT_SOA");
    return ACM_SUCCESS;
}

}  // namespace acm

using namespace acm;

// ====================================================================== C-ABI
extern "C" {

ACM_API int acm_num_params(int model) {
    switch (model) {
    case ACM_PINHOLE: return 4;
    case ACM_RADTAN: return 9;
    case ACM_KANNALA_BRANDT: return 8;
    case ACM_DOUBLE_SPHERE: return 6;
    case ACM_UCM: return 5;
    case ACM_EUCM: return 6;
    case ACM_FOV: return 5;
    default: return -1;
    }
}

ACM_API int acm_validate_params(const acm_camera* cam) {
    if (!cam) return fail(ACM_ERR_INVALID_ARGUMENT, "camera is NULL");
    const double* p = cam->params;
    // validation::validate_intrinsics (src/camera/mod.rs:362-371)
    if (p[0] <= 0.0 || p[1] <= 0.0) return ACM_FOCAL_LENGTH_MUST_BE_POSITIVE;
    if (!std::isfinite(p[2]) || !std::isfinite(p[3])) return ACM_PRINCIPAL_POINT_MUST_BE_FINITE;
    switch (cam->model) {
    case ACM_DOUBLE_SPHERE:  // double_sphere.rs:592-607
        if (p[4] <= 0.0 || p[4] > 1.0) return fail(ACM_INVALID_DISTORTION, "alpha must be in (0, 1]");
        if (!std::isfinite(p[5])) return fail(ACM_INVALID_DISTORTION, "xi must be finite");
        break;
    case ACM_UCM:  // ucm.rs:467-477
        if (!std::isfinite(p[4])) return fail(ACM_INVALID_DISTORTION, "alpha must be finite");
        break;
    case ACM_EUCM:  // eucm.rs:501-517
        if (!std::isfinite(p[4])) return fail(ACM_INVALID_DISTORTION, "alpha must be finite");
        if (!std::isfinite(p[5])) return fail(ACM_INVALID_DISTORTION, "beta must be finite");
        break;
    case ACM_FOV:  // fov.rs:457-468
        if (!std::isfinite(p[4]) || p[4] <= kEps || p[4] > 3.0)
            return fail(ACM_INVALID_DISTORTION, "w must be in range (epsilon, 3.0]");
        break;
    default: break;
    }
    return ACM_VALID;
}

ACM_API int acm_camera_init(acm_camera* cam, int model, const double* params, size_t num_params,
                            uint32_t width, uint32_t height) {
    if (!cam || (!params && num_params)) return fail(ACM_ERR_INVALID_ARGUMENT, "NULL argument");
    const int p = acm_num_params(model);
    if (p < 0) return fail(ACM_ERR_INVALID_MODEL, "unknown camera model id");
    if ((size_t)p != num_params)
        return fail(ACM_ERR_INVALID_PARAMS, "Expected " + std::to_string(p) + " parameters, got " +
                                                std::to_string(num_params));
    std::memset(cam, 0, sizeof(*cam));
    cam->model = model;
    cam->width = width;
    cam->height = height;
    cam->num_params = (uint32_t)p;
    for (int i = 0; i < p; ++i) cam->params[i] = params[i];
    if (model == ACM_PINHOLE || model == ACM_RADTAN) {  // pinhole.rs:80, rad_tan.rs:135
        const int v = acm_validate_params(cam);
        if (v != ACM_VALID) return fail(ACM_ERR_INVALID_PARAMS, "validate_params failed");
    }
    return ACM_SUCCESS;
}

ACM_API int acm_project(const acm_camera* cam, size_t n, const double* points_3d, int layout,
                        double* points_2d, uint8_t* status, double* jacobian, void* stream) {
    int rc = check_cam(cam);
    if (rc) return rc;
    const bool exact = (layout & ACM_EXACT_MATH) != 0;
    layout &= ~ACM_EXACT_MATH;
    if ((rc = check_layout(layout))) return rc;
    if (n == 0) return ACM_SUCCESS;
    if (!points_3d || !points_2d || !status) return fail(ACM_ERR_INVALID_ARGUMENT, "NULL buffer");
    hipStream_t s = (hipStream_t)stream;
    if (exact && (cam->model == ACM_KANNALA_BRANDT || cam->model == ACM_FOV)) {
        return dispatch_model(cam->model, [&](auto tag) -> int {
            using TagT = decltype(tag);
            const dim3 g(grid_for(n)), b(kBlock);
#define ACM_EX(L, WJ)                                                                          \
    hipLaunchKernelGGL((k_project_exact<TagT, L, WJ>), g, b, 0, s, prep(*cam), n, points_3d,     \
                       points_2d, status, jacobian)
            if (layout == ACM_LAYOUT_AOS) {
                if (jacobian) ACM_EX(ACM_LAYOUT_AOS, true); else ACM_EX(ACM_LAYOUT_AOS, false);
            } else {
                if (jacobian) ACM_EX(ACM_LAYOUT_SOA, true); else ACM_EX(ACM_LAYOUT_SOA, false);
            }
#undef ACM_EX
            return check_launch("acm_project (exact math)");
        });
    }
    int var = g_project_variant;
    if (var < 0) {
        const size_t out_bytes =
            n * (17 + (jacobian ? 16 * (size_t)acm_num_params(cam->model) : 0));
        var = (out_bytes > kNtThresholdBytes ? kVarNT : 0) | (g_nt_loads == 1 ? kVarNTL : 0);
    }
    const int P = acm_num_params(cam->model);
    (void)P;
    const bool align = jacobian && g_align_j != 0;
    if (align) {  // line-aligned store windows (always non-temporal: measured faster)
        return dispatch_model(cam->model, [&](auto tag) -> int {
            using TagT = decltype(tag);
            if (layout == ACM_LAYOUT_AOS)
                launch_al<TagT, ACM_LAYOUT_AOS, false>(s, prep(*cam), n, points_3d, nullptr, 0,
                                                       points_2d, status, jacobian);
            else
                launch_al<TagT, ACM_LAYOUT_SOA, false>(s, prep(*cam), n, points_3d, nullptr, 0,
                                                       points_2d, status, jacobian);
            return check_launch("acm_project");
        });
    }
    return dispatch_model(cam->model, [&](auto tag) -> int {
        using TagT = decltype(tag);
        auto launch = [&](auto lay_c, auto wj_c, auto var_c) {
            constexpr int L = decltype(lay_c)::value;
            constexpr bool WJ = decltype(wj_c)::value;
            constexpr int V = decltype(var_c)::value;
            unsigned blocks = grid_for(n);
            if ((V & kVarGrid) && blocks > 256u * 8u) blocks = 256u * 8u;
            hipLaunchKernelGGL((k_project<TagT, L, WJ, V>), dim3(blocks), dim3(kBlock), 0, s,
                               prep(*cam), n, points_3d, points_2d, status, jacobian);
        };
        auto by_var = [&](auto lay_c, auto wj_c) {
            switch (var) {
            case 1: launch(lay_c, wj_c, std::integral_constant<int, 1>{}); break;
            case 2: launch(lay_c, wj_c, std::integral_constant<int, 2>{}); break;
            case 3: launch(lay_c, wj_c, std::integral_constant<int, 3>{}); break;
            case 4: launch(lay_c, wj_c, std::integral_constant<int, 4>{}); break;
            case 5: launch(lay_c, wj_c, std::integral_constant<int, 5>{}); break;
            case 6: launch(lay_c, wj_c, std::integral_constant<int, 6>{}); break;
            case 7: launch(lay_c, wj_c, std::integral_constant<int, 7>{}); break;
            default: launch(lay_c, wj_c, std::integral_constant<int, 0>{}); break;
            }
        };
        using AOS = std::integral_constant<int, ACM_LAYOUT_AOS>;
        using SOA = std::integral_constant<int, ACM_LAYOUT_SOA>;
        if (layout == ACM_LAYOUT_AOS) {
            if (jacobian) by_var(AOS{}, std::true_type{});
            else by_var(AOS{}, std::false_type{});
        } else {
            if (jacobian) by_var(SOA{}, std::true_type{});
            else by_var(SOA{}, std::false_type{});
        }
        return check_launch("acm_project");
    });
}

ACM_API int acm_project_f32(const acm_camera* cam, size_t n, const float* points_3d, int layout,
                            float* points_2d, uint8_t* status, float* jacobian, void* stream) {
    int rc = check_cam(cam);
    if (rc) return rc;
    if ((rc = check_layout(layout))) return rc;
    if (n == 0) return ACM_SUCCESS;
    if (!points_3d || !points_2d || !status) return fail(ACM_ERR_INVALID_ARGUMENT, "NULL buffer");
    hipStream_t s = (hipStream_t)stream;
    const size_t out_bytes = n * (9 + (jacobian ? 8 * (size_t)acm_num_params(cam->model) : 0));
    const bool nt = out_bytes > kNtThresholdBytes;
    return dispatch_model(cam->model, [&](auto tag) -> int {
        using TagT = decltype(tag);
        const dim3 g(grid_for(n)), b(kBlock);
#define ACM_F32(L, WJ, NT)                                                                     \
    hipLaunchKernelGGL((k_project_f32<TagT, L, WJ, NT>), g, b, 0, s, prep(*cam), n, points_3d,       \
                       points_2d, status, jacobian)
        if (layout == ACM_LAYOUT_AOS) {
            if (jacobian) { if (nt) ACM_F32(ACM_LAYOUT_AOS, true, true); else ACM_F32(ACM_LAYOUT_AOS, true, false); }
            else { if (nt) ACM_F32(ACM_LAYOUT_AOS, false, true); else ACM_F32(ACM_LAYOUT_AOS, false, false); }
        } else {
            if (jacobian) { if (nt) ACM_F32(ACM_LAYOUT_SOA, true, true); else ACM_F32(ACM_LAYOUT_SOA, true, false); }
            else { if (nt) ACM_F32(ACM_LAYOUT_SOA, false, true); else ACM_F32(ACM_LAYOUT_SOA, false, false); }
        }
#undef ACM_F32
        return check_launch("acm_project_f32");
    });
}

ACM_API int acm_unproject(const acm_camera* cam, size_t n, const double* points_2d, double* rays,
                          int layout, uint8_t* status, void* stream) {
    int rc = check_cam(cam);
    if (rc) return rc;
    const bool refn = (layout & ACM_REFERENCE_NEWTON) != 0;
    layout &= ~ACM_REFERENCE_NEWTON;
    if ((rc = check_layout(layout))) return rc;
    if (n == 0) return ACM_SUCCESS;
    if (!points_2d || !rays || !status) return fail(ACM_ERR_INVALID_ARGUMENT, "NULL buffer");
    hipStream_t s = (hipStream_t)stream;
    return dispatch_model(cam->model, [&](auto tag) -> int {
        using TagT = decltype(tag);
        const dim3 g(grid_for(n)), b(kBlock);
        const bool nt = n * 25 > kNtThresholdBytes;  // rays + status written once
        const bool ntl = g_nt_loads_unproject == 1;
        // knob: -1 auto = 2 pixels per lane, AoS stores LDS-staged per
        // UnprojectStaged; 1 / 2 = pixels per lane with three 8-B stores per
        // AoS ray; 3 = 1 pixel per lane with LDS-staged stores
        // (tools/diag_unproject_ppt.py)
        const int ppt = g_unproject_ppt;
        const bool stg = (ppt == 3 || (ppt < 0 && UnprojectStaged<TagT>::on)) &&
                         (reinterpret_cast<uintptr_t>(rays) & 15u) == 0;
        auto go = [&](auto lay_c) {
            constexpr int L = decltype(lay_c)::value;
            auto pick = [&](auto ppt_c, auto stg_c) {
                constexpr int K = decltype(ppt_c)::value;
                constexpr bool PR = decltype(stg_c)::value && L == ACM_LAYOUT_AOS;
                auto kern = nt ? (ntl ? k_unproject<TagT, L, true, true, K, PR> : k_unproject<TagT, L, true, false, K, PR>)
                               : (ntl ? k_unproject<TagT, L, false, true, K, PR> : k_unproject<TagT, L, false, false, K, PR>);
                const dim3 gk((unsigned)((n + (size_t)kBlock * K - 1) / ((size_t)kBlock * K)));
                hipLaunchKernelGGL(kern, gk, b, 0, s, prep(*cam, refn, true), n, points_2d, rays, status);
            };
            using One = std::integral_constant<int, 1>;
            using Two = std::integral_constant<int, 2>;
            if (ppt == 1) pick(One{}, std::false_type{});
            else if (ppt == 3) {  // staged only on a 16-B aligned ray buffer (st2)
                if (stg) pick(One{}, std::true_type{});
                else pick(One{}, std::false_type{});
            }
            else if (stg) pick(Two{}, std::true_type{});
            else pick(Two{}, std::false_type{});
        };
        if (layout == ACM_LAYOUT_AOS) go(std::integral_constant<int, ACM_LAYOUT_AOS>{});
        else go(std::integral_constant<int, ACM_LAYOUT_SOA>{});
        return check_launch("acm_unproject");
    });
}

ACM_API int acm_project_unproject(const acm_camera* cam, size_t n, const double* points_3d,
                                  int layout, double* points_2d, uint8_t* status, double* rays,
                                  uint8_t* ray_status, void* stream) {
    int rc = check_cam(cam);
    if (rc) return rc;
    if (layout & (ACM_EXACT_MATH | ACM_REFERENCE_NEWTON)) {  // the two calls, in order
        rc = acm_project(cam, n, points_3d, layout & ~ACM_REFERENCE_NEWTON, points_2d, status,
                         nullptr, stream);
        if (rc) return rc;
        return acm_unproject(cam, n, points_2d, rays, layout & ~ACM_EXACT_MATH, ray_status,
                             stream);
    }
    if ((rc = check_layout(layout))) return rc;
    if (n == 0) return ACM_SUCCESS;
    if (!points_3d || !points_2d || !status || !rays || !ray_status)
        return fail(ACM_ERR_INVALID_ARGUMENT, "NULL buffer");
    hipStream_t s = (hipStream_t)stream;
    return dispatch_model(cam->model, [&](auto tag) -> int {
        using TagT = decltype(tag);
        const int knob = g_round_trip.load(std::memory_order_relaxed);
        const int ppt = knob < 0 ? RoundTripDefault<TagT>::ppt : (knob & 7);
        const int smode = knob < 0 ? 0 : (knob >> 3);
        const bool nt = n * 42 > kNtThresholdBytes;
        const bool want_stg = smode == 0 ? RoundTripDefault<TagT>::staged : smode == 1;
        const bool stg = want_stg && (reinterpret_cast<uintptr_t>(rays) & 15u) == 0;
        const dim3 b(kBlock);
        auto go = [&](auto lay_c, auto ppt_c, auto stg_c) {
            constexpr int L = decltype(lay_c)::value;
            constexpr int K = decltype(ppt_c)::value;
            constexpr bool ST = decltype(stg_c)::value && L == ACM_LAYOUT_AOS;
            const dim3 gk((unsigned)((n + (size_t)kBlock * K - 1) / ((size_t)kBlock * K)));
            auto kern = nt ? k_round_trip<TagT, L, true, K, ST> : k_round_trip<TagT, L, false, K, ST>;
            hipLaunchKernelGGL(kern, gk, b, 0, s, prep(*cam, false, true), n, points_3d, points_2d,
                               status, rays, ray_status);
        };
        using AOS = std::integral_constant<int, ACM_LAYOUT_AOS>;
        using One = std::integral_constant<int, 1>;
        using Two = std::integral_constant<int, 2>;
        using Four = std::integral_constant<int, 4>;
        auto by_ppt = [&](auto stg_c) {
            if (ppt == 1) go(AOS{}, One{}, stg_c);
            else if (ppt == 4) go(AOS{}, Four{}, stg_c);
            else go(AOS{}, Two{}, stg_c);
        };
        if (layout == ACM_LAYOUT_AOS) {
            if (stg) by_ppt(std::true_type{});
            else by_ppt(std::false_type{});
        } else {
            go(std::integral_constant<int, ACM_LAYOUT_SOA>{}, Two{}, std::false_type{});
        }
        return check_launch("acm_project_unproject");
    });
}

ACM_API int acm_residual_jacobian(const acm_camera* cam, size_t n, const double* points_3d,
                                  int layout, const double* points_2d_obs, int invalid_policy,
                                  double* residual, double* jacobian, uint8_t* status,
                                  void* stream) {
    int rc = check_cam(cam);
    if (rc) return rc;
    if ((rc = check_layout(layout))) return rc;
    if (invalid_policy != ACM_INVALID_SKIP && invalid_policy != ACM_INVALID_SENTINEL)
        return fail(ACM_ERR_INVALID_ARGUMENT, "invalid_policy must be SKIP or SENTINEL");
    if (n == 0) return ACM_SUCCESS;
    if (!points_3d || !points_2d_obs || !residual)
        return fail(ACM_ERR_INVALID_ARGUMENT, "NULL buffer");
    hipStream_t s = (hipStream_t)stream;
    return dispatch_model(cam->model, [&](auto tag) -> int {
        using TagT = decltype(tag);
        const dim3 g(grid_for(n)), b(kBlock);
        const size_t out_bytes =
            n * (17 + (jacobian ? 16 * (size_t)acm_num_params(cam->model) : 0));
        const bool nt = g_residual_nt < 0 ? out_bytes > kNtThresholdBytes : g_residual_nt == 1;
        const bool align = jacobian && g_align_j != 0;
        if (align) {  // line-aligned store windows (always non-temporal: measured faster)
            if (layout == ACM_LAYOUT_AOS)
                launch_al<TagT, ACM_LAYOUT_AOS, true>(s, prep(*cam), n, points_3d, points_2d_obs,
                                                      invalid_policy, residual, status, jacobian);
            else
                launch_al<TagT, ACM_LAYOUT_SOA, true>(s, prep(*cam), n, points_3d, points_2d_obs,
                                                      invalid_policy, residual, status, jacobian);
            return check_launch("acm_residual_jacobian");
        }
#define ACM_LAUNCH_RES(L, WJ)                                                                   \
    do {                                                                                        \
        if (nt)                                                                                 \
            hipLaunchKernelGGL((k_residual<TagT, L, WJ, true>), g, b, 0, s, prep(*cam), n, points_3d, \
                               points_2d_obs, invalid_policy, residual, jacobian, status);      \
        else                                                                                    \
            hipLaunchKernelGGL((k_residual<TagT, L, WJ, false>), g, b, 0, s, prep(*cam), n,           \
                               points_3d, points_2d_obs, invalid_policy, residual, jacobian,    \
                               status);                                                         \
    } while (0)
        if (layout == ACM_LAYOUT_AOS) {
            if (jacobian) ACM_LAUNCH_RES(ACM_LAYOUT_AOS, true);
            else ACM_LAUNCH_RES(ACM_LAYOUT_AOS, false);
        } else {
            if (jacobian) ACM_LAUNCH_RES(ACM_LAYOUT_SOA, true);
            else ACM_LAUNCH_RES(ACM_LAYOUT_SOA, false);
        }
#undef ACM_LAUNCH_RES
        return check_launch("acm_residual_jacobian");
    });
}

ACM_API size_t acm_normal_equations_workspace_size(int model, size_t n) {
    const int P = acm_num_params(model);
    if (P < 0) return 0;
    const int D = P - 4;
    const int K = 10 + 5 * D + D * (D + 1) / 2 + 2;  // = NE<P>::K
    return ((size_t)nq_blocks(n) + 1) * (size_t)K * sizeof(double);
}

extern "C++" {
namespace acm {
// flag / seq: see k_ne_finish_cols / k_ne_publish (the LM's polled path in solver.hip)
// cells / grid (r06): the observations as grid cells (ObsCells) instead of
// pixels; the kernel is then the per-model default (NE_WAVES / NE_UNROLL do
// not apply), which is what makes its sums the pixel form's bit for bit.
int check_cell_grid(const acm_cell_grid* grid) {
    if (!grid) return fail(ACM_ERR_INVALID_ARGUMENT, "NULL cell grid");
    if (!grid->num_cells_x || !grid->num_cells_y || !grid->width || !grid->height ||
        (uint64_t)grid->num_cells_x * grid->num_cells_y > 0xFFFFFFFFull)
        return fail(ACM_ERR_INVALID_ARGUMENT, "cell grid: empty, or more than 2^32 - 1 cells");
    return ACM_SUCCESS;
}
static ObsCells obs_cells(const uint32_t* cells, const acm_cell_grid& g) {
    ObsCells o;
    o.p = cells;
    o.ncx = g.num_cells_x;
    o.inv_ncx = 1.0 / (double)g.num_cells_x;
    o.cw = (double)g.width / (double)g.num_cells_x;   // point_sampling.rs:57-58, as
    o.ch = (double)g.height / (double)g.num_cells_y;  // acm_sample_points_ex computes them
    return o;
}
// (r06) whether normal_equations_impl can run the pre-queued evaluation
// (k_normal_eq_dev, instantiated for the default configuration only): AoS
// points, the default waves / unroll knobs and NT loads on
bool ne_dev_ok(int layout) {
    return layout == ACM_LAYOUT_AOS && g_nt_loads != 0 && g_ne_waves == 0 && g_ne_unroll == 0;
}

int normal_equations_impl(const acm_camera* cam, size_t n, const double* points_3d, int layout,
                          const double* points_2d_obs, int invalid_policy, double* result,
                          void* workspace, size_t workspace_bytes, void* stream,
                          unsigned long long* flag, unsigned long long seq,
                          unsigned int* ticket, const uint32_t* cells,
                          const acm_cell_grid* grid, const LmDoorbell* db) {
    int rc = check_cam(cam);
    if (rc) return rc;
    if ((rc = check_layout(layout))) return rc;
    if (invalid_policy != ACM_INVALID_SKIP && invalid_policy != ACM_INVALID_SENTINEL)
        return fail(ACM_ERR_INVALID_ARGUMENT, "invalid_policy must be SKIP or SENTINEL");
    if (cells && (rc = check_cell_grid(grid))) return rc;
    if (!result || !workspace || (n && (!points_3d || !(cells ? (const void*)cells
                                                               : (const void*)points_2d_obs))))
        return fail(ACM_ERR_INVALID_ARGUMENT, "NULL buffer");
    if (workspace_bytes < acm_normal_equations_workspace_size(cam->model, n))
        return fail(ACM_ERR_WORKSPACE_TOO_SMALL, "normal-equations workspace too small");
    hipStream_t s = (hipStream_t)stream;
    const int nb_max = nq_blocks(n);
    return dispatch_model(cam->model, [&](auto tag) -> int {
        using TagT = decltype(tag);
        using M = typename TagT::template type<double>;
        constexpr int P = M::P;
        double* parts = (double*)workspace;
        int nb = nb_max;
        using Def = NeDefault<TagT>;
        const int wv0 = g_ne_waves, un0 = g_ne_unroll;
        const int wv = wv0 ? wv0 : Def::W;
        const int un = un0 ? un0 : Def::U;
        auto go_cells = [&](auto lay_c) {
            constexpr int LAY = decltype(lay_c)::value;
            const bool ntl = g_nt_loads != 0;
            auto kern = ntl ? k_normal_eq<TagT, LAY, Def::W, Def::U, true, ObsCells>
                            : k_normal_eq<TagT, LAY, Def::W, Def::U, false, ObsCells>;
            // the pixel form's workgroup count (its occupancy, not the cell
            // form's): the same grid-stride partition of the points, so the
            // same summation order and the same bits
            auto kpix = ntl ? k_normal_eq<TagT, LAY, Def::W, Def::U, true, ObsPixels>
                            : k_normal_eq<TagT, LAY, Def::W, Def::U, false, ObsPixels>;
            const int cap = resident_blocks(reinterpret_cast<const void*>(kpix));
            if (nb > cap) nb = cap;
            if (db) {  // (r06) the pre-queued LM evaluation: AoS, NT loads (ne_dev_ok)
                hipLaunchKernelGGL((k_normal_eq_dev<TagT, ACM_LAYOUT_AOS, Def::W, Def::U, true,
                                                    ObsCells>),
                                   dim3(nb), dim3(kBlock), 0, s, *db, n, points_3d,
                                   obs_cells(cells, *grid), invalid_policy, parts);
                return;
            }
            hipLaunchKernelGGL(kern, dim3(nb), dim3(kBlock), 0, s, prep(*cam), n, points_3d,
                               obs_cells(cells, *grid), invalid_policy, parts);
        };
        auto go = [&](auto lay_c, auto w_c) {
            constexpr int LAY = decltype(lay_c)::value, W = decltype(w_c)::value;
            const bool ntl = g_nt_loads != 0;
            auto kern = ntl ? k_normal_eq<TagT, LAY, W, 1, true> : k_normal_eq<TagT, LAY, W, 1, false>;
            if (un == 2) kern = ntl ? k_normal_eq<TagT, LAY, W, 2, true> : k_normal_eq<TagT, LAY, W, 2, false>;
            if (un == 3) kern = ntl ? k_normal_eq<TagT, LAY, W, 3, true> : k_normal_eq<TagT, LAY, W, 3, false>;
            // 4, 5: loads 3, 4 steps ahead (KB only; others take 3)
            if constexpr (std::is_same<TagT, Tag<KannalaBrandt>>::value) {
                if (un == 4) kern = ntl ? k_normal_eq<TagT, LAY, W, 4, true> : k_normal_eq<TagT, LAY, W, 4, false>;
                if (un == 5) kern = ntl ? k_normal_eq<TagT, LAY, W, 5, true> : k_normal_eq<TagT, LAY, W, 5, false>;
            } else {
                if (un >= 4) kern = ntl ? k_normal_eq<TagT, LAY, W, 3, true> : k_normal_eq<TagT, LAY, W, 3, false>;
            }
            const int cap = resident_blocks(reinterpret_cast<const void*>(kern));
            if (nb > cap) nb = cap;
            if (db) {  // (ne_dev_ok: the default W, U; AoS; NT loads)
                hipLaunchKernelGGL((k_normal_eq_dev<TagT, ACM_LAYOUT_AOS, Def::W, Def::U, true>),
                                   dim3(nb), dim3(kBlock), 0, s, *db, n, points_3d,
                                   ObsPixels{points_2d_obs}, invalid_policy, parts);
                return;
            }
            hipLaunchKernelGGL(kern, dim3(nb), dim3(kBlock), 0, s, prep(*cam), n, points_3d,
                               ObsPixels{points_2d_obs}, invalid_policy, parts);
        };
        auto by_waves = [&](auto lay_c) {
            if (db) {  // the default kernel's partition (nb), then the doorbell form
                if constexpr (Def::W == 1) go(lay_c, std::integral_constant<int, 1>{});
                else if constexpr (Def::W == 4) go(lay_c, std::integral_constant<int, 4>{});
                else go(lay_c, std::integral_constant<int, 3>{});
                return;
            }
            switch (wv) {
            case 1: go(lay_c, std::integral_constant<int, 1>{}); break;
            case 4: go(lay_c, std::integral_constant<int, 4>{}); break;
            default: go(lay_c, std::integral_constant<int, 3>{}); break;
            }
        };
        if (cells) {
            if (layout == ACM_LAYOUT_AOS) go_cells(std::integral_constant<int, ACM_LAYOUT_AOS>{});
            else go_cells(std::integral_constant<int, ACM_LAYOUT_SOA>{});
        } else if (layout == ACM_LAYOUT_AOS) {
            by_waves(std::integral_constant<int, ACM_LAYOUT_AOS>{});
        } else {
            by_waves(std::integral_constant<int, ACM_LAYOUT_SOA>{});
        }
        // (r04) with a ticket the finish kernel's last workgroup releases
        // the completion word itself: one launch fewer per LM evaluation
        // (host loop 1.275 -> 1.252 ms at config 3, three interleaved runs,
        // profiles/r04t2_lm_ticket_ab.log)
        unsigned int* tk = ticket;
        if (flag) {
            hipLaunchKernelGGL((k_ne_finish_cols<P, true>), dim3(NE<P>::K + 1), dim3(kBlock), 0, s,
                               parts, nb, result, tk, flag, seq);
            if (!tk) hipLaunchKernelGGL(k_ne_publish, dim3(1), dim3(1), 0, s, flag, seq);
        } else {
            hipLaunchKernelGGL((k_ne_finish_cols<P, false>), dim3(NE<P>::K + 1), dim3(kBlock), 0, s,
                               parts, nb, result, nullptr, nullptr, 0ull);
        }
        return check_launch("acm_normal_equations");
    });
}

}  // namespace acm
}  // extern "C++"

ACM_API int acm_normal_equations(const acm_camera* cam, size_t n, const double* points_3d,
                                 int layout, const double* points_2d_obs, int invalid_policy,
                                 double* result, void* workspace, size_t workspace_bytes,
                                 void* stream) {
    return acm::normal_equations_impl(cam, n, points_3d, layout, points_2d_obs, invalid_policy,
                                      result, workspace, workspace_bytes, stream, nullptr, 0,
                                      nullptr, nullptr, nullptr, nullptr);
}

ACM_API int acm_normal_equations_cells(const acm_camera* cam, size_t n, const double* points_3d,
                                       int layout, const uint32_t* cells,
                                       const acm_cell_grid* grid, int invalid_policy,
                                       double* result, void* workspace, size_t workspace_bytes,
                                       void* stream) {
    if (n && !cells) return fail(ACM_ERR_INVALID_ARGUMENT, "NULL buffer");
    if (!cells) {  // n = 0: nothing is read
        static const uint32_t none = 0;
        cells = &none;
    }
    return acm::normal_equations_impl(cam, n, points_3d, layout, nullptr, invalid_policy,
                                      result, workspace, workspace_bytes, stream, nullptr, 0,
                                      nullptr, cells, grid, nullptr);
}

ACM_API size_t acm_reprojection_stats_workspace_size(size_t n) {
    // errors (N) + per-workgroup partials (nb * 7) + totals (7)
    const size_t nb = (size_t)ne_blocks(n);
    return (n + nb * kReprojW + kReprojW) * sizeof(double);
}

// hparts != nullptr: also the median's first histogram per workgroup
// (k_reproj_pass1<HIST>); *nb_out = the workgroups launched
static SelWs sel_ws(void* workspace);
// median_ws != nullptr: the finish kernel also initialises that median
// workspace for n_valid (acm_reprojection_error)
static int reprojection_stats_impl(const acm_camera* cam, size_t n, const double* points_3d,
                                   int layout, const double* points_2d, double* result,
                                   double* errors, void* workspace, hipStream_t s,
                                   unsigned int* hparts, int* nb_out,
                                   void* median_ws = nullptr, const uint32_t* cells = nullptr,
                                   const acm_cell_grid* grid = nullptr) {
    int rc = check_cam(cam);
    if (rc) return rc;
    if ((rc = check_layout(layout))) return rc;
    const int nb_max = ne_blocks(n);
    double* ws = (double*)workspace;
    double* errs = errors ? errors : ws;
    double* p1 = ws + n;
    double* tot = p1 + (size_t)nb_max * kReprojW;
    const bool ntl = g_nt_loads != 0;
    return dispatch_model(cam->model, [&](auto tag) -> int {
        using TagT = decltype(tag);
        int nb1 = nb_max;
        const bool nts = n * sizeof(double) > kNtThresholdBytes;
        auto go = [&](auto lay_c) {
            constexpr int LAY = decltype(lay_c)::value;
            auto kern = ntl ? k_reproj_pass1<TagT, LAY, true, false, false>
                            : k_reproj_pass1<TagT, LAY, false, false, false>;
            if (nts) kern = ntl ? k_reproj_pass1<TagT, LAY, true, true, false>
                                : k_reproj_pass1<TagT, LAY, false, true, false>;
            if (hparts) {
                kern = ntl ? k_reproj_pass1<TagT, LAY, true, false, true>
                           : k_reproj_pass1<TagT, LAY, false, false, true>;
                if (nts) kern = ntl ? k_reproj_pass1<TagT, LAY, true, true, true>
                                    : k_reproj_pass1<TagT, LAY, false, true, true>;
            }
            nb1 = std::min(nb1, resident_blocks(reinterpret_cast<const void*>(kern)));
            if (cells) {  // (r06) the cell form, on the pixel form's partition
                auto kc = ntl ? k_reproj_pass1<TagT, LAY, true, false, false, ObsCells>
                              : k_reproj_pass1<TagT, LAY, false, false, false, ObsCells>;
                if (nts) kc = ntl ? k_reproj_pass1<TagT, LAY, true, true, false, ObsCells>
                                  : k_reproj_pass1<TagT, LAY, false, true, false, ObsCells>;
                if (hparts) {
                    kc = ntl ? k_reproj_pass1<TagT, LAY, true, false, true, ObsCells>
                             : k_reproj_pass1<TagT, LAY, false, false, true, ObsCells>;
                    if (nts) kc = ntl ? k_reproj_pass1<TagT, LAY, true, true, true, ObsCells>
                                      : k_reproj_pass1<TagT, LAY, false, true, true, ObsCells>;
                }
                hipLaunchKernelGGL(kc, dim3(nb1), dim3(kBlock), 0, s, prep(*cam), n, points_3d,
                                   acm::obs_cells(cells, *grid), errs, p1, hparts);
            } else {
                hipLaunchKernelGGL(kern, dim3(nb1), dim3(kBlock), 0, s, prep(*cam), n, points_3d,
                                   ObsPixels{points_2d}, errs, p1, hparts);
            }
        };
        if (layout == ACM_LAYOUT_AOS) go(std::integral_constant<int, ACM_LAYOUT_AOS>{});
        else go(std::integral_constant<int, ACM_LAYOUT_SOA>{});
        hipLaunchKernelGGL(k_reproj_finish, dim3(1), dim3(kBlock), 0, s, p1, nb1, tot, result,
                           median_ws ? sel_ws(median_ws) : SelWs{});
        if (nb_out) *nb_out = nb1;
        return check_launch("acm_reprojection_stats");
    });
}

ACM_API int acm_reprojection_stats(const acm_camera* cam, size_t n, const double* points_3d,
                                   int layout, const double* points_2d, double* result,
                                   double* errors, void* workspace, size_t workspace_bytes,
                                   void* stream) {
    if (!result || !workspace || (n && (!points_3d || !points_2d)))
        return fail(ACM_ERR_INVALID_ARGUMENT, "NULL buffer");
    if (workspace_bytes < acm_reprojection_stats_workspace_size(n))
        return fail(ACM_ERR_WORKSPACE_TOO_SMALL, "reprojection-stats workspace too small");
    return reprojection_stats_impl(cam, n, points_3d, layout, points_2d, result, errors,
                                   workspace, (hipStream_t)stream, nullptr, nullptr);
}

ACM_API size_t acm_error_stats_workspace_size(size_t n) {
    return ((size_t)ne_blocks(n) * kReprojW + kReprojW) * sizeof(double);
}

ACM_API int acm_error_stats(size_t n, const double* errors, double* result, void* workspace,
                            size_t workspace_bytes, void* stream) {
    if (!result || !workspace || (n && !errors)) return fail(ACM_ERR_INVALID_ARGUMENT, "NULL buffer");
    if (workspace_bytes < acm_error_stats_workspace_size(n))
        return fail(ACM_ERR_WORKSPACE_TOO_SMALL, "error-stats workspace too small");
    hipStream_t s = (hipStream_t)stream;
    double* p1 = (double*)workspace;
    int nb = ne_blocks(n);
    nb = std::max(1, std::min(nb, resident_blocks(reinterpret_cast<const void*>(k_errstats_pass1))));
    double* tot = p1 + (size_t)nb * kReprojW;
    hipLaunchKernelGGL(k_errstats_pass1, dim3(nb), dim3(kBlock), 0, s, n, errors, p1);
    hipLaunchKernelGGL(k_reproj_finish, dim3(1), dim3(kBlock), 0, s, p1, nb, tot, result, SelWs{});
    return check_launch("acm_error_stats");
}

ACM_API int acm_reprojection_stats_merge(size_t nparts, const double* parts, double* result) {
    if (!result || (nparts && !parts)) return fail(ACM_ERR_INVALID_ARGUMENT, "NULL argument");
    // parts: nparts x [rmse, min, max, mean, stddev, n_valid, sum, sumsq]
    // (acm_reprojection_stats results of disjoint shards), merged in order:
    // sums add, extrema combine, (n, mean, M2 = n stddev^2) by Chan's update
    double n = 0.0, sum = 0.0, sumsq = 0.0, mn = INFINITY, mx = -INFINITY, m = 0.0, M2 = 0.0;
    for (size_t r = 0; r < nparts; ++r) {
        const double* p = parts + 8 * r;
        const double nr = p[5];
        if (!(nr > 0.0)) continue;
        sum += p[6];
        sumsq += p[7];
        mn = std::fmin(mn, p[1]);
        mx = std::fmax(mx, p[2]);
        const double mr = p[3], M2r = p[4] * p[4] * nr;
        if (n == 0.0) {
            n = nr; m = mr; M2 = M2r;
        } else {
            const double t = n + nr, d = mr - m;
            m = m + d * (nr / t);
            M2 = M2 + M2r + d * d * (n * (nr / t));
            n = t;
        }
    }
    result[0] = std::sqrt(sumsq / n);
    result[1] = mn;
    result[2] = mx;
    result[3] = sum / n;  // error_metrics.rs:88-89: sum / n
    result[4] = std::sqrt(std::fmax(M2, 0.0) / n);
    result[5] = n;
    result[6] = sum;
    result[7] = sumsq;
    return ACM_SUCCESS;
}

ACM_API int acm_sample_points_grid(uint32_t width, uint32_t height, size_t n_requested,
                                   uint32_t* num_cells_x, uint32_t* num_cells_y) {
    if (!num_cells_x || !num_cells_y) return fail(ACM_ERR_INVALID_ARGUMENT, "NULL argument");
    const double w = (double)width, h = (double)height;  // point_sampling.rs:50-54
    const double fx = std::round(std::sqrt((double)n_requested * (w / h)));
    const double fy = std::round(std::sqrt((double)n_requested * (h / w)));
    if (!(fx >= 1.0) || !(fy >= 1.0) || fx > 4e9 || fy > 4e9)
        return fail(ACM_ERR_INVALID_ARGUMENT, "sample grid is empty or too large");
    *num_cells_x = (uint32_t)fx;
    *num_cells_y = (uint32_t)fy;
    return ACM_SUCCESS;
}

// Workspace words of every path: two-pass = counts + offsets (2 per
// kSampleCells tile); single pass = one status word per kFusedCells tile (+1);
// segment path = one u32 count per 64-cell segment + block sums and block
// offsets (2 per kSegBlockCells workgroup).
static size_t sample_ws_words(size_t cells) {
    const size_t nb = cells ? (cells + kSampleCells - 1) / kSampleCells : 1;
    const size_t nt = cells ? (cells + kFusedCells - 1) / kFusedCells : 1;
    const size_t nseg = cells ? (cells + kSegCells - 1) / kSegCells : 1;
    const size_t nsb = cells ? (cells + kSegBlockCells - 1) / kSegBlockCells : 1;
    return std::max(std::max(2 * nb, nt + 1), (nseg + 1) / 2 + 2 * nsb);
}

ACM_API size_t acm_sample_points_workspace_size(const acm_camera* cam, size_t n_requested) {
    uint32_t ncx, ncy;
    if (!cam || acm_sample_points_grid(cam->width, cam->height, n_requested, &ncx, &ncy))
        return 0;
    return sample_ws_words((size_t)ncx * ncy) * sizeof(uint64_t);
}

// The cell form of the kept pixels for the sample_points paths whose write
// kernels do not emit it (ACM_TUNE_SAMPLE_FUSED 0-3): j = u / cw - 0.5 and
// i = v / ch - 0.5 rounded -- exact, since u = RN((j + 0.5) cw) is within
// half an ulp of the centre and the cells are a whole cw apart.
__global__ __launch_bounds__(kBlock) void k_cells_of_uv(const double* __restrict__ uv,
                                                        const uint64_t* __restrict__ counts,
                                                        Grid g, uint32_t* __restrict__ cells_out) {
    const size_t n = counts[0];
    for (size_t t = (size_t)blockIdx.x * kBlock + threadIdx.x; t < n;
         t += (size_t)gridDim.x * kBlock) {
        const double2 p = ld2<false>(uv + 2 * t);
        const uint32_t j = (uint32_t)rint(p.x / g.cw - 0.5);
        const uint32_t i = (uint32_t)rint(p.y / g.ch - 0.5);
        cells_out[t] = i * g.ncx + j;
    }
}

static int sample_points_impl(const acm_camera* cam, size_t n_requested, size_t cell_begin,
                              size_t cell_end, int flags, double* points_2d_out,
                              double* points_3d_out, uint32_t* cells_out, uint64_t* counts,
                              void* workspace, size_t workspace_bytes, void* stream);

ACM_API int acm_sample_points_ex(const acm_camera* cam, size_t n_requested, size_t cell_begin,
                                 size_t cell_end, int flags, double* points_2d_out,
                                 double* points_3d_out, uint64_t* counts, void* workspace,
                                 size_t workspace_bytes, void* stream) {
    return sample_points_impl(cam, n_requested, cell_begin, cell_end, flags, points_2d_out,
                              points_3d_out, nullptr, counts, workspace, workspace_bytes, stream);
}

// (r06) the same, also writing each kept point's cell c = i * ncx + j
// (cells_out: device uint32[cap]) for the cell forms of the solver
// (acm_lm_optimize_cells); the grid must have at most 2^32 - 1 cells
ACM_API int acm_sample_points_cells(const acm_camera* cam, size_t n_requested, size_t cell_begin,
                                    size_t cell_end, int flags, double* points_2d_out,
                                    double* points_3d_out, uint32_t* cells_out, uint64_t* counts,
                                    void* workspace, size_t workspace_bytes, void* stream) {
    if (!cells_out) return fail(ACM_ERR_INVALID_ARGUMENT, "NULL buffer");
    return sample_points_impl(cam, n_requested, cell_begin, cell_end, flags, points_2d_out,
                              points_3d_out, cells_out, counts, workspace, workspace_bytes,
                              stream);
}

static int sample_points_impl(const acm_camera* cam, size_t n_requested, size_t cell_begin,
                              size_t cell_end, int flags, double* points_2d_out,
                              double* points_3d_out, uint32_t* cells_out, uint64_t* counts,
                              void* workspace, size_t workspace_bytes, void* stream) {
    int rc = check_cam(cam);
    if (rc) return rc;
    if (flags & ~ACM_REFERENCE_NEWTON)
        return fail(ACM_ERR_INVALID_ARGUMENT, "flags must be 0 or ACM_REFERENCE_NEWTON");
    const bool refn = (flags & ACM_REFERENCE_NEWTON) != 0;
    uint32_t ncx, ncy;
    if ((rc = acm_sample_points_grid(cam->width, cam->height, n_requested, &ncx, &ncy))) return rc;
    const size_t total = (size_t)ncx * ncy;
    if (cell_end > total) cell_end = total;
    if (cell_begin > cell_end) return fail(ACM_ERR_INVALID_ARGUMENT, "cell_begin > cell_end");
    if (!points_2d_out || !points_3d_out || !counts || !workspace)
        return fail(ACM_ERR_INVALID_ARGUMENT, "NULL buffer");
    const size_t cells = cell_end - cell_begin;
    const size_t nb = cells ? (cells + kSampleCells - 1) / kSampleCells : 1;
    const size_t nt = cells ? (cells + kFusedCells - 1) / kFusedCells : 1;
    if (workspace_bytes < sample_ws_words(cells) * sizeof(uint64_t))
        return fail(ACM_ERR_WORKSPACE_TOO_SMALL, "sample_points workspace too small");
    if (nt > 0x7fffffffull) return fail(ACM_ERR_INVALID_ARGUMENT, "sample grid too large");
    if (cells_out && total > 0xFFFFFFFFull)
        return fail(ACM_ERR_INVALID_ARGUMENT, "cell form: the grid has more than 2^32 - 1 cells");
    Grid g;
    g.ncx = ncx;
    g.ncy = ncy;
    g.cw = (double)cam->width / (double)ncx;  // point_sampling.rs:57
    g.ch = (double)cam->height / (double)ncy;
    g.cell0 = cell_begin;
    const int pat = g_sample_patience;
    g.patience = pat < 0 ? kLbPatience : pat;
    hipStream_t s = (hipStream_t)stream;
    CamArg ca = prep(*cam, refn, true);
    if (cam->model == ACM_KANNALA_BRANDT && !refn) {
        // the certified kept interval + initial guess for ray_certified, in
        // every sample_points path alike (same rays whichever kernels run)
        const SegCert kc = kb_seg_cert_cached(cam->params);
        if (kc.on && (kc.ig_ok || kc.rp_ok) && kc.all_hi > kc.all_lo) {
            ca.kc[0] = kc.all_lo;
            ca.kc[1] = kc.all_hi;
            // ray_certified: 3 = the ray polynomials, else its Newton steps
            ca.kc[2] = kc.rp_ok ? 3 : kc.ig_ok;
            for (int i = 0; i < 9; ++i) ca.kc[3 + i] = kc.ig[i];
            for (int i = 0; i < 2 * kRayPolyN; ++i) ca.rp[i] = kc.rp[i];
        }
    }
    if (!cells) {  // nothing to launch: counts = [0 kept, 0 cells]
        if (hipMemsetAsync(counts, 0, 2 * sizeof(uint64_t), s) != hipSuccess)
            return check_launch("acm_sample_points: counts");
        return ACM_SUCCESS;
    }
    // (plain stores: non-temporal ones measured slower for these compacted
    // outputs, 1.41 -> 1.47 ms at 1e8 KB cells, profiles/r02_diag_sample_phases.log)
    int mode = g_sample_fused;
    // RadTan has no keep certificate (its Newton runs in (x, y), not on r2):
    // the segment path would count every cell with the full Newton, so auto
    // keeps the single pass for it (1.32 vs 1.78 ms at 1e8 cells,
    // profiles/r03c_diag_sample.log)
    // ... and the speculative segment path beats both when (as for the
    // sample camera) nothing or little is dropped: 0.99 vs 1.32 ms at 1e8
    // cells (profiles/r03m_diag_sample.log)
    if (mode < 0 && cam->model == ACM_RADTAN) mode = 4;
    const bool spec = mode == 4;
    // KB's certified rays from the ray polynomials (TagKbPoly) when the host
    // fit holds; the count kernels take SampleTag<>::count either way
    const bool poly = cam->model == ACM_KANNALA_BRANDT && ca.kc[2] == 3.0;
    auto dispatch_sample = [&](auto&& f) -> int {
        if (poly) return f(TagKbPoly{});
        return dispatch_model(cam->model, f);
    };
    if (mode < 0 || spec) {  // segment two-pass (default) / speculative segments
        const size_t nseg = (cells + kSegCells - 1) / kSegCells;
        const size_t nsb = (cells + kSegBlockCells - 1) / kSegBlockCells;
        uint32_t* seg_cnt = (uint32_t*)workspace;
        uint64_t* blk_sum = (uint64_t*)workspace + (nseg + 1) / 2;
        uint64_t* blk_off = blk_sum + nsb;
        const SegCert cert = seg_cert(*cam);
        return dispatch_sample([&](auto tag) -> int {
            using TagT = decltype(tag);
            using TagC = typename SampleTag<TagT>::count;
            // ACM_TUNE_SAMPLE_WRITE: segments per write wave and order
            // (-1 auto = 16 interleaved; 1 = 64 contiguous, 2 = 16
            // interleaved, 3 = 4 interleaved, 4 = 16 contiguous, 5 = 16
            // interleaved with non-temporal stores)
            // auto: 4 segments per wave for the cheapest unprojections (UCM,
            // EUCM, FOV: 0.71 vs 0.84 ms at 1e8 cells) and, since its rays
            // come from the LDS-staged polynomials (r04), for KB (0.745 vs
            // 0.847 ms, profiles/r04j_sample_write_layout.log); 16 for DS
            // (0.787 vs 0.827) and Pinhole (0.763 vs 0.752, even)
            const int wv0 = g_sample_write.load(std::memory_order_relaxed);
            const bool cheap = cam->model == ACM_UCM || cam->model == ACM_EUCM ||
                               cam->model == ACM_FOV || cam->model == ACM_KANNALA_BRANDT;
            const int wv = wv0 < 0 ? (cheap ? 3 : 2) : wv0;
            auto wlaunch = [&](auto kern, int spw) {
                const size_t nwb = (nseg + 4 * (size_t)spw - 1) / (4 * (size_t)spw);
                hipLaunchKernelGGL(kern, dim3((unsigned)nwb), dim3(kBlock), 0, s, ca, g, cells,
                                   seg_cnt, blk_off, points_2d_out, points_3d_out,
                                   (const uint64_t*)counts, cells_out);
            };
            if (spec) {
                hipLaunchKernelGGL((k_seg_spec<TagT>), dim3((unsigned)nsb), dim3(kBlock), 0, s, ca,
                                   g, cells, seg_cnt, blk_sum, points_2d_out, points_3d_out,
                                   cells_out);
                hipLaunchKernelGGL(k_scan_counts, dim3(1), dim3(1024), 0, s, blk_sum, nsb, blk_off,
                                   counts, (uint64_t)cells);
                wlaunch(k_seg_write<TagT, 16, true, false, true>, 16);
                return check_launch("acm_sample_points");
            }
            hipLaunchKernelGGL((k_seg_count<TagC>), dim3((unsigned)nsb), dim3(kBlock), 0, s, ca, g,
                               cells, cert, seg_cnt, blk_sum);
            hipLaunchKernelGGL(k_scan_counts, dim3(1), dim3(1024), 0, s, blk_sum, nsb, blk_off,
                               counts, (uint64_t)cells);
            if (wv == 5) wlaunch(k_seg_write<TagT, 16, true, true>, 16);
            else if (wv == 1) wlaunch(k_seg_write<TagT, 64, false>, 64);
            else if (wv == 3) wlaunch(k_seg_write<TagT, 4, true>, 4);
            else if (wv == 4) wlaunch(k_seg_write<TagT, 16, false>, 16);
            else wlaunch(k_seg_write<TagT, 16, true>, 16);
            return check_launch("acm_sample_points");
        });
    }
    if (mode > 0) {  // single pass with the decoupled look-back
        uint64_t* status = (uint64_t*)workspace + 1;
        if (hipMemsetAsync(workspace, 0, (nt + 1) * sizeof(uint64_t), s) != hipSuccess)
            return check_launch("acm_sample_points: workspace clear");
        return dispatch_sample([&](auto tag) -> int {
            using TagT = decltype(tag);
            const int rr = mode == 1 ? 2 : mode == 2 ? 4 : 8;
            const size_t ntr = (cells + (size_t)kBlock * rr - 1) / ((size_t)kBlock * rr);
            auto kern = k_sample_fused<TagT, 4>;
            if (rr == 2) kern = k_sample_fused<TagT, 2>;
            if (rr == 8) kern = k_sample_fused<TagT, 8>;
            hipLaunchKernelGGL(kern, dim3((unsigned)ntr), dim3(kBlock), 0, s, ca, g, cells,
                               status, points_2d_out, points_3d_out, counts);
            if (cells_out)
                hipLaunchKernelGGL(k_cells_of_uv, dim3((unsigned)std::min<size_t>(nb, 4096)),
                                   dim3(kBlock), 0, s, points_2d_out, counts, g, cells_out);
            return check_launch("acm_sample_points");
        });
    }
    uint64_t* cnt = (uint64_t*)workspace;
    uint64_t* off = cnt + nb;
    return dispatch_sample([&](auto tag) -> int {
        using TagT = decltype(tag);
        hipLaunchKernelGGL((k_sample_count<typename SampleTag<TagT>::count>), dim3((unsigned)nb),
                           dim3(kBlock), 0, s, ca, g, cells, cnt);
        hipLaunchKernelGGL(k_scan_counts, dim3(1), dim3(1024), 0, s, cnt, nb, off, counts,
                           (uint64_t)cells);
        hipLaunchKernelGGL((k_sample_write<TagT>), dim3((unsigned)nb), dim3(kBlock), 0, s, ca, g,
                           cells, off, points_2d_out, points_3d_out);
        if (cells_out)
            hipLaunchKernelGGL(k_cells_of_uv, dim3((unsigned)std::min<size_t>(nb, 4096)),
                               dim3(kBlock), 0, s, points_2d_out, counts, g, cells_out);
        return check_launch("acm_sample_points");
    });
}

ACM_API int acm_sample_points_certificate(const acm_camera* cam, double* out) {
    int rc = check_cam(cam);
    if (rc) return rc;
    if (!out) return fail(ACM_ERR_INVALID_ARGUMENT, "NULL buffer");
    const SegCert c = seg_cert(*cam);
    out[0] = c.on;
    out[1] = c.all_lo;
    out[2] = c.all_hi;
    out[3] = c.none_lo;
    out[4] = c.none_hi;
    return ACM_SUCCESS;
}

ACM_API int acm_unproject_certificate(const acm_camera* cam, double* out) {
    int rc = check_cam(cam);
    if (rc) return rc;
    if (!out) return fail(ACM_ERR_INVALID_ARGUMENT, "NULL buffer");
    out[0] = out[1] = 0.0;
    if (cam->model != ACM_RADTAN) return ACM_SUCCESS;
    const CamArg a = prep(*cam, false, true);
    out[0] = a.uk[1];
    out[1] = a.uk[0] == a.uk[0] ? 1.0 : 0.0;
    return ACM_SUCCESS;
}

ACM_API int acm_sample_points_ray_fit(const acm_camera* cam, double* out) {
    int rc = check_cam(cam);
    if (rc) return rc;
    if (!out) return fail(ACM_ERR_INVALID_ARGUMENT, "NULL buffer");
    for (int i = 0; i < 6; ++i) out[i] = 0.0;
    if (cam->model != ACM_KANNALA_BRANDT) return ACM_SUCCESS;
    const SegCert c = seg_cert(*cam);
    const bool use = c.on && (c.ig_ok || c.rp_ok) && c.all_hi > c.all_lo;
    out[0] = use ? (c.rp_ok ? 3 : c.ig_ok) : 0;
    out[1] = c.on ? c.M : 0.0;
    out[2] = c.on ? c.ef : 0.0;
    out[3] = c.on ? c.rp_err : 0.0;
    out[4] = c.all_lo;
    out[5] = c.all_hi;
    return ACM_SUCCESS;
}

ACM_API int acm_sample_points_ray_poly(const acm_camera* cam, double* out) {
    static_assert(ACM_RAY_POLY_N == kRayPolyN, "acm.h ACM_RAY_POLY_N");
    static_assert(ACM_RAY_GUESS_N == sizeof(SegCert::ig) / sizeof(double), "acm.h ACM_RAY_GUESS_N");
    int rc = check_cam(cam);
    if (rc) return rc;
    if (!out) return fail(ACM_ERR_INVALID_ARGUMENT, "NULL buffer");
    constexpr int NO = 2 * kRayPolyN + ACM_RAY_GUESS_N + 1;
    for (int i = 0; i < NO; ++i) out[i] = 0.0;
    if (cam->model != ACM_KANNALA_BRANDT) return ACM_SUCCESS;
    const SegCert c = seg_cert(*cam);
    if (c.on && c.all_hi > c.all_lo) {
        for (int i = 0; i < 2 * kRayPolyN; ++i) out[i] = c.rp[i];
        for (int i = 0; i < ACM_RAY_GUESS_N; ++i) out[2 * kRayPolyN + i] = c.ig[i];
        out[NO - 1] = c.ig_err;
    }
    return ACM_SUCCESS;
}

ACM_API int acm_sample_points_range(const acm_camera* cam, size_t n_requested, size_t cell_begin,
                                    size_t cell_end, double* points_2d_out, double* points_3d_out,
                                    uint64_t* counts, void* workspace, size_t workspace_bytes,
                                    void* stream) {
    return acm_sample_points_ex(cam, n_requested, cell_begin, cell_end, 0, points_2d_out,
                                points_3d_out, counts, workspace, workspace_bytes, stream);
}

ACM_API int acm_sample_points(const acm_camera* cam, size_t n_requested, double* points_2d_out,
                              double* points_3d_out, uint64_t* counts, void* workspace,
                              size_t workspace_bytes, void* stream) {
    return acm_sample_points_ex(cam, n_requested, 0, ~(size_t)0, 0, points_2d_out, points_3d_out,
                                counts, workspace, workspace_bytes, stream);
}

ACM_API int acm_linear_system_columns(int model) {
    switch (model) {
    case ACM_KANNALA_BRANDT: return 4;
    case ACM_RADTAN: return 3;
    case ACM_DOUBLE_SPHERE:
    case ACM_UCM:
    case ACM_EUCM: return 1;
    default: return -1;
    }
}

static size_t tsqr_blocks(size_t n) {
    size_t nb = (n + kBlock - 1) / kBlock;
    if (nb > (size_t)kTsqrMaxBlocks) nb = kTsqrMaxBlocks;
    return nb ? nb : 1;
}

ACM_API size_t acm_linear_system_qr_workspace_size(int model, size_t n) {
    const int k = acm_linear_system_columns(model);
    if (k < 0) return 0;
    const int M = k + 1, S = M * (M + 1) / 2;
    return tsqr_blocks(n) * S * sizeof(double);
}

ACM_API int acm_linear_system_qr(const acm_camera* cam, size_t n, const double* points_3d,
                                 int layout, const double* points_2d, double* r_factor,
                                 int* error_flag, void* workspace, size_t workspace_bytes,
                                 void* stream) {
    int rc = check_cam(cam);
    if (rc) return rc;
    if ((rc = check_layout(layout))) return rc;
    const int k = acm_linear_system_columns(cam->model);
    if (k < 0) return fail(ACM_ERR_NOT_SUPPORTED, "model has no linear_estimation");
    if (!r_factor || !error_flag || !workspace || (n && (!points_3d || !points_2d)))
        return fail(ACM_ERR_INVALID_ARGUMENT, "NULL buffer");
    if (workspace_bytes < acm_linear_system_qr_workspace_size(cam->model, n))
        return fail(ACM_ERR_WORKSPACE_TOO_SMALL, "linear-system workspace too small");
    hipStream_t s = (hipStream_t)stream;
    double* parts = (double*)workspace;
    if (hipMemsetAsync(error_flag, 0, sizeof(int), s) != hipSuccess)
        return check_launch("acm_linear_system_qr (memset)");
    auto go = [&](auto model_c) {
        constexpr int MOD = decltype(model_c)::value;
        constexpr int M = LinRows<MOD>::K + 1;
        auto kern = layout == ACM_LAYOUT_AOS ? k_tsqr<MOD, ACM_LAYOUT_AOS, void, false, kTsqrNtl>
                                             : k_tsqr<MOD, ACM_LAYOUT_SOA, void, false, kTsqrNtl>;
        const int nb = std::min((int)tsqr_blocks(n),
                                resident_blocks(reinterpret_cast<const void*>(kern)));
        hipLaunchKernelGGL(kern, dim3(nb), dim3(kBlock), 0, s, prep(*cam), n, points_3d,
                           ObsPixels{points_2d}, parts, error_flag, nullptr, nullptr, nullptr);
        hipLaunchKernelGGL((k_tsqr_final<M>), dim3(1), dim3(kBlock), 0, s, parts, nb, r_factor);
    };
    switch (cam->model) {
    case ACM_KANNALA_BRANDT: go(std::integral_constant<int, ACM_KANNALA_BRANDT>{}); break;
    case ACM_RADTAN: go(std::integral_constant<int, ACM_RADTAN>{}); break;
    case ACM_DOUBLE_SPHERE: go(std::integral_constant<int, ACM_DOUBLE_SPHERE>{}); break;
    case ACM_UCM: go(std::integral_constant<int, ACM_UCM>{}); break;
    default: go(std::integral_constant<int, ACM_EUCM>{}); break;
    }
    return check_launch("acm_linear_system_qr");
}

static size_t reproj_error_hist_offset(size_t n);
static size_t reproj_error_median_offset(size_t n);
static int median_impl(size_t n, const double* values, const double* n_valid_device,
                       uint64_t n_valid, double* out, void* workspace,
                       acm_allreduce_fn allreduce, void* allreduce_ctx, void* stream,
                       const unsigned int* hparts, int hnb, bool inited);
static SelWs sel_ws(void* workspace);

extern "C++" {
namespace acm {
// acm_linear_estimation_with_error's device half (solver.hip): one pass of
// k_tsqr<MOD, LAYOUT, TagR> builds the R factor of [A | b] and the
// reprojection error of *cam as given, then the factor merge, the error
// statistics and the median follow on the stream.  ws_err is laid out as
// acm_reprojection_error's workspace (errors first); result: its 9 f64.
// host_out != nullptr (pinned, 25 f64; acm_linear_estimation_with_error_async):
// right after the statistics -- before the median -- R and the flag (17 f64
// from r_factor, the flag in r_factor[16]) and result[0..7] are copied there
// and `ready` is recorded, so the host can solve while the median runs.
// hist_nb != nullptr (the sharded opening, sharded.hip): the shard's R, flag
// and 8 statistics only -- no median state, no host copy, no median; the
// pass-0 histogram partials stay in ws_err and *hist_nb = their workgroups.
// cells / grid (r06): the observations in the cell form (ObsCells), the
// partition of the pixel form's launch (its occupancy), so the same bits.
int linear_system_qr_error(const acm_camera* cam, size_t n, const double* points_3d, int layout,
                           const double* points_2d, double* r_factor, int* error_flag,
                           double* result, void* ws_qr, void* ws_err, void* stream,
                           double* host_out, hipEvent_t ready, int* hist_nb,
                           const uint32_t* cells, const acm_cell_grid* grid) {
    int rc = check_cam(cam);
    if (rc) return rc;
    if ((rc = check_layout(layout))) return rc;
    if (acm_linear_system_columns(cam->model) < 0)
        return fail(ACM_ERR_NOT_SUPPORTED, "model has no linear_estimation");
    hipStream_t s = (hipStream_t)stream;
    double* parts = (double*)ws_qr;
    double* errs = (double*)ws_err;
    double* p1 = errs + n;
    double* tot = p1 + (size_t)ne_blocks(n) * kReprojW;
    unsigned int* hparts = (unsigned int*)((char*)ws_err + reproj_error_hist_offset(n));
    if (hipMemsetAsync(error_flag, 0, sizeof(int), s) != hipSuccess)
        return check_launch("acm_linear_estimation_with_error (memset)");
    int nb = 1;
    auto go = [&](auto model_c, auto tag) {
        constexpr int MOD = decltype(model_c)::value;
        using TagR = decltype(tag);
        constexpr int M = LinRows<MOD>::K + 1;
        auto kern = layout == ACM_LAYOUT_AOS ? k_tsqr<MOD, ACM_LAYOUT_AOS, TagR, true, kTsqrNtl>
                                             : k_tsqr<MOD, ACM_LAYOUT_SOA, TagR, true, kTsqrNtl>;
        nb = std::min((int)tsqr_blocks(n), resident_blocks(reinterpret_cast<const void*>(kern)));
        if (cells) {
            auto kc = layout == ACM_LAYOUT_AOS
                          ? k_tsqr<MOD, ACM_LAYOUT_AOS, TagR, true, kTsqrNtl, ObsCells>
                          : k_tsqr<MOD, ACM_LAYOUT_SOA, TagR, true, kTsqrNtl, ObsCells>;
            hipLaunchKernelGGL(kc, dim3(nb), dim3(kBlock), 0, s, prep(*cam), n, points_3d,
                               obs_cells(cells, *grid), parts, error_flag, errs, p1, hparts);
        } else {
            hipLaunchKernelGGL(kern, dim3(nb), dim3(kBlock), 0, s, prep(*cam), n, points_3d,
                               ObsPixels{points_2d}, parts, error_flag, errs, p1, hparts);
        }
        hipLaunchKernelGGL((k_tsqr_final<M>), dim3(1), dim3(kBlock), 0, s, parts, nb, r_factor);
    };
    switch (cam->model) {
    case ACM_KANNALA_BRANDT:
        go(std::integral_constant<int, ACM_KANNALA_BRANDT>{}, Tag<KannalaBrandt>{});
        break;
    case ACM_RADTAN: go(std::integral_constant<int, ACM_RADTAN>{}, Tag<RadTan>{}); break;
    case ACM_DOUBLE_SPHERE:
        go(std::integral_constant<int, ACM_DOUBLE_SPHERE>{}, Tag<DoubleSphere>{});
        break;
    case ACM_UCM: go(std::integral_constant<int, ACM_UCM>{}, Tag<Ucm>{}); break;
    default: go(std::integral_constant<int, ACM_EUCM>{}, Tag<Eucm>{}); break;
    }
    void* mws = (char*)ws_err + reproj_error_median_offset(n);
    hipLaunchKernelGGL(k_reproj_finish, dim3(1), dim3(kBlock), 0, s, p1, nb, tot, result,
                       hist_nb ? SelWs{} : sel_ws(mws));
    if ((rc = check_launch("acm_linear_estimation_with_error"))) return rc;
    if (hist_nb) {
        *hist_nb = nb;
        return ACM_SUCCESS;
    }
    if (host_out) {
        if (hipMemcpyAsync(host_out, r_factor, 17 * sizeof(double), hipMemcpyDeviceToHost, s) !=
                hipSuccess ||
            hipMemcpyAsync(host_out + 17, result, 8 * sizeof(double), hipMemcpyDeviceToHost, s) !=
                hipSuccess ||
            hipEventRecord(ready, s) != hipSuccess)
            return check_launch("acm_linear_estimation_with_error (copy)");
    }
    return median_impl(n, errs, result + 5, 0, result + 8, mws, nullptr, nullptr, stream, hparts,
                       nb, true);
}

// The sharded conversion's pieces (sharded.hip): the workspace layout of
// acm_reprojection_error, its statistics pass with the pass-0 histogram
// partials but no median state, and the median of the union of the ranks'
// values for a global n_valid known on the host, every histogram summed
// through `allreduce`.
size_t reproj_error_hist_off(size_t n) { return reproj_error_hist_offset(n); }
size_t reproj_error_median_off(size_t n) { return reproj_error_median_offset(n); }
int reprojection_stats_hist(const acm_camera* cam, size_t n, const double* points_3d, int layout,
                            const double* points_2d, double* result, double* errors,
                            void* workspace, void* stream, int* hist_nb,
                            const uint32_t* cells, const acm_cell_grid* grid) {
    unsigned int* hparts = (unsigned int*)((char*)workspace + reproj_error_hist_offset(n));
    return reprojection_stats_impl(cam, n, points_3d, layout, points_2d, result, errors,
                                   workspace, (hipStream_t)stream, hparts, hist_nb, nullptr,
                                   cells, grid);
}
int median_union(size_t n, const double* values, uint64_t n_valid_global, double* out,
                 void* median_ws, acm_allreduce_fn allreduce, void* allreduce_ctx, void* stream,
                 const unsigned int* hparts, int hist_nb) {
    return median_impl(n, values, nullptr, n_valid_global, out, median_ws, allreduce,
                       allreduce_ctx, stream, hparts, hist_nb, false);
}
}  // namespace acm
}

// FOV linear_estimation grid (fov.rs:153-251); the selection is host code
// in solver.hip (acm_fov_grid_select).
// Chunks of >= 256 points, at most the workgroups resident at once (a grid
// of 1.33 rounds left a third of the chip idle for the last round).
static int fov_cap(const void* k, int block) {
    int per_cu = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k, block, 0) != hipSuccess ||
        per_cu <= 0) {
        (void)hipGetLastError();
        per_cu = 4;
    }
    return std::min(kFovMaxBlocks, per_cu * cu_count());
}
// the grid-lane forms: chunks of >= 256 points
static size_t fov_blocks_rec(size_t n) {
    static const int cap = fov_cap(reinterpret_cast<const void*>(k_fov_grid_rec<ACM_LAYOUT_AOS>),
                                   kFovBlock);
    size_t nb = (n + kBlock - 1) / kBlock;
    if (nb > (size_t)cap) nb = cap;
    return nb ? nb : 1;
}
// the point-lane form: >= one group per wave
static size_t fov_blocks_pl(size_t n) {
    static const int cap = fov_cap(
        reinterpret_cast<const void*>(k_fov_grid_pl<ACM_LAYOUT_AOS, kFovPlP, kFovPlNW>),
        kFovPlBlock);
    const size_t per_block = (size_t)kFovPlBlock * kFovPlP;
    size_t nb = (n + per_block - 1) / per_block;
    if (nb > (size_t)cap) nb = cap;
    return nb ? nb : 1;
}
// the partial-sum rows of the workspace: enough for either form
static size_t fov_blocks(size_t n) { return std::max(fov_blocks_rec(n), fov_blocks_pl(n)); }

static const double* fov_grid_table() {
    static double table[5 * kFovGrid];
    static const bool init = [] {
        for (int i = 10; i < 10 + kFovGrid; ++i) {
            const double w = (double)i / 100.0;          // :180
            const double tan_w_half = std::tan(w / 2.0);  // :195
            table[3 * (i - 10)] = w;
            table[3 * (i - 10) + 1] = 2.0 * tan_w_half;          // :196, exact
            table[3 * (i - 10) + 2] = 2.0 * tan_w_half / w;      // :202
            table[3 * kFovGrid + 2 * (i - 10)] = 1.0 / w;
            table[3 * kFovGrid + 2 * (i - 10) + 1] = 1.0 / (2.0 * tan_w_half);
        }
        return true;
    }();
    (void)init;
    return table;
}

ACM_API size_t acm_fov_grid_workspace_size(size_t n) {
    return (fov_blocks(n) * 2 * kFovGrid + 5 * kFovGrid) * sizeof(double);
}

ACM_API int acm_fov_grid_errors(const acm_camera* cam, size_t n, const double* points_3d,
                                int layout, const double* points_2d, double* grid_sums,
                                void* workspace, size_t workspace_bytes, void* stream) {
    int rc = check_cam(cam);
    if (rc) return rc;
    if ((rc = check_layout(layout))) return rc;
    if (cam->model != ACM_FOV) return fail(ACM_ERR_NOT_SUPPORTED, "grid search is FOV-only");
    if (!grid_sums || !workspace || (n && (!points_3d || !points_2d)))
        return fail(ACM_ERR_INVALID_ARGUMENT, "NULL buffer");
    if (workspace_bytes < acm_fov_grid_workspace_size(n))
        return fail(ACM_ERR_WORKSPACE_TOO_SMALL, "FOV grid workspace too small");
    hipStream_t s = (hipStream_t)stream;
    const int fu = g_fov_unroll;
    const size_t nb = fu < 0 ? fov_blocks_pl(n) : fov_blocks_rec(n);
    const size_t chunk = (n + nb - 1) / nb;
    double* parts = (double*)workspace;
    double* table = parts + fov_blocks(n) * 2 * kFovGrid;
    if (hipMemcpyAsync(table, fov_grid_table(), 5 * kFovGrid * sizeof(double),
                       hipMemcpyHostToDevice, s) != hipSuccess)
        return check_launch("acm_fov_grid_errors (table)");
    auto go = [&](auto lay_c, auto u_c) {
        constexpr int LAY = decltype(lay_c)::value, U = decltype(u_c)::value;
        if (fu < 0) {  // point-lane form (default)
            hipLaunchKernelGGL((k_fov_grid_pl<LAY, kFovPlP, kFovPlNW>), dim3(nb),
                               dim3(kFovPlBlock), 0, s, *cam, n, points_3d, points_2d, table, parts);
        } else if (fu == 0) {  // record form
            hipLaunchKernelGGL((k_fov_grid_rec<LAY>), dim3(nb), dim3(kFovBlock), 0, s, *cam, n,
                               chunk, points_3d, points_2d, table, parts);
        } else {  // the LDS form, U points per lane step
            hipLaunchKernelGGL((k_fov_grid<LAY, U>), dim3(nb), dim3(kFovBlock), 0, s, *cam, n,
                               chunk, points_3d, points_2d, table, parts);
        }
    };
    auto by_unroll = [&](auto lay_c) {
        switch (fu) {
        case 2: go(lay_c, std::integral_constant<int, 2>{}); break;
        case 4: go(lay_c, std::integral_constant<int, 4>{}); break;
        default: go(lay_c, std::integral_constant<int, 1>{}); break;
        }
    };
    if (layout == ACM_LAYOUT_AOS) by_unroll(std::integral_constant<int, ACM_LAYOUT_AOS>{});
    else by_unroll(std::integral_constant<int, ACM_LAYOUT_SOA>{});
    hipLaunchKernelGGL(k_fov_finish, dim3(2 * kFovGrid), dim3(kBlock), 0, s, parts, (int)nb,
                       grid_sums);
    return check_launch("acm_fov_grid_errors");
}

// workspace: 2 SelState | 2 x 2048 f64 histogram | candidate count | n f64 candidates
ACM_API size_t acm_median_workspace_size(size_t n) {
    return 2 * sizeof(SelState) + 2 * kSelBins * sizeof(double) + 16 + n * sizeof(double);
}

// hparts / hnb: pass 0's histogram already counted per workgroup by
// k_reproj_pass1<HIST> (acm_reprojection_error): merged instead of read.
static SelWs sel_ws(void* workspace) {
    SelWs w;
    w.st = (SelState*)workspace;
    w.hist = (double*)(w.st + 2);
    w.count = (unsigned long long*)(w.hist + 2 * kSelBins);
    w.cbuf = (double*)(w.count + 2);
    return w;
}

// inited: the caller's k_reproj_finish already ran sel_init_wg on this
// workspace (acm_reprojection_error, acm_linear_estimation_with_error)
static int median_impl(size_t n, const double* values, const double* n_valid_device,
                       uint64_t n_valid, double* out, void* workspace,
                       acm_allreduce_fn allreduce, void* allreduce_ctx, void* stream,
                       const unsigned int* hparts, int hnb, bool inited) {
    hipStream_t s = (hipStream_t)stream;
    const SelWs w = sel_ws(workspace);
    SelState* st = w.st;
    double* hist = w.hist;
    // one 1024-lane workgroup per CU (fewer for small n)
    const unsigned nb = (unsigned)std::max<size_t>(
        1, std::min<size_t>((size_t)cu_count(), (n + kSelBlock * kSelU - 1) / (kSelBlock * kSelU)));
    const bool ntl = g_nt_loads != 0;
    // passes 0-1 read every value (pass 0 aggregates its exponent digits per
    // wave); then the candidates sharing either state's 22-bit prefix are
    // compacted and passes 2-5 read only them.  (Picking in the histogram
    // kernels' last workgroup instead of a k_sel_pick launch was measured in
    // r05: the ticket's fan-in and the fences cost more than the launches,
    // reproj_error 1.10 -> 1.46 ms at 92.9M, profiles/r05q_median_ab.log.)
    constexpr int kFullPasses = 2;
    if (!inited)
        hipLaunchKernelGGL(k_sel_init, dim3(1), dim3(kBlock), 0, s, w, n_valid_device,
                           (unsigned long long)n_valid);
    for (int pass = 0; pass < kSelPasses; ++pass) {
        if (pass == kFullPasses)
            hipLaunchKernelGGL((ntl ? k_sel_compact<true> : k_sel_compact<false>), dim3(nb),
                               dim3(kSelBlock), 0, s, n, values, st, w.cbuf, w.count);
        if (pass == 0 && hparts)
            hipLaunchKernelGGL(k_sel_hist_merge, dim3(kSelBins / kBlock, kSelMergeG), dim3(kBlock),
                               0, s, hparts, hnb, hist);
        else if (pass == 0)
            hipLaunchKernelGGL((ntl ? k_sel_hist<true, true> : k_sel_hist<true, false>), dim3(nb),
                               dim3(kSelBlock), 0, s, n, nullptr, values, st, pass, hist);
        else if (pass < kFullPasses)
            hipLaunchKernelGGL((ntl ? k_sel_hist<false, true> : k_sel_hist<false, false>),
                               dim3(nb), dim3(kSelBlock), 0, s, n, nullptr, values, st, pass,
                               hist);
        else
            hipLaunchKernelGGL((k_sel_hist<false, false>), dim3(nb), dim3(kSelBlock),
                               0, s, (size_t)0, w.count, w.cbuf, st, pass, hist);
        if (allreduce) {  // every rank then picks the same digits
            int rc = check_launch("acm_median_valid (histogram)");
            if (rc) return rc;
            if (allreduce(allreduce_ctx, hist, 2 * kSelBins, stream) != 0)
                return fail(ACM_ERR_INVALID_ARGUMENT, "allreduce callback failed");
        }
        hipLaunchKernelGGL(k_sel_pick, dim3(1), dim3(kBlock), 0, s, st, pass, hist);
    }
    hipLaunchKernelGGL(k_sel_finish, dim3(1), dim3(64), 0, s, st, st + 1, n_valid_device,
                       (unsigned long long)n_valid, out);
    return check_launch("acm_median_valid");
}

ACM_API int acm_median_valid_allreduce(size_t n, const double* values,
                                       const double* n_valid_device, uint64_t n_valid,
                                       double* out, void* workspace, size_t workspace_bytes,
                                       acm_allreduce_fn allreduce, void* allreduce_ctx,
                                       void* stream) {
    if (!out || !workspace || (n && !values)) return fail(ACM_ERR_INVALID_ARGUMENT, "NULL buffer");
    if (workspace_bytes < acm_median_workspace_size(n))
        return fail(ACM_ERR_WORKSPACE_TOO_SMALL, "median workspace too small");
    return median_impl(n, values, n_valid_device, n_valid, out, workspace, allreduce,
                       allreduce_ctx, stream, nullptr, 0, false);
}

// compute_reprojection_error in one call: [errors n f64 (when the caller
// passes none)] | reprojection partials | pass-0 histogram partials
// (nb x 2048 u32) | median workspace
static size_t reproj_error_hist_offset(size_t n) {
    return (acm_reprojection_stats_workspace_size(n) + 255) / 256 * 256;
}
static size_t reproj_error_median_offset(size_t n) {
    return reproj_error_hist_offset(n) +
           ((size_t)ne_blocks(n) * kSelBins * sizeof(unsigned int) + 255) / 256 * 256;
}
ACM_API size_t acm_reprojection_error_workspace_size(size_t n) {
    return reproj_error_median_offset(n) + acm_median_workspace_size(n);
}

ACM_API int acm_reprojection_error(const acm_camera* cam, size_t n, const double* points_3d,
                                   int layout, const double* points_2d, double* result,
                                   double* errors, void* workspace, size_t workspace_bytes,
                                   void* stream) {
    if (!result || !workspace || (n && (!points_3d || !points_2d)))
        return fail(ACM_ERR_INVALID_ARGUMENT, "NULL buffer");
    if (workspace_bytes < acm_reprojection_error_workspace_size(n))
        return fail(ACM_ERR_WORKSPACE_TOO_SMALL, "reprojection-error workspace too small");
    char* ws = (char*)workspace;
    unsigned int* hparts = (unsigned int*)(ws + reproj_error_hist_offset(n));
    int nb = 0;
    void* mws = ws + reproj_error_median_offset(n);
    int rc = reprojection_stats_impl(cam, n, points_3d, layout, points_2d, result, errors,
                                     workspace, (hipStream_t)stream, hparts, &nb, mws);
    if (rc) return rc;
    const double* errs = errors ? errors : (const double*)workspace;
    // n_valid from result[5] on the device: no host round trip in between
    return median_impl(n, errs, result + 5, 0, result + 8, mws, nullptr, nullptr, stream, hparts,
                       nb, true);
}

// (r06) the same from the cell form of the observations (acm_cell_grid)
ACM_API int acm_reprojection_error_cells(const acm_camera* cam, size_t n, const double* points_3d,
                                         int layout, const uint32_t* cells,
                                         const acm_cell_grid* grid, double* result,
                                         double* errors, void* workspace, size_t workspace_bytes,
                                         void* stream) {
    int rc = acm::check_cell_grid(grid);
    if (rc) return rc;
    if (!result || !workspace || (n && (!points_3d || !cells)))
        return fail(ACM_ERR_INVALID_ARGUMENT, "NULL buffer");
    if (workspace_bytes < acm_reprojection_error_workspace_size(n))
        return fail(ACM_ERR_WORKSPACE_TOO_SMALL, "reprojection-error workspace too small");
    static const uint32_t none = 0;
    char* ws = (char*)workspace;
    unsigned int* hparts = (unsigned int*)(ws + reproj_error_hist_offset(n));
    int nb = 0;
    void* mws = ws + reproj_error_median_offset(n);
    rc = reprojection_stats_impl(cam, n, points_3d, layout, nullptr, result, errors, workspace,
                                 (hipStream_t)stream, hparts, &nb, mws, cells ? cells : &none,
                                 grid);
    if (rc) return rc;
    const double* errs = errors ? errors : (const double*)workspace;
    return median_impl(n, errs, result + 5, 0, result + 8, mws, nullptr, nullptr, stream, hparts,
                       nb, true);
}

ACM_API int acm_median_valid(size_t n, const double* values, const double* n_valid_device,
                             uint64_t n_valid, double* out, void* workspace,
                             size_t workspace_bytes, void* stream) {
    return acm_median_valid_allreduce(n, values, n_valid_device, n_valid, out, workspace,
                                      workspace_bytes, nullptr, nullptr, stream);
}


ACM_API int acm_undistort_image(const acm_camera* cam, const double* target_intrinsics,
                                int interpolation, const uint8_t* image, uint8_t* output,
                                void* stream) {
    int rc = check_cam(cam);
    if (rc) return rc;
    if (!image || !output) return fail(ACM_ERR_INVALID_ARGUMENT, "NULL buffer");
    if (interpolation != ACM_INTERP_NEAREST && interpolation != ACM_INTERP_BILINEAR)
        return fail(ACM_ERR_INVALID_ARGUMENT, "interpolation must be NEAREST or BILINEAR");
    const double* t = target_intrinsics ? target_intrinsics : cam->params;  // :30
    if (cam->width == 0 || cam->height == 0) return ACM_SUCCESS;
    hipStream_t s = (hipStream_t)stream;
    const dim3 g((cam->width + 63) / 64, (cam->height + kBlock / 64 - 1) / (kBlock / 64));
    return dispatch_model(cam->model, [&](auto tag) -> int {
        using TagT = decltype(tag);
        if (interpolation == ACM_INTERP_BILINEAR)
            hipLaunchKernelGGL((k_undistort<TagT, true>), g, dim3(kBlock), 0, s, prep(*cam), t[0], t[1],
                               t[2], t[3], image, output);
        else
            hipLaunchKernelGGL((k_undistort<TagT, false>), g, dim3(kBlock), 0, s, prep(*cam), t[0],
                               t[1], t[2], t[3], image, output);
        return check_launch("acm_undistort_image");
    });
}

static int hip_rc(hipError_t e, const char* what) {
    if (e == hipSuccess) return ACM_SUCCESS;
    g_last_hip_error = (int)e;
    return fail(ACM_ERR_HIP, std::string(what) + ": " + hipGetErrorString(e));
}

ACM_API int acm_set_device(int device) { return hip_rc(hipSetDevice(device), "hipSetDevice"); }

ACM_API int acm_device_malloc(void** ptr, size_t bytes) {
    if (!ptr) return fail(ACM_ERR_INVALID_ARGUMENT, "NULL argument");
    return hip_rc(hipMalloc(ptr, bytes), "hipMalloc");
}

ACM_API int acm_device_free(void* ptr) { return hip_rc(hipFree(ptr), "hipFree"); }

ACM_API int acm_memcpy_htod(void* dst, const void* src, size_t bytes, void* stream) {
    return hip_rc(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, (hipStream_t)stream),
                  "hipMemcpyAsync(H2D)");
}

ACM_API int acm_memcpy_dtoh(void* dst, const void* src, size_t bytes, void* stream) {
    return hip_rc(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, (hipStream_t)stream),
                  "hipMemcpyAsync(D2H)");
}

ACM_API int acm_stream_synchronize(void* stream) {
    return hip_rc(hipStreamSynchronize((hipStream_t)stream), "hipStreamSynchronize");
}

ACM_API int acm_set_tuning(int key, int value) {
    // Every knob is a std::atomic<int> read with one load per launch, so
    // concurrent callers and concurrent acm_set_tuning calls are race-free
    // (each launch sees either the old or the new value; results are
    // identical for every setting).
    struct Knob {
        int key;
        std::atomic<int>* v;
        int lo, hi;
        const char* msg;
    };
    static const Knob knobs[] = {
        {ACM_TUNE_PROJECT_VARIANT, &g_project_variant, -1, 7, "variant must be -1 (auto) or 0..7"},
        {ACM_TUNE_RESIDUAL_NT, &g_residual_nt, -1, 1, "value must be -1..1"},
        {ACM_TUNE_NE_WAVES, &g_ne_waves, 0, 4, "value must be 0 (per-model default), 1, 3 or 4"},
        {ACM_TUNE_FOV_UNROLL, &g_fov_unroll, -1, 4, "value must be -1, 0, 1, 2 or 4"},
        {ACM_TUNE_NE_UNROLL, &g_ne_unroll, 0, 5, "value must be 0 (per-model default) or 1..5"},
        {ACM_TUNE_ALIGN_J, &g_align_j, -1, 1, "value must be -1..1"},
        {ACM_TUNE_NT_LOADS, &g_nt_loads, -1, 1, "value must be -1..1"},
        {ACM_TUNE_NT_LOADS_UNPROJECT, &g_nt_loads_unproject, -1, 1, "value must be -1..1"},
        {ACM_TUNE_LM_HOST_RESULT, &g_lm_host_result, -1, 3, "value must be -1..3"},
        {ACM_TUNE_SAMPLE_FUSED, &g_sample_fused, -1, 4, "value must be -1..4"},
        {ACM_TUNE_UNPROJECT_RCP, &g_unproject_rcp, -1, 1, "value must be -1..1"},
        {ACM_TUNE_SAMPLE_PATIENCE, &g_sample_patience, -1, 1 << 20, "value must be -1..2^20"},
        {ACM_TUNE_SAMPLE_CERT, &g_sample_cert, -1, 0, "value must be -1 (auto) or 0"},
        {ACM_TUNE_SAMPLE_WRITE, &g_sample_write, -1, 5, "value must be -1..5"},
        {ACM_TUNE_UNPROJECT_PPT, &g_unproject_ppt, -1, 3, "value must be -1..3"},
        {ACM_TUNE_ROUND_TRIP, &g_round_trip, -1, 20, "value must be -1 or PPT (1, 2, 4) + 8 x stores (0..2)"},
    };
    if (key == ACM_TUNE_NEWTON_FAST)  // removed (r03): numerics are chosen per call
        return fail(ACM_ERR_NOT_SUPPORTED,
                    "ACM_TUNE_NEWTON_FAST was removed: OR ACM_REFERENCE_NEWTON into the call's "
                    "layout / flags instead (acm_unproject, acm_sample_points_ex)");
    if (key == ACM_TUNE_LM_DEVICE)  // removed (r05): slower than the host loop
        return fail(ACM_ERR_NOT_SUPPORTED,
                    "ACM_TUNE_LM_DEVICE was removed: acm_lm_optimize runs the host loop");
    for (const Knob& k : knobs) {
        if (k.key != key) continue;
        bool ok = value >= k.lo && value <= k.hi;
        if (key == ACM_TUNE_NE_WAVES) ok = ok && value != 2;
        if (key == ACM_TUNE_FOV_UNROLL) ok = ok && value != 3;
        if (key == ACM_TUNE_UNPROJECT_PPT) ok = ok && value != 0;
        if (key == ACM_TUNE_ROUND_TRIP)
            ok = ok && (value == -1 || ((value & 7) == 1 || (value & 7) == 2 || (value & 7) == 4));
        if (!ok) return fail(ACM_ERR_INVALID_ARGUMENT, k.msg);
        return k.v->exchange(value);
    }
    return fail(ACM_ERR_INVALID_ARGUMENT, "unknown tuning key");
}

ACM_API int acm_last_hip_error(void) { return g_last_hip_error; }
ACM_API const char* acm_last_error(void) { return g_last_error.c_str(); }
// The version string names the compile-time variant of the build (the
// diagnostic / A-B defines), so a counter file collected on one variant
// cannot be attributed to another (bench.py load_traffic).
// ACM_BUILD_DEFINES: the Makefile passes every extra define of an A/B or
// diagnostic build (AB=..., HIPFLAGS additions) as a string, so the version
// names them whatever the library file is called.
#ifndef ACM_BUILD_DEFINES
#define ACM_BUILD_DEFINES ""
#endif
ACM_API const char* acm_version(void) {
    static const std::string v = std::string("acm 0.4.0 (gfx950") +
#ifdef ACM_IEEE_MATH
                                 "; ACM_IEEE_MATH" +
#endif
                                 (ACM_BUILD_DEFINES[0] ? std::string("; ") + ACM_BUILD_DEFINES
                                                       : std::string()) +
                                 ")";
    return v.c_str();
}

}  // extern "C"
