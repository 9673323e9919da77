// hbm_probe.hip -- zero-compute HBM ceilings for the hot path's access
// patterns (a measuring tool, not part of libacm.so).
//
//   acm_probe_read   : grid-stride sum of a buffer (the normal-equations
//                      kernel's pure 40 B/pt read stream, no math)
//   acm_probe_read_pts: the same stream in its real shape (AoS xyz + 16-B
//                      observations), per-lane strided or LDS-staged loads
//   acm_probe_write  : fill a buffer with 16-B stores (plain or nt)
//   acm_probe_mimic  : the exact traffic of k_project<*, J>: read 24 B/pt
//                      (AoS xyz), write 16 B uv + 1 B status + `cols` 16-B
//                      Jacobian column pairs (2N x cols column-major), with a
//                      trivial function of the inputs instead of the camera
//                      model -- the same bytes, in the same instruction shape,
//                      with (almost) no VALU work.
//
// Built by tools/Makefile (hipcc --offload-arch=gfx950); driven by
// tools/hbm_ceiling.py.
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef double dbl2 __attribute__((ext_vector_type(2)));

template <bool NT>
__device__ __forceinline__ void put2(double* p, double a, double b) {
    dbl2 v = {a, b};
    if (NT) __builtin_nontemporal_store(v, reinterpret_cast<dbl2*>(p));
    else *reinterpret_cast<dbl2*>(p) = v;
}

// U independent 16-B loads in flight per lane per step; NT = non-temporal loads
template <int U, bool NT>
__global__ __launch_bounds__(256) void k_read(const dbl2* __restrict__ p, size_t n2,
                                              double* __restrict__ out) {
    // one partial per wave (no same-address atomics: they would serialise)
    double s = 0.0;
    const size_t stride = (size_t)gridDim.x * 256;
    size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
    for (; i + (U - 1) * stride < n2; i += U * stride) {
        dbl2 a[U];
#pragma unroll
        for (int u = 0; u < U; ++u)
            a[u] = NT ? __builtin_nontemporal_load(p + i + u * stride) : p[i + u * stride];
#pragma unroll
        for (int u = 0; u < U; ++u) s += a[u].x + a[u].y;
    }
    for (; i < n2; i += stride) { const dbl2 a = p[i]; s += a.x + a.y; }
    for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off, 64);
    if ((threadIdx.x & 63) == 0) out[(size_t)blockIdx.x * 4 + (threadIdx.x >> 6)] = s;
}

// The normal-equations read stream with no math: AoS xyz (24 B/pt) + 16-B
// observations, one 64-point chunk per wave step.  STAGE = 0: three 8-B loads
// per lane at a 24-B stride; STAGE = 1: the chunk's 1536 B as three dense
// 512-B wave loads, redistributed through LDS.
template <bool STAGE>
__global__ __launch_bounds__(256) void k_read_pts(const double* __restrict__ xyz,
                                                  const double* __restrict__ obs, size_t n,
                                                  double* __restrict__ out) {
    __shared__ double st[4][192];
    double s = 0.0;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const size_t nw = (size_t)gridDim.x * 4;
    for (size_t b = ((size_t)blockIdx.x * 4 + w) * 64; b < n; b += nw * 64) {
        const size_t i = b + lane;
        double x = 0.0, y = 0.0, z = 0.0;
        if (STAGE && b + 64 <= n) {
            const double* src = xyz + 3 * b + lane;
            const double d0 = __builtin_nontemporal_load(src);
            const double d1 = __builtin_nontemporal_load(src + 64);
            const double d2 = __builtin_nontemporal_load(src + 128);
            st[w][lane] = d0;
            st[w][64 + lane] = d1;
            st[w][128 + lane] = d2;
            __builtin_amdgcn_wave_barrier();
            x = st[w][3 * lane];
            y = st[w][3 * lane + 1];
            z = st[w][3 * lane + 2];
            __builtin_amdgcn_wave_barrier();
        } else if (i < n) {
            x = __builtin_nontemporal_load(xyz + 3 * i);
            y = __builtin_nontemporal_load(xyz + 3 * i + 1);
            z = __builtin_nontemporal_load(xyz + 3 * i + 2);
        }
        if (i < n) {
            const dbl2 o = __builtin_nontemporal_load(reinterpret_cast<const dbl2*>(obs) + i);
            s += x + y + z + o.x + o.y;
        }
    }
    for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off, 64);
    if (lane == 0) out[(size_t)blockIdx.x * 4 + w] = s;
}

template <bool NT>
__global__ __launch_bounds__(256) void k_write(double* __restrict__ p, size_t n2, double v) {
    const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (i < n2) put2<NT>(p + 2 * i, v, v);
}

// OBS: also read a 16-B observation per point (the residual kernel's traffic)
template <bool NT, int COLS, bool OBS>
__global__ __launch_bounds__(256) void k_mimic(size_t n, const double* __restrict__ xyz,
                                               double* __restrict__ uv, uint8_t* __restrict__ st,
                                               double* __restrict__ jac) {
    const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    double x = xyz[3 * i], y = xyz[3 * i + 1], z = xyz[3 * i + 2];
    if (OBS) {
        const dbl2 o = *reinterpret_cast<const dbl2*>(xyz + 3 * n + 2 * i);
        x += o.x;
        y += o.y;
    }
    put2<NT>(uv + 2 * i, x + z, y + z);
    if (NT) __builtin_nontemporal_store((uint8_t)(z < 0.0), st + i);
    else st[i] = (uint8_t)(z < 0.0);
#pragma unroll
    for (int c = 0; c < COLS; ++c) put2<NT>(jac + (size_t)c * 2 * n + 2 * i, x * c, y * c);
}

static unsigned blocks(size_t n) { return (unsigned)((n + 255) / 256); }

extern "C" {

int acm_probe_read(const void* buf, size_t bytes, double* out, int grid, int unroll, int nt,
                   void* stream) {
    const size_t n2 = bytes / 16;
    hipStream_t s = (hipStream_t)stream;
#define RD(U)                                                                                   \
    if (unroll == U) {                                                                          \
        if (nt) hipLaunchKernelGGL((k_read<U, true>), dim3(grid), dim3(256), 0, s, (const dbl2*)buf, \
                                   n2, out);                                                    \
        else hipLaunchKernelGGL((k_read<U, false>), dim3(grid), dim3(256), 0, s, (const dbl2*)buf, \
                                n2, out);                                                       \
        return (int)hipGetLastError();                                                          \
    }
    RD(1) RD(2) RD(4) RD(8)
#undef RD
    return -1;
}

// xyz: n AoS points (16-B aligned), obs: n 16-B observations
int acm_probe_read_pts(const double* xyz, const double* obs, size_t n, double* out, int grid,
                       int stage, void* stream) {
    if (stage) hipLaunchKernelGGL(k_read_pts<true>, dim3(grid), dim3(256), 0, (hipStream_t)stream,
                                  xyz, obs, n, out);
    else hipLaunchKernelGGL(k_read_pts<false>, dim3(grid), dim3(256), 0, (hipStream_t)stream, xyz,
                            obs, n, out);
    return (int)hipGetLastError();
}

int acm_probe_write(void* buf, size_t bytes, int nt, void* stream) {
    const size_t n2 = bytes / 16;
    if (nt) hipLaunchKernelGGL(k_write<true>, dim3(blocks(n2)), dim3(256), 0, (hipStream_t)stream,
                               (double*)buf, n2, 1.0);
    else hipLaunchKernelGGL(k_write<false>, dim3(blocks(n2)), dim3(256), 0, (hipStream_t)stream,
                            (double*)buf, n2, 1.0);
    return (int)hipGetLastError();
}

// obs != 0: xyz must hold 3n + 2n doubles (points, then observations)
int acm_probe_mimic(size_t n, const double* xyz, double* uv, uint8_t* st, double* jac, int cols,
                    int nt, int obs, void* stream) {
    hipStream_t s = (hipStream_t)stream;
#define MIMIC(C)                                                                          \
    if (cols == C) {                                                                      \
        if (obs) hipLaunchKernelGGL((k_mimic<true, C, true>), dim3(blocks(n)), dim3(256), 0, s, \
                                    n, xyz, uv, st, jac);                                 \
        else if (nt) hipLaunchKernelGGL((k_mimic<true, C, false>), dim3(blocks(n)), dim3(256), 0, \
                                        s, n, xyz, uv, st, jac);                          \
        else hipLaunchKernelGGL((k_mimic<false, C, false>), dim3(blocks(n)), dim3(256), 0, s, n, \
                                xyz, uv, st, jac);                                        \
        return (int)hipGetLastError();                                                    \
    }
    MIMIC(0) MIMIC(4) MIMIC(5) MIMIC(6) MIMIC(8) MIMIC(9)
#undef MIMIC
    return -1;
}

}  // extern "C"

// ---------------------------------------------------------------------------
// acm_probe_write_sample: the store ceiling of the sample_points write pass
//  -- write-only kernels in its output shape (a 16-B pixel
// stream and a 24-B ray stream per kept point, 3.72 GB at config 5), no loads
// and no arithmetic; driven by tools/diag_store.py.
namespace {

// variant 0: one 16-B store per lane per stream, grid-stride over points
// (uv: point i -> 16 B at 16 i; rays: 24 B at 24 i as 3 x 8 B)
__global__ __launch_bounds__(256) void k_store_aos(double2* __restrict__ uv,
                                                   double* __restrict__ xyz, uint64_t n) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        uv[i] = make_double2((double)i, 1.0);
        xyz[3 * i + 0] = 0.5;
        xyz[3 * i + 1] = 0.25;
        xyz[3 * i + 2] = 1.0;
    }
}

// variant 1: both streams as flat 16-B vectors (uv: 1 per point, rays: 1.5
// per point), every lane one dwordx4 per step -- the best case for the
// store unit
__global__ __launch_bounds__(256) void k_store_v4(double2* __restrict__ a, uint64_t na,
                                                  double2* __restrict__ b, uint64_t nb) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const double2 v = make_double2(1.0, 2.0);
    for (uint64_t i = t; i < na; i += stride) a[i] = v;
    for (uint64_t i = t; i < nb; i += stride) b[i] = v;
}

// variant 2: like 1 but each wave writes a contiguous 64 x 16 B run per
// step from a per-wave chunk (the write pass's "one contiguous run per wave")
__global__ __launch_bounds__(256) void k_store_runs(double2* __restrict__ a, uint64_t na,
                                                    double2* __restrict__ b, uint64_t nb,
                                                    uint64_t chunk) {
    const uint64_t wave = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const unsigned lane = threadIdx.x & 63;
    const double2 v = make_double2(1.0, 2.0);
    uint64_t lo = wave * chunk, hi = lo + chunk;
    for (uint64_t i = lo + lane; i < hi && i < na; i += 64) a[i] = v;
    lo = wave * chunk * 3 / 2;
    hi = lo + chunk * 3 / 2;
    for (uint64_t i = lo + lane; i < hi && i < nb; i += 64) b[i] = v;
}

}  // namespace

extern "C" int acm_probe_write_sample(int variant, void* uv, void* xyz, uint64_t n, int blocks,
                           uint64_t chunk, hipStream_t s) {
    switch (variant) {
    case 0:
        hipLaunchKernelGGL(k_store_aos, dim3(blocks), dim3(256), 0, s, (double2*)uv,
                           (double*)xyz, n);
        break;
    case 1:
        hipLaunchKernelGGL(k_store_v4, dim3(blocks), dim3(256), 0, s, (double2*)uv, n,
                           (double2*)xyz, n * 3 / 2);
        break;
    case 2:
        hipLaunchKernelGGL(k_store_runs, dim3(blocks), dim3(256), 0, s, (double2*)uv, n,
                           (double2*)xyz, n * 3 / 2, chunk);
        break;
    default:
        return -1;
    }
    return hipGetLastError() == hipSuccess ? 0 : -2;
}

// ---------------------------------------------------------------------------
// acm_probe_reproj: the traffic of k_reproj_pass1 (compute_reprojection_error,
// DESIGN.md 8) with no camera model -- AoS xyz (24 B) + a 16-B observation
// read per point, software-pipelined in A static slots exactly like the real
// kernel, and (STORE) one 8-B value written per point (NTS: non-temporal).
// STORE = false is the normal-equations kernel's pure read stream in the
// same loop shape.  Driven by tools/diag_reproj_ceiling.py.
namespace {

template <int A, bool STORE, bool NTS>
__global__ __launch_bounds__(256) void k_reproj_mimic(size_t n, const double* __restrict__ xyz,
                                                      const double* __restrict__ obs,
                                                      double* __restrict__ err,
                                                      double* __restrict__ out) {
    const size_t stride = (size_t)gridDim.x * 256;
    size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
    double xs[A], ys[A], zs[A];
    dbl2 os[A];
    auto load_slot = [&](int q, size_t iq) {
        const size_t ic = iq < n ? iq : n - 1;
        xs[q] = __builtin_nontemporal_load(xyz + 3 * ic);
        ys[q] = __builtin_nontemporal_load(xyz + 3 * ic + 1);
        zs[q] = __builtin_nontemporal_load(xyz + 3 * ic + 2);
        os[q] = __builtin_nontemporal_load(reinterpret_cast<const dbl2*>(obs) + ic);
    };
    double s = 0.0;
    if (n) {
#pragma unroll
        for (int q = 0; q < A; ++q) load_slot(q, i + (size_t)q * stride);
    }
    for (; i < n; i += (size_t)A * stride) {
#pragma unroll
        for (int q = 0; q < A; ++q) {
            const size_t iq = i + (size_t)q * stride;
            if (iq < n) {
                const double e = xs[q] * zs[q] + ys[q] - os[q].x * os[q].y;
                s += e;
                if (STORE) {
                    if (NTS) __builtin_nontemporal_store(e, err + iq);
                    else err[iq] = e;
                }
            }
            load_slot(q, iq + (size_t)A * stride);
        }
    }
    for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off, 64);
    if ((threadIdx.x & 63) == 0) out[(size_t)blockIdx.x * 4 + (threadIdx.x >> 6)] = s;
}

}  // namespace

// store: 0 = none, 1 = non-temporal 8-B stores, 2 = plain 8-B stores
extern "C" int acm_probe_reproj(size_t n, const double* xyz, const double* obs, double* err,
                                double* out, int grid, int slots, int store, void* stream) {
    hipStream_t s = (hipStream_t)stream;
#define RP(AA)                                                                               \
    if (slots == AA) {                                                                       \
        if (store == 0) hipLaunchKernelGGL((k_reproj_mimic<AA, false, false>), dim3(grid), dim3(256), \
                                           0, s, n, xyz, obs, err, out);                     \
        else if (store == 1) hipLaunchKernelGGL((k_reproj_mimic<AA, true, true>), dim3(grid),  \
                                                dim3(256), 0, s, n, xyz, obs, err, out);     \
        else hipLaunchKernelGGL((k_reproj_mimic<AA, true, false>), dim3(grid), dim3(256), 0, s, n, \
                                xyz, obs, err, out);                                         \
        return (int)hipGetLastError();                                                       \
    }
    RP(2) RP(4) RP(6)
#undef RP
    return -1;
}

// ---------------------------------------------------------------------------
// acm_probe_round_trip: the traffic of k_round_trip (config 4, one point per
// lane) with no camera model: AoS xyz read (24 B), pixel pair (16 B) and
// status byte written, then the AoS ray (24 B, LDS-staged into 16-B stores
// per wave like the real kernel) and a second status byte.  66 B per point.
namespace {

__global__ __launch_bounds__(256) void k_rt_mimic(size_t n, const double* __restrict__ xyz,
                                                  double* __restrict__ uv, uint8_t* __restrict__ st,
                                                  double* __restrict__ rays,
                                                  uint8_t* __restrict__ st2) {
    __shared__ double s_ray[4][192];
    const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const size_t wfirst = i - lane;
    if (wfirst >= n) return;
    double x = 0.0, y = 0.0, z = 1.0;
    if (i < n) {
        x = xyz[3 * i];
        y = xyz[3 * i + 1];
        z = xyz[3 * i + 2];
        put2<true>(uv + 2 * i, x + z, y + z);
        __builtin_nontemporal_store((uint8_t)(z < 0.0), st + i);
    }
    if (wfirst + 64 <= n) {
        double* sr = s_ray[wid];
        sr[3 * lane] = x * 0.5;
        sr[3 * lane + 1] = y * 0.5;
        sr[3 * lane + 2] = z * 0.5;
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        double* dst = rays + 3 * wfirst;
        put2<true>(dst + 2 * lane, sr[2 * lane], sr[2 * lane + 1]);
        if (lane < 32) put2<true>(dst + 128 + 2 * lane, sr[128 + 2 * lane], sr[129 + 2 * lane]);
    } else if (i < n) {
        rays[3 * i] = x * 0.5;
        rays[3 * i + 1] = y * 0.5;
        rays[3 * i + 2] = z * 0.5;
    }
    if (i < n) __builtin_nontemporal_store((uint8_t)(z > 8.0), st2 + i);
}

}  // namespace

extern "C" int acm_probe_round_trip(size_t n, const double* xyz, double* uv, uint8_t* st,
                                    double* rays, uint8_t* st2, void* stream) {
    hipLaunchKernelGGL(k_rt_mimic, dim3(blocks(n)), dim3(256), 0, (hipStream_t)stream, n, xyz, uv,
                       st, rays, st2);
    return (int)hipGetLastError();
}

// (r06) camera_models.hpp's sqrt_rn against the compiler's sqrt, bit for bit
// (tests/test_gpu_sqrt_rn.py): *mismatches counts the inputs whose results
// differ; the first few (input, sqrt, sqrt_rn) triples go to `first`.
#include "../apex-camera-models_amd/csrc/camera_models.hpp"

__global__ __launch_bounds__(256) void k_sqrt_rn_check(const double* __restrict__ a, size_t n,
                                                       unsigned long long* mismatches,
                                                       double* first) {
    const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const double x = a[i];
    const double r0 = sqrt(x);
    const double r1 = acm::sqrt_rn(x);
    if (__double_as_longlong(r0) != __double_as_longlong(r1)) {
        const unsigned long long k = atomicAdd(mismatches, 1ull);
        if (k < 8) {
            first[3 * k] = x;
            first[3 * k + 1] = r0;
            first[3 * k + 2] = r1;
        }
    }
}

extern "C" int acm_probe_sqrt_rn(const double* a, size_t n, unsigned long long* mismatches,
                                 double* first, void* stream) {
    if (n == 0) return 0;
    hipLaunchKernelGGL(k_sqrt_rn_check, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                       (hipStream_t)stream, a, n, mismatches, first);
    return hipGetLastError() == hipSuccess ? 0 : 1;
}
