// Experiment (not part of libacm.so): Kannala-Brandt unprojection with two
// pixels per lane and the two Newton loops merged into one, so every wave
// carries two independent FP64 dependency chains, against the production
// one-pixel-per-lane form (KannalaBrandt::unproject).  Outputs must be
// bit-identical: each pixel runs the same operations in the same order
// (kannala_brandt.rs:445-562); only the interleaving differs.
//
//   make -C tools build/libexp_u2.so ; python tools/exp_unproject2.py
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../apex-camera-models_amd/csrc/camera_models.hpp"

using acm::Cam;
using KB = acm::KannalaBrandt<double>;

struct ExpCam {
    double p[9];
    uint32_t width, height;
    double ifx, ify;
};

__device__ __forceinline__ Cam<double> mk(const ExpCam& e) {
    Cam<double> c;
#pragma unroll
    for (int i = 0; i < 9; ++i) c.p[i] = e.p[i];
    c.w = (double)e.width;
    c.h = (double)e.height;
    c.wi = e.width;
    c.hi = e.height;
    c.ifx = e.ifx;
    c.ify = e.ify;
    c.uk[0] = c.uk[1] = 0.0;
    return c;
}

__device__ __forceinline__ void st_nt(double* p, double v) { __builtin_nontemporal_store(v, p); }

__global__ __launch_bounds__(256) void k_one(ExpCam e, size_t n, const double* __restrict__ uv,
                                              double* __restrict__ rays,
                                              uint8_t* __restrict__ status) {
    const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const Cam<double> c = mk(e);
    const double2 q = *reinterpret_cast<const double2*>(uv + 2 * i);
    double X, Y, Z;
    const uint8_t st = KB::unproject(c, q.x, q.y, X, Y, Z);
    if (st != acm::ST_OK) X = Y = Z = __builtin_nan("");
    st_nt(rays + 3 * i, X);
    st_nt(rays + 3 * i + 1, Y);
    st_nt(rays + 3 * i + 2, Z);
    status[i] = st;
}

// The production unprojection split at the Newton loop (same operations).
struct Pre {
    double mx, my, ru, theta;
    bool out, conv, act;
};

__device__ __forceinline__ Pre pre(const Cam<double>& c, double u, double v) {
    Pre s;
    const double fx = c.p[0], fy = c.p[1], cx = c.p[2], cy = c.p[3];
    s.out = c.wi > 0 && c.hi > 0 && (u < 0.0 || u >= c.w || v < 0.0 || v >= c.h);
    s.mx = acm::div_by_f(u - cx, fx, c.ifx);
    s.my = acm::div_by_f(v - cy, fy, c.ify);
    double ru = sqrt(s.mx * s.mx + s.my * s.my);
    ru = fmin(ru, acm::kPi / 2.0);
    s.ru = ru;
    s.theta = ru;
    s.conv = true;
    s.act = ru > 1e-6;
    if (!s.act) {
        if (ru > 0.0) s.conv = false;
        else s.theta = 0.0;
    }
    return s;
}

__device__ __forceinline__ void newton_pass(const Cam<double>& c, Pre& s, int i) {
    const double k1 = c.p[4], k2 = c.p[5], k3 = c.p[6], k4 = c.p[7];
    const double theta = s.theta;
    double theta2 = theta * theta;
    double theta4 = theta2 * theta2;
    double theta6 = theta4 * theta2;
    double theta8 = theta4 * theta4;
    double k1t2 = k1 * theta2, k2t4 = k2 * theta4, k3t6 = k3 * theta6, k4t8 = k4 * theta8;
    double f = theta * (1.0 + k1t2 + k2t4 + k3t6 + k4t8) - s.ru;
    double fp = 1.0 + (3.0 * k1t2) + (5.0 * k2t4) + (7.0 * k3t6) + (9.0 * k4t8);
    const bool flat = fabs(fp) < acm::kEps;
    double delta = f / fp;
    const bool a = s.act;
    if (a && flat) {
        s.conv = false;
        s.act = false;
    } else if (a) {
        s.theta = theta - delta;
        if (fabs(delta) < 1e-6) s.act = false;
        else if (i == 9) {
            s.conv = false;
            s.act = false;
        }
    }
}

__device__ __forceinline__ uint8_t post(const Pre& s, double& X, double& Y, double& Z) {
    if (s.out) {
        X = Y = Z = __builtin_nan("");
        return acm::ST_POINT_IS_OUT_SIDE_IMAGE;
    }
    const bool small = fabs(s.ru) < acm::kEps;
    double sn, co;
    acm::sincos_0_2(s.theta, &sn, &co);
    const double ir = acm::nr_range(s.ru) ? acm::rcp_nr(s.ru) : 1.0 / s.ru;
    const double xc = small ? 0.0 : s.mx * ir;
    const double yc = small ? 0.0 : s.my * ir;
    const double px = sn * xc, py = sn * yc;
    const double n2 = px * px + py * py + co * co;
    const double in = acm::nr_range(n2) ? acm::rsq_nr(n2) : 1.0 / sqrt(n2);
    X = px * in;
    Y = py * in;
    Z = co * in;
    return s.conv ? acm::ST_OK : acm::ST_NUMERICAL_ERROR;
}

__global__ __launch_bounds__(256) void k_two(ExpCam e, size_t n, const double* __restrict__ uv,
                                              double* __restrict__ rays,
                                              uint8_t* __restrict__ status) {
    const size_t i0 = 2 * ((size_t)blockIdx.x * 256 + threadIdx.x);
    if (i0 >= n) return;
    const bool has1 = i0 + 1 < n;
    const Cam<double> c = mk(e);
    const double2 q0 = *reinterpret_cast<const double2*>(uv + 2 * i0);
    const double2 q1 = has1 ? *reinterpret_cast<const double2*>(uv + 2 * i0 + 2) : q0;
    Pre s0 = pre(c, q0.x, q0.y), s1 = pre(c, q1.x, q1.y);
    if (s0.out) s0.act = false;  // the production code returns before Newton
    if (s1.out) s1.act = false;
    for (int i = 0; i < 10 && (s0.act || s1.act); ++i) {
        newton_pass(c, s0, i);
        newton_pass(c, s1, i);
    }
    double X0, Y0, Z0, X1, Y1, Z1;
    uint8_t st0 = post(s0, X0, Y0, Z0), st1 = post(s1, X1, Y1, Z1);
    if (st0 != acm::ST_OK) X0 = Y0 = Z0 = __builtin_nan("");
    if (st1 != acm::ST_OK) X1 = Y1 = Z1 = __builtin_nan("");
    st_nt(rays + 3 * i0, X0);
    st_nt(rays + 3 * i0 + 1, Y0);
    st_nt(rays + 3 * i0 + 2, Z0);
    status[i0] = st0;
    if (has1) {
        st_nt(rays + 3 * i0 + 3, X1);
        st_nt(rays + 3 * i0 + 4, Y1);
        st_nt(rays + 3 * i0 + 5, Z1);
        status[i0 + 1] = st1;
    }
}

extern "C" int exp_unproject(int variant, const ExpCam* cam, size_t n, const double* uv,
                             double* rays, uint8_t* status, void* stream) {
    hipStream_t s = (hipStream_t)stream;
    if (variant == 1) {
        hipLaunchKernelGGL(k_one, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, *cam, n, uv,
                           rays, status);
    } else {
        const size_t lanes = (n + 1) / 2;
        hipLaunchKernelGGL(k_two, dim3((unsigned)((lanes + 255) / 256)), dim3(256), 0, s, *cam, n,
                           uv, rays, status);
    }
    return hipGetLastError() == hipSuccess ? 0 : -4;
}
