// lm_core.hpp -- the bounded Levenberg-Marquardt state machine of
// acm_lm_optimize (solver.hip), host code: start() clamps the start point,
// then the driver alternates one normal-equations evaluation on the GPU
// (k_normal_eq + k_ne_finish_cols) with consume(), which advances the state
// to the next parameter vector to evaluate or ends the run.  (r04 also ran
// this state machine on the device, behind each evaluation; it measured
// slower than the host loop and was removed in r05.)
//
// Reference: bin/camera_converter.rs:381-420 (apex-solver LM with bounds,
// max_iterations = 100, cost_tolerance = 1e-6, parameter_tolerance = 1e-8,
// gradient_tolerance = 1e-6).  apex-solver 0.1.5's LM source is absent, so
// this is a standard bounded LM (Nielsen damping update, Marquardt diagonal
// scaling floored at 1e-12 max(diag, 1), projection onto the bounds);
// DESIGN.md §8 documents the (unpinned) choice.
#pragma once

#include <math.h>

#include "acm.h"

namespace acm {
namespace lm {

enum : int { NEED_EVAL = 0, DONE = 1 };

// Everything the loop carries between evaluations.  phase 0: the first
// evaluation (at the clamped start) is pending; 1: a trial step's.
struct State {
    int P, it, evals, term, phase, pad;
    double x[9], xn[9], h[9];
    double A[81], g[9];
    double F, nv, mu, nu, dmax, initial_cost;
};

inline bool cholesky_solve(int P, const double* A, const double* b, double* x) {
    double L[81];
    for (int i = 0; i < P; ++i)
        for (int j = 0; j <= i; ++j) {
            double s = A[i * P + j];
            for (int q = 0; q < j; ++q) s -= L[i * P + q] * L[j * P + q];
            if (i == j) {
                if (!(s > 0.0)) return false;
                L[i * P + i] = sqrt(s);
            } else {
                L[i * P + j] = s / L[j * P + j];
            }
        }
    double y[9];
    for (int i = 0; i < P; ++i) {
        double s = b[i];
        for (int q = 0; q < i; ++q) s -= L[i * P + q] * y[q];
        y[i] = s / L[i * P + i];
    }
    for (int i = P - 1; i >= 0; --i) {
        double s = y[i];
        for (int q = i + 1; q < P; ++q) s -= L[q * P + i] * x[q];
        x[i] = s / L[i * P + i];
    }
    return true;
}

inline void clamp(const acm_lm_config& cfg, int P, double* x) {
    if (!cfg.has_bounds) return;
    for (int i = 0; i < P; ++i) x[i] = fmin(fmax(x[i], cfg.lower[i]), cfg.upper[i]);
}

inline double ginf(int P, const double* g) {
    double m = 0.0;
    for (int i = 0; i < P; ++i) m = fmax(m, fabs(g[i]));
    return m;
}

// The start point: the parameters, clamped; the first evaluation is at xn.
inline void start(State& s, const acm_lm_config& cfg, int P, const double* params) {
    s.P = P;
    s.it = 0;
    s.evals = 0;
    s.term = ACM_LM_MAX_ITERATIONS;
    s.phase = 0;
    s.pad = 0;
    for (int i = 0; i < 9; ++i) s.x[i] = s.xn[i] = s.h[i] = 0.0;
    for (int i = 0; i < P; ++i) s.x[i] = params[i];
    clamp(cfg, P, s.x);
    for (int i = 0; i < P; ++i) s.xn[i] = s.x[i];
    s.F = s.nv = s.mu = s.nu = s.dmax = s.initial_cost = 0.0;
}

// Iterate until the next evaluation is needed (NEED_EVAL, s.xn and s.h set)
// or the run ends (DONE, s.term set).  Cholesky failures raise the damping
// and retry without an evaluation, as does nothing else.
inline int advance(State& s, const acm_lm_config& cfg, int P) {
    while (s.term == ACM_LM_MAX_ITERATIONS && s.it < cfg.max_iterations) {
        ++s.it;
        // (JtJ + mu * diag(JtJ)) h = -g   (Marquardt scaling, floored)
        double Ad[81], mg[9], hstep[9];
        for (int i = 0; i < P * P; ++i) Ad[i] = s.A[i];
        for (int i = 0; i < P; ++i) {
            Ad[i * P + i] += s.mu * fmax(s.A[i * P + i], 1e-12 * fmax(s.dmax, 1.0));
            mg[i] = -s.g[i];
        }
        if (!cholesky_solve(P, Ad, mg, hstep)) {
            s.mu *= s.nu;
            s.nu *= 2.0;
            continue;
        }
        double xnorm = 0.0, hnorm = 0.0;
        for (int i = 0; i < P; ++i) s.xn[i] = s.x[i] + hstep[i];
        clamp(cfg, P, s.xn);
        for (int i = 0; i < P; ++i) {
            s.h[i] = s.xn[i] - s.x[i];
            hnorm += s.h[i] * s.h[i];
            xnorm += s.x[i] * s.x[i];
        }
        hnorm = sqrt(hnorm);
        xnorm = sqrt(xnorm);
        if (hnorm <= cfg.parameter_tolerance * (xnorm + cfg.parameter_tolerance)) {
            s.term = ACM_LM_PARAMETER;
            break;
        }
        return NEED_EVAL;
    }
    return DONE;
}

// Take the evaluation at s.xn -- res = [JtJ (P x P) | Jtr (P) | 0.5 r.r |
// n_valid], acm_normal_equations' layout -- then advance.  P == s.P (a
// compile-time constant in the device step kernel).
inline int consume(State& s, const acm_lm_config& cfg, const double* res,
                                      int P) {
    ++s.evals;
    const double* An = res;
    const double* gn = res + P * P;
    const double Fn = res[P * P + P], nvn = res[P * P + P + 1];
    if (s.phase == 0) {
        for (int i = 0; i < P * P; ++i) s.A[i] = An[i];
        for (int i = 0; i < P; ++i) s.g[i] = gn[i];
        s.F = Fn;
        s.nv = nvn;
        s.initial_cost = Fn;
        s.dmax = 0.0;
        for (int i = 0; i < P; ++i) s.dmax = fmax(s.dmax, s.A[i * P + i]);
        s.mu = cfg.initial_damping;
        s.nu = 2.0;
        if (!isfinite(s.F)) s.term = ACM_LM_FAILED;
        else if (ginf(P, s.g) <= cfg.gradient_tolerance) s.term = ACM_LM_GRADIENT;
        s.phase = 1;
        return advance(s, cfg, P);
    }
    // predicted reduction L(0) - L(h) = -(g.h + 0.5 h.A.h)
    double gh = 0.0, hAh = 0.0;
    for (int i = 0; i < P; ++i) {
        gh += s.g[i] * s.h[i];
        double t = 0.0;
        for (int j = 0; j < P; ++j) t += s.A[i * P + j] * s.h[j];
        hAh += s.h[i] * t;
    }
    const double pred = -(gh + 0.5 * hAh);
    const double rho = (isfinite(Fn) && pred > 0.0) ? (s.F - Fn) / pred : -1.0;
    if (rho > 0.0) {
        const double dF = s.F - Fn;
        const double Fold = s.F;
        for (int i = 0; i < P; ++i) s.x[i] = s.xn[i];
        for (int i = 0; i < P * P; ++i) s.A[i] = An[i];
        for (int i = 0; i < P; ++i) s.g[i] = gn[i];
        s.F = Fn;
        s.nv = nvn;
        const double t = 2.0 * rho - 1.0;
        s.mu *= fmax(1.0 / 3.0, 1.0 - t * t * t);
        s.nu = 2.0;
        if (ginf(P, s.g) <= cfg.gradient_tolerance) s.term = ACM_LM_GRADIENT;
        else if (dF <= cfg.cost_tolerance * Fold) s.term = ACM_LM_COST;
    } else {
        s.mu *= s.nu;
        s.nu *= 2.0;
        if (!isfinite(s.mu) || s.mu > 1e32) {
            s.term = ACM_LM_FAILED;
            return DONE;
        }
    }
    return advance(s, cfg, P);
}

}  // namespace lm
}  // namespace acm
