/* Exercises every oracle entry point on edge-heavy inputs; built by
 * tests/test_oracle_sanitized.py with -fsanitize=address,undefined so that
 * any out-of-bounds access, leak, overflow or undefined shift in the CPU
 * checker fails the CPU suite (sanitizers on the
 * oracle).  Prints "ok" and exits 0 when the run is clean. */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "acm_oracle.h"

static const double PARAMS[7][9] = {
    {460.0, 460.0, 320.0, 240.0},                                             /* Pinhole */
    {461.6, 460.3, 366.3, 249.1, -0.28, 0.07, 0.0002, 0.00002, 0.0},           /* RadTan */
    {190.97, 190.97, 254.93, 256.90, 0.0034, 0.0008, -0.0023, 0.0003},          /* KB */
    {157.9, 157.8, 254.9, 256.9, 0.64, -0.2},                                  /* DS */
    {349.1, 349.1, 254.9, 256.9, 0.56},                                        /* UCM */
    {313.4, 313.4, 254.9, 256.9, 0.59, 1.06},                                  /* EUCM */
    {370.0, 370.0, 255.0, 257.0, 0.9},                                         /* FOV */
};
static const uint32_t W = 512, H = 512;

int main(void) {
    enum { N = 4096 };
    double *xyz = malloc(sizeof(double) * 3 * N), *uv = malloc(sizeof(double) * 2 * N);
    double *ray = malloc(sizeof(double) * 3 * N), *res = malloc(sizeof(double) * 2 * N);
    double *jac = malloc(sizeof(double) * 2 * N * 9);
    uint8_t *st = malloc(N);
    unsigned s = 12345u;
    for (int i = 0; i < N; ++i) {
        s = s * 1103515245u + 12345u;
        double a = ((s >> 8) & 0xFFFF) / 32768.0 - 1.0;
        s = s * 1103515245u + 12345u;
        double b = ((s >> 8) & 0xFFFF) / 32768.0 - 1.0;
        s = s * 1103515245u + 12345u;
        double c = ((s >> 8) & 0xFFFF) / 16384.0 - 0.5;
        xyz[3 * i] = a;
        xyz[3 * i + 1] = b;
        xyz[3 * i + 2] = c;
    }
    /* edge points: origin, behind, on axis, tiny z, NaN, inf, huge */
    const double edge[][3] = {{0, 0, 0}, {0, 0, -1}, {0, 0, 1}, {1e-300, 0, 1e-300},
                              {NAN, 0, 1}, {INFINITY, 1, 1}, {1e300, 1e300, 1}, {0, 0, 1e-9}};
    for (unsigned k = 0; k < sizeof(edge) / sizeof(edge[0]); ++k)
        memcpy(xyz + 3 * k, edge[k], sizeof(edge[k]));
    double acc = 0.0;
    for (int m = 0; m < 7; ++m) {
        const double *p = PARAMS[m];
        oracle_project_batch(m, p, W, H, N, xyz, uv, st, jac);
        for (int i = 0; i < 2 * N; ++i)
            if (isnan(uv[i])) uv[i] = (i & 1) ? -5.0 : 1e9;  /* out-of-image pixels too */
        oracle_unproject_batch(m, p, W, H, N, uv, ray, st);
        oracle_residual_jacobian_batch(m, p, W, H, N, xyz, uv, m & 1, res, jac, st);
        double JtJ[81], Jtr[9], cost;
        uint64_t nv;
        oracle_normal_equations(m, p, W, H, N, xyz, uv, m & 1, JtJ, Jtr, &cost, &nv);
        double out[6];
        oracle_reprojection_error(m, p, W, H, N, xyz, uv, out);
        size_t total = 0, cap = 600;
        double *suv = malloc(sizeof(double) * 2 * cap), *sxyz = malloc(sizeof(double) * 3 * cap);
        size_t kept = oracle_sample_points(m, p, W, H, 500, cap, suv, sxyz, &total);
        if (kept > 1) {
            double *A = malloc(sizeof(double) * 2 * kept * 4), *bv = malloc(sizeof(double) * 2 * kept);
            oracle_linear_estimation_system(m, p, kept, sxyz, suv, A, bv);
            free(A);
            free(bv);
        }
        if (m == 6) {
            double es[ORACLE_FOV_GRID], vc[ORACLE_FOV_GRID];
            acc += oracle_fov_grid_search(p, kept, sxyz, suv, es, vc);
        }
        uint8_t *img = malloc(64 * 48 * 3), *outimg = malloc(64 * 48 * 3);
        for (int i = 0; i < 64 * 48 * 3; ++i) img[i] = (uint8_t)(i * 7);
        const double target[4] = {p[0] / 8, p[1] / 8, 32, 24};
        oracle_undistort_image(m, p, 64, 48, target, m & 1, img, outimg);
        acc += outimg[100] + cost + (double)kept;
        free(img);
        free(outimg);
        free(suv);
        free(sxyz);
    }
    free(xyz);
    free(uv);
    free(ray);
    free(res);
    free(jac);
    free(st);
    printf("ok %g\n", isfinite(acc) ? 1.0 : 0.0);
    return 0;
}
