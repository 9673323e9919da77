// Host-side C-ABI hygiene: drives the host-only entry points of libacm
// (camera init / validation for every model and parameter count, the
// linear-estimation R-factor merge and SVD solve on random factors, the FOV
// grid selection, the sample grid, every tuning key and value, workspace
// sizes) under AddressSanitizer + UndefinedBehaviorSanitizer.  Built by
// tests/test_capi_sanitized.py: acm.hip and solver.hip with host-side
// -fsanitize=address,undefined.  Needs no GPU.
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include "acm.h"
int main() {
    unsigned s = 7u;
    auto rnd = [&]() { s = s * 1103515245u + 12345u; return ((s >> 8) & 0xFFFF) / 65536.0; };
    double acc = 0;
    for (int m = 0; m < 8; ++m) {
        int P = acm_num_params(m);
        acm_camera cam;
        double p[9] = {300, 300, 250, 250, 0.5, 0.1, 0.01, 0.001, 0.0};
        for (size_t cnt = 0; cnt <= 10; ++cnt) acm_camera_init(&cam, m, p, cnt, 512, 512);
        if (P < 0) continue;
        if (acm_camera_init(&cam, m, p, P, 512, 512) == 0) acc += acm_validate_params(&cam);
        int k = acm_linear_system_columns(m);
        if (k > 0) {
            int M = k + 1, S = M * (M + 1) / 2;
            std::vector<double> a(S), b(S);
            for (int t = 0; t < 200; ++t) {
                for (int i = 0; i < S; ++i) { a[i] = rnd() - 0.3; b[i] = rnd() - 0.6; }
                acm_linear_system_r_merge(m, a.data(), b.data());
                acm_camera c2 = cam;
                acm_linear_estimation_solve(&c2, 1000, a.data(), 0);
                acm_linear_estimation_solve(&c2, 1, a.data(), 0);
                acm_linear_estimation_solve(&c2, 1000, a.data(), 1);
                acc += c2.params[4];
            }
        }
    }
    acm_camera fov;
    double fp[5] = {300, 300, 250, 250, 1.0};
    acm_camera_init(&fov, ACM_FOV, fp, 5, 512, 512);
    std::vector<double> grid(2 * ACM_FOV_GRID_SIZE);
    for (auto& g : grid) g = rnd();
    acm_fov_grid_select(&fov, grid.data());
    uint32_t nx, ny;
    acm_sample_points_grid(752, 480, 100000000, &nx, &ny);
    acm_sample_points_grid(0, 480, 10, &nx, &ny);
    acm_lm_config cfg;
    acm_lm_default_config(&cfg);
    for (int key = 0; key < 13; ++key)
        for (int v = -3; v < 10; ++v) acm_set_tuning(key, v);
    for (int key = 0; key < 12; ++key) acm_set_tuning(key, key == 2 || key == 4 ? 0 : -1);
    acm_set_tuning(3, 1);
    acc += acm_normal_equations_workspace_size(2, 12345) + acm_median_workspace_size(999);
    double parts[16] = {1, 0.1, 2, 1, 0.5, 10, 10, 20, 1, 0.2, 3, 1.2, 0.6, 5, 6, 9}, mres[8];
    acm_reprojection_stats_merge(2, parts, mres);
    acm_reprojection_stats_merge(0, nullptr, mres);
    acc += mres[5];
    printf("ok %d\n", std::isfinite(acc) ? 1 : 0);
    return 0;
}
