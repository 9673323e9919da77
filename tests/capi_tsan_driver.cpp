// Concurrency hygiene of libacm's host code (reentrant C-ABI,
// the `&self` / Send + Sync use of trait CameraModel, mod.rs:241-340):
// threads call acm_set_tuning on every knob while other threads run the
// host-side entry points (camera init / validation, R-factor merge and SVD
// solve, FOV grid selection, sample grid, statistics merge, workspace sizes,
// error strings).  Built by tests/test_capi_sanitized.py with host-side
// -fsanitize=thread; any data race fails the run.  Needs no GPU (no kernel
// is launched).
#include <atomic>
#include <cmath>
#include <cstdio>
#include <thread>
#include <vector>

#include "acm.h"

static std::atomic<int> g_bad{0};

static void tuner(int seed) {
    for (int it = 0; it < 2000; ++it) {
        const int key = (it + seed) % 12;
        const int v = (it * 7 + seed) % 5 - 1;
        acm_set_tuning(key, v);
    }
}

static void host_api(int seed) {
    unsigned s = 12345u + (unsigned)seed;
    auto rnd = [&]() { s = s * 1103515245u + 12345u; return ((s >> 8) & 0xFFFF) / 65536.0; };
    for (int it = 0; it < 300; ++it) {
        const int m = it % 7;
        acm_camera cam;
        double p[9] = {300, 300, 250, 250, 0.5, 0.1, 0.01, 0.001, 0.0};
        const int P = acm_num_params(m);
        if (acm_camera_init(&cam, m, p, P, 512, 512) != 0) g_bad++;
        (void)acm_validate_params(&cam);
        const int k = acm_linear_system_columns(m);
        if (k > 0) {
            const int M = k + 1, S = M * (M + 1) / 2;
            std::vector<double> a(S), b(S);
            for (int i = 0; i < S; ++i) { a[i] = rnd() - 0.3; b[i] = rnd() - 0.6; }
            acm_linear_system_r_merge(m, a.data(), b.data());
            acm_camera c2 = cam;
            acm_linear_estimation_solve(&c2, 1000, a.data(), 0);
        }
        if (m == ACM_FOV) {
            std::vector<double> grid(2 * ACM_FOV_GRID_SIZE);
            for (auto& g : grid) g = rnd() + 1.0;
            acm_fov_grid_select(&cam, grid.data());
        }
        uint32_t nx, ny;
        acm_sample_points_grid(752, 480, 1000 + it, &nx, &ny);
        double parts[16] = {1, 0.1, 2, 1, 0.5, 10, 10, 20, 1, 0.2, 3, 1.2, 0.6, 5, 6, 9};
        double res[8];
        acm_reprojection_stats_merge(2, parts, res);
        if (!(res[5] == 15.0)) g_bad++;
        (void)acm_normal_equations_workspace_size(m, 1000 + it);
        (void)acm_sample_points_workspace_size(&cam, 5000);
        acm_set_tuning(99, 0);  // an error: writes this thread's error string
        (void)acm_last_error();
    }
}

int main() {
    std::vector<std::thread> th;
    for (int t = 0; t < 2; ++t) th.emplace_back(tuner, t);
    for (int t = 0; t < 3; ++t) th.emplace_back(host_api, t);
    for (auto& x : th) x.join();
    for (int key = 0; key < 12; ++key) acm_set_tuning(key, key == 2 || key == 4 ? 0 : -1);
    acm_set_tuning(3, 1);
    printf("ok %d\n", g_bad.load() == 0 ? 1 : 0);
    return g_bad.load() == 0 ? 0 : 1;
}
