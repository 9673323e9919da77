/* Torch-free host program over the C-ABI, the same calls a Rust `extern "C"`
 * binding makes.  Projects the reference's five
 * test points (tests/model_conversions.rs:9-17) with the KB sample camera
 * (samples/kannala_brandt.yaml), prints uv + status + the 2x8 Jacobian rows
 * and the round trip through unproject.
 *   gcc -O2 -I include examples/c_host_project.c \
 *       -L apex-camera-models_amd/lib -lacm -Wl,-rpath,$PWD/apex-camera-models_amd/lib -lm
 */
#include <math.h>
#include <stdio.h>
#include <stdlib.h>

#include "acm.h"

#define CHECK(x)                                                                 \
    do {                                                                         \
        int rc_ = (x);                                                           \
        if (rc_ < 0) {                                                           \
            fprintf(stderr, "%s failed: %d %s\n", #x, rc_, acm_last_error());    \
            return 1;                                                            \
        }                                                                        \
    } while (0)

int main(void) {
    const double params[8] = {190.97847715128717, 190.9733070521226, 254.93170605935475,
                              256.8974428996504, 0.0034823894022493434, 0.0007150348452162257,
                              -0.0020532361418706202, 0.00020293673591811182};
    enum { N = 7, P = 8 };
    const double xyz[3 * N] = {0.1, 0.1, 1.0, 0.3, 0.0, 1.5, -0.2, 0.3, 2.0, -0.3, -0.2, 1.8,
                               0.15, -0.25, 2.5, 0.0, 0.0, 0.0, 0.1, 0.2, -1.0};
    acm_camera cam;
    CHECK(acm_set_device(0));
    CHECK(acm_camera_init(&cam, ACM_KANNALA_BRANDT, params, 8, 512, 512));
    double *d_xyz, *d_uv, *d_jac, *d_ray;
    uint8_t *d_st, *d_st2;
    CHECK(acm_device_malloc((void **)&d_xyz, sizeof xyz));
    CHECK(acm_device_malloc((void **)&d_uv, 2 * N * sizeof(double)));
    CHECK(acm_device_malloc((void **)&d_jac, 2 * N * P * sizeof(double)));
    CHECK(acm_device_malloc((void **)&d_ray, 3 * N * sizeof(double)));
    CHECK(acm_device_malloc((void **)&d_st, N));
    CHECK(acm_device_malloc((void **)&d_st2, N));
    CHECK(acm_memcpy_htod(d_xyz, xyz, sizeof xyz, NULL));
    CHECK(acm_project(&cam, N, d_xyz, ACM_LAYOUT_AOS, d_uv, d_st, d_jac, NULL));
    CHECK(acm_unproject(&cam, N, d_uv, d_ray, ACM_LAYOUT_AOS, d_st2, NULL));
    double uv[2 * N], jac[2 * N * P], ray[3 * N];
    uint8_t st[N], st2[N];
    CHECK(acm_memcpy_dtoh(uv, d_uv, sizeof uv, NULL));
    CHECK(acm_memcpy_dtoh(jac, d_jac, sizeof jac, NULL));
    CHECK(acm_memcpy_dtoh(ray, d_ray, sizeof ray, NULL));
    CHECK(acm_memcpy_dtoh(st, d_st, sizeof st, NULL));
    CHECK(acm_memcpy_dtoh(st2, d_st2, sizeof st2, NULL));
    CHECK(acm_stream_synchronize(NULL));
    int bad = 0;
    for (int i = 0; i < N; ++i) {
        printf("p%d status %u uv %.17g %.17g  dudfx %.17g dvdk4 %.17g", i, st[i], uv[2 * i],
               uv[2 * i + 1], jac[0 * 2 * N + 2 * i], jac[7 * 2 * N + 2 * i + 1]);
        if (st[i] == 0 && st2[i] == 0) {
            const double *p = xyz + 3 * i, *r = ray + 3 * i;
            double n = sqrt(p[0] * p[0] + p[1] * p[1] + p[2] * p[2]);
            double dot = (p[0] * r[0] + p[1] * r[1] + p[2] * r[2]) / n;
            printf("  round-trip dot %.17g", dot);
            if (!(dot > 0.99)) bad = 1; /* tests/model_conversions.rs:41-59 */
        }
        printf("\n");
    }
    /* reference KATs: (0,0,0) -> PointAtCameraCenter, z<0 -> PointIsOutSideImage */
    if (st[5] != ACM_STATUS_POINT_AT_CAMERA_CENTER || st[6] != ACM_STATUS_POINT_IS_OUT_SIDE_IMAGE)
        bad = 1;
    acm_device_free(d_xyz); acm_device_free(d_uv); acm_device_free(d_jac);
    acm_device_free(d_ray); acm_device_free(d_st); acm_device_free(d_st2);
    printf(bad ? "FAIL\n" : "OK\n");
    return bad;
}
