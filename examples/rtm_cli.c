/*
 * rtm_cli — a compiled C caller of the rtm ABI (include/rtm.h), standing in for
 * the reference's own driver (testscene_closelyOrbitingSphere, main.rs:1468-1633:
 * build the scene of frame f, rasterize + march the shadow viewport, rasterize
 * the eye viewport, renderColorImage, writeColorImage to imgNNNNNN.ppm).  The
 * Rust binding a maintainer would add is in INTEGRATION.md; Rust is not in this
 * image, so this program is the compiled, linked proof that the boundary is a
 * plain C ABI: it includes only rtm.h and links only librtm.so.
 *
 *   rtm_cli [-w W] [-h H] [-k STEPS] [-f FIRST_FRAME] [-n FRAMES] [-b]
 *           [--ppm PATH] [--raw PATH]
 *
 *   -b          Scene A-bench's tilted patch instead of the
 *               reference's hard-coded one (main.rs:2024-2029)
 *   --ppm PATH  writeColorImage of the last frame (P3 text, main.rs:660-704),
 *               encoded on the host from rtm_encode_thresholds
 *   --raw PATH  the last frame's RGBA f32 bytes (row-major y*W+x)
 *
 * Prints one line per run: frames, seconds, Mpixels/s of rtm_render (blocking,
 * frame returned to host memory: the PCIe-inclusive drop-in rate).
 */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "rtm.h"

/* testscene_closelyOrbitingSphere frame f (main.rs:1475-1522): two blue spheres
 * on the z axis and a red one orbiting in the y-z plane */
static void scene_a(int frame, rtm_sphere sph[3]) {
    const double f = (double)frame;
    const double blue[3] = {0.02, 0.02, 1.0}, red[3] = {0.9, 0.2, 0.2};
    memset(sph, 0, 3 * sizeof *sph);
    sph[0].id = 0;
    sph[0].pos[2] = 0.5;
    sph[0].r = 0.2;
    sph[1].id = 1;
    sph[1].pos[2] = 0.5 + 0.2 * 2.0;
    sph[1].r = 0.2;
    sph[2].id = 2;
    sph[2].pos[0] = -0.0;
    sph[2].pos[1] = sin(f * 0.025) * 0.7;
    sph[2].pos[2] = cos(f * 0.025) * 0.7;
    sph[2].r = 0.1;
    for (int k = 0; k < 3; k++) {
        sph[0].color[k] = blue[k];
        sph[1].color[k] = blue[k];
        sph[2].color[k] = red[k];
    }
}

static void camera(rtm_camera* c, double px, double dx, double dy, double dz, double ux, double uy, double uz,
                   double sx, double sy, double sz) {
    memset(c, 0, sizeof *c);
    c->type = RTM_CAMERA_ORTHOGONAL;
    c->pos[0] = px;
    c->dir[0] = dx, c->dir[1] = dy, c->dir[2] = dz;
    c->up[0] = ux, c->up[1] = uy, c->up[2] = uz;
    c->side[0] = sx, c->side[1] = sy, c->side[2] = sz;
}

/* writeColorImage's byte per channel: c.max(0.0).min(1.0), powf(1/2.2), *255,
 * truncated -- evaluated as the rank of v among the library's 256 exact
 * thresholds (T[k] = the smallest v whose byte is >= k) */
static int enc(float c, const float t[256]) {
    float v = fmaxf(c, 0.0f); /* NaN -> 0, as f32::max */
    v = fminf(v, 1.0f);
    int lo = 0, hi = 255; /* largest k with t[k] <= v */
    while (lo < hi) {
        const int mid = (lo + hi + 1) / 2;
        if (t[mid] <= v) lo = mid;
        else hi = mid - 1;
    }
    return lo;
}

static int write_ppm(const char* path, const float* rgba, int w, int h) {
    float t[256];
    if (rtm_encode_thresholds(t) != RTM_OK) return -1;
    FILE* f = fopen(path, "wb");
    if (!f) return -1;
    fprintf(f, "P3\n%d %d\n255\n", w, h);
    for (int y = 0; y < h; y++) {
        for (int x = 0; x < w; x++) {
            const float* p = rgba + ((size_t)y * w + x) * 4;
            fprintf(f, "%d %d %d  ", enc(p[0], t), enc(p[1], t), enc(p[2], t));
        }
        fputc('\n', f);
    }
    return fclose(f);
}

static double now(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec + ts.tv_nsec * 1e-9;
}

int main(int argc, char** argv) {
    int w = 512, h = 512, steps = 500, first = 0, frames = 1, bench_patch = 0;
    const char *ppm = NULL, *raw = NULL;
    for (int i = 1; i < argc; i++) {
        const char* a = argv[i];
        const int more = i + 1 < argc;
        if (!strcmp(a, "-w") && more) w = atoi(argv[++i]);
        else if (!strcmp(a, "-h") && more) h = atoi(argv[++i]);
        else if (!strcmp(a, "-k") && more) steps = atoi(argv[++i]);
        else if (!strcmp(a, "-f") && more) first = atoi(argv[++i]);
        else if (!strcmp(a, "-n") && more) frames = atoi(argv[++i]);
        else if (!strcmp(a, "-b")) bench_patch = 1;
        else if (!strcmp(a, "--ppm") && more) ppm = argv[++i];
        else if (!strcmp(a, "--raw") && more) raw = argv[++i];
        else {
            fprintf(stderr, "usage: %s [-w W] [-h H] [-k STEPS] [-f FIRST] [-n FRAMES] [-b] [--ppm P] [--raw P]\n",
                    argv[0]);
            return 2;
        }
    }
    if (rtm_abi_version() != RTM_ABI_VERSION) {
        fprintf(stderr, "librtm ABI %d, header %d\n", rtm_abi_version(), RTM_ABI_VERSION);
        return 1;
    }
    if (w <= 0 || h <= 0 || frames <= 0) {
        fprintf(stderr, "bad size or frame count\n");
        return 2;
    }
    /* the shadow camera looks along +z (main.rs:1552-1563), the eye along +x from (-1,0,0) (main.rs:1598-1609) */
    rtm_camera shadow, eye;
    camera(&shadow, 0.0, 0.0, 0.0, 1.0, 0.0, 1.0, 0.0, 1.0, 0.0, 0.0);
    camera(&eye, -1.0, 1.0, 0.0, 0.0, 0.0, 1.0, 0.0, 0.0, 0.0, 1.0);
    const rtm_patch patch = bench_patch ? (rtm_patch){0.3, 2.1, 0.9, 2.7} : (rtm_patch){0.1, 0.1, 0.1, 0.1};
    float* img = (float*)malloc((size_t)w * h * 4 * sizeof(float));
    if (!img) return 1;
    double t0 = 0.0;
    for (int i = 0; i < frames; i++) {
        rtm_sphere sph[3];
        scene_a(first + i, sph);
        rtm_scene sc;
        memset(&sc, 0, sizeof sc);
        sc.spheres = sph;
        sc.n_spheres = 3;
        sc.patches = &patch;
        sc.n_patches = 1;
        if (i == 1 || frames == 1) t0 = now(); /* frame 0 pays the context/table set-up when frames > 1 */
        const int rc = rtm_render(&sc, &eye, &shadow, w, h, steps, 0, img);
        if (rc != RTM_OK) {
            fprintf(stderr, "rtm_render: %d (%s)\n", rc, rtm_last_error());
            free(img);
            return 1;
        }
    }
    const double dt = now() - t0;
    const int timed = frames > 1 ? frames - 1 : 1;
    printf("{\"frames\": %d, \"width\": %d, \"height\": %d, \"steps\": %d, \"seconds\": %.6f, "
           "\"mpixels_per_s\": %.2f, \"path\": \"rtm_render (host output)\"}\n",
           timed, w, h, steps, dt, (double)w * h * timed / dt / 1e6);
    int rc = 0;
    if (raw) {
        FILE* f = fopen(raw, "wb");
        rc |= !f || fwrite(img, sizeof(float), (size_t)w * h * 4, f) != (size_t)w * h * 4;
        if (f) rc |= fclose(f) != 0;
    }
    if (ppm) rc |= write_ppm(ppm, img, w, h) != 0;
    free(img);
    return rc ? 1 : 0;
}
