/*
 * rtm_cli — a compiled C caller of the rtm ABI (include/rtm.h), standing in for
 * the reference's own driver (testscene_closelyOrbitingSphere, main.rs:1468-1633:
 * build the scene of frame f, rasterize + march the shadow viewport, rasterize
 * the eye viewport, renderColorImage, writeColorImage to imgNNNNNN.ppm).  The
 * Rust binding a maintainer would add is in INTEGRATION.md; Rust is not in this
 * image, so this program is the compiled, linked proof that the boundary is a
 * plain C ABI: it includes only rtm.h and links only librtm.so.
 *
 *   rtm_cli [-s SCENE] [-w W] [-h H] [-k STEPS] [-f FIRST_FRAME] [-n FRAMES] [-b]
 *           [-g N] [--ppm PATH] [--ppm-gpu PATH] [--raw PATH]
 *
 *   -s SCENE    orbit   testscene_closelyOrbitingSphere (main.rs:1468-1633, default)
 *               plane0  testscene_raytracingPlane0, main()'s default scene
 *                       (main.rs:910-1046, 1652): one capped cylinder, PERSPECTIVE eye
 *               plane0-disc  the same with the circle plane it has commented out
 *                       (main.rs:916-929)
 *               persp1  testscene_perspectiveSimple1 (main.rs:1059-1182)
 *               persp2  testscene_perspectiveSimple2 (main.rs:1184-1316)
 *               The non-orbit scenes have their shadow passes commented out in the
 *               reference (main.rs:998-1003, 1115-1120): RTM_FLAG_NO_MARCH |
 *               RTM_FLAG_NO_SHADOW_RASTER, and -k is ignored.
 *   -b          Scene A-bench's tilted patch instead of the
 *               reference's hard-coded one (main.rs:2024-2029)
 *   -g N        render every frame through an RCCL group of devices 0..N-1
 *               (rtm_group_create: ncclCommInitAll in this process; each device renders
 *               a row band, ONE gather assembles the frame on device 0,
 *               rtm_group_render returns it to host memory): the north star's
 *               tile-partitioned frame, called as a Rust host would call it
 *   --ppm PATH  writeColorImage of the last frame (P3 text, main.rs:660-704),
 *               encoded on the host from rtm_encode_thresholds
 *   --ppm-gpu PATH  the same file from the library's RGB8 output format
 *               (rtm_render_ex, RTM_FORMAT_RGB8: the encode runs in the eye pass)
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

/* normalize (main.rs:105-108): v.scale(1.0 / |v|) */
static void normalize3(double v[3]) {
    const double m = sqrt(v[0] * v[0] + v[1] * v[1] + v[2] * v[2]);
    const double inv = 1.0 / m;
    for (int k = 0; k < 3; k++) v[k] = v[k] * inv;
}

/* viewport0's PERSPECTIVE camera (main.rs:1016-1027; perspectiveSimple2 moves it to y = 1.5, main.rs:1283-1295) */
static void persp_camera(rtm_camera* c, double py) {
    memset(c, 0, sizeof *c);
    c->type = RTM_CAMERA_PERSPECTIVE;
    c->pos[1] = py;
    c->dir[2] = 1.0;
    c->up[1] = 1.0;
    c->side[0] = 1.0;
}

/* the non-orbit scenes: testscene_raytracingPlane0 (main.rs:931-943 cylinder, 916-929 disc)
 * and testscene_perspectiveSimple1/2 (main.rs:1069-1080, 1196-1221) */
static int other_scene(const char* name, rtm_scene* sc, rtm_sphere sph[2], rtm_capped_cylinder* cyl,
                       rtm_circle_plane* disc, rtm_camera* eye) {
    memset(sc, 0, sizeof *sc);
    persp_camera(eye, 0.0);
    if (!strcmp(name, "plane0") || !strcmp(name, "plane0-disc")) {
        memset(cyl, 0, sizeof *cyl);
        cyl->pa[0] = 0.01, cyl->pa[1] = 10.01, cyl->pa[2] = 10.01;
        cyl->pb[0] = 0.01, cyl->pb[1] = 0.01, cyl->pb[2] = 10.01;
        cyl->ra = 0.3, cyl->rb = 0.2;
        cyl->color[0] = 1.0, cyl->color[1] = 0.02, cyl->color[2] = 0.02;
        sc->capped_cylinders = cyl;
        sc->n_capped_cylinders = 1;
        if (!strcmp(name, "plane0-disc")) {
            memset(disc, 0, sizeof *disc);
            disc->pos[0] = 0.01, disc->pos[1] = 0.01, disc->pos[2] = 2.0;
            disc->n[0] = -1.0, disc->n[1] = 0.0, disc->n[2] = 1.0;
            normalize3(disc->n);
            disc->radius = 0.5;
            disc->color[0] = 0.02, disc->color[1] = 0.02, disc->color[2] = 1.0;
            sc->circle_planes = disc;
            sc->n_circle_planes = 1;
        }
        return 0;
    }
    if (!strcmp(name, "persp1") || !strcmp(name, "persp2")) {
        memset(sph, 0, 2 * sizeof *sph);
        for (int i = 0; i < 2; i++) {
            sph[i].id = i;
            sph[i].pos[0] = 0.01, sph[i].pos[1] = 0.01, sph[i].pos[2] = i ? 6.0 : 4.0;
            sph[i].r = 0.5;
            sph[i].color[0] = 0.02, sph[i].color[1] = i ? 1.0 : 0.02, sph[i].color[2] = i ? 0.02 : 1.0;
        }
        sc->spheres = sph;
        sc->n_spheres = strcmp(name, "persp1") ? 2 : 1;
        if (!strcmp(name, "persp2")) persp_camera(eye, 1.5);
        return 0;
    }
    return -1;
}

static int write_ppm_rgb8(const char* path, const uint8_t* rgb, int w, int h) {
    FILE* f = fopen(path, "wb");
    if (!f) return -1;
    fprintf(f, "P3\n%d %d\n255\n", w, h);
    for (int y = 0; y < h; y++) {
        for (int x = 0; x < w; x++) {
            const uint8_t* p = rgb + ((size_t)y * w + x) * 3;
            fprintf(f, "%d %d %d  ", p[0], p[1], p[2]);
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
    int w = 512, h = 512, steps = 500, first = 0, frames = 1, bench_patch = 0, group_n = 0;
    const char *ppm = NULL, *ppm_gpu = NULL, *raw = NULL, *scene_name = "orbit";
    for (int i = 1; i < argc; i++) {
        const char* a = argv[i];
        const int more = i + 1 < argc;
        if (!strcmp(a, "-w") && more) w = atoi(argv[++i]);
        else if (!strcmp(a, "-h") && more) h = atoi(argv[++i]);
        else if (!strcmp(a, "-k") && more) steps = atoi(argv[++i]);
        else if (!strcmp(a, "-f") && more) first = atoi(argv[++i]);
        else if (!strcmp(a, "-n") && more) frames = atoi(argv[++i]);
        else if (!strcmp(a, "-b")) bench_patch = 1;
        else if (!strcmp(a, "-g") && more) group_n = atoi(argv[++i]);
        else if (!strcmp(a, "-s") && more) scene_name = argv[++i];
        else if (!strcmp(a, "--ppm-gpu") && more) ppm_gpu = argv[++i];
        else if (!strcmp(a, "--ppm") && more) ppm = argv[++i];
        else if (!strcmp(a, "--raw") && more) raw = argv[++i];
        else {
            fprintf(stderr,
                    "usage: %s [-s orbit|plane0|plane0-disc|persp1|persp2] [-w W] [-h H] [-k STEPS] [-f FIRST] "
                    "[-n FRAMES] [-b] [-g N] [--ppm P] [--ppm-gpu P] [--raw P]\n",
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
    const int orbit = !strcmp(scene_name, "orbit");
    rtm_scene other;
    rtm_sphere osph[2];
    rtm_capped_cylinder ocyl;
    rtm_circle_plane odisc;
    int flags = 0;
    if (!orbit) {
        if (other_scene(scene_name, &other, osph, &ocyl, &odisc, &eye)) {
            fprintf(stderr, "unknown scene %s\n", scene_name);
            return 2;
        }
        flags = RTM_FLAG_NO_MARCH | RTM_FLAG_NO_SHADOW_RASTER;
        steps = 0;
    }
    float* img = (float*)malloc((size_t)w * h * 4 * sizeof(float));
    if (!img) return 1;
    rtm_group* group = NULL;
    if (group_n > 0) {
        const int rc = rtm_group_create(group_n, NULL, &group);
        if (rc != RTM_OK) {
            fprintf(stderr, "rtm_group_create: %d (%s)\n", rc, rtm_last_error());
            free(img);
            return 1;
        }
    }
    double t0 = 0.0;
    rtm_scene sc;
    rtm_sphere sph[3];
    for (int i = 0; i < frames; i++) {
        if (orbit) {
            scene_a(first + i, sph);
            memset(&sc, 0, sizeof sc);
            sc.spheres = sph;
            sc.n_spheres = 3;
            sc.patches = &patch;
            sc.n_patches = 1;
        } else {
            sc = other;
        }
        if (i == 1 || frames == 1) t0 = now(); /* frame 0 pays the context/table set-up when frames > 1 */
        const int rc = group ? rtm_group_render(group, &sc, &eye, &shadow, w, h, steps, flags, RTM_FORMAT_RGBA32F, img)
                             : rtm_render(&sc, &eye, &shadow, w, h, steps, flags, img);
        if (rc != RTM_OK) {
            fprintf(stderr, "%s: %d (%s)\n", group ? "rtm_group_render" : "rtm_render", rc, rtm_last_error());
            if (group) rtm_group_destroy(group);
            free(img);
            return 1;
        }
    }
    const double dt = now() - t0;
    if (group) rtm_group_destroy(group); /* (ncclCommDestroy: ~0.5 s, outside the timed frames) */
    const int timed = frames > 1 ? frames - 1 : 1;
    printf("{\"scene\": \"%s\", \"frames\": %d, \"width\": %d, \"height\": %d, \"steps\": %d, "
           "\"seconds\": %.6f, \"mpixels_per_s\": %.2f, \"path\": \"%s (host output)\", \"gpus\": %d}\n",
           scene_name, timed, w, h, steps, dt, (double)w * h * timed / dt / 1e6,
           group_n > 0 ? "rtm_group_render" : "rtm_render", group_n > 0 ? group_n : 1);
    int rc = 0;
    if (ppm_gpu) {
        uint8_t* rgb = (uint8_t*)malloc((size_t)w * h * 3);
        if (!rgb) rc = 1;
        else {
            const int r = rtm_render_ex(&sc, &eye, &shadow, w, h, steps, flags, RTM_FORMAT_RGB8, rgb);
            if (r != RTM_OK) {
                fprintf(stderr, "rtm_render_ex: %d (%s)\n", r, rtm_last_error());
                rc = 1;
            } else {
                rc |= write_ppm_rgb8(ppm_gpu, rgb, w, h) != 0;
            }
            free(rgb);
        }
    }
    if (raw) {
        FILE* f = fopen(raw, "wb");
        rc |= !f || fwrite(img, sizeof(float), (size_t)w * h * 4, f) != (size_t)w * h * 4;
        if (f) rc |= fclose(f) != 0;
    }
    if (ppm) rc |= write_ppm(ppm, img, w, h) != 0;
    free(img);
    return rc ? 1 : 0;
}
