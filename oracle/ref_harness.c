/*
 * oracle/ref_harness.c — TEST INFRASTRUCTURE ONLY (never shipped, never measured as the product).
 *
 * A harness `main` that links the UNMODIFIED reference sources
 *   /root/reference/cpu/src/{bvh,triangle,vec,raytracer,cam,light,bmp_writer}.c
 * compiled where they lie (recipe: oracle/Makefile; outputs only into oracle/_ref/).
 * It replaces the reference's cpu/src/main.c (which hard-wires WIDTH/HEIGHT/SCENE at compile time)
 * with a command-line driven front end that reproduces main.c's setup byte for byte:
 *   - srand(SEED=1) before anything else                      (cpu/src/main.c:91-95)
 *   - camera pos (0,-9,3), fov M_PI/3.2, rot.x = -M_PI/12      (cpu/src/main.c:105-106)
 *   - scene load or random-triangle mode                      (cpu/src/main.c:112-131)
 *   - bvh_build                                               (cpu/src/main.c:138)
 *   - per-thread screen coords + inc_x/inc_y                  (cpu/src/main.c:243-250)
 *   - render_pixel: dir = ((ul - pos) + inc_x*x) + inc_y*y     (cpu/src/main.c:228-239)
 *   - row tiles handed out by an atomic counter (TILE_SIZE = WIDTH) (cpu/src/main.c:252-261)
 *
 * Commands (all binary outputs little-endian):
 *   render <obj> <mtl> <lights> <W> <H> <threads> <out>
 *       out = int32 hit[N] | f32 t[N] | f32 rgb[3N]; hit/t = primary closest hit
 *       (bvh_traverse from the camera, exactly the first traversal raytrace() performs,
 *       cpu/src/raytracer.c:113), rgb = vec_constrain(raytrace(pos,dir,0)) (main.c:234-237).
 *   random <ntris> <W> <H> <threads> <out>        (random-triangle mode, main.c:115-131, lights_len=0)
 *   bvh <obj> <mtl> <out>                          out = int32 bvh_len | bvh_t[bvh_len] | int32 tri_idx[n]
 *   bvhrand <ntris> <out>                          same, for random mode
 *   bmp <obj> <mtl> <lights> <W> <H> <threads> <out.bmp>   bmp_write_file of the frame (bmp_writer.c:177)
 *   time <obj> <mtl> <lights> <W> <H> <threads> <row_offset> <row_stride> <reps>
 *       renders rows y = row_offset + k*row_stride (timing baseline), prints one JSON line with
 *       the median wall ms over <reps> frames; the BVH build is outside the timed region,
 *       as in main.c:169-185.
 */
#define _POSIX_C_SOURCE 199506L
#include <float.h>
#include <math.h>
#include <pthread.h>
#include <stdatomic.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "bmp_writer.h"
#include "bvh.h"
#include "cam.h"
#include "light.h"
#include "raytracer.h"
#include "triangle.h"
#include "vec.h"

#ifndef M_PI
#define M_PI 3.14159265358979323846
#endif

/* Globals the reference's main.c defines and raytracer.c / bvh.c reference (main.c:27-37). */
size_t triangles_len;
triangle_t* triangles;
size_t lights_len;
light_t* lights;
vec_t amb_light = {.r = 0.5, .g = 0.5, .b = 0.5};
cam_t cam;

extern bvh_t* bvh;
extern int* tri_idx;
extern int bvh_len;

static int W, H;
static int row_offset = 0, row_stride = 1, n_rows;
static atomic_int row_counter;
static int32_t* out_hit;
static float* out_t;
static vec_t* out_rgb;
static int want_primary = 1;

static void* thread_render(void* arg) {
    (void)arg;
    vec_t sp[3];
    cam_calculate_screen_coords(&cam, sp, (float)W / H); /* main.c:243 */
    vec_t ul = sp[0], ur = sp[1], dl = sp[2];
    vec_t inc_x = vec_sub(&ur, &ul);
    inc_x = vec_div(&inc_x, W);
    vec_t inc_y = vec_sub(&dl, &ul);
    inc_y = vec_div(&inc_y, H);
    for (;;) {
        int k = atomic_fetch_add(&row_counter, 1);
        if (k >= n_rows) break;
        int y = row_offset + k * row_stride;
        for (int x = 0; x < W; x++) {
            size_t idx = (size_t)y * W + x;
            /* render_pixel, main.c:228-239 */
            vec_t dir = vec_sub(&ul, &cam.pos);
            vec_t pos_x = vec_mul(&inc_x, x);
            vec_t pos_y = vec_mul(&inc_y, y);
            dir = vec_add(&dir, &pos_x);
            dir = vec_add(&dir, &pos_y);
            if (want_primary) {
                int nd = 0, ti = -1;
                float t = FLT_MAX;
                bvh_traverse(0, &cam.pos, &dir, &nd, &t, &ti);
                out_hit[idx] = ti;
                out_t[idx] = t;
            }
            vec_t col = raytrace(cam.pos, dir, 0);
            const vec_t v0 = {0, 0, 0};
            const vec_t v1 = {1, 1, 1};
            vec_constrain(&col, &v0, &v1);
            out_rgb[idx] = col;
        }
    }
    return NULL;
}

static void render_rows(int nthreads) {
    pthread_t th[256];
    if (nthreads < 1) nthreads = 1;
    if (nthreads > 256) nthreads = 256;
    atomic_store(&row_counter, 0);
    for (int i = 0; i < nthreads; i++) pthread_create(&th[i], NULL, thread_render, NULL);
    for (int i = 0; i < nthreads; i++) pthread_join(th[i], NULL);
}

static void setup_camera(void) {
    cam_init(&cam, &(vec_t){0, -9, 3}, M_PI / 3.2); /* main.c:105 */
    cam.rot.x = -M_PI / 12;                          /* main.c:106 */
}

static void load_scene(const char* obj, const char* mtl, const char* lts) {
    triangles = triangles_load(obj, mtl, &triangles_len);
    if (lts) lights = lights_load(lts, &lights_len);
    else lights_len = 0;
}

static void random_scene(int n) { /* main.c:116-130 */
    triangles_len = n;
    triangles = (triangle_t*)malloc(sizeof(triangle_t) * triangles_len);
    for (int i = 0; i < n; i++) {
        vec_t vec0 = {0.0f, 0.0f, 0.0f};
        vec_t vec1 = {1.0f, 1.0f, 1.0f};
        vec_t r0 = {(float)rand() / RAND_MAX, (float)rand() / RAND_MAX, (float)rand() / RAND_MAX};
        vec_t r1 = {(float)rand() / RAND_MAX, (float)rand() / RAND_MAX, (float)rand() / RAND_MAX};
        vec_t r2 = {(float)rand() / RAND_MAX, (float)rand() / RAND_MAX, (float)rand() / RAND_MAX};
        vec_t a = vec_mul(&r0, 10);
        a.x -= 5; a.y -= 5; a.z -= 5;
        vec_t b = vec_add(&a, &r1);
        vec_t c = vec_add(&b, &r2);
        triangle_init(&triangles[i], &a, &b, &c, &vec1, &vec0, &vec0);
    }
    lights_len = 0;
}

static void write_frame(const char* path) {
    size_t N = (size_t)W * H;
    FILE* f = fopen(path, "wb");
    if (!f) { perror(path); exit(2); }
    fwrite(out_hit, sizeof(int32_t), N, f);
    fwrite(out_t, sizeof(float), N, f);
    for (size_t i = 0; i < N; i++) fwrite(out_rgb[i].arr, sizeof(float), 3, f);
    fclose(f);
}

static void write_bvh(const char* path) {
    FILE* f = fopen(path, "wb");
    if (!f) { perror(path); exit(2); }
    int32_t len = bvh_len;
    fwrite(&len, 4, 1, f);
    fwrite(bvh, sizeof(bvh_t), (size_t)bvh_len, f);
    fwrite(tri_idx, sizeof(int), triangles_len, f);
    fclose(f);
}

static void alloc_frame(void) {
    size_t N = (size_t)W * H;
    out_hit = (int32_t*)calloc(N, sizeof(int32_t));
    out_t = (float*)calloc(N, sizeof(float));
    out_rgb = (vec_t*)calloc(N, sizeof(vec_t));
    if (!out_hit || !out_t || !out_rgb) { fprintf(stderr, "oom\n"); exit(2); }
}

static double now_ms(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec * 1e3 + ts.tv_nsec / 1e6;
}

static int cmp_d(const void* a, const void* b) {
    double d = *(const double*)a - *(const double*)b;
    return (d > 0) - (d < 0);
}

int main(int argc, char** argv) {
    srand(1); /* SEED 1, main.c:94 */
    setup_camera();
    if (argc < 2) { fprintf(stderr, "usage: see header\n"); return 2; }
    const char* cmd = argv[1];
    if (!strcmp(cmd, "render") || !strcmp(cmd, "bmp")) {
        if (argc != 9) { fprintf(stderr, "%s <obj> <mtl> <lights> <W> <H> <threads> <out>\n", cmd); return 2; }
        load_scene(argv[2], argv[3], argv[4]);
        W = atoi(argv[5]); H = atoi(argv[6]);
        bvh_build(triangles, triangles_len);
        alloc_frame();
        n_rows = H;
        render_rows(atoi(argv[7]));
        if (!strcmp(cmd, "render")) write_frame(argv[8]);
        else return bmp_write_file(out_rgb, W, H, argv[8]) ? 1 : 0;
        return 0;
    }
    if (!strcmp(cmd, "random")) {
        if (argc != 7) { fprintf(stderr, "random <ntris> <W> <H> <threads> <out>\n"); return 2; }
        random_scene(atoi(argv[2]));
        W = atoi(argv[3]); H = atoi(argv[4]);
        bvh_build(triangles, triangles_len);
        alloc_frame();
        n_rows = H;
        render_rows(atoi(argv[5]));
        write_frame(argv[6]);
        return 0;
    }
    if (!strcmp(cmd, "bvh")) {
        if (argc != 5) { fprintf(stderr, "bvh <obj> <mtl> <out>\n"); return 2; }
        load_scene(argv[2], argv[3], NULL);
        bvh_build(triangles, triangles_len);
        write_bvh(argv[4]);
        return 0;
    }
    if (!strcmp(cmd, "bvhrand")) {
        if (argc != 4) { fprintf(stderr, "bvhrand <ntris> <out>\n"); return 2; }
        random_scene(atoi(argv[2]));
        bvh_build(triangles, triangles_len);
        write_bvh(argv[3]);
        return 0;
    }
    if (!strcmp(cmd, "time")) {
        if (argc != 11) {
            fprintf(stderr, "time <obj|random:N> <mtl> <lights> <W> <H> <threads> <row_offset> <row_stride> <reps>\n");
            return 2;
        }
        if (!strncmp(argv[2], "random:", 7)) random_scene(atoi(argv[2] + 7)); /* random mode, main.c:115-131 */
        else load_scene(argv[2], argv[3], argv[4]);
        W = atoi(argv[5]); H = atoi(argv[6]);
        int threads = atoi(argv[7]);
        row_offset = atoi(argv[8]);
        row_stride = atoi(argv[9]);
        int reps = atoi(argv[10]);
        if (row_stride < 1) row_stride = 1;
        if (reps < 1) reps = 1;
        if (reps > 64) reps = 64;
        n_rows = (H - row_offset + row_stride - 1) / row_stride;
        double t0 = now_ms();
        bvh_build(triangles, triangles_len);
        double bvh_ms = now_ms() - t0;
        alloc_frame();
        want_primary = 0;
        double times[64];
        for (int r = 0; r < reps; r++) {
            double s = now_ms();
            render_rows(threads);
            times[r] = now_ms() - s;
        }
        qsort(times, reps, sizeof(double), cmp_d);
        double med = reps % 2 ? times[reps / 2] : 0.5 * (times[reps / 2 - 1] + times[reps / 2]);
        printf("{\"median_ms\": %.4f, \"min_ms\": %.4f, \"bvh_ms\": %.4f, \"rows\": %d, \"threads\": %d, \"reps\": %d}\n",
               med, times[0], bvh_ms, n_rows, threads, reps);
        return 0;
    }
    fprintf(stderr, "unknown command %s\n", cmd);
    return 2;
}
