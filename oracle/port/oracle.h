/*
 * oracle/port/oracle.h — TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement ("port") of the reference cpu/ renderer (deluf/parallel-ray-tracer @ 2025-10-31),
 * used by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg as the CHECKER.
 * It is never linked into, loaded by, or called from the product (librt_hip.so / librt_host.so).
 *
 * Pinned against the reference itself: tests/test_oracle.py compares it with oracle/_ref/rt_ref_strict
 * (the unmodified reference sources + ref_harness.c) through the committed fixtures in tests/golden/.
 * Built strict (-O2 -ffp-contract=off): SURVEY §8c "O-strict".
 */
#ifndef PRT_ORACLE_H
#define PRT_ORACLE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct orc_scene orc_scene;

enum {
    ORC_C_PRIMARY = 0,   /* primary rays (1 per pixel)                            */
    ORC_C_REFLECT,       /* traced reflection rays (iter 1..BOUNCES-1)             */
    ORC_C_SHADOW,        /* traced shadow rays (light_v calls past back-face test) */
    ORC_C_SHADOW_SKIP,   /* light_v early-outs, raytracer.c:66-67                  */
    ORC_C_CH_INNER,      /* closest-hit interior pops (2 box tests each)          */
    ORC_C_CH_LEAF,       /* closest-hit leaf pops                                  */
    ORC_C_CH_TRI,        /* closest-hit triangle tests                             */
    ORC_C_SH_INNER,      /* shadow interior pops                                   */
    ORC_C_SH_LEAF,       /* shadow leaf pops                                       */
    ORC_C_SH_TRI,        /* shadow triangle tests                                  */
    ORC_C_HITS,          /* closest-hit rays that hit                              */
    ORC_NCOUNTERS = 16
};

/* Scene creation seeds the C library generator with srand(seed) exactly where the reference's main()
 * does (cpu/src/main.c:91-95); random mode consumes rand() first, bvh build continues the sequence. */
orc_scene* orc_scene_load(const char* obj, const char* mtl, const char* lights, unsigned seed);
orc_scene* orc_scene_random(int ntris, unsigned seed);
void orc_scene_free(orc_scene* s);
int orc_scene_ntris(const orc_scene* s);
int orc_scene_nlights(const orc_scene* s);
/* triangle_t AoS (108 B each, cpu/include/triangle.h:8-16) and light_t (24 B) views */
const void* orc_scene_triangles(const orc_scene* s);
const void* orc_scene_lights(const orc_scene* s);

/* bvh.c:360-388; heuristic 3 (cpu default) or 6 (gpu default); returns bvh_len or <0 */
int orc_bvh_build(orc_scene* s, int heuristic);
/* copies bvh_t[bvh_len] (32 B each, cpu/include/bvh.h:14-23) and tri_idx[n] */
int orc_bvh_export(const orc_scene* s, void* nodes, int32_t* tri_idx);
/* disable the BVH (USE_BVH 0, raytracer.c:85-96,114-129): brute-force known-answer mode */
void orc_set_use_bvh(orc_scene* s, int use_bvh);
void orc_set_bounces(orc_scene* s, int bounces);

/* camera constants for a W x H frame: pos[3] ul[3] inc_x[3] inc_y[3] (main.c:105-106,243-250) */
void orc_camera(int W, int H, float out12[12]);

/* Render rows y = row_offset + k*row_stride, k < n_rows; outputs are full-frame arrays indexed y*W+x.
 * hit/t: primary closest hit (nullable); rgb: clamped colour [3N] (nullable);
 * bounce_hit: [4N] closest-hit triangle index per bounce, -1 miss, -2 not traced (nullable);
 * counters: ORC_NCOUNTERS uint64 (nullable). threads <= 0 -> 1. */
int orc_render(const orc_scene* s, int W, int H, int row_offset, int row_stride, int n_rows, int threads,
               int32_t* hit, float* t, float* rgb, int32_t* bounce_hit, uint64_t* counters);

/* spp > 1: stratified sub-pixel grid (car_boxed 64-spp config): sample (i,j) of an
 * s x s grid (s*s = spp) shoots from x + (i+0.5)/s, y + (j+0.5)/s; the pixel is the mean of the
 * clamped samples accumulated in sample order. spp = 1 is the reference's corner ray. */
int orc_render_spp(const orc_scene* s, int W, int H, int spp, int row_offset, int row_stride, int n_rows,
                   int threads, float* rgb, uint64_t* counters);

#ifdef __cplusplus
}
#endif
#endif
