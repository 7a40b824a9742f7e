/*
 * rt_host.h — C-ABI of librt_host.so, the host half of the drop-in (pure C++17, no GPU).
 *
 * It keeps the reference cpu/ renderer's scene loader, camera, BVH builder, random-triangle mode
 * and BMP output (BASELINE.json north_star: "keeps the cpu/ renderer's scene loader, camera and
 * command-line surface"). Every function names the reference interface it replaces. Buffers
 * returned through `out` pointers are malloc'd and released with rth_free().
 */
#ifndef RT_HOST_H
#define RT_HOST_H

#include <stddef.h>
#include <stdint.h>

#include "rt_types.h"

#ifdef __cplusplus
extern "C" {
#endif

/* ---- glibc random()/rand() restatement (TYPE_3 additive feedback, r[i] = r[i-3] + r[i-31]).
 * Replaces the reference's srand(SEED)/rand() (cpu/src/main.c:91-95, bvh.c:229-231,
 * main.c:121-123) with an explicit state so results do not depend on hidden libc state. */
typedef struct rth_rng {
    int32_t r[34];
    int pos;
} rth_rng;
void rth_srand(rth_rng* g, unsigned seed); /* srand(seed) */
int rth_rand(rth_rng* g);                  /* rand(): 0 .. RAND_MAX (2^31 - 1) */

/* ---- scene loading (text formats unchanged) */
/* triangles_load(objname, mtlname, &size)        cpu/src/triangle.c:74-126
 * OBJ: 'v x y z', 'f a b c' (1-based), 'usemtl'; MTL: Kd/Ks/Kr within 5 lines after 'newmtl';
 * lines are read as fgets(256) chunks; a material key absent from the MTL is 0. */
int rth_triangles_load(const char* obj, const char* mtl, rt_triangle** out, size_t* n);
/* lights_load(filename, &size)                   cpu/src/light.c:6-29 ('px py pz r g b' per line) */
int rth_lights_load(const char* path, rt_light** out, size_t* n);
/* triangle_init(t, a, b, c, ks, kd, kr)          cpu/src/triangle.c:6-24 */
void rth_triangle_init(rt_triangle* t, const rt_vec3* a, const rt_vec3* b, const rt_vec3* c,
                       const rt_vec3* ks, const rt_vec3* kd, const rt_vec3* kr);
/* random-triangle mode: `raytracer <threads> <ntris>`  cpu/src/main.c:115-131 (uses g) */
int rth_triangles_random(size_t n, rth_rng* g, rt_triangle** out);

/* ---- BVH build: bvh_build(triangles, n)          cpu/src/bvh.c:360-388
 * heuristic: 0 axis-0 centre, 1 largest-axis centre, 3 random axis/position (cpu default,
 *   options.h:34; consumes g), 6 32-bin SAH with the reference's FLT_MIN box seed (gpu default,
 *   options.cuh:50), RTH_BVH_BINNED_SAH: this library's O(n log n) binned SAH (surface-area cost,
 *   leaf <= 8, depth <= 24) for large meshes. Leaves: tr_len <= 2 or depth 32 (bvh.c:84). Output uses the
 *   reference's node layout; nodes has bvh_len entries. */
enum { RTH_BVH_BINNED_SAH = 16 };
typedef struct rth_bvh_stats {
    int leaves, min_leaf, max_leaf, max_depth;
    double avg_leaf; /* "avg number of triangle" (bvh.c:384) */
} rth_bvh_stats;
int rth_bvh_build(const rt_triangle* tris, size_t n, int heuristic, rth_rng* g, rt_bvh_node** nodes,
                  int* bvh_len, int** tri_idx, rth_bvh_stats* stats);

/* ---- binary scene cache (no reference counterpart). `cache` is a file path (NULL: no
 * cache). An entry is keyed by a 64-bit hash of everything the result depends on and checksummed; a
 * stale, foreign or damaged file is ignored and replaced, so the cached call returns exactly what the
 * uncached one would. *from_cache (nullable) = 1 when the result was read from the cache. */
/* triangles_load of an OBJ/MTL pair (key: both files' bytes) */
int rth_triangles_load_cached(const char* obj, const char* mtl, const char* cache, rt_triangle** out, size_t* n,
                              int* from_cache);
/* bvh_build (key: the triangles, heuristic and RNG state; the RNG is left as after the real build) */
int rth_bvh_build_cached(const rt_triangle* tris, size_t n, int heuristic, rth_rng* g, const char* cache,
                         rt_bvh_node** nodes, int* bvh_len, int** tri_idx, rth_bvh_stats* stats, int* from_cache);

/* ---- 8-wide quantised BVH: the fast walk's device layout (rt_device.hpp DWide), built
 * from any reference-layout binary BVH (bvh + tri_idx as rth_bvh_build returns them). Interior nodes
 * hold up to 8 children; child boxes are grown by `inflate` and quantised outward to 8 bits per
 * plane; leaves hold <= 4 triangles. Replaces no reference function: it is the acceleration structure
 * behind RT_ACCEL_AUTO. nodes: 20 x uint32 per node, root = node 0; tri_order: wide-leaf position
 * -> triangle index (a permutation of 0..n_tris-1). Buffers are released with rth_free(). */
typedef struct rth_wbvh_info {
    int n_nodes, n_tris, depth, max_children;
} rth_wbvh_info;
int rth_wbvh_build(const rt_bvh_node* bvh, int n_nodes, const int* tri_idx, const rt_triangle* tris, int n_tris,
                   float inflate, uint32_t** nodes, int** tri_order, rth_wbvh_info* info);
/* the same with the collapse's price of a wide-node visit in triangle tests (c_node <= 0: the default, 2) */
int rth_wbvh_build_cost(const rt_bvh_node* bvh, int n_nodes, const int* tri_idx, const rt_triangle* tris, int n_tris,
                        float inflate, float c_node, uint32_t** nodes, int** tri_order, rth_wbvh_info* info);

/* ---- camera: cam_init + cam.rot.x + cam_calculate_screen_coords + inc_x/inc_y
 * (cpu/src/cam.c:5-48, main.c:105-106, main.c:243-250) for a width x height frame:
 * pos (0,-9,3), fov pi/3.2, rot.x = -pi/12. */
int rth_camera(int width, int height, rt_camera* out);

/* ---- output: bmp_write_file(pixels, width, height, filename)   cpu/src/bmp_writer.c:177-211
 * rgb: height x width x 3 floats in [0,1], row 0 = top; 32-bpp BGRA, bottom-up, (uint8_t)(c*255). */
int rth_bmp_write(const float* rgb, int width, int height, const char* path);
/* the same conversion into a caller buffer of 54 + 4*width*height bytes */
int rth_bmp_encode(const float* rgb, int width, int height, uint8_t* out, size_t cap);
/* its 54-byte header alone (bmp_writer.c:97-120) */
int rth_bmp_header(int width, int height, uint8_t out[54]);

void rth_free(void* p);

#ifdef __cplusplus
}
#endif
#endif
