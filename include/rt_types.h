/*
 * rt_types.h — plain-old-data types shared by the host library (rt_host.h) and the HIP device
 * layer (rt_hip.h). Each struct is layout-identical to the reference's own type, so buffers the
 * reference's C code produces can be handed over unchanged (and vice versa):
 *
 *   rt_vec3      == vec_t       cpu/include/vec.h:4-18        (12 B)
 *   rt_triangle  == triangle_t  cpu/include/triangle.h:8-16   (108 B: coords, centroid, ks, kd, kr, norm[2])
 *   rt_light     == light_t     cpu/include/light.h:8-11      (24 B)
 *   rt_bvh_node  == bvh_t       cpu/include/bvh.h:9-23        (32 B; child doubles as tr_idx when tr_len > 0)
 */
#ifndef RT_TYPES_H
#define RT_TYPES_H

#ifdef __cplusplus
extern "C" {
#endif

typedef struct rt_vec3 {
    float x, y, z;
} rt_vec3;

typedef struct rt_triangle {
    rt_vec3 coords[3];
    float centroid[3];
    rt_vec3 ks;
    rt_vec3 kd;
    rt_vec3 kr;
    rt_vec3 norm[2];
} rt_triangle;

typedef struct rt_light {
    rt_vec3 pos;
    rt_vec3 kl;
} rt_light;

typedef struct rt_bvh_node {
    rt_vec3 min;
    rt_vec3 max;
    int tr_len; /* > 0: leaf with tr_len triangles starting at tri_idx[child] */
    int child;  /* interior: children at child, child + 1; child == 0 && tr_len == 0: empty */
} rt_bvh_node;

/* Camera constants of one frame (cpu/src/main.c:243-250): a pixel (x, y) shoots
 * dir = ((ul - pos) + inc_x * x) + inc_y * y from pos (main.c:228-233), unnormalised. */
typedef struct rt_camera {
    rt_vec3 pos;
    rt_vec3 ul;
    rt_vec3 inc_x;
    rt_vec3 inc_y;
} rt_camera;

/* status codes returned by every rt_* / rth_* call (0 = ok) */
enum {
    RT_OK = 0,
    RT_E_ARG = -1,      /* invalid argument */
    RT_E_IO = -2,       /* file cannot be opened / written */
    RT_E_NOMEM = -3,    /* host allocation failed */
    RT_E_HIP = -4,      /* HIP runtime error (see rt_last_error) */
    RT_E_STATE = -5,    /* call out of order (e.g. render before upload) */
    RT_E_NODEVICE = -6, /* no GPU visible */
    RT_E_EMPTY = -7,    /* no triangles: "no triangles, cannot build bvh." (bvh.c:361-364) */
    RT_E_KERNEL = -8,   /* a kernel reported an error: a traversal stack overflowed (the frame is not trustworthy) */
    RT_E_TIMEOUT = -9   /* a collective did not complete within its deadline (the communicator is aborted) */
};

#ifdef __cplusplus
}
#endif
#endif
