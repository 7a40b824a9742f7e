/*
 * oracle/ref_count_wrap.c — TEST INFRASTRUCTURE ONLY. Counts the reference's own traversal calls
 * by linker wrapping (-Wl,--wrap=bvh_traverse,--wrap=bvh_light_traverse), without touching its
 * sources: closest-hit rays = bvh_traverse calls (raytracer.c:113) minus the harness's one primary
 * probe per pixel; traced shadow rays = bvh_light_traverse calls (raytracer.c:74).
 * Printed to stderr at exit as "COUNTS trav=<n> light=<n>".
 */
#include <stdatomic.h>
#include <stdbool.h>
#include <stdio.h>

#include "bvh.h"

static atomic_ulong n_trav, n_light;
void __real_bvh_traverse(int, const vec_t*, const vec_t*, int*, float*, int*);
bool __real_bvh_light_traverse(int, const vec_t*, const vec_t*, float*, float);

void __wrap_bvh_traverse(int a, const vec_t* o, const vec_t* d, int* nd, float* t, int* ti) {
    atomic_fetch_add(&n_trav, 1);
    __real_bvh_traverse(a, o, d, nd, t, ti);
}
bool __wrap_bvh_light_traverse(int a, const vec_t* o, const vec_t* d, float* t, float l) {
    atomic_fetch_add(&n_light, 1);
    return __real_bvh_light_traverse(a, o, d, t, l);
}
__attribute__((destructor)) static void report(void) {
    fprintf(stderr, "COUNTS trav=%lu light=%lu\n", (unsigned long)n_trav, (unsigned long)n_light);
}
