/*
 * oracle/port/oracle.c — TEST INFRASTRUCTURE ONLY: the CPU restatement ("port") of the reference
 * cpu/ renderer. Every function cites the reference file:line it restates. It is the checker for
 * the HIP path (tests/, __graft_entry__.smoke(), bench.py cpu_baseline) and is never part of the
 * product. Compile strict (-O2 -ffp-contract=off) for parity: each float expression below keeps
 * the reference's operand order so that the roundings are identical.
 *
 * Pinned: tests/test_oracle.py checks it bit-for-bit against oracle/_ref/rt_ref_strict (the
 * reference's own sources) via the fixtures in tests/golden/ (made by tests/golden/make_golden.py).
 */
#define _GNU_SOURCE
#include "oracle.h"

#include <float.h>
#include <math.h>
#include <pthread.h>
#include <stdatomic.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

/* ---------------------------------------------------------------- vec (cpu/src/vec.c) */
typedef struct { float x, y, z; } v3;

static inline float dot3(v3 a, v3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }   /* vec.c:4-6 */
static inline float mag3(v3 a) { return sqrtf(a.x * a.x + a.y * a.y + a.z * a.z); } /* vec.c:15-17 */
static inline v3 mul3(v3 a, float s) { return (v3){a.x * s, a.y * s, a.z * s}; }    /* vec.c:23-25 */
static inline v3 add3(v3 a, v3 b) { return (v3){a.x + b.x, a.y + b.y, a.z + b.z}; } /* vec.c:27-29 */
static inline v3 sub3(v3 a, v3 b) { return (v3){a.x - b.x, a.y - b.y, a.z - b.z}; } /* vec.c:31-33 */
static inline v3 div3(v3 a, float s) { return (v3){a.x / s, a.y / s, a.z / s}; }    /* vec.c:35-37 */
static inline v3 cross3(v3 a, v3 b) {                                               /* vec.c:39-45 */
    return (v3){a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x};
}
static inline v3 norm3(v3 a) { return div3(a, mag3(a)); }                           /* vec.c:19-21 */
static inline v3 vmin3(v3 a, v3 b) { return (v3){fminf(a.x, b.x), fminf(a.y, b.y), fminf(a.z, b.z)}; }
static inline v3 vmax3(v3 a, v3 b) { return (v3){fmaxf(a.x, b.x), fmaxf(a.y, b.y), fmaxf(a.z, b.z)}; }
static inline float comp(v3 a, int i) { return i == 0 ? a.x : (i == 1 ? a.y : a.z); }

/* ---------------------------------------------------------------- data model */
typedef struct {            /* cpu/include/triangle.h:8-16 (108 bytes) */
    v3 coords[3];
    float centroid[3];
    v3 ks, kd, kr;
    v3 norm[2];
} tri_t;
typedef struct { v3 pos, kl; } light_t;            /* cpu/include/light.h:8-11 */
typedef struct { v3 min, max; int tr_len; int idx; } node_t; /* cpu/include/bvh.h:9-23; idx = tr_idx | child */

struct orc_scene {
    tri_t* tris;
    int n;
    light_t* lights;
    int nl;
    node_t* bvh;
    int bvh_len;
    int* tri_idx;
    int use_bvh;
    int bounces;
};

static const float EPS = 1e-3f;          /* raytracer.c:19 */
static const v3 AMB = {0.5f, 0.5f, 0.5f}; /* main.c:37 */

/* triangle.c:6-24 */
static void tri_init(tri_t* t, v3 a, v3 b, v3 c, v3 ks, v3 kd, v3 kr) {
    t->coords[0] = a; t->coords[1] = b; t->coords[2] = c;
    t->ks = ks; t->kd = kd; t->kr = kr;
    v3 e1 = sub3(b, a), e2 = sub3(c, a);
    t->norm[0] = norm3(cross3(e1, e2));
    t->norm[1] = norm3(cross3(e2, e1));
    t->centroid[0] = (a.x + b.x + c.x) / 3.0f;
    t->centroid[1] = (a.y + b.y + c.y) / 3.0f;
    t->centroid[2] = (a.z + b.z + c.z) / 3.0f;
}

/* ---------------------------------------------------------------- loaders (triangle.c:26-126, light.c:6-29) */
/* fgets(buf, 256) chunking, triangle.c:34-42: a physical line longer than 255 chars becomes several. */
static char** read_chunks(const char* path, int* count) {
    FILE* f = fopen(path, "r");
    if (!f) return NULL;
    char** lines = NULL;
    int n = 0, cap = 0;
    char buf[256];
    while (fgets(buf, sizeof buf, f)) {
        if (n == cap) {
            cap = cap ? cap * 2 : 1024;
            lines = (char**)realloc(lines, sizeof(char*) * cap);
        }
        lines[n++] = strdup(buf);
    }
    fclose(f);
    *count = n;
    if (!lines) lines = (char**)malloc(sizeof(char*));
    return lines;
}

typedef struct { char name[256]; v3 kd, ks, kr; } mat_t;

orc_scene* orc_scene_load(const char* obj, const char* mtl, const char* lights, unsigned seed) {
    srand(seed);
    int no = 0, nm = 0;
    char** ol = read_chunks(obj, &no);
    if (!ol) return NULL;
    char** ml = read_chunks(mtl, &nm);
    if (!ml) return NULL;
    v3* verts = (v3*)calloc(no + 1, sizeof(v3));
    int nv = 0;
    for (int i = 0; i < no; i++)                                   /* triangle.c:82-87 */
        if (ol[i][0] == 'v' && ol[i][1] == ' ') {
            sscanf(ol[i], "v %f %f %f", &verts[nv].x, &verts[nv].y, &verts[nv].z);
            nv++;
        }
    mat_t* mats = (mat_t*)calloc(128, sizeof(mat_t));             /* triangle.c:89; unset keys = 0 */
    int nmat = 0;
    for (int i = 0; i < nm; i++) {                                 /* triangle.c:54-72 */
        if (strncmp(ml[i], "newmtl", 6) == 0 && nmat < 128) {
            sscanf(ml[i], "newmtl %255s", mats[nmat].name);
            for (int j = i + 1; j < i + 6 && j < nm; j++) {
                if (strncmp(ml[j], "Kd", 2) == 0)
                    sscanf(ml[j], "Kd %f %f %f", &mats[nmat].kd.x, &mats[nmat].kd.y, &mats[nmat].kd.z);
                else if (strncmp(ml[j], "Ks", 2) == 0)
                    sscanf(ml[j], "Ks %f %f %f", &mats[nmat].ks.x, &mats[nmat].ks.y, &mats[nmat].ks.z);
                else if (strncmp(ml[j], "Kr", 2) == 0)
                    sscanf(ml[j], "Kr %f %f %f", &mats[nmat].kr.x, &mats[nmat].kr.y, &mats[nmat].kr.z);
            }
            nmat++;
        }
    }
    orc_scene* s = (orc_scene*)calloc(1, sizeof(orc_scene));
    s->tris = (tri_t*)malloc(sizeof(tri_t) * (no + 1));
    v3 cks = {0, 0, 0}, ckd = {0, 0, 0}, ckr = {0, 0, 0};          /* triangle.c:92 */
    int nt = 0;
    for (int i = 0; i < no; i++) {                                 /* triangle.c:96-115 */
        if (strncmp(ol[i], "usemtl", 6) == 0) {
            char name[256] = {0};
            sscanf(ol[i], "usemtl %255s", name);
            for (int m = 0; m < nmat; m++)
                if (strcmp(name, mats[m].name) == 0) {
                    ckd = mats[m].kd; cks = mats[m].ks; ckr = mats[m].kr;
                    break;
                }
        } else if (ol[i][0] == 'f') {
            int a = 0, b = 0, c = 0;
            sscanf(ol[i], "f %d %d %d", &a, &b, &c);
            tri_init(&s->tris[nt], verts[a - 1], verts[b - 1], verts[c - 1], cks, ckd, ckr);
            nt++;
        }
    }
    s->n = nt;
    for (int i = 0; i < no; i++) free(ol[i]);
    for (int i = 0; i < nm; i++) free(ml[i]);
    free(ol); free(ml); free(verts); free(mats);
    s->use_bvh = 1;
    s->bounces = 4;
    if (lights) {                                                  /* light.c:6-29 */
        FILE* f = fopen(lights, "r");
        if (!f) { orc_scene_free(s); return NULL; }
        char line[256];
        s->lights = (light_t*)malloc(sizeof(light_t));
        while (fgets(line, sizeof line, f)) {
            light_t l;
            memset(&l, 0, sizeof l);
            sscanf(line, "%f %f %f %f %f %f", &l.pos.x, &l.pos.y, &l.pos.z, &l.kl.x, &l.kl.y, &l.kl.z);
            s->lights = (light_t*)realloc(s->lights, sizeof(light_t) * (s->nl + 1));
            s->lights[s->nl++] = l;
        }
        fclose(f);
    }
    return s;
}

/* main.c:115-131 */
orc_scene* orc_scene_random(int ntris, unsigned seed) {
    srand(seed);
    orc_scene* s = (orc_scene*)calloc(1, sizeof(orc_scene));
    s->tris = (tri_t*)malloc(sizeof(tri_t) * (ntris > 0 ? ntris : 1));
    s->n = ntris;
    for (int i = 0; i < ntris; i++) {
        v3 v0 = {0.0f, 0.0f, 0.0f}, v1 = {1.0f, 1.0f, 1.0f};
        /* C evaluates each initializer in order; draws are sequenced x, y, z */
        float r[9];
        for (int k = 0; k < 9; k++) r[k] = (float)rand() / RAND_MAX;
        v3 r0 = {r[0], r[1], r[2]}, r1 = {r[3], r[4], r[5]}, r2 = {r[6], r[7], r[8]};
        v3 a = mul3(r0, 10);
        a.x -= 5; a.y -= 5; a.z -= 5;
        v3 b = add3(a, r1);
        v3 c = add3(b, r2);
        tri_init(&s->tris[i], a, b, c, v1, v0, v0);
    }
    s->use_bvh = 1;
    s->bounces = 4;
    return s;
}

void orc_scene_free(orc_scene* s) {
    if (!s) return;
    free(s->tris); free(s->lights); free(s->bvh); free(s->tri_idx);
    free(s);
}
int orc_scene_ntris(const orc_scene* s) { return s->n; }
int orc_scene_nlights(const orc_scene* s) { return s->nl; }
const void* orc_scene_triangles(const orc_scene* s) { return s->tris; }
const void* orc_scene_lights(const orc_scene* s) { return s->lights; }
void orc_set_use_bvh(orc_scene* s, int u) { s->use_bvh = u; }
void orc_set_bounces(orc_scene* s, int b) { s->bounces = b; }

/* ---------------------------------------------------------------- BVH build (bvh.c:38-267,360-388) */
static v3 box_center(v3 mn, v3 mx) { return mul3(add3(mn, mx), 0.5f); }           /* bvh.c:38-41 */
static float box_area(v3 mn, v3 mx) { v3 s = sub3(mx, mn); return dot3(s, s); }  /* bvh.c:43-46 */
static void grow_tri(const orc_scene* s, v3* mn, v3* mx, int t) {                  /* bvh.c:61-71 */
    for (int k = 0; k < 3; k++) {
        *mn = vmin3(*mn, s->tris[t].coords[k]);
        *mx = vmax3(*mx, s->tris[t].coords[k]);
    }
}

static void split(orc_scene* s, int heuristic, int ni, int depth) {
    node_t* p = &s->bvh[ni];
    if (s->bvh_len >= 2 * s->n) return;                            /* bvh.c:80-83 */
    if (depth == 32 || p->tr_len <= 2) {                           /* bvh.c:84-96 */
        if (!p->tr_len) p->idx = 0;
        return;
    }
    int ci = s->bvh_len;
    s->bvh_len += 2;
    node_t* L = &s->bvh[ci];
    node_t* R = &s->bvh[ci + 1];
    L->idx = p->idx; L->min = (v3){1e10f, 1e10f, 1e10f}; L->max = (v3){-1e10f, -1e10f, -1e10f};
    R->idx = p->idx; R->min = (v3){1e10f, 1e10f, 1e10f}; R->max = (v3){-1e10f, -1e10f, -1e10f};
    int axis = 0;
    float pos = 0;
    v3 center = box_center(p->min, p->max);
    v3 size = sub3(p->max, p->min);
    if (heuristic == 6) {                                          /* bvh.c:138-177, SAH_BIN_SIZE 32 */
        float best = FLT_MAX;
        for (int a = 0; a < 3; a++) {
            for (int i = 0; i < 32; i++) {
                v3 lmn = {FLT_MAX, FLT_MAX, FLT_MAX}, lmx = {FLT_MIN, FLT_MIN, FLT_MIN};
                v3 rmn = lmn, rmx = lmx;
                float sp = comp(p->min, a) + comp(size, a) * ((float)i / 32);
                int cl = 0, cr = 0;
                for (int j = p->idx; j < p->idx + p->tr_len; j++) {
                    int t = s->tri_idx[j];
                    if (s->tris[t].centroid[a] < sp) { grow_tri(s, &lmn, &lmx, t); cl++; }
                    else { grow_tri(s, &rmn, &rmx, t); cr++; }
                }
                float score = cl * box_area(lmn, lmx) + cr * box_area(rmn, rmx);
                if (score < best) { best = score; axis = a; pos = sp; }
            }
        }
    } else if (heuristic == 3) {                                   /* bvh.c:228-241 */
        int okA = 0, okB = 0;
        while (!okA || !okB) {
            okA = okB = 0;
            axis = rand() % 4;
            if (axis == 3) {
                /* rand() % 4 == 3 reads center.arr[3], size.arr[3] and centroid[3] past their arrays
                 * (bvh.c:229-231,237,247). O-strict (gcc -O2) keeps `size` right after
                 * `center` on the stack and the vec_add(min, max) temporary right after `size`, so it
                 * reads center.arr[3] = size.x and size.arr[3] = (min + max).x; centroid[3] is ks.r by
                 * the triangle_t layout. Pinned by the reference's own BVH dumps (tests/golden). */
                pos = size.x;
                pos += ((float)rand() / RAND_MAX - 0.5f) * (p->min.x + p->max.x);
            } else {
                pos = comp(center, axis);
                pos += ((float)rand() / RAND_MAX - 0.5f) * (comp(size, axis));
            }
            for (int i = p->idx; i < p->idx + p->tr_len && (!okA || !okB); i++) {
                const tri_t* t = &s->tris[s->tri_idx[i]];
                int inA = (axis == 3 ? t->ks.x : t->centroid[axis]) < pos;
                okA |= inA;
                okB |= !inA;
            }
        }
    } else {
        /* heuristic 0 (axis 0 centre) / 1 (largest axis centre), bvh.c:214-223 */
        axis = 0;
        if (heuristic == 1) {
            if (size.y > size.x) axis = 1;
            if (size.z > size.x && size.z > size.y) axis = 2;
        }
        pos = comp(center, axis);
    }
    for (int i = p->idx; i < p->idx + p->tr_len; i++) {           /* bvh.c:244-259 */
        int t = s->tri_idx[i];
        int inA = (axis == 3 ? s->tris[t].ks.x : s->tris[t].centroid[axis]) < pos;
        node_t* c = inA ? L : R;
        grow_tri(s, &c->min, &c->max, t);
        c->tr_len += 1;
        if (inA) {
            int sw = L->idx + L->tr_len - 1;
            int tmp = s->tri_idx[i];
            s->tri_idx[i] = s->tri_idx[sw];
            s->tri_idx[sw] = tmp;
            R->idx += 1;
        }
    }
    p->idx = ci;                                                   /* bvh.c:262-266 */
    p->tr_len = 0;
    split(s, heuristic, ci, depth + 1);
    split(s, heuristic, ci + 1, depth + 1);
}

int orc_bvh_build(orc_scene* s, int heuristic) {                   /* bvh.c:360-388 */
    if (!s || s->n <= 0) return -1;
    if (heuristic != 0 && heuristic != 1 && heuristic != 3 && heuristic != 6) return -2;
    free(s->bvh); free(s->tri_idx);
    s->tri_idx = (int*)malloc(sizeof(int) * s->n);
    for (int i = 0; i < s->n; i++) s->tri_idx[i] = i;
    s->bvh = (node_t*)calloc((size_t)2 * s->n, sizeof(node_t));
    s->bvh_len = 1;
    s->bvh[0].tr_len = s->n;
    s->bvh[0].min = (v3){1e10f, 1e10f, 1e10f};
    s->bvh[0].max = (v3){-1e10f, -1e10f, -1e10f};
    for (int i = 0; i < s->n; i++) grow_tri(s, &s->bvh[0].min, &s->bvh[0].max, i);
    split(s, heuristic, 0, 0);
    return s->bvh_len;
}

int orc_bvh_export(const orc_scene* s, void* nodes, int32_t* tri_idx) {
    if (!s->bvh) return -1;
    if (nodes) memcpy(nodes, s->bvh, sizeof(node_t) * s->bvh_len);
    if (tri_idx) memcpy(tri_idx, s->tri_idx, sizeof(int) * s->n);
    return s->bvh_len;
}

/* ---------------------------------------------------------------- hot path */
typedef struct { uint64_t c[ORC_NCOUNTERS]; } ctr_t;

/* raytracer.c:35-59 */
static float hit_tri(v3 o, v3 d, const tri_t* tr, int* nd) {
    v3 e1 = sub3(tr->coords[1], tr->coords[0]);
    v3 e2 = sub3(tr->coords[2], tr->coords[0]);
    v3 n = cross3(e1, e2);
    float det = -dot3(d, n);
    *nd = det < 0.0f;
    if (fabsf(det) < EPS) return FLT_MAX;
    float inv = 1.0f / det;
    v3 ao = sub3(o, tr->coords[0]);
    v3 dao = cross3(ao, d);
    float u = dot3(e2, dao) * inv;
    float v = -dot3(e1, dao) * inv;
    float t = dot3(ao, n) * inv;
    if (t > EPS && u >= 0.0f && v >= 0.0f && (u + v) <= 1.0f) return t;
    return FLT_MAX;
}

/* bvh.c:48-59 */
static float box_hit(v3 mn, v3 mx, v3 o, v3 d) {
    float tx1 = (mn.x - o.x) / d.x, tx2 = (mx.x - o.x) / d.x;
    float tmin = fminf(tx1, tx2), tmax = fmaxf(tx1, tx2);
    float ty1 = (mn.y - o.y) / d.y, ty2 = (mx.y - o.y) / d.y;
    tmin = fmaxf(tmin, fminf(ty1, ty2)), tmax = fminf(tmax, fmaxf(ty1, ty2));
    float tz1 = (mn.z - o.z) / d.z, tz2 = (mx.z - o.z) / d.z;
    tmin = fmaxf(tmin, fminf(tz1, tz2)), tmax = fminf(tmax, fmaxf(tz1, tz2));
    if (tmax >= tmin && tmax > 0) return tmin;
    return FLT_MAX;
}

/* bvh.c:317-358 */
static void traverse(const orc_scene* s, v3 o, v3 d, int* nd, float* t, int* ti, ctr_t* c) {
    int stack[64], sp = 0;
    stack[sp++] = 0;
    while (sp) {
        const node_t* node = &s->bvh[stack[--sp]];
        if (node->tr_len) {
            c->c[ORC_C_CH_LEAF]++;
            for (int i = node->idx; i < node->idx + node->tr_len; i++) {
                int k, idx = s->tri_idx[i];
                c->c[ORC_C_CH_TRI]++;
                float tt = hit_tri(o, d, &s->tris[idx], &k);
                if (tt < *t) { *t = tt; *nd = k; *ti = idx; }
            }
        } else if (node->idx) {
            c->c[ORC_C_CH_INNER]++;
            int ni = node->idx, fi = node->idx + 1;
            float nt = box_hit(s->bvh[ni].min, s->bvh[ni].max, o, d);
            float ft = box_hit(s->bvh[fi].min, s->bvh[fi].max, o, d);
            if (ft < nt) { int ti2 = ni; float tt = nt; ni = fi; nt = ft; fi = ti2; ft = tt; }
            if (ft < *t) stack[sp++] = fi;
            if (nt < *t) stack[sp++] = ni;
        }
    }
}

/* bvh.c:269-315 */
static int light_traverse(const orc_scene* s, v3 o, v3 d, float* t, float ld2, ctr_t* c) {
    int stack[64], sp = 0;
    stack[sp++] = 0;
    while (sp) {
        const node_t* node = &s->bvh[stack[--sp]];
        if (node->tr_len) {
            c->c[ORC_C_SH_LEAF]++;
            for (int i = node->idx; i < node->idx + node->tr_len; i++) {
                int k, idx = s->tri_idx[i];
                c->c[ORC_C_SH_TRI]++;
                float tt = hit_tri(o, d, &s->tris[idx], &k);
                if (tt < *t) {
                    *t = tt;
                    v3 ip = add3(o, mul3(d, *t));
                    v3 oi = sub3(o, ip);
                    if (ld2 > dot3(oi, oi)) return 0;
                }
            }
        } else if (node->idx) {
            c->c[ORC_C_SH_INNER]++;
            int ni = node->idx, fi = node->idx + 1;
            float nt = box_hit(s->bvh[ni].min, s->bvh[ni].max, o, d);
            float ft = box_hit(s->bvh[fi].min, s->bvh[fi].max, o, d);
            if (ft < nt) { int ti2 = ni; float tt = nt; ni = fi; nt = ft; fi = ti2; ft = tt; }
            if (ft < *t) stack[sp++] = fi;
            if (nt < *t) stack[sp++] = ni;
        }
    }
    return 1;
}

/* brute force closest hit, raytracer.c:114-129 */
static void brute_closest(const orc_scene* s, v3 o, v3 d, int* nd, float* t, int* ti, ctr_t* c) {
    float dist = FLT_MAX;
    for (int i = 0; i < s->n; i++) {
        int k;
        c->c[ORC_C_CH_TRI]++;
        float tt = hit_tri(o, d, &s->tris[i], &k);
        if (tt > EPS) {
            v3 ip = add3(o, mul3(d, tt));
            v3 df = sub3(o, ip);
            float dd = sqrtf(df.x * df.x + df.y * df.y + df.z * df.z);  /* vec_dist, vec.c:8-13 */
            if (dd < dist) { *ti = i; dist = dd; *t = tt; *nd = k; }
        }
    }
}

/* raytracer.c:62-99 */
static int light_v(const orc_scene* s, v3 o, v3 d, v3 n, v3 L, ctr_t* c) {
    v3 tmp = sub3(o, L), tmp2 = sub3(L, o);
    float ld2 = dot3(tmp, tmp);
    if (dot3(tmp2, n) < 0) { c->c[ORC_C_SHADOW_SKIP]++; return 0; }
    c->c[ORC_C_SHADOW]++;
    float t = FLT_MAX;
    if (s->use_bvh) return light_traverse(s, o, d, &t, ld2, c);
    for (int i = 0; i < s->n; i++) {                               /* raytracer.c:86-96 */
        int k;
        c->c[ORC_C_SH_TRI]++;
        float tt = hit_tri(o, d, &s->tris[i], &k);
        if (tt > EPS) {
            v3 ip = add3(o, mul3(d, tt));
            v3 oi = sub3(o, ip);
            if (ld2 > dot3(oi, oi)) return 0;
        }
    }
    return 1;
}

/* raytracer.c:21-33 */
static v3 lambert_blinn(v3 ks, v3 kd, v3 n, v3 l, v3 v, float dt) {
    v3 h = norm3(add3(l, v));
    float coeff = (float)fmax(0, dot3(n, h));
    v3 out;
    out.x = kd.x * fmaxf(0, dt) + ks.x * coeff;
    out.y = kd.y * fmaxf(0, dt) + ks.y * coeff;
    out.z = kd.z * fmaxf(0, dt) + ks.z * coeff;
    return out;
}

/* raytracer.c:101-177 */
static v3 raytrace(const orc_scene* s, v3 o, v3 d, int iter, ctr_t* c, int32_t* bh) {
    v3 col = {0, 0, 0};
    if (iter == s->bounces) return col;
    if (iter == 0) c->c[ORC_C_PRIMARY]++;
    else c->c[ORC_C_REFLECT]++;
    int index = -1, nd = 0;
    float t = FLT_MAX;
    if (s->use_bvh) traverse(s, o, d, &nd, &t, &index, c);
    else brute_closest(s, o, d, &nd, &t, &index, c);
    if (bh && iter < 4) bh[iter] = index;
    if (index == -1) {
        col.x += AMB.x; col.y += AMB.y; col.z += AMB.z;
        return col;
    }
    c->c[ORC_C_HITS]++;
    v3 ip = add3(o, mul3(d, t));
    const tri_t* tr = &s->tris[index];
    v3 ks = tr->ks, kd = tr->kd, kr = tr->kr, n = tr->norm[nd];
    col.x += kd.x * AMB.x; col.y += kd.y * AMB.y; col.z += kd.z * AMB.z;
    d = mul3(d, -1.0f);
    for (int i = 0; i < s->nl; i++) {
        v3 l = sub3(s->lights[i].pos, ip);
        float mag = mag3(l);
        l = div3(l, mag);
        mag *= mag;
        float ndl = dot3(n, l);
        v3 cr = lambert_blinn(ks, kd, n, l, d, ndl);
        int V = light_v(s, ip, l, n, s->lights[i].pos, c);
        col.x += V * s->lights[i].kl.x * cr.x / mag;
        col.y += V * s->lights[i].kl.y * cr.y / mag;
        col.z += V * s->lights[i].kl.z * cr.z / mag;
    }
    d = mul3(d, -1);
    v3 ns = mul3(n, 2 * fabsf(dot3(d, n)));
    v3 r = norm3(add3(d, ns));
    if (mag3(kr) > 0.0) {
        v3 cr = raytrace(s, ip, r, iter + 1, c, bh);
        col.x += kr.x * cr.x; col.y += kr.y * cr.y; col.z += kr.z * cr.z;
    }
    return col;
}

/* ---------------------------------------------------------------- camera (cam.c:5-48, main.c:105-106) */
typedef struct { v3 pos, rot; float fov; } cam_t;

static void rot_all(const cam_t* c, v3* p) {                      /* cam.c:11-33, order Y, X, Z */
    v3 t = *p;
    p->x = t.x * cosf(c->rot.y) + t.z * sinf(c->rot.y);
    p->z = -t.x * sinf(c->rot.y) + t.z * cosf(c->rot.y);
    t = *p;
    p->y = t.y * cosf(c->rot.x) - t.z * sinf(c->rot.x);
    p->z = t.y * sinf(c->rot.x) + t.z * cosf(c->rot.x);
    t = *p;
    p->x = t.x * cosf(c->rot.z) - t.y * sinf(c->rot.z);
    p->y = t.x * sinf(c->rot.z) + t.y * cosf(c->rot.z);
}

void orc_camera(int W, int H, float out[12]) {
    cam_t c;
    float fov = (float)(M_PI / 3.2);                               /* cam_init(.., M_PI/3.2) */
    c.pos = (v3){0, -9, 3};
    c.rot = (v3){0, 0, 0};
    c.fov = 1.0 / tanf(fov / 2.0f);
    c.rot.x = -M_PI / 12;
    float ar = (float)W / H;
    v3 sp[3] = {{-1 * ar, c.fov, +1}, {+1 * ar, c.fov, +1}, {-1 * ar, c.fov, -1}};
    for (int i = 0; i < 3; i++) { rot_all(&c, &sp[i]); sp[i] = add3(sp[i], c.pos); }
    v3 ix = div3(sub3(sp[1], sp[0]), W);
    v3 iy = div3(sub3(sp[2], sp[0]), H);
    float* o = out;
    o[0] = c.pos.x; o[1] = c.pos.y; o[2] = c.pos.z;
    o[3] = sp[0].x; o[4] = sp[0].y; o[5] = sp[0].z;
    o[6] = ix.x; o[7] = ix.y; o[8] = ix.z;
    o[9] = iy.x; o[10] = iy.y; o[11] = iy.z;
}

/* ---------------------------------------------------------------- frame driver (main.c:214-264) */
typedef struct {
    const orc_scene* s;
    int W, H, spp, row_offset, row_stride, n_rows;
    atomic_int next;
    int32_t *hit, *bh;
    float *t, *rgb;
    v3 pos, ul, ix, iy;
    ctr_t tot;
    pthread_mutex_t mu;
} job_t;

static void* worker(void* arg) {
    job_t* j = (job_t*)arg;
    ctr_t c;
    memset(&c, 0, sizeof c);
    const orc_scene* s = j->s;
    int g = 1;
    while (g * g < j->spp) g++;
    for (;;) {
        int k = atomic_fetch_add(&j->next, 1);
        if (k >= j->n_rows) break;
        int y = j->row_offset + k * j->row_stride;
        for (int x = 0; x < j->W; x++) {
            size_t idx = (size_t)y * j->W + x;
            if (j->spp <= 1) {
                v3 d = sub3(j->ul, j->pos);                        /* main.c:229-233 */
                d = add3(d, mul3(j->ix, x));
                d = add3(d, mul3(j->iy, y));
                if (j->hit || j->t) {
                    int nd = 0, ti = -1;
                    float t = FLT_MAX;
                    ctr_t dummy;
                    memset(&dummy, 0, sizeof dummy);
                    if (s->use_bvh) traverse(s, j->pos, d, &nd, &t, &ti, &dummy);
                    else brute_closest(s, j->pos, d, &nd, &t, &ti, &dummy);
                    if (j->hit) j->hit[idx] = ti;
                    if (j->t) j->t[idx] = t;
                }
                int32_t bh[4] = {-2, -2, -2, -2};
                v3 col = raytrace(s, j->pos, d, 0, &c, bh);
                col.x = fminf(fmaxf(col.x, 0), 1);                  /* vec_constrain, vec.c:47-54 */
                col.y = fminf(fmaxf(col.y, 0), 1);
                col.z = fminf(fmaxf(col.z, 0), 1);
                if (j->rgb) { j->rgb[3 * idx] = col.x; j->rgb[3 * idx + 1] = col.y; j->rgb[3 * idx + 2] = col.z; }
                if (j->bh) memcpy(&j->bh[4 * idx], bh, sizeof bh);
            } else {
                v3 acc = {0, 0, 0};
                for (int sj = 0; sj < g; sj++)
                    for (int si = 0; si < g; si++) {
                        float fx = (float)x + ((float)si + 0.5f) / (float)g;
                        float fy = (float)y + ((float)sj + 0.5f) / (float)g;
                        v3 d = sub3(j->ul, j->pos);
                        d = add3(d, mul3(j->ix, fx));
                        d = add3(d, mul3(j->iy, fy));
                        v3 col = raytrace(s, j->pos, d, 0, &c, NULL);
                        col.x = fminf(fmaxf(col.x, 0), 1);
                        col.y = fminf(fmaxf(col.y, 0), 1);
                        col.z = fminf(fmaxf(col.z, 0), 1);
                        acc = add3(acc, col);
                    }
                float inv_n = (float)(g * g);
                if (j->rgb) {
                    j->rgb[3 * idx] = acc.x / inv_n;
                    j->rgb[3 * idx + 1] = acc.y / inv_n;
                    j->rgb[3 * idx + 2] = acc.z / inv_n;
                }
            }
        }
    }
    pthread_mutex_lock(&j->mu);
    for (int i = 0; i < ORC_NCOUNTERS; i++) j->tot.c[i] += c.c[i];
    pthread_mutex_unlock(&j->mu);
    return NULL;
}

static int run(const orc_scene* s, int W, int H, int spp, int ro, int rs, int nr, int threads,
               int32_t* hit, float* t, float* rgb, int32_t* bh, uint64_t* counters) {
    if (!s || W <= 0 || H <= 0 || rs <= 0 || nr < 0) return -1;
    if (s->use_bvh && !s->bvh) return -2;
    if (ro < 0 || (nr > 0 && ro + (nr - 1) * rs >= H)) return -3;
    job_t* j = (job_t*)calloc(1, sizeof(job_t));
    j->s = s; j->W = W; j->H = H; j->spp = spp; j->row_offset = ro; j->row_stride = rs; j->n_rows = nr;
    atomic_store(&j->next, 0);
    j->hit = hit; j->t = t; j->rgb = rgb; j->bh = bh;
    pthread_mutex_init(&j->mu, NULL);
    float cam[12];
    orc_camera(W, H, cam);
    j->pos = (v3){cam[0], cam[1], cam[2]};
    j->ul = (v3){cam[3], cam[4], cam[5]};
    j->ix = (v3){cam[6], cam[7], cam[8]};
    j->iy = (v3){cam[9], cam[10], cam[11]};
    if (threads <= 0) threads = 1;
    if (threads > 256) threads = 256;
    pthread_t th[256];
    for (int i = 0; i < threads; i++) pthread_create(&th[i], NULL, worker, j);
    for (int i = 0; i < threads; i++) pthread_join(th[i], NULL);
    if (counters) memcpy(counters, j->tot.c, sizeof(uint64_t) * ORC_NCOUNTERS);
    pthread_mutex_destroy(&j->mu);
    free(j);
    return 0;
}

int orc_render(const orc_scene* s, int W, int H, int ro, int rs, int nr, int threads,
               int32_t* hit, float* t, float* rgb, int32_t* bh, uint64_t* counters) {
    return run(s, W, H, 1, ro, rs, nr, threads, hit, t, rgb, bh, counters);
}

int orc_render_spp(const orc_scene* s, int W, int H, int spp, int ro, int rs, int nr, int threads,
                   float* rgb, uint64_t* counters) {
    return run(s, W, H, spp < 1 ? 1 : spp, ro, rs, nr, threads, NULL, NULL, rgb, NULL, counters);
}
