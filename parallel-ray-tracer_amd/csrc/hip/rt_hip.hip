// librt_hip.so — the rt_* C-ABI (include/rt_hip.h) over the HIP kernels in rt_kernels.hpp.
//
// Replaces load_to_gpu / render_frame / load_from_gpu (gpu/include/gpu.cuh:23-26, gpu/src/gpu.cu:98-228)
// and the CPU render_frame (cpu/src/main.c:214-264). All state is per context; every call returns a
// status; HIP errors are captured into rt_last_error() instead of being printed and ignored.
#include <hip/hip_runtime.h>
#include <dlfcn.h>
#include <rccl/rccl.h>

#include <type_traits>

#include <algorithm>
#include <climits>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <memory>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#include "rt_hip.h"
#include "rt_host.h"
#include "rt_kernels.hpp"
#include "rt_shpool.hpp"
#include "rt_coop.hpp"
#include "rt_output.hpp"
#include "rt_build.hpp"
#include "rt_comm_logic.hpp"
#include "rt_treelet.hpp"
#include "rt_feedback.hpp"
#ifndef PRT_TREELET
#define PRT_TREELET 2  // treelet-restructuring passes over the GPU-built binary tree (0: none)
#endif

#include <chrono>
#include <hipcub/hipcub.hpp>

#include <cstdlib>

namespace {

// One BVH view in device memory (rt_device.hpp DBvh) and its host-side build.
struct DevView {
    float4* nodes = nullptr;
    int2* leaves = nullptr;
    float4* tris = nullptr;
    int* orig = nullptr;
    int* path = nullptr;  // [n_tris: original triangle -> its leaf][n_leaves: leaf -> parent record] (ref view)
    int root = 0, n_inner = 0, n_leaves = 0;
    size_t bytes = 0;
};

struct HostView {
    std::vector<float4> nodes, tris;
    std::vector<int2> leaves;
    std::vector<int> orig;
    std::vector<int> path;  // DevView::path
    int root = 0;
};

// The multi-process communicator whose send / recv groups a context's stream holds (rt_ctx::comm_link): shared by both,
// so that a host wait on that stream (rt_sync, rt_download, rt_destroy, ...) first waits, bounded, for the
// communicator's outstanding groups -- a peer that never joins turns into RT_E_TIMEOUT there too, not into a hang --
// and so that either side may be destroyed first (rt_comm_destroy clears cm).
struct CommLink {
    rt_comm* cm = nullptr;
};

}  // namespace

struct rt_ctx {
    int device = 0;
    unsigned flags = 0;
    hipStream_t stream = nullptr;
    bool own_stream = false;
    std::string err;
    // device scene
    DevView ref, acc;  // acc.nodes == nullptr: acc aliases ref
    // 8-wide quantised view of acc (rt_wide.cpp); wide_nodes == nullptr: none
    float4 *wide_nodes = nullptr, *wide_tris = nullptr;
    int* wide_orig = nullptr;
    int wide_n = 0, wide_depth = 0;
    // the unit-direction view (rtd::DScene::unit): the wide BVH over the triangles a unit-length ray can hit
    float4 *unit_nodes = nullptr, *unit_tris = nullptr;
    int* unit_orig = nullptr;
    int unit_n = 0, unit_depth = 0, unit_tris_n = 0;
    // the primary view (rtd::DScene::prim): the wide BVH over the triangles a direction of length <= PRIMARY_D can hit
    float4 *prim_nodes = nullptr, *prim_tris = nullptr;
    int* prim_orig = nullptr;
    int prim_n = 0, prim_depth = 0, prim_tris_n = 0;
    float4* d_shade = nullptr;
    float4* d_mats = nullptr;
    float4* d_lights = nullptr;
    int n_lights = 0, n_tris = 0;
    // the packed builds' bounds: 5-byte stack entries hold a 24-bit child base (rtd::WIDE_MAX_NODES wide nodes per
    // view), packed triangle-test jobs a 26-bit triangle (rtd::TQ_MAX_TRIS); larger scenes run the unpacked builds
    bool pk_ok = true, tq_ok = true;
    float amb[3] = {0.5f, 0.5f, 0.5f};
    // every face coordinate of the reference tree's child boxes, per axis, sorted; on the device one after another
    // (rtd::DScene::faces)
    std::vector<float> faces[3];
    float* d_faces = nullptr;
    bool has_scene = false;
    rt_scene_info info{};  // what the last upload built (rt_get_scene_info)
    float t_ploc = 0.0f, t_treelet = 0.0f, t_collapse = 0.0f;  // the upload's build stages (ms; rt_scene_info)
    // outputs / bookkeeping
    float* d_rgb_own = nullptr;
    size_t rgb_cap = 0;
    float* last_rgb = nullptr;
    unsigned* last_bgra = nullptr;  // the last render's BGRA8 output (rt_outputs.bgra), or a gathered full frame
    int* last_hit = nullptr;
    size_t last_pixels = 0;
    int last_W = 0, last_H = 0, last_off = 0, last_stride = 1, last_rows = 0, last_block = 1;  // the last frame's rows
    int last_shift = 0;
    int last_frames = 1;     // frames of the last render (rt_render_frames)
    bool batch_sum = false;  // set while rt_render_frames launches frames one by one (counters add up)
    // frame batches: the cameras on the device (d_cams, read by the kernels in stream order) and a ring of pinned host
    // slots they are copied from (upload_cams): a slot is rewritten only once its earlier copy has run, so a changed
    // camera set never waits for the renders in flight
    static constexpr int CAM_SLOTS = 8;
    float* d_cams = nullptr;
    hipEvent_t cam_ev[CAM_SLOTS] = {};
    int cam_slot = 0;
    std::vector<float> cams_last;  // the set d_cams holds (after its copy)
    rt_launch_info last_launch{};  // rt_get_launch_info
    float4* d_pathbuf = nullptr;  // PB kernels: per-wave path levels (rtd::KArgs::pathbuf)
    float4* d_lanebuf = nullptr;  // k_persist's multi-sample builds: one slot per resident lane (rtd::KArgs::lanebuf)
    int* d_gstack = nullptr;      // DYN kernels: the binary walks' stacks (rtd::KArgs::gstack)
    float* h_cams = nullptr;  // pinned: CAM_SLOTS x cams_cap cameras
    int cams_cap = 0;
    // output stage (rt_gather, rt_download_bmp)
    float* d_full = nullptr;
    int* d_full_hit = nullptr;
    size_t full_cap = 0, full_hit_cap = 0;
    char* d_stage = nullptr;
    size_t stage_cap = 0;
    unsigned* d_bmp = nullptr;
    size_t bmp_cap = 0;
    unsigned* d_full_bgra = nullptr;  // gathered BGRA8 frames (rt_gather / rt_comm_gather of bgra renders)
    size_t full_bgra_cap = 0;
    unsigned long long* d_counters = nullptr;  // rtd::NCOUNT
    unsigned long long* h_err = nullptr;       // pinned: the last render's error counter (rtd::C_ERR), read by rt_sync / rt_download
    std::unordered_map<long long, int*> orders;  // tile dealing orders (rt_frame.dealing), per tx x ty tile grid
    unsigned int* d_work = nullptr;
    static constexpr int NEV = 64;  // ring of per-launch event pairs (rt_kernel_times)
    hipEvent_t ev0s[NEV] = {}, ev1s[NEV] = {};
    hipEvent_t ev0 = nullptr, ev1 = nullptr;  // the last launch's pair
    hipEvent_t gather_ev = nullptr;           // completion of the last rt_gather into this (root) context
    hipEvent_t copy_ev = nullptr;             // rt_gather: this (source) context's peer copies issued
    long long launches = 0;
    bool rendered = false;
    std::shared_ptr<CommLink> comm_link;  // the communicator with a send / recv group on this stream (CommLink)
    // the default rule of frame batches and spp > 1 (PERSIST4 or SHPOOL), measured per shape (render_batch)
    struct BatchRule {
        long long scene = -1;
        int W = 0, rows = 0, off = 0, stride = 0, block = 0, shift = 0, bounces = 0, spp = 0, frames = 0, dealing = 0,
            cap_req = 0;
        // trials per candidate: 3, decided by the minimum -- or, for launches longer than LONG_MS, the median (the
        // 64-spp configuration's 190-ms launches of one kernel ranged 186-199 ms on one box; the minimum of two trials
        // picked either kernel)
        static constexpr int ROUNDS = 3;
        static constexpr float LONG_MS = 50.0f;
        long long launch[2][ROUNDS] = {{-1, -1, -1}, {-1, -1, -1}};
        int choice = -1;
    };
    std::vector<BatchRule> brules;
    long long scene_gen = 0;  // bumped by every upload
    // RT_VARIANT_HYBRID (single 1-spp frames), keyed by the frame's SHAPE: the per-tile times of a measuring k_persist
    // frame, the candidates' tile lists they give (the hot kernel's tiles of the costliest 8x8 tiles; the rest for the
    // cold kernel), the trials and the choice
    struct Hybrid {
        long long scene = -1;
        int W = 0, rows = 0, off = 0, stride = 0, block = 0, bounces = 0, dealing = 0, pct_req = 0, hk_req = 0;
        int state = 0;  // 0: measure next; 1: a measuring frame's tile times are on their way to h_tr; 2: lists ready
        long long frames = 0;  // frames since the choice or the last list refresh
        static constexpr int NCAND = 12;
        static constexpr int ROUNDS = 4;    // trial frames per candidate, back to back: the first untimed (its per-tile
                                            // times feed the next one's lists), the best median of the other three
                                            // chosen (single frames are noisy, and some two-stream launches bimodal).
                                            // Back to back, not round robin: a hybrid candidate's lists are built from
                                            // the frame before it, and after another candidate's frame they are not the
                                            // lists it renders with once chosen (a car_boxed walkthrough priced its hot
                                            // candidates 30-60 % slow and settled on none of them)
        static constexpr int WARM = 1;
        static constexpr int REFRESH = 64;  // frames of a shape between measuring frames once it is decided
        // candidates: hot threshold (0 = the cold kernel over the whole frame), lanes per ray of k_coop for the hot
        // tiles, the cold tiles' kernel (RT_VARIANT_PERSIST / SHPOOL); their lists at d_lists + at[c]
        int nc = 0, choice = -1;
        int pct[NCAND] = {}, lanes[NCAND] = {}, cold[NCAND] = {}, n_hot[NCAND] = {}, n_cold[NCAND] = {};
        bool lpt[NCAND] = {};
        size_t at[NCAND] = {};
        long long launch[NCAND][ROUNDS] = {};
        float ms[NCAND] = {};
        unsigned long long* d_tr = nullptr;  // [tiles][4], rtd::k_persist's TRACE records
        unsigned long long* h_tr = nullptr;  // pinned
        size_t tr_cap = 0, n_tiles = 0;
        int* d_lists = nullptr;  // per candidate: [hot tiles][cold 8x8 tiles: XCD region layout or order]
        int* h_lists = nullptr;  // pinned staging of d_lists (stream-ordered copies)
        size_t lists_cap = 0, hl_cap = 0;
        bool cold_regions = false;
        int cold_mode = 0;  // the cold lists' region layout (xcd_mode) when cold_regions
        hipEvent_t ev = nullptr, fork = nullptr, join = nullptr;
        hipStream_t s2 = nullptr;
        // per-frame feedback (rt_feedback.hpp): every frame of the shape records its 8x8 tiles' durations in d_cost (and
        // their maximum after them); a decided shape's frames build their lists from the previous frame's on the device
        // (d_fb: [hot: 4 x n_tiles][cold: 9 + n_tiles][counts: 4][the builder's table: FB_G x FB_TK][its partials:
        // 3 FB_G]); h_fb_cnt: a
        // recent frame's hot count, read back without waiting (grid sizes)
        unsigned* d_cost = nullptr;  // two buffers of fb_cap + 1 words: the last frame's (cost_at(cost_cur)), the next
        int cost_cur = 0;            // frame's (cleared by the list builder, k_fb_max: no memset launch per frame)
        unsigned* cost_at(int i) const { return d_cost + (size_t)i * (fb_cap + 1); }
        int* d_fb = nullptr;
        unsigned char* d_info = nullptr;  // rtd::fb_tile_info of every tile, for info_mode
        int info_mode = -1;
        size_t fb_cap = 0;
        bool fb_ok = false;  // d_cost holds a whole frame of this shape (stream order)
        int* h_fb_cnt = nullptr;
        hipEvent_t fb_ev = nullptr;
        bool fb_pending = false;
        int fb_est_c = -1, fb_pend_c = -1;  // the candidates whose hot counts fb_hot_est / the pending copy hold
        float fb_cam[12] = {};  // the last feedback frame's camera (pos, ul, ix, iy)
        bool fb_cam_ok = false;
        int fb_hot_est = -1;
    } hy;
};

namespace {

// RT_VARIANT_HYBRID candidates: pct = 0: the cold kernel over the whole frame; else the 8x8 tiles slower than pct % of the
// slowest tile of the measuring frame go to k_coop with `lanes` lanes per ray while the cold kernel renders the rest
// (each candidate is tried ROUNDS times; hybrid_pick). Measured: car_boxed hot > 45 % k_coop<4>,
// sportscar hot > 60 % k_coop<2> / <4>, dragon the whole-frame kernels; k_fan and k_relay hot tiles never won
// (both removed).
// lpt: the cold tiles dealt costliest first by the measuring frame's per-tile times (longest processing time first,
// the classic makespan heuristic: a single frame ends with its slowest tile) instead of centre-out; with pct = 0 the
// whole frame that way.
struct HotCand {
    int pct, lanes, cold;
    bool lpt;
};
// The candidates are the configurations that won on some BASELINE scene (dragon the shadow pool in LPT
// order, car_boxed hot > 45 % k_coop<4> with LPT cold tiles, sportscar hot > 60 % k_coop<4> / <2>) plus k_persist in
// LPT order: few candidates keep the trial frames few (3 each) and the choice robust to frame-to-frame noise (a moving
// camera changes every trial frame's cost; nine candidates picked a 12 % slower one on a walkthrough).
// (RT_VARIANT_SHPOOL here stands for the rule's pool kernel: RT_VARIANT_SHDEFER where its path buffer fits.)
constexpr HotCand HYBRID_CANDS[] = {{0, 0, RT_VARIANT_SHPOOL, true},   {0, 0, RT_VARIANT_PERSIST, true},
                                    {45, 4, RT_VARIANT_PERSIST, true}, {60, 4, RT_VARIANT_PERSIST, false},
                                    {60, 2, RT_VARIANT_PERSIST, false}};
// Per-frame feedback (rt_feedback.hpp) for a decided shape: its frames deal their tiles by the previous frame's
// per-tile durations, the lists built on the device, instead of a measuring frame's every REFRESH frames
#ifndef PRT_FEEDBACK
#define PRT_FEEDBACK 1
#endif
// pixel tile of a group kernel (rtd::GTile): k_coop<2> 8x4, k_coop<4> 4x4
inline void hot_tile(int g, int& tw, int& th) {
    tw = g == 2 ? 8 : 4;
    th = 4;
}

const char* variant_name(int v) {
    switch (v) {
        case RT_VARIANT_PERSIST: return "persist";
        case RT_VARIANT_PERSIST4: return "persist4";
        case RT_VARIANT_COOP2: return "coop2";
        case RT_VARIANT_COOP4: return "coop4";
        case RT_VARIANT_HYBRID: return "hybrid";
        case RT_VARIANT_SHPOOL: return "shpool";
        case RT_VARIANT_SHDEFER: return "shdefer";
        default: return "default";
    }
}

int fail(rt_ctx* c, hipError_t e, const char* what) {
    if (c) c->err = std::string(what) + ": " + hipGetErrorString(e);
    return RT_E_HIP;
}
#define HIPC(call)                                          \
    do {                                                    \
        hipError_t e_ = (call);                             \
        if (e_ != hipSuccess) return fail(ctx, e_, #call); \
    } while (0)

int arg_err(rt_ctx* c, const char* msg) {
    if (c) c->err = msg;
    return RT_E_ARG;
}

void free_view(DevView& v) {
    for (void* p : {(void*)v.nodes, (void*)v.leaves, (void*)v.tris, (void*)v.orig, (void*)v.path})
        if (p) (void)hipFree(p);
    v = DevView();
}

void free_scene(rt_ctx* ctx) {
    free_view(ctx->ref);
    free_view(ctx->acc);
    for (void* p : {(void*)ctx->wide_nodes, (void*)ctx->wide_tris, (void*)ctx->wide_orig})
        if (p) (void)hipFree(p);
    ctx->wide_nodes = ctx->wide_tris = nullptr;
    ctx->wide_orig = nullptr;
    ctx->wide_n = ctx->wide_depth = 0;
    for (void* p : {(void*)ctx->unit_nodes, (void*)ctx->unit_tris, (void*)ctx->unit_orig})
        if (p) (void)hipFree(p);
    ctx->unit_nodes = ctx->unit_tris = nullptr;
    ctx->unit_orig = nullptr;
    ctx->unit_n = ctx->unit_depth = ctx->unit_tris_n = 0;
    for (void* p : {(void*)ctx->prim_nodes, (void*)ctx->prim_tris, (void*)ctx->prim_orig})
        if (p) (void)hipFree(p);
    ctx->prim_nodes = ctx->prim_tris = nullptr;
    ctx->prim_orig = nullptr;
    ctx->prim_n = ctx->prim_depth = ctx->prim_tris_n = 0;
    for (void* p : {(void*)ctx->d_shade, (void*)ctx->d_mats, (void*)ctx->d_lights, (void*)ctx->d_faces})
        if (p) (void)hipFree(p);
    ctx->d_faces = nullptr;
    for (auto& f : ctx->faces) f.clear();
    ctx->d_shade = nullptr;
    ctx->d_mats = nullptr;
    ctx->d_lights = nullptr;
    ctx->has_scene = false;
}

template <class T>
int upload(rt_ctx* ctx, T** dst, const std::vector<T>& src, size_t* bytes = nullptr) {
    size_t b = sizeof(T) * (src.empty() ? 1 : src.size());
    HIPC(hipMalloc((void**)dst, b));
    if (!src.empty()) HIPC(hipMemcpy(*dst, src.data(), sizeof(T) * src.size(), hipMemcpyHostToDevice));
    if (bytes) *bytes += b;
    return RT_OK;
}

inline float i2f(int i) {
    float f;
    std::memcpy(&f, &i, 4);
    return f;
}

// leaf-ordered triangle planes: v0, e1, e2, n = e1 x e2 (raytracer.c:36-38, same roundings)
void tri_records(const rt_triangle* T, const int* order, int n, std::vector<float4>& tris, std::vector<int>& orig) {
    tris.resize(3 * (size_t)n);
    orig.resize(n);
    for (int i = 0; i < n; i++) {
        const rt_triangle& t = T[order[i]];
        orig[i] = order[i];
        const rt_vec3 &a = t.coords[0], &b = t.coords[1], &c = t.coords[2];
        const float e1x = b.x - a.x, e1y = b.y - a.y, e1z = b.z - a.z;
        const float e2x = c.x - a.x, e2y = c.y - a.y, e2z = c.z - a.z;
        const float nx = e1y * e2z - e1z * e2y, ny = e1z * e2x - e1x * e2z, nz = e1x * e2y - e1y * e2x;
        tris[3 * i + 0] = make_float4(a.x, a.y, a.z, e1x);
        tris[3 * i + 1] = make_float4(e1y, e1z, e2x, e2y);
        tris[3 * i + 2] = make_float4(e2z, nx, ny, nz);
    }
}

// Reference-layout BVH (bvh_t[], tri_idx) -> device view. `inflate` > 0 grows every child box by that
// absolute amount (acceleration BVH: keeps the reciprocal-FMA slab test conservative); 0 keeps the
// reference's boxes bit-for-bit (strict walk).
int build_view(rt_ctx* ctx, const rt_bvh_node* B, int nn, const int* tri_idx, const rt_triangle* T, int n,
               float inflate, HostView& v) {
    std::vector<char> seen(n, 0);
    for (int i = 0; i < n; i++) {
        int t = tri_idx[i];
        if (t < 0 || t >= n || seen[t]) return arg_err(ctx, "rt_upload_scene: tri_idx is not a permutation");
        seen[t] = 1;
    }
    // refs: interior -> record index (DFS preorder), leaf -> ~leaf id, empty -> EMPTY_REF
    std::vector<int> ref(nn, rtd::EMPTY_REF);
    std::vector<int> inner;
    std::vector<int> st{0};
    std::vector<char> visited(nn, 0);
    while (!st.empty()) {
        int i = st.back();
        st.pop_back();
        if (i < 0 || i >= nn || visited[i]) return arg_err(ctx, "rt_upload_scene: malformed bvh (child index)");
        visited[i] = 1;
        const rt_bvh_node& b = B[i];
        if (b.tr_len > 0) {
            if (b.child < 0 || (long long)b.child + b.tr_len > n)
                return arg_err(ctx, "rt_upload_scene: leaf range outside tri_idx");
            ref[i] = ~(int)v.leaves.size();
            v.leaves.push_back(make_int2(b.child, b.tr_len));
        } else if (b.child != 0) {
            if (b.child < 1 || b.child + 1 >= nn) return arg_err(ctx, "rt_upload_scene: child index out of range");
            ref[i] = (int)inner.size();
            inner.push_back(i);
            st.push_back(b.child + 1);
            st.push_back(b.child);  // left first: preorder, near-first locality
        }
    }
    if (ref[0] == rtd::EMPTY_REF) return arg_err(ctx, "rt_upload_scene: empty root");
    v.root = ref[0];
    v.nodes.resize(4 * inner.size());
    // parents: a record's in its 4th float4's z (-1: the root), a leaf's in path[n + leaf]; path[t]: triangle t's leaf
    std::vector<int> parent(inner.size(), -1);
    v.path.assign((size_t)n + v.leaves.size(), -1);
    for (size_t r = 0; r < inner.size(); r++) {
        const rt_bvh_node& p = B[inner[r]];
        for (int k = 0; k < 2; k++) {
            const int c = ref[p.child + k];
            if (c >= 0) parent[c] = (int)r;
            else if (c != rtd::EMPTY_REF) v.path[(size_t)n + ~c] = (int)r;
        }
    }
    for (size_t l = 0; l < v.leaves.size(); l++)
        for (int i = v.leaves[l].x; i < v.leaves[l].x + v.leaves[l].y; i++) v.path[tri_idx[i]] = (int)l;
    for (size_t r = 0; r < inner.size(); r++) {
        const rt_bvh_node& p = B[inner[r]];
        rt_bvh_node L = B[p.child], R = B[p.child + 1];
        if (inflate > 0)
            for (rt_bvh_node* c : {&L, &R}) {
                c->min.x -= inflate;
                c->min.y -= inflate;
                c->min.z -= inflate;
                c->max.x += inflate;
                c->max.y += inflate;
                c->max.z += inflate;
            }
        v.nodes[4 * r + 0] = make_float4(L.min.x, L.min.y, L.min.z, L.max.x);
        v.nodes[4 * r + 1] = make_float4(L.max.y, L.max.z, R.min.x, R.min.y);
        v.nodes[4 * r + 2] = make_float4(R.min.z, R.max.x, R.max.y, R.max.z);
        v.nodes[4 * r + 3] = make_float4(i2f(ref[p.child]), i2f(ref[p.child + 1]), i2f(parent[r]), 0.0f);
    }
    tri_records(T, tri_idx, n, v.tris, v.orig);
    return RT_OK;
}

int upload_view(rt_ctx* ctx, const HostView& h, DevView& d) {
    int rc;
    d.bytes = 0;
    if ((rc = upload(ctx, &d.nodes, h.nodes, &d.bytes)) || (rc = upload(ctx, &d.leaves, h.leaves, &d.bytes)) ||
        (rc = upload(ctx, &d.tris, h.tris, &d.bytes)) || (rc = upload(ctx, &d.orig, h.orig, &d.bytes)) ||
        (rc = upload(ctx, &d.path, h.path, &d.bytes)))
        return rc;
    d.root = h.root;
    d.n_inner = (int)(h.nodes.size() / 4);
    d.n_leaves = (int)h.leaves.size();
    return RT_OK;
}

}  // namespace

extern "C" int rt_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

extern "C" const char* rt_version(void) { return "prt-mi355x 0.2 (gfx950)"; }

extern "C" int rt_create(const rt_opts* opts, rt_ctx** out) {
    if (!out) return RT_E_ARG;
    *out = nullptr;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return RT_E_NODEVICE;
    rt_ctx* ctx = new rt_ctx();
    if (opts) {
        ctx->device = opts->device;
        ctx->flags = opts->flags;
        ctx->stream = (hipStream_t)opts->stream;
    }
    if (ctx->device < 0 || ctx->device >= n) {
        delete ctx;
        return RT_E_ARG;
    }
    hipError_t e = hipSetDevice(ctx->device);
    if (e == hipSuccess && !ctx->stream) {
        e = hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking);
        ctx->own_stream = true;
    }
    for (int i = 0; i < rt_ctx::NEV && e == hipSuccess; i++) {
        e = hipEventCreate(&ctx->ev0s[i]);
        if (e == hipSuccess) e = hipEventCreate(&ctx->ev1s[i]);
    }
    if (e == hipSuccess) e = hipMalloc((void**)&ctx->d_counters, sizeof(unsigned long long) * rtd::NCOUNT);
    if (e == hipSuccess) e = hipMalloc((void**)&ctx->d_work, 1024);
    if (e == hipSuccess) e = hipMemset(ctx->d_counters, 0, sizeof(unsigned long long) * rtd::NCOUNT);
    if (e == hipSuccess) e = hipHostMalloc((void**)&ctx->h_err, sizeof(unsigned long long), hipHostMallocDefault);
    if (e != hipSuccess) {
        rt_destroy(ctx);
        return RT_E_HIP;
    }
    *out = ctx;
    return RT_OK;
}

// load_to_gpu (gpu/src/gpu.cu:129-201): reference layouts -> device layout (rt_device.hpp).
namespace {
// host threads of the acceleration build's CPU stages (the treelet passes, rt_treelet.hpp): the machine's, at most 16
// (the GPU box's CPU quota; nproc there reports the whole host)
int build_threads() {
    const unsigned hc = std::thread::hardware_concurrency();
    return (int)std::max(1u, std::min(16u, hc));
}
// GPU-built acceleration BVH (rt_build.hpp, PLOC) in the reference layout: children of a node at child and
// child + 1, single-triangle leaves numbered depth-first (every subtree's triangles are one range of idx).
// Returns RT_OK, or RT_E_STATE when the tree is unusable (the caller falls back to the host build).
int gpu_ploc(rt_ctx* ctx, const rt_triangle* T, int n, int R, std::vector<rt_bvh_node>& out, std::vector<int>& idx,
             int& depth_out) {
    hipStream_t st = ctx->stream;
    const auto t_gpu = std::chrono::steady_clock::now();
    std::vector<float> hv(9 * (size_t)n);
    for (int i = 0; i < n; i++)
        for (int k = 0; k < 3; k++) {
            hv[9 * (size_t)i + 3 * k] = T[i].coords[k].x;
            hv[9 * (size_t)i + 3 * k + 1] = T[i].coords[k].y;
            hv[9 * (size_t)i + 3 * k + 2] = T[i].coords[k].z;
        }
    const size_t nn2 = 2 * (size_t)n;
    float* dv = nullptr;
    float4 *plo = nullptr, *phi = nullptr, *nlo = nullptr, *nhi = nullptr;
    unsigned *keys = nullptr, *keys2 = nullptr;
    int *vals = nullptr, *sorted = nullptr, *cb = nullptr, *C = nullptr, *C2 = nullptr, *nnb = nullptr, *mflag = nullptr,
        *keep = nullptr, *moff = nullptr, *koff = nullptr, *left = nullptr, *right = nullptr;
    void* tmp = nullptr;
    size_t tmp_bytes = 0;
    int* tot = nullptr;  // pinned: a merge round's merge and survivor totals
    int rc = RT_OK;
    auto done = [&]() {
        if (tot) (void)hipHostFree(tot);
        tot = nullptr;
        for (void* p : {(void*)dv, (void*)plo, (void*)phi, (void*)nlo, (void*)nhi, (void*)keys, (void*)keys2, (void*)vals,
                        (void*)sorted, (void*)cb, (void*)C, (void*)C2, (void*)nnb, (void*)mflag, (void*)keep, (void*)moff,
                        (void*)koff, (void*)left, (void*)right, tmp})
            if (p) (void)hipFree(p);
        return rc;
    };
#define PLOC(call)                                   \
    do {                                             \
        hipError_t e_ = (call);                      \
        if (e_ != hipSuccess) {                      \
            rc = fail(ctx, e_, #call);               \
            return done();                           \
        }                                            \
    } while (0)
    PLOC(hipMalloc((void**)&dv, sizeof(float) * hv.size()));
    PLOC(hipMalloc((void**)&plo, sizeof(float4) * n));
    PLOC(hipMalloc((void**)&phi, sizeof(float4) * n));
    PLOC(hipMalloc((void**)&nlo, sizeof(float4) * nn2));
    PLOC(hipMalloc((void**)&nhi, sizeof(float4) * nn2));
    PLOC(hipMalloc((void**)&keys, sizeof(unsigned) * n));
    PLOC(hipMalloc((void**)&keys2, sizeof(unsigned) * n));
    for (int** p : {&vals, &sorted, &C, &C2, &nnb, &mflag, &keep, &moff, &koff}) PLOC(hipMalloc((void**)p, sizeof(int) * n));
    PLOC(hipMalloc((void**)&left, sizeof(int) * std::max(1, n - 1)));
    PLOC(hipMalloc((void**)&right, sizeof(int) * std::max(1, n - 1)));
    PLOC(hipMalloc((void**)&cb, sizeof(int) * 8));
    PLOC(hipMemcpyAsync(dv, hv.data(), sizeof(float) * hv.size(), hipMemcpyHostToDevice, st));
    const int cb_init[6] = {0x7FFFFFFF, 0x7FFFFFFF, 0x7FFFFFFF, (int)0x80000000, (int)0x80000000, (int)0x80000000};
    PLOC(hipMemcpyAsync(cb, cb_init, sizeof cb_init, hipMemcpyHostToDevice, st));
    const int g = (n + 255) / 256;
    rtb::k_prim_boxes<<<g, 256, 0, st>>>(dv, n, plo, phi, cb);
    rtb::k_morton<<<g, 256, 0, st>>>(plo, phi, n, cb, keys, vals);
    PLOC(hipGetLastError());
    size_t sort_bytes = 0, scan_bytes = 0;
    PLOC(hipcub::DeviceRadixSort::SortPairs(nullptr, sort_bytes, keys, keys2, vals, sorted, n, 0, 30, st));
    PLOC(hipcub::DeviceScan::ExclusiveSum(nullptr, scan_bytes, mflag, moff, n, st));
    tmp_bytes = std::max(sort_bytes, scan_bytes);
    PLOC(hipMalloc(&tmp, tmp_bytes));
    PLOC(hipcub::DeviceRadixSort::SortPairs(tmp, sort_bytes, keys, keys2, vals, sorted, n, 0, 30, st));
    rtb::k_leaves<<<g, 256, 0, st>>>(sorted, plo, phi, n, nlo, nhi, C);
    PLOC(hipGetLastError());
    int m = n, next = n;
    PLOC(hipHostMalloc((void**)&tot, sizeof(int) * 4, hipHostMallocDefault));
    while (m > 1) {
        const int gm = (m + 255) / 256;
        rtb::k_nn<<<gm, 256, 0, st>>>(C, m, nlo, nhi, nnb, R);
        rtb::k_flags<<<gm, 256, 0, st>>>(nnb, m, mflag, keep);
        size_t b1 = tmp_bytes, b2 = tmp_bytes;
        PLOC(hipcub::DeviceScan::ExclusiveSum(tmp, b1, mflag, moff, m, st));
        PLOC(hipcub::DeviceScan::ExclusiveSum(tmp, b2, keep, koff, m, st));
        PLOC(hipMemcpyAsync(tot, moff + m - 1, sizeof(int), hipMemcpyDeviceToHost, st));
        PLOC(hipMemcpyAsync(tot + 1, mflag + m - 1, sizeof(int), hipMemcpyDeviceToHost, st));
        PLOC(hipMemcpyAsync(tot + 2, koff + m - 1, sizeof(int), hipMemcpyDeviceToHost, st));
        PLOC(hipMemcpyAsync(tot + 3, keep + m - 1, sizeof(int), hipMemcpyDeviceToHost, st));
        rtb::k_merge<<<gm, 256, 0, st>>>(C, nnb, mflag, moff, m, n, next, nlo, nhi, left, right);
        rtb::k_compact<<<gm, 256, 0, st>>>(C, keep, koff, m, C2);
        PLOC(hipGetLastError());
        PLOC(hipStreamSynchronize(st));
        const int merges = tot[0] + tot[1], survivors = tot[2] + tot[3];
        if (merges <= 0 || survivors != m - merges) {  // no progress: never expected (a mutual pair always exists)
            rc = RT_E_STATE;
            return done();
        }
        next += merges;
        m = survivors;
        std::swap(C, C2);
    }
    // the tree back to the host
    const int ni = n - 1;
    std::vector<int> hl(std::max(ni, 1)), hr(std::max(ni, 1)), hs(n);
    std::vector<float4> hlo(nn2), hhi(nn2);
    int root = 0;
    PLOC(hipMemcpyAsync(&root, C, sizeof(int), hipMemcpyDeviceToHost, st));
    if (ni > 0) {
        PLOC(hipMemcpyAsync(hl.data(), left, sizeof(int) * ni, hipMemcpyDeviceToHost, st));
        PLOC(hipMemcpyAsync(hr.data(), right, sizeof(int) * ni, hipMemcpyDeviceToHost, st));
    }
    PLOC(hipMemcpyAsync(hs.data(), sorted, sizeof(int) * n, hipMemcpyDeviceToHost, st));
    PLOC(hipMemcpyAsync(hlo.data(), nlo, sizeof(float4) * nn2, hipMemcpyDeviceToHost, st));
    PLOC(hipMemcpyAsync(hhi.data(), nhi, sizeof(float4) * nn2, hipMemcpyDeviceToHost, st));
    PLOC(hipStreamSynchronize(st));
#undef PLOC
    using clk = std::chrono::steady_clock;
    auto since = [](clk::time_point t) { return std::chrono::duration<float, std::milli>(clk::now() - t).count(); };
    ctx->t_ploc += since(t_gpu);
    auto t_host = clk::now();
    if (PRT_TREELET > 0 && n >= 3) {  // treelet restructuring on the host (rt_treelet.hpp)
        rtt::Tree T;
        T.n = n;
        T.root = root;
        T.left.assign(hl.begin(), hl.begin() + ni);
        T.right.assign(hr.begin(), hr.begin() + ni);
        T.box.resize(2 * (size_t)n - 1);
        for (size_t i = 0; i < T.box.size(); i++)
            T.box[i] = rtt::Box{{hlo[i].x, hlo[i].y, hlo[i].z}, {hhi[i].x, hhi[i].y, hhi[i].z}};
        for (int p = 0; p < PRT_TREELET; p++) rtt::optimize_pass(T, build_threads());
        std::copy(T.left.begin(), T.left.end(), hl.begin());
        std::copy(T.right.begin(), T.right.end(), hr.begin());
        for (size_t i = (size_t)n; i < T.box.size(); i++) {
            hlo[i] = make_float4(T.box[i].lo[0], T.box[i].lo[1], T.box[i].lo[2], hlo[i].w);
            hhi[i] = make_float4(T.box[i].hi[0], T.box[i].hi[1], T.box[i].hi[2], hhi[i].w);
        }
    }
    ctx->t_treelet += since(t_host);
    t_host = clk::now();
    // reference layout, depth-first: children at consecutive indices, leaves numbered left to right
    out.clear();
    out.reserve(nn2);
    idx.assign(n, 0);
    out.push_back(rt_bvh_node{});
    struct Item {
        int node, at, depth;
    };
    std::vector<Item> stack{{root, 0, 0}};
    int pos = 0, depth = 0;
    while (!stack.empty()) {
        const Item it = stack.back();
        stack.pop_back();
        depth = std::max(depth, it.depth);
        rt_bvh_node& o = out[it.at];
        const float4 l = hlo[it.node], h = hhi[it.node];
        o.min = rt_vec3{l.x, l.y, l.z};
        o.max = rt_vec3{h.x, h.y, h.z};
        if (it.node < n) {  // leaf: one triangle
            o.tr_len = 1;
            o.child = pos;
            idx[pos++] = hs[it.node];
        } else {
            const int c = (int)out.size();
            out[it.at].tr_len = 0;
            out[it.at].child = c;
            out.push_back(rt_bvh_node{});
            out.push_back(rt_bvh_node{});
            stack.push_back({hr[it.node - n], c + 1, it.depth + 1});  // right after left: depth-first, left first
            stack.push_back({hl[it.node - n], c, it.depth + 1});
        }
    }
    depth_out = depth;
    ctx->t_collapse += since(t_host);
    return done();
}
}  // namespace

namespace {
// Reflection and shadow rays have unit-length directions (raytracer.c:153,166), and hit_triangle culls
// |det| < EPSILON with det = -d . n (raytracer.c:41-45): in float, |det| <= |n| |d| (1 + 7 u) with |d| <= 1 + 3 u,
// so a triangle whose (precomputed, tri_records) |n| is below EPS (1 - 1e-5) can never be hit by such a ray. On the
// BASELINE scenes that is 22 % (dragon stand-in), 23 % (car_boxed), 28 % (two_cars), 81 % (sportscar stand-in) and
// 99.7 % (dragon871k) of the triangles: the wide view built without them serves the unit-direction walks, the
// full one the primary rays (whose directions are not normalised, main.c:229-233).
// Primary rays are not normalised (main.c:229-233): a launch whose primary directions are all at most PRIMARY_D
// long (the reference camera's are 1.87-2.77) walks a view without the triangles no such direction can hit.
constexpr double UNIT_KEEP = 1.0 - 1e-5;  // x EPSILON (1e-3f, raytracer.c:19)
constexpr double PRIMARY_D = 3.0;
// can a direction of length <= dmax hit the triangle (|n| >= EPSILON (1 - 1e-5) / dmax)?
bool hittable(const rt_triangle& t, double dmax) {
    const rt_vec3 &a = t.coords[0], &b = t.coords[1], &c = t.coords[2];  // n as tri_records forms it
    const float e1x = b.x - a.x, e1y = b.y - a.y, e1z = b.z - a.z;
    const float e2x = c.x - a.x, e2y = c.y - a.y, e2z = c.z - a.z;
    const float nx = e1y * e2z - e1z * e2y, ny = e1z * e2x - e1x * e2z, nz = e1x * e2y - e1y * e2x;
    return std::sqrt((double)nx * nx + (double)ny * ny + (double)nz * nz) >= UNIT_KEEP * (double)rtd::EPS / dmax;
}

// Upper bound on |d| of every primary ray of a frame, d = ((ul - pos) + inc_x * fx) + inc_y * fy for
// fx in [0, W], fy in [0, H] (main.c:229-233; spp samples stay inside their pixel): |d| is convex in (fx, fy), so
// its maximum is at a corner; the float evaluation adds at most a few ulp of the terms' magnitudes (1e-5 of them
// here, ~80x that).
double primary_dmax(const rt_camera* c, int W, int H) {
    const double bx = (double)c->ul.x - c->pos.x, by = (double)c->ul.y - c->pos.y, bz = (double)c->ul.z - c->pos.z;
    double m = 0.0;
    for (int cx = 0; cx < 2; cx++)
        for (int cy = 0; cy < 2; cy++) {
            const double x = cx ? W : 0, y = cy ? H : 0;
            const double dx = bx + c->inc_x.x * x + c->inc_y.x * y, dy = by + c->inc_x.y * x + c->inc_y.y * y,
                         dz = bz + c->inc_x.z * x + c->inc_y.z * y;
            m = std::max(m, std::sqrt(dx * dx + dy * dy + dz * dz));
        }
    const double terms = std::sqrt(bx * bx + by * by + bz * bz) +
                         W * std::sqrt((double)c->inc_x.x * c->inc_x.x + (double)c->inc_x.y * c->inc_x.y +
                                       (double)c->inc_x.z * c->inc_x.z) +
                         H * std::sqrt((double)c->inc_y.x * c->inc_y.x + (double)c->inc_y.y * c->inc_y.y +
                                       (double)c->inc_y.z * c->inc_y.z);
    return m * (1.0 + 1e-5) + 1e-5 * terms;
}

// The 8-wide quantised view of a triangle set, built as the full view was (`method`: RT_ACCEL_GPU = PLOC on the
// device, else the host binned SAH), same inflation and node price. RT_E_STATE: none (too deep for the wide walk).
int wide_view(rt_ctx* ctx, const rt_triangle* T, int n, int method, int R, float inflate, float cnode,
              std::vector<float4>& wn, std::vector<float4>& wt, std::vector<int>& wo, int& depth) {
    rt_bvh_node* nodes = nullptr;
    int nlen = 0;
    int* idx = nullptr;
    std::vector<rt_bvh_node> gnodes;
    std::vector<int> gidx;
    bool gpu = false;
    if (method == RT_ACCEL_GPU) {
        int gdepth = 0;
        const int rc = gpu_ploc(ctx, T, n, R, gnodes, gidx, gdepth);
        if (rc == RT_E_HIP) return rc;
        gpu = rc == RT_OK;
    }
    if (gpu) {
        nodes = gnodes.data();
        nlen = (int)gnodes.size();
        idx = gidx.data();
    } else if (rth_bvh_build(T, (size_t)n, RTH_BVH_BINNED_SAH, nullptr, &nodes, &nlen, &idx, nullptr) != RT_OK) {
        return RT_E_STATE;
    }
    uint32_t* words = nullptr;
    int* order = nullptr;
    rth_wbvh_info wi{};
    int rc = RT_E_STATE;
    const auto t_c = std::chrono::steady_clock::now();
    const bool wide_ok = rth_wbvh_build_cost(nodes, nlen, idx, T, n, inflate, cnode, &words, &order, &wi) == RT_OK;
    ctx->t_collapse += std::chrono::duration<float, std::milli>(std::chrono::steady_clock::now() - t_c).count();
    if (wide_ok && wi.depth <= rtd::WSTACK) {
        wn.resize(5 * (size_t)wi.n_nodes);
        std::memcpy(wn.data(), words, sizeof(uint32_t) * 20 * (size_t)wi.n_nodes);
        tri_records(T, order, n, wt, wo);
        depth = wi.depth;
        rc = RT_OK;
    }
    rth_free(words);
    rth_free(order);
    if (!gpu) {
        rth_free(nodes);
        rth_free(idx);
    }
    return rc;
}
}  // namespace

extern "C" int rt_upload_scene(rt_ctx* ctx, const rt_scene* sc) {
    if (!ctx) return RT_E_ARG;
    if (!sc || !sc->triangles || !sc->bvh || !sc->tri_idx || sc->n_triangles <= 0 || sc->n_nodes <= 0)
        return arg_err(ctx, "rt_upload_scene: empty scene or missing bvh");
    if (sc->n_lights < 0 || (sc->n_lights > 0 && !sc->lights)) return arg_err(ctx, "rt_upload_scene: bad lights");
    if (sc->accel < RT_ACCEL_AUTO || sc->accel > RT_ACCEL_HOST) return arg_err(ctx, "rt_upload_scene: bad accel");
    HIPC(hipSetDevice(ctx->device));
    const int n = sc->n_triangles;
    HostView hr, ha;
    std::vector<float4> wide_nodes, wide_tris;
    std::vector<int> wide_orig;
    int wide_depth = 0;
    int rc = build_view(ctx, sc->bvh, sc->n_nodes, sc->tri_idx, sc->triangles, n, 0.0f, hr);
    if (rc) return rc;
    // the reference tree's child-box faces per axis, sorted (rtd::DScene::faces), uploaded with the scene below
    std::vector<float> faces[3], all_faces;
    for (size_t r = 0; r + 3 < hr.nodes.size(); r += 4) {  // node record: L.min, L.max, R.min, R.max (build_view)
        const float4 p = hr.nodes[r], q = hr.nodes[r + 1], e = hr.nodes[r + 2];
        const float fx[4] = {p.x, p.w, q.z, e.y}, fy[4] = {p.y, q.x, q.w, e.z}, fz[4] = {p.z, q.y, e.x, e.w};
        for (int k = 0; k < 4; k++) {
            faces[0].push_back(fx[k]);
            faces[1].push_back(fy[k]);
            faces[2].push_back(fz[k]);
        }
    }
    for (int a = 0; a < 3; a++) {
        std::sort(faces[a].begin(), faces[a].end());
        faces[a].erase(std::unique(faces[a].begin(), faces[a].end()), faces[a].end());
        all_faces.insert(all_faces.end(), faces[a].begin(), faces[a].end());
    }
    bool own_acc = sc->accel != RT_ACCEL_REFERENCE;
    int built = sc->accel == RT_ACCEL_REFERENCE ? RT_ACCEL_REFERENCE : RT_ACCEL_HOST;
    float gpu_ms = 0.0f;
    ctx->t_ploc = ctx->t_treelet = ctx->t_collapse = 0.0f;
    const auto t_build = std::chrono::steady_clock::now();
    std::vector<rt_bvh_node> gnodes;
    std::vector<int> gidx;
    // The default (AUTO) is the GPU build: measured same box, 16-frame batches, the PLOC tree collapsed to 8-wide
    // renders faster than the host binned SAH's (dragon 0.847 vs 0.911 ms per frame, dragon871k 0.588 vs 0.640,
    // sportscar 1.370 vs 1.435) and builds in 58 vs 86 ms (dragon; 444 vs 883 ms at 871k triangles)
    if (sc->accel == RT_ACCEL_GPU || sc->accel == RT_ACCEL_AUTO) {  // PLOC on the device; its binary tree is not traversed
        int gdepth = 0;
        const auto t0 = std::chrono::steady_clock::now();
        const int R = sc->ploc_radius > 0 ? std::min(sc->ploc_radius, rtb::PLOC_R_MAX) : rtb::PLOC_R;
        rc = gpu_ploc(ctx, sc->triangles, n, R, gnodes, gidx, gdepth);
        gpu_ms = std::chrono::duration<float, std::milli>(std::chrono::steady_clock::now() - t0).count();
        if (rc == RT_E_HIP) return rc;
        if (rc == RT_OK) built = RT_ACCEL_GPU;
        rc = RT_OK;
    }
    if (own_acc) {
        // the fast walk's BVH: binned SAH over the same triangles (librt_host.so), boxes inflated by
        // 2^-16 of the scene's coordinate magnitude (>= 20x the slab tests' rounding reach); or the GPU-built tree
        rt_bvh_node* nodes = nullptr;
        int nlen = 0;
        int* idx = nullptr;
        if (built == RT_ACCEL_GPU) {
            nodes = (rt_bvh_node*)std::malloc(sizeof(rt_bvh_node) * gnodes.size());
            idx = (int*)std::malloc(sizeof(int) * gidx.size());
            if (!nodes || !idx) {
                std::free(nodes);
                std::free(idx);
                return arg_err(ctx, "rt_upload_scene: out of host memory");
            }
            std::memcpy(nodes, gnodes.data(), sizeof(rt_bvh_node) * gnodes.size());
            std::memcpy(idx, gidx.data(), sizeof(int) * gidx.size());
            nlen = (int)gnodes.size();
        } else if (rth_bvh_build(sc->triangles, (size_t)n, RTH_BVH_BINNED_SAH, nullptr, &nodes, &nlen, &idx, nullptr) != RT_OK) {
            return arg_err(ctx, "rt_upload_scene: acceleration BVH build failed");
        }
        float mx = 16.0f;
        for (int i = 0; i < n; i++)
            for (const rt_vec3& c : sc->triangles[i].coords)
                mx = std::max(mx, std::max(std::fabs(c.x), std::max(std::fabs(c.y), std::fabs(c.z))));
        const float inflate = std::ldexp(mx, -16);
        // the binary fast walk's view (used only without a wide view): not for a GPU-built tree, whose depth is
        // not bounded by the binary walks' 34-entry stack (the reference tree serves instead)
        if (built != RT_ACCEL_GPU) rc = build_view(ctx, nodes, nlen, idx, sc->triangles, n, inflate, ha);
        // ... and its 8-wide quantised form (same inflation, planes rounded outward)
        uint32_t* words = nullptr;
        int* order = nullptr;
        rth_wbvh_info wi{};
        const auto t_c = std::chrono::steady_clock::now();
        const bool wide_ok = !rc && rth_wbvh_build_cost(nodes, nlen, idx, sc->triangles, n, inflate,
                                                        sc->collapse_node_cost, &words, &order, &wi) == RT_OK;
        ctx->t_collapse += std::chrono::duration<float, std::milli>(std::chrono::steady_clock::now() - t_c).count();
        if (wide_ok && wi.depth <= rtd::WSTACK) {
            wide_nodes.resize(5 * (size_t)wi.n_nodes);
            std::memcpy(wide_nodes.data(), words, sizeof(uint32_t) * 20 * (size_t)wi.n_nodes);
            tri_records(sc->triangles, order, n, wide_tris, wide_orig);
            wide_depth = wi.depth;
        }
        rth_free(words);
        rth_free(order);
        if (built == RT_ACCEL_GPU) {
            std::free(nodes);
            std::free(idx);
        } else {
            rth_free(nodes);
            rth_free(idx);
        }
        if (rc) return rc;
        if (built == RT_ACCEL_GPU && wide_nodes.empty()) {  // too deep for the wide walk's stack: host build instead
            rt_scene s2 = *sc;
            s2.accel = RT_ACCEL_HOST;
            const int r2 = rt_upload_scene(ctx, &s2);
            if (r2 == RT_OK) ctx->info.gpu_build_ms = gpu_ms;
            return r2;
        }
        own_acc = built != RT_ACCEL_GPU;  // (no binary acceleration view for a GPU-built tree)
    }
    // the unit-direction view (reflection and shadow rays): the same build over the triangles such a ray can hit
    std::vector<float4> unit_nodes, unit_tris;
    std::vector<int> unit_orig;
    int unit_depth = 0, unit_tris_n = 0;
    if (!wide_nodes.empty()) {
        std::vector<rt_triangle> sub;
        std::vector<int> sub_id;
        for (int i = 0; i < n; i++)
            if (hittable(sc->triangles[i], 1.0)) {
                sub.push_back(sc->triangles[i]);
                sub_id.push_back(i);
            }
        if (!sub.empty() && (int)sub.size() < n) {
            float mx = 16.0f;  // the full view's inflation (all triangles' coordinate magnitude)
            for (int i = 0; i < n; i++)
                for (const rt_vec3& c : sc->triangles[i].coords)
                    mx = std::max(mx, std::max(std::fabs(c.x), std::max(std::fabs(c.y), std::fabs(c.z))));
            const int R = sc->ploc_radius > 0 ? std::min(sc->ploc_radius, rtb::PLOC_R_MAX) : rtb::PLOC_R;
            rc = wide_view(ctx, sub.data(), (int)sub.size(), built, R, std::ldexp(mx, -16), sc->collapse_node_cost,
                           unit_nodes, unit_tris, unit_orig, unit_depth);
            if (rc == RT_E_HIP) return rc;
            if (rc == RT_OK) {
                for (int& o : unit_orig) o = sub_id[o];  // subset position -> original triangle index
                unit_tris_n = (int)sub.size();
            } else {  // no usable view: the full one serves every ray
                unit_nodes.clear();
                unit_tris.clear();
                unit_orig.clear();
                unit_depth = 0;
            }
            rc = RT_OK;
        }
    }
    // the primary view: the same build over the triangles a direction of length <= PRIMARY_D can hit (only when
    // that leaves out at least 2 % of them)
    std::vector<float4> prim_nodes, prim_tris;
    std::vector<int> prim_orig;
    int prim_depth = 0, prim_tris_n = 0;
    if (!wide_nodes.empty()) {
        std::vector<rt_triangle> sub;
        std::vector<int> sub_id;
        for (int i = 0; i < n; i++)
            if (hittable(sc->triangles[i], PRIMARY_D)) {
                sub.push_back(sc->triangles[i]);
                sub_id.push_back(i);
            }
        if (!sub.empty() && sub.size() < (size_t)n - (size_t)n / 50) {
            float mx = 16.0f;
            for (int i = 0; i < n; i++)
                for (const rt_vec3& c : sc->triangles[i].coords)
                    mx = std::max(mx, std::max(std::fabs(c.x), std::max(std::fabs(c.y), std::fabs(c.z))));
            const int R = sc->ploc_radius > 0 ? std::min(sc->ploc_radius, rtb::PLOC_R_MAX) : rtb::PLOC_R;
            rc = wide_view(ctx, sub.data(), (int)sub.size(), built, R, std::ldexp(mx, -16), sc->collapse_node_cost,
                           prim_nodes, prim_tris, prim_orig, prim_depth);
            if (rc == RT_E_HIP) return rc;
            if (rc == RT_OK) {
                for (int& o : prim_orig) o = sub_id[o];
                prim_tris_n = (int)sub.size();
            } else {
                prim_nodes.clear();
                prim_tris.clear();
                prim_orig.clear();
                prim_depth = 0;
            }
            rc = RT_OK;
        }
    }
    const float build_ms = std::chrono::duration<float, std::milli>(std::chrono::steady_clock::now() - t_build).count();
    // materials: distinct (ks, kd, kr) triples of triangle_t (the reference stores them per triangle)
    std::unordered_map<std::string, int> mat_id;
    std::vector<float4> mats;
    std::vector<float4> shade(2 * (size_t)n);
    for (int i = 0; i < n; i++) {
        const rt_triangle& t = sc->triangles[i];
        std::string key((const char*)&t.ks, 36);
        auto it = mat_id.find(key);
        int m;
        if (it == mat_id.end()) {
            m = (int)(mats.size() / 3);
            mat_id.emplace(key, m);
            mats.push_back(make_float4(t.ks.x, t.ks.y, t.ks.z, 0.0f));
            mats.push_back(make_float4(t.kd.x, t.kd.y, t.kd.z, 0.0f));
            mats.push_back(make_float4(t.kr.x, t.kr.y, t.kr.z, 0.0f));
        } else {
            m = it->second;
        }
        shade[2 * i + 0] = make_float4(t.norm[0].x, t.norm[0].y, t.norm[0].z, i2f(m));
        shade[2 * i + 1] = make_float4(t.norm[1].x, t.norm[1].y, t.norm[1].z, 0.0f);
    }
    std::vector<float4> lights(2 * (size_t)sc->n_lights);
    for (int j = 0; j < sc->n_lights; j++) {
        const rt_light& l = sc->lights[j];
        lights[2 * j] = make_float4(l.pos.x, l.pos.y, l.pos.z, 0.0f);
        lights[2 * j + 1] = make_float4(l.kl.x, l.kl.y, l.kl.z, 0.0f);
    }
    free_scene(ctx);
    if ((rc = upload_view(ctx, hr, ctx->ref)) || (own_acc && (rc = upload_view(ctx, ha, ctx->acc))) ||
        (rc = upload(ctx, &ctx->d_shade, shade)) || (rc = upload(ctx, &ctx->d_mats, mats)) ||
        (rc = upload(ctx, &ctx->d_lights, lights)) || (rc = upload(ctx, &ctx->d_faces, all_faces)) ||
        (!wide_nodes.empty() && ((rc = upload(ctx, &ctx->wide_nodes, wide_nodes)) ||
                                 (rc = upload(ctx, &ctx->wide_tris, wide_tris)) ||
                                 (rc = upload(ctx, &ctx->wide_orig, wide_orig)))) ||
        (!unit_nodes.empty() && ((rc = upload(ctx, &ctx->unit_nodes, unit_nodes)) ||
                                 (rc = upload(ctx, &ctx->unit_tris, unit_tris)) ||
                                 (rc = upload(ctx, &ctx->unit_orig, unit_orig)))) ||
        (!prim_nodes.empty() && ((rc = upload(ctx, &ctx->prim_nodes, prim_nodes)) ||
                                 (rc = upload(ctx, &ctx->prim_tris, prim_tris)) ||
                                 (rc = upload(ctx, &ctx->prim_orig, prim_orig))))) {
        free_scene(ctx);
        return rc;
    }
    for (int a = 0; a < 3; a++) ctx->faces[a].swap(faces[a]);
    ctx->wide_n = (int)(wide_nodes.size() / 5);
    ctx->wide_depth = wide_depth;
    ctx->unit_n = (int)(unit_nodes.size() / 5);
    ctx->unit_depth = unit_depth;
    ctx->unit_tris_n = unit_nodes.empty() ? 0 : unit_tris_n;
    ctx->prim_n = (int)(prim_nodes.size() / 5);
    ctx->prim_depth = prim_depth;
    ctx->prim_tris_n = prim_nodes.empty() ? 0 : prim_tris_n;
    ctx->n_lights = sc->n_lights;
    ctx->n_tris = n;
    ctx->pk_ok = std::max(ctx->wide_n, std::max(ctx->unit_n, ctx->prim_n)) <= rtd::WIDE_MAX_NODES &&
                 !(ctx->flags & RT_FLAG_UNPACKED_STACK);
    ctx->tq_ok = n < rtd::TQ_MAX_TRIS && !(ctx->flags & RT_FLAG_UNPACKED_TRIS);
    ctx->amb[0] = sc->amb.x;
    ctx->amb[1] = sc->amb.y;
    ctx->amb[2] = sc->amb.z;
    ctx->has_scene = true;
    ctx->scene_gen++;
    ctx->info = rt_scene_info{};
    ctx->info.n_triangles = n;
    ctx->info.n_lights = sc->n_lights;
    ctx->info.wide_nodes = ctx->wide_n;
    ctx->info.wide_depth = wide_depth;
    ctx->info.unit_triangles = ctx->unit_tris_n;
    ctx->info.unit_nodes = ctx->unit_n;
    ctx->info.unit_depth = unit_depth;
    ctx->info.primary_triangles = ctx->prim_tris_n;
    ctx->info.primary_nodes = ctx->prim_n;
    ctx->info.accel_built = built;
    ctx->info.build_ms = build_ms;
    ctx->info.gpu_build_ms = gpu_ms;
    ctx->info.ploc_ms = ctx->t_ploc;
    ctx->info.treelet_ms = ctx->t_treelet;
    ctx->info.collapse_ms = ctx->t_collapse;
    return RT_OK;
}

extern "C" int rt_get_scene_info(rt_ctx* ctx, rt_scene_info* info) {
    if (!ctx || !info) return RT_E_ARG;
    if (!ctx->has_scene) {
        ctx->err = "rt_get_scene_info: no scene uploaded";
        return RT_E_STATE;
    }
    *info = ctx->info;
    return RT_OK;
}

namespace {

// resident workgroups per CU of a persistent kernel (occupancy API, capped at 8)
template <class K>
int resident(K kernel, int device, int cap = 8, size_t dyn_lds = 0, int block = rtd::BLOCK) {
    if (cap <= 0) cap = 8;
    int per_cu = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kernel, block, dyn_lds) != hipSuccess || per_cu < 1)
        per_cu = 1;
    int cus = 256;
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device);
    return std::max(1, std::min(per_cu, cap)) * cus;
}

// The persistent kernels run their frame-batch builds for single frames too: with KArgs::cams null a BATCH kernel
// takes its one camera from the kernel arguments (rt_kernels.hpp cam_of), so one instantiation serves both.
using KFn = void (*)(rtd::KArgs);

// the 4-wave k_persist instantiation of a launch: path buffer in LDS (pbl) or global memory, the spp = 1 build,
// counters; SHP: the per-wave shadow pool (rt_shpool.hpp; 1: one pool per level, 2: one for all levels), which needs
// the LDS path buffer
template <int MAXB, int SHP>
KFn persist4(bool pbl, bool spp1, bool count) {
    using rtd::k_persist;
    if (pbl) {
        if (spp1) return count ? k_persist<MAXB, false, true, true, 4, false, true, 2, true, true, SHP>
                               : k_persist<MAXB, false, false, true, 4, false, true, 2, true, true, SHP>;
        return count ? k_persist<MAXB, false, true, true, 4, false, true, 2, true, false, SHP>
                     : k_persist<MAXB, false, false, true, 4, false, true, 2, true, false, SHP>;
    }
    if constexpr (!SHP) {  // (deep trees: the LDS holds no path buffer next to the stack)
        if (spp1) return count ? k_persist<MAXB, false, true, true, 4, false, true, 1, false, true>
                               : k_persist<MAXB, false, false, true, 4, false, true, 1, false, true>;
        return count ? k_persist<MAXB, false, true, true, 4, false, true, 1, false, false>
                     : k_persist<MAXB, false, false, true, 4, false, true, 1, false, false>;
    }
    return nullptr;
}

// the spp > 1 sample-sum slots of an LDS-path-buffer launch (one float4 per lane, after the rest of its layout)
size_t slot_bytes(const rtd::KArgs& A) { return A.spp > 1 ? sizeof(float4) * rtd::BLOCK : 0; }
// the kernel arguments of a launch with `dyn` bytes of dynamic LDS: its slots' offset (ints) when it has them
rtd::KArgs with_slots(const rtd::KArgs& A, size_t dyn) {
    rtd::KArgs B = A;
    B.slot_off = dyn && slot_bytes(A) ? (int)((dyn - slot_bytes(A)) / sizeof(int)) : -1;
    return B;
}

// dynamic LDS of the 4-wave kernels' LDS layout: the wide stack sized to the scene's wide depth, then the path levels
// (and, for the all-levels pool, each level's hit triangle)
// (and, for spp > 1, the lanes' sample-sum slots at the end: rtd::KArgs::slot_off)
template <int MAXB>
size_t pbl_bytes(const rtd::KArgs& A, int shp = 0) {
    return sizeof(int) * (size_t)rtd::wstack_words(A.wcap, shp > 0) * rtd::BLOCK + sizeof(float4) * rtd::BLOCK * MAXB +
           (shp == 2 ? sizeof(int) * (rtd::BLOCK * MAXB + rtd::BLOCK / 64 * rtd::TQ_WORDS) : 0) +
           (shp == 1 || shp == 3 ? sizeof(int) * (rtd::BLOCK / 64 * rtd::TQ_WORDS) : 0) + slot_bytes(A);
}
// Does that layout fit 4 workgroups per CU for this scene? (the LDS path buffer measured 1.2 % faster than the global
// slab on dragon, 2.3 % on car_boxed; the shadow pool needs it)
template <int MAXB>
bool pbl_fits(const rtd::KArgs& A, int device, int shp = 0) {
    if (!A.gstack || A.wcap <= 0) return false;
    (void)device;
    int per_cu = 0;
    return hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, persist4<MAXB, 0>(true, true, false), rtd::BLOCK,
                                                        pbl_bytes<MAXB>(A, shp)) == hipSuccess &&
           per_cu >= 4;
}

// k_persist (the persistent one-lane-per-path kernel) in configuration `variant`, and its dynamic LDS:
//   RT_VARIANT_PERSIST   <= 168 VGPRs (3 waves per SIMD), path levels in registers (spp = 1: packed triangle tests);
//   RT_VARIANT_PERSIST4  <= 128 VGPRs (4 waves per SIMD), path levels in a path buffer: in LDS after the wide stack
//                        (packed stack entries and triangle tests, SHP = 3) when 4 workgroups of that fit a CU, else
//                        a global slab;
//   RT_VARIANT_SHPOOL    PERSIST4 with each bounce level's shadow rays walked as a per-wave pool (rt_shpool.hpp);
//                        PERSIST4 where the LDS path buffer does not fit;
//   RT_VARIANT_SHDEFER   PERSIST4 with every level's shadow rays walked as ONE per-wave pool after the closest hits
//                        (the path buffer plus a hit-triangle array in LDS; else PERSIST4);
// a tile trace (A.tile_trace: the hybrid launch's measuring frame, PRT_TILE_TRACE) runs the 3-wave build with
// per-tile timestamps.
template <int MAXB>
KFn persist_kernel(const rtd::KArgs& A, int variant, bool count, int device, size_t& dyn, bool pk_ok, bool tq_ok,
                   unsigned* build = nullptr) {
    dyn = 0;
    unsigned bd = 0;  // rt_launch_info.build of the instantiation returned (RT_BUILD_*)
    struct Report {
        unsigned* out;
        unsigned& v;
        ~Report() {
            if (out) *out = v;
        }
    } report{build, bd};
    // (the k_persist builds are made either for spp = 1 (SPP1) or for spp > 1 only: each launch takes the one its spp
    // needs; a tile trace -- the hybrid rule's measuring frame, PRT_TILE_TRACE -- is single-sample)
    if (A.tile_trace) {
        bd = RT_BUILD_TRACE;
        return count ? rtd::k_persist<MAXB, false, true, true, 3, true, true, 0, false, true>
                     : rtd::k_persist<MAXB, false, false, true, 3, true, true, 0, false, true>;
    }
    if ((variant == RT_VARIANT_SHPOOL || variant == RT_VARIANT_SHDEFER) && pk_ok && tq_ok) {
        const int shp = variant == RT_VARIANT_SHDEFER ? 2 : 1;
        if (pbl_fits<MAXB>(A, device, shp)) {
            dyn = pbl_bytes<MAXB>(A, shp);
            bd = RT_BUILD_WAVES4 | RT_BUILD_PACKED_STACK | RT_BUILD_PACKED_TRIS | RT_BUILD_LDS_PATHS |
                 (shp == 2 ? RT_BUILD_POOL_ALL : RT_BUILD_POOL_LEVEL);
            return shp == 2 ? persist4<MAXB, 2>(true, A.spp <= 1, count) : persist4<MAXB, 1>(true, A.spp <= 1, count);
        }
    }
    // PERSIST4 with packed stack entries and packed triangle tests (SHP = 3) where its LDS fits: sportscar 20-frame
    // batches 0.922 -> 0.895 ms per frame, car_boxed 0.860 -> 0.841; car_boxed 4K at 64 spp 194.3 -> 191.6 ms per
    // frame although that build spills 144 B (same box)
    if ((variant == RT_VARIANT_PERSIST4 || variant == RT_VARIANT_SHPOOL || variant == RT_VARIANT_SHDEFER) && pk_ok &&
        tq_ok && pbl_fits<MAXB>(A, device, 3)) {
        dyn = pbl_bytes<MAXB>(A, 3);
        bd = RT_BUILD_WAVES4 | RT_BUILD_PACKED_STACK | RT_BUILD_PACKED_TRIS | RT_BUILD_LDS_PATHS;
        return persist4<MAXB, 3>(true, A.spp <= 1, count);
    }
    if (variant == RT_VARIANT_PERSIST4 || variant == RT_VARIANT_SHPOOL || variant == RT_VARIANT_SHDEFER) {
        const bool pbl = pbl_fits<MAXB>(A, device);
        if (pbl) dyn = pbl_bytes<MAXB>(A);
        bd = RT_BUILD_WAVES4 | (pbl ? RT_BUILD_LDS_PATHS : 0u);
        // (the bench's batches: the spp = 1 build)
        return persist4<MAXB, 0>(pbl, A.spp <= 1, count);
    }
    // the 3-wave kernel's spp = 1 build with packed triangle tests (queues in static LDS): same box, single frames
    // dragon 1.27 -> 1.16 ms, sportscar 2.40 -> 2.29, car_boxed 1.96 -> 1.84; the default rule's single frames (its
    // cold tiles) sportscar 1.708 -> 1.671, car_boxed 1.210 -> 1.183
    if (A.spp <= 1 && tq_ok) {
        bd = RT_BUILD_PACKED_TRIS;
        return count ? rtd::k_persist<MAXB, false, true, true, 3, false, true, 0, false, true, 3>
                     : rtd::k_persist<MAXB, false, false, true, 3, false, true, 0, false, true, 3>;
    }
    if (A.spp <= 1)  // (scenes past the packed tests' triangle bound)
        return count ? rtd::k_persist<MAXB, false, true, true, 3, false, true, 0, false, true>
                     : rtd::k_persist<MAXB, false, false, true, 3, false, true, 0, false, true>;
    return count ? rtd::k_persist<MAXB, false, true, true, 3, false, true> : rtd::k_persist<MAXB, false, false, true, 3, false, true>;
}

// `cap`: workgroups per CU at most (0: the occupancy limit); the grid never exceeds the tiles / 4.
template <int MAXB>
void launch_paths(const rtd::KArgs& A, int variant, bool count, int device, hipStream_t s, int cap, bool pk_ok,
                  bool tq_ok, unsigned* build = nullptr) {
    size_t dyn = 0;
    const KFn k = persist_kernel<MAXB>(A, variant, count, device, dyn, pk_ok, tq_ok, build);
    const int blocks = std::max(1, std::min(resident(k, device, cap > 0 ? cap : 8, dyn), (A.n_tiles * A.n_frames + 3) / 4));
    k<<<blocks, rtd::BLOCK, dyn, s>>>(with_slots(A, dyn));
}

rtd::DBvh dview(const DevView& v) { return rtd::DBvh{v.nodes, v.leaves, v.tris, v.orig, v.root}; }

// k_coop (rt_coop.hpp): G = 2 or 4 lanes per ray; one wave per tile of 64 / G pixels
template <int MAXB>
KFn coop_kernel(int G, bool count) {
    using rtd::k_coop;
    if (G == 2) return count ? k_coop<MAXB, true, 2, 3, false, true> : k_coop<MAXB, false, 2, 3, false, true>;
    return count ? k_coop<MAXB, true, 4, 3, false, true> : k_coop<MAXB, false, 4, 3, false, true>;
}
// never more workgroups than tiles / 4
template <int MAXB>
int launch_group(const rtd::KArgs& A, int g, bool count, int device, hipStream_t s, int cap) {
    const KFn k = coop_kernel<MAXB>(g, count);
    const int blocks = std::max(1, std::min(resident(k, device, cap), (A.n_tiles * A.n_frames + 3) / 4));
    k<<<blocks, rtd::BLOCK, 0, s>>>(A);
    return RT_OK;
}

}  // namespace

namespace {
// Centre-out order of a tx x ty tile grid (the persistent kernels' default dealing order), by runs of SUPER tiles
// side by side in a row: an 8x8 tile of 4-B pixels stores 32-B row pieces, so SUPER = 4 neighbouring tiles fill
// whole 128-B lines, and dealt back to back they are written while the line is still in the XCD's L2 (a line
// left partly written leaves L2 once per piece: WRITE_SIZE).
constexpr int SUPER = 4;
std::vector<int> centre_out(int tx, int ty) {
    const int n = tx * ty;
    std::vector<int> ord(n);
    for (int i = 0; i < n; i++) ord[i] = i;
    const float cx = 0.5f * tx, cy = 0.5f * ty;
    auto d2 = [&](int t) {
        const int x0 = (t % tx) / SUPER * SUPER, x1 = std::min(tx, x0 + SUPER);
        const float dx = 0.5f * (x0 + x1) - cx, dy = t / tx + 0.5f - cy;
        return dx * dx + dy * dy;
    };
    std::stable_sort(ord.begin(), ord.end(), [&](int a, int b) {
        const float da = d2(a), db = d2(b);
        if (da != db) return da < db;
        return a / tx != b / tx ? a / tx < b / tx : a < b;  // a run's tiles together, left to right
    });
    return ord;
}

// XCD-aware layout of a dealing order (rtd::next_item): 9 region offsets into the tile part, then the tiles of
// region 0..7, each region in the order's order. mode 1: 8 bands of tile rows, 2: 8 bands of tile columns,
// 3: 4 x 2 blocks.
std::vector<int> region_layout(const std::vector<int>& ord, int tx, int ty, int mode) {
    std::vector<int> dev(9 + ord.size());
    int at = 9;
    for (int r = 0; r < 8; r++) {
        dev[r] = at;
        for (int t : ord) {
            const int reg = mode == 1 ? (t / tx) * 8 / ty : mode == 2 ? (t % tx) * 8 / tx
                                                                    : (t % tx) * 4 / tx + 4 * ((t / tx) * 2 / ty);
            if (reg == r) dev[at++] = t;
        }
    }
    dev[8] = at;
    for (int r = 0; r <= 8; r++) dev[r] -= 9;  // offsets into the order part
    return dev;
}

template <int MAXB>
int launch_hybrid(rt_ctx* ctx, const rtd::KArgs& A, bool count, int c, unsigned* build = nullptr);  // below
template <int MAXB>
int launch_hybrid_fb(rt_ctx* ctx, const rtd::KArgs& A, bool count, int c, unsigned* build);  // below

// A frame batch's cameras to d_cams when they differ from the set it holds. The copy runs in stream order (after the
// renders in flight, which read the old set) from a ring of pinned slots; only a slot whose previous copy has not
// run yet -- CAM_SLOTS camera sets in flight -- makes the host wait.
int upload_cams(rt_ctx* ctx, const rt_camera* cams, int n_frames) {
    static_assert(sizeof(rt_camera) == 48, "rt_camera = 4 x rt_vec3");
    const size_t nf = 12 * (size_t)n_frames;
    if ((int)ctx->cams_last.size() == (int)nf && std::memcmp(ctx->cams_last.data(), cams, sizeof(float) * nf) == 0)
        return RT_OK;
    if (ctx->cams_cap < n_frames) {  // (rare: a larger batch; hipFree waits for the device)
        if (ctx->d_cams) HIPC(hipFree(ctx->d_cams));
        if (ctx->h_cams) {
            HIPC(hipStreamSynchronize(ctx->stream));
            HIPC(hipHostFree(ctx->h_cams));
        }
        ctx->d_cams = nullptr;
        ctx->h_cams = nullptr;
        ctx->cams_cap = 0;
        const int cap = std::max(n_frames, 32);
        HIPC(hipMalloc((void**)&ctx->d_cams, sizeof(float) * 12 * cap));
        HIPC(hipHostMalloc((void**)&ctx->h_cams, sizeof(float) * 12 * cap * rt_ctx::CAM_SLOTS, hipHostMallocDefault));
        ctx->cams_cap = cap;
    }
    const int sl = ctx->cam_slot;
    ctx->cam_slot = (sl + 1) % rt_ctx::CAM_SLOTS;
    if (!ctx->cam_ev[sl]) HIPC(hipEventCreateWithFlags(&ctx->cam_ev[sl], hipEventDisableTiming));
    else HIPC(hipEventSynchronize(ctx->cam_ev[sl]));  // done long ago unless CAM_SLOTS sets are in flight
    float* h = ctx->h_cams + (size_t)sl * 12 * ctx->cams_cap;
    std::memcpy(h, cams, sizeof(float) * nf);
    HIPC(hipMemcpyAsync(ctx->d_cams, h, sizeof(float) * nf, hipMemcpyHostToDevice, ctx->stream));
    HIPC(hipEventRecord(ctx->cam_ev[sl], ctx->stream));
    ctx->cams_last.assign(reinterpret_cast<const float*>(cams), reinterpret_cast<const float*>(cams) + nf);
    return RT_OK;
}

// rt_render / rt_render_frames: n_frames frames of the same shape (cameras cams[0..n_frames-1]); outputs
// [n_frames][n_rows][width]... Persistent fast configurations trace the whole batch in ONE launch (frames'
// tiles interleaved in the dealing order); other kernels launch once per frame.
int render_batch(rt_ctx* ctx, const rt_camera* cams, int n_frames, const rt_frame* f, const rt_outputs* out) {
    if (!ctx) return RT_E_ARG;
    if (!ctx->has_scene) {
        ctx->err = "rt_render: no scene uploaded";
        return RT_E_STATE;
    }
    if (!cams || !f) return arg_err(ctx, "rt_render: null camera/frame");
    if (n_frames < 1 || n_frames > 4096) return arg_err(ctx, "rt_render_frames: n_frames must be 1..4096");
    const rt_camera* cam = cams;
    const int rb = f->row_block > 1 ? f->row_block : 1;
    const int fs = f->frame_shift;
    if (f->width <= 0 || f->height <= 0 || f->row_stride <= 0 || f->n_rows <= 0 || f->row_offset < 0 ||
        f->row_block < 0 || fs < 0 || (f->n_rows > rb && f->row_stride < rb) ||
        (fs == 0 && (long long)f->row_offset + (long long)((f->n_rows - 1) / rb) * f->row_stride +
                            (f->n_rows - 1) % rb >= f->height) ||
        (fs > 0 && (f->row_offset >= f->row_stride || f->row_offset >= f->height ||
                    (long long)f->n_rows > (long long)f->row_stride * f->height)))
        return arg_err(ctx, "rt_render: rows outside the frame");
    if (fs > 0 && f->kernel != RT_KERNEL_FAST && f->kernel != RT_KERNEL_AUTO)
        return arg_err(ctx, "rt_render: frame_shift needs RT_KERNEL_FAST");
    if (f->bounces < 1 || f->bounces > 8) return arg_err(ctx, "rt_render: bounces must be 1..8");
    int g = 1;
    while (g * g < f->spp) g++;
    if (f->spp < 1 || g * g != f->spp || g > 16) return arg_err(ctx, "rt_render: spp must be a square 1..256");
    if (f->kernel < RT_KERNEL_AUTO || f->kernel > RT_KERNEL_FAST) return arg_err(ctx, "rt_render: bad kernel");
    if (f->spp > 1 && (f->width > 65535 || f->n_rows > 65535))  // (k_persist's multi-sample slots pack x and the row)
        return arg_err(ctx, "rt_render: spp > 1 frames are at most 65535 pixels wide and 65535 rows high");
    // (variants 3, 6, 7, 8, 9, 10, 12, 14 -- the split pipeline, k_coop<8>, k_fan, k_chain, k_pool, k_relay, k_stream
    // -- measured slower than k_persist and were removed: refused)
    const bool known = f->variant == RT_VARIANT_DEFAULT || f->variant == RT_VARIANT_PERSIST ||
                       f->variant == RT_VARIANT_PERSIST4 || f->variant == RT_VARIANT_COOP2 ||
                       f->variant == RT_VARIANT_COOP4 || f->variant == RT_VARIANT_HYBRID ||
                       f->variant == RT_VARIANT_SHPOOL || f->variant == RT_VARIANT_SHDEFER;
    if (!known || f->hot_pct < 0 || f->hot_pct > 100 || f->hot_kernel < RT_HOT_COOP4 || f->hot_kernel > RT_HOT_COOP2 ||
        f->tune < 0 || f->tune > 1 ||
        f->waves_cap < 0 || f->waves_cap > 8 || f->dealing < RT_DEAL_DEFAULT || f->dealing > RT_DEAL_ROW_MAJOR ||
        f->regroup < 0 || f->regroup > 64)
        return arg_err(ctx, "rt_render: bad launch configuration (variant / tune / waves_cap / dealing / regroup)");
    HIPC(hipSetDevice(ctx->device));
    const size_t pixels = (size_t)f->width * f->n_rows;  // per frame
    const size_t all_px = pixels * (size_t)n_frames;
    if (all_px > (size_t)INT_MAX)  // (the kernels index a launch's output pixels with 32-bit integers)
        return arg_err(ctx, "rt_render: the launch's frames x pixels exceed 2^31 - 1");
    float* rgb = out ? out->rgb : nullptr;
    unsigned* bgra = out ? out->bgra : nullptr;
    if (!rgb && !bgra) {  // a quantised-only frame writes no f32 pixels at all
        if (ctx->rgb_cap < all_px) {
            if (ctx->d_rgb_own) HIPC(hipFree(ctx->d_rgb_own));
            ctx->d_rgb_own = nullptr;
            ctx->rgb_cap = 0;
            HIPC(hipMalloc((void**)&ctx->d_rgb_own, sizeof(float) * 3 * all_px));
            ctx->rgb_cap = all_px;
        }
        rgb = ctx->d_rgb_own;
    }
    rtd::KArgs A;
    std::memset(&A, 0, sizeof A);
    A.s.ref = dview(ctx->ref);
    A.s.acc = ctx->acc.nodes ? dview(ctx->acc) : A.s.ref;
    A.s.wide = rtd::DWide{ctx->wide_nodes, ctx->wide_tris, ctx->wide_orig, ctx->wide_n};
    A.s.unit = rtd::DWide{ctx->unit_nodes, ctx->unit_tris, ctx->unit_orig, ctx->unit_n};
    // the primary view when every primary direction of every frame of the launch is short enough for it
    bool prim_ok = ctx->prim_nodes != nullptr;
    for (int i = 0; i < n_frames && prim_ok; i++) prim_ok = primary_dmax(cams + i, f->width, f->height) <= PRIMARY_D;
    if (prim_ok) A.s.prim = rtd::DWide{ctx->prim_nodes, ctx->prim_tris, ctx->prim_orig, ctx->prim_n};
    A.s.shade = ctx->d_shade;
    A.s.mats = ctx->d_mats;
    A.s.lights = ctx->d_lights;
    A.s.n_lights = ctx->n_lights;
    A.s.amb_x = ctx->amb[0];
    A.s.amb_y = ctx->amb[1];
    A.s.amb_z = ctx->amb[2];
    A.s.faces = ctx->d_faces;  // (rt_kernels.hpp degenerate_ok)
    A.s.ref_path = ctx->ref.path;  // (rt_kernels.hpp ref_reaches)
    A.s.n_tris = ctx->n_tris;
    for (int a = 0; a < 3; a++) A.s.n_face[a] = (int)ctx->faces[a].size();
    const rt_vec3* cv[4] = {&cam->pos, &cam->ul, &cam->inc_x, &cam->inc_y};
    float* dst[4] = {A.pos, A.ul, A.ix, A.iy};
    for (int i = 0; i < 4; i++) {
        dst[i][0] = cv[i]->x;
        dst[i][1] = cv[i]->y;
        dst[i][2] = cv[i]->z;
    }
    A.W = f->width;
    A.H = f->height;
    A.row_offset = f->row_offset;
    A.row_stride = f->row_stride;
    A.row_block = rb;
    A.frame_shift = fs;
    A.n_rows = f->n_rows;
    A.bounces = f->bounces;
    A.spp = f->spp;
    A.spp_grid = g;
    A.rgb = rgb;
    A.bgra = bgra;
    A.hit = out ? out->hit : nullptr;
    A.t = out ? out->t : nullptr;
    A.bounce_hit = out ? out->bounce_hit : nullptr;
    A.counters = ctx->d_counters;
    A.work = ctx->d_work;
    A.tiles_x = (f->width + 7) / 8;
    A.n_tiles = A.tiles_x * ((f->n_rows + 7) / 8);
    A.tiles_x8 = A.tiles_x;
    const int kernel = f->kernel == RT_KERNEL_AUTO ? RT_KERNEL_FAST : f->kernel;
    if (n_frames > 1 && kernel != RT_KERNEL_FAST) {  // one launch per frame, outputs at frame offsets
        for (int i = 0; i < n_frames; i++) {
            rt_outputs o{rgb ? rgb + 3 * pixels * i : nullptr, A.hit ? A.hit + pixels * i : nullptr,
                         A.t ? A.t + pixels * i : nullptr,
                         A.bounce_hit ? A.bounce_hit + pixels * f->bounces * i : nullptr,
                         bgra ? bgra + pixels * i : nullptr};
            ctx->batch_sum = i > 0;
            const int rc = render_batch(ctx, cams + i, 1, f, &o);
            ctx->batch_sum = false;
            if (rc) return rc;
        }
        ctx->last_rgb = rgb;
        ctx->last_bgra = bgra;
        ctx->last_hit = A.hit;
        ctx->last_pixels = all_px;
        ctx->last_frames = n_frames;
        return RT_OK;
    }
    A.n_frames = n_frames;
    A.frame_px = pixels;
    if (kernel == RT_KERNEL_FAST && (!ctx->d_pathbuf || !ctx->d_gstack || !ctx->d_lanebuf)) {
        // (each buffer its own check: a failed allocation of one of them leaves the others, and the next render
        // retries the missing one instead of launching with a null buffer)
        int cus = 256;
        (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, ctx->device);
        const size_t waves = (size_t)cus * 8 * (rtd::BLOCK / 64);  // <= 8 workgroups per CU (resident() cap)
        // path buffer of the PB kernels: every resident wave, MAXB <= 8 levels
        if (!ctx->d_pathbuf) HIPC(hipMalloc((void**)&ctx->d_pathbuf, sizeof(float4) * waves * 8 * 64));
        // DYN kernels' binary-walk stacks: STACK ints per lane of every resident workgroup (<= 8 per CU)
        if (!ctx->d_gstack) HIPC(hipMalloc((void**)&ctx->d_gstack, sizeof(int) * (size_t)cus * 8 * rtd::STACK * rtd::BLOCK));
        // the multi-sample builds' per-lane slots (the running sum and the pixel between samples): every resident lane
        if (!ctx->d_lanebuf) HIPC(hipMalloc((void**)&ctx->d_lanebuf, sizeof(float4) * (size_t)cus * 8 * rtd::BLOCK));
    }
    A.pathbuf = ctx->d_pathbuf;
    A.lanebuf = ctx->d_lanebuf;
    A.gstack = ctx->d_gstack;
    A.wcap = ctx->wide_n > 0 ? std::max(1, std::max(ctx->wide_depth, std::max(ctx->unit_depth, ctx->prim_depth))) : 0;
    if (n_frames > 1) {  // the batch's cameras, uploaded when they change
        if (int rc = upload_cams(ctx, cams, n_frames)) return rc;
        A.cams = ctx->d_cams;
    }
    A.regroup = f->regroup > 0 ? f->regroup : 16;
    const bool count = (ctx->flags & RT_FLAG_COUNTERS) != 0;
    dim3 grid((f->width + 15) / 16, (f->n_rows + 15) / 16);
    const int slot = (int)(ctx->launches % rt_ctx::NEV);
    ctx->ev0 = ctx->ev0s[slot];
    ctx->ev1 = ctx->ev1s[slot];
    // diagnostics: PRT_TILE_TRACE=<file> writes 4 x uint64 per tile of a k_persist frame (rt_kernels.hpp)
    // (s_memrealtime, 100 MHz); synchronous, never used by tests or the bench
    const char* trace_path = std::getenv("PRT_TILE_TRACE");
    unsigned long long* d_trace = nullptr;
    const size_t trace_n = (size_t)A.n_tiles;
    if (trace_path && kernel == RT_KERNEL_FAST && n_frames == 1 && f->spp == 1) {
        HIPC(hipMalloc((void**)&d_trace, sizeof(unsigned long long) * 4 * trace_n));
        HIPC(hipMemsetAsync(d_trace, 0, sizeof(unsigned long long) * 4 * trace_n, ctx->stream));
        A.tile_trace = d_trace;
    }
    // Tile dealing order of the persistent kernels: centre-out (default). The frame ends when the slowest
    // tile does (PRT_TILE_TRACE: 8x8 tiles range from 2 us to ~1.9 ms; expensive ones are deep reflection
    // chains, usually on the object in view); dealing from the centre starts them first (bench frame
    // -7 %). RT_DEAL_ROW_MAJOR: row-major. One cached permutation per tile grid.
    const bool dealt_centre_out = kernel == RT_KERNEL_FAST && f->dealing != RT_DEAL_ROW_MAJOR;
    auto order_for = [&](int tx, int ty, const int*& out_ord) -> int {
        out_ord = nullptr;
        if (!dealt_centre_out) return RT_OK;
        const long long key = ((long long)tx << 32) | (unsigned)ty;
        auto it = ctx->orders.find(key);
        if (it != ctx->orders.end()) {
            out_ord = it->second;
            return RT_OK;
        }
        const std::vector<int> ord = centre_out(tx, ty);
        int* d = nullptr;
        HIPC(hipMalloc((void**)&d, sizeof(int) * ord.size()));
        HIPC(hipMemcpy(d, ord.data(), sizeof(int) * ord.size(), hipMemcpyHostToDevice));
        ctx->orders[key] = d;
        out_ord = d;
        return RT_OK;
    };
    if (int rc = order_for(A.tiles_x, A.n_tiles / A.tiles_x, A.tile_order)) return rc;
    // XCD-aware dealing of k_persist: the centre-out order split into 8 spatial regions, region r drained first by
    // the workgroups on XCD r (rtd::next_item), so each XCD's L2 holds the part of the scene its region's rays
    // touch. rt_frame.dealing: BLOCKS = 4 x 2 blocks of tiles, ROWS = 8 bands of tile rows, COLUMNS = 8 bands of
    // tile columns, GLOBAL = one counter. Same-box, ms per frame: 16-frame batches of the full frame, dragon 1.060
    // (global) / 0.938 (blocks) / 0.980 (rows) / 0.942 (columns), sportscar 0.599 / 0.504, car_boxed 1.067 / 1.041;
    // a single frame 1.862 / 1.871 (blocks) / 1.732 (rows); an 8-GPU rank's rows, batched, 0.220 / 0.208 (blocks) /
    // 0.202 (rows). Default: blocks for batches of the full frame, row bands otherwise. Device layout: 9 region
    // offsets, then the concatenated regions' tiles.
    const int* region_off = nullptr;
    const int* region_order = nullptr;
    const bool full_frame = f->row_offset == 0 && f->n_rows == f->height;
    const int xcd_mode = f->dealing == RT_DEAL_DEFAULT ? (n_frames > 1 && full_frame ? 3 : 1)
                         : f->dealing == RT_DEAL_ROWS    ? 1
                         : f->dealing == RT_DEAL_COLUMNS ? 2
                         : f->dealing == RT_DEAL_BLOCKS  ? 3
                                                         : 0;
    auto regions_for = [&](int tx, int ty, const int*& roff, const int*& rord) -> int {
        roff = rord = nullptr;
        if (!(dealt_centre_out && xcd_mode >= 1 && xcd_mode <= 3)) return RT_OK;
        const long long key = ((long long)xcd_mode << 58) | ((long long)tx << 32) | (unsigned)ty;
        auto it = ctx->orders.find(key);
        if (it == ctx->orders.end()) {
            const std::vector<int> dev = region_layout(centre_out(tx, ty), tx, ty, xcd_mode);
            int* d = nullptr;
            HIPC(hipMalloc((void**)&d, sizeof(int) * dev.size()));
            HIPC(hipMemcpy(d, dev.data(), sizeof(int) * dev.size(), hipMemcpyHostToDevice));
            it = ctx->orders.emplace(key, d).first;
        }
        roff = it->second;
        rord = it->second + 9;
        return RT_OK;
    };
    if (int rc = regions_for(A.tiles_x, A.n_tiles / A.tiles_x, region_off, region_order)) return rc;
    // RT_KERNEL_FAST launch configurations (rt_frame.variant; every one renders the same bits):
    //   PERSIST / PERSIST4  k_persist, one lane per pixel path, walks in lockstep, 8x8 tiles;
    //   SHPOOL              k_persist at 4 waves with each level's shadow rays walked as a per-wave pool;
    //   COOP2/4             k_coop (rt_coop.hpp): G lanes per ray, 64/G-pixel tiles — shorter chains per tile,
    //                       which is what a frame split over many GPUs (few tiles per wave) is bound by;
    //   HYBRID              single frames: the costliest tiles through k_coop on a second stream (§3e).
    const bool wide_ok = kernel == RT_KERNEL_FAST && ctx->wide_n > 0;
    // the shadow pool: 1..32 lights (a 32-bit visibility word per pixel) and the LDS path buffer at 4 workgroups per CU
    const bool shp_ok = wide_ok && ctx->n_lights >= 1 && ctx->n_lights <= 32 && ctx->pk_ok && ctx->tq_ok &&
                        (f->bounces <= 4 ? pbl_fits<4>(A, ctx->device, 1) : pbl_fits<8>(A, ctx->device, 1));
    const bool shd_ok = shp_ok && ctx->n_lights <= 8 && (f->bounces <= 4 ? pbl_fits<4>(A, ctx->device, 2) : pbl_fits<8>(A, ctx->device, 2));
    auto usable = [&](int v) {
        if (A.tile_trace) return v == RT_VARIANT_PERSIST;  // (diagnostics: the 3-wave kernel's tile trace)
        if (v == RT_VARIANT_COOP2 || v == RT_VARIANT_COOP4) return wide_ok;
        if (v == RT_VARIANT_SHPOOL) return shp_ok;
        if (v == RT_VARIANT_SHDEFER) return shd_ok;
        if (v == RT_VARIANT_HYBRID) return wide_ok && n_frames == 1 && fs == 0 && f->spp == 1;
        return true;
    };
    // The default rule (measured): frame batches and spp > 1 fill the chip, so the kernel with the best
    // throughput — the shadow pool for scenes of 2+ lights whose LDS path buffer fits (dragon 0.708 -> 0.666 ms per
    // frame in 20-frame batches; one light leaves nothing to pool: car_boxed 0.868 vs 0.902), else k_persist at 4
    // waves; a single 1-spp frame is tail-bound: the hybrid launch, which measures its candidates on the frames of
    // the shape and keeps the fastest (k_persist where it cannot run).
    const bool pool_rule = shp_ok && ctx->n_lights >= 2;
    // the pool kernel of the rules: one pool for all levels where its larger LDS path buffer fits (dragon 20-frame
    // batches 0.655 -> 0.639 ms per frame, single frames 1.145 -> 1.091 ms; SIMD efficiency 0.59 -> 0.68), else one
    // per level
    const int pool_v = shd_ok ? RT_VARIANT_SHDEFER : RT_VARIANT_SHPOOL;
    int mode = f->variant;
    if (mode == RT_VARIANT_DEFAULT)
        mode = (n_frames > 1 || f->spp > 1) ? (pool_rule ? pool_v : RT_VARIANT_PERSIST4) : RT_VARIANT_HYBRID;
    if ((mode == RT_VARIANT_SHPOOL && !shp_ok) || (mode == RT_VARIANT_SHDEFER && !shd_ok))
        mode = RT_VARIANT_PERSIST4;  // (no room for the pool: PERSIST4 itself)
    if (!usable(mode)) mode = RT_VARIANT_PERSIST;  // (no wide view, or a diagnostics trace)
    // the whole-frame kernel of a single frame while the hybrid launch measures or tries its candidates
    const int single_rule = pool_rule ? pool_v : RT_VARIANT_PERSIST;
    const int cap = f->waves_cap;
    rt_launch_info li{};  // what this render runs (rt_get_launch_info)
    li.settled = 1;
    // The default rule for frame batches and spp > 1 where the shadow pool can run: measured, not guessed. Whether the
    // pool pays depends on the scene (dragon 20-frame batches 0.708 -> 0.666 ms per frame; two_cars 4K 1.881 vs 1.917,
    // car_boxed 0.868 vs 0.902), so the first launches of a shape try PERSIST4 and SHPOOL ROUNDS times each (their own
    // HIP events, read by a query once the last has run) and the faster per frame renders from then on. A context with
    // traversal counters never tries (the counters of a trial would be another kernel's): it keeps the static rule.
    if (f->variant == RT_VARIANT_DEFAULT && kernel == RT_KERNEL_FAST && !A.tile_trace && !count &&
        (n_frames > 1 || f->spp > 1) && shp_ok) {
        rt_ctx::BatchRule* br = nullptr;
        for (auto& b : ctx->brules)
            if (b.scene == ctx->scene_gen && b.W == f->width && b.rows == f->n_rows && b.off == f->row_offset &&
                b.stride == f->row_stride && b.block == rb && b.shift == fs && b.bounces == f->bounces &&
                b.spp == f->spp && b.frames == n_frames && b.dealing == f->dealing && b.cap_req == f->waves_cap)
                br = &b;
        if (!br) {
            if (ctx->brules.size() >= 16) ctx->brules.erase(ctx->brules.begin());
            ctx->brules.emplace_back();
            br = &ctx->brules.back();
            *br = rt_ctx::BatchRule{ctx->scene_gen, f->width, f->n_rows, f->row_offset, f->row_stride, rb, fs,
                                     f->bounces, f->spp, n_frames, f->dealing, f->waves_cap};
        }
        rt_ctx::BatchRule& b = *br;
        const int cand[2] = {RT_VARIANT_PERSIST4, pool_v};
        const int nc = 2;
        int pick = -1;
        if (b.choice < 0) {
            for (int r = 0; r < rt_ctx::BatchRule::ROUNDS && pick < 0; r++)
                for (int c = 0; c < nc && pick < 0; c++)
                    if (b.launch[c][r] < 0 || ctx->launches - b.launch[c][r] >= rt_ctx::NEV) {  // untried (or events reused)
                        b.launch[c][r] = ctx->launches;
                        pick = c;
                    }
            if (pick < 0) {  // every trial enqueued: decide once the last has run (a query, never a wait)
                long long last = 0;
                for (int c = 0; c < nc; c++)
                    for (long long x : b.launch[c]) last = std::max(last, x);
                const hipError_t q = hipEventQuery(ctx->ev1s[last % rt_ctx::NEV]);
                if (q == hipSuccess) {
                    float ms[2] = {1e30f, 1e30f};
                    constexpr int R = rt_ctx::BatchRule::ROUNDS;
                    float t[2][R];
                    float med_max = 0.0f;
                    for (int c = 0; c < nc; c++) {
                        for (int r = 0; r < R; r++) {
                            const int sl = (int)(b.launch[c][r] % rt_ctx::NEV);
                            HIPC(hipEventElapsedTime(&t[c][r], ctx->ev0s[sl], ctx->ev1s[sl]));
                        }
                        std::sort(t[c], t[c] + R);
                        med_max = std::max(med_max, t[c][R / 2]);
                    }
                    // one statistic for every candidate (like with like): the median when the launches are long
                    // (some candidate's median over LONG_MS), else the minimum
                    const bool by_median = med_max > rt_ctx::BatchRule::LONG_MS;
                    for (int c = 0; c < nc; c++) ms[c] = by_median ? t[c][R / 2] : t[c][0];
                    b.choice = 0;
                    for (int c = 1; c < nc; c++)
                        if (ms[c] < ms[b.choice]) b.choice = c;
                    if (const char* l = std::getenv("PRT_TUNE_LOG"); l && std::atoi(l) == 1)
                        std::fprintf(stderr, "[prt batch] %dx%d f%d spp%d: persist4 %.3f ms, %s %.3f ms -> %s\n",
                                     f->width, f->n_rows, n_frames, f->spp, ms[0], variant_name(cand[1]), ms[1],
                                     variant_name(cand[b.choice]));
                } else if (q != hipErrorNotReady) {
                    return fail(ctx, q, "rt_render: batch rule trials");
                } else {
                    (void)hipGetLastError();  // not an error: the trials are still running
                }
            }
        }
        if (b.choice >= 0) {
            mode = cand[b.choice];
        } else {
            mode = pick >= 0 ? cand[pick] : (pool_rule ? pool_v : RT_VARIANT_PERSIST4);
            li.trial = 1;
            li.settled = 0;
        }
    }
    // RT_VARIANT_HYBRID: what this single frame runs. The state is keyed by the frame's SHAPE, not its camera (a
    // walkthrough moves it every frame). The first frame of a shape measures: k_persist with per-tile times, copied to
    // pinned host memory behind it. Once they have arrived (an event query, never a wait) the tile lists of every
    // candidate are built and copied in stream order, and the next frames try the candidates ROUNDS times each,
    // timed by their own HIP events; when the last trial has finished (a query) the fastest minimum renders from then
    // on (PRT_TUNE_LOG=1 prints them). Every REFRESH frames of the shape a measuring frame renews the tile lists for
    // a moving camera (the choice stays). While a measurement or the trials are in flight, a frame runs the static
    // rule's whole-frame kernel. rt_frame.hot_pct > 0 fixes the threshold (no trials).
    // kind 0: measuring frame; 1: whole-frame variant c; 2: hybrid candidate c's launch (lists at ctx->hy)
    struct Pick {
        int kind, c;
    };
    auto hybrid_pick = [&](int& rc) -> Pick {
        rt_ctx::Hybrid& h = ctx->hy;
        const bool same = h.scene == ctx->scene_gen && h.W == f->width && h.rows == f->n_rows && h.off == f->row_offset &&
                          h.stride == f->row_stride && h.block == rb && h.bounces == f->bounces &&
                          h.dealing == f->dealing && h.pct_req == f->hot_pct && h.hk_req == f->hot_kernel;
        auto err = [&](hipError_t e, const char* what) { rc = fail(ctx, e, what); return Pick{1, single_rule}; };
        auto in_flight = [&](hipEvent_t e, bool& done) -> hipError_t {  // query, never wait
            const hipError_t q = hipEventQuery(e);
            done = q == hipSuccess;
            if (q == hipErrorNotReady) {
                (void)hipGetLastError();  // not an error: still running
                return hipSuccess;
            }
            return q;
        };
        if (!h.ev) {
            hipError_t e = hipEventCreateWithFlags(&h.ev, hipEventDisableTiming);
            if (e == hipSuccess) e = hipEventCreateWithFlags(&h.fork, hipEventDisableTiming);
            if (e == hipSuccess) e = hipEventCreateWithFlags(&h.join, hipEventDisableTiming);
            if (e == hipSuccess) e = hipStreamCreateWithFlags(&h.s2, hipStreamNonBlocking);
            if (e != hipSuccess) return err(e, "rt_render: hybrid events / stream");
        }
        // a decided shape's frames -- its periodic refresh (a measuring frame, li.refresh) and the frames while that
        // measurement is in flight included -- are the rule's steady state (settled); a new shape's are trials
        const bool decided = same && h.choice >= 0;
        li.settled = decided ? 1 : 0;
        li.trial = decided ? 0 : 1;
        if (!same) {  // a new shape: measure it, once an earlier measurement in flight has landed in h_tr
            if (h.state == 1) {
                bool done = false;
                if (hipError_t e = in_flight(h.ev, done); e != hipSuccess) return err(e, "rt_render: hybrid measurement");
                if (!done) return Pick{1, single_rule};
            }
            h.scene = ctx->scene_gen;
            h.W = f->width;
            h.rows = f->n_rows;
            h.off = f->row_offset;
            h.stride = f->row_stride;
            h.block = rb;
            h.bounces = f->bounces;
            h.dealing = f->dealing;
            h.pct_req = f->hot_pct;
            h.hk_req = f->hot_kernel;
            h.choice = -1;
            h.n_tiles = (size_t)A.n_tiles;
            if (h.tr_cap < h.n_tiles) {  // (no measurement in flight writes h_tr now)
                if (h.d_tr) (void)hipFree(h.d_tr);
                if (h.h_tr) (void)hipHostFree(h.h_tr);
                h.d_tr = h.h_tr = nullptr;
                h.tr_cap = 0;
                hipError_t e = hipMalloc((void**)&h.d_tr, sizeof(unsigned long long) * 4 * h.n_tiles);
                if (e == hipSuccess) e = hipHostMalloc((void**)&h.h_tr, sizeof(unsigned long long) * 4 * h.n_tiles,
                                                       hipHostMallocDefault);
                if (e != hipSuccess) return err(e, "rt_render: hybrid tile times");
                h.tr_cap = h.n_tiles;
            }
            if (h.fb_cap < h.n_tiles) {  // the feedback's buffers (rt_feedback.hpp); no frame of the old shape runs now
                if (h.fb_pending) (void)hipEventSynchronize(h.fb_ev);
                if (h.d_cost) (void)hipFree(h.d_cost);
                if (h.d_fb) (void)hipFree(h.d_fb);
                if (h.d_info) (void)hipFree(h.d_info);
                h.d_cost = nullptr;
                h.d_fb = nullptr;
                h.d_info = nullptr;
                h.fb_cap = 0;
                hipError_t e = hipMalloc((void**)&h.d_cost, sizeof(unsigned) * 2 * (h.n_tiles + 1));
                if (e == hipSuccess) e = hipMalloc((void**)&h.d_fb, sizeof(int) * (5 * h.n_tiles + 13 + rtd::FB_G * (rtd::FB_TK + 3)));
                if (e == hipSuccess) e = hipMalloc((void**)&h.d_info, h.n_tiles);
                if (e == hipSuccess && !h.h_fb_cnt) e = hipHostMalloc((void**)&h.h_fb_cnt, sizeof(int) * 4, hipHostMallocDefault);
                if (e == hipSuccess && !h.fb_ev) e = hipEventCreateWithFlags(&h.fb_ev, hipEventDisableTiming);
                if (e != hipSuccess) return err(e, "rt_render: hybrid feedback buffers");
                h.fb_cap = h.n_tiles;
            }
            h.fb_ok = false;
            h.fb_cam_ok = false;
            h.fb_hot_est = -1;
            h.info_mode = -1;
            h.state = 0;
        }
        // renew a decided shape's lists with a measuring frame every REFRESH frames -- unless its frames feed their own
        // tile times forward (PRT_FEEDBACK), which keeps the lists one frame old
        if (!PRT_FEEDBACK && h.state == 2 && h.choice >= 0 && ++h.frames >= rt_ctx::Hybrid::REFRESH) h.state = 0;
        if (h.state == 0) return Pick{0, 0};
        if (h.state == 1) {
            bool done = false;
            if (hipError_t e = in_flight(h.ev, done); e != hipSuccess) return err(e, "rt_render: hybrid measurement");
            if (!done) return Pick{1, h.choice >= 0 && h.pct[h.choice] == 0 ? h.cold[h.choice] : single_rule};
            // the tile lists of every candidate threshold: [hot tiles][cold 8x8 tiles], one after another
            const int tx = A.tiles_x, ty = A.n_tiles / A.tiles_x;
            std::vector<long long> dur(h.n_tiles);
            long long cmax = 1, dsum = 0;
            for (size_t t = 0; t < h.n_tiles; t++) {
                dur[t] = (long long)(h.h_tr[4 * t + 1] - h.h_tr[4 * t]);
                cmax = std::max(cmax, dur[t]);
                dsum += dur[t];
            }
            std::vector<int> ord = centre_out(tx, ty);
            if (!dealt_centre_out)
                for (int t = 0; t < (int)ord.size(); t++) ord[t] = t;  // RT_DEAL_ROW_MAJOR
            h.cold_regions = xcd_mode >= 1 && xcd_mode <= 3 && dealt_centre_out;
            h.cold_mode = h.cold_regions ? xcd_mode : 0;
            const bool keep = h.choice >= 0;  // a refresh: new lists, the same candidates and choice
            if (!keep) {
                h.nc = 0;
                auto add = [&](int pct, int lanes, int cold, bool lpt) {
                    if (cold == RT_VARIANT_SHPOOL) cold = pool_v;  // (HYBRID_CANDS: "the pool kernel")
                    if (h.nc >= rt_ctx::Hybrid::NCAND || !usable(cold)) return;
                    h.pct[h.nc] = pct;
                    h.lanes[h.nc] = lanes;
                    h.lpt[h.nc] = lpt;
                    h.cold[h.nc++] = cold;
                };
                if (f->hot_pct > 0) {
                    add(f->hot_pct, f->hot_kernel == RT_HOT_COOP2 ? 2 : 4, RT_VARIANT_PERSIST, false);
                } else {
                    for (const HotCand& hc : HYBRID_CANDS) add(hc.pct, hc.lanes, hc.cold, hc.lpt);
                }
            }
            std::vector<int> lists;
            for (int c = 0; c < h.nc; c++) {
                h.at[c] = lists.size();
                h.n_hot[c] = h.n_cold[c] = 0;
                if (h.pct[c] == 0 && !h.lpt[c]) continue;
                std::vector<int> hot8;
                for (size_t t = 0; t < h.n_tiles && h.pct[c] > 0; t++)
                    if (dur[t] * 100 > (long long)h.pct[c] * cmax && dur[t] * (long long)h.n_tiles > 2 * dsum)
                        hot8.push_back((int)t);  // (and over twice the mean: rt_feedback.hpp fb_tile)
                std::stable_sort(hot8.begin(), hot8.end(), [&](int a, int b) { return dur[a] > dur[b]; });
                if (hot8.size() > h.n_tiles / 2) hot8.resize(h.n_tiles / 2);  // k_coop costs ~2x the wave time
                std::vector<char> is_hot(h.n_tiles, 0);
                // each 8x8 tile = (8 / TW) x (8 / TH) tiles of the hot kernel (rtd::GTile), hottest first
                int tw, th;
                hot_tile(h.lanes[c], tw, th);
                const int ctw = (f->width + tw - 1) / tw, cth = (f->n_rows + th - 1) / th;
                for (int t : hot8) {
                    is_hot[t] = 1;
                    for (int qy = 0; qy < 8 / th; qy++)
                        for (int qx = 0; qx < 8 / tw; qx++) {
                            const int cx = (t % tx) * (8 / tw) + qx, cy = (t / tx) * (8 / th) + qy;
                            if (cx < ctw && cy < cth) lists.push_back(cy * ctw + cx);
                        }
                }
                h.n_hot[c] = (int)(lists.size() - h.at[c]);
                std::vector<int> cold;
                for (int t : ord)
                    if (!is_hot[t]) cold.push_back(t);
                if (h.lpt[c])  // costliest first (ties: centre-out)
                    std::stable_sort(cold.begin(), cold.end(), [&](int a, int b) { return dur[a] > dur[b]; });
                h.n_cold[c] = (int)cold.size();
                if (h.cold_regions) cold = region_layout(cold, tx, ty, xcd_mode);
                lists.insert(lists.end(), cold.begin(), cold.end());
            }
            if (!lists.empty()) {
                // pinned staging: the last copy out of it ran before the measuring frame (stream order), which has
                // finished; the device copy is stream-ordered after every frame that read the old lists
                if (h.hl_cap < lists.size()) {
                    if (h.h_lists) (void)hipHostFree(h.h_lists);
                    h.h_lists = nullptr;
                    h.hl_cap = 0;
                    const hipError_t e = hipHostMalloc((void**)&h.h_lists, sizeof(int) * lists.size(), hipHostMallocDefault);
                    if (e != hipSuccess) return err(e, "rt_render: hybrid lists");
                    h.hl_cap = lists.size();
                }
                if (h.lists_cap < lists.size()) {  // (rare: a new shape; hipFree waits for the device)
                    if (h.d_lists) (void)hipFree(h.d_lists);
                    h.d_lists = nullptr;
                    h.lists_cap = 0;
                    const hipError_t e = hipMalloc((void**)&h.d_lists, sizeof(int) * lists.size());
                    if (e != hipSuccess) return err(e, "rt_render: hybrid lists");
                    h.lists_cap = lists.size();
                }
                std::memcpy(h.h_lists, lists.data(), sizeof(int) * lists.size());
                const hipError_t e = hipMemcpyAsync(h.d_lists, h.h_lists, sizeof(int) * lists.size(),
                                                    hipMemcpyHostToDevice, ctx->stream);
                if (e != hipSuccess) return err(e, "rt_render: hybrid lists");
            }
            if (!keep) {
                for (int c = 0; c < h.nc; c++)
                    for (int r = 0; r < rt_ctx::Hybrid::ROUNDS; r++) h.launch[c][r] = -1;
                h.choice = h.nc == 1 ? 0 : -1;
            }
            h.frames = 0;
            h.state = 2;
        }
        auto pick_of = [&](int c) { return h.pct[c] == 0 && !h.lpt[c] ? Pick{1, h.cold[c]} : Pick{2, c}; };
        if (h.choice >= 0) {
            li.settled = 1;
            li.trial = 0;
            return pick_of(h.choice);
        }
        for (int c = 0; c < h.nc; c++)
            for (int r = 0; r < rt_ctx::Hybrid::ROUNDS; r++)
                if (h.launch[c][r] < 0 || ctx->launches - h.launch[c][r] >= rt_ctx::NEV) {  // untried (or events reused)
                    h.launch[c][r] = ctx->launches;
                    return pick_of(c);
                }
        long long last = 0;
        for (int c = 0; c < h.nc; c++)
            for (int r = 0; r < rt_ctx::Hybrid::ROUNDS; r++) last = std::max(last, h.launch[c][r]);
        bool done = false;
        if (hipError_t e = in_flight(ctx->ev1s[last % rt_ctx::NEV], done); e != hipSuccess) return err(e, "rt_render: hybrid trials");
        if (!done) return Pick{1, single_rule};  // the trials are still running
        int best = 0;
        for (int c = 0; c < h.nc; c++) {
            constexpr int W = rt_ctx::Hybrid::WARM, NT = rt_ctx::Hybrid::ROUNDS - W;
            float t[NT];
            for (int r = 0; r < NT; r++) {
                const int sl = (int)(h.launch[c][W + r] % rt_ctx::NEV);
                const hipError_t e = hipEventElapsedTime(&t[r], ctx->ev0s[sl], ctx->ev1s[sl]);
                if (e != hipSuccess) return err(e, "rt_render: hybrid trials");
            }
            std::sort(t, t + NT);
            h.ms[c] = t[NT / 2];  // the median of the timed trials
            if (h.ms[c] < h.ms[best]) best = c;
        }
        h.choice = best;
        h.frames = 0;
        if (const char* l = std::getenv("PRT_TUNE_LOG"); l && std::atoi(l) == 1) {
            std::fprintf(stderr, "[prt hybrid] %dx%d b%d:", f->width, f->n_rows, f->bounces);
            for (int c = 0; c < h.nc; c++)
                std::fprintf(stderr, " %s%d/coop%d/%s%s %.3f ms", h.pct[c] ? "hot>" : "whole", h.pct[c], h.lanes[c],
                             variant_name(h.cold[c]), h.lpt[c] ? "/lpt" : "", h.ms[c]);
            std::fprintf(stderr, " -> %d\n", best);
        }
        li.settled = 1;
        li.trial = 0;
        return pick_of(best);
    };
    // one frame of configuration (variant, cap); d_work holds the persistent grids' work counters, and the
    // ray counters restart with every launch (rt_get_stats reports the frame, not the trial launches)
    auto dispatch = [&](int md, int cp) -> int {
        auto clear = [&]() -> int {
            if (!ctx->batch_sum)  // a per-frame loop of a batch keeps adding to the batch's counters
                HIPC(hipMemsetAsync(ctx->d_counters, 0, sizeof(unsigned long long) * rtd::NCOUNT, ctx->stream));
            HIPC(hipMemsetAsync(ctx->d_work, 0, 1024, ctx->stream));
            return RT_OK;
        };
        // (a hybrid frame on device-built lists has its list builder clear them instead: after the pick)
        if (!(PRT_FEEDBACK && md == RT_VARIANT_HYBRID))
            if (int rc = clear()) return rc;
        li.variant = md;
        if (kernel == RT_KERNEL_STRICT) {
            li.variant = 0;
            auto k = count ? rtd::k_tiles<4, true, true> : rtd::k_tiles<4, true, false>;
            if (f->bounces > 4) k = count ? rtd::k_tiles<8, true, true> : rtd::k_tiles<8, true, false>;
            k<<<grid, rtd::BLOCK, 0, ctx->stream>>>(A);
            return RT_OK;
        }
        if (md == RT_VARIANT_COOP2 || md == RT_VARIANT_COOP4) {
            rtd::KArgs B = A;
            const int gr = md == RT_VARIANT_COOP2 ? 2 : 4;
            int tw, th;
            hot_tile(gr, tw, th);  // rtd::GTile<gr>
            B.tiles_x = (f->width + tw - 1) / tw;
            const int ty = (f->n_rows + th - 1) / th;
            B.n_tiles = B.tiles_x * ty;
            if (int rc = order_for(B.tiles_x, ty, B.tile_order)) return rc;
            return f->bounces <= 4 ? launch_group<4>(B, gr, count, ctx->device, ctx->stream, cp)
                                   : launch_group<8>(B, gr, count, ctx->device, ctx->stream, cp);
        }
        rtd::KArgs P = A;
        if (region_off) {
            P.region_off = region_off;
            P.tile_order = region_order;
        }
        if (md == RT_VARIANT_HYBRID) {
            int rc = RT_OK;
            const Pick pk = hybrid_pick(rc);
            if (rc) return rc;
            rt_ctx::Hybrid& h = ctx->hy;
            const bool fb = PRT_FEEDBACK && pk.kind == 2 && h.fb_ok && h.d_cost;
            if (PRT_FEEDBACK && !fb)
                if (int rc2 = clear()) return rc2;
            // the frame's HIP-event time starts here, after the host work of the pick (the trials compare them)
            HIPC(hipEventRecord(ctx->ev0, ctx->stream));
            // every frame of the shape records its tiles' durations (rt_feedback.hpp); a hybrid candidate's frame --
            // tried or chosen -- builds its lists from the previous frame's first, on the device (the memset follows
            // that build: k_coop's hot tiles combine their group tiles' times by atomic max). The trials too: with a
            // moving camera the measuring frame's lists age frame by frame, and a candidate tried later would be
            // priced with older lists than one tried first (a car_boxed walkthrough settled on the wrong candidate).
            if (PRT_FEEDBACK && h.d_cost) {
                if (fb) {
                    li.hot_pct = h.pct[pk.c];
                    li.hot_lanes = h.lanes[pk.c];
                    li.cold_variant = h.cold[pk.c];
                    const int r2 = f->bounces <= 4 ? launch_hybrid_fb<4>(ctx, A, count, pk.c, &li.build)
                                                   : launch_hybrid_fb<8>(ctx, A, count, pk.c, &li.build);
                    h.fb_ok = r2 == RT_OK;
                    return r2;
                }
                unsigned* w = h.cost_at(h.cost_cur ^ 1);
                HIPC(hipMemsetAsync(w, 0, sizeof(unsigned) * (h.n_tiles + 1), ctx->stream));
                P.tile_cost = w;
                A.tile_cost = w;
                h.cost_cur ^= 1;
                h.fb_ok = true;  // (this frame, in stream order, fills it)
            }
            if (pk.kind == 2) {
                li.hot_pct = ctx->hy.pct[pk.c];
                li.hot_lanes = ctx->hy.lanes[pk.c];
                li.cold_variant = ctx->hy.cold[pk.c];
                return f->bounces <= 4 ? launch_hybrid<4>(ctx, A, count, pk.c, &li.build)
                                       : launch_hybrid<8>(ctx, A, count, pk.c, &li.build);
            }
            if (pk.kind == 0) {  // measuring frame: k_persist with per-tile times, copied to the host behind it
                li.variant = RT_VARIANT_PERSIST;
                li.refresh = h.choice >= 0 ? 1 : 0;  // a decided shape's periodic list refresh (settled)
                li.trial = li.refresh ? 0 : 1;
                li.settled = li.refresh;
                P.tile_trace = h.d_tr;
                if (f->bounces <= 4) launch_paths<4>(P, RT_VARIANT_PERSIST, count, ctx->device, ctx->stream, cp, ctx->pk_ok, ctx->tq_ok, &li.build);
                else launch_paths<8>(P, RT_VARIANT_PERSIST, count, ctx->device, ctx->stream, cp, ctx->pk_ok, ctx->tq_ok, &li.build);
                HIPC(hipGetLastError());
                HIPC(hipMemcpyAsync(h.h_tr, h.d_tr, sizeof(unsigned long long) * 4 * h.n_tiles, hipMemcpyDeviceToHost,
                                    ctx->stream));
                HIPC(hipEventRecord(h.ev, ctx->stream));
                h.state = 1;
                return RT_OK;
            }
            md = pk.c;  // a whole-frame kernel: chosen, tried, or while the measurement / trials are on their way
            li.variant = md;
        }
        if (f->bounces <= 4) launch_paths<4>(P, md, count, ctx->device, ctx->stream, cp, ctx->pk_ok, ctx->tq_ok, &li.build);
        else launch_paths<8>(P, md, count, ctx->device, ctx->stream, cp, ctx->pk_ok, ctx->tq_ok, &li.build);
        return RT_OK;
    };
    {
        HIPC(hipEventRecord(ctx->ev0, ctx->stream));
        const int rc = dispatch(mode, cap);
        if (rc) return rc;
    }
    HIPC(hipGetLastError());
    HIPC(hipEventRecord(ctx->ev1, ctx->stream));
    if (d_trace) {
        std::vector<unsigned long long> h(4 * trace_n);
        HIPC(hipStreamSynchronize(ctx->stream));
        HIPC(hipMemcpy(h.data(), d_trace, sizeof(unsigned long long) * h.size(), hipMemcpyDeviceToHost));
        HIPC(hipFree(d_trace));
        if (FILE* fp = std::fopen(trace_path, "wb")) {
            std::fwrite(h.data(), sizeof(unsigned long long), h.size(), fp);
            std::fclose(fp);
        }
    }
    ctx->last_launch = li;
    ctx->launches++;
    ctx->last_rgb = rgb;
    ctx->last_bgra = bgra;
    ctx->last_hit = A.hit;
    ctx->last_pixels = all_px;
    ctx->last_frames = n_frames;
    ctx->last_W = f->width;
    ctx->last_H = f->height;
    ctx->last_off = f->row_offset;
    ctx->last_stride = f->row_stride;
    ctx->last_rows = f->n_rows;
    ctx->last_block = rb;
    ctx->last_shift = fs;
    ctx->rendered = true;
    return RT_OK;
}
}  // namespace

extern "C" int rt_render(rt_ctx* ctx, const rt_camera* cam, const rt_frame* f, const rt_outputs* out) {
    return render_batch(ctx, cam, 1, f, out);
}

extern "C" int rt_render_frames(rt_ctx* ctx, const rt_camera* cams, int n_frames, const rt_frame* f,
                                const rt_outputs* out) {
    return render_batch(ctx, cams, n_frames, f, out);
}

extern "C" int rt_get_launch_info(rt_ctx* ctx, rt_launch_info* info) {
    if (!ctx || !info) return RT_E_ARG;
    if (!ctx->rendered) {
        ctx->err = "rt_get_launch_info: nothing rendered";
        return RT_E_STATE;
    }
    *info = ctx->last_launch;
    return RT_OK;
}

namespace {
int comm_settle_ctx(rt_ctx* ctx, const char* who);  // (below, with the communicators)
// Waits for the context stream; with a render behind it, reads that render's error counter (rtd::C_ERR: a traversal
// stack overflowed, rt_kernels.hpp) in the same wait, so that a frame computed with a truncated walk never passes as
// good: RT_E_KERNEL. A stream holding a multi-process gather's send / recv group is first waited for through the
// communicator's bounded wait (comm_settle): a peer that never joins fails the call with RT_E_TIMEOUT instead of
// blocking in hipStreamSynchronize.
int sync_checked(rt_ctx* ctx, const char* who) {
    if (int rc = comm_settle_ctx(ctx, who)) return rc;
    if (ctx->rendered)
        HIPC(hipMemcpyAsync(ctx->h_err, ctx->d_counters + rtd::C_ERR, sizeof(unsigned long long), hipMemcpyDeviceToHost,
                            ctx->stream));
    HIPC(hipStreamSynchronize(ctx->stream));
    if (ctx->rendered && *ctx->h_err) {
        ctx->err = std::string(who) + ": the render's traversal stack overflowed " + std::to_string(*ctx->h_err) +
                   " times (BVH deeper than the walks' stacks): the frame is not valid";
        return RT_E_KERNEL;
    }
    return RT_OK;
}
}  // namespace

extern "C" int rt_sync(rt_ctx* ctx, float* kernel_ms) {
    if (!ctx) return RT_E_ARG;
    HIPC(hipSetDevice(ctx->device));
    if (int rc = sync_checked(ctx, "rt_sync")) return rc;
    if (kernel_ms) {
        *kernel_ms = 0.0f;
        if (ctx->rendered) HIPC(hipEventElapsedTime(kernel_ms, ctx->ev0, ctx->ev1));
    }
    return RT_OK;
}

extern "C" int rt_kernel_times(rt_ctx* ctx, float* ms, int n) {
    if (!ctx || !ms || n < 0) return RT_E_ARG;
    HIPC(hipSetDevice(ctx->device));
    if (int rc = comm_settle_ctx(ctx, "rt_kernel_times")) return rc;
    HIPC(hipStreamSynchronize(ctx->stream));
    long long avail = ctx->launches < rt_ctx::NEV ? ctx->launches : rt_ctx::NEV;
    if (n > avail) n = (int)avail;
    for (int i = 0; i < n; i++) {  // oldest first among the last n launches
        int slot = (int)((ctx->launches - n + i) % rt_ctx::NEV);
        HIPC(hipEventElapsedTime(&ms[i], ctx->ev0s[slot], ctx->ev1s[slot]));
    }
    return n;
}

extern "C" int rt_download(rt_ctx* ctx, float* h_rgb, int* h_hit) {
    if (!ctx) return RT_E_ARG;
    if (!ctx->rendered) {
        ctx->err = "rt_download: nothing rendered";
        return RT_E_STATE;
    }
    HIPC(hipSetDevice(ctx->device));
    if (int rc = sync_checked(ctx, "rt_download")) return rc;
    if (h_rgb && !ctx->last_rgb) {
        ctx->err = "rt_download: last frame was rendered to a bgra output only";
        return RT_E_STATE;
    }
    if (h_rgb)
        HIPC(hipMemcpy(h_rgb, ctx->last_rgb, sizeof(float) * 3 * ctx->last_pixels, hipMemcpyDeviceToHost));
    if (h_hit) {
        if (!ctx->last_hit) {
            ctx->err = "rt_download: last frame had no hit output";
            return RT_E_STATE;
        }
        HIPC(hipMemcpy(h_hit, ctx->last_hit, sizeof(int) * ctx->last_pixels, hipMemcpyDeviceToHost));
    }
    return RT_OK;
}

namespace {
template <class T>
int grow(rt_ctx* ctx, T** p, size_t& cap, size_t n) {
    if (*p && cap >= n) return RT_OK;
    if (*p) HIPC(hipFree(*p));
    *p = nullptr;
    cap = 0;
    HIPC(hipMalloc((void**)p, sizeof(T) * std::max<size_t>(n, 1)));
    cap = n;
    return RT_OK;
}
}  // namespace

namespace {
// RT_VARIANT_HYBRID, one frame: the hot tiles (ctx->hy lists) through k_coop on the context's second stream
// while the cold kernel (k_persist, or the shadow pool) renders the cold 8x8 tiles on the context stream; both
// persistent grids together fill the chip (the hot grid is sized to start every hot tile at once, at most half the
// chip), and the context stream waits for both.
template <int MAXB>
int launch_hybrid(rt_ctx* ctx, const rtd::KArgs& A, bool count, int c, unsigned* build) {
    rt_ctx::Hybrid& h = ctx->hy;
    const int n_hot = h.n_hot[c], n_cold = h.n_cold[c];
    int* lists = h.d_lists + h.at[c];
    const int g = h.lanes[c];
    const KFn kc = coop_kernel<MAXB>(g, count);
    int tw, th;
    hot_tile(g, tw, th);
    rtd::KArgs B = A;  // the hot kernel's tiles, dealt hottest first from their own work counter
    B.tiles_x = (A.W + tw - 1) / tw;
    B.n_tiles = n_hot;
    B.tile_order = lists;
    B.region_off = nullptr;
    B.work = A.work + 224;
    rtd::KArgs P = A;
    P.n_tiles = n_cold;
    P.region_off = h.cold_regions ? lists + n_hot : nullptr;
    P.tile_order = lists + n_hot + (h.cold_regions ? 9 : 0);
    size_t dyn = 0;
    const KFn kp = persist_kernel<MAXB>(P, h.cold[c], count, ctx->device, dyn, ctx->pk_ok, ctx->tq_ok, build);
    const int rp = resident(kp, ctx->device, 8, dyn);
    const int rcp = resident(kc, ctx->device);
    const int nc = n_hot > 0 ? std::max(1, std::min((n_hot + 3) / 4, rcp / 2)) : 0;
    const int np = std::max(1, std::min(rp - (int)((long long)nc * rp / rcp), (n_cold + 3) / 4));
    if (n_hot == 0) {  // (a whole frame in the measured order)
        if (n_cold > 0) kp<<<np, rtd::BLOCK, dyn, ctx->stream>>>(with_slots(P, dyn));
        HIPC(hipGetLastError());
        return RT_OK;
    }
    HIPC(hipEventRecord(h.fork, ctx->stream));  // after the work / counter resets
    HIPC(hipStreamWaitEvent(h.s2, h.fork, 0));
    if (n_hot > 0) kc<<<nc, rtd::BLOCK, 0, h.s2>>>(B);
    HIPC(hipGetLastError());
    if (n_cold > 0) kp<<<np, rtd::BLOCK, dyn, ctx->stream>>>(with_slots(P, dyn));
    HIPC(hipGetLastError());
    HIPC(hipEventRecord(h.join, h.s2));
    HIPC(hipStreamWaitEvent(ctx->stream, h.join, 0));
    return RT_OK;
}

// A decided shape's frame under the per-frame feedback (rt_feedback.hpp): candidate c's lists built on the device from
// the previous frame's tile durations (k_fb_max, k_fb_count, k_fb_place), the durations cleared, then c's kernels as launch_hybrid launches
// them, every one reading its list and count from the device and recording this frame's durations. The grids are sized
// by a recent frame's hot count, read back without a wait.
template <int MAXB>
int launch_hybrid_fb(rt_ctx* ctx, const rtd::KArgs& A, bool count, int c, unsigned* build) {
    rt_ctx::Hybrid& h = ctx->hy;
    const int g = h.lanes[c] == 2 ? 2 : 4;
    const bool hot = h.pct[c] > 0;
    int tw, th;
    hot_tile(g, tw, th);
    const int ctw = (A.W + tw - 1) / tw, cth = (A.n_rows + th - 1) / th;
    int* d_hot = h.d_fb;
    int* d_cold = h.d_fb + 4 * h.n_tiles;
    int* d_cnt = d_cold + 9 + h.n_tiles;
    const int tx = A.tiles_x, ty = A.n_tiles / A.tiles_x;
    if (h.info_mode != h.cold_mode) {  // the shape's per-tile region and hot-kernel tile counts, once
        std::vector<unsigned char> info(h.n_tiles);
        for (int t = 0; t < A.n_tiles; t++) info[t] = rtd::fb_tile_info(t, tx, ty, h.cold_mode, A.W, A.n_rows);
        HIPC(hipMemcpy(h.d_info, info.data(), info.size(), hipMemcpyHostToDevice));
        h.info_mode = h.cold_mode;
    }
    // (hot set: at most half the 8x8 tiles, as the host's lists, counted in hot-kernel tiles)
    // (d_cost holds n_tiles + 1 words: A.n_tiles is this shape's n_tiles, the maximum's word right after the tiles)
    // the last frame's times in, this frame's buffer cleared by k_fb_max (with the frame's counters and work words)
    unsigned* const cost_in = h.cost_at(h.cost_cur);
    unsigned* const cost_out = h.cost_at(h.cost_cur ^ 1);
    rtd::FbArgs F{cost_in, A.n_tiles, tx, ty, h.pct[c], (int)(h.n_tiles / 2) * (8 / tw) * (8 / th), tw, th, ctw, cth, h.cold_mode,
                  h.d_info, d_hot, d_cold, d_cnt, (unsigned*)(d_cnt + 4), (unsigned*)(d_cnt + 4) + rtd::FB_G * rtd::FB_TK, 0,
                  cost_out,
                  ctx->batch_sum ? nullptr : ctx->d_counters, rtd::NCOUNT, ctx->d_work, 1024 / 4};
    {  // the camera against the last feedback frame's (rt_feedback.hpp FbArgs::moved)
        float cam[12];
        std::memcpy(cam, A.pos, sizeof(float) * 3);
        std::memcpy(cam + 3, A.ul, sizeof(float) * 3);
        std::memcpy(cam + 6, A.ix, sizeof(float) * 3);
        std::memcpy(cam + 9, A.iy, sizeof(float) * 3);
        F.moved = h.fb_cam_ok && std::memcmp(cam, h.fb_cam, sizeof cam) != 0;
        std::memcpy(h.fb_cam, cam, sizeof cam);
        h.fb_cam_ok = true;
    }
    rtd::k_fb_max<<<rtd::FB_G, rtd::FB_THREADS, 0, ctx->stream>>>(F);
    rtd::k_fb_count<<<rtd::FB_G, rtd::FB_THREADS, 0, ctx->stream>>>(F);
    rtd::k_fb_place<<<rtd::FB_G, rtd::FB_THREADS, 0, ctx->stream>>>(F);
    HIPC(hipGetLastError());
    h.cost_cur ^= 1;
    if (h.fb_pending) {  // a recent frame's hot count (grid size), if its copy has landed: a query, never a wait
        const hipError_t q = hipEventQuery(h.fb_ev);
        if (q == hipSuccess) {
            h.fb_hot_est = h.h_fb_cnt[0];
            h.fb_est_c = h.fb_pend_c;
            h.fb_pending = false;
        } else if (q == hipErrorNotReady) {
            (void)hipGetLastError();
        } else {
            return fail(ctx, q, "rt_render: hybrid feedback count");
        }
    }
    if (hot && !h.fb_pending) {
        HIPC(hipMemcpyAsync(h.h_fb_cnt, d_cnt, sizeof(int), hipMemcpyDeviceToHost, ctx->stream));
        HIPC(hipEventRecord(h.fb_ev, ctx->stream));
        h.fb_pending = true;
        h.fb_pend_c = c;
    }
    const KFn kc = coop_kernel<MAXB>(g, count);
    rtd::KArgs B = A;  // the hot kernel's tiles, hottest first, their number on the device
    B.tiles_x = ctw;
    B.n_tiles = 4 * (int)h.n_tiles;
    B.n_tiles_dev = d_cnt;
    B.tile_order = d_hot;
    B.region_off = nullptr;
    B.work = A.work + 224;
    B.tile_cost = cost_out;
    rtd::KArgs P = A;  // the cold 8x8 tiles by region, costliest first (the region offsets hold their number)
    P.region_off = d_cold;
    P.tile_order = d_cold + 9;
    P.tile_cost = cost_out;
    size_t dyn = 0;
    const KFn kp = persist_kernel<MAXB>(P, h.cold[c], count, ctx->device, dyn, ctx->pk_ok, ctx->tq_ok, build);
    if (build) *build |= RT_BUILD_FEEDBACK;
    const int rp = resident(kp, ctx->device, 8, dyn);
    const int rcp = resident(kc, ctx->device);
    const int est = h.fb_hot_est >= 0 && h.fb_est_c == c ? h.fb_hot_est : h.n_hot[c];  // (another candidate's: its own)
    // the hot kernel's grid from a count a few frames old: with headroom (2x + 64 tiles), since a hot set that grew
    // past its grid's waves -- a moving camera's, after frames of few hot tiles -- is rendered by too few waves (dragon
    // walkthrough frames of 3-6 ms among ~1.1 ms ones); a persistent grid's waves that find no tile exit at once
    const int est_h = 2 * est + 64;
    const int nc = hot ? std::max(1, std::min((est_h + 3) / 4, rcp / 2)) : 0;
    const int np = std::max(1, std::min(rp - (int)((long long)nc * rp / rcp), (A.n_tiles + 3) / 4));
    if (!hot) {  // (the whole frame, costliest first)
        kp<<<np, rtd::BLOCK, dyn, ctx->stream>>>(with_slots(P, dyn));
        HIPC(hipGetLastError());
        return RT_OK;
    }
    HIPC(hipEventRecord(h.fork, ctx->stream));  // after the lists, the counters' and the durations' resets
    HIPC(hipStreamWaitEvent(h.s2, h.fork, 0));
    kc<<<nc, rtd::BLOCK, 0, h.s2>>>(B);
    HIPC(hipGetLastError());
    kp<<<np, rtd::BLOCK, dyn, ctx->stream>>>(with_slots(P, dyn));
    HIPC(hipGetLastError());
    HIPC(hipEventRecord(h.join, h.s2));
    HIPC(hipStreamWaitEvent(ctx->stream, h.join, 0));
    return RT_OK;
}
}  // namespace

namespace {
// a rank's part of a gathered frame batch, the layout checks (rt_comm_logic.hpp: host-only, unit-tested with g++)
using rtc::check_parts;
using rtc::Part;
using rtc::part_px;

Part part_of(const rt_ctx* c) {
    Part p{};
    p.W = c->last_W;
    p.H = c->last_H;
    p.frames = c->last_frames;
    p.rows = c->last_rows;
    p.off = c->last_off;
    p.stride = c->last_stride;
    p.block = c->last_block;
    p.shift = c->last_shift;
    p.words = c->last_bgra ? 1 : 3;
    p.hit = c->last_hit ? 1 : 0;
    return p;
}
const void* payload_of(const rt_ctx* c) { return c->last_bgra ? (const void*)c->last_bgra : (const void*)c->last_rgb; }

// compact part -> full frames on stream s (root's device)
int unshuffle(rt_ctx* ctx, const void* src, void* dst, const Part& p, int words, hipStream_t s) {
    const size_t n = part_px(p);
    if (!n) return RT_OK;
    const int grid = (int)std::max<size_t>(1, std::min<size_t>((n + 255) / 256, 4096));
    rtd::k_unshuffle_frames<<<grid, 256, 0, s>>>((const unsigned*)src, (unsigned*)dst, p.W, p.H, p.frames, p.rows,
                                                   p.off, p.stride, p.block, p.shift, words);
    HIPC(hipGetLastError());
    return RT_OK;
}

// the root's full frames (its own buffers unless the caller gave one); afterwards its last render IS them
int full_target(rt_ctx* ctx, const Part& a, void* user, void** dst, int** dst_hit, bool want_hit) {
    const size_t px = (size_t)a.frames * a.W * a.H;
    int rc;
    if (user) *dst = user;
    else if (a.words == 1) {
        if ((rc = grow(ctx, &ctx->d_full_bgra, ctx->full_bgra_cap, px))) return rc;
        *dst = ctx->d_full_bgra;
    } else {
        if ((rc = grow(ctx, &ctx->d_full, ctx->full_cap, 3 * px))) return rc;
        *dst = ctx->d_full;
    }
    *dst_hit = nullptr;
    if (want_hit) {
        if ((rc = grow(ctx, &ctx->d_full_hit, ctx->full_hit_cap, px))) return rc;
        *dst_hit = ctx->d_full_hit;
    }
    return RT_OK;
}

int finish_gather(rt_ctx* ctx, const Part& a, void* dst, int* dst_hit) {
    // the gather's completion has its own event: ev0s / ev1s stay the render launches' (rt_kernel_times)
    if (!ctx->gather_ev) HIPC(hipEventCreateWithFlags(&ctx->gather_ev, hipEventDisableTiming));
    HIPC(hipEventRecord(ctx->gather_ev, ctx->stream));
    ctx->last_rgb = a.words == 3 ? (float*)dst : nullptr;
    ctx->last_bgra = a.words == 1 ? (unsigned*)dst : nullptr;
    ctx->last_hit = dst_hit;
    ctx->last_pixels = (size_t)a.frames * a.W * a.H;
    ctx->last_off = 0;
    ctx->last_stride = 1;
    ctx->last_rows = a.H;
    ctx->last_block = 1;
    ctx->last_shift = 0;
    return RT_OK;
}
}  // namespace

extern "C" int rt_gather(rt_ctx* const* ctxs, int n, int root) { return rt_gather_to(ctxs, n, root, nullptr); }

extern "C" int rt_gather_to(rt_ctx* const* ctxs, int n, int root, void* d_dst) {
    if (!ctxs || n <= 0 || root < 0 || root >= n || !ctxs[root]) return RT_E_ARG;
    rt_ctx* ctx = ctxs[root];
    std::vector<Part> ps;
    bool all_hit = true;
    for (int i = 0; i < n; i++) {
        rt_ctx* c = ctxs[i];
        if (!c || !c->rendered) return arg_err(ctx, "rt_gather: a context has not rendered");
        ps.push_back(part_of(c));
        all_hit = all_hit && c->last_hit;
    }
    const std::string why = check_parts(ps);
    if (!why.empty()) return arg_err(ctx, ("rt_gather: " + why).c_str());
    const Part& a = ps[0];
    const int words = a.words;
    // staging on the root for the parts of other devices, in rank order: payload, then hit
    size_t stage = 0;
    for (int i = 0; i < n; i++)
        if (ctxs[i]->device != ctx->device) stage += part_px(ps[i]) * 4 * (words + (all_hit ? 1 : 0));
    HIPC(hipSetDevice(ctx->device));
    int rc;
    if (stage && (rc = grow(ctx, &ctx->d_stage, ctx->stage_cap, stage))) return rc;
    void* dst;
    int* dst_hit;
    if ((rc = full_target(ctx, a, d_dst, &dst, &dst_hit, all_hit))) return rc;
    size_t at = 0;
    for (int i = 0; i < n; i++) {
        rt_ctx* c = ctxs[i];
        const size_t cpx = part_px(ps[i]);
        const void* src = payload_of(c);
        const int* src_hit = c->last_hit;
        if (c->device != ctx->device) {
            // xGMI peer copies issued on the SOURCE's stream (after its render; the copies of different sources
            // run on their own devices' engines at once), then the root waits for them
            void* d1 = ctx->d_stage + at;
            at += cpx * 4 * words;
            HIPC(hipSetDevice(c->device));
            // the root's staging area may still be read by the previous gather's un-interleaving (root stream):
            // the source's copy into it waits for that gather's completion (write after read)
            if (ctx->gather_ev) HIPC(hipStreamWaitEvent(c->stream, ctx->gather_ev, 0));
            int can = 0;
            (void)hipDeviceCanAccessPeer(&can, c->device, ctx->device);
            if (can) {  // direct xGMI copies (else the runtime stages through the host)
                const hipError_t e = hipDeviceEnablePeerAccess(ctx->device, 0);
                if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled) return fail(ctx, e, "hipDeviceEnablePeerAccess");
                (void)hipGetLastError();
            }
            HIPC(hipMemcpyPeerAsync(d1, ctx->device, src, c->device, cpx * 4 * words, c->stream));
            src = d1;
            if (all_hit) {
                int* d2 = (int*)(ctx->d_stage + at);
                at += cpx * 4;
                HIPC(hipMemcpyPeerAsync(d2, ctx->device, src_hit, c->device, cpx * 4, c->stream));
                src_hit = d2;
            }
            if (!c->copy_ev) HIPC(hipEventCreateWithFlags(&c->copy_ev, hipEventDisableTiming));
            HIPC(hipEventRecord(c->copy_ev, c->stream));
            HIPC(hipSetDevice(ctx->device));
            HIPC(hipStreamWaitEvent(ctx->stream, c->copy_ev, 0));
        } else if (c != ctx) {
            HIPC(hipStreamWaitEvent(ctx->stream, c->ev1, 0));  // after the source's last render
        }
        if ((rc = unshuffle(ctx, src, dst, ps[i], words, ctx->stream))) return rc;
        if (all_hit && (rc = unshuffle(ctx, src_hit, dst_hit, ps[i], 1, ctx->stream))) return rc;
    }
    return finish_gather(ctx, a, dst, dst_hit);
}

// ---------------------------------------------------------------- RCCL communicator (rt_comm_*)
struct rt_comm {
    std::vector<rt_ctx*> ctxs;  // rt_comm_init: the local ranks rank0 .. rank0 + n - 1; rt_comm_init_rank: this rank's
    std::vector<int> devices;   // their devices
    std::vector<ncclComm_t> comms;
    int nranks = 0, rank0 = 0;
    bool multi = false;  // rt_comm_init_rank: one rank of a multi-process job (row sets exchanged over RCCL)
    // multi-process: the layout -- every rank's descriptor as last exchanged (ncclAllGather), and this rank's part
    // at that exchange. A gather exchanges again only on what every rank sees the same way (rtc::layout_step: the
    // first gather, a new frame size / count / pixel kind, or rt_comm_relayout on every rank).
    std::vector<Part> layout;
    Part mine{};
    bool have_layout = false;
    Part* d_desc = nullptr;  // every rank's descriptor (ncclAllGather) + this rank's staging slot, on its device
    Part* h_desc = nullptr;  // pinned
    unsigned long long* d_count = nullptr;  // the root's coverage check of a layout's first gather
    hipStream_t side = nullptr;  // the exchange's stream: the host waits for the exchange only, not for renders
    hipEvent_t done = nullptr;   // after the last send / recv group: the next operation on the communicator waits
    bool issued = false;
    // the issued send / recv groups not yet seen complete, oldest first: `pre` recorded on the source's stream before
    // the group (after its render: the group's local part), `done` after it (rtc::settle: the deadline covers the
    // collective, not the render before it); events reused from ev_pool
    struct Pending {
        hipEvent_t pre, done;
    };
    std::vector<Pending> pending;
    std::vector<hipEvent_t> ev_pool;
    std::shared_ptr<CommLink> link = std::make_shared<CommLink>();
    bool aborted = false;     // a collective missed its deadline: the communicator was aborted (ncclCommAbort)
    double timeout_s = 120.0;  // host waits on a collective (rt_comm_set_timeout)
    rt_comm_info info{};
    std::string err;
};

namespace {
// RCCL is opened on first use (dlopen of librccl.so.1), not linked: a process that never builds a communicator
// never loads it, and one that already has it (torch.distributed's RCCL) gets that same library (matched by
// soname) instead of a second copy next to it.
struct Rccl {
    bool tried = false, ok = false;
    std::string why;
    ncclResult_t (*GetUniqueId)(ncclUniqueId*) = nullptr;
    ncclResult_t (*CommInitAll)(ncclComm_t*, int, const int*) = nullptr;
    ncclResult_t (*CommInitRank)(ncclComm_t*, int, ncclUniqueId, int) = nullptr;
    ncclResult_t (*CommDestroy)(ncclComm_t) = nullptr;
    ncclResult_t (*CommAbort)(ncclComm_t) = nullptr;
    ncclResult_t (*AllGather)(const void*, void*, size_t, ncclDataType_t, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*Send)(const void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*Recv)(void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*GroupStart)() = nullptr;
    ncclResult_t (*GroupEnd)() = nullptr;
    const char* (*GetErrorString)(ncclResult_t) = nullptr;
};
Rccl& rccl() {
    static Rccl R;
    if (R.tried) return R;
    R.tried = true;
    void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
    if (!h) h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
    if (!h) {
        R.why = std::string("cannot load librccl.so.1: ") + dlerror();
        return R;
    }
    bool all = true;
    auto sym = [&](auto& fp, const char* name) {
        fp = reinterpret_cast<std::remove_reference_t<decltype(fp)>>(dlsym(h, name));
        if (!fp) all = false;
    };
    sym(R.GetUniqueId, "ncclGetUniqueId");
    sym(R.CommInitAll, "ncclCommInitAll");
    sym(R.CommInitRank, "ncclCommInitRank");
    sym(R.CommDestroy, "ncclCommDestroy");
    sym(R.CommAbort, "ncclCommAbort");
    sym(R.AllGather, "ncclAllGather");
    sym(R.Send, "ncclSend");
    sym(R.Recv, "ncclRecv");
    sym(R.GroupStart, "ncclGroupStart");
    sym(R.GroupEnd, "ncclGroupEnd");
    sym(R.GetErrorString, "ncclGetErrorString");
    R.ok = all;
    if (!all) R.why = "librccl.so.1 lacks a symbol";
    return R;
}

int comm_fail(rt_comm* cm, ncclResult_t r, const char* what) {
    cm->err = std::string(what) + ": " + (rccl().GetErrorString ? rccl().GetErrorString(r) : "RCCL error");
    if (!cm->ctxs.empty() && cm->ctxs[0]) cm->ctxs[0]->err = cm->err;  // (null: that context was destroyed)
    return RT_E_HIP;
}
int comm_arg(rt_comm* cm, const std::string& what) {
    cm->err = what;
    for (rt_ctx* c : cm->ctxs)
        if (c) c->err = what;
    return RT_E_ARG;
}
#define NCCLC(call)                                       \
    do {                                                  \
        ncclResult_t r_ = (call);                         \
        if (r_ != ncclSuccess) return comm_fail(cm, r_, #call); \
    } while (0)

// A collective that misses its deadline: every RCCL communicator of `cm` is aborted (its kernels stop waiting for
// the missing peer, so the streams drain), and the communicator refuses further gathers.
int comm_abort(rt_comm* cm, const std::string& what) {
    for (size_t l = 0; l < cm->comms.size(); l++)
        if (cm->comms[l]) {
            (void)hipSetDevice(cm->devices[l]);
            (void)rccl().CommAbort(cm->comms[l]);
            cm->comms[l] = nullptr;
        }
    cm->aborted = true;
    cm->err = what;
    for (rt_ctx* c : cm->ctxs)
        if (c) c->err = what;
    // (the aborted groups' kernels stop waiting, the streams drain: nothing outstanding is waited for again)
    for (const rt_comm::Pending& p : cm->pending) {
        cm->ev_pool.push_back(p.pre);
        cm->ev_pool.push_back(p.done);
    }
    cm->pending.clear();
    return RT_E_TIMEOUT;
}
// A host wait on work behind a collective (a stream or an event), bounded by the communicator's timeout
// (rtc::bounded_wait): RT_E_TIMEOUT and an aborted communicator instead of a hang when a peer never arrives.
template <class Q>
int comm_wait(rt_comm* cm, Q query_hip, const char* what) {
    int err = 0;
    const rtc::Wait w = rtc::bounded_wait(
        [&]() -> int {
            const hipError_t e = query_hip();
            if (e == hipSuccess) return 0;
            if (e == hipErrorNotReady) {
                (void)hipGetLastError();  // not an error: still running
                return 1;
            }
            return -(int)e;
        },
        cm->timeout_s, err);
    if (w == rtc::Wait::Done) return RT_OK;
    if (w == rtc::Wait::Error) {
        cm->err = std::string(what) + ": " + hipGetErrorString((hipError_t)(-err));
        for (rt_ctx* c : cm->ctxs)
            if (c) c->err = cm->err;
        return RT_E_HIP;
    }
    return comm_abort(cm, std::string(what) + ": no completion within " + std::to_string(cm->timeout_s) +
                              " s (a peer rank never joined the collective); the communicator is aborted");
}

int event_state(hipEvent_t e) {  // rtc query convention: 0 complete, 1 not yet, < 0 -(hipError_t)
    const hipError_t q = hipEventQuery(e);
    if (q == hipSuccess) return 0;
    if (q == hipErrorNotReady) {
        (void)hipGetLastError();  // not an error: still running
        return 1;
    }
    return -(int)q;
}

// Waits for every outstanding send / recv group of a multi-process communicator, in issue order (rtc::settle): each
// group's render without a deadline, its collective within the communicator's timeout from the moment that render has
// completed. RT_E_TIMEOUT (the communicator aborted) when a peer never joins.
int comm_settle(rt_comm* cm, const char* what) {
    if (cm->aborted) {
        cm->err = std::string(what) + ": the communicator was aborted";
        return RT_E_TIMEOUT;
    }
    if (cm->pending.empty()) return RT_OK;
    (void)hipSetDevice(cm->devices[0]);
    int err = 0, n_done = 0;
    const rtc::Wait w = rtc::settle((int)cm->pending.size(), [&](int j) { return event_state(cm->pending[j].pre); },
                                    [&](int j) { return event_state(cm->pending[j].done); }, cm->timeout_s, err, n_done);
    for (int j = 0; j < n_done; j++) {
        cm->ev_pool.push_back(cm->pending[j].pre);
        cm->ev_pool.push_back(cm->pending[j].done);
    }
    cm->pending.erase(cm->pending.begin(), cm->pending.begin() + n_done);
    if (w == rtc::Wait::Done) return RT_OK;
    if (w == rtc::Wait::Error) {
        cm->err = std::string(what) + ": " + hipGetErrorString((hipError_t)(-err));
        for (rt_ctx* c : cm->ctxs)
            if (c) c->err = cm->err;
        return RT_E_HIP;
    }
    return comm_abort(cm, std::string(what) + ": a gather's collective did not complete within " +
                              std::to_string(cm->timeout_s) +
                              " s of its render (a peer rank never joined it); the communicator is aborted");
}
// the same for a context whose stream holds a group (sync_checked, rt_kernel_times, rt_destroy)
int comm_settle_ctx(rt_ctx* ctx, const char* who) {
    if (!ctx->comm_link || !ctx->comm_link->cm) return RT_OK;
    rt_comm* cm = ctx->comm_link->cm;
    if (cm->aborted) return RT_OK;  // (aborted: its groups no longer block the stream)
    const int rc = comm_settle(cm, who);
    (void)hipSetDevice(ctx->device);
    if (rc) ctx->err = cm->err;
    return rc;
}
// completed groups off the front of the list, without waiting (each gather: the list stays short)
void comm_prune(rt_comm* cm) {
    size_t k = 0;
    while (k < cm->pending.size() && event_state(cm->pending[k].done) == 0) {
        cm->ev_pool.push_back(cm->pending[k].pre);
        cm->ev_pool.push_back(cm->pending[k].done);
        k++;
    }
    cm->pending.erase(cm->pending.begin(), cm->pending.begin() + k);
}
hipError_t comm_event(rt_comm* cm, hipEvent_t* e) {
    if (!cm->ev_pool.empty()) {
        *e = cm->ev_pool.back();
        cm->ev_pool.pop_back();
        return hipSuccess;
    }
    return hipEventCreateWithFlags(e, hipEventDisableTiming);
}
}  // namespace

extern "C" int rt_comm_get_id(unsigned char* id) {
    if (!id) return RT_E_ARG;
    static_assert(sizeof(ncclUniqueId) == RT_COMM_ID_BYTES, "ncclUniqueId size");
    if (!rccl().ok) return RT_E_STATE;
    ncclUniqueId u;
    if (rccl().GetUniqueId(&u) != ncclSuccess) return RT_E_HIP;
    std::memcpy(id, &u, sizeof u);
    return RT_OK;
}

extern "C" int rt_comm_init(rt_ctx* const* ctxs, int n, rt_comm** out) {
    if (!ctxs || n <= 0 || !out) return RT_E_ARG;
    *out = nullptr;
    std::vector<int> devs;
    for (int i = 0; i < n; i++) {
        if (!ctxs[i]) return RT_E_ARG;
        for (int d : devs)
            if (d == ctxs[i]->device) {
                ctxs[i]->err = "rt_comm_init: RCCL takes one rank per device (two contexts share a device: use rt_gather)";
                return RT_E_ARG;
            }
        devs.push_back(ctxs[i]->device);
    }
    if (!rccl().ok) {
        ctxs[0]->err = "rt_comm_init: " + rccl().why;
        return RT_E_STATE;
    }
    rt_comm* cm = new rt_comm;
    cm->ctxs.assign(ctxs, ctxs + n);
    cm->devices = devs;
    cm->comms.resize(n);
    cm->nranks = n;
    cm->info.nranks = n;
    const ncclResult_t r = rccl().CommInitAll(cm->comms.data(), n, devs.data());
    if (r != ncclSuccess) {
        comm_fail(cm, r, "ncclCommInitAll");
        delete cm;
        return RT_E_HIP;
    }
    *out = cm;
    return RT_OK;
}

extern "C" int rt_comm_init_rank(rt_ctx* ctx, int nranks, int rank, const unsigned char* id, rt_comm** out) {
    if (!ctx || !id || !out || nranks <= 0 || rank < 0 || rank >= nranks) return RT_E_ARG;
    *out = nullptr;
    if (!rccl().ok) {
        ctx->err = "rt_comm_init_rank: " + rccl().why;
        return RT_E_STATE;
    }
    HIPC(hipSetDevice(ctx->device));
    rt_comm* cm = new rt_comm;
    cm->ctxs = {ctx};
    cm->devices = {ctx->device};
    cm->comms.resize(1);
    cm->nranks = nranks;
    cm->rank0 = rank;
    cm->multi = true;
    cm->info.nranks = nranks;
    cm->info.rank = rank;
    ncclUniqueId u;
    std::memcpy(&u, id, sizeof u);
    ncclResult_t r = rccl().CommInitRank(&cm->comms[0], nranks, u, rank);
    if (r != ncclSuccess) {
        comm_fail(cm, r, "ncclCommInitRank");
        delete cm;
        return RT_E_HIP;
    }
    hipError_t e = hipMalloc((void**)&cm->d_desc, sizeof(Part) * (nranks + 1));
    if (e == hipSuccess) e = hipHostMalloc((void**)&cm->h_desc, sizeof(Part) * (nranks + 1));
    if (e == hipSuccess) e = hipMalloc((void**)&cm->d_count, sizeof(unsigned long long));
    if (e == hipSuccess) e = hipStreamCreateWithFlags(&cm->side, hipStreamNonBlocking);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&cm->done, hipEventDisableTiming);
    if (e != hipSuccess) {
        fail(ctx, e, "rt_comm_init_rank: descriptor buffers");
        rt_comm_destroy(cm);
        return RT_E_HIP;
    }
    *out = cm;
    return RT_OK;
}

namespace {
// The multi-process gather: `src` (a context of this rank on the communicator's device) sends its last render to
// the root. One communicator serves every context of the rank (bench.py alternates two on two streams): each
// gather's send / recv group runs on its source's stream (so after that render) and after the previous group on
// the communicator (an event), so every rank runs the communicator's operations in one order.
int comm_gather_multi(rt_comm* cm, rt_ctx* src, int root, void* d_dst) {
    rt_ctx* ctx = src;
    HIPC(hipSetDevice(ctx->device));
    if (cm->aborted) return comm_arg(cm, "rt_comm_gather: the communicator was aborted (" + cm->err + ")");
    // this rank's part; a rank whose context has not rendered still takes part (W = 0), so that every rank fails
    // together in check_parts instead of the others waiting in the collective for it
    const Part mine = ctx->rendered ? part_of(ctx) : Part{};
    const rtc::Step step = rtc::layout_step(mine, cm->mine, cm->have_layout);
    if (step == rtc::Step::RowsChanged)  // (refused before any collective call: the peers' next wait times out)
        return comm_arg(cm, "rt_comm_gather: this rank's rows changed without a layout change every rank sees "
                            "(frame size, frame count, pixel kind): call rt_comm_relayout on every rank first");
    const bool fresh = step == rtc::Step::Exchange;
    if (fresh) {  // a new layout: exchange the 64-B descriptors (ncclAllGather) and check that they partition the frames
        // (the groups before it first: their renders unbounded, their collectives bounded -- the exchange's own
        // deadline then covers the AllGather only)
        if (int rc = comm_settle(cm, "rt_comm_gather: the gathers before a row-set exchange")) return rc;
        cm->h_desc[cm->nranks] = mine;
        if (cm->issued) HIPC(hipStreamWaitEvent(cm->side, cm->done, 0));
        HIPC(hipMemcpyAsync(cm->d_desc + cm->nranks, cm->h_desc + cm->nranks, sizeof(Part), hipMemcpyHostToDevice, cm->side));
        NCCLC(rccl().AllGather(cm->d_desc + cm->nranks, cm->d_desc, sizeof(Part) / 4, ncclInt32, cm->comms[0], cm->side));
        HIPC(hipMemcpyAsync(cm->h_desc, cm->d_desc, sizeof(Part) * cm->nranks, hipMemcpyDeviceToHost, cm->side));
        if (int rc = comm_wait(cm, [&] { return hipStreamQuery(cm->side); }, "rt_comm_gather: row-set exchange"))
            return rc;
        cm->info.exchanges++;
        cm->layout.assign(cm->h_desc, cm->h_desc + cm->nranks);
        cm->have_layout = false;
        const std::string why = check_parts(cm->layout);
        if (!why.empty()) return comm_arg(cm, "rt_comm_gather: " + why);
        cm->mine = mine;
        cm->have_layout = true;
    }
    const std::vector<Part>& ps = cm->layout;
    const Part& a = ps[0];
    const int words = a.words;
    const bool is_root = cm->rank0 == root;
    std::vector<size_t> at(cm->nranks, 0);
    void* dst = nullptr;
    int* dst_hit = nullptr;
    if (is_root) {
        size_t stage = 0;
        for (int q = 0; q < cm->nranks; q++) {
            at[q] = stage;
            if (q != root) stage += part_px(ps[q]) * 4 * words;
        }
        int rc;
        if (stage && (rc = grow(ctx, &ctx->d_stage, ctx->stage_cap, stage))) return rc;
        if ((rc = full_target(ctx, a, d_dst, &dst, &dst_hit, false))) return rc;
    }
    if (cm->issued) HIPC(hipStreamWaitEvent(ctx->stream, cm->done, 0));
    const size_t full_px = (size_t)a.frames * a.W * a.H;
    if (is_root && fresh)  // coverage check of a layout's first gather: no render writes this value (k_count_unwritten)
        HIPC(hipMemsetAsync(dst, words == 1 ? 0 : 0xFF, full_px * 4 * words, ctx->stream));
    comm_prune(cm);
    rt_comm::Pending pend{};
    HIPC(comm_event(cm, &pend.pre));
    if (hipError_t e = comm_event(cm, &pend.done); e != hipSuccess) {
        cm->ev_pool.push_back(pend.pre);
        return fail(ctx, e, "rt_comm_gather: events");
    }
    cm->ev_pool.push_back(pend.pre);  // (back to the pool unless the group is issued below)
    cm->ev_pool.push_back(pend.done);
    HIPC(hipEventRecord(pend.pre, ctx->stream));  // the group's local part (the render) ends here
    NCCLC(rccl().GroupStart());
    if (!is_root) {
        NCCLC(rccl().Send(payload_of(ctx), part_px(ps[cm->rank0]) * words, ncclUint32, root, cm->comms[0], ctx->stream));
    } else {
        for (int q = 0; q < cm->nranks; q++)
            if (q != root)
                NCCLC(rccl().Recv(ctx->d_stage + at[q], part_px(ps[q]) * words, ncclUint32, q, cm->comms[0], ctx->stream));
    }
    NCCLC(rccl().GroupEnd());
    HIPC(hipEventRecord(cm->done, ctx->stream));
    cm->ev_pool.pop_back();
    cm->ev_pool.pop_back();
    HIPC(hipEventRecord(pend.done, ctx->stream));
    cm->pending.push_back(pend);
    ctx->comm_link = cm->link;
    cm->issued = true;
    cm->info.gathers++;
    if (!is_root) return RT_OK;
    int rc;
    for (int q = 0; q < cm->nranks; q++) {
        const void* s = q == root ? payload_of(ctx) : (const void*)(ctx->d_stage + at[q]);
        if ((rc = unshuffle(ctx, s, dst, ps[q], words, ctx->stream))) return rc;
    }
    if ((rc = finish_gather(ctx, a, dst, dst_hit))) return rc;
    if (fresh) {  // the layout's first gather, checked pixel by pixel on the root (once per layout: a host wait)
        unsigned long long left = 0;
        HIPC(hipMemsetAsync(cm->d_count, 0, sizeof left, ctx->stream));
        const int grid = (int)std::max<size_t>(1, std::min<size_t>((full_px + 255) / 256, 4096));
        rtd::k_count_unwritten<<<grid, 256, 0, ctx->stream>>>((const unsigned*)dst, full_px, words, cm->d_count);
        HIPC(hipGetLastError());
        HIPC(hipMemcpyAsync(&left, cm->d_count, sizeof left, hipMemcpyDeviceToHost, ctx->stream));
        // the group (its render unbounded, its collective bounded), then the local unshuffle and count behind it
        if (int rc2 = comm_settle(cm, "rt_comm_gather: coverage check")) return rc2;
        if (int rc2 = comm_wait(cm, [&] { return hipStreamQuery(ctx->stream); }, "rt_comm_gather: coverage check"))
            return rc2;
        cm->info.checked++;
        if (left)  // (the layout stays: every rank keeps the same view of it, so the next gathers stay matched)
            return comm_arg(cm, "rt_comm_gather: the gathered frames miss " + std::to_string(left) + " pixels");
    }
    return RT_OK;
}
}  // namespace

extern "C" int rt_comm_gather_from(rt_comm* cm, rt_ctx* src, int root, void* d_dst) {
    if (!cm || root < 0 || root >= cm->nranks) return RT_E_ARG;
    if (cm->multi) {
        if (!src) src = cm->ctxs[0];
        if (!src) return comm_arg(cm, "rt_comm_gather_from: the communicator's context was destroyed");
        if (src->device != cm->devices[0])
            return comm_arg(cm, "rt_comm_gather_from: the context is not on the communicator's device");
        return comm_gather_multi(cm, src, root, d_dst);
    }
    if (src && src != cm->ctxs[0]) return comm_arg(cm, "rt_comm_gather_from: a one-process communicator gathers its own contexts");
    const int nl = (int)cm->ctxs.size();
    // one process: every rank's descriptor at hand
    std::vector<Part> ps(cm->nranks);
    for (rt_ctx* c : cm->ctxs)
        if (!c || !c->rendered) return comm_arg(cm, "rt_comm_gather: a context has not rendered (or was destroyed)");
    for (int i = 0; i < nl; i++) ps[i] = part_of(cm->ctxs[i]);
    const std::string why = check_parts(ps);
    if (!why.empty()) return comm_arg(cm, "rt_comm_gather: " + why);
    const Part& a = ps[0];
    const int words = a.words;
    rt_ctx* rctx = cm->ctxs[root];
    std::vector<size_t> at(cm->nranks, 0);
    void* dst = nullptr;
    int* dst_hit = nullptr;
    {
        rt_ctx* ctx = rctx;
        size_t stage = 0;
        for (int q = 0; q < cm->nranks; q++) {
            at[q] = stage;
            if (q != root) stage += part_px(ps[q]) * 4 * words;
        }
        HIPC(hipSetDevice(ctx->device));
        int rc;
        if (stage && (rc = grow(ctx, &ctx->d_stage, ctx->stage_cap, stage))) return rc;
        if ((rc = full_target(ctx, a, d_dst, &dst, &dst_hit, false))) return rc;
    }
    // one group: every non-root rank sends its compact frames (on its stream: after its render), the root receives
    // every peer's into its staging slot
    NCCLC(rccl().GroupStart());
    for (int l = 0; l < nl; l++) {
        rt_ctx* c = cm->ctxs[l];
        if (l != root) {
            NCCLC(rccl().Send(payload_of(c), part_px(ps[l]) * words, ncclUint32, root, cm->comms[l], c->stream));
        } else {
            for (int q = 0; q < cm->nranks; q++)
                if (q != root)
                    NCCLC(rccl().Recv(rctx->d_stage + at[q], part_px(ps[q]) * words, ncclUint32, q, cm->comms[l], c->stream));
        }
    }
    NCCLC(rccl().GroupEnd());
    cm->info.gathers++;
    rt_ctx* ctx = rctx;
    HIPC(hipSetDevice(ctx->device));
    int rc;
    for (int q = 0; q < cm->nranks; q++) {
        const void* s = q == root ? payload_of(ctx) : (const void*)(ctx->d_stage + at[q]);
        if ((rc = unshuffle(ctx, s, dst, ps[q], words, ctx->stream))) return rc;
    }
    return finish_gather(ctx, a, dst, dst_hit);
}

extern "C" int rt_comm_gather(rt_comm* cm, int root, void* d_dst) { return rt_comm_gather_from(cm, nullptr, root, d_dst); }

extern "C" int rt_comm_relayout(rt_comm* cm) {
    if (!cm) return RT_E_ARG;
    cm->have_layout = false;  // the next gather exchanges (every rank calls this before the same gather)
    return RT_OK;
}

extern "C" int rt_comm_set_timeout(rt_comm* cm, double seconds) {
    if (!cm || !(seconds > 0.0)) return RT_E_ARG;
    cm->timeout_s = seconds;
    return RT_OK;
}

extern "C" int rt_comm_wait(rt_comm* cm) {
    if (!cm) return RT_E_ARG;
    if (cm->aborted) return RT_E_TIMEOUT;
    if (!cm->issued || !cm->done) return RT_OK;
    (void)hipSetDevice(cm->devices[0]);
    if (cm->multi) return comm_settle(cm, "rt_comm_wait: the gathers issued");
    return comm_wait(cm, [&] { return hipEventQuery(cm->done); }, "rt_comm_wait: the last gather");
}

extern "C" int rt_comm_get_info(rt_comm* cm, rt_comm_info* info) {
    if (!cm || !info) return RT_E_ARG;
    *info = cm->info;
    return RT_OK;
}

extern "C" const char* rt_comm_last_error(rt_comm* cm) { return cm ? cm->err.c_str() : "null communicator"; }

extern "C" void rt_comm_destroy(rt_comm* cm) {
    if (!cm) return;
    // (the contexts may be gone already: only the communicator's own devices, events and streams are touched)
    // the last send / recv group (any context's stream) has run -- or its peers never came and the bounded wait
    // aborted the communicator (comm_abort): nothing left to wait for
    if (cm->issued && cm->done && !cm->aborted) (void)rt_comm_wait(cm);
    for (size_t l = 0; l < cm->comms.size(); l++) {
        (void)hipSetDevice(cm->devices[l]);
        if (!cm->multi && !cm->aborted) (void)hipDeviceSynchronize();  // (one process: the groups ran on the contexts' streams)
        if (cm->comms[l]) (void)rccl().CommDestroy(cm->comms[l]);
    }
    if (cm->side && !cm->aborted) (void)hipStreamSynchronize(cm->side);
    if (cm->d_desc) (void)hipFree(cm->d_desc);
    if (cm->d_count) (void)hipFree(cm->d_count);
    if (cm->h_desc) (void)hipHostFree(cm->h_desc);
    if (cm->side) (void)hipStreamDestroy(cm->side);
    if (cm->done) (void)hipEventDestroy(cm->done);
    for (const rt_comm::Pending& p : cm->pending) cm->ev_pool.insert(cm->ev_pool.end(), {p.pre, p.done});
    for (hipEvent_t e : cm->ev_pool) (void)hipEventDestroy(e);
    cm->link->cm = nullptr;  // (the contexts that still hold the link see the communicator gone)
    delete cm;
}

extern "C" int rt_download_bmp(rt_ctx* ctx, unsigned char* h_bmp, size_t cap) {
    if (!ctx || !h_bmp) return RT_E_ARG;
    if (!ctx->rendered) {
        ctx->err = "rt_download_bmp: nothing rendered";
        return RT_E_STATE;
    }
    if (ctx->last_frames != 1) return arg_err(ctx, "rt_download_bmp: the last render was a frame batch");
    if (!ctx->last_rgb && !ctx->last_bgra) return arg_err(ctx, "rt_download_bmp: no pixels in the last render");
    const int W = ctx->last_W, H = ctx->last_H;
    if (ctx->last_off != 0 || ctx->last_stride != ctx->last_block || ctx->last_rows != H) {
        ctx->err = "rt_download_bmp: the last frame is not a full frame (gather it first)";
        return RT_E_STATE;
    }
    const size_t px = (size_t)W * H;
    if (cap < 54 + 4 * px) return arg_err(ctx, "rt_download_bmp: buffer too small");
    HIPC(hipSetDevice(ctx->device));
    int rc;
    if ((rc = grow(ctx, &ctx->d_bmp, ctx->bmp_cap, px))) return rc;
    const int grid = (int)std::max<size_t>(1, std::min<size_t>((px + 255) / 256, 4096));
    if (ctx->last_rgb) rtd::k_bgra<<<grid, 256, 0, ctx->stream>>>(ctx->last_rgb, ctx->d_bmp, W, H);
    else rtd::k_flip_rows<<<grid, 256, 0, ctx->stream>>>(ctx->last_bgra, ctx->d_bmp, W, H);  // already quantised
    HIPC(hipGetLastError());
    if (rth_bmp_header(W, H, h_bmp) != RT_OK) return arg_err(ctx, "rt_download_bmp: bad frame size");
    HIPC(hipMemcpyAsync(h_bmp + 54, ctx->d_bmp, 4 * px, hipMemcpyDeviceToHost, ctx->stream));
    return sync_checked(ctx, "rt_download_bmp");
}

extern "C" int rt_get_stats(rt_ctx* ctx, rt_stats* st) {
    if (!ctx || !st) return RT_E_ARG;
    HIPC(hipSetDevice(ctx->device));
    HIPC(hipStreamSynchronize(ctx->stream));
    unsigned long long c[rtd::NCOUNT];
    HIPC(hipMemcpy(c, ctx->d_counters, sizeof c, hipMemcpyDeviceToHost));
    std::memset(st, 0, sizeof *st);
    st->primary = c[rtd::C_PRIM];
    st->reflection = c[rtd::C_REFL];
    st->shadow = c[rtd::C_SHAD];
    st->shadow_skipped = c[rtd::C_SKIP];
    st->hits = c[rtd::C_HITS];
    st->ch_inner = c[rtd::C_CHI];
    st->ch_leaf = c[rtd::C_CHL];
    st->ch_tri = c[rtd::C_CHT];
    st->sh_inner = c[rtd::C_SHI];
    st->sh_leaf = c[rtd::C_SHL];
    st->sh_tri = c[rtd::C_SHT];
    st->pixels = c[rtd::C_PIX];
    st->fallbacks = c[rtd::C_FALLBACK];
    st->stack_overflows = c[rtd::C_ERR];
    st->node_bytes = 8 * c[rtd::C_NB];
    st->wave_steps = c[rtd::C_WS];
    st->shadow_wave_steps = c[rtd::C_WSH];
    st->steps_lanes_16 = c[rtd::C_Q1];
    st->steps_lanes_32 = c[rtd::C_Q2];
    st->steps_lanes_48 = c[rtd::C_Q3];
    st->steps_lanes_64 = c[rtd::C_Q4];
    std::memcpy(st->steps_hist, c + rtd::C_HIST, sizeof st->steps_hist);
    static_assert(sizeof st->steps_hist == 32 * sizeof(unsigned long long), "histogram slots");
    if (c[rtd::C_ERR]) {
        ctx->err = "rt_get_stats: the render's traversal stack overflowed (BVH deeper than the walks' stacks)";
        return RT_E_KERNEL;
    }
    return RT_OK;
}

extern "C" const char* rt_last_error(rt_ctx* ctx) { return ctx ? ctx->err.c_str() : "null context"; }

extern "C" void rt_destroy(rt_ctx* ctx) {
    if (!ctx) return;
    (void)hipSetDevice(ctx->device);
    // a send / recv group on this stream: waited for through the communicator (bounded; aborted if a peer never
    // joins), and the communicator forgets this context
    (void)comm_settle_ctx(ctx, "rt_destroy");
    if (ctx->comm_link && ctx->comm_link->cm)
        for (rt_ctx*& c : ctx->comm_link->cm->ctxs)
            if (c == ctx) c = nullptr;
    if (ctx->stream) (void)hipStreamSynchronize(ctx->stream);
    free_scene(ctx);
    if (ctx->gather_ev) (void)hipEventDestroy(ctx->gather_ev);
    if (ctx->copy_ev) (void)hipEventDestroy(ctx->copy_ev);
    if (ctx->d_rgb_own) (void)hipFree(ctx->d_rgb_own);
    if (ctx->d_cams) (void)hipFree(ctx->d_cams);
    if (ctx->d_pathbuf) (void)hipFree(ctx->d_pathbuf);
    if (ctx->d_lanebuf) (void)hipFree(ctx->d_lanebuf);
    if (ctx->d_gstack) (void)hipFree(ctx->d_gstack);
    if (ctx->h_cams) (void)hipHostFree(ctx->h_cams);
    if (ctx->d_counters) (void)hipFree(ctx->d_counters);
    if (ctx->h_err) (void)hipHostFree(ctx->h_err);
    for (auto& o : ctx->orders) (void)hipFree(o.second);
    for (void* p : {(void*)ctx->d_full, (void*)ctx->d_full_hit, (void*)ctx->d_stage, (void*)ctx->d_bmp,
                    (void*)ctx->d_full_bgra})
        if (p) (void)hipFree(p);
    if (ctx->d_work) (void)hipFree(ctx->d_work);
    for (int i = 0; i < rt_ctx::NEV; i++) {
        if (ctx->ev0s[i]) (void)hipEventDestroy(ctx->ev0s[i]);
        if (ctx->ev1s[i]) (void)hipEventDestroy(ctx->ev1s[i]);
    }
    if (ctx->hy.s2) (void)hipStreamSynchronize(ctx->hy.s2);
    if (ctx->hy.d_tr) (void)hipFree(ctx->hy.d_tr);
    if (ctx->hy.d_cost) (void)hipFree(ctx->hy.d_cost);
    if (ctx->hy.d_fb) (void)hipFree(ctx->hy.d_fb);
    if (ctx->hy.d_info) (void)hipFree(ctx->hy.d_info);
    if (ctx->hy.h_fb_cnt) (void)hipHostFree(ctx->hy.h_fb_cnt);
    if (ctx->hy.fb_ev) (void)hipEventDestroy(ctx->hy.fb_ev);
    if (ctx->hy.h_tr) (void)hipHostFree(ctx->hy.h_tr);
    if (ctx->hy.d_lists) (void)hipFree(ctx->hy.d_lists);
    if (ctx->hy.h_lists) (void)hipHostFree(ctx->hy.h_lists);
    for (hipEvent_t e : ctx->cam_ev)
        if (e) (void)hipEventDestroy(e);
    for (hipEvent_t e : {ctx->hy.ev, ctx->hy.fork, ctx->hy.join})
        if (e) (void)hipEventDestroy(e);
    if (ctx->hy.s2) (void)hipStreamDestroy(ctx->hy.s2);
    if (ctx->own_stream && ctx->stream) (void)hipStreamDestroy(ctx->stream);
    delete ctx;
}
