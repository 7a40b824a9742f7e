/*
 * rt_hip.h — C-ABI of librt_hip.so, the device half of the drop-in (HIP, gfx950 / MI355X).
 *
 * It replaces the reference's render seam:
 *   GPU  gpu/include/gpu.cuh:23-26   void load_to_gpu(void); float render_frame(bool,int,int);
 *                                     void load_from_gpu(void);
 *   CPU  cpu/src/main.c:214-264       void render_frame(void) over the globals cam, triangles,
 *                                     lights, amb_light, bvh, tri_idx -> vec_t pixels[W*H]
 * with explicit, reentrant calls: state lives in an rt_ctx (one per device), inputs are the
 * reference's own data (triangle_t / bvh_t / light_t layouts, rt_types.h), every call returns an
 * int status (0 = ok, < 0 = RT_E_*), nothing calls exit(). A context is not thread-safe; distinct
 * contexts may be driven from distinct host threads.
 *
 * The per-pixel hot path (ray generation, BVH traversal, ray-triangle intersection, Lambert/Blinn
 * shading with shadow rays, the BOUNCES reflection loop, clamp) runs in ONE HIP kernel per frame
 * (or per batch of frames, rt_render_frames). Every launch configuration is chosen through the
 * arguments below (rt_frame.variant / waves_cap / dealing / regroup / hot_pct); the library reads no
 * environment variable on the render path except two diagnostics (PRT_TILE_TRACE, PRT_TUNE_LOG).
 */
#ifndef RT_HIP_H
#define RT_HIP_H

#include <stddef.h>

#include "rt_types.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct rt_ctx rt_ctx;

/* rt_opts.flags */
enum {
    RT_FLAG_COUNTERS = 1,       /* also count traversal work (node visits, triangle tests): slower */
    /* The kernels' packed builds have field bounds: 5-byte stack entries hold a 24-bit child base (at most 2^24 wide
     * nodes per view), packed triangle-test jobs a 26-bit triangle index (fewer than 2^26 triangles). Scenes past them
     * run the unpacked builds. These two flags select those builds for any scene, so that they can be checked on
     * scenes of test size (tests/test_gpu_unpacked.py). The result is bit-identical either way. */
    RT_FLAG_UNPACKED_STACK = 2, /* as for a scene of more than 2^24 wide nodes: no packed stack entries (no pool
                                   kernels, PERSIST4 with two-word entries) */
    RT_FLAG_UNPACKED_TRIS = 4   /* as for a scene of 2^26 or more triangles: no packed triangle tests */
};

typedef struct rt_opts {
    int device;      /* HIP device ordinal */
    unsigned flags;  /* RT_FLAG_* */
    void* stream;    /* hipStream_t to launch on; NULL = the context creates its own */
} rt_opts;

/* Scene = the globals load_to_gpu() reads (gpu/src/gpu.cu:16-29, 129-201). Deep-copied by
 * rt_upload_scene; the caller keeps ownership. bvh/tri_idx are bvh_build()'s output
 * (cpu/src/bvh.c:360-388) for ANY builder that keeps the reference layout. */
typedef struct rt_scene {
    const rt_triangle* triangles;
    int n_triangles;
    const rt_bvh_node* bvh;
    int n_nodes;
    const int* tri_idx;
    const rt_light* lights;
    int n_lights;
    rt_vec3 amb; /* amb_light (cpu/src/main.c:37): 0.5, 0.5, 0.5 */
    int accel;   /* RT_ACCEL_*: acceleration structure of the fast kernel */
    int ploc_radius; /* RT_ACCEL_GPU / AUTO: the GPU build's nearest-neighbour radius (0 = 32, at most 64) */
    float collapse_node_cost; /* the 8-wide collapse's price of a wide-node visit in triangle tests (0 = 2) */
} rt_scene;

/* rt_scene.accel */
enum {
    RT_ACCEL_AUTO = 0,      /* the library builds the fast walk's BVH: RT_ACCEL_GPU, falling back to RT_ACCEL_HOST;
                               `bvh` serves the strict walk */
    RT_ACCEL_REFERENCE = 1, /* traverse the given `bvh` in both walks */
    RT_ACCEL_GPU = 2,       /* build the fast walk's BVH on the GPU (PLOC over Morton-sorted triangles, rt_build.hpp),
                               then collapse it to the 8-wide quantised layout; falls back to RT_ACCEL_HOST when the
                               tree is too deep for the wide walk (rt_scene_info.accel_built says which) */
    RT_ACCEL_HOST = 3       /* build it on the host: binned SAH (librt_host.so), then the same collapse */
};

/* what rt_upload_scene built (rt_get_scene_info) */
typedef struct rt_scene_info {
    int n_triangles, n_lights;
    int wide_nodes, wide_depth; /* the fast walk's 8-wide BVH (0: none, the binary fast walk) */
    int accel_built;            /* RT_ACCEL_* of the fast walk's BVH as built (RT_ACCEL_HOST = host binned SAH, RT_ACCEL_GPU = PLOC on the device) */
    float build_ms;             /* host wall time of the acceleration build (binary tree + wide collapse) */
    float gpu_build_ms;         /* of which the GPU tree build (RT_ACCEL_GPU; incl. transfers) */
    int unit_triangles;         /* triangles a unit-length ray can hit (|e1 x e2| >= EPSILON: hit_triangle's det cull,
                                   cpu/src/raytracer.c:41-45), indexed by the view reflection and shadow rays walk;
                                   0: that view is the full one */
    int unit_nodes, unit_depth; /* its 8-wide BVH */
    int primary_triangles;      /* triangles a direction of length <= 3 can hit, indexed by the view primary rays walk
                                   when every primary direction of a launch is that short (the reference camera's are
                                   1.87-2.77); 0: no such view (it would leave out < 2 % of the triangles) */
    int primary_nodes;
    /* build_ms by stage, summed over the views: */
    float ploc_ms;     /* the GPU tree builds (PLOC, incl. transfers) */
    float treelet_ms;  /* the treelet restructuring of the GPU-built trees (host threads, rt_treelet.hpp) */
    float collapse_ms; /* the layout and the 8-wide collapse with its quantisation (host threads, rt_wide.cpp) */
} rt_scene_info;

/* rt_frame.kernel */
enum {
    RT_KERNEL_AUTO = 0,   /* RT_KERNEL_FAST */
    RT_KERNEL_STRICT = 1, /* reference-order traversal, exact slab divisions: bit-exact by construction */
    RT_KERNEL_FAST = 2    /* the fast walk (8-wide quantised BVH) in the launch configuration rt_frame.variant
                             names; every variant renders the same bits as RT_KERNEL_STRICT */
};

/* rt_frame.variant: launch configuration of RT_KERNEL_FAST */
enum {
    RT_VARIANT_DEFAULT = 0,  /* the library's rule, measured per frame shape: frame batches and spp > 1 try
                                RT_VARIANT_PERSIST4 and the pool kernel -- RT_VARIANT_SHDEFER where its LDS path buffer
                                fits, else RT_VARIANT_SHPOOL -- three times each on their first launches and keep the
                                faster, by the minimum of each candidate's trials, or by their medians when a
                                candidate's median exceeds 50 ms (RT_VARIANT_PERSIST4 alone where no pool fits); single 1-spp frames
                                run RT_VARIANT_HYBRID (RT_VARIANT_PERSIST where it cannot run); rt_get_launch_info */
    RT_VARIANT_PERSIST = 1,  /* k_persist: one lane per pixel path, walks in lockstep, 3 waves per SIMD */
    RT_VARIANT_PERSIST4 = 2, /* k_persist at 4 waves per SIMD (path levels in LDS) */
    /* 3: the split pipeline (closest chains / shadow batches / resolve), measured slower, removed in round 4: refused */
    RT_VARIANT_COOP2 = 4,    /* k_coop: 2 lanes per ray (shorter chains for small row sets) */
    RT_VARIANT_COOP4 = 5,    /* k_coop: 4 lanes per ray */
    /* 6: k_coop with 8 lanes per ray, 3x slower, removed in round 4: refused */
    /* 7: k_fan (1 + lights lanes per pixel, shadow fan-out), never chosen by a rule nor won a trial, removed in
       round 5: refused */
    /* 8, 9: k_chain (each lane's walks back to back), measured slower and removed in round 2: refused */
    /* 10: k_pool (tile-local LDS ray queues behind workgroup barriers), measured slower, removed in round 4: refused */
    RT_VARIANT_HYBRID = 11,  /* single 1-spp frames: the tiles a measuring frame of the same SHAPE found costliest through
                                k_coop (2 or 4 lanes per ray) on a second stream while k_persist or the shadow pool renders
                                the rest. The first frame of a shape measures (k_persist with per-tile times), the next
                                ones try the candidates -- including the whole-frame kernels -- four frames each, back
                                to back, and the best median of the last three renders from then on, each frame's tile lists built on the device from the
                                previous frame's per-tile times (RT_BUILD_FEEDBACK: a moving camera's lists stay one
                                frame old). Nothing waits on the host: measurements and trials are read by event queries
                                (rt_frame.hot_pct > 0: that threshold and rt_frame.hot_kernel, no trials) */
    /* 12: k_relay (1 + lights waves per tile, LDS hand-off), measured slower, removed in round 4: refused */
    RT_VARIANT_SHPOOL = 13,  /* k_persist at 4 waves per SIMD with each bounce level's shadow rays (every pixel's, every
                                light's) walked as ONE per-wave pool: a lane whose walk ends takes the next unassigned ray,
                                lanes of ended paths included (rt_frame.regroup = idle lanes per refill; 1..32 lights; the
                                LDS path buffer must fit 4 workgroups per CU, else RT_VARIANT_PERSIST4 runs) */
    /* 14: k_stream (a lane whose path ends takes its tile's next pixel; paths at mixed levels), measured slower in
       round 4 (dragon 0.781 vs 0.654 ms per frame in 20-frame batches) and removed: refused */
    RT_VARIANT_SHDEFER = 15  /* RT_VARIANT_SHPOOL with ONE pool for all bounce levels: a wave's paths find their closest
                                hits level by level first, then the shadow rays of every level, pixel and light are walked
                                as one pool and the levels are shaded after it (RT_VARIANT_PERSIST4 where the larger LDS
                                path buffer does not fit) */
};

/* rt_frame.hot_kernel: the kernel RT_VARIANT_HYBRID sends the hot tiles to when rt_frame.hot_pct > 0 */
enum {
    RT_HOT_COOP4 = 0, /* k_coop, 4 lanes per ray */
    RT_HOT_COOP2 = 1  /* k_coop, 2 lanes per ray */
    /* 2: k_fan, removed in round 5; 3: k_relay, removed in round 4: refused */
};

/* rt_frame.dealing: order in which persistent waves take their tiles (k_persist 8x8, k_pool 16x16) */
enum {
    RT_DEAL_DEFAULT = 0,  /* XCD-aware: 4 x 2 regions for batches of full frames, 8 row bands otherwise */
    RT_DEAL_GLOBAL = 1,   /* one counter over the centre-out order */
    RT_DEAL_ROWS = 2,     /* 8 bands of tile rows, band r drained first by the workgroups of XCD r */
    RT_DEAL_COLUMNS = 3,  /* 8 bands of tile columns */
    RT_DEAL_BLOCKS = 4,   /* 4 x 2 blocks */
    RT_DEAL_ROW_MAJOR = 5 /* one counter, row-major tile order */
};

/* Rows rendered: y = row_offset + (k / B) * row_stride + k % B for k in [0, n_rows), B = max(1, row_block)
 * (B = 1: y = row_offset + k * row_stride). Output rows are compact: row k of the output holds image
 * row y. A full frame is {W, H, 0, 1, H, ...}. Rank q of N, cyclic rows: {.., q, N, ..}; block-cyclic
 * rows (blocks of B rows dealt cyclically, so a rank's 8x8 pixel tiles stay 8x8 in the image):
 * {.., q * B, N * B, .., row_block = B}. */
typedef struct rt_frame {
    int width, height;
    int row_offset, row_stride, n_rows;
    int bounces; /* BOUNCES (cpu/include/options.h:52), 1..8; the reference uses 4 */
    int spp;     /* 1 = the reference's pixel-corner ray; s*s = s x s stratified grid, mean of clamped samples */
    int kernel;  /* RT_KERNEL_* */
    int row_block; /* 0 or 1: single rows; B > 1: rows in blocks of B (row_stride >= B) */
    int frame_shift; /* 0: every frame of a batch renders the rows above. S > 0 (RT_KERNEL_FAST only): frame f
                      * of rt_render_frames starts at (row_offset + f * S) % row_stride, so that ranks dealt
                      * block-cyclic rows rotate through every block residue over a batch and their costs
                      * even out; compact rows whose image row falls at or past height are skipped. */
    /* launch configuration (RT_KERNEL_FAST; all zero = the library's defaults) */
    int variant;   /* RT_VARIANT_* */
    int tune;      /* 0 or 1, both the default rule (which measures its candidates itself). Until round 4, 1 selected
                      a separate autotuner whose candidates left out the hybrid launch; it was slower than the default
                      rule on every BASELINE scene and was removed. Other values are refused. */
    int waves_cap; /* persistent grids: at most this many workgroups (4 waves each) per CU; 0 = occupancy limit */
    int dealing;   /* RT_DEAL_* */
    int regroup;   /* RT_VARIANT_SHPOOL: idle lanes of a wave that trigger a refill from the pool; 0 = 16 */
    int hot_pct;   /* RT_VARIANT_HYBRID: tiles whose measured time exceeds hot_pct % of the costliest tile's go to the
                      kernel hot_kernel names; 0 = try several thresholds and hot kernels and keep the fastest */
    int hot_kernel; /* RT_HOT_* (with hot_pct > 0) */
} rt_frame;

/* Device output pointers (all nullable). rgb: [n_rows][width][3] f32 in [0,1] = vec_t pixels
 * (main.c:39); NULL -> a buffer owned by the context (read it with rt_download).
 * hit: [n_rows][width] int32 primary closest-hit triangle index (-1 = miss); t: its distance.
 * bounce_hit: [n_rows][width][bounces] int32 closest-hit triangle index of every recursion level
 * (raytrace(.., iter), raytracer.c:101-135): -1 = miss, -2 = level not reached (first sample when spp > 1).
 * bgra: [n_rows][width] uint32, the pixel quantised as the BMP writer does (vec_to_bgra,
 * cpu/src/bmp_writer.c:88-95: B | G << 8 | R << 16 | 255 << 24, little-endian bytes B,G,R,A) in the frame's
 * top-down row order (the BMP file stores rows bottom-up); written by the kernel itself, so a frame bound for
 * a gather or a file moves 4 bytes per pixel instead of 12. With bgra set and rgb NULL no f32 pixels are
 * written (rt_download of rgb, rt_gather and rt_download_bmp then refuse the frame). */
typedef struct rt_outputs {
    float* rgb;
    int* hit;
    float* t;
    int* bounce_hit;
    unsigned int* bgra;
} rt_outputs;

typedef struct rt_stats {
    unsigned long long primary;        /* primary rays                                     */
    unsigned long long reflection;     /* traced reflection rays                           */
    unsigned long long shadow;         /* traced shadow rays (past the back-face test)     */
    unsigned long long shadow_skipped; /* light_v early-outs (raytracer.c:66-67)           */
    unsigned long long hits;           /* closest-hit rays that hit a triangle             */
    unsigned long long ch_inner, ch_leaf, ch_tri; /* closest-hit interior visits / leaf visits / tri tests (RT_FLAG_COUNTERS) */
    unsigned long long sh_inner, sh_leaf, sh_tri; /* same for shadow rays (RT_FLAG_COUNTERS)             */
    unsigned long long pixels;         /* pixels written                                    */
    unsigned long long fallbacks;      /* fast-kernel rays re-walked strictly (zero direction component or exact tie) */
    unsigned long long stack_overflows; /* must be 0 (rt_get_stats fails otherwise)          */
    unsigned long long node_bytes;     /* BVH node / leaf record bytes read (RT_FLAG_COUNTERS; fused kernels) */
    unsigned long long wave_steps;     /* wave-level wide-node steps (RT_FLAG_COUNTERS): SIMD efficiency =
                                          (ch_inner + sh_inner of the wide walk) / (64 * wave_steps) */
    unsigned long long shadow_wave_steps; /* of which shadow walks' (k_persist's walks; RT_FLAG_COUNTERS)     */
    unsigned long long steps_lanes_16, steps_lanes_32, steps_lanes_48, steps_lanes_64; /* k_persist's wave steps
                                          with 1-16 / 17-32 / 33-48 / 49-64 active lanes (RT_FLAG_COUNTERS)  */
    unsigned long long steps_hist[2][4][4]; /* k_persist's wave steps by walk kind (0 closest: primary + reflection,
                                          1 shadow) x bounce level (0, 1, 2, 3 and deeper) x active lanes (1-16,
                                          17-32, 33-48, 49-64) (RT_FLAG_COUNTERS)                               */
} rt_stats;

int rt_device_count(void);
const char* rt_version(void);

int rt_create(const rt_opts* opts, rt_ctx** out);
/* load_to_gpu(): converts the reference layouts into the device layout and uploads */
int rt_upload_scene(rt_ctx* ctx, const rt_scene* scene);
int rt_get_scene_info(rt_ctx* ctx, rt_scene_info* info);
/* render_frame(): enqueues ONE kernel on the context stream (asynchronous) */
int rt_render(rt_ctx* ctx, const rt_camera* cam, const rt_frame* frame, const rt_outputs* out);
/* A batch of n_frames frames of the same shape (a camera sequence; main.c:141-160's ITERATIONS loop when
 * the cameras are equal): frame i uses cams[i] and writes its outputs at frame offset i, i.e. rgb
 * [n_frames][n_rows][width][3], hit / t [n_frames][n_rows][width], bounce_hit [n_frames][n_rows][width]
 * [bounces]. RT_KERNEL_FAST traces the whole batch in ONE persistent launch whose tile dealing interleaves
 * the frames (the long reflection chains of every frame start first, so one frame's tail overlaps the
 * others' work); other kernels launch once per frame. Each frame equals its rt_render bit for bit; the
 * stats of the call are the batch's sums. rt_gather / rt_download_bmp need a single-frame render. */
int rt_render_frames(rt_ctx* ctx, const rt_camera* cams, int n_frames, const rt_frame* frame,
                     const rt_outputs* out);
/* What the last rt_render / rt_render_frames ran (no synchronisation): the default rule resolves RT_VARIANT_DEFAULT per
 * shape, trying candidates on the first frames of a shape. A caller timing the drop-in seam skips frames until
 * `settled` (the reference's own loop needs no such thing: every frame is bit-exact either way). */
typedef struct rt_launch_info {
    int variant;      /* RT_VARIANT_* the last render ran (0 for RT_KERNEL_STRICT) */
    int hot_pct;      /* RT_VARIANT_HYBRID with hot tiles: the threshold, else 0 */
    int hot_lanes;    /* its lanes per ray (k_coop) or per pixel (k_fan) */
    int cold_variant; /* its kernel of the cold tiles (RT_VARIANT_PERSIST or RT_VARIANT_SHPOOL) */
    int trial;        /* 1: a measuring or trial frame of the default rule */
    int settled;      /* 1: the configuration of this shape is decided: no trial frames follow */
    int refresh;      /* 1: a decided hybrid shape's measuring frame that renews its tile lists (k_persist with per-tile
                         times; settled = 1) -- only where the per-frame feedback is off (PRT_FEEDBACK=0 at build time:
                         a measuring frame every 64 frames of a shape); 0 with it */
    unsigned build;   /* the k_persist instantiation that ran (of the cold tiles, for a hybrid launch): RT_BUILD_* bits;
                         0 for the other kernels (strict, k_coop alone) */
} rt_launch_info;
/* rt_launch_info.build */
enum {
    RT_BUILD_WAVES4 = 1,       /* 4 waves per SIMD (<= 128 VGPRs); else 3 */
    RT_BUILD_PACKED_STACK = 2, /* 5-byte wide-stack entries */
    RT_BUILD_PACKED_TRIS = 4,  /* packed triangle tests through the wave's LDS queue */
    RT_BUILD_LDS_PATHS = 8,    /* the path levels in LDS (else a global slab, or registers at 3 waves) */
    RT_BUILD_POOL_LEVEL = 16,  /* the per-level shadow pool (RT_VARIANT_SHPOOL) */
    RT_BUILD_POOL_ALL = 32,    /* one shadow pool for all levels (RT_VARIANT_SHDEFER) */
    RT_BUILD_TRACE = 64,       /* the measuring build with per-tile times */
    RT_BUILD_FEEDBACK = 128    /* a decided single-frame shape's frame dealt by the previous frame's per-tile times, its
                                  tile lists built on the device (no measuring frames, no host round trip) */
};
int rt_get_launch_info(rt_ctx* ctx, rt_launch_info* info);
/* load_from_gpu(): copies the last frame's compact rows to host (synchronous); nullable args. RT_E_KERNEL when the
 * render reported a traversal-stack overflow (its frame is not valid). */
int rt_download(rt_ctx* ctx, float* h_rgb, int* h_hit);
/* waits for the stream; kernel_ms (nullable) = the last render's kernel time from HIP events; RT_E_KERNEL when the
 * last render reported a traversal-stack overflow */
int rt_sync(rt_ctx* ctx, float* kernel_ms);
/* per-launch kernel times (HIP events recorded on the context stream around each kernel) of the last
 * n launches (n <= 64), oldest first; synchronises; returns the number written or < 0 */
int rt_kernel_times(rt_ctx* ctx, float* ms, int n);
/* Multi-GPU in one process without RCCL (the fallback of the CLI's --gpus N; also several contexts on ONE
 * device): gathers the last render of n contexts -- a frame or a frame batch, f32 rgb or BGRA8 (rt_outputs.bgra),
 * the same kind on every context -- into ctxs[root]'s full frames [frames][height][width]. Every context must
 * have rendered the same shape, and their row sets must partition each frame (rank g of n: cyclic rows
 * {g, n}, block-cyclic rows {g*B, n*B, .., row_block = B}, rotated residues with frame_shift).
 * Each source's xGMI peer copies are issued on ITS stream after its render (the sources' copy engines run at
 * once), the root waits for them (events) and un-interleaves the rows. Afterwards the root's last render is
 * the full frame(s) (rgb or bgra, and hit when every context wrote one): rt_download / rt_download_bmp read a
 * single frame. Asynchronous like rt_render. */
int rt_gather(rt_ctx* const* ctxs, int n, int root);
/* rt_gather into a caller's device buffer d_dst on the root's device ([frames][height][width] x 3 floats or
 * x 1 uint32, the last renders' kind), e.g. to keep a gathered frame batch; d_dst NULL = rt_gather */
int rt_gather_to(rt_ctx* const* ctxs, int n, int root, void* d_dst);

/* RCCL communicator over contexts (the framebuffer gather over xGMI). Two ways to build one:
 *   rt_comm_init      -- one process driving n devices (the CLI's --gpus N): ncclCommInitAll over the contexts'
 *                        devices, rank i = ctxs[i] (one context per device);
 *   rt_comm_init_rank -- one rank per process (N processes, one GPU each): ncclCommInitRank with an id that
 *                        rank 0 made with rt_comm_get_id and handed to every rank (any channel: MPI, a file,
 *                        torch.distributed). One communicator per rank serves every context of that rank on its
 *                        device (rt_comm_gather_from).
 * rt_comm_gather(comm, root, d_dst): every rank's last render (a frame or frame batch, rgb or BGRA8; the row
 * sets must partition each frame, as for rt_gather) is sent to `root` with ncclSend / ncclRecv in one group,
 * on each context's stream (so after its render), and un-interleaved there into d_dst ([frames][height][width]
 * x 3 floats or x 1 uint32; a device pointer on the root's device) or, with d_dst NULL, into the root
 * context's own buffer, which then is its last render (rt_download / rt_download_bmp). Collective: every rank
 * calls it. Asynchronous on the streams. Hit indices are not gathered (rt_gather does).
 * Across processes the ranks exchange their 64-B row-set descriptors (one ncclAllGather, a host wait) only on what
 * every rank sees the same way: the first gather, a new frame size, frame count or pixel kind (fields every rank of
 * a valid layout shares), or rt_comm_relayout called by every rank. A rank whose own rows change without one of
 * those is refused (RT_E_ARG) before any collective call. The root checks each exchanged layout partitions every
 * frame and, on the layout's first gather, that every pixel of the gathered frames arrived (one host wait per
 * layout); later gathers of the same layout neither exchange nor wait. Every host wait on a collective is bounded
 * (rt_comm_set_timeout, default 120 s): a peer that never joins turns into RT_E_TIMEOUT and an aborted communicator
 * (ncclCommAbort), never a hang. */
typedef struct rt_comm rt_comm;
#define RT_COMM_ID_BYTES 128 /* sizeof(ncclUniqueId) */
typedef struct rt_comm_info {
    long long gathers;   /* rt_comm_gather / rt_comm_gather_from calls */
    long long exchanges; /* row-set descriptor exchanges (multi-process): one per layout */
    long long checked;   /* layouts whose first gather the root checked pixel by pixel */
    int nranks, rank;    /* the job's ranks; this communicator's (first local) rank */
} rt_comm_info;
int rt_comm_get_id(unsigned char* id /* RT_COMM_ID_BYTES */);
int rt_comm_init(rt_ctx* const* ctxs, int n, rt_comm** out);
int rt_comm_init_rank(rt_ctx* ctx, int nranks, int rank, const unsigned char* id, rt_comm** out);
int rt_comm_gather(rt_comm* comm, int root, void* d_dst);
/* rt_comm_gather of the last render of `src`, a context of this rank on the communicator's device (NULL: the
 * context the communicator was built with); multi-process communicators only. Successive gathers of one
 * communicator run in their call order, whatever streams their contexts use. */
int rt_comm_gather_from(rt_comm* comm, rt_ctx* src, int root, void* d_dst);
/* Collective: every rank calls it before the same gather, which then exchanges the row sets again (a rank's rows
 * may change there). */
int rt_comm_relayout(rt_comm* comm);
/* The deadline of every host wait on a collective of this communicator (seconds > 0; default 120). */
int rt_comm_set_timeout(rt_comm* comm, double seconds);
/* Waits, bounded by that deadline, until the communicator's last gather has run on the device: RT_OK, or
 * RT_E_TIMEOUT with the communicator aborted (a peer never joined). For a caller that would otherwise block in a
 * device synchronisation behind a collective that cannot complete. */
int rt_comm_wait(rt_comm* comm);
int rt_comm_get_info(rt_comm* comm, rt_comm_info* info);
const char* rt_comm_last_error(rt_comm* comm);
void rt_comm_destroy(rt_comm* comm);
/* bmp_write_file's bytes of the last frame (cpu/src/bmp_writer.c:88-211): 54-B header + BGRA8 rows
 * bottom-up, (uint8_t)(c * 255.0f) per channel (vec_to_bgra), quantised on the device. Needs a full
 * frame (all rows; after rt_gather for multi-GPU). cap >= 54 + 4 * width * height; synchronous. */
int rt_download_bmp(rt_ctx* ctx, unsigned char* h_bmp, size_t cap);
/* counters of the last rendered frame (synchronises) */
int rt_get_stats(rt_ctx* ctx, rt_stats* stats);
const char* rt_last_error(rt_ctx* ctx);
void rt_destroy(rt_ctx* ctx);

#ifdef __cplusplus
}
#endif
#endif
