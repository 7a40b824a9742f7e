// raytracer — command-line drop-in for the reference's cpu/raytracer (cpu/src/main.c:90-212).
//
//   raytracer [threads] [ntris] [--scene NAME] [--assets DIR] [--width W] [--height H]
//             [--bounces B] [--iterations K] [--warmup W] [--bvh-heuristic H] [--seed S]
//             [--gpus N] [--gather auto|rccl|peer] [--spp S] [--kernel fast|strict|VARIANT]
//             [--out FILE.bmp] [--cache DIR]
//   VARIANT: persist, persist4, coop2, coop4, hybrid, shpool, shdefer (rt_frame.variant; the fast
//   kernel's launch configurations, all rendering the same bits; default: the library's measured rule)
//
// Positional arguments and defaults are the reference's (options.h: 1920x1080, car_boxed, BOUNCES 4,
// ITERATIONS 1, BVH_HEURISTIC 3, SEED 1; main.c:97-131: `threads` in 1..63, `ntris` = random mode).
// Scenes load from <assets>/<scene>/{triangles.obj,triangles.mtl,lights.obj}, default assets "../assets"
// as in main.c:113-114. The frame renders on the GPU(s) through the rt_* C-ABI; with --gpus N the
// rows are dealt over N devices in 8-row blocks (one rt_ctx each, one host thread each) and gathered on
// GPU 0 with RCCL (rt_comm_gather; --gather peer: xGMI peer copies, rt_gather; --gather rccl at one GPU
// runs the RCCL path over a one-rank communicator). Output: <scene>.bmp (main.c:191, quantised on the GPU) and the reference's stdout metric
// lines, plus ray counts. --cache DIR keeps the parsed triangles and the BVH in binary cache files
// (rth_*_cached: identical results, no re-parse / re-build of unchanged scenes).
#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "rt_hip.h"
#include "rt_host.h"

namespace {

struct Args {
    int threads = 1;
    long ntris = -1;
    std::string scene = "car_boxed", assets = "../assets", out, kernel = "fast", cache, gather = "auto";
    int W = 1920, H = 1080, bounces = 4, iterations = 1, warmup = 0, heuristic = 3, gpus = 1, spp = 1;
    unsigned seed = 1;
};

[[noreturn]] void usage(const char* msg) {
    std::fprintf(stdout, "%s\n", msg);
    std::exit(-1);
}

Args parse(int argc, char** argv) {
    Args a;
    std::vector<std::string> pos;
    for (int i = 1; i < argc; i++) {
        std::string s = argv[i];
        auto val = [&](void) -> std::string {
            if (i + 1 >= argc) usage(("missing value for " + s).c_str());
            return argv[++i];
        };
        if (s == "--scene") a.scene = val();
        else if (s == "--assets") a.assets = val();
        else if (s == "--width") a.W = std::atoi(val().c_str());
        else if (s == "--height") a.H = std::atoi(val().c_str());
        else if (s == "--bounces") a.bounces = std::atoi(val().c_str());
        else if (s == "--iterations") a.iterations = std::atoi(val().c_str());
        else if (s == "--warmup") a.warmup = std::atoi(val().c_str());
        else if (s == "--bvh-heuristic") a.heuristic = std::atoi(val().c_str());
        else if (s == "--seed") a.seed = (unsigned)std::strtoul(val().c_str(), nullptr, 10);
        else if (s == "--gpus") a.gpus = std::atoi(val().c_str());
        else if (s == "--spp") a.spp = std::atoi(val().c_str());
        else if (s == "--kernel") a.kernel = val();
        else if (s == "--out") a.out = val();
        else if (s == "--gather") a.gather = val();
        else if (s == "--cache") a.cache = val();
        else if (s.rfind("--", 0) == 0) usage(("unknown option " + s).c_str());
        else pos.push_back(s);
    }
    if (pos.size() >= 1) {  // main.c:97-103
        a.threads = std::atoi(pos[0].c_str());
        if (a.threads <= 0 || a.threads >= 64) usage("Invalid number of threads");
    }
    if (pos.size() == 2) a.ntris = std::atol(pos[1].c_str());  // main.c:112-131 (argc == 3)
    if (a.W <= 0 || a.H <= 0 || a.iterations <= 0 || a.gpus <= 0) usage("invalid frame settings");
    if (a.gather != "auto" && a.gather != "rccl" && a.gather != "peer") usage("--gather: auto, rccl or peer");
    if (a.out.empty()) a.out = a.scene + ".bmp";
    return a;
}

double median(std::vector<double> v) {  // main.c:50-64
    std::sort(v.begin(), v.end());
    size_t n = v.size();
    return n % 2 ? v[n / 2] : (v[n / 2 - 1] + v[n / 2]) / 2.0;
}

}  // namespace

int main(int argc, char** argv) {
    Args a = parse(argc, argv);
    rth_rng rng;
    rth_srand(&rng, a.seed);  // main.c:91-95

    std::printf("Loading scene...\n");
    rt_triangle* tris = nullptr;
    size_t n = 0;
    rt_light* lights = nullptr;
    size_t nl = 0;
    if (a.ntris < 0) {
        std::string d = a.assets + "/" + a.scene + "/";
        const std::string tc = a.cache.empty() ? "" : a.cache + "/" + a.scene + ".tris.prtc";
        if (rth_triangles_load_cached((d + "triangles.obj").c_str(), (d + "triangles.mtl").c_str(),
                                      tc.empty() ? nullptr : tc.c_str(), &tris, &n, nullptr) != RT_OK)
            return EXIT_FAILURE;  // the loader printed "cannot load <file>" (triangle.c:29-30)
        if (rth_lights_load((d + "lights.obj").c_str(), &lights, &nl) != RT_OK) return EXIT_FAILURE;
    } else if (rth_triangles_random((size_t)a.ntris, &rng, &tris) == RT_OK) {
        n = (size_t)a.ntris;
    }

    std::printf("Building BVH...\n");
    auto t0 = std::chrono::steady_clock::now();
    rt_bvh_node* bvh = nullptr;
    int bvh_len = 0;
    int* tri_idx = nullptr;
    rth_bvh_stats bs{};
    const std::string bc = a.cache.empty() || a.ntris >= 0
                               ? ""
                               : a.cache + "/" + a.scene + ".bvh" + std::to_string(a.heuristic) + ".prtc";
    int rc = rth_bvh_build_cached(tris, n, a.heuristic, &rng, bc.empty() ? nullptr : bc.c_str(), &bvh, &bvh_len,
                                  &tri_idx, &bs, nullptr);
    if (rc == RT_E_EMPTY) return EXIT_FAILURE;  // "no triangles, cannot build bvh." (bvh.c:361-364)
    if (rc != RT_OK) usage("bvh build failed (heuristic must be 0, 1, 3, 6 or 16)");
    double bvh_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    std::printf("min number of triangle: %d\n", bs.min_leaf);  // bvh.c:381-387
    std::printf("max number of triangle: %d\n", bs.max_leaf);
    std::printf("avg number of triangle: %.2f\n", (float)bs.avg_leaf);
    std::printf("number of leaf: %d\n", bs.leaves);
    std::printf("bvh size (bytes): %lu\n", (unsigned long)(sizeof(rt_bvh_node) * bvh_len));
    std::printf("bvh built in %.3f ms\n", bvh_ms);
    std::printf("\n# BVH settings #\nMax depth: %d\nLeaf size threshold: %d\nSplit heuristic: %d\nSeed: %u\n"
                "Fast light: %d\n", 32, 2, a.heuristic, a.seed, 1);

    int ndev = rt_device_count();
    if (ndev <= 0) {
        std::fprintf(stderr, "no GPU visible: this renderer runs the hot path on MI355X only\n");
        return EXIT_FAILURE;
    }
    if (a.gpus > ndev) usage("--gpus exceeds the visible devices");
    std::printf("\n# Host settings #\nNumber of threads: %d\nNumber of GPUs: %d\n", a.threads, a.gpus);
    std::printf("\n# Scene complexity #\nResolution: %d x %d\nNumber of triangles: %zu\nNumber of lights: %zu\n"
                "Number of ray bounces: %d\n",
                a.W, a.H, n, nl, a.bounces);

    rt_scene sc{tris, (int)n, bvh, bvh_len, tri_idx, lights, (int)nl, rt_vec3{0.5f, 0.5f, 0.5f}};
    rt_camera cam;
    rth_camera(a.W, a.H, &cam);
    const int G = a.gpus;
    std::vector<rt_ctx*> ctx(G, nullptr);
    for (int g = 0; g < G; g++) {
        rt_opts o{g, 0, nullptr};
        if (rt_create(&o, &ctx[g]) != RT_OK || rt_upload_scene(ctx[g], &sc) != RT_OK) {
            std::fprintf(stderr, "GPU %d: %s\n", g, ctx[g] ? rt_last_error(ctx[g]) : "rt_create failed");
            return EXIT_FAILURE;
        }
    }
    static const struct {
        const char* name;
        int variant;
    } variants[] = {{"fast", RT_VARIANT_DEFAULT}, {"persist", RT_VARIANT_PERSIST}, {"persist4", RT_VARIANT_PERSIST4},
                    {"coop2", RT_VARIANT_COOP2},  {"coop4", RT_VARIANT_COOP4},
                    {"hybrid", RT_VARIANT_HYBRID}, {"shpool", RT_VARIANT_SHPOOL}, {"shdefer", RT_VARIANT_SHDEFER}};
    int kern = a.kernel == "strict" ? RT_KERNEL_STRICT : -1, variant = RT_VARIANT_DEFAULT;
    for (const auto& v : variants)
        if (kern < 0 && a.kernel == v.name) {
            kern = RT_KERNEL_FAST;
            variant = v.variant;
        }
    if (kern < 0) {
        std::fprintf(stderr, "unknown --kernel %s\n", a.kernel.c_str());
        return EXIT_FAILURE;
    }
    // the frame gather: RCCL over the G devices (one communicator per device, one process) by default at G > 1
    rt_comm* comm = nullptr;
    if (a.gather == "rccl" || (a.gather == "auto" && G > 1)) {
        if (rt_comm_init(ctx.data(), G, &comm) != RT_OK) {
            std::fprintf(stderr, "RCCL communicator: %s; gathering with peer copies\n", rt_last_error(ctx[0]));
            comm = nullptr;
        }
    }
    std::printf("Frame gather: %s\n", comm ? "RCCL" : G > 1 ? "peer copies" : "none (one GPU)");
    std::vector<float> frame((size_t)a.W * a.H * 3);
    unsigned long long rays = 0;
    auto render_all = [&]() {
        std::vector<std::thread> th;
        std::vector<int> status(G, 0);
        for (int g = 0; g < G; g++)
            th.emplace_back([&, g] {
                // 8-row blocks dealt cyclically to the GPUs (prt/dist.py::rank_rows): a GPU's 8x8 tiles stay
                // 8x8 image tiles; one GPU renders the frame as single rows
                const int B = G > 1 ? 8 : 1, nb = (a.H + B - 1) / B;
                int nr = 0;
                for (int j = g; j < nb; j += G) nr += std::min(B, a.H - j * B);
                rt_frame f{a.W, a.H, g * B, G * B, nr, a.bounces, a.spp, kern, B};
                f.variant = variant;
                int s = rt_render(ctx[g], &cam, &f, nullptr);
                if (s == RT_OK) s = rt_sync(ctx[g], nullptr);
                status[g] = s;
            });
        for (auto& t : th) t.join();
        for (int g = 0; g < G; g++)
            if (status[g] != RT_OK) {
                std::fprintf(stderr, "GPU %d: %s\n", g, rt_last_error(ctx[g]));
                std::exit(EXIT_FAILURE);
            }
    };
    std::printf("\nRendering...\n");
    for (int i = 0; i < a.warmup; i++) render_all();
    std::vector<double> times;
    for (int i = 0; i < a.iterations; i++) {  // main.c:171-185
        auto s = std::chrono::steady_clock::now();
        render_all();
        // every GPU's 8-row blocks -> GPU 0's frame: RCCL send / recv over xGMI (rt_comm_gather), or xGMI peer
        // copies (rt_gather) when RCCL is not wanted or not available; then to the host
        int gs = RT_OK;
        if (comm) gs = rt_comm_gather(comm, 0, nullptr);
        else if (G > 1) gs = rt_gather(ctx.data(), G, 0);
        if (gs != RT_OK || rt_download(ctx[0], frame.data(), nullptr) != RT_OK) {
            std::fprintf(stderr, "gather: %s\n", comm ? rt_comm_last_error(comm) : rt_last_error(ctx[0]));
            return EXIT_FAILURE;
        }
        double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - s).count();
        times.push_back(ms);
        std::printf("Iteration %d completed in %.3f ms\n", i + 1, ms);
    }
    rays = 0;
    for (int g = 0; g < G; g++) {
        rt_stats st;
        rt_get_stats(ctx[g], &st);
        rays += st.primary + st.reflection + st.shadow;
    }
    {  // main.c:191 bmp_write_file: quantised on GPU 0 (rt_download_bmp), written by the host
        std::vector<unsigned char> bmp(54 + (size_t)4 * a.W * a.H);
        if (rt_download_bmp(ctx[0], bmp.data(), bmp.size()) != RT_OK) {
            std::fprintf(stderr, "bmp: %s\n", rt_last_error(ctx[0]));
            return EXIT_FAILURE;
        }
        FILE* fo = std::fopen(a.out.c_str(), "wb");
        if (!fo || std::fwrite(bmp.data(), 1, bmp.size(), fo) != bmp.size()) return -1;
        std::fclose(fo);
    }

    double mean = 0;  // main.c:193-209
    for (double t : times) mean += t;
    mean /= times.size();
    double var = 0;
    for (double t : times) var += (t - mean) * (t - mean);
    double sd = std::sqrt(var / times.size());
    double ci = 2.5758293035489004 * sd / std::sqrt((double)times.size());
    std::printf("\n# Metrics #\n");
    std::printf("Total execution time of %d frames: %.3f ms\n", a.iterations, mean * a.iterations);
    if (a.iterations >= 30)
        std::printf("Frame time (mean +/- 99%% CI): %.3f +/- %.3f = [%.3f, %.3f] ms\n", mean, ci, mean - ci, mean + ci);
    else
        std::printf("Frame time (mean): %.3f ms\n", mean);
    std::printf("Frame time (median): %.3f ms\n", median(times));
    std::printf("Frame time (stddev): %.3f ms^2\n", sd);
    std::printf("Expected FPS: %.3f\n", 1000 / mean);
    std::printf("Rays per frame (primary+reflection+shadow): %llu\n", rays);
    std::printf("Throughput: %.1f Mrays/s\n", rays / (median(times) / 1e3) / 1e6);
    rt_comm_destroy(comm);
    for (auto* c : ctx) rt_destroy(c);
    rth_free(tris);
    rth_free(lights);
    rth_free(bvh);
    rth_free(tri_idx);
    return 0;
}
