// rt_comm_logic.hpp — the host-side decisions of the multi-process framebuffer gather (rt_comm_gather_from,
// rt_hip.hip), kept free of HIP and RCCL so that tests/c/comm_logic_test.cpp can check them with g++ alone:
//   * Part / check_parts: a rank's row-set descriptor and the root's check that the ranks' rows partition every frame
//     (the gather replaces gpu/src/gpu.cu:203-228's single-device load_from_gpu);
//   * layout_step: when the ranks exchange their descriptors (one ncclAllGather) -- a decision every rank must take
//     the same way, or one rank waits in the AllGather while its peers post their sends and receives;
//   * bounded_wait: a host wait on a collective with a deadline, so that a peer that never arrives turns into an
//     error (the caller aborts the communicator) instead of a process that hangs until something kills it.
#pragma once
#include <algorithm>
#include <chrono>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

namespace rtc {

// One rank's part of a gathered frame batch: its last render's compact rows (rt_frame) and payload. 16 ints: the
// descriptor the RCCL ranks of different processes exchange.
struct Part {
    int W, H, frames, rows, off, stride, block, shift;
    int words;  // 32-bit words per pixel: 1 = BGRA8 (rt_outputs.bgra), 3 = f32 rgb
    int hit;    // 1: the render wrote hit indices too (never gathered across processes: not part of the layout)
    int pad[6];
};
static_assert(sizeof(Part) == 64, "descriptor size");

inline size_t part_px(const Part& p) { return (size_t)p.frames * p.rows * p.W; }

// "" when the parts' rows partition every frame of the batch (rows a rotated rank renders past the image are
// skipped), else what is wrong
inline std::string check_parts(const std::vector<Part>& ps) {
    if (ps.empty()) return "no ranks";
    for (const Part& p : ps)
        if (p.W <= 0 || p.H <= 0) return "a rank has not rendered";
    const Part& a = ps[0];
    std::vector<char> cover((size_t)a.H);
    for (const Part& p : ps) {
        if (p.W != a.W || p.H != a.H) return "frame sizes differ";
        if (p.frames != a.frames) return "frame counts differ";
        if (p.words != a.words) return "outputs differ (bgra vs rgb)";
        if (p.rows < 0 || p.stride < 1 || p.block < 1) return "bad row set";
    }
    for (int f = 0; f < a.frames; f++) {
        std::fill(cover.begin(), cover.end(), 0);
        for (const Part& p : ps) {
            const long long start = p.shift ? (p.off + (long long)f * p.shift) % p.stride : p.off;
            for (int k = 0; k < p.rows; k++) {
                const long long y = start + (long long)(k / p.block) * p.stride + k % p.block;
                if (y >= a.H && p.shift) continue;
                if (y < 0 || y >= a.H || cover[y]) return "row sets do not partition the frame";
                cover[y] = 1;
            }
        }
        for (char v : cover)
            if (!v) return "row sets do not cover the frame";
    }
    return "";
}

// The fields every rank of a valid layout shares (check_parts refuses anything else): a change of one of them is a
// change on every rank at the same gather, so the ranks decide to exchange together.
inline bool same_uniform(const Part& a, const Part& b) {
    return a.W == b.W && a.H == b.H && a.frames == b.frames && a.words == b.words;
}
// This rank's own rows (they differ between ranks and need not change together).
inline bool same_rows(const Part& a, const Part& b) {
    return a.rows == b.rows && a.off == b.off && a.stride == b.stride && a.block == b.block && a.shift == b.shift;
}

enum class Step {
    Exchange,     // every rank exchanges its descriptor before this gather (collective)
    Reuse,        // the layout of the last exchange holds: no exchange, no host wait
    RowsChanged   // this rank's rows changed but nothing every rank sees did: refused (rt_comm_relayout first)
};
// have: a layout was exchanged (and not invalidated by rt_comm_relayout); last: this rank's part at that exchange.
// Decided only from what every rank sees the same way (the first gather, the uniform fields, a collective
// rt_comm_relayout), never from a field one rank may change alone (its hit output, its own rows).
inline Step layout_step(const Part& mine, const Part& last, bool have) {
    if (!have || !same_uniform(mine, last)) return Step::Exchange;
    return same_rows(mine, last) ? Step::Reuse : Step::RowsChanged;
}

enum class Wait { Done, Error, Timeout };
// Polls query() -- 0: complete, 1: not yet, < 0: an error (returned in err) -- until it completes, fails, or
// timeout_s seconds have passed; spins for the first ~200 us, then sleeps 50 us between polls. On Timeout the
// caller aborts the collective (ncclCommAbort) and reports RT_E_TIMEOUT.
template <class Query>
Wait bounded_wait(Query query, double timeout_s, int& err) {
    using clk = std::chrono::steady_clock;
    const auto t0 = clk::now();
    for (;;) {
        const int q = query();
        if (q == 0) return Wait::Done;
        if (q < 0) {
            err = q;
            return Wait::Error;
        }
        const double el = std::chrono::duration<double>(clk::now() - t0).count();
        if (el >= timeout_s) return Wait::Timeout;
        if (el > 2e-4) std::this_thread::sleep_for(std::chrono::microseconds(50));
    }
}

// A communicator's outstanding send / recv groups, waited for in issue order (rt_comm_wait, the exchange and coverage
// waits of a gather, and any host wait on a stream that holds a group: rt_sync, rt_download, ...). Group j's local
// part -- the render before it, marked by its `pre` event -- depends only on this rank's own work once group j - 1 has
// completed, so it is waited for without a deadline; the deadline covers the collective itself and starts when the
// local part has completed. A long render (a 64-spp 4K frame) therefore never turns into a timeout, and a peer that
// never joins still does. pre(j) / done(j): 0 complete, 1 not yet, < 0 an error (returned in err).
// Returns Done with n_done = n, else the Error or Timeout of group n_done (groups 0 .. n_done - 1 completed).
template <class PreQ, class DoneQ>
Wait settle(int n, PreQ pre, DoneQ done, double timeout_s, int& err, int& n_done) {
    using clk = std::chrono::steady_clock;
    n_done = 0;
    for (int j = 0; j < n; j++) {
        const auto t0 = clk::now();
        for (;;) {  // the local part: no deadline (spin ~200 us, then sleep between polls)
            const int q = pre(j);
            if (q == 0) break;
            if (q < 0) {
                err = q;
                return Wait::Error;
            }
            if (std::chrono::duration<double>(clk::now() - t0).count() > 2e-4)
                std::this_thread::sleep_for(std::chrono::microseconds(50));
        }
        const Wait w = bounded_wait([&] { return done(j); }, timeout_s, err);
        if (w != Wait::Done) return w;
        n_done = j + 1;
    }
    return Wait::Done;
}

}  // namespace rtc
