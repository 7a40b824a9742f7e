// Host-only checks of the multi-process gather's decisions (parallel-ray-tracer_amd/csrc/hip/rt_comm_logic.hpp),
// compiled with plain g++ by tests/test_comm_logic.py: no GPU, no HIP, no RCCL.
//   * bounded_wait over a stub "stream" that never completes returns Timeout after the deadline (and the caller's
//     abort runs once), one that completes returns Done, one that fails returns Error;
//   * layout_step: two ranks, one of which toggles its hit output between gathers, take the same decision (Reuse),
//     so neither waits in an AllGather the other never posts; frame-count changes make both exchange; a rank whose
//     rows alone changed is refused before any collective call;
//   * check_parts on block-cyclic and rotated layouts.
#include <cstdio>
#include <cstdlib>

#include "rt_comm_logic.hpp"

static int failures = 0;
#define CHECK(c)                                                          \
    do {                                                                  \
        if (!(c)) {                                                       \
            std::fprintf(stderr, "FAIL %s:%d: %s\n", __FILE__, __LINE__, #c); \
            failures++;                                                   \
        }                                                                 \
    } while (0)

using rtc::Part;

// a rank's part: rows block-cyclic over n ranks in blocks of b (prt/dist.py rank_rows)
static Part part(int W, int H, int frames, int q, int n, int b, int words = 1, int hit = 0, int shift = 0) {
    Part p{};
    p.W = W;
    p.H = H;
    p.frames = frames;
    int rows = 0;
    for (int y = 0; y < H; y++)
        if ((y / b) % n == q) rows++;
    if (shift) {  // rotated residues: every rank renders the largest rank's row count
        rows = 0;
        for (int y = 0; y < H; y++)
            if ((y / b) % n == 0) rows++;
    }
    p.rows = rows;
    p.off = q * b;
    p.stride = n * b;
    p.block = b;
    p.shift = shift;
    p.words = words;
    p.hit = hit;
    return p;
}

// the library's comm_wait, reduced to its logic: a bounded wait whose timeout aborts the communicator once
struct StubComm {
    bool aborted = false;
    int aborts = 0;
    double timeout_s = 0.2;
    template <class Q>
    int wait(Q q) {
        int err = 0;
        const rtc::Wait w = rtc::bounded_wait(q, timeout_s, err);
        if (w == rtc::Wait::Done) return 0;
        if (w == rtc::Wait::Error) return err;
        aborted = true;
        aborts++;
        return -9;  // RT_E_TIMEOUT
    }
};

int main() {
    using clk = std::chrono::steady_clock;
    {  // a stream that never completes: Timeout after the deadline, the abort once
        StubComm cm;
        long long polls = 0;
        const auto t0 = clk::now();
        const int rc = cm.wait([&] {
            polls++;
            return 1;
        });
        const double el = std::chrono::duration<double>(clk::now() - t0).count();
        CHECK(rc == -9);
        CHECK(cm.aborted && cm.aborts == 1);
        CHECK(el >= 0.2 && el < 2.0);
        CHECK(polls > 10);
        std::printf("never-completing stub: timeout after %.3f s, %lld polls, aborted %d time(s)\n", el, polls, cm.aborts);
    }
    {  // completes after 5 polls: Done, no abort
        StubComm cm;
        int n = 0;
        CHECK(cm.wait([&] { return ++n >= 5 ? 0 : 1; }) == 0);
        CHECK(!cm.aborted && n == 5);
    }
    {  // an error: reported, no abort
        StubComm cm;
        CHECK(cm.wait([&] { return -700; }) == -700);
        CHECK(!cm.aborted);
    }
    {  // settle: a render (the local part) far longer than the timeout does not abort; the collective after it is bounded
        using ms = std::chrono::milliseconds;
        const double timeout = 0.05;
        const auto t0 = clk::now();
        auto at = [&](double s) { return std::chrono::duration<double>(clk::now() - t0).count() >= s ? 0 : 1; };
        int err = 0, n_done = -1;
        // group 0: render done at 0.30 s (6x the timeout), collective 10 ms later; group 1: render at 0.35, done 0.36
        const double pre_t[2] = {0.30, 0.35}, done_t[2] = {0.31, 0.36};
        rtc::Wait w = rtc::settle(2, [&](int j) { return at(pre_t[j]); }, [&](int j) { return at(done_t[j]); }, timeout,
                                  err, n_done);
        const double el = std::chrono::duration<double>(clk::now() - t0).count();
        CHECK(w == rtc::Wait::Done && n_done == 2);
        CHECK(el >= 0.36 && el < 2.0);
        std::printf("settle: a 0.30 s render under a %.2f s timeout completes (%.3f s)\n", timeout, el);
        // a peer that never joins group 1: group 0 completes, group 1 times out one timeout after its render
        const auto t1 = clk::now();
        auto since = [&](double s) { return std::chrono::duration<double>(clk::now() - t1).count() >= s ? 0 : 1; };
        w = rtc::settle(2, [&](int j) { return since(j == 0 ? 0.02 : 0.1); }, [&](int j) { return j == 0 ? since(0.03) : 1; },
                        timeout, err, n_done);
        const double el1 = std::chrono::duration<double>(clk::now() - t1).count();
        CHECK(w == rtc::Wait::Timeout && n_done == 1);
        CHECK(el1 >= 0.1 + timeout && el1 < 2.0);
        // an error in a render: reported as such
        w = rtc::settle(1, [&](int) { return -700; }, [&](int) { return 0; }, timeout, err, n_done);
        CHECK(w == rtc::Wait::Error && err == -700 && n_done == 0);
        (void)ms(0);
    }
    {  // layout decisions of two ranks over a gather sequence; rank 1 toggles its hit output
        const int W = 64, H = 40;
        Part last[2] = {};
        bool have[2] = {false, false};
        struct G {
            int frames, hit1;
        };
        const G seq[] = {{4, 0}, {4, 1}, {4, 0}, {2, 0}, {2, 1}, {2, 1}};
        const rtc::Step want[] = {rtc::Step::Exchange, rtc::Step::Reuse, rtc::Step::Reuse,
                                  rtc::Step::Exchange, rtc::Step::Reuse, rtc::Step::Reuse};
        for (int g = 0; g < 6; g++) {
            rtc::Step st[2];
            for (int q = 0; q < 2; q++) {
                const Part mine = part(W, H, seq[g].frames, q, 2, 8, 1, q == 1 ? seq[g].hit1 : 0);
                st[q] = rtc::layout_step(mine, last[q], have[q]);
                if (st[q] == rtc::Step::Exchange) {
                    last[q] = mine;
                    have[q] = true;
                }
            }
            CHECK(st[0] == st[1]);  // the ranks agree: no rank alone in a collective
            CHECK(st[0] == want[g]);
        }
        // rank 0's rows alone change (no size / count / kind change): refused locally, before any collective
        Part moved = last[0];
        moved.off = 8;
        CHECK(rtc::layout_step(moved, last[0], true) == rtc::Step::RowsChanged);
        // ... unless every rank called rt_comm_relayout (have = false): all exchange
        CHECK(rtc::layout_step(moved, last[0], false) == rtc::Step::Exchange);
        // a pixel-kind change (bgra -> rgb) is one every rank sees
        Part rgb = last[0];
        rgb.words = 3;
        CHECK(rtc::layout_step(rgb, last[0], true) == rtc::Step::Exchange);
    }
    {  // check_parts: block-cyclic layouts partition; a missing rank or an overlap does not
        const int W = 32, H = 1080;
        for (int n : {1, 2, 3, 4, 8})
            for (int b : {1, 8}) {
                std::vector<Part> ps;
                for (int q = 0; q < n; q++) ps.push_back(part(W, H, 3, q, n, b));
                CHECK(rtc::check_parts(ps).empty());
                if (n > 1) {
                    std::vector<Part> miss(ps.begin(), ps.end() - 1);
                    CHECK(!rtc::check_parts(miss).empty());
                    std::vector<Part> dup = ps;
                    dup[1] = dup[0];
                    CHECK(!rtc::check_parts(dup).empty());
                }
            }
        // rotated residues (frame_shift = B): every frame still partitioned
        for (int n : {2, 3, 8}) {
            std::vector<Part> ps;
            for (int q = 0; q < n; q++) ps.push_back(part(W, 1080, 16, q, n, 8, 1, 0, 8));
            CHECK(rtc::check_parts(ps).empty());
        }
        std::vector<Part> ps = {part(W, H, 3, 0, 2, 8), part(W, H, 2, 1, 2, 8)};
        CHECK(rtc::check_parts(ps) == "frame counts differ");
        ps = {part(W, H, 3, 0, 2, 8, 1), part(W, H, 3, 1, 2, 8, 3)};
        CHECK(rtc::check_parts(ps) == "outputs differ (bgra vs rgb)");
        ps = {part(W, H, 3, 0, 2, 8, 1), Part{}};
        CHECK(rtc::check_parts(ps) == "a rank has not rendered");
    }
    if (failures) {
        std::fprintf(stderr, "%d check(s) failed\n", failures);
        return 1;
    }
    std::printf("comm logic: all checks passed\n");
    return 0;
}
