// Host planners under AddressSanitizer + UndefinedBehaviorSanitizer (SURVEY.md §5's
// sanitizer row). Built by tools/sanitize/run.sh with the library's own
// sources (host code sanitized, device code compiled as usual and never launched): drives
// every host-only entry that plans or checks a schedule over the sizes the CPU tests cover:
//   gaplac_plan_check          - the single-GPU schedule's launch footprints (every mode),
//                                which also builds / checks every tail task list
//                                (build_tail_tasks, sim_order_tail_tasks, check_tail_tasks,
//                                interleave_tail_tasks) on its first call;
//   gaplac_plan_check_schedule - the deferred-update accounting at every depth;
//   gaplac_dist_plan_check     - build_plan / check_plan of the distributed schedule;
//   gaplac_dist_plan           - the plan export;
//   gaplac_dist_plan_check_tail / gaplac_dist_plan_tail - the same with the tail gather.
// Exit 0 when every check passes and no sanitizer fired (halt_on_error=1).
#include <cstdio>
#include <vector>

#include "../../include/gaplac.h"

static int fails = 0;
#define EXPECT(cond, ...)                 \
    do {                                  \
        if (!(cond)) {                    \
            std::printf(__VA_ARGS__);     \
            std::printf("\n");            \
            ++fails;                      \
        }                                 \
    } while (0)

int main() {
    char msg[256];
    int64_t a = 0, b = 0;
    std::vector<int64_t> sizes;
    for (int64_t n = 1; n <= 300; ++n) sizes.push_back(n);
    for (int64_t n : {383, 384, 385, 511, 512, 513, 1000, 2047, 4095, 4096, 4097, 7000, 8192, 12000, 16384, 65536})
        sizes.push_back(n);
    long checks = 0;
    for (int spw : {1, 2, 4, 5, 8})
        for (int mode : {0, 1, 2})
            for (int64_t M : {1, 130, 1000, 6016, 6200}) {
                if (mode != 2 && M != 1) continue;
                for (int64_t N : sizes) {
                    if (mode == 1 && N > 16384) continue;
                    const int rc = gaplac_plan_check(N, mode, mode == 2 ? M : 0, spw, &a, &b, msg, sizeof msg);
                    EXPECT(rc == 0 && b == 0, "plan_check N=%lld mode=%d M=%lld spw=%d: rc %d violations %lld %s",
                           (long long)N, mode, (long long)M, spw, rc, (long long)b, msg);
                    ++checks;
                }
            }
    // negative control: a workspace one element short must be reported
    for (int64_t N : {1, 127, 255, 300, 4096}) {
        const int rc = gaplac_plan_check(N, 8, 0, 4, &a, &b, msg, sizeof msg);
        EXPECT(rc == 0 && b >= 1, "negative control N=%lld not reported", (long long)N);
    }
    for (int depth = 0; depth <= 8; ++depth) {
        if (depth == 1) continue;
        for (int ext : {0, 1})
            for (int64_t N : {1, 127, 1000, 4096, 10239, 10240, 12000, 16384, 20000, 33000, 40000, 50000, 65536})
                for (int sp : {0, 1, 2, 3}) {
                    const int spw[] = {4, 4, 2, 3}, pm[] = {40, 8, 24, 16};
                    const int rc = gaplac_plan_check_schedule(N, spw[sp], depth, ext, pm[sp], &a, msg, sizeof msg);
                    EXPECT(rc == 0 && a >= 1, "plan_check_schedule N=%lld spw=%d depth=%d ext=%d: %s", (long long)N,
                           spw[sp], depth, ext, msg);
                    ++checks;
                }
    }
    for (int depth : {1, 2, 3, 4, 5, 8})
        for (int spw : {1, 2, 4, 8})
            for (int pair_m : {0, 8, 40})
                for (int nt = 1; nt <= 600; ++nt) {
                    const int rc = gaplac_dist_plan_check(nt, spw, depth, pair_m, &a, msg, sizeof msg);
                    EXPECT(rc == 0, "dist_plan_check nt=%d spw=%d depth=%d pair_m=%d: %s", nt, spw, depth, pair_m, msg);
                    ++checks;
                    for (int tail : {1, 5, 48, 80, 128}) {
                        const int rt = gaplac_dist_plan_check_tail(nt, spw, depth, pair_m, tail, &a, msg, sizeof msg);
                        EXPECT(rt == 0, "dist_plan_check_tail nt=%d spw=%d depth=%d pair_m=%d tail=%d: %s", nt, spw,
                               depth, pair_m, tail, msg);
                        ++checks;
                        if (nt % 97 == 0) {
                            int64_t n = 0;
                            EXPECT(gaplac_dist_plan_tail(nt, spw, depth, pair_m, tail, nullptr, 0, &n) == 0 && n > 0,
                                   "dist_plan_tail size");
                            std::vector<int32_t> out((size_t)(5 * n));
                            EXPECT(gaplac_dist_plan_tail(nt, spw, depth, pair_m, tail, out.data(), 5 * n, &n) == 0,
                                   "dist_plan_tail export");
                        }
                    }
                    if (nt % 97 == 0) {  // the export, sized by a first call
                        int64_t n = 0;
                        EXPECT(gaplac_dist_plan(nt, spw, depth, pair_m, nullptr, 0, &n) == 0 && n > 0, "dist_plan size");
                        std::vector<int32_t> out((size_t)(5 * n));
                        EXPECT(gaplac_dist_plan(nt, spw, depth, pair_m, out.data(), 5 * n, &n) == 0, "dist_plan export");
                    }
                }
    std::printf("sanitized plan checks: %ld checks, %d failures\n", checks, fails);
    return fails ? 1 : 0;
}
