// ubench_fault.cpp — what filling a fresh 32 MiB caller buffer costs on this host (Decoder::get_decoded_data's
// copy-out): page faults on one thread vs several, with MADV_HUGEPAGE, with MADV_POPULATE_WRITE.
//   g++ -O2 -std=c++17 -pthread scripts/ubench_fault.cpp -o build/ubench_fault && build/ubench_fault
#include <sys/mman.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <string>
#include <thread>
#include <vector>

#ifndef MADV_POPULATE_WRITE
#define MADV_POPULATE_WRITE 23
#endif

static double now_us() {
    return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

static void par(int t, size_t n, uint8_t *p, const uint8_t *src, int mode) {
    std::vector<std::thread> th;
    const size_t per = ((n + t - 1) / t + 4095) & ~size_t(4095);
    for (int i = 0; i < t; ++i)
        th.emplace_back([=] {
            const size_t a = i * per, b = std::min(n, a + per);
            if (a >= b) return;
            if (mode == 1) madvise(p + a, b - a, MADV_POPULATE_WRITE);
            if (src) std::memcpy(p + a, src + a, b - a);
            else std::memset(p + a, 1, b - a);
        });
    for (auto &x : th) x.join();
}

int main() {
    for (const char *f : {"/sys/kernel/mm/transparent_hugepage/enabled", "/sys/kernel/mm/transparent_hugepage/defrag"}) {
        std::ifstream s(f);
        std::string l;
        std::getline(s, l);
        std::printf("{\"file\": \"%s\", \"value\": \"%s\"}\n", f, l.c_str());
    }
    const size_t n = (size_t(32) << 20) + 16;
    std::vector<uint8_t> src(n, 7);
    for (int threads : {1, 2, 4, 8, 16}) {
        for (int mode : {0, 1, 2}) {  // 0 plain first-touch, 1 MADV_POPULATE_WRITE per slice first, 2 MADV_HUGEPAGE
            double best = 1e18, sum = 0;
            const int reps = 7;
            for (int r = 0; r < reps; ++r) {
                uint8_t *p = static_cast<uint8_t *>(std::calloc(n, 1));
                const double t0 = now_us();
                if (mode == 2) {
                    const uintptr_t a = (reinterpret_cast<uintptr_t>(p) + 4095) & ~uintptr_t(4095);
                    madvise(reinterpret_cast<void *>(a), (reinterpret_cast<uintptr_t>(p) + n - a) & ~uintptr_t(4095), MADV_HUGEPAGE);
                }
                par(threads, n, p, src.data(), mode == 1 ? 1 : 0);
                const double dt = now_us() - t0;
                std::free(p);
                best = std::min(best, dt);
                sum += dt;
            }
            std::printf("{\"threads\": %d, \"mode\": \"%s\", \"best_us\": %.1f, \"mean_us\": %.1f}\n", threads,
                        mode == 0 ? "first-touch copy" : mode == 1 ? "populate_write + copy" : "hugepage + copy", best,
                        sum / reps);
            std::fflush(stdout);
        }
    }
    // warm: the same buffer again (no faults)
    uint8_t *p = static_cast<uint8_t *>(std::malloc(n));
    std::memset(p, 0, n);
    for (int threads : {1, 4, 8}) {
        double best = 1e18;
        for (int r = 0; r < 5; ++r) {
            const double t0 = now_us();
            par(threads, n, p, src.data(), 0);
            best = std::min(best, now_us() - t0);
        }
        std::printf("{\"threads\": %d, \"mode\": \"warm copy\", \"best_us\": %.1f}\n", threads, best);
    }
    std::free(p);
    return 0;
}
