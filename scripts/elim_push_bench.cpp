// elim_push_bench.cpp — host cost of one Decoder::decode coefficient push (the exact replica of
// DecoderMatrix::rref on [coeffs | E], elimination.cpp), per k: best-of-N whole decodes / k.  No device needed.
//   g++ -std=c++17 -O2 -Iinclude scripts/elim_push_bench.cpp -Lrlnc_amd -lrlnc_hip -Wl,-rpath,$PWD/rlnc_amd
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <random>
#include <vector>

#include "rlnc_hip.h"

int main() {
    std::mt19937 g(1);
    for (size_t k : {16, 32, 64, 128, 256}) {
        std::vector<uint8_t> C((k + 8) * k);
        for (auto &b : C) b = uint8_t(g());
        double best = 1e30;
        for (int rep = 0; rep < 30; ++rep) {
            rlnc_elimination *e = nullptr;
            rlnc_elimination_new(k, 0, &e);
            const auto t0 = std::chrono::steady_clock::now();
            int32_t slot, keep;
            for (size_t i = 0; i < k + 8 && rlnc_elimination_rank(e) < k; ++i)
                rlnc_elimination_push(e, &C[i * k], &slot, &keep);
            best = std::min(best, std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count());
            rlnc_elimination_free(e);
        }
        std::printf("{\"k\": %zu, \"us_per_push\": %.2f}\n", k, best / double(k));
    }
    return 0;
}
