// object_api_bench.cpp — the reference's own bench grid (benches/full_rlnc_{encoder,recoder,decoder}.rs: 1 / 16 / 32 MB
// × k = 16..256, recoders over k / 2 received pieces) on the drop-in object API (include/rlnc/full.hpp over
// librlnc_hip), timed per call the way divan times it: one call per sample, inputs built outside the timed region,
// the median over the samples.  A C++ caller, as a Rust caller of the crate would be: no interpreter between the
// timer and the C ABI.  Beside each row: the reference's published EPYC 9R14 single-thread median (README.md:2738-2850
// encode, :2859-2888 encode_zero_alloc, :3237-3349 recode, :3358-3387 recode_zero_alloc, :3736-3765 decode) and
// our/their ratio: the reference's five benches x its 15 shapes.
//
// decode: the reference's region is the loop of Decoder::decode calls until ReceivedAllPieces (full_rlnc_decoder.rs:
// 113-138: it never calls get_decoded_data).  Our decode() defers the data product to get_decoded_data, so each row
// reports the decode calls alone, get_decoded_data alone, and their sum -- the sum is the like-for-like figure.
//
//   g++ -std=c++17 -O2 -Iinclude scripts/object_api_bench.cpp -Lrlnc_amd -lrlnc_hip -Wl,-rpath,$PWD/rlnc_amd
//       -o build/object_api_bench; build/object_api_bench [--quick]
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "rlnc/full.hpp"

using rlnc::RLNCError;
using rlnc::full::Decoder;
using rlnc::full::Encoder;
using rlnc::full::Recoder;

namespace {

struct Rng {  // splitmix64; the coefficient bytes come from the caller's RNG as in the reference (encoder.rs:248)
    uint64_t s;
    explicit Rng(uint64_t seed) : s(seed) {}
    uint64_t next() {
        uint64_t z = (s += 0x9E3779B97F4A7C15ull);
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        return z ^ (z >> 31);
    }
    void fill_bytes(uint8_t *p, size_t n) {
        for (size_t i = 0; i < n; i += 8) {
            const uint64_t v = next();
            std::memcpy(p + i, &v, std::min<size_t>(8, n - i));
        }
    }
};

double now_us() {
    return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
double median(std::vector<double> v) {
    std::sort(v.begin(), v.end());
    return v[v.size() / 2];
}

struct Cfg {
    size_t bytes, k;
};
const Cfg kArgs[15] = {{1u << 20, 16}, {1u << 20, 32}, {1u << 20, 64}, {1u << 20, 128}, {1u << 20, 256},
                       {1u << 24, 16}, {1u << 24, 32}, {1u << 24, 64}, {1u << 24, 128}, {1u << 24, 256},
                       {1u << 25, 16}, {1u << 25, 32}, {1u << 25, 64}, {1u << 25, 128}, {1u << 25, 256}};
// EPYC 9R14 medians, microseconds (README.md rows in kArgs order)
const double kEncUs[15] = {22.3, 22.38, 19.58, 17.43, 17.47, 456, 414.4, 408.1, 405.3, 403.7,
                           1268, 1192, 1431, 1456, 1507};
// the allocating forms, encode (full_rlnc_encoder.rs:103-117: Encoder::code returns a fresh Vec) and recode
// (full_rlnc_recoder.rs:120-144: Recoder::recode), README.md:2738-2850 and :3237-3349
const double kEncAllocUs[15] = {23.1, 25.13, 18.91, 20.15, 20.09, 464.6, 411.7, 434.2, 440.1, 436,
                                1337, 1253, 1541, 1513, 1582};
const double kRecAllocUs[15] = {13.95, 11.49, 11.24, 18.42, 48.8, 288.5, 273.9, 277.7, 274.1, 308.7,
                                692.4, 636.3, 723.1, 821.8, 858.9};
const double kRecUs[15] = {11.86, 12.33, 11.1, 18.15, 50.01, 218.5, 218.4, 211.2, 213.6, 234.2,
                           655.9, 641.9, 720.4, 811.5, 805.6};
const double kDecUs[15] = {446, 834.3, 1681, 3850, 12700, 8655, 15410, 28740, 57290, 119300,
                           34520, 50680, 84020, 157300, 307000};
constexpr double kGiB = double(1u << 30);

int samples_for(double est_us, bool quick) {
    const double budget = quick ? 0.3e6 : 2e6;  // us of timed calls per row
    return int(std::max(5.0, std::min(100.0, budget / std::max(est_us, 1.0))));
}

}  // namespace

int main(int argc, char **argv) {
    const bool quick = argc > 1 && std::strcmp(argv[1], "--quick") == 0;
    const char *only = std::getenv("OBJ_BENCH_ONLY");  // "encode" / "recode" / "decode"
    Rng rng(0x524C4E43);
    for (int a = 0; a < 15; ++a) {
        const Cfg c = kArgs[a];
        if (quick && c.bytes > (1u << 24)) continue;
        if (std::getenv("OBJ_BENCH_SMALL") && c.bytes > (1u << 20)) continue;  // the 1 MB rows only
        if (const char *kk = std::getenv("OBJ_BENCH_K"))  // one k only (e.g. with RLNC_PIECE_TRACE=1)
            if (size_t(std::atoi(kk)) != c.k) continue;
        std::vector<uint8_t> data(c.bytes);
        rng.fill_bytes(data.data(), data.size());
        Encoder enc = Encoder::create(data, c.k).unwrap();
        const size_t L = enc.get_piece_byte_len(), full = enc.get_full_coded_piece_byte_len();
        // ---- encode_zero_alloc (full_rlnc_encoder.rs:124-138)
        if (!only || std::strcmp(only, "encode") == 0) {
            std::vector<uint8_t> buf(full);
            for (int i = 0; i < 5; ++i) enc.code_with_buf(rng, buf).unwrap();
            const int n = samples_for(kEncUs[a], quick);
            std::vector<double> t;
            for (int i = 0; i < n; ++i) {
                const double t0 = now_us();
                enc.code_with_buf(rng, buf).unwrap();
                t.push_back(now_us() - t0);
            }
            const double m = median(t), counter = double(c.k * L + full);  // :111-113
            std::printf("{\"bench\": \"encode_zero_alloc\", \"data_bytes\": %zu, \"k\": %zu, \"L\": %zu, \"samples\": %d, "
                        "\"median_us\": %.2f, \"GiBps\": %.2f, \"epyc_median_us\": %.2f, \"epyc_GiBps\": %.2f, "
                        "\"time_vs_epyc\": %.3f}\n",
                        c.bytes, c.k, L, n, m, counter / m * 1e6 / kGiB, kEncUs[a], counter / kEncUs[a] * 1e6 / kGiB,
                        m / kEncUs[a]);
            std::fflush(stdout);
        }
        // ---- encode (full_rlnc_encoder.rs:103-117): Encoder::code allocates the coded piece it returns; the returned
        // pieces are dropped outside the timed region (divan drops bench outputs after timing)
        if (!only || std::strcmp(only, "encode") == 0) {
            for (int i = 0; i < 5; ++i) (void)enc.code(rng);
            const int n = samples_for(kEncAllocUs[a], quick);
            std::vector<double> t;
            for (int i = 0; i < n; ++i) {
                double t1;
                {
                    const double t0 = now_us();
                    const std::vector<uint8_t> piece = enc.code(rng);
                    t1 = now_us();
                    t.push_back(t1 - t0);
                }  // dropped after the timer, as divan drops a sample's output
            }
            const double m = median(t), counter = double(c.k * L + full);
            std::printf("{\"bench\": \"encode\", \"data_bytes\": %zu, \"k\": %zu, \"L\": %zu, \"samples\": %d, "
                        "\"median_us\": %.2f, \"GiBps\": %.2f, \"epyc_median_us\": %.2f, \"epyc_GiBps\": %.2f, "
                        "\"time_vs_epyc\": %.3f}\n",
                        c.bytes, c.k, L, n, m, counter / m * 1e6 / kGiB, kEncAllocUs[a],
                        counter / kEncAllocUs[a] * 1e6 / kGiB, m / kEncAllocUs[a]);
            std::fflush(stdout);
        }
        // ---- recode_zero_alloc (full_rlnc_recoder.rs:148-173): a fresh Recoder over k/2 coded pieces per sample
        if (!only || std::strcmp(only, "recode") == 0) {
            const size_t nrec = c.k / 2;
            std::vector<uint8_t> coded;
            coded.reserve(nrec * full);
            for (size_t i = 0; i < nrec; ++i) {
                auto p = enc.code(rng);
                coded.insert(coded.end(), p.begin(), p.end());
            }
            std::vector<uint8_t> buf(full);
            {
                Recoder r = Recoder::create(coded, full, c.k).unwrap();
                for (int i = 0; i < 5; ++i) r.recode_with_buf(rng, buf).unwrap();
            }
            const int n = samples_for(kRecUs[a], quick);
            std::vector<double> t, tc;  // tc: Recoder::new itself (outside the bench's timed region, as in divan)
            for (int i = 0; i < n; ++i) {
                const double tc0 = now_us();
                Recoder r = Recoder::create(coded, full, c.k).unwrap();
                const double t0 = now_us();
                tc.push_back(t0 - tc0);
                r.recode_with_buf(rng, buf).unwrap();
                t.push_back(now_us() - t0);
            }
            const double m = median(t), counter = double(full * nrec + full);  // :137-142
            std::printf("{\"bench\": \"recode_zero_alloc\", \"data_bytes\": %zu, \"k\": %zu, \"received\": %zu, "
                        "\"samples\": %d, \"median_us\": %.2f, \"GiBps\": %.2f, \"epyc_median_us\": %.2f, "
                        "\"epyc_GiBps\": %.2f, \"time_vs_epyc\": %.3f, \"new_median_us\": %.2f}\n",
                        c.bytes, c.k, nrec, n, m, counter / m * 1e6 / kGiB, kRecUs[a], counter / kRecUs[a] * 1e6 / kGiB,
                        m / kRecUs[a], median(tc));
            std::fflush(stdout);
            // ---- recode (full_rlnc_recoder.rs:120-144): Recoder::recode allocates the recoded piece it returns
            std::vector<double> ta;
            for (int i = 0; i < n; ++i) {
                Recoder r = Recoder::create(coded, full, c.k).unwrap();
                const double t0 = now_us();
                const std::vector<uint8_t> piece = r.recode(rng);
                ta.push_back(now_us() - t0);
            }
            const double ma = median(ta);
            std::printf("{\"bench\": \"recode\", \"data_bytes\": %zu, \"k\": %zu, \"received\": %zu, "
                        "\"samples\": %d, \"median_us\": %.2f, \"GiBps\": %.2f, \"epyc_median_us\": %.2f, "
                        "\"epyc_GiBps\": %.2f, \"time_vs_epyc\": %.3f}\n",
                        c.bytes, c.k, nrec, n, ma, counter / ma * 1e6 / kGiB, kRecAllocUs[a],
                        counter / kRecAllocUs[a] * 1e6 / kGiB, ma / kRecAllocUs[a]);
            std::fflush(stdout);
        }
        // ---- decode (full_rlnc_decoder.rs:106-139): 2k coded pieces, a fresh Decoder per sample
        if (!only || std::strcmp(only, "decode") == 0) {
            const size_t np = 2 * c.k;
            std::vector<std::vector<uint8_t>> pieces(np);
            for (auto &p : pieces) p = enc.code(rng);
            const int n = samples_for(kDecUs[a] * 0.5, quick);
            std::vector<double> td, tg, ts;
            for (int i = 0; i < n + 1; ++i) {
                Decoder d = Decoder::create(L, c.k).unwrap();
                const double t0 = now_us();
                for (size_t p = 0; p < np; ++p) {
                    auto r = d.decode(pieces[p]);
                    if (r.is_err() && r.error() == RLNCError::ReceivedAllPieces) break;
                }
                const double t1 = now_us();
                auto got = d.get_decoded_data();
                const double t2 = now_us();
                if (got.is_err() || got.value() != data) {
                    std::fprintf(stderr, "decode mismatch at %zu B / k = %zu\n", c.bytes, c.k);
                    return 1;
                }
                if (i == 0) continue;  // warm-up sample
                td.push_back(t1 - t0);
                tg.push_back(t2 - t1);
                ts.push_back(t2 - t0);
            }
            const double counter = double(full * c.k);  // :118
            const double m = median(ts);
            std::printf("{\"bench\": \"decode\", \"data_bytes\": %zu, \"k\": %zu, \"samples\": %d, "
                        "\"decode_calls_median_us\": %.1f, \"get_decoded_data_median_us\": %.1f, "
                        "\"decode_total_median_us\": %.1f, \"GiBps_total\": %.3f, \"epyc_median_us\": %.1f, "
                        "\"epyc_GiBps\": %.3f, \"total_vs_epyc\": %.3f, \"calls_vs_epyc\": %.3f}\n",
                        c.bytes, c.k, n, median(td), median(tg), m, counter / m * 1e6 / kGiB, kDecUs[a],
                        counter / kDecUs[a] * 1e6 / kGiB, m / kDecUs[a], median(td) / kDecUs[a]);
            std::fflush(stdout);
        }
    }
    return 0;
}
