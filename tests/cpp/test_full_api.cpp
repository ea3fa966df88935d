// test_full_api.cpp — the reference's own tests, ported onto the C++ mirror (include/rlnc/full.hpp) of
// rlnc::full over librlnc_hip: error tables of encoder.rs:277-544 / decoder.rs:186-350 / recoder.rs:180-331 and
// the round-trip property tests of src/full/tests.rs:7-203 (sizes reduced).  Exit code 0 = all passed.
// Built and run by tests/test_gpu_cpp.py on the GPU box.
#include <cstdio>
#include <cstdlib>
#include <thread>
#include <vector>

#include "rlnc/full.hpp"

using rlnc::RLNCError;
using rlnc::full::Decoder;
using rlnc::full::Encoder;
using rlnc::full::Recoder;

namespace {

int g_fail = 0;
#define CHECK(c)                                                            \
    do {                                                                    \
        if (!(c)) {                                                         \
            std::fprintf(stderr, "FAIL %s:%d: %s\n", __FILE__, __LINE__, #c); \
            ++g_fail;                                                       \
        }                                                                   \
    } while (0)

struct SplitMix {  // the caller-owned RNG (rand::Rng stand-in)
    uint64_t s;
    explicit SplitMix(uint64_t seed) : s(seed) {}
    uint64_t next() {
        uint64_t z = (s += 0x9E3779B97F4A7C15ull);
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        return z ^ (z >> 31);
    }
    void fill_bytes(uint8_t *p, size_t n) {
        for (size_t i = 0; i < n; ++i) p[i] = uint8_t(next());
    }
    size_t range(size_t lo, size_t hi) { return lo + next() % (hi - lo + 1); }
    std::vector<uint8_t> bytes(size_t n) {
        std::vector<uint8_t> v(n);
        fill_bytes(v.data(), n);
        return v;
    }
};

void test_encoder_errors() {  // encoder.rs:277-358, 450-494
    SplitMix rng(1);
    CHECK(Encoder::create({}, 5).error() == RLNCError::DataLengthZero);
    CHECK(Encoder::create(rng.bytes(100), 0).error() == RLNCError::PieceCountZero);
    CHECK(Encoder::create({}, 0).error() == RLNCError::DataLengthZero);
    auto e = Encoder::create(rng.bytes(1024), 32).unwrap();
    std::vector<uint8_t> shortb(e.get_full_coded_piece_byte_len() - 1), longb(e.get_full_coded_piece_byte_len() + 1),
        empty, ok(e.get_full_coded_piece_byte_len());
    CHECK(e.code_with_buf(rng, shortb).error() == RLNCError::InvalidOutputBuffer);
    CHECK(e.code_with_buf(rng, longb).error() == RLNCError::InvalidOutputBuffer);
    CHECK(e.code_with_buf(rng, empty).error() == RLNCError::InvalidOutputBuffer);
    CHECK(e.code_with_buf(rng, ok).is_ok());
}

void test_encoder_getters() {  // encoder.rs:496-544
    SplitMix rng(2);
    auto a = Encoder::create(rng.bytes(100), 1).unwrap();
    CHECK(a.get_piece_count() == 1 && a.get_piece_byte_len() == 101 && a.get_full_coded_piece_byte_len() == 102);
    auto b = Encoder::create({42}, 1).unwrap();
    CHECK(b.get_piece_byte_len() == 2 && b.get_full_coded_piece_byte_len() == 3);
    auto c = Encoder::create(rng.bytes(10), 10).unwrap();
    CHECK(c.get_piece_byte_len() == 2 && c.get_full_coded_piece_byte_len() == 12);
    auto d = Encoder::create(rng.bytes(100), 50).unwrap();
    CHECK(d.get_piece_byte_len() == 3);
}

void test_decoder() {  // decoder.rs:186-350
    SplitMix rng(3);
    CHECK(Decoder::create(0, 10).error() == RLNCError::PieceLengthZero);
    CHECK(Decoder::create(10, 0).error() == RLNCError::PieceCountZero);
    CHECK(Decoder::create(0, 0).error() == RLNCError::PieceLengthZero);
    auto e = Encoder::create(rng.bytes(1024), 32).unwrap();
    auto d = Decoder::create(e.get_piece_byte_len(), e.get_piece_count()).unwrap();
    CHECK(d.decode(rng.bytes(e.get_full_coded_piece_byte_len() - 1)).error() == RLNCError::InvalidPieceLength);
    CHECK(d.decode(rng.bytes(e.get_full_coded_piece_byte_len() + 1)).error() == RLNCError::InvalidPieceLength);
    CHECK(d.decode({}).error() == RLNCError::InvalidPieceLength);
    CHECK(d.get_received_piece_count() == 0 && d.get_useful_piece_count() == 0 && !d.is_already_decoded());
    CHECK(d.get_decoded_data().error() == RLNCError::NotAllPiecesReceivedYet);
    size_t total = 0;
    while (!d.is_already_decoded()) {
        auto r = d.decode(e.code(rng));
        CHECK(r.is_ok() || r.error() == RLNCError::PieceNotUseful);
        ++total;
    }
    CHECK(d.get_received_piece_count() == total && d.get_remaining_piece_count() == 0);
    CHECK(d.decode(e.code(rng)).error() == RLNCError::ReceivedAllPieces);
}

void test_recoder() {  // recoder.rs:180-331
    SplitMix rng(4);
    auto e = Encoder::create(rng.bytes(1024), 32).unwrap();
    const size_t full = e.get_full_coded_piece_byte_len(), k = e.get_piece_count();
    CHECK(Recoder::create({}, full, k).error() == RLNCError::NotEnoughPiecesToRecode);
    CHECK(Recoder::create({1, 2, 3}, 0, k).error() == RLNCError::PieceLengthZero);
    CHECK(Recoder::create({1, 2, 3}, full, 0).error() == RLNCError::PieceCountZero);
    CHECK(Recoder::create({1, 2, 3}, k, k).error() == RLNCError::PieceLengthTooShort);
    CHECK(Recoder::create({1, 2, 3}, k - 1, k).error() == RLNCError::PieceLengthTooShort);
    std::vector<uint8_t> coded;
    for (int i = 0; i < 10; ++i) {
        auto p = e.code(rng);
        coded.insert(coded.end(), p.begin(), p.end());
    }
    auto r = Recoder::create(coded, full, k).unwrap();
    CHECK(r.get_num_pieces_recoded_together() == 10 && r.get_original_num_pieces_coded_together() == k);
    CHECK(r.get_piece_byte_len() == e.get_piece_byte_len() && r.get_full_coded_piece_byte_len() == full);
    std::vector<uint8_t> bad(full - 1), good(full);
    CHECK(r.recode_with_buf(rng, bad).error() == RLNCError::InvalidOutputBuffer);
    CHECK(r.recode_with_buf(rng, good).is_ok());
}

void prop_encoder_recoder_decoder(uint64_t seed) {  // full/tests.rs:49-119 and :121-203
    SplitMix rng(seed);
    const auto data = rng.bytes(rng.range(1 << 10, 1 << 15));
    const size_t k = rng.range(1 << 5, 1 << 7);
    auto e = Encoder::create(data, k).unwrap();
    auto d = Decoder::create(e.get_piece_byte_len(), e.get_piece_count()).unwrap();
    std::vector<uint8_t> seen;
    size_t nseen = 0;
    for (size_t i = 0; i < k / 2; ++i) {
        auto p = e.code(rng);
        auto s = d.decode(p);
        if (s.is_ok()) {
            seen.insert(seen.end(), p.begin(), p.end());
            ++nseen;
        } else {
            CHECK(s.error() == RLNCError::PieceNotUseful);
        }
    }
    auto r = Recoder::create(seen, e.get_full_coded_piece_byte_len(), k).unwrap();
    for (size_t i = 0; i < 2 * nseen; ++i) CHECK(d.decode(r.recode(rng)).error() == RLNCError::PieceNotUseful);
    while (d.get_remaining_piece_count() > 0) {
        auto s = d.decode(e.code(rng));
        CHECK(s.is_ok() || s.error() == RLNCError::PieceNotUseful);
    }
    auto out = d.get_decoded_data();
    CHECK(out.is_ok() && out.value() == data);
}

void test_threads_and_clone() {
    // An encoder built on a worker thread is used after that thread (and its thread-local context) has ended.
    SplitMix rng(77);
    const auto data = rng.bytes(40000);
    Encoder e;
    std::thread([&] { e = Encoder::create(data, 24).unwrap(); }).join();
    auto d = Decoder::create(e.get_piece_byte_len(), e.get_piece_count()).unwrap();
    while (!d.is_already_decoded()) {
        auto r = d.decode(e.code(rng));
        CHECK(r.is_ok() || r.error() == RLNCError::PieceNotUseful);
    }
    CHECK(d.get_decoded_data().value() == data);

    // code(&self) from 8 threads at once on ONE encoder (the reference Encoder is Send + Sync): every piece equals
    // the one a single thread computes afterwards from the same coefficient bytes.
    const int nth = 8, per = 24;
    std::vector<std::vector<std::vector<uint8_t>>> got(nth);
    std::vector<std::thread> th;
    for (int t = 0; t < nth; ++t)
        th.emplace_back([&, t] {
            SplitMix r(1000 + t);
            for (int i = 0; i < per; ++i) got[t].push_back(e.code(r));
        });
    for (auto &t : th) t.join();
    for (int t = 0; t < nth; ++t) {
        SplitMix r(1000 + t);
        for (int i = 0; i < per; ++i) CHECK(e.code(r) == got[t][i]);
    }

    // Clone: an encoder clone codes identically; a decoder cloned half-way finishes independently; a recoder
    // clone recodes identically.
    Encoder e2 = e.clone();
    SplitMix ra(5), rb(5);
    CHECK(e.code(ra) == e2.code(rb));
    auto d1 = Decoder::create(e.get_piece_byte_len(), e.get_piece_count()).unwrap();
    SplitMix rc(6);
    std::vector<uint8_t> coded;
    for (size_t i = 0; i < e.get_piece_count() / 2; ++i) {
        auto p = e.code(rc);
        CHECK(d1.decode(p).is_ok());
        coded.insert(coded.end(), p.begin(), p.end());
    }
    Decoder d2 = d1;  // Clone
    CHECK(d2.get_received_piece_count() == d1.get_received_piece_count() &&
          d2.get_useful_piece_count() == d1.get_useful_piece_count());
    SplitMix r1(8), r2(9);
    while (!d1.is_already_decoded()) (void)d1.decode(e.code(r1));
    while (!d2.is_already_decoded()) (void)d2.decode(e2.code(r2));
    CHECK(d1.get_decoded_data().value() == data && d2.get_decoded_data().value() == data);
    auto rec = Recoder::create(coded, e.get_full_coded_piece_byte_len(), e.get_piece_count()).unwrap();
    Recoder rec2 = rec.clone();
    SplitMix s1(11), s2(11);
    CHECK(rec.recode(s1) == rec2.recode(s2));
}

}  // namespace

int main() {
    test_encoder_errors();
    test_encoder_getters();
    test_decoder();
    test_recoder();
    for (uint64_t s = 10; s < 14; ++s) prop_encoder_recoder_decoder(s);
    test_threads_and_clone();
    std::printf("%s (%d failures)\n", g_fail ? "FAILED" : "all passed", g_fail);
    return g_fail ? 1 : 0;
}
