// rlnc/full.hpp — C++ mirror of rlnc::full::{Encoder, Decoder, Recoder} and rlnc::RLNCError
// (itzmeanjan/rlnc 0.8.5, src/full/*.rs, src/common/errors.rs) over the C ABI of librlnc_hip
// (include/rlnc_hip.h).  Header-only; link with -lrlnc_hip.
//
// Names follow the reference; `Encoder::create` stands for `Encoder::new` (a C++ keyword).  Result<T> carries
// RLNCError like Rust's Result.  Randomness stays with the caller exactly as in the reference: code()/recode()
// take any Rng with `void fill_bytes(uint8_t *, size_t)` and draw the coefficient bytes on the host
// (encoder.rs:248, recoder.rs:131).
#pragma once

#include <algorithm>
#include <cstddef>
#include <cstdint>
#include <cstdlib>
#include <new>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

#include <sys/mman.h>

#include "../rlnc_hip.h"

namespace rlnc {

// errors.rs:3-32, same order (C status = discriminant + 1)
enum class RLNCError : int {
    CodingVectorLengthMismatch = 0,
    DataLengthMismatch,
    PieceCountZero,
    DataLengthZero,
    PieceLengthZero,
    NotEnoughPiecesToRecode,
    PieceLengthTooShort,
    PieceNotUseful,
    ReceivedAllPieces,
    NotAllPiecesReceivedYet,
    InvalidDecodedDataFormat,
    InvalidPieceLength,
    InvalidOutputBuffer,
};

inline const char *to_string(RLNCError e) { return rlnc_status_message(int(e) + 1); }  // errors.rs:34-58

struct DeviceError : std::runtime_error {
    using std::runtime_error::runtime_error;
};

template <class T>
class Result {
   public:
    Result(T v) : ok_(true), v_(std::move(v)) {}
    Result(RLNCError e) : ok_(false), e_(e) {}
    bool is_ok() const { return ok_; }
    bool is_err() const { return !ok_; }
    RLNCError error() const { return e_; }
    T &value() {
        if (!ok_) throw std::logic_error(std::string("unwrap on Err: ") + to_string(e_));
        return v_;
    }
    T unwrap() { return std::move(value()); }

   private:
    bool ok_;
    T v_{};
    RLNCError e_{};
};

template <>
class Result<void> {
   public:
    Result() : ok_(true) {}
    Result(RLNCError e) : ok_(false), e_(e) {}
    bool is_ok() const { return ok_; }
    bool is_err() const { return !ok_; }
    RLNCError error() const { return e_; }
    void unwrap() const {
        if (!ok_) throw std::logic_error(std::string("unwrap on Err: ") + to_string(e_));
    }

   private:
    bool ok_;
    RLNCError e_{};
};

namespace detail {
inline Result<void> status(int s) {
    if (s == RLNC_OK) return {};
    if (s >= 1 && s <= 13) return RLNCError(s - 1);
    throw DeviceError(std::string(rlnc_status_name(s)) + ": " + rlnc_last_error());
}

// The default context of the calling thread.  Objects take their own reference on it (rlnc_hip.h, Lifetime), so
// an Encoder built on a worker thread stays valid after that thread -- and this thread_local -- is gone.
inline rlnc_context *context() {
    thread_local struct Holder {
        rlnc_context *c = nullptr;
        Holder() {
            const int s = rlnc_context_create(0, &c);
            if (s != RLNC_OK) throw DeviceError(std::string("rlnc_context_create: ") + rlnc_last_error());
        }
        ~Holder() { rlnc_context_destroy(c); }
    } h;
    return h.c;
}

// The allocator of Bytes: calloc'd storage, and value-initialisation of its bytes is a no-op -- they are zero
// already.  That is what the reference's `vec![0u8; n]` is (alloc_zeroed = calloc: a large buffer is a fresh mapping
// whose pages are zeroed lazily, on first write), where a std::vector<uint8_t>(n) would memset every byte on the
// calling thread first (32 MiB: most of a large decode's get_decoded_data).  Caveat: growing a Bytes
// that was shrunk does not re-zero the bytes it had before.
template <class T>
struct ZeroedAlloc {
    using value_type = T;
    ZeroedAlloc() = default;
    template <class U>
    ZeroedAlloc(const ZeroedAlloc<U> &) noexcept {}
    T *allocate(size_t n) {
        if (void *p = std::calloc(n ? n : 1, sizeof(T))) return static_cast<T *>(p);
        throw std::bad_alloc();
    }
    void deallocate(T *p, size_t) noexcept { std::free(p); }
    template <class U>
    void construct(U *) noexcept {}  // value-initialised = the calloc'd zero
    template <class U, class... A>
    void construct(U *p, A &&...a) {
        ::new (static_cast<void *>(p)) U(std::forward<A>(a)...);
    }
    template <class U>
    bool operator==(const ZeroedAlloc<U> &) const noexcept {
        return true;
    }
    template <class U>
    bool operator!=(const ZeroedAlloc<U> &) const noexcept {
        return false;
    }
};

using ZBytes = std::vector<uint8_t, ZeroedAlloc<uint8_t>>;

// A fresh result buffer this mirror allocated (get_decoded_data's Bytes) of >= 8 MiB: its whole 2 MiB-aligned pages
// may be backed by transparent huge pages (MADV_HUGEPAGE, a hint where the host's THP mode is "madvise"), so the
// library's parallel copy-out faults it in 2 MiB at a time (32 MiB rows 2.4-3.8 -> 1.7-2.3 ms).  The
// library itself does not advise memory it does not own (unless RLNC_COPY_HUGEPAGE=1).
inline void advise_huge_pages(void *p, size_t n) {
    if (n < (size_t(8) << 20)) return;
    constexpr uintptr_t kHuge = uintptr_t(2) << 20;
    const uintptr_t a = (reinterpret_cast<uintptr_t>(p) + kHuge - 1) & ~(kHuge - 1);
    const uintptr_t b = (reinterpret_cast<uintptr_t>(p) + n) & ~(kHuge - 1);
    if (b > a) (void)madvise(reinterpret_cast<void *>(a), b - a, MADV_HUGEPAGE);
}
inline bool operator==(const ZBytes &a, const std::vector<uint8_t> &b) {
    return a.size() == b.size() && std::equal(a.begin(), a.end(), b.begin());
}
inline bool operator==(const std::vector<uint8_t> &a, const ZBytes &b) { return b == a; }
inline bool operator!=(const ZBytes &a, const std::vector<uint8_t> &b) { return !(a == b); }
inline bool operator!=(const std::vector<uint8_t> &a, const ZBytes &b) { return !(b == a); }

template <class H, void (*Free)(H *)>
struct Handle {
    H *h = nullptr;
    Handle() = default;
    explicit Handle(H *p) : h(p) {}
    Handle(Handle &&o) noexcept : h(o.h) { o.h = nullptr; }
    Handle &operator=(Handle &&o) noexcept {
        std::swap(h, o.h);
        return *this;
    }
    Handle(const Handle &) = delete;
    ~Handle() {
        if (h) Free(h);
    }
};

// #[derive(Clone)] of the reference types: an independent librlnc_hip object
template <class H>
H *clone_handle(int (*fn)(const H *, H **), const H *h) {
    if (!h) return nullptr;
    H *c = nullptr;
    const int s = fn(h, &c);
    if (s != RLNC_OK) throw DeviceError(std::string("clone: ") + rlnc_last_error());
    return c;
}
}  // namespace detail

namespace full {

// Decoder::get_decoded_data's result: a byte vector allocated zeroed like the reference's vec![0u8; n]
using Bytes = detail::ZBytes;

// encoder.rs:19-270
class Encoder {
   public:
    Encoder() = default;
    Encoder(const Encoder &o) : h_(detail::clone_handle(rlnc_encoder_clone, o.h_.h)) {}  // Clone
    Encoder &operator=(const Encoder &o) {
        Encoder t(o);
        std::swap(h_.h, t.h_.h);
        return *this;
    }
    Encoder(Encoder &&) noexcept = default;
    Encoder &operator=(Encoder &&) noexcept = default;
    Encoder clone() const { return Encoder(*this); }
    static Result<Encoder> create(const std::vector<uint8_t> &data, size_t piece_count) {  // Encoder::new :85
        rlnc_encoder *h = nullptr;
        auto r = detail::status(rlnc_encoder_new(detail::context(), data.data(), data.size(), piece_count, &h));
        if (r.is_err()) return r.error();
        return Encoder(h);
    }
    size_t get_piece_count() const { return rlnc_encoder_get_piece_count(h_.h); }
    size_t get_piece_byte_len() const { return rlnc_encoder_get_piece_byte_len(h_.h); }
    size_t get_full_coded_piece_byte_len() const { return rlnc_encoder_get_full_coded_piece_byte_len(h_.h); }
    template <class Rng>
    Result<void> code_with_buf(Rng &rng, std::vector<uint8_t> &full) const {  // encoder.rs:241-250
        if (full.size() != get_full_coded_piece_byte_len()) return RLNCError::InvalidOutputBuffer;
        rng.fill_bytes(full.data(), get_piece_count());
        return detail::status(
            rlnc_encoder_code_with_buf(h_.h, full.data(), get_piece_count(), full.data(), full.size()));
    }
    template <class Rng>
    std::vector<uint8_t> code(Rng &rng) const {  // encoder.rs:264-269
        std::vector<uint8_t> v(get_full_coded_piece_byte_len());
        code_with_buf(rng, v).unwrap();
        return v;
    }

   private:
    explicit Encoder(rlnc_encoder *h) : h_(h) {}
    detail::Handle<rlnc_encoder, rlnc_encoder_free> h_;
};

// decoder.rs:9-178
class Decoder {
   public:
    Decoder() = default;
    Decoder(const Decoder &o) : h_(detail::clone_handle(rlnc_decoder_clone, o.h_.h)) {}  // Clone
    Decoder &operator=(const Decoder &o) {
        Decoder t(o);
        std::swap(h_.h, t.h_.h);
        return *this;
    }
    Decoder(Decoder &&) noexcept = default;
    Decoder &operator=(Decoder &&) noexcept = default;
    Decoder clone() const { return Decoder(*this); }
    static Result<Decoder> create(size_t piece_byte_len, size_t required_piece_count) {  // Decoder::new :65
        rlnc_decoder *h = nullptr;
        auto r = detail::status(rlnc_decoder_new(detail::context(), piece_byte_len, required_piece_count, &h));
        if (r.is_err()) return r.error();
        return Decoder(h);
    }
    Result<void> decode(const std::vector<uint8_t> &piece) {  // decoder.rs:96-118
        return detail::status(rlnc_decoder_decode(h_.h, piece.data(), piece.size()));
    }
    bool is_already_decoded() const { return rlnc_decoder_is_already_decoded(h_.h) != 0; }
    size_t get_num_pieces_coded_together() const { return rlnc_decoder_get_num_pieces_coded_together(h_.h); }
    size_t get_piece_byte_len() const { return rlnc_decoder_get_piece_byte_len(h_.h); }
    size_t get_full_coded_piece_byte_len() const { return rlnc_decoder_get_full_coded_piece_byte_len(h_.h); }
    size_t get_received_piece_count() const { return rlnc_decoder_get_received_piece_count(h_.h); }
    size_t get_useful_piece_count() const { return rlnc_decoder_get_useful_piece_count(h_.h); }
    size_t get_remaining_piece_count() const { return rlnc_decoder_get_remaining_piece_count(h_.h); }
    Result<Bytes> get_decoded_data() {  // decoder.rs:136-159
        Bytes out(get_num_pieces_coded_together() * get_piece_byte_len());
        detail::advise_huge_pages(out.data(), out.size());
        size_t n = 0;
        auto r = detail::status(rlnc_decoder_get_decoded_data(h_.h, out.data(), out.size(), &n));
        if (r.is_err()) return r.error();
        // out[n] holds the boundary marker and every byte after it is zero: clear the marker so that a later
        // resize(m > n) of the result regrows into zeros, as the crate's Vec does
        if (n < out.size()) out[n] = 0;
        out.resize(n);
        return out;
    }

   private:
    explicit Decoder(rlnc_decoder *h) : h_(h) {}
    detail::Handle<rlnc_decoder, rlnc_decoder_free> h_;
};

// recoder.rs:13-172
class Recoder {
   public:
    Recoder() = default;
    Recoder(const Recoder &o) : h_(detail::clone_handle(rlnc_recoder_clone, o.h_.h)) {}  // Clone
    Recoder &operator=(const Recoder &o) {
        Recoder t(o);
        std::swap(h_.h, t.h_.h);
        return *this;
    }
    Recoder(Recoder &&) noexcept = default;
    Recoder &operator=(Recoder &&) noexcept = default;
    Recoder clone() const { return Recoder(*this); }
    static Result<Recoder> create(const std::vector<uint8_t> &data, size_t full_coded_piece_byte_len,
                                  size_t num_pieces_coded_together) {  // Recoder::new :68
        rlnc_recoder *h = nullptr;
        auto r = detail::status(rlnc_recoder_new(detail::context(), data.data(), data.size(),
                                                 full_coded_piece_byte_len, num_pieces_coded_together, &h));
        if (r.is_err()) return r.error();
        return Recoder(h);
    }
    size_t get_original_num_pieces_coded_together() const {
        return rlnc_recoder_get_original_num_pieces_coded_together(h_.h);
    }
    size_t get_num_pieces_recoded_together() const { return rlnc_recoder_get_num_pieces_recoded_together(h_.h); }
    size_t get_piece_byte_len() const { return rlnc_recoder_get_piece_byte_len(h_.h); }
    size_t get_full_coded_piece_byte_len() const { return rlnc_recoder_get_full_coded_piece_byte_len(h_.h); }
    template <class Rng>
    Result<void> recode_with_buf(Rng &rng, std::vector<uint8_t> &full) {  // recoder.rs:122-153
        if (full.size() != get_full_coded_piece_byte_len()) return RLNCError::InvalidOutputBuffer;
        std::vector<uint8_t> r(get_num_pieces_recoded_together());
        rng.fill_bytes(r.data(), r.size());
        return detail::status(rlnc_recoder_recode_with_buf(h_.h, r.data(), r.size(), full.data(), full.size()));
    }
    template <class Rng>
    std::vector<uint8_t> recode(Rng &rng) {  // recoder.rs:166-171
        std::vector<uint8_t> v(get_full_coded_piece_byte_len());
        recode_with_buf(rng, v).unwrap();
        return v;
    }

   private:
    explicit Recoder(rlnc_recoder *h) : h_(h) {}
    detail::Handle<rlnc_recoder, rlnc_recoder_free> h_;
};

}  // namespace full
}  // namespace rlnc
