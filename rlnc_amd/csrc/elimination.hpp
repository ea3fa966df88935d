// elimination.hpp — the decoder's coefficient-side engine (host, exact).
//
// Decoder::decode (src/full/decoder.rs:96-118) appends the full piece [coeffs | data] and re-runs the
// diagonal-pivot RREF of DecoderMatrix (src/full/decoder_matrix.rs:99-244) over k + L columns.  Every
// decision of that algorithm (pivot tests, row swaps, which rows to eliminate, zero-row removal) reads
// only coefficient columns < k, and every row operation touches all columns >= i, i.e. always the whole
// data part.  So running the SAME algorithm on [coeffs | E], where E tracks each row as a combination of
// the received pieces (E starts as the unit vector of the piece's slot), makes the same decisions and
// ends with data rows == E × received data.  The host therefore answers useful / not-useful at once on a
// k × (k + slots) matrix, and the device applies E to the data rows in one matmul (kernels.hpp) —
// byte-identical to the reference, including its rank over-count on structured coefficients
// (SURVEY.md §0.5), because the elimination is replicated verbatim, not replaced by a "correct" one.
#pragma once
#include <cstddef>
#include <cstdint>
#include <vector>

namespace rlnc {

class Elimination {
   public:
    // fixed_slots > 0: slot of the p-th pushed piece is p (E has fixed_slots columns, no reuse; batch
    // decode).  fixed_slots == 0: slots are recycled once a piece no longer contributes to any row.
    explicit Elimination(size_t k, size_t fixed_slots = 0);

    // Decoder::decode semantics on the coefficient vector (k bytes).  Returns 0 (useful),
    // RLNC_ERR_PIECE_NOT_USEFUL or RLNC_ERR_RECEIVED_ALL_PIECES (no state change).  *slot = E column
    // given to the piece, *keep = whether its data row is still referenced (must be stored).
    int push(const uint8_t *coeffs, int *slot, bool *keep);

    size_t k() const { return k_; }
    size_t rank() const { return rows_; }
    size_t slots() const { return cap_; }  // E columns (high-water mark)
    bool decoded() const { return rows_ == k_; }
    // T[r][s] = E[r][s] for r < rank, s < slots; T has leading dimension ld >= slots.
    void transform(uint8_t *T, size_t ld) const;
    // Full matrix row r (k coefficient bytes then slots() E bytes) — for tests.
    const uint8_t *row(size_t r) const { return &m_[r * stride()]; }

   private:
    size_t stride() const { return k_ + cap_; }
    void grow(size_t new_cap);
    void rref();
    void clean_forward();
    void clean_backward();
    void remove_zero_rows();
    void row_muladd(size_t dst, size_t src, size_t from, uint8_t q);

    size_t k_;
    size_t cap_ = 0;
    size_t rows_ = 0;
    size_t pushed_ = 0;
    bool fixed_;
    std::vector<uint8_t> m_;  // (k_ + 1) rows × stride()
    std::vector<uint8_t> live_;
    std::vector<uint8_t> used_;  // push's scratch: OR of the rows' E parts
    std::vector<uint8_t> piv_, row_pad_;  // clean_backward's scratch: pivot flags, the row being scanned
};

}  // namespace rlnc
