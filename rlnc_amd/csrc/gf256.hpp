// gf256.hpp — GF(2^8) arithmetic shared by host and device code of librlnc_hip.
//
// Field: AES polynomial x^8+x^4+x^3+x+1 (0x11B), generator 3 — the field of the reference's
// src/common/gf256.rs:50-51,82-85.  Tables are computed at static-init time from the polynomial (the
// test-suite pins them against the reference's literal LOG/EXP tables).
#pragma once
#include <cstddef>
#include <cstdint>

namespace rlnc {

constexpr uint8_t kBoundaryMarker = 0x81;  // src/full/consts.rs:5

__host__ __device__ constexpr uint8_t gf_xtime(uint8_t a) {
    return static_cast<uint8_t>((a << 1) ^ ((a & 0x80) ? 0x1B : 0x00));
}

// Carry-less multiply reduced by 0x11B; used for table generation and on device for one-off products.
__host__ __device__ constexpr uint8_t gf_mul_slow(uint8_t a, uint8_t b) {
    uint8_t r = 0;
    for (int i = 0; i < 8; ++i) {
        if (b & 1) r ^= a;
        a = gf_xtime(a);
        b >>= 1;
    }
    return r;
}

// Host-side full product / inverse tables (64 KiB + 256 B): the decoder's coefficient elimination
// runs on k×(k+m)-byte matrices where a table lookup per byte is the fastest scalar form.
struct HostField {
    uint8_t mul[256][256];
    uint8_t inv[256];
    HostField() {
        for (int a = 0; a < 256; ++a)
            for (int b = 0; b < 256; ++b) mul[a][b] = gf_mul_slow(static_cast<uint8_t>(a), static_cast<uint8_t>(b));
        inv[0] = 0;
        for (int a = 1; a < 256; ++a)
            for (int b = 1; b < 256; ++b)
                if (mul[a][b] == 1) {
                    inv[a] = static_cast<uint8_t>(b);
                    break;
                }
    }
};

const HostField &host_field();

// The 3-bit-split product tables consumed by v_perm_b32 on device (see kernels.hip):
//   T0[v] = c·v        (v = 0..7)   -> bytes of {t0lo, t0hi}
//   T1[v] = c·(v<<3)   (v = 0..7)   -> bytes of {t1lo, t1hi}
//   T2[v] = c·(v<<6)   (v = 0..3)   -> bytes of t2
struct PermTable {
    uint32_t t0lo, t0hi, t1lo, t1hi, t2;
};

__host__ __device__ inline PermTable make_perm_table(uint8_t c) {
    uint8_t m[8];
    m[0] = c;
    for (int b = 1; b < 8; ++b) m[b] = gf_xtime(m[b - 1]);  // m[b] = c·2^b
    uint8_t t0[8], t1[8], t2[4];
    for (int v = 0; v < 8; ++v) {
        uint8_t a = 0, h = 0;
        for (int b = 0; b < 3; ++b)
            if (v & (1 << b)) {
                a ^= m[b];
                h ^= m[b + 3];
            }
        t0[v] = a;
        t1[v] = h;
    }
    for (int v = 0; v < 4; ++v) {
        uint8_t a = 0;
        for (int b = 0; b < 2; ++b)
            if (v & (1 << b)) a ^= m[b + 6];
        t2[v] = a;
    }
    auto pack = [](const uint8_t *p) -> uint32_t {
        return uint32_t(p[0]) | (uint32_t(p[1]) << 8) | (uint32_t(p[2]) << 16) | (uint32_t(p[3]) << 24);
    };
    return PermTable{pack(t0), pack(t0 + 4), pack(t1), pack(t1 + 4), pack(t2)};
}

}  // namespace rlnc
