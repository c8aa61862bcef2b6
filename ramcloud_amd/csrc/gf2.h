// GF(2)[x] / P arithmetic for CRC-32C, shared by host and device code.
//
// Representation: the *reflected* 32-bit form RAMCloud's Crc32C state uses
// (src/Crc32C.h:39-153): bit 31 holds the coefficient of x^0, bit 0 that of
// x^31.  P is the Castagnoli polynomial, reflected 0x82F63B78
// (src/Crc32C.cc:73, :96-100).
//
// Every CRC operator the kernels use is multiplication by a constant power of
// x, so all of them commute.  Writing raw(s, M) for the state after
// update(M) from state s, and X^n for "append n zero bytes":
//     X^n(v)         = v * x^(8n) mod P
//     raw(s, M)      = X^|M|(s) ^ raw(0, M)
//     raw(0, A || B) = X^|B|(raw(0, A)) ^ raw(0, B)
//     word w at byte offset o of an n-byte message contributes X^(n-o)(w).
// An X^d operator is applied with four byte-indexed tables (OpTable).
//
// Tables are generated from the polynomial at compile time (constexpr); none
// is copied from the reference.
#pragma once

#include <stdint.h>

#if defined(__HIPCC__)
#define RAMCRC_HD __host__ __device__
#else
#define RAMCRC_HD
#endif

namespace ramcrc {

constexpr uint32_t kPoly = 0x82F63B78u;   // reflected 0x1EDC6F41
constexpr uint32_t kOne = 0x80000000u;    // the polynomial 1
constexpr uint32_t kX8 = 0x00800000u;     // x^8 (one zero byte)

// a * b mod P.
RAMCRC_HD constexpr uint32_t mulmod(uint32_t a, uint32_t b)
{
    uint32_t p = 0;
    for (int i = 0; i < 32; i++) {
        if (a & (kOne >> i))
            p ^= b;
        b = (b >> 1) ^ ((b & 1u) ? kPoly : 0u);
    }
    return p;
}

// x^(8n) mod P: the constant of X^n.
RAMCRC_HD constexpr uint32_t xpow8(uint64_t n)
{
    uint32_t r = kOne, sq = kX8;
    while (n) {
        if (n & 1)
            r = mulmod(r, sq);
        sq = mulmod(sq, sq);
        n >>= 1;
    }
    return r;
}

// x^-1 mod P.  P = x^32 + p(x) with p(0) = 1, so x * ((P + 1) / x) = P + 1 = 1
// (mod P): the inverse is x^31 + (p(x) - 1) / x.  In reflected form the x^i
// coefficient of p sits at bit 31-i; dividing by x moves it to bit 32-i.
constexpr uint32_t kXInv = ((kPoly & 0x7FFFFFFFu) << 1) | 1u;

RAMCRC_HD constexpr uint32_t xinv8pow(uint64_t n)  // x^(-8n) mod P
{
    uint32_t inv8 = kOne;
    for (int i = 0; i < 8; i++)
        inv8 = mulmod(inv8, kXInv);
    uint32_t r = kOne, sq = inv8;
    while (n) {
        if (n & 1)
            r = mulmod(r, sq);
        sq = mulmod(sq, sq);
        n >>= 1;
    }
    return r;
}

// Four byte tables applying X^d: X^d(v) = t[0][v&255] ^ t[1][(v>>8)&255] ^
// t[2][(v>>16)&255] ^ t[3][v>>24].
struct OpTable {
    uint32_t t[4][256];
};

constexpr OpTable make_op(uint64_t d)
{
    OpTable op{};
    const uint32_t c = xpow8(d);
    for (int k = 0; k < 4; k++)
        for (uint32_t b = 0; b < 256; b++)
            op.t[k][b] = mulmod(b << (8 * k), c);
    return op;
}

RAMCRC_HD inline uint32_t apply_op(const OpTable& op, uint32_t v)
{
    return op.t[0][v & 0xFF] ^ op.t[1][(v >> 8) & 0xFF] ^ op.t[2][(v >> 16) & 0xFF] ^
           op.t[3][v >> 24];
}

// X^1 byte table: t0[b] = raw(0, byte b); equals OpTable(1).t[0].
struct ByteTable {
    uint32_t t[256];
};

constexpr ByteTable make_byte_table()
{
    ByteTable bt{};
    for (uint32_t i = 0; i < 256; i++) {
        uint32_t x = i;
        for (int j = 0; j < 8; j++)
            x = (x >> 1) ^ ((x & 1u) ? kPoly : 0u);
        bt.t[i] = x;
    }
    return bt;
}

}  // namespace ramcrc
