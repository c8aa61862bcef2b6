// Replaces RAMCloud's src/Crc32C.cc when include/ramcloud/Crc32C.h replaces
// src/Crc32C.h: defines the process-wide hardware flag (src/Crc32C.cc:41-45)
// and the reference's slicing-by-8 tables under their names
// (src/Crc32C.cc:108-537) -- generated here from the polynomial at compile
// time (constant initialisation, no static-init order dependence), with the
// same values as libramcrc's ramcrc_slice8_tables (tests/cpp/crc32c_test.cc
// compares them word for word).
//
// Compiled by the embedding project (RAMCloud's own build, or
// tests/cpp/Makefile here) next to its Buffer.h; link with -lramcrc.
#include "Crc32C.h"

namespace Crc32CSlicingBy8 {
namespace {

// Table k, byte b: the CRC state after feeding byte b followed by k zero bytes
// into a zero state (reflected Castagnoli polynomial 0x82F63B78), which is
// what slicing-by-8 looks up for the byte k positions before the end of an
// 8-byte group.  C++11 constexpr (RAMCloud builds with -std=c++11).
constexpr uint32_t bit_step(uint32_t c) { return (c >> 1) ^ ((c & 1u) ? 0x82F63B78u : 0u); }
constexpr uint32_t byte_step(uint32_t c)
{
    return bit_step(bit_step(bit_step(bit_step(bit_step(bit_step(bit_step(bit_step(c))))))));
}
constexpr uint32_t zero_step(uint32_t x) { return (x >> 8) ^ byte_step(x & 0xFFu); }
constexpr uint32_t entry(int k, uint32_t b) { return k == 0 ? byte_step(b) : zero_step(entry(k - 1, b)); }
static_assert(entry(0, 1) == 0xF26B8303u, "CRC-32C byte table");

}  // namespace

#define RAMCRC_E(k, i) entry(k, i)
#define RAMCRC_R4(k, i) RAMCRC_E(k, i), RAMCRC_E(k, i + 1), RAMCRC_E(k, i + 2), RAMCRC_E(k, i + 3)
#define RAMCRC_R16(k, i) RAMCRC_R4(k, i), RAMCRC_R4(k, i + 4), RAMCRC_R4(k, i + 8), RAMCRC_R4(k, i + 12)
#define RAMCRC_R64(k, i) \
    RAMCRC_R16(k, i), RAMCRC_R16(k, i + 16), RAMCRC_R16(k, i + 32), RAMCRC_R16(k, i + 48)
#define RAMCRC_R256(k) RAMCRC_R64(k, 0), RAMCRC_R64(k, 64), RAMCRC_R64(k, 128), RAMCRC_R64(k, 192)

const uint32_t crc_tableil8_o32[256] = {RAMCRC_R256(0)};
const uint32_t crc_tableil8_o40[256] = {RAMCRC_R256(1)};
const uint32_t crc_tableil8_o48[256] = {RAMCRC_R256(2)};
const uint32_t crc_tableil8_o56[256] = {RAMCRC_R256(3)};
const uint32_t crc_tableil8_o64[256] = {RAMCRC_R256(4)};
const uint32_t crc_tableil8_o72[256] = {RAMCRC_R256(5)};
const uint32_t crc_tableil8_o80[256] = {RAMCRC_R256(6)};
const uint32_t crc_tableil8_o88[256] = {RAMCRC_R256(7)};

#undef RAMCRC_E
#undef RAMCRC_R4
#undef RAMCRC_R16
#undef RAMCRC_R64
#undef RAMCRC_R256

}  // namespace Crc32CSlicingBy8

namespace RAMCloud {

bool Crc32C::haveHardware = ramcrc_cpu_has_hw() != 0;

}  // namespace RAMCloud
