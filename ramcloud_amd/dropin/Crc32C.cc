// Replaces RAMCloud's src/Crc32C.cc when include/ramcloud/Crc32C.h replaces
// src/Crc32C.h: defines the process-wide hardware flag (src/Crc32C.cc:41-45)
// and binds the reference's table names (src/Crc32C.cc:108-537) to the
// slicing tables libramcrc generates at compile time (ramcrc_host.cc).
//
// Compiled by the embedding project (RAMCloud's own build, or
// tests/cpp/Makefile here) next to its Buffer.h; link with -lramcrc.
#include "Crc32C.h"

namespace Crc32CSlicingBy8 {
namespace {
typedef const uint32_t Table[256];
Table& table(int k) { return *reinterpret_cast<Table*>(ramcrc_slice8_tables() + 256 * k); }
}  // namespace
const uint32_t (&crc_tableil8_o32)[256] = table(0);
const uint32_t (&crc_tableil8_o40)[256] = table(1);
const uint32_t (&crc_tableil8_o48)[256] = table(2);
const uint32_t (&crc_tableil8_o56)[256] = table(3);
const uint32_t (&crc_tableil8_o64)[256] = table(4);
const uint32_t (&crc_tableil8_o72)[256] = table(5);
const uint32_t (&crc_tableil8_o80)[256] = table(6);
const uint32_t (&crc_tableil8_o88)[256] = table(7);
}  // namespace Crc32CSlicingBy8

namespace RAMCloud {

bool Crc32C::haveHardware = ramcrc_cpu_has_hw() != 0;

}  // namespace RAMCloud
