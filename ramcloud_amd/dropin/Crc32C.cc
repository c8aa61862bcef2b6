// Replaces RAMCloud's src/Crc32C.cc when include/ramcloud/Crc32C.h replaces
// src/Crc32C.h: defines the process-wide hardware flag (src/Crc32C.cc:41-45).
// The slicing tables the reference file also holds (src/Crc32C.cc:108-537)
// are generated at compile time inside libramcrc (ramcrc_host.cc) instead.
//
// Compiled by the embedding project (RAMCloud's own build, or
// tests/cpp/Makefile here) next to its Buffer.h; link with -lramcrc.
#include "Crc32C.h"

namespace RAMCloud {

bool Crc32C::haveHardware = ramcrc_cpu_has_hw() != 0;

}  // namespace RAMCloud
