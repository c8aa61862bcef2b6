// Drop-in test: include/ramcloud/Crc32C.h + ramcloud_amd/dropin/Crc32C.cc +
// libramcrc, exercised the way src/Crc32CTest.cc exercises the reference
// class (parameterised over forceSoftware, src/Crc32CTest.cc:64-68):
//   single            every prefix of the known-answer input   (:70-75)
//   accumulated       byte-at-a-time chaining + getResult       (:77-82)
//   accumulatedVaried several split patterns                    (:84-109)
//   updateFromBuffer  pointer and multi-chunk Buffer paths agree (:111-127)
//   assignmentOperator / copy-and-extend                         (:129-134,
//                     src/Segment.cc:677-681)
// plus the Segment certificate and Object checksum goldens.  The vectors are
// read from a text file written by tests/test_cxx_dropin.py from
// tests/golden/crc32c_golden.json (no reference source is embedded here).
#define PRIVATE public  // like EXPOSE_PRIVATES (src/Minimal.h:40-54)
#include "Crc32C.h"

#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <string>
#include <vector>

using RAMCloud::Buffer;
using RAMCloud::Crc32C;

static int failures = 0;

#define EXPECT_EQ(a, b)                                                                   \
    do {                                                                                  \
        unsigned long long a_ = (a), b_ = (b);                                            \
        if (a_ != b_) {                                                                   \
            fprintf(stderr, "%s:%d: EXPECT_EQ(%s, %s) failed: 0x%llx != 0x%llx\n",        \
                    __FILE__, __LINE__, #a, #b, a_, b_);                                  \
            failures++;                                                                   \
        }                                                                                 \
    } while (0)

static std::vector<uint8_t> unhex(const std::string& s)
{
    std::vector<uint8_t> out;
    for (size_t i = 0; i + 1 < s.size(); i += 2)
        out.push_back(static_cast<uint8_t>(strtoul(s.substr(i, 2).c_str(), nullptr, 16)));
    return out;
}

struct Vectors {
    std::vector<uint8_t> input;
    std::vector<uint32_t> crcByLength;
    std::vector<std::pair<std::vector<uint8_t>, uint32_t>> golden;  // certs + objects
};

static Vectors load(const char* path)
{
    Vectors v;
    FILE* f = fopen(path, "r");
    if (!f) {
        perror(path);
        exit(2);
    }
    char key[32];
    static char buf[1 << 16];
    while (fscanf(f, "%31s %65535s", key, buf) == 2) {
        if (!strcmp(key, "INPUT")) {
            v.input = unhex(buf);
        } else if (!strcmp(key, "CRC")) {
            v.crcByLength.push_back(static_cast<uint32_t>(strtoul(buf, nullptr, 16)));
        } else if (!strcmp(key, "GOLDEN")) {
            unsigned crc = 0;
            if (fscanf(f, "%x", &crc) != 1)
                exit(2);
            v.golden.emplace_back(unhex(buf), crc);
        }
    }
    fclose(f);
    return v;
}

static void run(const Vectors& v, bool forceSoftware)
{
    const uint8_t* input = v.input.data();
    const uint32_t n = static_cast<uint32_t>(v.input.size());

    // single
    for (uint32_t i = 0; i <= n; i++)
        EXPECT_EQ(v.crcByLength[i], Crc32C(forceSoftware).update(input, i).getResult());

    // accumulated
    {
        Crc32C crc(forceSoftware);
        EXPECT_EQ(v.crcByLength[0], crc.getResult());
        for (uint32_t i = 0; i < n; i++)
            EXPECT_EQ(v.crcByLength[i + 1], crc.update(&input[i], 1).getResult());
    }

    // accumulatedVaried: every split point pair (a, b) of the input
    for (uint32_t a = 0; a <= n; a += 3) {
        for (uint32_t b = a; b <= n; b += 5) {
            Crc32C crc(forceSoftware);
            crc.update(input, a);
            EXPECT_EQ(v.crcByLength[a], crc.getResult());
            crc.update(input + a, b - a);
            EXPECT_EQ(v.crcByLength[b], crc.getResult());
            crc.update(input + b, n - b);
            EXPECT_EQ(v.crcByLength[n], crc.getResult());
        }
    }

    // updateFromBuffer: contiguous vs multi-chunk Buffer, whole and offset
    {
        static uint8_t big[65536 + 37];
        for (size_t i = 0; i < sizeof(big); i++)
            big[i] = static_cast<uint8_t>(i * 131 + (i >> 7));
        Buffer buffer;
        const uint32_t cuts[] = {1, 7, 64, 1000, 3, 30000, 4096};
        uint32_t pos = 0;
        for (uint32_t c : cuts) {
            buffer.appendExternal(big + pos, c);
            pos += c;
        }
        buffer.appendExternal(big + pos, sizeof(big) - pos);
        Crc32C a(forceSoftware), b(forceSoftware);
        a.update(big, sizeof(big));
        b.update(buffer);
        EXPECT_EQ(a.result, b.result);
        Crc32C c(forceSoftware), d(forceSoftware);
        c.update(&big[5], sizeof(big) - 11);
        d.update(buffer, 5, sizeof(big) - 11);
        EXPECT_EQ(c.result, d.result);
    }

    // assignmentOperator and the fork-and-extend of Segment::getAppendedLength
    {
        Crc32C a(forceSoftware);
        a.update(&a, sizeof(a));
        Crc32C b = a;
        EXPECT_EQ(a.result, b.result);
        Crc32C c(forceSoftware);
        c = a;
        EXPECT_EQ(a.result, c.result);
        Crc32C fork = a;
        fork.update(input, 4);
        Crc32C again = a;
        again.update(input, 4);
        EXPECT_EQ(fork.getResult(), again.getResult());
        EXPECT_EQ(a.result, c.result);  // the fork left the original untouched
    }

    // Segment certificate and Object checksum goldens
    for (const auto& g : v.golden)
        EXPECT_EQ(g.second, Crc32C(forceSoftware)
                                .update(g.first.data(), static_cast<uint32_t>(g.first.size()))
                                .getResult());

    // large buffers through the interleaved hardware path, odd offsets
    {
        std::vector<uint8_t> big(3 * 8192 * 4 + 123);
        for (size_t i = 0; i < big.size(); i++)
            big[i] = static_cast<uint8_t>((i * 2654435761u) >> 13);
        for (uint32_t off = 0; off < 9; off++) {
            const uint32_t len = static_cast<uint32_t>(big.size() - off - 3);
            Crc32C hw(false), sw(true);
            hw.update(big.data() + off, len);
            sw.update(big.data() + off, len);
            EXPECT_EQ(hw.getResult(), sw.getResult());
        }
    }
}

// The free functions and table names of the reference header
// (src/Crc32C.h:25-34,39-153): intelCrc32C / softwareCrc32C agree with the
// class on every known-answer prefix, and a slicing-by-8 written against the
// Crc32CSlicingBy8 names (byte j of an 8-byte block through the table of its
// distance 7 - j from the block end: o88 for byte 0 .. o32 for byte 7) gives
// the same states -- so each name holds the table the reference's does.
static uint32_t
slicing8(uint32_t crc, const uint8_t* p, size_t n)
{
    using namespace Crc32CSlicingBy8;
    for (; n >= 8; n -= 8, p += 8) {
        const uint32_t x = crc ^ (uint32_t(p[0]) | uint32_t(p[1]) << 8 | uint32_t(p[2]) << 16 |
                                  uint32_t(p[3]) << 24);
        crc = crc_tableil8_o88[x & 0xFF] ^ crc_tableil8_o80[(x >> 8) & 0xFF] ^
              crc_tableil8_o72[(x >> 16) & 0xFF] ^ crc_tableil8_o64[x >> 24] ^
              crc_tableil8_o56[p[4]] ^ crc_tableil8_o48[p[5]] ^ crc_tableil8_o40[p[6]] ^
              crc_tableil8_o32[p[7]];
    }
    for (; n; n--, p++)
        crc = crc_tableil8_o32[(crc ^ *p) & 0xFF] ^ (crc >> 8);
    return crc;
}

static void
free_functions(const Vectors& v)
{
    const uint8_t* in = reinterpret_cast<const uint8_t*>(v.input.data());
    for (size_t i = 0; i <= v.input.size(); i++) {
        EXPECT_EQ(v.crcByLength[i], ~RAMCloud::intelCrc32C(0xFFFFFFFFu, in, i));
        EXPECT_EQ(v.crcByLength[i], ~RAMCloud::softwareCrc32C(0xFFFFFFFFu, in, i));
        EXPECT_EQ(v.crcByLength[i], ~slicing8(0xFFFFFFFFu, in, i));
    }
    // the drop-in's arrays (real arrays, as the reference declares them) hold
    // libramcrc's tables word for word
    const uint32_t* const names[8] = {
        Crc32CSlicingBy8::crc_tableil8_o32, Crc32CSlicingBy8::crc_tableil8_o40,
        Crc32CSlicingBy8::crc_tableil8_o48, Crc32CSlicingBy8::crc_tableil8_o56,
        Crc32CSlicingBy8::crc_tableil8_o64, Crc32CSlicingBy8::crc_tableil8_o72,
        Crc32CSlicingBy8::crc_tableil8_o80, Crc32CSlicingBy8::crc_tableil8_o88};
    const uint32_t* lib = ramcrc_slice8_tables();
    for (int k = 0; k < 8; k++)
        for (int b = 0; b < 256; b++)
            EXPECT_EQ(lib[256 * k + b], names[k][b]);
    static_assert(sizeof(Crc32CSlicingBy8::crc_tableil8_o88) == 256 * sizeof(uint32_t),
                  "array type, as src/Crc32C.h:25-34 declares");
    std::vector<uint8_t> big(4099);
    for (size_t i = 0; i < big.size(); i++)
        big[i] = static_cast<uint8_t>((i * 40503u) >> 5);
    for (size_t off = 0; off < 8; off++) {
        const uint32_t s = static_cast<uint32_t>(0x9E3779B9u * (off + 1));
        EXPECT_EQ(RAMCloud::intelCrc32C(s, big.data() + off, big.size() - off),
                  slicing8(s, big.data() + off, big.size() - off));
    }
}

int main(int argc, char** argv)
{
    if (argc < 2) {
        fprintf(stderr, "usage: %s vectors.txt\n", argv[0]);
        return 2;
    }
    const Vectors v = load(argv[1]);
    if (v.input.empty() || v.crcByLength.size() != v.input.size() + 1) {
        fprintf(stderr, "bad vector file\n");
        return 2;
    }
    run(v, false);
    run(v, true);
    free_functions(v);
    printf("haveHardware=%d failures=%d\n", Crc32C::haveHardware ? 1 : 0, failures);
    return failures ? 1 : 0;
}
