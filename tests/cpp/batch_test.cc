// Crc32CBatch (include/ramcloud/Crc32CBatch.h) as an opt-in RAMCloud caller
// would use it: hostBuffers() over replica-sized and object-sized buffers must
// equal Crc32C().update(buf, len).getResult() for each buffer.
//   batch_test gpu     run on an MI355X and compare
//   batch_test nodev   no GPU present: the wrapper must throw, not crash
#include <stdio.h>
#include <string.h>

#include <stdexcept>
#include <vector>

#include "Crc32C.h"
#include "Crc32CBatch.h"

using namespace RAMCloud;

int main(int argc, char** argv)
{
    const bool gpu = argc > 1 && !strcmp(argv[1], "gpu");
    std::vector<std::vector<uint8_t> > bufs;
    const size_t sizes[] = {0, 1, 3, 4, 100, 1024, 4096, 65536, 1 << 20, 8 << 20, 8 * 1024 * 1024 + 13};
    uint32_t x = 12345;
    for (size_t s : sizes) {
        std::vector<uint8_t> b(s);
        for (size_t i = 0; i < s; i++) {
            x = x * 1103515245u + 12345u;
            b[i] = static_cast<uint8_t>(x >> 16);
        }
        bufs.push_back(b);
    }
    std::vector<std::pair<const void*, uint64_t> > in;
    for (size_t i = 0; i < bufs.size(); i++)
        in.push_back(std::make_pair(static_cast<const void*>(bufs[i].data()),
                                    static_cast<uint64_t>(bufs[i].size())));
    Crc32CBatch batch(0);
    try {
        std::vector<uint32_t> got = batch.hostBuffers(in);
        if (!gpu) {
            fprintf(stderr, "expected an exception without a GPU\n");
            return 1;
        }
        int bad = 0;
        for (size_t i = 0; i < bufs.size(); i++) {
            const uint32_t want = Crc32C().update(bufs[i].data(),
                                                  static_cast<uint32_t>(bufs[i].size())).getResult();
            if (got[i] != want) {
                fprintf(stderr, "buffer %zu (%zu B): 0x%08x != 0x%08x\n", i, bufs[i].size(),
                        got[i], want);
                bad++;
            }
        }
        // write path: assembleObjects stamps header.checksum = Crc32C over
        // bytes [4, len) (Object::computeChecksum, src/Object.cc:805-819)
        std::vector<std::pair<void*, uint64_t> > objs;
        for (size_t i = 0; i < bufs.size(); i++)
            objs.push_back(std::make_pair(static_cast<void*>(bufs[i].data()),
                                          static_cast<uint64_t>(bufs[i].size())));
        std::vector<std::vector<uint8_t> > before = bufs;
        batch.assembleObjects(objs);
        for (size_t i = 0; i < bufs.size(); i++) {
            std::vector<uint8_t> want = before[i];
            if (want.size() >= 24) {
                const uint32_t c = Crc32C().update(&want[4],
                                                   static_cast<uint32_t>(want.size() - 4)).getResult();
                memcpy(&want[0], &c, 4);
            }
            if (want != bufs[i]) {
                fprintf(stderr, "object %zu (%zu B): header checksum mismatch\n", i, want.size());
                bad++;
            }
        }
        printf("gpu batch: %zu buffers, %d mismatches\n", bufs.size(), bad);
        return bad ? 1 : 0;
    } catch (const std::runtime_error& e) {
        printf("exception: %s\n", e.what());
        return gpu ? 1 : 0;
    }
}
