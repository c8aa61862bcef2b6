// Test double for RAMCloud::Buffer (src/Buffer.h): just enough of the chunk
// list and Buffer::Iterator (src/Buffer.h:482-556, src/Buffer.cc:838-975) for
// the drop-in Crc32C.h to compile and for update(Buffer&, off, len) to walk
// real multi-chunk buffers in tests/cpp/crc32c_test.cc.  Not used by the
// library itself.
#ifndef RAMCRC_TEST_BUFFER_H
#define RAMCRC_TEST_BUFFER_H

#include <stddef.h>
#include <stdint.h>

#include <vector>

namespace RAMCloud {

class Buffer {
  public:
    void appendExternal(const void* data, uint32_t length)
    {
        chunks.push_back(Chunk{static_cast<const uint8_t*>(data), length});
        total += length;
    }
    uint32_t size() const { return total; }

    class Iterator {
      public:
        Iterator(Buffer* buffer, uint32_t offset, uint32_t length)
            : buf(buffer), index(0), skip(offset), remaining(length), data(nullptr), len(0)
        {
            settle();
        }
        bool isDone() const { return remaining == 0 || index >= buf->chunks.size(); }
        const void* getData() const { return data; }
        uint32_t getLength() const { return len; }
        void next()
        {
            remaining -= len;
            index++;
            skip = 0;
            settle();
        }

      private:
        void settle()
        {
            while (index < buf->chunks.size() && skip >= buf->chunks[index].length) {
                skip -= buf->chunks[index].length;
                index++;
            }
            if (isDone()) {
                data = nullptr;
                len = 0;
                return;
            }
            const Chunk& c = buf->chunks[index];
            data = c.data + skip;
            len = c.length - skip;
            if (len > remaining)
                len = remaining;
        }
        Buffer* buf;
        size_t index;
        uint32_t skip, remaining;
        const uint8_t* data;
        uint32_t len;
    };

  private:
    struct Chunk {
        const uint8_t* data;
        uint32_t length;
    };
    std::vector<Chunk> chunks;
    uint32_t total = 0;
};

}  // namespace RAMCloud

#endif
