// device_block.hpp -- per-call device staging from the process's device-block cache (geom_block_alloc /
// geom_block_release, csrc/extract.hip): one block carved into 256-byte aligned pieces and returned to the
// cache at scope exit, instead of a hipMalloc / hipFree pair per array per call (hipFree synchronises the
// device; fresh allocations map pages).  The owner synchronises its stream before the scope ends.
#pragma once

#include <algorithm>
#include <cstddef>

#include "mqr_common.hpp"

namespace mqr {

inline size_t block_al256(size_t x) { return (x + 255) & ~size_t(255); }

struct CachedBlock {
    int device;
    void* p = nullptr;
    size_t cap = 0, used = 0;
    CachedBlock(int d, size_t bytes) : device(d) { p = geom_block_alloc(d, std::max<size_t>(bytes, 256), &cap); }
    ~CachedBlock() { geom_block_release(device, p, cap); }
    CachedBlock(const CachedBlock&) = delete;
    CachedBlock& operator=(const CachedBlock&) = delete;
    // the next piece of b bytes, or nullptr when the block is missing or full
    void* take(size_t b) {
        if (!p || used + block_al256(b) > cap) return nullptr;
        char* r = static_cast<char*>(p) + used;
        used += block_al256(b);
        return r;
    }
};

}  // namespace mqr
