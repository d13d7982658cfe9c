// pack_block.hpp -- KIND_PACK block access for the general kernels (the
// whole 64-byte block in 16 registers, bytes picked by selects; layout in
// mbrwt_internal.hpp).  k_traverse_fast2 reads the same blocks its own way.
#pragma once

#include "device_access.hpp"
#include "mbrwt_internal.hpp"

namespace mbrwt {

struct PackBlock {
    uint32_t w[16];
    uint32_t total;  // set (child, position) pairs of the block
    __device__ __forceinline__ void load(uint64_t base, uint32_t j) {
        const uint64_t blk = base + (uint64_t)(j / kPackSpan) * kPackBlock;
#pragma unroll
        for (int h = 0; h < 4; ++h) {
            const uint4 q = gld_at<uint4>(blk + 16 * h);
            w[4 * h] = q.x;
            w[4 * h + 1] = q.y;
            w[4 * h + 2] = q.z;
            w[4 * h + 3] = q.w;
        }
        total = 0;
#pragma unroll
        for (int h = 0; h < 4; ++h) total += __builtin_popcount(w[4 * h]);
    }
    __device__ __forceinline__ uint32_t bits(uint32_t k) const {  // child k's 16 position bits
        uint32_t x = w[0];
#pragma unroll
        for (int h = 1; h < 4; ++h) x = (k >> 1) == (uint32_t)h ? w[4 * h] : x;
        return (k & 1) ? x >> 16 : x & 0xFFFFu;
    }
    // mask-area byte o (inline, or from the spill list)
    __device__ __forceinline__ uint32_t mask(uint32_t o) const {
        if (total > kPackArea) return gld_at<uint8_t>(((uint64_t)w[2] << 32 | w[1]) + o);
        const uint32_t by = pack_area_byte(o);
        uint32_t x = w[0];
#pragma unroll
        for (int i = 1; i < 16; ++i) x = (by >> 2) == (uint32_t)i ? w[i] : x;
        return (x >> (8 * (by & 3))) & 0xFFu;
    }
};

}  // namespace mbrwt

namespace mbrwt {

// KIND_PACK2 block access for the general kernels (layout in
// mbrwt_internal.hpp): the 64-byte block in 16 registers, record bytes
// picked by selects, or read from the spill list.
struct Pack2Block {
    uint32_t w[16];
    bool spilled;
    uint64_t sa;  // spill list address
    // j: position of the node; span: positions per block (DevNode::stride)
    __device__ __forceinline__ void load(uint64_t base, uint32_t j, uint32_t span) {
        const uint64_t blk = base + (uint64_t)(j / span) * kPack2Block;
#pragma unroll
        for (int h = 0; h < 4; ++h) {
            const uint4 q = gld_at<uint4>(blk + 16 * h);
            w[4 * h] = q.x;
            w[4 * h + 1] = q.y;
            w[4 * h + 2] = q.z;
            w[4 * h + 3] = q.w;
        }
        spilled = (w[0] & 0xFFu) == 0;
        sa = ((uint64_t)w[3] << 32) | w[2];
    }
    __device__ __forceinline__ uint32_t byte(uint32_t o) const {
        if (spilled) return gld_at<uint8_t>(sa + o);
        uint32_t x = w[0];
#pragma unroll
        for (int i = 1; i < 16; ++i) x = (o >> 2) == (uint32_t)i ? w[i] : x;
        return (x >> (8 * (o & 3))) & 0xFFu;
    }
    // byte offset of the record of position t (t = j % span)
    __device__ __forceinline__ uint32_t start(uint32_t t) const {
        if (spilled) return gld_at<uint16_t>(sa + 2ull * t);
        return byte(t);
    }
};

}  // namespace mbrwt

namespace mbrwt {

// DFS walk of the KIND_PACKT record (mbrwt_internal.hpp) of dnode u starting
// at byte o of `byte` (the record's bytes: count, then the masks): leaf(label) for every set leaf
// below u in pre-order (BRWT.cpp:45-51), inner(arity) for every visited
// internal node BELOW u.  Register shift-stack (static indices only).
// Returns false when the subtree is deeper than kPacktMaxDepth.
template <typename ByteFn, typename LeafFn, typename InnerFn>
__device__ __forceinline__ bool packt_walk(const DevNode *__restrict__ nodes, uint32_t u, ByteFn byte, uint32_t o,
                                           LeafFn leaf, InnerFn inner) {
    constexpr int D = (int)kPacktMaxDepth - 1;
    const DevNode nu = gld(nodes + u);
    ++o;  // the record's label count
    uint32_t top_m = byte(o++);
    if (nu.arity > 8) top_m |= byte(o++) << 8;
    uint32_t top_fc = nu.first_child;
    uint32_t sfc[D], sm[D];
#pragma unroll
    for (int k = 0; k < D; ++k) sfc[k] = sm[k] = 0;
    int sp = 0;
    while (true) {
        if (!top_m) {
            if (sp == 0) break;
            top_fc = sfc[0];
            top_m = sm[0];
#pragma unroll
            for (int k = 0; k < D - 1; ++k) {
                sfc[k] = sfc[k + 1];
                sm[k] = sm[k + 1];
            }
            --sp;
            continue;
        }
        const uint32_t c = (uint32_t)__builtin_ctz(top_m);
        top_m &= top_m - 1;
        const DevNode w = gld(nodes + top_fc + c);
        if (w.kind == KIND_LEAF) {
            leaf(w.label);
            continue;
        }
        uint32_t mw = byte(o++);
        if (w.arity > 8) mw |= byte(o++) << 8;
        inner((uint32_t)w.arity);
        if (top_m) {  // the parent still has children to visit
            if (sp == D) return false;
#pragma unroll
            for (int k = D - 1; k > 0; --k) {
                sfc[k] = sfc[k - 1];
                sm[k] = sm[k - 1];
            }
            sfc[0] = top_fc;
            sm[0] = top_m;
            ++sp;
        }
        top_fc = w.first_child;
        top_m = mw;
    }
    return true;
}

}  // namespace mbrwt
