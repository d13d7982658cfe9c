// rows_record.hpp -- reading one row record of the block layout (rows.hip):
// the block / spill addressing and the single-lane DFS walk of a record over
// the RWT table.  Shared by the row-record kernels (rows.hip) and the record
// classes (rows_class.hip).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "device_access.hpp"
#include "mbrwt_internal.hpp"

namespace mbrwt {

struct RowsView {
    uint64_t blocks, spill, magic, num_rows;
    uint32_t B, S;
    uint32_t nib;  // masks stored as nibble codes (RowsImage::nib)
};
__device__ __forceinline__ uint64_t rows_block(uint64_t r, uint32_t S, uint64_t magic) {
    return S == 1 ? r : __umul64hi(r, magic);
}
// the record of row r (< num_rows): address of its first mask byte, label count
__device__ __forceinline__ void rows_locate(const RowsView &v, uint64_t r, uint64_t &masks, uint32_t &count) {
    const uint64_t b = rows_block(r, v.S, v.magic);
    const uint32_t t = (uint32_t)(r - b * v.S);
    const uint64_t blk = v.blocks + b * v.B;
    const uint32_t e = gld_at<uint8_t>(blk + t);
    const uint32_t o = e & 0x7Fu;
    if (e & 0x80u) {
        uint32_t idx = 0;
        for (uint32_t k = 0; k < 4; ++k) idx |= (uint32_t)gld_at<uint8_t>(blk + o + 1 + k) << (8 * k);
        const uint64_t se = v.spill + (uint64_t)idx * 16;
        count = gld_at<uint32_t>(se);
        masks = se + 8;
    } else {
        count = gld_at<uint8_t>(blk + o);
        masks = blk + o + 1;
    }
}

// The masks of a record, one per call (mask(arity)), from the record's
// bytes byte(k): one byte per mask (two for arity > 8), or (RowsImage::nib,
// r06) NIBBLE CODES for arity <= 8 -- a mask with one bit set is the nibble
// of its bit's index (0..7), any other mask the nibble 8 and its two halves,
// low first; nibble k is in byte k / 2, low half first.  At the Kingsford
// shape most masks of a row's descent hold one bit (the leaf parents' and
// most of the level above), so a record takes 15.2 instead of 21.3 bytes.
template <class ByteFn>
struct RecMasks {
    ByteFn byte;
    uint32_t nib;
    uint32_t c;
    __device__ __forceinline__ uint32_t nibble(uint32_t k) { return (byte(k >> 1) >> ((k & 1u) * 4u)) & 15u; }
    __device__ __forceinline__ uint64_t operator()(uint32_t a) {
        if (!nib) {  // one byte per 8 children, little-endian (arity <= 64)
            uint64_t m = byte(c++);
            for (uint32_t k = 8; k < a; k += 8) m |= (uint64_t)byte(c++) << k;
            return m;
        }
        const uint32_t v = nibble(c);
        if (v < 8) {
            c += 1;
            return 1u << v;
        }
        const uint32_t m = nibble(c + 1) | nibble(c + 2) << 4;
        c += 3;
        return m;
    }
};
template <class ByteFn>
__device__ __forceinline__ RecMasks<ByteFn> rec_masks(ByteFn byte, uint32_t nib) {
    return RecMasks<ByteFn>{byte, nib, 0u};
}
// the nibbles one mask (arity <= 8, non-zero) takes as a nibble code
__host__ __device__ __forceinline__ uint32_t nib_codes(uint32_t m) { return (m && !(m & (m - 1))) ? 1u : 3u; }

// DFS walk of a record (its masks from `mask`, a RecMasks) over the RWT table
// `table` (mbrwt_internal.hpp): leaf(column) per set leaf in pre-order
// (BRWT.cpp:45-51), inner(arity) per mask read (the root's included).  One
// lane; false past kRowsMaxHeight pending frames, or when a mask names a
// child the table does not have (a corrupt record: an error, not a read past
// the table).  A descent pushes the parent's remaining children BEFORE it
// reads the child's mask, so no mask value lives across the push (r06: the
// other order, with an early return between, was miscompiled in the LDS
// variant below -- the child's mask replaced by the parent's).
template <class MaskFn, class LeafFn, class InnerFn>
__device__ bool rwt_walk(const uint32_t *table, MaskFn mask, LeafFn leaf, InnerFn inner) {
    const uint32_t nI = table[0], nE = table[1];
    const uint32_t *ntab = table + 4;
    const uint32_t *etab = ntab + nI;
    uint32_t nw = ntab[0];
    uint32_t a = nw >> 24;
    uint64_t m = mask(a);
    inner(a);
    uint32_t first = nw & 0xFFFFFFu;
    uint32_t sf[kRowsMaxHeight];
    uint64_t sm[kRowsMaxHeight];
    int sp = 0;
    bool ok = true;
    while (true) {
        if (!m) {
            if (!sp) break;
            --sp;
            first = sf[sp];
            m = sm[sp];
            continue;
        }
        const uint32_t c = (uint32_t)__builtin_ctzll(m);
        m &= m - 1;
        if (first + c >= nE) {
            ok = false;
            break;
        }
        const uint32_t e = etab[first + c];
        if (e & 0x80000000u) {
            leaf(e & 0x7FFFFFFFu);
            continue;
        }
        if (e >= nI || (m && sp == (int)kRowsMaxHeight)) {
            ok = false;
            break;
        }
        if (m) {
            sf[sp] = first;
            sm[sp] = m;
            ++sp;
        }
        nw = ntab[e];
        a = nw >> 24;
        m = mask(a);
        inner(a);
        first = nw & 0xFFFFFFu;
    }
    return ok;
}

// record classes (rows_class.hip): row r's class, bits [r w, r w + w) of the
// packed index (one dword-aligned 8-byte load; the index has a pad word)
__device__ __forceinline__ uint64_t class_field(const uint32_t *index, uint32_t w, uint64_t r) {
    typedef uint64_t u64a4 __attribute__((aligned(4)));
    const uint64_t bit = r * w;
    const uint64_t x = *(const AS_GLOBAL u64a4 *)(uintptr_t)(index + (bit >> 5));
    return (x >> (bit & 31)) & ((1ull << w) - 1);
}

}  // namespace mbrwt
