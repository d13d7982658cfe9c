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
    uint32_t nib;   // masks stored as nibble codes (RowsImage::nib)
    uint32_t term;  // terminal records (RowsImage::term): `table` is the TT table
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

// TERMINAL records (r06, MBRWT_BUILD_ROWS_CODE = 2; rows.hip
// build_term_tables): a row's descent as the leaf parents and leaves it
// reaches ("terminals"), in pre-order, each a w-bit field {terminal id
// [0, ib), its children mask [ib, w)} packed LSB-first -- the internal
// nodes' masks are implied by the terminals below them.  The TT table: [0]
// w | ib << 8, [1] nT, [2..3] 0, nT RWT2 entry words (leaf / leaf parent /
// listed leaf parent: term_label's forms), then the u16 column lists.  The
// fields are read until the record's count of labels is reached.
__device__ __forceinline__ uint32_t tt_label(uint32_t e, const uint16_t *lst, uint32_t bit) {
    const uint32_t i = (e & 0xFFFFu) + bit;
    return ((e >> 29) & 1u) ? (uint32_t)lst[i] : i;
}
struct NoTerm {
    __device__ void operator()(uint32_t) const {}
};
template <class ByteFn, class LeafFn, class TermFn = NoTerm>
__device__ bool term_walk(const uint32_t *tt, ByteFn byte, uint32_t count, LeafFn leaf, TermFn onterm = TermFn()) {
    const uint32_t hdr = tt[0], w = hdr & 0xFFu, ib = (hdr >> 8) & 0xFFu, nT = tt[1];
    const uint32_t *ent = tt + 4;
    const uint16_t *lst = reinterpret_cast<const uint16_t *>(ent + nT);
    uint32_t left = count, bit = 0;
    while (left) {
        const uint32_t b0 = bit >> 3, sh = bit & 7u;
        uint64_t v = 0;
        for (uint32_t k = 0; 8u * k < sh + w; ++k) v |= (uint64_t)byte(b0 + k) << (8u * k);
        const uint32_t f = (uint32_t)(v >> sh) & ((1u << w) - 1u);
        bit += w;
        const uint32_t id = f & ((1u << ib) - 1u);
        if (id >= nT) return false;
        const uint32_t e = ent[id];
        uint32_t x = (e >> 30) == 3u ? (f >> ib) : 1u;  // a leaf parent: its set children; a leaf: itself
        if (!x) return false;
        onterm(id);
        for (; x && left; x &= x - 1u, --left) leaf(tt_label(e, lst, (uint32_t)__builtin_ctz(x)));
        if (x) return false;  // (more labels than the record's count)
    }
    return true;
}
// one record's labels in pre-order, whatever its form: leaf(column) per
// label, inner(arity) per mask read (the mask forms only)
template <class ByteFn, class LeafFn, class InnerFn>
__device__ __forceinline__ bool record_walk_bytes(const RowsView &v, const uint32_t *table, ByteFn byte, uint32_t count,
                                                  LeafFn leaf, InnerFn inner) {
    if (v.term) return term_walk(table, byte, count, leaf);
    return rwt_walk(table, rec_masks(byte, v.nib), leaf, inner);
}
template <class LeafFn, class InnerFn>
__device__ __forceinline__ bool record_walk(const RowsView &v, const uint32_t *table, uint64_t masks, uint32_t count,
                                            LeafFn leaf, InnerFn inner) {
    return record_walk_bytes(v, table, [&](uint32_t o) { return (uint32_t)gld_at<uint8_t>(masks + o); }, count, leaf,
                             inner);
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
