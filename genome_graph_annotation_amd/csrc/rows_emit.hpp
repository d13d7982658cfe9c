// rows_emit.hpp -- the masks of a row's descent over a node image (any of
// its kinds), in DFS pre-order: what the row-record builders (rows.hip,
// rows_var.hip) store per row.  Device code shared by both translation units.
#pragma once

#include "device_access.hpp"
#include "mbrwt_internal.hpp"
#include "pack_block.hpp"

namespace mbrwt {
namespace {

// ------------------------------------------------------------------------
// build: the masks of a row's descent over a node image
// ------------------------------------------------------------------------
// one byte per 8 children (r06: arity up to 64; one or two bytes up to 16)
__device__ __forceinline__ uint32_t rec_mask_bytes(uint32_t arity) { return (arity + 7u) >> 3; }

constexpr int kEmitFrames = 34;  // PLANE levels on a path (<= 32) + the super-root

// the children bits of PLANE node image `nd` at position j (arity <= 64)
__device__ __forceinline__ uint64_t plane_mask(const DevNode &nd, uint32_t j) {
    const uint64_t blk = nd.base + (uint64_t)(j >> 5) * nd.stride;
    const uint32_t t = j & 31;
    uint64_t m = 0;
    for (uint32_t c = 0; c < nd.arity; ++c) m |= (uint64_t)((gld_at<uint2>(blk + 8u * c).y >> t) & 1u) << c;
    return m;
}
__device__ __forceinline__ uint64_t mask_at(const DevNode &nd, uint32_t j) {
    if (nd.kind == KIND_MASK8) return gld_at<uint8_t>(nd.base + j);
    if (nd.kind == KIND_MASK16) return gld_at<uint16_t>(nd.base + 2ull * j);
    if (nd.kind == KIND_MASK32) return gld_at<uint32_t>(nd.base + 4ull * j);
    return gld_at<uint64_t>(nd.base + 8ull * j);
}

// Row r of a node image: emit(mask (u64), arity, dnode) for the children mask of
// every internal node its descent reaches, in DFS pre-order -- the row's record.
// Returns the row's labels (set leaves), or ~0u when the descent is deeper
// than the walker's frames.  Handles every node kind of the images
// (PLANE, MASK*, PACK, PACK2, PACKT, a folded root).
template <class Emit>
__device__ uint32_t emit_row_masks(const DevNode *__restrict__ nodes, bool folded, uint32_t r, Emit emit) {
    uint32_t fv[kEmitFrames], fj[kEmitFrames];
    uint64_t fm[kEmitFrames];
    int sp = 0;
    uint32_t leaves = 0;
    bool bad = false;
    auto push = [&](uint32_t v, uint32_t j, uint64_t m) {
        if (sp == kEmitFrames) {
            bad = true;
            return;
        }
        fv[sp] = v;
        fj[sp] = j;
        fm[sp] = m;
        ++sp;
    };
    // internal dnode v at position j of its image (v's index bit is set there)
    auto visit = [&](uint32_t v, uint32_t j) {
        const DevNode nd = gld(nodes + v);
        const uint32_t a = nd.arity;
        if (nd.kind == KIND_PLANE) {
            const uint64_t m = plane_mask(nd, j);
            emit(m, a, v);
            push(v, j, m);
        } else if (nd.kind >= KIND_MASK8 && nd.kind <= KIND_MASK64) {
            const uint64_t m = mask_at(nd, j);
            emit(m, a, v);
            leaves += (uint32_t)__builtin_popcountll(m);
        } else if (nd.kind == KIND_PACK) {  // children: MASK8 nodes inline
            PackBlock pb;
            pb.load(nd.base, j);
            const uint32_t t = j % kPackSpan;
            uint32_t m = 0;
            for (uint32_t k = 0; k < a; ++k) m |= ((pb.bits(k) >> t) & 1u) << k;
            emit(m, a, v);
            uint32_t o = 0;
            for (uint32_t k = 0; k < a; ++k) {
                const uint32_t bk = pb.bits(k);
                if ((bk >> t) & 1u) {
                    const uint32_t cm = pb.mask(o + (uint32_t)__builtin_popcount(bk & ((1u << t) - 1u)));
                    emit(cm, gld(nodes + nd.first_child + k).arity, nd.first_child + k);
                    leaves += (uint32_t)__builtin_popcount(cm);
                }
                o += (uint32_t)__builtin_popcount(bk);
            }
        } else if (nd.kind == KIND_PACK2) {  // the 3-level subtree inline (level order in the block)
            Pack2Block pb;
            pb.load(nd.base, j, nd.stride);
            const uint32_t s = pb.start(j % nd.stride);
            const uint32_t m2 = pb.byte(s);
            emit(m2, a, v);
            uint32_t o1 = s + 1, o2 = s + 1 + (uint32_t)__builtin_popcount(m2);
            for (uint32_t A = 0; A < a; ++A) {
                if (!((m2 >> A) & 1u)) continue;
                const DevNode na = gld(nodes + nd.first_child + A);
                const uint32_t m1 = pb.byte(o1++);
                emit(m1, na.arity, nd.first_child + A);
                for (uint32_t x = m1; x; x &= x - 1) {
                    const uint32_t bid = na.first_child + (uint32_t)__builtin_ctz(x);
                    const DevNode nb = gld(nodes + bid);
                    const uint32_t lm = pb.byte(o2++);
                    emit(lm, nb.arity, bid);
                    leaves += (uint32_t)__builtin_popcount(lm);
                }
            }
        } else if (nd.kind == KIND_PACKT) {  // the whole subtree inline, already DFS pre-order
            Pack2Block pb;
            pb.load(nd.base, j, nd.stride);
            uint32_t o = pb.start(j % nd.stride) + 1;  // (the record's label count)
            uint32_t m = pb.byte(o++);
            if (a > 8) m |= pb.byte(o++) << 8;
            emit(m, a, v);
            constexpr int D = (int)kPacktMaxDepth;
            uint32_t sfc[D], sm[D];
            int tp = 0;
            sfc[0] = nd.first_child;
            sm[0] = m;
            tp = 1;
            while (tp) {
                const int t = tp - 1;
                if (!sm[t]) {
                    --tp;
                    continue;
                }
                const uint32_t c = (uint32_t)__builtin_ctz(sm[t]);
                sm[t] &= sm[t] - 1;
                const uint32_t wid = sfc[t] + c;
                const DevNode w = gld(nodes + wid);
                if (w.kind == KIND_LEAF) {
                    ++leaves;
                    continue;
                }
                uint32_t mw = pb.byte(o++);
                if (w.arity > 8) mw |= pb.byte(o++) << 8;
                emit(mw, w.arity, wid);
                if (tp == D) {
                    bad = true;
                    return;
                }
                sfc[tp] = w.first_child;
                sm[tp] = mw;
                ++tp;
            }
        } else {
            bad = true;
        }
    };
    const DevNode d0 = gld(nodes);
    if (folded) {  // dnode 0 holds the root's children over rows
        const uint64_t m = d0.kind == KIND_PLANE ? plane_mask(d0, r) : mask_at(d0, r);
        if (!m) return 0;
        emit(m, d0.arity, 0u);
        if (d0.kind == KIND_PLANE) push(0, r, m);
        else leaves += (uint32_t)__builtin_popcountll(m);
    } else {  // dnode 0: the root's own column
        uint32_t bit, jr = 0;
        if (d0.kind == KIND_PLANE) {
            const uint2 rb = gld_at<uint2>(d0.base + (uint64_t)(r >> 5) * d0.stride);
            bit = (rb.y >> (r & 31)) & 1u;
            jr = rb.x + (uint32_t)__builtin_popcount(rb.y & ((1u << (r & 31)) - 1u));
        } else {
            bit = mask_at(d0, r) & 1u;
        }
        if (!bit) return 0;
        if (gld(nodes + d0.first_child).kind == KIND_LEAF) return 1;
        visit(d0.first_child, jr);
    }
    while (sp > 0 && !bad) {
        const int t = sp - 1;
        if (!fm[t]) {
            --sp;
            continue;
        }
        const uint32_t c = (uint32_t)__builtin_ctzll(fm[t]);
        fm[t] &= fm[t] - 1;
        const DevNode nu = gld(nodes + fv[t]);
        const uint32_t w = nu.first_child + c;
        if (gld(nodes + w).kind == KIND_LEAF) {
            ++leaves;
            continue;
        }
        const uint32_t j = fj[t];
        const uint2 rb = gld_at<uint2>(nu.base + (uint64_t)(j >> 5) * nu.stride + 8u * c);
        visit(w, rb.x + (uint32_t)__builtin_popcount(rb.y & ((1u << (j & 31)) - 1u)));
    }
    return bad ? ~0u : leaves;
}

}  // namespace
}  // namespace mbrwt
