// image.cpp -- builds the device image of a BRWT from a tree description
// (include/mbrwt.h mbrwt_tree_desc), replacing BRWT::load (BRWT.cpp:87-111)
// as the way structure enters the engine.  Layout: mbrwt_internal.hpp.
#include <algorithm>
#include <chrono>
#include <thread>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "mbrwt_internal.hpp"

namespace mbrwt {

namespace {

inline uint64_t popc(uint64_t x) { return (uint64_t)__builtin_popcountll(x); }

// MBRWT_BUILD_TIMING=1: phase times of the image build on stderr
struct PhaseTimer {
    bool on;
    std::chrono::steady_clock::time_point t;
    PhaseTimer() : t(std::chrono::steady_clock::now()) {
        const char *e = std::getenv("MBRWT_BUILD_TIMING");
        on = e && e[0] == '1';
    }
    void lap(const char *what) {
        if (!on) return;
        const auto now = std::chrono::steady_clock::now();
        std::fprintf(stderr, "[mbrwt image] %s %.1f ms\n", what, std::chrono::duration<double, std::milli>(now - t).count());
        t = now;
    }
};



uint64_t count_ones(const uint64_t *w, uint64_t size) {
    uint64_t c = 0, W = size / 64;
    for (uint64_t k = 0; k < W; ++k) c += popc(w[k]);
    if (size & 63) c += popc(w[W] & ((1ull << (size & 63)) - 1));
    return c;
}

// hipMalloc + copy of a host image; large images are page-locked for the
// copy (pageable copies of freshly built images measured ~0.3 GB/s)
hipError_t upload_bytes(const void *src, size_t bytes, void **out) {
    void *d = nullptr;
    hipError_t e = hipMalloc(&d, bytes);
    if (e != hipSuccess) return e;
    void *h = const_cast<void *>(src);
    const bool reg = bytes >= (1u << 20) && hipHostRegister(h, bytes, hipHostRegisterDefault) == hipSuccess;
    e = hipMemcpy(d, src, bytes, hipMemcpyHostToDevice);
    if (reg) (void)hipHostUnregister(h);
    if (e != hipSuccess) {
        (void)hipFree(d);
        return e;
    }
    *out = d;
    return hipSuccess;
}

// 32-bit chunk b of a bit vector, tail bits past `size` cleared
inline uint32_t chunk32(const uint64_t *w, uint64_t size, uint64_t b) {
    uint64_t lo = b * 32;
    if (lo >= size) return 0;
    uint32_t v = (uint32_t)(w[b >> 1] >> (32 * (b & 1)));
    uint64_t valid = size - lo;
    if (valid < 32) v &= (1u << valid) - 1;
    return v;
}

// Build the children image of one internal dnode: children vectors are
// child_words[c] (length L each).
int upload_image(const std::vector<const uint64_t *> &child_words, const std::vector<bool> &child_is_leaf,
                 uint64_t L, DevNode &dn, std::vector<void *> &images, uint64_t &image_bytes) {
    const uint32_t a = (uint32_t)child_words.size();
    bool all_leaves = std::all_of(child_is_leaf.begin(), child_is_leaf.end(), [](bool b) { return b; });
    std::vector<uint8_t> host;
    if (all_leaves) {
        dn.kind = mask_kind(a);
        const uint32_t w = mask_bytes(dn.kind);
        host.assign(L * w + kImagePad, 0);
        for (uint32_t c = 0; c < a; ++c) {
            const uint64_t *cw = child_words[c];
            const uint64_t W = (L + 63) / 64;
            for (uint64_t k = 0; k < W; ++k) {
                uint64_t x = cw[k];
                if (k == W - 1 && (L & 63)) x &= (1ull << (L & 63)) - 1;
                while (x) {
                    uint64_t j = k * 64 + (uint64_t)__builtin_ctzll(x);
                    x &= x - 1;
                    uint8_t *p = &host[j * w];
                    uint64_t m = 0;
                    std::memcpy(&m, p, w);
                    m |= 1ull << c;
                    std::memcpy(p, &m, w);
                }
            }
        }
    } else {
        dn.kind = KIND_PLANE;
        dn.stride = plane_stride(a);
        const uint64_t blocks = (L + 31) / 32;
        host.assign(blocks * dn.stride + kImagePad, 0);
        for (uint32_t c = 0; c < a; ++c) {
            uint32_t rank = 0;
            for (uint64_t b = 0; b < blocks; ++b) {
                uint32_t bits = chunk32(child_words[c], L, b);
                uint8_t *p = &host[b * dn.stride + 8ull * c];
                std::memcpy(p, &rank, 4);
                std::memcpy(p + 4, &bits, 4);
                rank += (uint32_t)__builtin_popcount(bits);
            }
        }
    }
    dn.arity = (uint16_t)a;
    dn.length = L;
    void *d = nullptr;
    MBRWT_HIP(upload_bytes(host.data(), host.size(), &d));
    images.push_back(d);
    dn.base = (uint64_t)(uintptr_t)d;
    image_bytes += host.size();
    return MBRWT_OK;
}

std::vector<uint8_t> child_masks(const mbrwt_tree_desc &desc, uint32_t v, uint64_t len);


// KIND_PACK image of desc node u (mbrwt_internal.hpp): returns false (and
// builds nothing) when more than 1 block in 20 would spill.
bool build_pack_image(const mbrwt_tree_desc &desc, uint32_t u, uint64_t L, DevNode &dn, std::vector<void *> &images,
                      uint64_t &image_bytes, int &rc) {
    rc = MBRWT_OK;
    const uint32_t a = desc.num_children[u], fc = desc.first_child[u];
    const uint64_t blocks = (L + kPackSpan - 1) / kPackSpan;
    std::vector<uint8_t> host(blocks * kPackBlock + kImagePad, 0);
    std::vector<uint8_t> spill;
    std::vector<std::pair<uint64_t, uint64_t>> spilled;  // (block, offset in spill)
    std::vector<uint64_t> rank(a, 0);
    std::vector<std::vector<uint8_t>> cm(a);  // each MASK8 child's masks over its positions
    for (uint32_t c = 0; c < a; ++c) cm[c] = child_masks(desc, fc + c, desc.vec_size[desc.first_child[fc + c]]);
    std::vector<uint8_t> masks;
    for (uint64_t b = 0; b < blocks; ++b) {
        uint8_t *blk = &host[b * kPackBlock];
        masks.clear();
        for (uint32_t c = 0; c < a; ++c) {
            const uint32_t ch = fc + c;
            const uint64_t *cw = desc.vec_words[ch];
            // bits b*16 .. b*16+15 of the child's column (tail past L cleared)
            const uint64_t j0 = b * kPackSpan;
            uint32_t bits = (uint32_t)(cw[j0 >> 6] >> (j0 & 63)) & 0xFFFFu;
            if (L - j0 < kPackSpan) bits &= (1u << (L - j0)) - 1u;
            const uint16_t b16 = (uint16_t)bits;
            std::memcpy(blk + 16 * (c / 2) + 2 * (c % 2), &b16, 2);
            for (uint32_t x = bits; x; x &= x - 1) masks.push_back(cm[c][rank[c]++]);
        }
        if (masks.size() <= kPackArea) {
            for (uint32_t o = 0; o < masks.size(); ++o) blk[pack_area_byte(o)] = masks[o];
        } else {
            spilled.emplace_back(b, spill.size());
            spill.insert(spill.end(), masks.begin(), masks.end());
        }
    }
    if (spilled.size() * 20 > blocks) return false;
    void *ds = nullptr;
    if (!spill.empty()) {
        spill.resize(spill.size() + kImagePad, 0);
        if (hipMalloc(&ds, spill.size()) != hipSuccess || hipMemcpy(ds, spill.data(), spill.size(),
                                                                      hipMemcpyHostToDevice) != hipSuccess) {
            rc = hip_fail(hipErrorOutOfMemory, "pack spill upload");
            return true;
        }
        images.push_back(ds);
        image_bytes += spill.size();
        for (const auto &sb : spilled) {  // area bytes 0..7 = spill address
            const uint64_t addr = (uint64_t)(uintptr_t)ds + sb.second;
            for (uint32_t k = 0; k < 8; ++k) host[sb.first * kPackBlock + pack_area_byte(k)] = (uint8_t)(addr >> (8 * k));
        }
    }
    void *d = nullptr;
    if (upload_bytes(host.data(), host.size(), &d) != hipSuccess) {
        rc = hip_fail(hipErrorOutOfMemory, "pack image upload");
        return true;
    }
    images.push_back(d);
    image_bytes += host.size();
    dn.kind = KIND_PACK;
    dn.arity = (uint16_t)a;
    dn.stride = kPackBlock;
    dn.length = L;
    dn.base = (uint64_t)(uintptr_t)d;
    return true;
}

// desc node u may become KIND_PACK: 1..8 children, each with 1..8 leaf
// children (MASK8 nodes; their labels are consecutive pre-order indices)
bool pack_candidate(const mbrwt_tree_desc &desc, uint32_t u) {
    const uint32_t a = desc.num_children[u];
    if (a == 0 || a > 8) return false;
    for (uint32_t c = 0; c < a; ++c) {
        const uint32_t ch = desc.first_child[u] + c, gc = desc.num_children[ch];
        if (gc == 0 || gc > 8) return false;
        // (any leaf columns: leaves are labelled by pre-order index, so the
        // leaves below one node are consecutive labels -- finalize_tree)
        for (uint32_t k = 0; k < gc; ++k)
            if (desc.num_children[desc.first_child[ch] + k] != 0) return false;
    }
    return true;
}

// desc node u may become KIND_PACK2: 1..8 children, each a KIND_PACK candidate
bool pack2_candidate(const mbrwt_tree_desc &desc, uint32_t u) {
    const uint32_t a = desc.num_children[u];
    if (a == 0 || a > 8) return false;
    for (uint32_t c = 0; c < a; ++c)
        if (!pack_candidate(desc, desc.first_child[u] + c)) return false;
    return true;
}

// children bits of desc node v (<= 8 children) at each of its len positions,
// by walking the set bits of every child's index column
std::vector<uint8_t> child_masks(const mbrwt_tree_desc &desc, uint32_t v, uint64_t len) {
    std::vector<uint8_t> mk(len, 0);
    const uint64_t W = (len + 63) / 64;
    for (uint32_t k = 0; k < desc.num_children[v]; ++k) {
        const uint64_t *cw = desc.vec_words[desc.first_child[v] + k];
        for (uint64_t w = 0; w < W; ++w) {
            uint64_t x = cw[w];
            if (w == W - 1 && (len & 63)) x &= (1ull << (len & 63)) - 1;
            for (; x; x &= x - 1) mk[w * 64 + (uint64_t)__builtin_ctzll(x)] |= (uint8_t)(1u << k);
        }
    }
    return mk;
}

// The 64-byte record blocks of KIND_PACK2 / KIND_PACKT (mbrwt_internal.hpp)
// from the records of positions 0..L-1 (recs, offsets roff[L+1]): the
// largest span (8, 4, 2, 1 positions per block; any of 8..1 with any_span)
// at which at most 1 block in 20 spills; false (nothing built) when no span qualifies.  Sets dn's
// stride (span), length and base.
bool upload_record_blocks(const std::vector<uint8_t> &recs, const std::vector<uint64_t> &roff, uint64_t L,
                          DevNode &dn, std::vector<void *> &images, uint64_t &image_bytes, int &rc,
                          bool any_span = false) {
    rc = MBRWT_OK;
    for (uint64_t j = 0; j < L; ++j)
        if (roff[j + 1] - roff[j] > kPack2Block) return false;  // a record must fit a block (mbrwt_internal.hpp)
    auto block_bytes = [&](uint64_t b, uint32_t S) {
        return roff[std::min<uint64_t>(L, (b + 1) * S)] - roff[std::min<uint64_t>(L, b * S)];
    };
    uint32_t S = 0;
    uint64_t blocks = 0;
    for (uint32_t span = kPack2MaxSpan; span >= 1 && !S; span = any_span ? span - 1 : span / 2) {
        const uint64_t nb = (L + span - 1) / span;
        uint64_t spills = 0;
        for (uint64_t b = 0; b < nb; ++b) spills += block_bytes(b, span) > pack2_inline(span);
        if (spills * 20 <= nb) {
            S = span;
            blocks = nb;
        }
    }
    if (!S) return false;
    std::vector<uint8_t> host(blocks * kPack2Block + kImagePad, 0);
    std::vector<uint8_t> spill;
    std::vector<std::pair<uint64_t, uint64_t>> spilled;  // (block, offset in spill)
    for (uint64_t b = 0; b < blocks; ++b) {
        const uint64_t j0 = b * S, r0 = roff[std::min<uint64_t>(L, j0)];
        const uint64_t bytes = block_bytes(b, S);
        uint8_t *blk = &host[b * kPack2Block];
        if (bytes <= pack2_inline(S)) {
            for (uint32_t t = 0; t < S; ++t) blk[t] = (uint8_t)(S + roff[std::min<uint64_t>(L, j0 + t)] - r0);
            std::memcpy(blk + S, recs.data() + r0, bytes);
        } else {  // start[0] = 0 marks the block; list = u16 start[S+1], then the records
            spilled.emplace_back(b, spill.size());
            for (uint32_t t = 0; t <= S; ++t) {
                const uint16_t st = (uint16_t)(2 * (S + 1) + roff[std::min<uint64_t>(L, j0 + t)] - r0);
                spill.push_back((uint8_t)st);
                spill.push_back((uint8_t)(st >> 8));
            }
            spill.insert(spill.end(), recs.begin() + r0, recs.begin() + r0 + bytes);
            if (spill.size() & 1) spill.push_back(0);  // keep the u16 starts aligned
        }
    }
    if (!spill.empty()) {
        void *ds = nullptr;
        spill.resize(spill.size() + kImagePad, 0);
        if (hipMalloc(&ds, spill.size()) != hipSuccess || hipMemcpy(ds, spill.data(), spill.size(),
                                                                      hipMemcpyHostToDevice) != hipSuccess) {
            rc = hip_fail(hipErrorOutOfMemory, "record spill upload");
            return true;
        }
        images.push_back(ds);
        image_bytes += spill.size();
        for (const auto &sb : spilled) {
            const uint64_t addr = (uint64_t)(uintptr_t)ds + sb.second;
            std::memcpy(&host[sb.first * kPack2Block + 8], &addr, 8);
        }
    }
    void *d = nullptr;
    if (upload_bytes(host.data(), host.size(), &d) != hipSuccess) {
        rc = hip_fail(hipErrorOutOfMemory, "record image upload");
        return true;
    }
    images.push_back(d);
    image_bytes += host.size();
    dn.stride = S;  // positions per block
    dn.length = L;
    dn.base = (uint64_t)(uintptr_t)d;
    return true;
}

// KIND_PACK2 image of desc node u (mbrwt_internal.hpp) with the largest span
// (8, 4, 2, 1 positions per block) at which at most 1 block in 20 spills;
// returns false (and builds nothing) when no span qualifies.
bool build_pack2_image(const mbrwt_tree_desc &desc, uint32_t u, uint64_t L, DevNode &dn, std::vector<void *> &images,
                       uint64_t &image_bytes, int &rc) {
    rc = MBRWT_OK;
    const uint32_t a = desc.num_children[u], fc = desc.first_child[u];
    // the record of every position (flat, with offsets), from the children
    // masks of u, of every child A and of every grandchild B (set-bit walks)
    PhaseTimer timer;
    const std::vector<uint8_t> m2s = child_masks(desc, u, L);
    std::vector<std::vector<uint8_t>> m1s(a);
    std::vector<std::vector<std::vector<uint8_t>>> lms(a);
    std::vector<uint64_t> lenA(a, 0);
    for (uint32_t A = 0; A < a; ++A) {
        const uint32_t na = fc + A;
        lenA[A] = desc.vec_size[desc.first_child[na]];  // = ones of A's column
        m1s[A] = child_masks(desc, na, lenA[A]);
        lms[A].resize(desc.num_children[na]);
        for (uint32_t B = 0; B < desc.num_children[na]; ++B) {
            const uint32_t nb = desc.first_child[na] + B;
            lms[A][B] = child_masks(desc, nb, desc.vec_size[desc.first_child[nb]]);
        }
    }
    std::vector<uint8_t> recs;
    recs.reserve(L * 4);
    std::vector<uint64_t> roff(L + 1, 0);
    std::vector<uint64_t> rA(a, 0), rB(8 * a, 0);  // running ranks of the A and B columns
    for (uint64_t j = 0; j < L; ++j) {
        const uint32_t m2 = m2s[j];
        recs.push_back((uint8_t)m2);
        uint32_t m1[8] = {0}, jA[8] = {0};
        for (uint32_t x = m2; x; x &= x - 1) {
            const uint32_t A = (uint32_t)__builtin_ctz(x);
            jA[A] = (uint32_t)rA[A]++;
            m1[A] = m1s[A][jA[A]];
            recs.push_back((uint8_t)m1[A]);
        }
        for (uint32_t x = m2; x; x &= x - 1) {
            const uint32_t A = (uint32_t)__builtin_ctz(x);
            for (uint32_t y = m1[A]; y; y &= y - 1) {
                const uint32_t B = (uint32_t)__builtin_ctz(y);
                recs.push_back(lms[A][B][rB[8 * A + B]++]);
            }
        }
        roff[j + 1] = recs.size();
    }
    timer.lap("pack2: masks + records");
    if (!upload_record_blocks(recs, roff, L, dn, images, image_bytes, rc)) return false;
    timer.lap("pack2: blocks + upload");
    dn.kind = KIND_PACK2;
    dn.arity = (uint16_t)a;
    return true;
}

// children bits of desc node v (<= 16 children) at each of its len positions
std::vector<uint16_t> child_masks16(const mbrwt_tree_desc &desc, uint32_t v, uint64_t len) {
    std::vector<uint16_t> mk(len, 0);
    const uint64_t W = (len + 63) / 64;
    for (uint32_t k = 0; k < desc.num_children[v]; ++k) {
        const uint64_t *cw = desc.vec_words[desc.first_child[v] + k];
        for (uint64_t w = 0; w < W; ++w) {
            uint64_t x = cw[w];
            if (w == W - 1 && (len & 63)) x &= (1ull << (len & 63)) - 1;
            for (; x; x &= x - 1) mk[w * 64 + (uint64_t)__builtin_ctzll(x)] |= (uint16_t)(1u << k);
        }
    }
    return mk;
}

// height of desc node u's subtree (0 for a leaf), or UINT32_MAX past
// kPacktMaxDepth / with an arity above kPacktMaxArity
uint32_t packt_height(const mbrwt_tree_desc &desc, uint32_t u) {
    const uint32_t a = desc.num_children[u];
    if (a == 0) return 0;
    if (a > kPacktMaxArity) return UINT32_MAX;
    uint32_t h = 0;
    for (uint32_t c = 0; c < a; ++c) {
        const uint32_t hc = packt_height(desc, desc.first_child[u] + c);
        if (hc == UINT32_MAX) return UINT32_MAX;
        h = std::max(h, hc);
    }
    return h + 1 > kPacktMaxDepth ? UINT32_MAX : h + 1;
}

// KIND_PACKT image of desc node u (mbrwt_internal.hpp): the DFS records of
// its whole subtree; false (nothing built) when a record exceeds 64 bytes or
// no span keeps spills at <= 1 block in 20
bool build_packt_image(const mbrwt_tree_desc &desc, uint32_t u, uint64_t L, const std::vector<uint64_t> &ones,
                       DevNode &dn, std::vector<void *> &images, uint64_t &image_bytes, int &rc) {
    rc = MBRWT_OK;
    std::vector<uint32_t> inner{u};  // internal nodes of the subtree (BFS)
    for (size_t h = 0; h < inner.size(); ++h)
        for (uint32_t c = 0; c < desc.num_children[inner[h]]; ++c) {
            const uint32_t w = desc.first_child[inner[h]] + c;
            if (desc.num_children[w]) inner.push_back(w);
        }
    std::vector<std::vector<uint16_t>> masks(desc.num_nodes);
    std::vector<uint64_t> cnt(desc.num_nodes, 0);
    for (uint32_t v : inner) masks[v] = child_masks16(desc, v, ones[v]);
    std::vector<uint8_t> recs;
    recs.reserve(L * 8);
    std::vector<uint64_t> roff(L + 1, 0);
    auto put = [&](uint32_t v, uint32_t m) {
        recs.push_back((uint8_t)m);
        if (packt_mask_bytes(desc.num_children[v]) == 2) recs.push_back((uint8_t)(m >> 8));
    };
    std::vector<std::pair<uint32_t, uint32_t>> st;  // (node, children still to visit)
    for (uint64_t j = 0; j < L; ++j) {
        const uint32_t m = masks[u][j];
        const size_t at = recs.size();
        recs.push_back(0);  // the label count, set below
        uint32_t labels = 0;
        put(u, m);
        st.assign(1, {u, m});
        while (!st.empty()) {
            auto &top = st.back();
            if (!top.second) {
                st.pop_back();
                continue;
            }
            const uint32_t c = (uint32_t)__builtin_ctz(top.second);
            top.second &= top.second - 1;
            const uint32_t w = desc.first_child[top.first] + c;
            if (!desc.num_children[w]) {
                ++labels;
                continue;
            }
            const uint32_t mw = masks[w][cnt[w]++];
            put(w, mw);
            st.push_back({w, mw});
        }
        if (labels > 255) return false;
        recs[at] = (uint8_t)labels;
        roff[j + 1] = recs.size();
        if (roff[j + 1] - roff[j] > kPack2Block) return false;  // a record must fit a block
    }
    if (!upload_record_blocks(recs, roff, L, dn, images, image_bytes, rc, true)) return false;
    dn.kind = KIND_PACKT;
    dn.arity = (uint16_t)desc.num_children[u];
    return true;
}

}  // namespace


int build_from_desc(const mbrwt_tree_desc &desc, int device, Tree &tree) {
    PhaseTimer timer;
    MBRWT_HIP(hipSetDevice(device));
    tree = Tree();
    tree.num_rows = desc.num_rows;
    tree.num_columns = desc.num_columns;
    const uint32_t N = desc.num_nodes;
    tree.num_nodes = N;
    if (N == 0) {  // BRWT(): no columns, no rows (test_BRWT.cpp:15-19)
        if (desc.num_columns != 0 || desc.num_rows != 0) {
            set_error("empty tree description with nonzero shape");
            return MBRWT_ERR_INVALID;
        }
        return finalize_tree(tree);
    }
    if (!desc.num_children || !desc.first_child || !desc.leaf_column || !desc.vec_size || !desc.vec_words) {
        set_error("null array in tree description");
        return MBRWT_ERR_INVALID;
    }
    if (desc.num_rows > kMaxRows) {
        set_error("num_rows >= 2^32 is not supported by this build");
        return MBRWT_ERR_UNSUPPORTED;
    }
    if (desc.vec_size[0] != desc.num_rows) {
        set_error("root index column length != num_rows");
        return MBRWT_ERR_INVALID;
    }
    // structural validation: BFS numbering, children contiguous, each child
    // column as long as its parent's popcount (BRWT invariant, BRWT.cpp:43)
    std::vector<uint8_t> seen(N, 0);
    std::vector<uint64_t> ones(N);
    uint64_t leaves = 0;
    for (uint32_t u = 0; u < N; ++u) {
        if (!desc.vec_words[u] && desc.vec_size[u]) {
            set_error("null index column");
            return MBRWT_ERR_INVALID;
        }
        ones[u] = desc.vec_size[u] ? count_ones(desc.vec_words[u], desc.vec_size[u]) : 0;
    }
    std::vector<uint8_t> col_seen(desc.num_columns, 0);
    for (uint32_t u = 0; u < N; ++u) {
        const uint32_t a = desc.num_children[u];
        if (a == 0) {
            ++leaves;
            uint32_t col = desc.leaf_column[u];
            if (col >= desc.num_columns || col_seen[col]) {
                set_error("leaf column out of range or duplicated");
                return MBRWT_ERR_INVALID;
            }
            col_seen[col] = 1;
            continue;
        }
        if (a > kMaxArity) {
            set_error("node arity > 64 is not supported by this build");
            return MBRWT_ERR_UNSUPPORTED;
        }
        const uint64_t fc = desc.first_child[u];
        if (fc <= u || fc + a > N) {
            set_error("children not in BFS order");
            return MBRWT_ERR_INVALID;
        }
        for (uint32_t c = 0; c < a; ++c) {
            if (seen[fc + c]++) {
                set_error("node has two parents");
                return MBRWT_ERR_INVALID;
            }
            if (desc.vec_size[fc + c] != ones[u]) {
                set_error("child index column length != parent popcount");
                return MBRWT_ERR_INVALID;
            }
        }
    }
    if (leaves != desc.num_columns) {
        set_error("number of leaves != num_columns");
        return MBRWT_ERR_INVALID;
    }

    tree.nodes.assign(N + 1, DevNode{});
    // leaves and node wiring
    for (uint32_t u = 0; u < N; ++u) {
        DevNode &dn = tree.nodes[u + 1];
        if (desc.num_children[u] == 0) {
            dn.kind = KIND_LEAF;
            dn.label = desc.leaf_column[u];
            tree.num_relations += ones[u];
        } else {
            dn.first_child = desc.first_child[u] + 1;
            dn.label = UINT32_MAX;
        }
        tree.max_arity = std::max<uint32_t>(tree.max_arity, desc.num_children[u]);
    }
    // super-root: its single child is the root -- or, when the root column is
    // at least half full, the root's children expanded to row positions
    // (root folding, mbrwt_internal.hpp)
    timer.lap("validate");
    tree.folded = fold_root_enabled() && desc.num_children[0] > 0 && 2 * ones[0] >= desc.num_rows;
    if (tree.folded) {
        const uint32_t a = desc.num_children[0], fc = desc.first_child[0];
        const uint64_t n = desc.num_rows, W = (n + 63) / 64;
        std::vector<std::vector<uint64_t>> expanded(a, std::vector<uint64_t>(W, 0));
        std::vector<const uint64_t *> cw(a);
        std::vector<bool> leaf(a);
        const uint64_t *root = desc.vec_words[0];
        uint64_t jpos = 0;
        for (uint64_t k = 0; k < W; ++k) {
            uint64_t x = root[k];
            if (k == W - 1 && (n & 63)) x &= (1ull << (n & 63)) - 1;
            while (x) {
                const uint64_t r = k * 64 + (uint64_t)__builtin_ctzll(x);
                x &= x - 1;
                for (uint32_t c = 0; c < a; ++c)
                    if ((desc.vec_words[fc + c][jpos >> 6] >> (jpos & 63)) & 1) expanded[c][r >> 6] |= 1ull << (r & 63);
                ++jpos;
            }
        }
        for (uint32_t c = 0; c < a; ++c) {
            cw[c] = expanded[c].data();
            leaf[c] = desc.num_children[fc + c] == 0;
        }
        DevNode &sr = tree.nodes[0];
        sr.first_child = fc + 1;
        sr.label = UINT32_MAX;
        int rc = upload_image(cw, leaf, n, sr, tree.images, tree.image_bytes);
        if (rc) return rc;
        DevNode &rt = tree.nodes[1];  // absorbed: never visited
        rt.kind = KIND_FOLDED;
        rt.arity = 0;
        rt.first_child = 0;
    } else {
        DevNode &sr = tree.nodes[0];
        sr.first_child = 1;
        sr.label = UINT32_MAX;
        int rc = upload_image({desc.vec_words[0]}, {desc.num_children[0] == 0}, desc.num_rows, sr, tree.images,
                              tree.image_bytes);
        if (rc) return rc;
    }
    timer.lap("super-root");
    // KIND_PACKT: every internal child of the folded root whose subtree fits
    // (any shape), unless the tree is the PACK2 shape of k_traverse_p2w
    std::vector<bool> in_packt(N, false);  // PACKT roots and the internal nodes below them
    if (tree.folded && packt_enabled()) {
        const uint32_t a0 = desc.num_children[0], fc0 = desc.first_child[0];
        bool p2_shape = pack2_enabled();
        for (uint32_t k = 0; k < a0; ++k)
            if (!desc.num_children[fc0 + k] || !pack2_candidate(desc, fc0 + k)) p2_shape = false;
        struct PT {
            uint32_t u;
            bool built = false;
            int rc = MBRWT_OK;
            DevNode dn{};
            std::vector<void *> images;
            uint64_t bytes = 0;
        };
        std::vector<PT> pt;
        // (k_traverse_ptw reads at most 16 root children: a wider root keeps
        // the per-node layout)
        for (uint32_t k = 0; k < a0 && !p2_shape && a0 <= kPacktMaxArity; ++k)
            if (desc.num_children[fc0 + k] && packt_height(desc, fc0 + k) != UINT32_MAX) {
                pt.emplace_back();
                pt.back().u = fc0 + k;
            }
        // one host thread per candidate, at most 16 at a time; the started
        // threads are joined on every path (a failed thread start included)
        for (size_t i0 = 0; i0 < pt.size(); i0 += 16) {
            std::vector<std::thread> pool;
            struct Joiner {
                std::vector<std::thread> &p;
                ~Joiner() {
                    for (auto &t : p)
                        if (t.joinable()) t.join();
                }
            } joiner{pool};
            for (size_t i = i0; i < std::min(pt.size(), i0 + 16); ++i)
                pool.emplace_back([&, i]() {
                    PT &r = pt[i];
                    if (hipSetDevice(device) != hipSuccess) {
                        r.rc = MBRWT_ERR_DEVICE;
                        return;
                    }
                    try {
                        r.built = build_packt_image(desc, r.u, ones[r.u], ones, r.dn, r.images, r.bytes, r.rc);
                    } catch (...) {
                        r.rc = MBRWT_ERR_NOMEM;
                    }
                });
        }
        for (const PT &r : pt) {
            tree.images.insert(tree.images.end(), r.images.begin(), r.images.end());
            tree.image_bytes += r.bytes;
        }
        for (const PT &r : pt) {
            if (r.rc) return r.rc;
            if (!r.built) continue;
            DevNode &dn = tree.nodes[r.u + 1];
            dn.kind = KIND_PACKT;
            dn.arity = r.dn.arity;
            dn.stride = r.dn.stride;
            dn.length = r.dn.length;
            dn.base = r.dn.base;
            in_packt[r.u] = true;
            std::vector<uint32_t> st{r.u};
            while (!st.empty()) {
                const uint32_t v = st.back();
                st.pop_back();
                for (uint32_t c = 0; c < desc.num_children[v]; ++c) {
                    const uint32_t w = desc.first_child[v] + c;
                    if (!desc.num_children[w]) continue;
                    in_packt[w] = true;
                    DevNode &wn = tree.nodes[w + 1];
                    wn.kind = KIND_PACKT_IN;
                    wn.arity = (uint16_t)desc.num_children[w];
                    wn.length = ones[w];
                    wn.base = 0;
                    st.push_back(w);
                }
            }
        }
        timer.lap("packt images");
    }
    // PACK2 candidates are disjoint subtrees (a candidate's descendants are
    // PACK/MASK8-shaped): their images are built concurrently, one host thread
    // per candidate (at most 16 at a time)
    struct P2 {
        uint32_t u;
        bool built = false;
        int rc = MBRWT_OK;
        DevNode dn{};
        std::vector<void *> images;
        uint64_t bytes = 0;
    };
    std::vector<P2> p2;
    if (pack2_enabled())
        for (uint32_t u = 0; u < N; ++u)
            if (desc.num_children[u] && !(u == 0 && tree.folded) && !in_packt[u] && pack2_candidate(desc, u)) {
                p2.emplace_back();
                p2.back().u = u;
            }
    for (size_t i0 = 0; i0 < p2.size(); i0 += 16) {
        std::vector<std::thread> pool;
        struct Joiner {
            std::vector<std::thread> &p;
            ~Joiner() {
                for (auto &t : p)
                    if (t.joinable()) t.join();
            }
        } joiner{pool};
        for (size_t i = i0; i < std::min(p2.size(), i0 + 16); ++i)
            pool.emplace_back([&, i]() {
                P2 &r = p2[i];
                if (hipSetDevice(device) != hipSuccess) {
                    r.rc = MBRWT_ERR_DEVICE;
                    return;
                }
                try {
                    r.built = build_pack2_image(desc, r.u, ones[r.u], r.dn, r.images, r.bytes, r.rc);
                } catch (...) {
                    r.rc = MBRWT_ERR_NOMEM;
                }
            });
        for (auto &t : pool) t.join();
    }
    std::vector<int> p2_of(N, -1);
    for (size_t i = 0; i < p2.size(); ++i) {  // every allocation joins the tree (freed with it)
        tree.images.insert(tree.images.end(), p2[i].images.begin(), p2[i].images.end());
        tree.image_bytes += p2[i].bytes;
        if (p2[i].rc) return p2[i].rc;
        p2_of[p2[i].u] = (int)i;
    }
    timer.lap("pack2 images");
    std::vector<bool> in_pack(N, false);  // MASK8 children of a KIND_PACK node: no image
    for (uint32_t u = 0; u < N; ++u) {
        const uint32_t a = desc.num_children[u];
        if (!a || (u == 0 && tree.folded) || in_pack[u] || in_packt[u]) continue;
        if (p2_of[u] >= 0) {
            const P2 &r = p2[p2_of[u]];
            if (r.built) {
                DevNode &dn = tree.nodes[u + 1];
                dn.kind = r.dn.kind;
                dn.arity = r.dn.arity;
                dn.stride = r.dn.stride;
                dn.length = r.dn.length;
                dn.base = r.dn.base;
                for (uint32_t c = 0; c < a; ++c) {  // children: PACK-shaped records, grandchildren: MASK8 records
                    const uint32_t ch = desc.first_child[u] + c;
                    in_pack[ch] = true;
                    DevNode &cn = tree.nodes[ch + 1];
                    cn.kind = KIND_PACK;
                    cn.arity = (uint16_t)desc.num_children[ch];
                    cn.stride = kPackBlock;
                    cn.length = ones[ch];
                    cn.base = 0;
                    for (uint32_t g = 0; g < desc.num_children[ch]; ++g) {
                        const uint32_t gc = desc.first_child[ch] + g;
                        in_pack[gc] = true;
                        DevNode &gn = tree.nodes[gc + 1];
                        gn.kind = KIND_MASK8;
                        gn.arity = (uint16_t)desc.num_children[gc];
                        gn.length = ones[gc];
                        gn.base = 0;
                    }
                }
                continue;
            }
        }
        if (pack_enabled() && pack_candidate(desc, u)) {
            int rc = MBRWT_OK;
            if (build_pack_image(desc, u, ones[u], tree.nodes[u + 1], tree.images, tree.image_bytes, rc)) {
                if (rc) return rc;
                for (uint32_t c = 0; c < a; ++c) {
                    const uint32_t ch = desc.first_child[u] + c;
                    in_pack[ch] = true;
                    DevNode &cn = tree.nodes[ch + 1];
                    cn.kind = KIND_MASK8;
                    cn.arity = (uint16_t)desc.num_children[ch];
                    cn.length = ones[ch];
                    cn.base = 0;
                }
                continue;
            }
        }
        std::vector<const uint64_t *> cw(a);
        std::vector<bool> leaf(a);
        for (uint32_t c = 0; c < a; ++c) {
            cw[c] = desc.vec_words[desc.first_child[u] + c];
            leaf[c] = desc.num_children[desc.first_child[u] + c] == 0;
        }
        int rc = upload_image(cw, leaf, ones[u], tree.nodes[u + 1], tree.images, tree.image_bytes);
        if (rc) return rc;
    }
    timer.lap("node images");
    const int rc = finalize_tree(tree);
    timer.lap("finalize");
    return rc;
}

int finalize_tree(Tree &tree) {
    const uint32_t D = (uint32_t)tree.nodes.size();
    if (D == 0) return MBRWT_OK;
    // leaves labelled by pre-order index (Tree::label_perm): a DFS from the
    // super-root in child order (the folded root's children hang off dnode 0)
    {
        std::vector<uint32_t> perm;
        std::vector<uint32_t> st{0};
        bool identity = true;
        while (!st.empty()) {
            const uint32_t v = st.back();
            st.pop_back();
            DevNode &dn = tree.nodes[v];
            if (dn.kind == KIND_LEAF && v != 0) {
                identity &= dn.label == (uint32_t)perm.size();
                perm.push_back(dn.label);
                continue;
            }
            if (dn.kind == KIND_FOLDED || dn.kind == KIND_LEAF) continue;
            for (uint32_t c = dn.arity; c-- > 0;) st.push_back(dn.first_child + c);
        }
        tree.label_perm.clear();
        if (!identity) {
            uint32_t k = 0;
            st.assign(1, 0);
            while (!st.empty()) {
                const uint32_t v = st.back();
                st.pop_back();
                DevNode &dn = tree.nodes[v];
                if (dn.kind == KIND_LEAF && v != 0) {
                    dn.label = k++;
                    continue;
                }
                if (dn.kind == KIND_FOLDED || dn.kind == KIND_LEAF) continue;
                for (uint32_t c = dn.arity; c-- > 0;) st.push_back(dn.first_child + c);
            }
            tree.label_perm = std::move(perm);
        }
    }
    // consecutive-label flag for MASK nodes
    for (uint32_t v = 0; v < D; ++v) {
        DevNode &dn = tree.nodes[v];
        if (!is_mask_kind(dn.kind)) continue;
        bool consec = true;
        for (uint32_t c = 0; c < dn.arity; ++c)
            if (tree.nodes[dn.first_child + c].label != tree.nodes[dn.first_child].label + c) consec = false;
        if (consec) {
            dn.flags |= FLAG_CONSEC_LABELS;
            dn.label = tree.nodes[dn.first_child].label;
        }
    }
    // PLANE nodes whose children are all MASK8 nodes with consecutive labels
    for (uint32_t v = 0; v < D; ++v) {
        DevNode &dn = tree.nodes[v];
        if (dn.kind != KIND_PLANE) continue;
        bool all = dn.arity > 0;
        for (uint32_t c = 0; c < dn.arity; ++c) {
            const DevNode &ch = tree.nodes[dn.first_child + c];
            if (ch.kind != KIND_MASK8 || !(ch.flags & FLAG_CONSEC_LABELS)) all = false;
        }
        if (all) dn.flags |= FLAG_MASK_CHILDREN;
    }
    tree.has_pack2 = tree.has_mask_children = tree.has_packt = false;
    for (uint32_t v = 0; v < D; ++v) {
        tree.has_pack2 |= tree.nodes[v].kind == KIND_PACK2;
        tree.has_packt |= tree.nodes[v].kind == KIND_PACKT;
        tree.has_mask_children |= tree.nodes[v].kind == KIND_PLANE && (tree.nodes[v].flags & FLAG_MASK_CHILDREN);
    }
    // shape eligible for the specialised kernel: internal nodes PLANE/MASK8 with
    // arity <= 8, MASK8 labels consecutive, no leaf directly under a PLANE node
    tree.fast_shape = true;
    for (uint32_t v = 0; v < D; ++v) {
        const DevNode &dn = tree.nodes[v];
        if (dn.kind == KIND_LEAF || dn.kind == KIND_FOLDED) continue;
        if (dn.arity > 8 ||
            (dn.kind != KIND_PLANE && dn.kind != KIND_MASK8 && dn.kind != KIND_PACK && dn.kind != KIND_PACK2))
            tree.fast_shape = false;
        if (dn.kind == KIND_MASK8 && !(dn.flags & FLAG_CONSEC_LABELS)) tree.fast_shape = false;
        if (dn.kind == KIND_PLANE)
            for (uint32_t c = 0; c < dn.arity; ++c)
                if (tree.nodes[dn.first_child + c].kind == KIND_LEAF) tree.fast_shape = false;
    }
    // depth-first walk: stack depth (KIND_PLANE frames) and column paths
    std::vector<uint32_t> parent(D, UINT32_MAX), cidx(D, 0), depth(D, 0), planes(D, 0);
    uint32_t max_depth = 0;
    for (uint32_t v = 0; v < D; ++v) {
        const DevNode &dn = tree.nodes[v];
        if (dn.kind == KIND_LEAF || dn.kind == KIND_FOLDED) continue;
        for (uint32_t c = 0; c < dn.arity; ++c) {
            uint32_t w = dn.first_child + c;
            parent[w] = v;
            cidx[w] = c;
            depth[w] = depth[v] + 1;
            planes[w] = planes[v] + (dn.kind == KIND_PLANE ? 1 : 0);
            max_depth = std::max(max_depth, depth[w]);
            tree.stack_depth = std::max(tree.stack_depth, planes[w]);
        }
    }
    tree.path_len = std::max<uint32_t>(1, max_depth);
    if (tree.stack_depth > kFastMaxDepth) tree.fast_shape = false;
    // frames the fast kernels push: PLANE nodes not resolved inline (no FLAG_MASK_CHILDREN)
    {
        std::vector<uint32_t> fr(D, 0);
        tree.push_frames = 0;
        for (uint32_t v = 0; v < D; ++v) {  // BFS order: parents first
            const DevNode &dn = tree.nodes[v];
            const uint32_t here = (parent[v] == UINT32_MAX ? 0 : fr[parent[v]]) +
                                  ((dn.kind == KIND_PLANE && !(dn.flags & FLAG_MASK_CHILDREN)) ? 1 : 0);
            fr[v] = here;
            tree.push_frames = std::max(tree.push_frames, here);
        }
    }
    tree.lds_records = 1;
    for (uint32_t v = 0; v < D; ++v)
        if (tree.nodes[v].kind != KIND_LEAF) tree.lds_records = v + 1;
    tree.lds_complete = tree.lds_records <= kLdsNodes;
    build_p2w_table(tree);
    build_ptw_table(tree);
    tree.col_path.assign(tree.num_columns * tree.path_len, 0);
    tree.col_leaf.assign(tree.num_columns, 0);
    for (uint32_t v = 0; v < D; ++v) {
        const DevNode &dn = tree.nodes[v];
        if (dn.kind != KIND_LEAF || v == 0) continue;
        const uint32_t col = tree.label_perm.empty() ? dn.label : tree.label_perm[dn.label];
        tree.col_leaf[col] = v;
        // path from the super-root down to the leaf
        std::vector<uint8_t> rev;
        for (uint32_t w = v; parent[w] != UINT32_MAX; w = parent[w]) rev.push_back((uint8_t)cidx[w]);
        std::reverse(rev.begin(), rev.end());
        for (size_t k = 0; k < rev.size(); ++k) tree.col_path[(uint64_t)col * tree.path_len + k] = rev[k];
    }
    return MBRWT_OK;
}

// The shape k_traverse_p2w takes: dnode 0 a PLANE node of arity <= 8 whose
// children u are all KIND_PACK2 (arity <= 8), every child A of such u with
// 1..8 children B, every B a KIND_MASK8 node with consecutive labels -- the
// basic arity-8 trees at the Kingsford and RefSeq shapes.  A and B nodes are
// numbered consecutively (BFS), so the table indexes them from the first one.
void build_p2w_table(Tree &tree) {
    tree.p2w_table.clear();
    const auto &N = tree.nodes;
    if (N.empty() || N[0].kind != KIND_PLANE || N[0].arity == 0 || N[0].arity > 8) return;
    const uint32_t R = N[0].arity;
    uint32_t a_lo = UINT32_MAX, a_hi = 0, b_lo = UINT32_MAX, b_hi = 0;
    for (uint32_t k = 0; k < R; ++k) {
        const DevNode &u = N[N[0].first_child + k];
        if (u.kind != KIND_PACK2 || u.arity == 0 || u.arity > 8 || u.stride == 0 || u.stride > kPack2MaxSpan) return;
        for (uint32_t h = 0; h < u.arity; ++h) {
            const uint32_t a = u.first_child + h;
            const DevNode &A = N[a];
            if (A.arity == 0 || A.arity > 8) return;
            a_lo = std::min(a_lo, a);
            a_hi = std::max(a_hi, a);
            for (uint32_t e = 0; e < A.arity; ++e) {
                const uint32_t b = A.first_child + e;
                const DevNode &B = N[b];
                if (B.kind != KIND_MASK8 || !(B.flags & FLAG_CONSEC_LABELS) || B.arity == 0 || B.arity > 8) return;
                b_lo = std::min(b_lo, b);
                b_hi = std::max(b_hi, b);
            }
        }
    }
    const uint32_t nA = a_hi - a_lo + 1, nB = b_hi - b_lo + 1;
    if (4 + 4 * R + nA + nB > kP2wMaxWords) return;
    std::vector<uint32_t> t(4 + 4 * R + nA + nB, 0);
    t[0] = R;
    t[1] = nA;
    t[2] = nB;
    for (uint32_t k = 0; k < R; ++k) {
        const DevNode &u = N[N[0].first_child + k];
        uint32_t lg = 0;
        while ((1u << lg) < u.stride) ++lg;
        t[4 + 4 * k + 0] = (uint32_t)u.base;
        t[4 + 4 * k + 1] = (uint32_t)(u.base >> 32);
        t[4 + 4 * k + 2] = lg;
        t[4 + 4 * k + 3] = u.first_child - a_lo;
    }
    for (uint32_t a = a_lo; a <= a_hi; ++a) t[4 + 4 * R + (a - a_lo)] = N[a].arity ? N[a].first_child - b_lo : 0;
    for (uint32_t b = b_lo; b <= b_hi; ++b) t[4 + 4 * R + nA + (b - b_lo)] = N[b].label;
    tree.p2w_table = std::move(t);
}

// The shape k_traverse_ptw takes: dnode 0 a PLANE node of arity <= 16 (the
// folded root) whose children are leaves or KIND_PACKT nodes; columns and
// local node indices below 2^15 (u16 entries).  The leaf entries hold the
// GLOBAL columns (the walk's order is the output order; no label map
// afterwards).  Layout: mbrwt_internal.hpp.
void build_ptw_table(Tree &tree) {
    tree.ptw_table.clear();
    const auto &N = tree.nodes;
    if (N.empty() || N[0].kind != KIND_PLANE || N[0].arity == 0 || N[0].arity > 16) return;
    const uint32_t R = N[0].arity;
    std::vector<uint32_t> local(N.size(), UINT32_MAX), inner;
    uint32_t height = 0;
    for (uint32_t k = 0; k < R; ++k) {
        const uint32_t u = N[0].first_child + k;
        if (N[u].kind == KIND_LEAF) continue;
        if (N[u].kind != KIND_PACKT || N[u].stride == 0 || N[u].stride > kPack2MaxSpan) return;
        // the subtree's internal nodes, BFS
        const size_t b = inner.size();
        inner.push_back(u);
        std::vector<uint32_t> lvl(1, 1);
        for (size_t h = b; h < inner.size(); ++h) {
            const DevNode &v = N[inner[h]];
            height = std::max(height, lvl[h - b]);
            for (uint32_t c = 0; c < v.arity; ++c)
                if (N[v.first_child + c].kind != KIND_LEAF) {
                    inner.push_back(v.first_child + c);
                    lvl.push_back(lvl[h - b] + 1);
                }
        }
    }
    if (inner.size() >= 0x8000) return;
    for (uint32_t i = 0; i < inner.size(); ++i) local[inner[i]] = i;
    std::vector<uint32_t> nodew(inner.size());
    std::vector<uint16_t> ent;
    for (uint32_t i = 0; i < inner.size(); ++i) {
        const DevNode &v = N[inner[i]];
        if (ent.size() >= 0x10000 || v.arity > kPacktMaxArity) return;
        nodew[i] = (uint32_t)ent.size() | ((uint32_t)v.arity << 24);
        for (uint32_t c = 0; c < v.arity; ++c) {
            const DevNode &w = N[v.first_child + c];
            if (w.kind == KIND_LEAF) {
                const uint32_t col = tree.label_perm.empty() ? w.label : tree.label_perm[w.label];
                if (col >= 0x8000) return;
                ent.push_back((uint16_t)(0x8000u | col));
            } else {
                ent.push_back((uint16_t)local[v.first_child + c]);
            }
        }
    }
    const uint32_t nI = (uint32_t)inner.size(), nE = (uint32_t)ent.size();
    const size_t words = 4 + 4 * (size_t)R + nI + (nE + 1) / 2;
    if (words > kPtwMaxWords) return;
    std::vector<uint32_t> t(words, 0);
    t[0] = R;
    t[1] = nI;
    t[2] = nE;
    t[3] = height;
    for (uint32_t k = 0; k < R; ++k) {
        const uint32_t u = N[0].first_child + k;
        const DevNode &d = N[u];
        uint32_t *e = &t[4 + 4 * k];
        if (d.kind == KIND_LEAF) {
            e[3] = 0x80000000u | (tree.label_perm.empty() ? d.label : tree.label_perm[d.label]);
            continue;
        }
        e[0] = (uint32_t)d.base;
        e[1] = (uint32_t)(d.base >> 32);
        e[2] = d.stride;  // span
        e[3] = local[u];
    }
    std::memcpy(&t[4 + 4 * R], nodew.data(), nI * 4);
    std::memcpy(&t[4 + 4 * R + nI], ent.data(), nE * 2);
    tree.ptw_table = std::move(t);
}

void free_tree(Tree &tree) {
    for (void *p : tree.images) (void)hipFree(p);
    tree.images.clear();
}

}  // namespace mbrwt
