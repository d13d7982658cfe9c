// rows.hip -- ROW RECORDS: the BRWT's index bits regrouped by row, and the
// row-record query kernels (layout in mbrwt_internal.hpp "ROW RECORDS",
// DESIGN.md §4/§5).
//
// The reference answers get_row(r) (BRWT.cpp:26-53) by a descent that reads,
// at every internal node u it reaches, the index bits of u's children at
// j = rank1(u, i) - 1 (BRWT.cpp:30, :43).  Those bits -- the children mask of
// u at the row's position -- belong to row r alone: every bit of every index
// column is reached by exactly one row.  A row's RECORD is the masks of its
// descent in DFS pre-order (the order the reference visits them, BRWT.cpp:
// 45-51), so the records of all rows are a permutation of the tree's index
// bits, and get_row is one 64- or 128-byte block read plus a walk of the
// record over the tree's shape (the RWT table, in LDS): the rank1 remaps are
// resolved once, when the image is built from a node image (any of its
// layouts), not per query.
//
// Build (rows_build_*): per range of rows, one thread per row walks the node
// image and measures its record (k_rows_measure); the first range decides
// the block size B and rows per block S from the records' sizes
// (k_rows_plan: spilled rows and spill bytes per candidate); one thread per
// block then writes the block and its spill entries (k_rows_write).
//
// Query (rows_get_rows): k_traverse_rows -- one wave per tile of 64 query
// rows: the 64 blocks are read as coalesced 16-byte quarters (one request per
// block) into LDS, a wave scan of the records' label counts places every
// row's labels, the 64 lanes walk their records in lockstep over the RWT table
// writing u16 labels into an LDS stage, which leaves as full-line stores into
// the tile's temp region; one scan over the tile totals and k_compact_tiles
// (u16 -> the caller's u32 CSR, the call's status) follow.  Tiles with more
// labels than their region, or with a record longer than a block, are walked
// by k_compact_tiles itself from the records in global memory.
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <type_traits>
#include <cmath>
#include <cstdio>
#include <cstring>

#include "device_access.hpp"
#include "mbrwt_internal.hpp"
#include "pack_block.hpp"
#include "rows_emit.hpp"
#include "rows_record.hpp"
#include "wave_scan.hpp"

namespace mbrwt {

// ------------------------------------------------------------------------
// layout selection
// ------------------------------------------------------------------------
static thread_local int g_build_layout = LAYOUT_AUTO;  // AUTO: the automatic choice
static thread_local BuildTuning g_build_tuning;        // MBRWT_BUILD_ROWS_VAR .. _ROWS_WGS_PER_CU
BuildTuning &build_tuning() { return g_build_tuning; }
void set_build_tuning(const BuildTuning &t) { g_build_tuning = t; }

int build_layout() { return g_build_layout; }

void set_build_layout(int layout) { g_build_layout = layout; }
int thread_build_layout() { return g_build_layout; }
static thread_local int g_rows_footprint = 0;  // MBRWT_ROWS_FAST
void set_rows_footprint(int v) { g_rows_footprint = v; }
int rows_footprint() { return g_rows_footprint; }

// ------------------------------------------------------------------------
// RWT table
// ------------------------------------------------------------------------
bool build_rwt_table(const Tree &tree, std::vector<uint32_t> &table, uint32_t &height, uint32_t &max_arity) {
    table.clear();
    height = 0;
    max_arity = 0;
    const auto &N = tree.nodes;
    if (N.size() < 2) return false;
    // the logical root: the folded root's children hang off dnode 0
    const bool folded = tree.folded;
    const uint32_t root = folded ? 0u : 1u;
    if (!folded && N[0].arity != 1) return false;
    if (N[root].kind == KIND_LEAF || N[root].arity == 0) return false;  // one-column tree
    auto column_of = [&](const DevNode &d) { return tree.label_perm.empty() ? d.label : tree.label_perm[d.label]; };
    std::vector<uint32_t> inner{root}, level{1};
    std::vector<uint32_t> local(N.size(), UINT32_MAX);
    local[root] = 0;
    for (size_t h = 0; h < inner.size(); ++h) {
        const DevNode &v = N[inner[h]];
        height = std::max(height, level[h]);
        if (v.arity == 0 || v.arity > kRowsMaxArity) return false;
        max_arity = std::max<uint32_t>(max_arity, v.arity);
        for (uint32_t c = 0; c < v.arity; ++c) {
            const uint32_t w = v.first_child + c;
            if (w >= N.size()) return false;
            if (N[w].kind != KIND_LEAF) {
                local[w] = (uint32_t)inner.size();
                inner.push_back(w);
                level.push_back(level[h] + 1);
            }
        }
    }
    if (height > kRowsMaxHeight || inner.size() >= 0x8000) return false;
    std::vector<uint32_t> nodew(inner.size());
    std::vector<uint32_t> ent;  // (r06: u32 entries -- columns up to 2^16; u16 with 15-bit columns before)
    for (size_t i = 0; i < inner.size(); ++i) {
        const DevNode &v = N[inner[i]];
        if (ent.size() + v.arity > 0xFFFFFF) return false;
        nodew[i] = (uint32_t)ent.size() | ((uint32_t)v.arity << 24);
        for (uint32_t c = 0; c < v.arity; ++c) {
            const DevNode &w = N[v.first_child + c];
            if (w.kind == KIND_LEAF) {
                const uint32_t col = column_of(w);
                if (col >= 0x10000) return false;  // (the label stage and temp regions hold u16 labels)
                ent.push_back(0x80000000u | col);
            } else {
                ent.push_back(local[v.first_child + c]);
            }
        }
    }
    const size_t nI = inner.size(), nE = ent.size();
    const size_t words = 4 + nI + nE;
    // (the RWT table stays in global memory -- the one-lane walks read it
    // there -- so only the LDS-staged RWT2 table has kRowsMaxTableWords)
    if (words > (1u << 22)) return false;
    table.assign(words, 0);
    table[0] = (uint32_t)nI;
    table[1] = (uint32_t)nE;
    table[2] = height;
    std::memcpy(&table[4], nodew.data(), nI * 4);
    std::memcpy(&table[4 + nI], ent.data(), nE * 4);
    return true;
}

// RWT2 table (k_traverse_rows): one u32 ENTRY per child of every internal
// node that is not a leaf parent ("LP" nodes, whose labels are base column +
// bit, or entry bit of a column list: no entries, no frame), u32 words
//   [0] the root's entry, [1] nE, [2] frames (non-LP internal levels on a
//   path), [3] 0 (or the path table's offset, append_path_table), nE
//   entries, then the column lists (u16) of the leaf parents whose columns
//   are not consecutive (the greedy partitioner's groups); an entry is
//     leaf      0x80000000 | column
//     LP node   0xC0000000 | arity << 16 | first column
//     LP list   0xE0000000 | arity << 16 | first u16 of its column list
//     internal  arity << 16 | first entry of its children
// so the walk reads ONE table word per visited child.
bool build_rwt2_table(const Tree &tree, std::vector<uint32_t> &t2, uint32_t &frames, std::vector<uint32_t> *slot_dnode) {
    t2.clear();
    frames = 0;
    const auto &N = tree.nodes;
    if (N.size() < 2) return false;
    const bool folded = tree.folded;
    const uint32_t root = folded ? 0u : 1u;
    if (N[root].kind == KIND_LEAF || N[root].arity == 0) return false;
    auto column_of = [&](const DevNode &d) { return tree.label_perm.empty() ? d.label : tree.label_perm[d.label]; };
    // a leaf parent: base = its first column (consecutive: cons) 
    auto is_lp2 = [&](uint32_t v, uint32_t &base, bool &cons) {
        const DevNode &d = N[v];
        cons = true;
        for (uint32_t c = 0; c < d.arity; ++c) {
            const DevNode &w = N[d.first_child + c];
            if (w.kind != KIND_LEAF) return false;
            if (c == 0) base = column_of(w);
            else if (column_of(w) != base + c) cons = false;
        }
        return d.arity > 0;
    };
    auto is_lp = [&](uint32_t v, uint32_t &base) {
        bool cons;
        return is_lp2(v, base, cons);
    };
    std::vector<uint16_t> lists;  // the column lists of non-consecutive leaf parents
    // non-LP internal nodes in BFS order, each with its first entry
    std::vector<uint32_t> order{root}, depth{1}, first;
    uint32_t nE = 0;
    std::vector<uint32_t> first_of(N.size(), 0);
    uint32_t rb = 0;
    bool root_cons = false;
    const bool root_lp = is_lp2(root, rb, root_cons) && root_cons;  // (a listed root: an internal node)
    if (!root_lp) {
        for (size_t h = 0; h < order.size(); ++h) {
            const uint32_t v = order[h];
            const DevNode &d = N[v];
            if (d.arity == 0 || d.arity > kRowsMaxArity) return false;
            frames = std::max(frames, depth[h]);
            first_of[v] = nE;
            nE += d.arity;
            for (uint32_t c = 0; c < d.arity; ++c) {
                const uint32_t w = d.first_child + c;
                uint32_t b;
                if (N[w].kind == KIND_LEAF || is_lp(w, b)) continue;
                order.push_back(w);
                depth.push_back(depth[h] + 1);
            }
        }
    } else if (N[root].arity > kRowsMaxArity) {
        return false;
    }
    if (nE >= 0x10000 || 4 + (size_t)nE > kRowsMaxTableWords) return false;
    auto entry = [&](uint32_t w, uint32_t &out) -> bool {
        const DevNode &d = N[w];
        if (d.kind == KIND_LEAF) {
            const uint32_t col = column_of(d);
            if (col >= 0x10000) return false;
            out = 0x80000000u | col;
            return true;
        }
        if (d.arity == 0 || d.arity > kRowsMaxArity) return false;
        uint32_t b;
        bool cons;
        if (is_lp2(w, b, cons)) {
            if (cons) {
                if (b + d.arity > 0x10000) return false;
                out = 0xC0000000u | ((uint32_t)d.arity << 16) | b;
                return true;
            }
            if (lists.size() + d.arity > 0x10000) return false;
            out = 0xE0000000u | ((uint32_t)d.arity << 16) | (uint32_t)lists.size();
            for (uint32_t c = 0; c < d.arity; ++c) {
                const uint32_t col = column_of(N[d.first_child + c]);
                if (col >= 0x10000) return false;
                lists.push_back((uint16_t)col);
            }
            return true;
        }
        out = ((uint32_t)d.arity << 16) | first_of[w];
        return true;
    };
    t2.assign(4 + nE, 0);
    if (slot_dnode) {  // (terminal records: the dnode of every entry; slot nE = the root)
        slot_dnode->assign(nE + 1, ~0u);
        (*slot_dnode)[nE] = root;
        if (!root_lp)
            for (const uint32_t v : order)
                for (uint32_t c = 0; c < N[v].arity; ++c) (*slot_dnode)[first_of[v] + c] = N[v].first_child + c;
    }
    if (!entry(root, t2[0])) return false;
    t2[1] = nE;
    t2[2] = frames;
    if (!root_lp)
        for (const uint32_t v : order) {
            const DevNode &d = N[v];
            for (uint32_t c = 0; c < d.arity; ++c)
                if (!entry(d.first_child + c, t2[4 + first_of[v] + c])) return false;
        }
    for (size_t i = 0; i < lists.size(); i += 2)
        t2.push_back((uint32_t)lists[i] | (i + 1 < lists.size() ? (uint32_t)lists[i + 1] << 16 : 0u));
    return t2.size() <= kRowsMaxTableWords;
}

// K when every root-to-leaf path of the RWT2 table crosses exactly K internal
// entries (the root included) and then a leaf parent (rows_walk_uni), else 0
uint32_t rwt2_uniform_levels(const std::vector<uint32_t> &t2) {
    if (t2.size() < 4 || (t2[0] >> 30) != 0u) return 0;  // the root is a leaf parent (or a leaf)
    const uint32_t K = t2[2];
    if (K < 1 || K > 5) return 0;
    std::vector<uint32_t> lev{t2[0]};
    for (uint32_t d = 1; d <= K; ++d) {
        std::vector<uint32_t> next;
        for (const uint32_t w : lev) {
            const uint32_t a = (w >> 16) & 0x7Fu, f = w & 0xFFFFu;
            for (uint32_t c = 0; c < a; ++c) {
                if (4 + (size_t)f + c >= t2.size()) return 0;
                const uint32_t e = t2[4 + f + c];
                if ((e >> 29) != (d == K ? 6u : 0u)) return 0;  // consecutive leaf parents exactly at depth K + 1
                if (d < K) next.push_back(e);
            }
        }
        lev.swap(next);
    }
    return K;
}

// The PATH TABLE of a uniform tree (rows_walk_path): every leaf parent's
// first column indexed by the child indices on its path from the root,
// idx = ((c_0 A_1 + c_1) A_2 + ...) A_{K-1} + c_{K-1}, A_k = the largest
// arity at level k (level 0 = the root).  Appended to the RWT2 table: t2[3]
// = its word offset, word 0 = A_1..A_{K-1} (4 bits each), then the u16
// columns.  The odometer then never reads the table to follow a level: it
// keeps the path index, and the leaf parent's column is one LDS read.
// Empty (t2[3] = 0) when the table would exceed kRowsMaxPathEntries.
constexpr uint32_t kRowsMaxPathEntries = 4096;
void append_path_table(std::vector<uint32_t> &t2, uint32_t K) {
    if (!K || t2.size() < 4) return;
    std::vector<uint32_t> A(K, 0);
    std::vector<uint32_t> lev{t2[0]};
    for (uint32_t d = 0; d < K; ++d) {  // A[d] = the largest arity at level d
        std::vector<uint32_t> next;
        for (const uint32_t w : lev) {
            const uint32_t a = (w >> 16) & 0x7Fu, f = w & 0xFFFFu;
            A[d] = std::max(A[d], a);
            if (d + 1 < K)
                for (uint32_t c = 0; c < a; ++c) next.push_back(t2[4 + f + c]);
        }
        lev.swap(next);
    }
    uint64_t entries = 1;
    for (uint32_t d = 0; d < K; ++d) entries *= A[d];
    if (entries > kRowsMaxPathEntries || entries == 0) return;
    std::vector<uint16_t> col(entries, 0);
    std::vector<uint8_t> set(entries, 0);
    // depth-first over the paths
    struct F {
        uint32_t w, idx, d;
    };
    std::vector<F> st{{t2[0], 0, 0}};
    while (!st.empty()) {
        const F fr = st.back();
        st.pop_back();
        const uint32_t a = (fr.w >> 16) & 0x7Fu, f = fr.w & 0xFFFFu;
        for (uint32_t c = 0; c < a; ++c) {
            const uint32_t e = t2[4 + f + c];
            const uint32_t idx = fr.idx * A[fr.d] + c;
            if (fr.d + 1 == K) {  // a leaf parent: its first column
                col[idx] = (uint16_t)(e & 0xFFFFu);
                set[idx] = 1;
            }
            else st.push_back(F{e, idx, fr.d + 1});
        }
    }
    uint32_t packed = 0;
    for (uint32_t d = 1; d < K; ++d) packed |= A[d] << (4 * (d - 1));
    // a LINEAR path table (every leaf parent's first column = its path index
    // << s: the basic partitioner's trees, whose only incomplete nodes are the
    // last of their level -- C2-C4 with s = 3) is flagged in bit 31, s in bits
    // 24..28: the walk then computes the column instead of reading it
    for (uint32_t sh = 0; sh < 16; ++sh) {
        bool lin = true;
        for (uint64_t i = 0; i < entries && lin; ++i) lin = !set[i] || col[i] == (uint32_t)(i << sh);
        if (lin) {
            packed |= 0x80000000u | sh << 24;
            break;
        }
    }
    t2[3] = (uint32_t)t2.size();
    t2.push_back(packed);
    for (size_t i = 0; i < col.size(); i += 2)
        t2.push_back((uint32_t)col[i] | (i + 1 < col.size() ? (uint32_t)col[i + 1] << 16 : 0u));
}

// TERMINAL records (r06, MBRWT_BUILD_ROWS_CODE = 2; rows_record.hpp
// term_walk): every RWT2 entry that is a leaf or a leaf parent is a
// terminal.  TT = [w | ib << 8, nT, 0, 0, nT entry words, the RWT2 column
// lists]; the build table BT = [root entry, the root's terminal id (a
// one-level tree), nE, 0, nE entries, nE terminal ids (internal: ~0)] for
// the build's walk.  False when the fields would not fit 28 bits (more than
// 4,096 terminals or a leaf parent wider than 16).
bool build_term_tables(const std::vector<uint32_t> &t2, std::vector<uint32_t> &tt, std::vector<uint32_t> &bt,
                       std::vector<uint32_t> &term_slot) {
    tt.clear();
    bt.clear();
    term_slot.clear();
    if (t2.size() < 4) return false;
    const uint32_t root = t2[0], nE = t2[1];
    const size_t lists_end = t2[3] ? (size_t)t2[3] : t2.size();
    if (4 + (size_t)nE > lists_end) return false;
    std::vector<uint32_t> ent, tid(nE, ~0u);
    uint32_t mbits = 0;
    auto is_term = [](uint32_t e) { return (e >> 31) != 0u; };
    auto lp_arity = [](uint32_t e) { return (e >> 30) == 3u ? (e >> 16) & 0x7Fu : 0u; };
    if ((root >> 30) == 3u) {  // a one-level tree: the root is the only terminal
        ent.push_back(root);
        term_slot.push_back(nE);
        mbits = lp_arity(root);
    } else {
        for (uint32_t i = 0; i < nE; ++i) {
            const uint32_t e = t2[4 + i];
            if (!is_term(e)) continue;
            tid[i] = (uint32_t)ent.size();
            ent.push_back(e);
            term_slot.push_back(i);
            mbits = std::max(mbits, lp_arity(e));
        }
    }
    const uint32_t nT = (uint32_t)ent.size();
    uint32_t ib = 1;
    while ((1u << ib) < nT) ++ib;
    if (nT == 0 || nT > 4096 || mbits > 16 || ib + mbits > 28) return false;
    const uint32_t w = ib + mbits;
    tt = {w | ib << 8, nT, 0u, 0u};
    tt.insert(tt.end(), ent.begin(), ent.end());
    tt.insert(tt.end(), t2.begin() + 4 + nE, t2.begin() + lists_end);
    bt = {root, 0u, nE, 0u};
    bt.insert(bt.end(), t2.begin() + 4, t2.begin() + 4 + nE);
    bt.insert(bt.end(), tid.begin(), tid.end());
    return tt.size() <= kRowsMaxTableWords;
}

// WT (terminal records' V accounting): every terminal's chain of ancestor
// dnodes from the root down, their arities, the chain's length and the
// terminal's own arity (a leaf parent's; 0 for a leaf).  The parents come
// from the logical tree below the root (as build_rwt_table walks it).
bool build_work_table(const Tree &tree, const std::vector<uint32_t> &term_dnode, std::vector<uint32_t> &wt) {
    const auto &N = tree.nodes;
    const uint32_t root = tree.folded ? 0u : 1u;
    std::vector<uint32_t> parent(N.size(), ~0u), q{root};
    for (size_t h = 0; h < q.size(); ++h) {
        const DevNode &v = N[q[h]];
        if (v.kind == KIND_LEAF) continue;
        for (uint32_t c = 0; c < v.arity; ++c) {
            const uint32_t w = v.first_child + c;
            if (w >= N.size()) return false;
            parent[w] = q[h];
            if (N[w].kind != KIND_LEAF) q.push_back(w);
        }
    }
    const uint32_t nT = (uint32_t)term_dnode.size();
    std::vector<std::vector<uint32_t>> chains(nT);
    uint32_t D = 1;
    for (uint32_t t = 0; t < nT; ++t) {
        const uint32_t u = term_dnode[t];
        if (u >= N.size()) return false;
        for (uint32_t a = u == root ? ~0u : parent[u]; a != ~0u; a = a == root ? ~0u : parent[a]) {
            chains[t].push_back(a);
            if (chains[t].size() > 32) return false;
        }
        std::reverse(chains[t].begin(), chains[t].end());
        D = std::max<uint32_t>(D, (uint32_t)chains[t].size());
    }
    wt.assign(4 + (size_t)nT * (2 * D + 2), 0u);
    wt[0] = D;
    wt[1] = nT;
    for (uint32_t t = 0; t < nT; ++t) {
        const uint32_t u = term_dnode[t];
        for (uint32_t k = 0; k < chains[t].size(); ++k) {
            wt[4 + (size_t)t * D + k] = chains[t][k];
            wt[4 + (size_t)nT * D + (size_t)t * D + k] = N[chains[t][k]].arity;
        }
        wt[4 + (size_t)2 * nT * D + t] = (uint32_t)chains[t].size();
        wt[4 + (size_t)2 * nT * D + nT + t] = N[u].kind == KIND_LEAF ? 0u : N[u].arity;
    }
    return true;
}

namespace {

// the terminals of row r's descent in pre-order, term(id, children mask):
// the row's masks (emit_row_masks) walked over the build table BT
// (build_term_tables).  False when the row has more than kTermMaxMasks masks
// or its masks do not follow the table.
constexpr uint32_t kTermMaxMasks = 256;
template <class Term>
__device__ bool row_terms(const DevNode *nodes, bool folded, uint32_t r, const uint32_t *bt, Term term,
                          uint32_t &labels) {
    uint16_t mb[kTermMaxMasks];
    uint32_t nm = 0;
    labels = emit_row_masks(nodes, folded, r, [&](uint64_t mk, uint32_t, uint32_t) {
        if (nm < kTermMaxMasks) mb[nm] = (uint16_t)mk;
        ++nm;
    });
    if (labels == ~0u || nm > kTermMaxMasks) return false;
    if (!nm) return labels == 0;
    const uint32_t root = gld(bt);
    if ((root >> 30) == 3u) {  // a one-level tree
        term(gld(bt + 1), (uint32_t)mb[0]);
        return nm == 1;
    }
    const uint32_t nE = gld(bt + 2);
    const uint32_t *ent = bt + 4, *tid = bt + 4 + nE;
    uint32_t pos = 1, m = mb[0], f = root & 0xFFFFu;
    uint32_t sf[kRowsMaxHeight], sm[kRowsMaxHeight];
    int sp = 0;
    while (true) {
        if (!m) {
            if (!sp) break;
            --sp;
            f = sf[sp];
            m = sm[sp];
            continue;
        }
        const uint32_t c = (uint32_t)__builtin_ctz(m);
        m &= m - 1u;
        const uint32_t sl = f + c;
        if (sl >= nE) return false;
        const uint32_t e = gld(ent + sl);
        if ((e >> 31) == 0u) {  // an internal node: its mask, one level down
            if (pos >= nm || (m && sp == (int)kRowsMaxHeight)) return false;
            if (m) {
                sf[sp] = f;
                sm[sp] = m;
                ++sp;
            }
            f = e & 0xFFFFu;
            m = mb[pos++];
        } else if ((e >> 30) == 3u) {  // a leaf parent: a terminal with its mask
            if (pos >= nm) return false;
            term(gld(tid + sl), (uint32_t)mb[pos++]);
        } else {  // a leaf: a terminal of its own
            term(gld(tid + sl), 0u);
        }
    }
    return pos == nm;
}
// row r's terminal fields (w bits: id | mask << ib) from byte p on; the
// bytes written, or ~0u
__device__ __forceinline__ uint32_t write_row_terms(const DevNode *nodes, bool folded, uint32_t r, uint8_t *p,
                                                    const uint32_t *bt, uint32_t w, uint32_t ib, uint32_t &labels) {
    uint64_t acc = 0;
    uint32_t nb = 0, wr = 0;
    const bool ok = row_terms(
        nodes, folded, r, bt,
        [&](uint32_t id, uint32_t m) {
            acc |= (uint64_t)(id | (m << ib)) << nb;
            nb += w;
            while (nb >= 8u) {
                p[wr++] = (uint8_t)acc;
                acc >>= 8;
                nb -= 8u;
            }
        },
        labels);
    if (nb) p[wr++] = (uint8_t)acc;
    return ok ? wr : ~0u;
}

// per row of a range: record size (1 + mask bytes, < 2^15) | 0x8000 when the
// row has >= 255 labels (its count does not fit the inline byte)
// (nib: the masks as nibble codes, rows_record.hpp RecMasks)
__global__ __launch_bounds__(256) void k_rows_measure(const DevNode *nodes, uint32_t folded, uint64_t n, uint16_t *sz,
                                                      unsigned long long *acc, uint32_t code, const uint32_t *bt,
                                                      uint32_t w) {
    const bool nib = code == 1u;
    unsigned long long lab = 0, bytes = 0, bad = 0, bytes1 = 0;
    const uint64_t gs = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; r < n; r += gs) {
        uint32_t b = 1, nn = 0, b1 = 1;
        uint32_t L = emit_row_masks(nodes, folded != 0, (uint32_t)r, [&](uint64_t mk, uint32_t a, uint32_t) {
            if (nib) nn += nib_codes((uint32_t)mk);
            else b += rec_mask_bytes(a);
            b1 += rec_mask_bytes(a);
        });
        b += (nn + 1) / 2;
        if (code == 2u && L != ~0u) {  // terminal records: the fields' bytes
            uint32_t nt = 0, L2 = 0;
            b = row_terms(nodes, folded != 0, (uint32_t)r, bt, [&](uint32_t, uint32_t) { ++nt; }, L2) && L2 == L
                    ? 1u + (nt * w + 7u) / 8u
                    : 0x8000u;  // (a row the fields cannot hold: bad)
        }
        bytes1 += b1;
        if (L == ~0u || b >= 0x8000) {
            ++bad;
            sz[r] = 0x7FFF;
            continue;
        }
        sz[r] = (uint16_t)(b | (L >= 255 ? 0x8000u : 0u));
        lab += L;
        bytes += b;
    }
    for (int off = 32; off > 0; off >>= 1) {
        lab += __shfl_down(lab, off);
        bytes += __shfl_down(bytes, off);
        bad += __shfl_down(bad, off);
        bytes1 += __shfl_down(bytes1, off);
    }
    if ((threadIdx.x & 63) == 0) {
        if (lab) atomicAdd(acc + 0, lab);
        if (bytes) atomicAdd(acc + 1, bytes);
        if (bad) atomicAdd(acc + 2, bad);
        if (bytes1) atomicAdd(acc + 3, bytes1);  // (the byte-coded size, beside a nibble measure)
    }
}

// which rows of a block spill: rows with >= 255 labels always; then, while
// the block overflows, the largest inline record (a spilled entry takes 5
// bytes in the block)
__device__ __forceinline__ uint32_t block_spills(const uint32_t *s, uint32_t nrows, uint32_t S, uint32_t B) {
    uint32_t used = S, spilled = 0;
    for (uint32_t t = 0; t < nrows; ++t) {
        if (s[t] & 0x8000u) {
            spilled |= 1u << t;
            used += 5;
        } else {
            used += s[t];
        }
    }
    while (used > B) {
        uint32_t best = 0, bt = 0;
        for (uint32_t t = 0; t < nrows; ++t)
            if (!((spilled >> t) & 1u) && s[t] >= best) {
                best = s[t];
                bt = t;
            }
        spilled |= 1u << bt;
        used = used - best + 5;
    }
    return spilled;
}
__device__ __forceinline__ uint32_t spill_units(uint32_t s) { return (8 + ((s & 0x7FFFu) - 1) + 15) / 16; }

// a candidate (B, S): spilled rows, spill units, rows whose spill entry is
// longer than a block (direct pass)
__global__ __launch_bounds__(256) void k_rows_plan(const uint16_t *sz, uint64_t n, uint32_t B, uint32_t S,
                                                   unsigned long long *acc) {
    unsigned long long sp = 0, units = 0, lng = 0;
    const uint64_t nb = (n + S - 1) / S;
    const uint64_t gs = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t b = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; b < nb; b += gs) {
        uint32_t s[16];
        const uint32_t nr = (uint32_t)std::min<uint64_t>(S, n - b * S);
        for (uint32_t t = 0; t < nr; ++t) s[t] = gld(sz + b * S + t);
        const uint32_t m = block_spills(s, nr, S, B);
        for (uint32_t t = 0; t < nr; ++t)
            if ((m >> t) & 1u) {
                ++sp;
                units += spill_units(s[t]);
                lng += (8 + (s[t] & 0x7FFFu) - 1 > B) ? 1u : 0u;
            }
    }
    for (int off = 32; off > 0; off >>= 1) {
        sp += __shfl_down(sp, off);
        units += __shfl_down(units, off);
        lng += __shfl_down(lng, off);
    }
    if ((threadIdx.x & 63) == 0) {
        if (sp) atomicAdd(acc + 0, sp);
        if (units) atomicAdd(acc + 1, units);
        if (lng) atomicAdd(acc + 2, lng);
    }
}

// the masks of row r written from byte p on (bytes, or nibble codes); the
// bytes written
__device__ __forceinline__ uint32_t write_row_masks(const DevNode *nodes, bool folded, uint32_t r, uint8_t *p,
                                                    uint32_t nib, uint32_t &labels) {
    uint32_t w = 0;
    auto put = [&](uint32_t v) {  // nibble w: byte w / 2, low half first
        if (w & 1u) p[w >> 1] |= (uint8_t)(v << 4);
        else p[w >> 1] = (uint8_t)v;
        ++w;
    };
    labels = emit_row_masks(nodes, folded, r, [&](uint64_t mk, uint32_t a, uint32_t) {
        if (nib) {  // (arity <= 8)
            if (nib_codes((uint32_t)mk) == 1u) {
                put((uint32_t)__builtin_ctzll(mk));
            } else {
                put(8u);
                put((uint32_t)mk & 15u);
                put((uint32_t)(mk >> 4) & 15u);
            }
        } else {  // one byte per 8 children, little-endian
            for (uint32_t k = 0; k < a; k += 8) p[w++] = (uint8_t)(mk >> k);
        }
    });
    return nib ? (w + 1) / 2 : w;
}

// one thread per block of the range: header, inline records, spill entries
__global__ __launch_bounds__(256) void k_rows_write(const DevNode *nodes, uint32_t folded, uint64_t nr_range,
                                                    const uint16_t *sz, uint32_t B, uint32_t S, uint8_t *blocks,
                                                    uint8_t *spill, unsigned long long *spill_used, uint32_t code,
                                                    const uint32_t *bt, uint32_t w, uint32_t ib) {
    const uint32_t nib = code == 1u ? 1u : 0u;
    auto write = [&](uint32_t r, uint8_t *p, uint32_t &L) -> uint32_t {
        return code == 2u ? write_row_terms(nodes, folded != 0, r, p, bt, w, ib, L)
                          : write_row_masks(nodes, folded != 0, r, p, nib, L);
    };
    const uint64_t nb = (nr_range + S - 1) / S;
    const uint64_t gs = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t b = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; b < nb; b += gs) {
        uint32_t s[16];
        const uint32_t nr = (uint32_t)std::min<uint64_t>(S, nr_range - b * S);
        for (uint32_t t = 0; t < nr; ++t) s[t] = gld(sz + b * S + t);
        const uint32_t m = block_spills(s, nr, S, B);
        uint8_t *blk = blocks + b * B;
        uint32_t o = S;
        for (uint32_t t = 0; t < nr; ++t) {
            const uint32_t r = (uint32_t)(b * S + t);
            if ((m >> t) & 1u) {
                const uint64_t idx = atomicAdd(spill_used, (unsigned long long)spill_units(s[t]));
                uint8_t *se = spill + idx * 16;
                uint32_t L = 0;
                const uint32_t nw = write(r, se + 8, L);
                *reinterpret_cast<uint32_t *>(se) = L;
                *reinterpret_cast<uint32_t *>(se + 4) = nw;
                blk[t] = (uint8_t)(o | 0x80u);
                blk[o] = (uint8_t)std::min<uint32_t>(L, 255);
                for (uint32_t k = 0; k < 4; ++k) blk[o + 1 + k] = (uint8_t)(idx >> (8 * k));
                o += 5;
            } else {
                blk[t] = (uint8_t)o;
                uint32_t L = 0;
                const uint32_t nw = write(r, blk + o + 1, L);
                blk[o] = (uint8_t)L;
                o += 1 + nw;
            }
        }
    }
}

int build_grid(uint64_t items) { return (int)std::max<uint64_t>(1, std::min<uint64_t>((items + 255) / 256, 65536)); }

}  // namespace

// ------------------------------------------------------------------------
// build driver
// ------------------------------------------------------------------------
struct RowsBuild {
    Ctx *top = nullptr;
    uint64_t n = 0, align = 1;
    bool decided = false;
    bool auto_layout = false;  // layout AUTO: decline records that cost more than kAutoMaxCost requests per row
    int footprint = 0;         // MBRWT_BUILD_ROWS_FOOTPRINT of the creating thread
    VarScratch vws;            // variable-length records (rows_var.hip)
    double var_bytes_per_row = 0;  // their size per row, measured on the first range
    RowsImage img;
    unsigned long long *d_acc = nullptr;  // [0..3] measure, [4..7] plan
    uint16_t *d_sz = nullptr;
    uint64_t sz_cap = 0;
    hipStream_t s = nullptr;
    uint32_t *d_bt = nullptr;  // terminal records: the build table (build_term_tables)
};

void free_rows(RowsImage &r) {
    for (void *p : r.var_chunks) (void)hipFree(p);
    if (r.var_lines) (void)hipFree(r.var_lines);
    if (r.d_var_units) (void)hipFree(r.d_var_units);
    if (r.d_var_anc) (void)hipFree(r.d_var_anc);
    if (r.d_unit_of) (void)hipFree(r.d_unit_of);
    if (r.blocks) (void)hipFree(r.blocks);
    if (r.spill) (void)hipFree(r.spill);
    if (r.d_spill_used) (void)hipFree(r.d_spill_used);
    if (r.d_table) (void)hipFree(r.d_table);
    if (r.d_table2) (void)hipFree(r.d_table2);
    if (r.d_table3) (void)hipFree(r.d_table3);
    if (r.d_table4) (void)hipFree(r.d_table4);
    if (r.classes) (void)hipFree(r.classes);
    r = RowsImage();
}

RowsBuild *rows_build_begin(Ctx &top, uint64_t num_rows, uint64_t align, bool auto_layout) {
    RowsBuild *rb = new (std::nothrow) RowsBuild();
    if (!rb) return nullptr;
    rb->top = &top;
    rb->auto_layout = auto_layout;
    rb->footprint = g_rows_footprint;
    rb->n = num_rows;
    rb->align = std::max<uint64_t>(1, align);
    rb->s = top.stream;
    if (hipMalloc(&rb->d_acc, 8 * sizeof(unsigned long long)) != hipSuccess ||
        hipMalloc(&rb->img.d_spill_used, sizeof(unsigned long long)) != hipSuccess ||
        hipMemset(rb->img.d_spill_used, 0, sizeof(unsigned long long)) != hipSuccess) {
        rows_build_abort(rb);
        return nullptr;
    }
    return rb;
}

void rows_build_abort(RowsBuild *rb) {
    if (!rb) return;
    if (rb->d_acc) (void)hipFree(rb->d_acc);
    if (rb->d_sz) (void)hipFree(rb->d_sz);
    if (rb->d_bt) (void)hipFree(rb->d_bt);
    var_free_scratch(rb->vws);
    free_rows(rb->img);
    delete rb;
}

static int read_acc(RowsBuild &rb, unsigned long long *h, int k) {
    MBRWT_HIP(hipMemcpyAsync(h, rb.d_acc, k * sizeof(unsigned long long), hipMemcpyDeviceToHost, rb.s));
    MBRWT_HIP(hipStreamSynchronize(rb.s));
    return MBRWT_OK;
}

// grow the spill area to hold `bytes` (entries keep their offsets: copy)
static int ensure_spill(RowsBuild &rb, uint64_t bytes) {
    RowsImage &im = rb.img;
    const uint64_t need = bytes + im.B + 256;
    if (need <= im.spill_cap) return MBRWT_OK;
    const uint64_t cap = std::max<uint64_t>(need, im.spill_cap + im.spill_cap / 4);
    uint8_t *p = nullptr;
    MBRWT_HIP(hipMalloc(&p, cap));
    MBRWT_HIP(hipMemsetAsync(p, 0, cap, rb.s));
    if (im.spill) {
        MBRWT_HIP(hipMemcpyAsync(p, im.spill, im.spill_cap, hipMemcpyDeviceToDevice, rb.s));
        MBRWT_HIP(hipStreamSynchronize(rb.s));
        MBRWT_HIP(hipFree(im.spill));
    }
    im.spill = p;
    im.spill_cap = cap;
    return MBRWT_OK;
}

int rows_build_range(RowsBuild *rbp, Ctx &range, uint64_t row0) {
    if (!rbp) return MBRWT_ERR_NOMEM;
    RowsBuild &rb = *rbp;
    RowsImage &im = rb.img;
    const uint64_t nr = range.tree.num_rows;
    if (!nr) return MBRWT_OK;
    if (!range.d_nodes || range.tree.nodes.empty()) {
        set_error("row records need a node image");
        return MBRWT_ERR_UNSUPPORTED;
    }
    if (row0 % rb.align) {
        set_error("row-record range not aligned");
        return MBRWT_ERR_INVALID;
    }
    if (im.table.empty()) {
        if (!build_rwt_table(range.tree, im.table, im.height, im.max_arity) ||
            !build_rwt2_table(range.tree, im.table2, im.frames, &im.slot_dnode)) {
            im.table.clear();
            set_error("tree shape outside the row-record limits (arity <= 64, columns < 2^16, height <= 16, a walk table of <= 8192 words)");
            return MBRWT_ERR_UNSUPPORTED;
        }
        // one-byte masks everywhere (rows_walk6): the root and every internal
        // or leaf-parent entry of arity <= 8
        auto ar8 = [](uint32_t e) { return (e >> 30) == 2u || ((e >> 16) & 0x7Fu) <= 8; };
        im.mask1 = ar8(im.table2[0]);
        for (size_t i = 4; i < 4 + (size_t)im.table2[1]; ++i) im.mask1 = im.mask1 && ar8(im.table2[i]);
        im.uni = im.mask1 ? rwt2_uniform_levels(im.table2) : 0u;
        if (im.uni) append_path_table(im.table2, im.uni);
        // masks wider than 16 bits (r06: arity up to 64) are read by the tree
        // odometer and the one-lane walks only: such a tree needs the tree
        // odometer's depth
        // (im.max_arity: over the nodes the walk reaches -- record-only
        // dnodes such as PACKT_IN carry other arities)
        if (im.max_arity > 16 && im.frames > kRowsOdoLevels) {
            im.table.clear();
            set_error("row records: a node wider than 16 children in a tree deeper than the tree odometer (8 levels)");
            return MBRWT_ERR_UNSUPPORTED;
        }
        // nibble-coded masks (MBRWT_BUILD_ROWS_CODE = 1, r06): read by the
        // path-table odometer and the one-lane walks, so uniform trees of
        // one-byte masks with a path table only (the others keep bytes)
        im.nib = build_tuning().rows_code == 1 && im.uni && im.table2.size() > 3 && im.table2[3] != 0;
        // terminal records (r06; MBRWT_BUILD_ROWS_CODE 0 = AUTO, the default,
        // or 2): trees of masks up to 16 bits whose terminals fit the fields
        im.term = false;
        // (AUTO, code 0: where they are smaller than byte masks -- decided on
        // the first range below; code 3 forces byte masks)
        const int code = build_tuning().rows_code;
        if ((code == 0 || code == 2) && im.max_arity <= 16) {
            std::vector<uint32_t> bt, term_slot;
            bool ok = build_term_tables(im.table2, im.table3, bt, term_slot);
            if (ok) {
                im.term_dnode.resize(term_slot.size());
                for (size_t i = 0; i < term_slot.size(); ++i)
                    im.term_dnode[i] = term_slot[i] < im.slot_dnode.size() ? im.slot_dnode[term_slot[i]] : ~0u;
                ok = build_work_table(range.tree, im.term_dnode, im.table4);
            }
            if (ok) {
                if (!rb.d_bt) {
                    if (hipMalloc(&rb.d_bt, bt.size() * 4) != hipSuccess) return hip_fail(hipGetLastError(), "build table");
                    MBRWT_HIP(hipMemcpy(rb.d_bt, bt.data(), bt.size() * 4, hipMemcpyHostToDevice));
                }
                im.term = true;
            }
        }
    }
    const uint32_t tw = im.term ? im.table3[0] & 0xFFu : 0u, tib = im.term ? (im.table3[0] >> 8) & 0xFFu : 0u;
    auto code_of = [&]() -> uint32_t { return im.term ? 2u : im.nib ? 1u : 0u; };
    if (nr > rb.sz_cap) {
        if (rb.d_sz) MBRWT_HIP(hipFree(rb.d_sz));
        rb.d_sz = nullptr;
        MBRWT_HIP(hipMalloc(&rb.d_sz, nr * sizeof(uint16_t)));
        rb.sz_cap = nr;
    }
    unsigned long long h[8];
    auto measure = [&]() -> int {
        MBRWT_HIP(hipMemsetAsync(rb.d_acc, 0, 8 * sizeof(unsigned long long), rb.s));
        hipLaunchKernelGGL(k_rows_measure, dim3(build_grid(nr)), dim3(256), 0, rb.s, range.d_nodes,
                           range.tree.folded ? 1u : 0u, nr, rb.d_sz, rb.d_acc, code_of(), (const uint32_t *)rb.d_bt, tw);
        MBRWT_HIP(hipGetLastError());
        return read_acc(rb, h, 4);
    };
    if (int rc = measure()) return rc;
    // nibble codes or terminal records that do not shrink the first range's
    // records (dense rows: most masks hold several bits), or terminal
    // fields a row of the range cannot take, give way to bytes for the
    // whole image
    if (im.term && !rb.decided && (h[2] || h[1] >= h[3])) {
        im.term = false;
        im.table3.clear();
        if (int rc = measure()) return rc;
    }
    if (im.nib && !rb.decided && h[2] == 0 && h[1] >= h[3]) {
        im.nib = false;
        if (int rc = measure()) return rc;
    }
    if (h[2]) {
        set_error("row record deeper than the build walker supports");
        return MBRWT_ERR_UNSUPPORTED;
    }
    if (h[0] != range.tree.num_relations) {
        set_error("row records: label count differs from the node image");
        return MBRWT_ERR_DEVICE;
    }
    if (!im.var) im.record_bytes += h[1];
    auto plan = [&](uint32_t B, uint32_t S, unsigned long long out[3]) -> int {
        MBRWT_HIP(hipMemsetAsync(rb.d_acc, 0, 8 * sizeof(unsigned long long), rb.s));
        hipLaunchKernelGGL(k_rows_plan, dim3(build_grid((nr + S - 1) / S)), dim3(256), 0, rb.s, rb.d_sz, nr, B, S,
                           rb.d_acc);
        MBRWT_HIP(hipGetLastError());
        return read_acc(rb, out, 3);
    };
    if (!rb.decided) {
        // (B, S): the fewest requests per row -- one block read plus one per
        // spilled row, a 128-byte block costing kCost128 of a 64-byte one
        // (measured ceilings), a record longer than a block a
        // direct-pass row (x50) -- among the images that fit the device,
        // then the smallest within 2 % of that
        // a 128-byte block costs more than its request (random 128-byte reads
        // run at 52.6 vs 53.7 G/s, profiles/r03/v01_probe_sweep.json): its
        // LDS slots halve the traversal's resident waves -- the greedy +
        // relax shape at 3.7 B rows took 0.859 ms with 128-byte blocks of 3
        // rows against 0.522 ms with 64-byte blocks of one row
        // (profiles/r04/v09_tree_odometer/)
        constexpr double kCost128 = 1.6;
        size_t free_b = 0, total_b = 0;
        MBRWT_HIP(hipMemGetInfo(&free_b, &total_b));
        const double budget = (double)free_b - 4.0 * (1ull << 30);
        struct Cand {
            uint32_t B, S;
            double t, mem;
        };
        std::vector<Cand> cands;
        const double scale = (double)rb.n / (double)nr;
        for (uint32_t B : {64u, 128u})
            for (uint32_t S = 1; S <= (B == 64 ? 8u : 15u); ++S) {
                if (rb.align % S) continue;
                unsigned long long o[3];
                if (int rc = plan(B, S, o)) return rc;
                const double fs = (double)o[0] / nr, fl = (double)o[2] / nr;
                Cand c{B, S, (B == 128 ? kCost128 : 1.0) * (1.0 + fs + 50.0 * fl),
                       (double)((rb.n + S - 1) / S) * B + (double)o[1] * 16.0 * scale};
                cands.push_back(c);
            }
        double tmin = 1e300;
        for (const Cand &c : cands)
            if (c.mem <= budget) tmin = std::min(tmin, c.t);
        // the variable-length records (rows_var.hip: uniform trees, ranges
        // on directory lines): for rows too long for the blocks -- a block
        // layout costing more than kAutoMaxCost requests per row (most rows
        // spilled, or records longer than a block) or none that fits.
        // The build option MBRWT_BUILD_ROWS_VAR = 1 / 0 forces / forbids them.
        constexpr double kAutoMaxCost = 1.25;
        const int force_var = build_tuning().rows_var;
        bool var_ok = force_var != 0 && rb.align % 13 == 0 && var_prepare(range.tree, im);
        // the lanes per row the decode will run with (the build option, else
        // automatic): the LDS gate below must judge that geometry
        uint32_t var_G = build_tuning().var_lanes;
        if (var_G & (var_G - 1) || var_G > 16) var_G = 0;  // (1, 2, 4, 8 or 16; 0: automatic)
        im.var_G = var_G;
        double var_mem = 1e300;
        if (var_ok && (force_var == 1 || tmin > kAutoMaxCost)) {
            uint64_t vb = 0;
            const int rc = var_measure_range(im, range, rb.vws, &vb, rb.s);
            if (rc && rc != MBRWT_ERR_UNSUPPORTED) return rc;
            var_ok = rc == MBRWT_OK;
            var_mem = (double)vb * scale * 1.02 + (double)((rb.n + 12) / 13) * 64.0 + 64.0 * (1 + rb.n / rb.align);
            rb.var_bytes_per_row = (double)vb / (double)nr;
            // a unit table so large that the decode's LDS cannot hold a mean
            // tile beside it: AUTO keeps the other layouts (forced: allowed,
            // every such tile then takes the decode's global path)
            if (var_ok && force_var != 1 &&
                !var_lds_fits(im, (double)range.tree.num_relations / std::max<double>(1.0, (double)range.tree.num_rows),
                              rb.var_bytes_per_row))
                var_ok = false;
        }
        if (var_ok && var_mem <= budget && (force_var == 1 || tmin > kAutoMaxCost)) {
            im.var = true;
            im.var_G = var_G;
            const uint64_t nlines = (rb.n + 12) / 13;
            MBRWT_HIP(hipMalloc(&im.var_lines, nlines * 64));
            MBRWT_HIP(hipMemsetAsync(im.var_lines, 0, nlines * 64, rb.s));
            rb.decided = true;
        } else {
            if (tmin == 1e300) {
                set_error("row-record image does not fit the device");
                return MBRWT_ERR_NOMEM;
            }
            // layout AUTO keeps the per-node images when the records are long
            // enough that most rows would take a second (spill) request or the
            // direct pass and no variable-length layout applies
            if (rb.auto_layout && tmin > kAutoMaxCost) {
                set_error("row records too long for the block layout");
                return MBRWT_ERR_UNSUPPORTED;
            }
            // The smallest image within `tol` of the fewest modelled requests.
            // The model prices a spilled row as a whole second request, which
            // holds on the odometer's uniform trees (request-bound: C4 with
            // three rows per block, 0.321 against 0.268 ms, profiles/r05), so
            // there FAST keeps within 2 %.  Under the tree odometer (greedy +
            // relax, non-uniform) the reloads overlap the other waves' walks
            // (20 % of the rows spilled: +2 % kernel time, profiles/r04/v15_*),
            // so from r05 such trees take the COMPACT tolerance (30 %) by
            // default: two rows per block, 158.9 GB instead of 236.9 GB at
            // 3.7 B rows.  MBRWT_BUILD_ROWS_FOOTPRINT = COMPACT takes 30 % always.
            const bool compact = rb.footprint == 1 || !im.uni;
            const double tol = compact ? 1.30 : 1.02;
            const Cand *best = nullptr;
            for (const Cand &c : cands)
                if (c.mem <= budget && c.t <= tmin * tol && (!best || c.mem < best->mem)) best = &c;
            im.B = best->B;
            im.S = best->S;
            if (const uint32_t bs = build_tuning().rows_block) {  // MBRWT_BUILD_ROWS_BLOCK: B << 8 | S
                const uint32_t Bv = bs >> 8, Sv = bs & 0xFFu;
                if ((Bv == 64 || Bv == 128) && Sv >= 1 && Sv <= (Bv == 64 ? 8u : 15u) && rb.align % Sv == 0) {
                    im.B = Bv;
                    im.S = Sv;
                }
            }
            // row / S = umulhi(row, floor(2^64 / S) + 1), exact for rows < 2^59 and S <= 16
            im.magic = im.S > 1 ? ((uint64_t)((((unsigned __int128)1) << 64) / im.S) + 1) : 0;
            im.num_blocks = (rb.n + im.S - 1) / im.S;
            MBRWT_HIP(hipMalloc(&im.blocks, im.num_blocks * im.B));
            MBRWT_HIP(hipMemsetAsync(im.blocks, 0, im.num_blocks * im.B, rb.s));
            rb.decided = true;
        }
    }
    if (im.var) return var_build_range(im, range, row0, rb.vws, rb.s);
    unsigned long long o[3];
    if (int rc = plan(im.B, im.S, o)) return rc;
    unsigned long long used = 0;
    MBRWT_HIP(hipMemcpyAsync(&used, im.d_spill_used, sizeof(used), hipMemcpyDeviceToHost, rb.s));
    MBRWT_HIP(hipStreamSynchronize(rb.s));
    // a spilled entry stores its offset as u32 16-byte units: the spill area
    // addresses 64 GiB
    if (used + o[1] >= (1ull << 32)) {
        set_error("row-record spill area beyond 64 GiB");
        return MBRWT_ERR_UNSUPPORTED;
    }
    // the first range sizes the area for the whole image (extrapolated)
    const double scale = row0 == 0 ? (double)rb.n / (double)nr : 1.0;
    if (int rc = ensure_spill(rb, (uint64_t)(used * 16 + o[1] * 16 * scale * (row0 == 0 ? 1.05 : 1.0)) + 16 * o[1]))
        return rc;
    im.spilled_rows += o[0];
    im.long_rows += o[2];
    im.spill_bytes += o[1] * 16;
    hipLaunchKernelGGL(k_rows_write, dim3(build_grid((nr + im.S - 1) / im.S)), dim3(256), 0, rb.s, range.d_nodes,
                       range.tree.folded ? 1u : 0u, nr, rb.d_sz, im.B, im.S, im.blocks + (row0 / im.S) * im.B,
                       im.spill, im.d_spill_used, code_of(), (const uint32_t *)rb.d_bt, tw, tib);
    MBRWT_HIP(hipGetLastError());
    MBRWT_HIP(hipStreamSynchronize(rb.s));
    return MBRWT_OK;
}

// device bytes the records of `rows` more rows will still allocate (the
// variable-length records are allocated per range; blocks up front)
uint64_t rows_build_pending_bytes(const RowsBuild *rb, uint64_t rows) {
    return rb && rb->img.var ? (uint64_t)(rb->var_bytes_per_row * 1.02 * (double)rows) + (64ull << 20) : 0;
}

int rows_build_finish(RowsBuild *rbp) {
    if (!rbp) return MBRWT_ERR_NOMEM;
    RowsBuild &rb = *rbp;
    RowsImage &im = rb.img;
    int rc = MBRWT_OK;
    if (!rb.decided) {  // no rows
        set_error("row records of an empty matrix");
        rc = MBRWT_ERR_UNSUPPORTED;
    }
    if (!rc && (hipMalloc(&im.d_table, im.table.size() * 4) != hipSuccess ||
                hipMemcpy(im.d_table, im.table.data(), im.table.size() * 4, hipMemcpyHostToDevice) != hipSuccess ||
                hipMalloc(&im.d_table2, im.table2.size() * 4) != hipSuccess ||
                hipMemcpy(im.d_table2, im.table2.data(), im.table2.size() * 4, hipMemcpyHostToDevice) != hipSuccess))
        rc = hip_fail(hipGetLastError(), "row-record table upload");
    if (!rc && im.term &&
        (hipMalloc(&im.d_table3, im.table3.size() * 4) != hipSuccess ||
         hipMemcpy(im.d_table3, im.table3.data(), im.table3.size() * 4, hipMemcpyHostToDevice) != hipSuccess ||
         hipMalloc(&im.d_table4, im.table4.size() * 4) != hipSuccess ||
         hipMemcpy(im.d_table4, im.table4.data(), im.table4.size() * 4, hipMemcpyHostToDevice) != hipSuccess))
        rc = hip_fail(hipGetLastError(), "terminal table upload");
    if (rc) {
        rows_build_abort(rbp);
        return rc;
    }
    if (im.var) {
        // (+32 zero entries: the decoder's speculative unit reads past the last word)
        if (hipMalloc(&im.d_var_units, (im.var_units.size() + 32) * 4) != hipSuccess ||
            hipMemset(im.d_var_units, 0, (im.var_units.size() + 32) * 4) != hipSuccess ||
            hipMemcpy(im.d_var_units, im.var_units.data(), im.var_units.size() * 4, hipMemcpyHostToDevice) != hipSuccess ||
            hipMalloc(&im.d_var_anc, std::max<size_t>(1, im.var_anc.size()) * 4) != hipSuccess ||
            hipMemcpy(im.d_var_anc, im.var_anc.data(), im.var_anc.size() * 4, hipMemcpyHostToDevice) != hipSuccess) {
            rc = hip_fail(hipGetLastError(), "variable-length record tables");
            rows_build_abort(rbp);
            return rc;
        }
        im.bytes = (rb.n + 12) / 13 * 64 + im.var_rec_bytes;
    } else {
        if (!im.spill && ensure_spill(rb, 0)) {
            rows_build_abort(rbp);
            return MBRWT_ERR_NOMEM;
        }
        im.bytes = im.num_blocks * im.B + im.spill_bytes;
    }
    if (!im.var) {  // record classes where rows repeat few distinct records (rows_class.hip)
        rc = rows_classes_build(im, rb.n, build_tuning().rows_classes, &im.class_sample_distinct, rb.s);
        if (rc) {
            rows_build_abort(rbp);
            return rc;
        }
    }
    im.occ_cap = build_tuning().rows_wgs_per_cu;  // (MBRWT_BUILD_ROWS_WGS_PER_CU: occupancy sweeps)
    im.ready = true;
    free_rows(rb.top->rows);
    rb.top->rows = im;
    rb.img = RowsImage();  // ownership moved
    if (rb.d_acc) (void)hipFree(rb.d_acc);
    if (rb.d_sz) (void)hipFree(rb.d_sz);
    if (rb.d_bt) (void)hipFree(rb.d_bt);
    var_free_scratch(rb.vws);
    delete rbp;
    return MBRWT_OK;
}


// ------------------------------------------------------------------------
// queries
// ------------------------------------------------------------------------
namespace {

// rwt_walk with its pending frames {first entry, mask} in a per-lane LDS
// stack (stk[128 k], stk[128 k + 64], k < lim <= kRowsMaxHeight: the tree's
// height) instead
// of registers: the compaction kernel walks direct tiles with it, so its
// register budget (and occupancy) stays that of its copy loop
template <class MaskFn, class LeafFn>
__device__ bool rwt_walk_lds(const uint32_t *table, MaskFn mask, LeafFn leaf, AS_LDS uint32_t *stk, uint32_t lim) {
    const uint32_t nI = table[0], nE = table[1];
    const uint32_t *ntab = table + 4;
    const uint32_t *etab = ntab + nI;
    uint32_t nw = ntab[0];
    uint32_t a = nw >> 24;
    uint32_t m = (uint32_t)mask(a);  // (arity <= 16 here: wide trees take rwt_walk)
    uint32_t first = nw & 0xFFFFFFu;
    uint32_t sp = 0;
    bool ok = true;
    while (true) {
        if (!m) {
            if (!sp) break;
            --sp;
            first = stk[128 * sp];
            m = stk[128 * sp + 64];
            continue;
        }
        const uint32_t c = (uint32_t)__builtin_ctz(m);
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
        if (e >= nI || (m && sp == lim)) {
            ok = false;
            break;
        }
        if (m) {  // (the push before the child's mask read: rwt_walk)
            stk[128 * sp] = first;
            stk[128 * sp + 64] = m;
            ++sp;
        }
        nw = ntab[e];
        a = nw >> 24;
        m = (uint32_t)mask(a);
        first = nw & 0xFFFFFFu;
    }
    return ok;
}

// walk families of k_traverse_rows (RowsImage::walk)
enum : uint32_t { WALK_GENERAL = 0, WALK_MASK1 = 1, WALK_ODOMETER = 2, WALK_TREE_ODOMETER = 3 };

struct RowsParams {
    const uint64_t *rows;
    uint64_t n;
    uint64_t num_rows;
    uint64_t blocks, spill, magic;
    uint32_t S;
    uint32_t table_words;
    const uint32_t *table;        // RWT2
    uint32_t C;                   // labels per tile region (multiple of 64)
    uint8_t *temp;                // tiles x (128 + 2 C) bytes: u16 counts[64], u16 labels[C]
    uint32_t *tile_counts;        // [tiles] labels (bit 31: the tile goes to the direct pass)
    unsigned long long *scalars;  // the kernel's counters: [2] error flags (bit 0: row out of range)
    unsigned long long *status;   // the call's {needed, status, sticky}: status is reset here
    uint32_t uni;                 // the odometer: the tree's internal levels K (1..5)
    uint32_t path_walk;           // the odometer over the path table when the tree has one
    uint32_t stk_words;           // per-lane LDS stack slots (general walks)
    uint32_t frames;              // the tree odometer: internal levels on the longest path (1..kRowsOdoLevels)
    uint32_t mask1;               // every mask one byte
    const uint32_t *classes;      // record classes: the packed class index (null: none; rows_class.hip)
    uint32_t class_bits;
};

__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// a u16 store at a 32-bit byte offset from a wave-uniform base (the saddr +
// 32-bit voffset form of global_store_short: no 64-bit address arithmetic)
__device__ __forceinline__ void st16(uint16_t *base, uint32_t idx, uint32_t v) {
    *(AS_GLOBAL uint16_t *)((uintptr_t)base + (uint64_t)(idx * 2u)) = (uint16_t)v;
}

// The general walk (masks of 1 or 2 bytes: arity <= 16): one lock-step
// iteration per reached child, the top frame in two registers, the pending
// frames in a per-lane LDS stack (one write / one read per push / pop), one
// emission loop for leaves and leaf parents, mask bytes read as two bytes
// masked by the arity.
// a terminal entry's label for bit `bit` of its mask: a leaf's column (bit
// 0), a leaf parent's first column + bit, or entry `bit` of its column list
__device__ __forceinline__ uint32_t term_label(uint32_t e, const AS_LDS uint16_t *lst, uint32_t bit) {
    const uint32_t i = (e & 0xFFFFu) + bit;
    return ((e >> 29) & 1u) ? (uint32_t)lst[i] : i;
}

__device__ __forceinline__ void rows_walk4(const AS_LDS uint8_t *pb, uint32_t o, bool live, uint32_t root,
                                           const AS_LDS uint32_t *ent, const AS_LDS uint16_t *lst,
                                           AS_LDS uint32_t *stk, uint16_t *out, uint32_t pos) {
    const uint32_t ra = (root >> 16) & 0x7Fu;
    const uint32_t rm = ((uint32_t)pb[o] | ((uint32_t)pb[o + 1] << 8)) & ((1u << ra) - 1u);
    o += ra > 8 ? 2u : 1u;
    if ((root >> 30) == 3u) {  // a one-level tree: the root is a leaf parent
        if (live)
            for (uint32_t x = rm; x; x &= x - 1) st16(out, pos++, (root & 0xFFFFu) + (uint32_t)__builtin_ctz(x));
        return;
    }
    uint32_t f = root & 0xFFFFu, m = live ? rm : 0u;
    uint32_t sp = 0;
    while (__any(m != 0)) {
        const bool act = m != 0;
        const uint32_t c = (uint32_t)__builtin_ctz(m | 0x10000u);
        m &= m - 1;
        const uint32_t e = ent[act ? f + c : 0u];
        const uint32_t a = act ? (e >> 16) & 0x7Fu : 0u;  // leaf: 0
        const uint32_t mw = ((uint32_t)pb[o] | ((uint32_t)pb[o + 1] << 8)) & ((1u << a) - 1u);
        o += a ? (a > 8 ? 2u : 1u) : 0u;
        const bool inner = act && (e >> 31) == 0u;
        uint32_t x = (act && (e >> 31)) ? (a ? mw : 1u) : 0u;  // a leaf: its column; a leaf parent: its set children
        const uint32_t base = e & 0xFFFFu;
        for (; x; x &= x - 1) st16(out, pos++, term_label(e, lst, (uint32_t)__builtin_ctz(x)));
        if (inner && m) {
            stk[sp * 64] = f | (m << 16);
            ++sp;
        }
        if (inner) {
            f = base;
            m = mw;
        }
        if (act && !m && sp) {
            --sp;
            const uint32_t w = stk[sp * 64];
            f = w & 0xFFFFu;
            m = w >> 16;
        }
    }
}

// The walk when every mask is one byte (arity <= 8 everywhere): rows_walk4's
// steps in about half the vector instructions -- the record cursor is an LDS
// byte address, the stack pointer a per-lane LDS address (slot stride 256
// bytes), finished lanes leave the loop (exec mask) instead of being carried
// by selects, and leaves / leaf parents and internal children take
// exec-masked branches.  Labels are stored one by one into the tile's temp
// region (global u16).
__device__ __forceinline__ void rows_walk6(const AS_LDS uint8_t *pb, uint32_t o, bool live, uint32_t root,
                                           const AS_LDS uint32_t *ent, const AS_LDS uint16_t *lst,
                                           AS_LDS uint32_t *stk, AS_GLOBAL uint16_t *out, uint32_t pos) {
    const AS_LDS uint8_t *rc = pb + o;  // record cursor
    const uint32_t rm = rc[0];
    ++rc;
    if ((root >> 30) == 3u) {  // a one-level tree: the root is a leaf parent
        if (live)
            for (uint32_t x = rm; x; x &= x - 1) out[pos++] = (uint16_t)((root & 0xFFFFu) + (uint32_t)__builtin_ctz(x));
        return;
    }
    if (!live) return;
    uint32_t f = root & 0xFFFFu, m = rm;
    AS_LDS uint32_t *sp = stk;
    uint32_t ob = pos * 2u;  // byte offset of the next label
    while (m != 0u) {
        const uint32_t c = (uint32_t)__builtin_ctz(m);
        m &= m - 1u;
        const uint32_t e = ent[f + c];
        const uint32_t mw = *rc;
        if ((int32_t)e < 0) {  // a leaf (its column) or a leaf parent (its set children)
            const bool lp = (e >> 30) & 1u;
            uint32_t x = lp ? mw : 1u;
            rc += lp ? 1 : 0;
            do {
                *(AS_GLOBAL uint16_t *)((uintptr_t)out + ob) = (uint16_t)term_label(e, lst, (uint32_t)__builtin_ctz(x));
                ob += 2u;
                x &= x - 1u;
            } while (x);
        } else {  // an internal child: push the rest of this frame, descend
            if (m) {
                *sp = f | (m << 16);
                sp += 64;
            }
            f = e & 0xFFFFu;
            m = mw;
            ++rc;
        }
        if (m == 0u && sp != stk) {
            sp -= 64;
            const uint32_t w = *sp;
            f = w & 0xFFFFu;
            m = w >> 16;
        }
    }
}

// The odometer walk (uniform trees: every root-to-leaf path crosses K
// internal levels and then a leaf parent with consecutive columns, one-byte
// masks -- the basic partitioner's trees without singleton groups, i.e.
// C2-C4).  rows_walk6 spends one lock-step iteration per reached node (19.3
// per C4 row, 34 per 64-row tile in lock step); here one iteration reaches
// the NEXT LEAF PARENT of the row in pre-order (7.9 per C4 row, 15 per tile):
// the remaining-children masks r[0..K-1] of the current path form an
// odometer -- level k takes its next child when every level below it is
// exhausted (top-down, so a level refilled in this iteration feeds the level
// under it), reading that child's mask as the record's next byte, which is
// exactly BRWT::get_row's pre-order (BRWT.cpp:43-51); the leaf-parent step
// then reads the leaf mask and stores base + bit for its set bits into the
// wave's LDS label stage.  No stack, no per-lane frame state beyond 2K
// registers.
template <int K>
__device__ __forceinline__ void rows_walk_uni(const AS_LDS uint8_t *pb, uint32_t o, bool live, uint32_t root,
                                              const AS_LDS uint32_t *ent, AS_LDS uint16_t *out, uint32_t pos) {
    const AS_LDS uint8_t *rc = pb + o;  // record cursor
    uint32_t r[K], f[K];
    f[0] = root & 0xFFFFu;
    r[0] = live ? (uint32_t)rc[0] : 0u;
    ++rc;
#pragma unroll
    for (int k = 1; k < K; ++k) r[k] = f[k] = 0u;
    uint32_t ob = pos * 2u;  // byte offset of the next label
    while (true) {
        uint32_t any = 0;
#pragma unroll
        for (int k = 0; k < K; ++k) any |= r[k];
        if (!any) break;
        bool nd[K];  // nd[k]: levels k..K-1 are exhausted
        nd[K - 1] = r[K - 1] == 0u;
#pragma unroll
        for (int k = K - 2; k >= 1; --k) nd[k] = nd[k + 1] && r[k] == 0u;
#pragma unroll
        for (int k = 1; k < K; ++k) {
            if (nd[k]) {
                const uint32_t c = (uint32_t)__builtin_ctz(r[k - 1]);
                r[k - 1] &= r[k - 1] - 1u;
                f[k] = ent[f[k - 1] + c] & 0xFFFFu;
                r[k] = *rc;
                ++rc;
            }
        }
        const uint32_t c = (uint32_t)__builtin_ctz(r[K - 1]);
        r[K - 1] &= r[K - 1] - 1u;
        const uint32_t base = ent[f[K - 1] + c] & 0xFFFFu;  // a leaf parent: its first column
        uint32_t x = *rc;
        ++rc;
        do {
            *(AS_LDS uint16_t *)((uintptr_t)out + ob) = (uint16_t)(base + (uint32_t)__builtin_ctz(x));
            ob += 2u;
            x &= x - 1u;
        } while (x);
    }
}

// The odometer over the PATH TABLE (append_path_table): the same lock-step
// iteration per reached leaf parent as rows_walk_uni, but a level keeps the
// path index of its node instead of its table entry, so refilling a level is
// register arithmetic (no dependent LDS read per level) and the leaf
// parent's first column is ONE LDS read; the level refills are selects (at
// the Kingsford shape nearly every iteration refills the level above the
// leaf parents in some lane, so branches only added exec-mask work), and a
// leaf parent's first label is stored unconditionally (1.01 labels per leaf
// parent at C4), the loop only for the rest.
// a * b + c in one full-rate v_mad_u32_u24 (a, b < 2^24; b wave-uniform):
// the compiler folds __umul24(a, b) + c into the quarter-rate 64-bit
// v_mad_u64_u32, so the instruction is named here
__device__ __forceinline__ uint32_t mad_u24(uint32_t a, uint32_t b, uint32_t c) {
    uint32_t r;
    asm("v_mad_u32_u24 %0, %1, %2, %3" : "=v"(r) : "v"(a), "s"(b), "v"(c));
    return r;
}

// a record's next mask at cursor c (bytes: byte c; nibble codes, r06:
// nibble c, rows_record.hpp RecMasks) and the cursor's advance.  The nibble
// form reads the two bytes the code can span (LDS: a read past the record
// stays inside the wave's slots)
struct MaskAt {
    uint32_t m, adv;
};
template <bool NIB>
__device__ __forceinline__ MaskAt rec_mask_at(const AS_LDS uint8_t *rec, uint32_t c) {
    if constexpr (!NIB) {
        return MaskAt{(uint32_t)rec[c], 1u};
    } else {
        // (two byte reads: one unaligned 4-byte ds_read_b32 instead took the
        // C4 kernel from 0.30 to 0.43 ms, profiles/r06/v04_nibble_codes)
        const uint32_t i = c >> 1;
        const uint32_t w = ((uint32_t)rec[i] | ((uint32_t)rec[i + 1] << 8)) >> ((c & 1u) * 4u);
        const uint32_t v = w & 15u;
        return v < 8u ? MaskAt{1u << v, 1u} : MaskAt{(w >> 4) & 0xFFu, 3u};
    }
}

template <int K, bool LIN, bool NIB>
__device__ __forceinline__ void rows_walk_path(const AS_LDS uint8_t *pb, uint32_t o, bool live,
                                               const AS_LDS uint16_t *ptab, uint32_t A, AS_LDS uint16_t *out,
                                               uint32_t pos) {
    const AS_LDS uint8_t *rec = pb + o;  // the record's masks
    uint32_t rc = 0;                     // cursor (bytes or nibbles)
    uint32_t r[K], idx[K];
    {
        const MaskAt m0 = rec_mask_at<NIB>(rec, 0);
        r[0] = live ? m0.m : 0u;
        rc = m0.adv;
    }
    idx[0] = 0;
#pragma unroll
    for (int k = 1; k < K; ++k) r[k] = idx[k] = 0u;
    uint32_t ob = pos * 2u;  // byte offset of the next label
    while (true) {
        uint32_t any = 0;
#pragma unroll
        for (int k = 0; k < K; ++k) any |= r[k];
        if (!any) break;
        bool nd[K];  // nd[k]: levels k..K-1 are exhausted
        nd[K - 1] = r[K - 1] == 0u;
#pragma unroll
        for (int k = K - 2; k >= 1; --k) nd[k] = nd[k + 1] && r[k] == 0u;
#pragma unroll
        for (int k = 1; k < K; ++k) {
            const uint32_t c = (uint32_t)__builtin_ctz(r[k - 1]);
            const MaskAt bm = rec_mask_at<NIB>(rec, rc);
            const uint32_t b = bm.m;
            // the node at level k is child c of the level-(k-1) node: A_{k-1}
            // (the largest arity at level k-1) scales the parent's index
            const uint32_t Ak = k >= 2 ? (A >> (4 * (k - 2))) & 0xFu : 0u;  // (wave-uniform)
            // (24-bit multiplies: v_mad_u32_u24 issues at full rate, the
            // 32-bit v_mad_u64_u32 the compiler picks otherwise does not)
            const uint32_t ni = k == 1 ? c : mad_u24(idx[k - 1], Ak, c);
            idx[k] = nd[k] ? ni : idx[k];
            r[k - 1] = nd[k] ? (r[k - 1] & (r[k - 1] - 1u)) : r[k - 1];
            r[k] = nd[k] ? b : r[k];
            rc += nd[k] ? bm.adv : 0u;
        }
        const uint32_t c = (uint32_t)__builtin_ctz(r[K - 1]);
        r[K - 1] &= r[K - 1] - 1u;
        const uint32_t AK = K > 1 ? (A >> (4 * (K > 1 ? K - 2 : 0))) & 0xFu : 0u;
        const uint32_t pidx = K > 1 ? mad_u24(idx[K - 1], AK, c) : c;
        // the leaf parent's first column: computed on a linear path table (no
        // LDS round trip per iteration), else read
        const uint32_t base = LIN ? pidx << ((A >> 24) & 0x1Fu) : (uint32_t)ptab[pidx];
        const MaskAt xm = rec_mask_at<NIB>(rec, rc);
        uint32_t x = xm.m;
        rc += xm.adv;
        *(AS_LDS uint16_t *)((uintptr_t)out + ob) = (uint16_t)(base + (uint32_t)__builtin_ctz(x));
        ob += 2u;
        x &= x - 1u;
        while (x) {
            *(AS_LDS uint16_t *)((uintptr_t)out + ob) = (uint16_t)(base + (uint32_t)__builtin_ctz(x));
            ob += 2u;
            x &= x - 1u;
        }
    }
}

// The odometer for ANY tree shape (r04; the greedy + relax trees of the
// reference's production build: leaf parents at different depths, leaf
// parents whose columns are not consecutive -- walked as internal nodes with
// leaf children -- and masks of up to 16 bits).  As in rows_walk_uni one
// lock-step iteration reaches the row's next TERMINAL in pre-order (a leaf
// parent with consecutive columns, or a leaf): the deepest level with a
// remaining child takes it, and while that child is internal the walk
// descends in the same iteration, each level reading its node's mask as the
// record's next byte(s) -- BRWT::get_row's pre-order (BRWT.cpp:43-51), the
// record format unchanged.  Levels are unrolled and predicated: a level no
// lane of the wave needs costs a skipped branch.  State: 2 KM registers.
template <int KM, bool M1, bool WIDE = false>
__device__ __forceinline__ void rows_walk_tree(const AS_LDS uint8_t *pb, uint32_t o, bool live, uint32_t root,
                                               const AS_LDS uint32_t *ent, const AS_LDS uint16_t *lst,
                                               AS_LDS uint16_t *out, uint32_t pos) {
    // masks: one byte (M1), up to two (arity <= 16), or (WIDE, r06) up to
    // eight -- arity <= 64, one byte per 8 children
    using MT = typename std::conditional<WIDE, uint64_t, uint32_t>::type;
    const AS_LDS uint8_t *rc = pb + o;  // record cursor
    // a node's mask of arity a at the cursor; its width in bytes
    auto mask_at = [&](uint32_t a) -> MT {
        MT m = rc[0];
        if constexpr (WIDE) {
            for (uint32_t k = 8; k < a; k += 8) m |= (MT)rc[k >> 3] << k;  // (rare: a loop, not reads in every lane)
            return a >= 64 ? m : (m & (((MT)1 << a) - 1u));
        } else {
            if (!M1 && a > 8) m |= (uint32_t)rc[1] << 8;  // (rare: a branch, not a read in every lane)
            return m & ((1u << a) - 1u);
        }
    };
    auto width = [](uint32_t a) -> uint32_t { return WIDE ? (a + 7u) >> 3 : (M1 || a <= 8) ? 1u : 2u; };
    uint32_t ob = pos * 2u;  // byte offset of the next label
    auto ctz = [](MT x) -> uint32_t { return WIDE ? (uint32_t)__builtin_ctzll((uint64_t)x) : (uint32_t)__builtin_ctz((uint32_t)x); };
    auto emit = [&](uint32_t e, MT x) {
        *(AS_LDS uint16_t *)((uintptr_t)out + ob) = (uint16_t)term_label(e, lst, ctz(x));
        ob += 2u;
        x &= x - 1u;
        while (x) {
            *(AS_LDS uint16_t *)((uintptr_t)out + ob) = (uint16_t)term_label(e, lst, ctz(x));
            ob += 2u;
            x &= x - 1u;
        }
    };
    const uint32_t ra = (root >> 16) & 0x7Fu;
    if ((root >> 30) == 3u) {  // a one-level tree: the root is a leaf parent
        if (live) {
            const MT x = mask_at(ra);
            if (x) emit(root, x);
        }
        return;
    }
    MT r[KM];
    uint32_t f[KM];
    r[0] = live ? mask_at(ra) : (MT)0;
    f[0] = root & 0xFFFFu;
    rc += width(ra);
#pragma unroll
    for (int k = 1; k < KM; ++k) {
        r[k] = 0;
        f[k] = 0u;
    }
    while (true) {
        uint32_t nz = 0;
#pragma unroll
        for (int k = 0; k < KM; ++k) nz |= (r[k] != 0 ? 1u : 0u) << k;
        if (!nz) break;
        const uint32_t ks = 31u - (uint32_t)__builtin_clz(nz);  // the deepest level with a child left
        bool go = true;
        uint32_t term = 0;
#pragma unroll
        for (int k = 0; k < KM; ++k) {
            if (go && (uint32_t)k >= ks) {
                const uint32_t c = ctz(r[k]);
                r[k] &= r[k] - 1u;
                const uint32_t e = ent[f[k] + c];
                if ((int32_t)e >= 0) {  // an internal child: its mask, one level down
                    const uint32_t a = (e >> 16) & 0x7Fu;
                    const MT m = mask_at(a);
                    rc += width(a);
                    if (k + 1 < KM) {
                        r[k + 1] = m;
                        f[k + 1] = e & 0xFFFFu;
                    }
                } else {
                    term = e;
                    go = false;
                }
            }
        }
        // the terminal: a leaf parent (its set children) or a leaf (its column)
        MT x = 1u;
        if ((term >> 30) == 3u) {
            const uint32_t a = (term >> 16) & 0x7Fu;
            x = mask_at(a);
            rc += width(a);
        }
        emit(term, x);
    }
}

// The walk of a TERMINAL record (r06, rows_record.hpp term_walk): no tree
// to walk -- each field names a leaf parent (its children mask beside) or a
// leaf, in pre-order, so a lane reads its fields one after the other (two
// aligned LDS words and a funnel shift per field) until its row's count of
// labels is out.  The TT table is in LDS: hdr = its word 0, ent its entries,
// lst its column lists.
__device__ __forceinline__ void rows_walk_terms(const AS_LDS uint8_t *pb, uint32_t o, bool live, uint32_t cnt,
                                                uint32_t hdr, const AS_LDS uint32_t *ent, const AS_LDS uint16_t *lst,
                                                AS_LDS uint16_t *out, uint32_t pos) {
    const uint32_t w = hdr & 0xFFu, ib = (hdr >> 8) & 0xFFu;
    const uint32_t fmask = (1u << w) - 1u, imask = (1u << ib) - 1u;
    const uint32_t a0 = (uint32_t)(uintptr_t)(pb + o);
    const AS_LDS uint32_t *wp = (const AS_LDS uint32_t *)(uintptr_t)(a0 & ~3u);
    uint32_t bit = 8u * (a0 & 3u);
    uint32_t left = live ? cnt : 0u;
    uint32_t ob = pos * 2u;  // byte offset of the next label
    // (fixed-width fields: the next field's words are read before this
    // field's entry and labels, off the dependency chain)
    uint32_t lo = 0, hi = 0;
    if (left) {
        lo = wp[bit >> 5];
        hi = wp[(bit >> 5) + 1];
    }
    while (left) {
        const uint32_t f = __builtin_amdgcn_alignbit(hi, lo, bit & 31u) & fmask;
        bit += w;
        lo = wp[bit >> 5];
        hi = wp[(bit >> 5) + 1];
        const uint32_t e = ent[f & imask];
        uint32_t x = (e >> 30) == 3u ? (f >> ib) : 1u;  // a leaf parent: its set children; a leaf: itself
        x = x ? x : 1u;  // (a corrupt field: one label, so the loop still ends)
        do {
            *(AS_LDS uint16_t *)((uintptr_t)out + ob) = (uint16_t)term_label(e, lst, (uint32_t)__builtin_ctz(x));
            ob += 2u;
            x &= x - 1u;
            --left;
        } while (x && left);
    }
}

// Tiles per wave (r05).  A persistent grid (every wave a fixed share of the
// tiles) lasts as long as its slowest wave, and its waves are not equally
// fast: the workgroups dispatched last lose issue arbitration by age (per-wave
// phase stamps at C4: the third workgroup of each CU took 27.5k cycles per
// tile against 22.3k for the first, lifetimes 396k..623k cycles around a mean
// of 507k; profiles/r05/v03_balance).  A grid of one tile per wave lets the
// dispatcher refill each CU as its waves finish: 0.263-0.271 ms against
// 0.280-0.284 ms per 8 M rows on the same boxes.  Rejected (same boxes):
// claiming the second half of the tiles from per-XCD atomic counters (0.316:
// the claims' returns sit in the waves' vmcnt queue ahead of their block
// loads), s_setprio for the later workgroups (0.2855), and requesting the
// next tile's blocks before walking this one (register prefetch with the
// spill reloads issued first: 0.2865 persistent, 0.2775 at 4 tiles per wave).
// (The r05 A/B variants of this kernel -- phase stamps, gather-only, no-walk,
// no-store, cache-resident blocks -- were retired in r06; their results are
// in profiles/r05 and DESIGN.md §16.)
constexpr uint32_t kRowsTilesPerWave = 1;

// k_traverse_rows: one wave per tile of 64 query rows (file comment).
// B: block bytes; WPB: waves per workgroup (the RWT2 table is staged once per
// workgroup); WALK: the walk family.  (r06: a one-pass form that wrote the
// CSR itself, its place found by a decoupled look-back, measured 0.44-0.48
// against 0.33 ms per C4 step and was retired: profiles/r06/v01_one_pass.)
// VAR: the record variant -- 0 byte masks, VAR_NIB nibble codes (the path
// odometer), VAR_WIDE masks of up to 64 bits (the tree odometer, r06)
enum : uint32_t { VAR_BYTE = 0, VAR_NIB = 1, VAR_WIDE = 2, VAR_TERM = 3 };
template <int B, int WPB, bool NT, uint32_t WALK, uint32_t VAR = VAR_BYTE>
__global__ __launch_bounds__(64 * WPB) void k_traverse_rows(RowsParams p) {
    constexpr bool NIB = VAR == VAR_NIB;
    extern __shared__ __attribute__((aligned(16))) uint32_t lds_rows[];
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint64_t ntiles = (p.n + 63) / 64;
    const uint64_t tstride = (uint64_t)gridDim.x * WPB;  // (one tile per wave unless the grid is capped)
    uint64_t t = (uint64_t)blockIdx.x * WPB + wv;
    uint64_t row_n = 0;  // the row of this lane in the wave's next tile (its load overlaps the table's)
    if (t < ntiles && t * 64 + lane < p.n) row_n = gld(p.rows + t * 64 + lane);
    for (uint32_t i = threadIdx.x; i < p.table_words; i += blockDim.x) lds_rows[i] = gld(p.table + i);
    if (blockIdx.x == 0 && threadIdx.x == 0) p.status[1] = MBRWT_OK;  // k_compact_tiles raises it
    __syncthreads();
    const uint32_t root = __builtin_amdgcn_readfirstlane(lds_rows[0]);
    const AS_LDS uint32_t *ent = (const AS_LDS uint32_t *)lds_rows + 4;
    // the leaf parents' column lists after the entries
    const AS_LDS uint16_t *lst = (const AS_LDS uint16_t *)(ent + __builtin_amdgcn_readfirstlane(lds_rows[1]));
    // the path table of a uniform tree (append_path_table; 0: none)
    const uint32_t ptw = p.path_walk ? __builtin_amdgcn_readfirstlane(lds_rows[3]) : 0u;
    const uint32_t pA = ptw ? __builtin_amdgcn_readfirstlane(lds_rows[ptw]) : 0u;
    const uint32_t C = p.C;
    // a row's block at a stride of B + 4 bytes: lanes reading their records
    // at similar offsets hit different LDS banks (a B-byte stride puts every
    // other lane in the same bank)
    constexpr uint32_t PB = B + 4;
    AS_LDS uint8_t *wb = (AS_LDS uint8_t *)(lds_rows + ((p.table_words + 3) & ~3u)) +
                         wv * (64u * PB + 256u * p.stk_words + (WALK >= WALK_ODOMETER ? 2u * C : 0u));
    AS_LDS uint8_t *mine = wb + lane * PB;
    AS_LDS uint32_t *stk = (AS_LDS uint32_t *)(wb + 64u * PB) + lane;
    constexpr uint32_t LPB = B / 16, RPI = 64 / LPB;
    const uint32_t S = p.S;
    // a tile's 64 blocks as coalesced quarters: load k brings rows RPI k ..
    // RPI k + RPI - 1, lane L its 16 bytes L % LPB (row addresses by __shfl)
    auto issue_blocks = [&](uint64_t addr, u32x4_t (&qq)[LPB]) {
#pragma unroll
        for (uint32_t k = 0; k < LPB; ++k) {
            const int src = (int)(RPI * k + lane / LPB);
            const uint32_t lo = (uint32_t)__shfl((int)(uint32_t)addr, src, 64);
            const uint32_t hi = (uint32_t)__shfl((int)(uint32_t)(addr >> 32), src, 64);
            qq[k] = gld_at_nt<u32x4_t, NT>((((uint64_t)hi << 32) | lo) + 16u * (lane % LPB));
        }
    };
    auto block_of = [&](uint64_t row, bool ok) -> uint64_t { return ok ? rows_block(row, S, p.magic) : 0; };
    u32x4_t q[LPB];
    for (uint64_t tn; t < ntiles; t = tn) {
        const uint64_t r0 = t * 64;
        const uint32_t nr = (uint32_t)(p.n - r0 < 64 ? p.n - r0 : 64);
        const uint64_t row = row_n;
        tn = t + tstride;
        if (tn < ntiles && tn * 64 + lane < p.n) row_n = gld(p.rows + tn * 64 + lane);
        const bool valid = lane < nr && row < p.num_rows;
        if (lane < nr && !valid) atomicOr(&p.scalars[2], 1ull);
        // record classes: the row's class is its record's row in the
        // dictionary (S = 1); the class index is the random HBM read, the
        // dictionary's blocks mostly cache hits
        const uint64_t rec_row = (p.classes && valid) ? class_field(p.classes, p.class_bits, row) : row;
        const uint64_t b = block_of(rec_row, valid);
        const uint32_t sub = (uint32_t)(rec_row - b * S);
        issue_blocks(p.blocks + b * B, q);
#pragma unroll
        for (uint32_t k = 0; k < LPB; ++k) {
            AS_LDS uint32_t *d = (AS_LDS uint32_t *)(wb + (RPI * k + lane / LPB) * PB + 16u * (lane % LPB));
            d[0] = q[k].x;
            d[1] = q[k].y;
            d[2] = q[k].z;
            d[3] = q[k].w;
        }
        wave_sync();
        uint32_t cnt = 0, o = 0;
        bool spl = false;
        if (valid) {
            const uint32_t e = mine[sub];
            o = e & 0x7Fu;
            spl = (e & 0x80u) != 0;
            cnt = mine[o];
            ++o;
        }
        bool lng = false;
        // spilled rows: the entry (<= B bytes of it) replaces the block in
        // the lane's own slot; masks from byte 8
        const bool any_spl = __any(spl);
        u32x4_t sq[LPB];
        if (any_spl && spl) {
            const uint32_t idx = (uint32_t)mine[o] | ((uint32_t)mine[o + 1] << 8) | ((uint32_t)mine[o + 2] << 16) |
                                 ((uint32_t)mine[o + 3] << 24);
            const uint64_t sa = p.spill + (uint64_t)idx * 16;
            *(AS_LDS uint32_t *)(mine + B) = idx;  // (the slot's pad word: a long record's copy below)
#pragma unroll
            for (uint32_t k = 0; k < LPB; ++k) sq[k] = gld_at<u32x4_t>(sa + 16u * k);
        }
        if (any_spl && spl) {
#pragma unroll
            for (uint32_t k = 0; k < LPB; ++k) {
                AS_LDS uint32_t *d = (AS_LDS uint32_t *)mine + 4 * k;
                d[0] = sq[k].x;
                d[1] = sq[k].y;
                d[2] = sq[k].z;
                d[3] = sq[k].w;
            }
            cnt = sq[0].x;
            lng = 8 + sq[0].y > B;
            o = 8;
        }
        const uint32_t x = wave_incl_sum(cnt);
        const uint32_t total = __builtin_amdgcn_readlane(x, 63);
        const uint32_t pos = x - cnt;
        // a tile whose labels exceed its region is walked by k_compact_tiles
        // from global memory; so is a record longer than a block (its count
        // flagged with bit 15; its labels' places in the tile are kept)
        const bool direct = total > C;
        // the lane's record in LDS: its block slot, or (r05) for a record
        // longer than a block, a copy of its whole spill entry in the free tail
        // of the wave's label stage (the tile's labels take its first 2 total
        // bytes), so the odometers walk it here instead of walking it byte by
        // byte from global memory (the greedy + relax shape: 0.13 % of rows,
        // 8 % of tiles; its compaction took 266 us of a 0.76 ms step,
        // profiles/r05)
        const AS_LDS uint8_t *rec = mine;
        AS_LDS uint16_t *stage = (AS_LDS uint16_t *)(wb + 64u * PB + 256u * p.stk_words);
        if constexpr (WALK == WALK_ODOMETER || WALK == WALK_TREE_ODOMETER) {
            if (!direct && __any(lng)) {
                // each long row's entry (16-byte chunks) below the previous
                // one's from the stage's end; all of them, or none
                // (the entry's mask bytes and index from the lane's slot)
                const uint32_t need = lng ? ((8u + *(const AS_LDS uint32_t *)(mine + 4) + 15u) & ~15u) : 0u;
                const uint32_t incl = wave_incl_sum(need);
                if (2u * total + __builtin_amdgcn_readlane(incl, 63) <= 2u * C) {
                    AS_LDS uint8_t *stg = (AS_LDS uint8_t *)stage + 2u * C - incl;
                    if (lng) {
                        const uint64_t sa = p.spill + (uint64_t)*(const AS_LDS uint32_t *)(mine + B) * 16;
#pragma unroll 1
                        for (uint32_t b = 0; b < need; b += 16u) *(AS_LDS u32x4_t *)(stg + b) = gld_at<u32x4_t>(sa + b);
                        rec = stg;  // masks from byte 8, as in a spilled row's slot
                        lng = false;
                    }
                    wave_sync();
                }
            }
        }
        const bool has_long = __any(lng);
        uint8_t *treg = p.temp + t * (uint64_t)(128 + 2 * C);
        // (non-temporal: the temp region is read once, by k_compact_tiles;
        // the stores then disturb the random block reads less -- C4 kernel
        // 0.262 -> 0.255 ms, step 0.348 -> 0.333 ms; the same hint on the
        // compaction's CSR stores made the two-stream step slower again,
        // 0.344 ms: profiles/r05/v21_temp_stores)
        if (lane < nr)
            __builtin_nontemporal_store((uint16_t)(cnt | (lng ? 0x8000u : 0u)),
                                        (AS_GLOBAL uint16_t *)(uintptr_t)(reinterpret_cast<uint16_t *>(treg) + lane));
        if (!direct) {
            const bool live = valid && cnt > 0 && !lng;
            if constexpr (WALK == WALK_ODOMETER || WALK == WALK_TREE_ODOMETER) {
                // the odometer into the wave's LDS label stage, then the
                // tile's labels as 16-byte vector stores (a few wide stores
                // instead of one scattered 2-byte store per label: the r03
                // SQ/TA counters showed the texture-address unit as the
                // busiest unit)
                if constexpr (WALK == WALK_TREE_ODOMETER && VAR == VAR_TERM) {
                    rows_walk_terms(rec, o, live, cnt, root, ent, lst, stage, pos);
                } else if constexpr (WALK == WALK_TREE_ODOMETER) {
#define MBRWT_TREE_CASE(K)                                                              \
    case K:                                                                             \
        if constexpr (VAR == VAR_WIDE)                                                  \
            rows_walk_tree<K, false, true>(rec, o, live, root, ent, lst, stage, pos);   \
        else if (p.mask1)                                                               \
            rows_walk_tree<K, true>(rec, o, live, root, ent, lst, stage, pos);          \
        else                                                                            \
            rows_walk_tree<K, false>(rec, o, live, root, ent, lst, stage, pos);         \
        break;
                    switch (p.frames) {
                        MBRWT_TREE_CASE(1)
                        MBRWT_TREE_CASE(2)
                        MBRWT_TREE_CASE(3)
                        MBRWT_TREE_CASE(4)
                        MBRWT_TREE_CASE(5)
                        MBRWT_TREE_CASE(6)
                        MBRWT_TREE_CASE(7)
                        default:
                            if constexpr (VAR == VAR_WIDE)
                                rows_walk_tree<8, false, true>(rec, o, live, root, ent, lst, stage, pos);
                            else
                                rows_walk_tree<8, false>(rec, o, live, root, ent, lst, stage, pos);
                            break;
                    }
#undef MBRWT_TREE_CASE
                } else if (ptw) {
                    const AS_LDS uint16_t *ptab = (const AS_LDS uint16_t *)((const AS_LDS uint32_t *)lds_rows + ptw + 1);
                    const bool lin = (pA >> 31) != 0u;
#define MBRWT_PATH_CASE(K)                                                      \
    case K:                                                                     \
        if (lin)                                                                \
            rows_walk_path<K, true, NIB>(rec, o, live, ptab, pA, stage, pos);   \
        else                                                                    \
            rows_walk_path<K, false, NIB>(rec, o, live, ptab, pA, stage, pos);  \
        break;
                    switch (p.uni) {
                        MBRWT_PATH_CASE(1)
                        MBRWT_PATH_CASE(2)
                        MBRWT_PATH_CASE(3)
                        MBRWT_PATH_CASE(4)
                        default:
                        MBRWT_PATH_CASE(5)
                    }
#undef MBRWT_PATH_CASE
                } else {
                    switch (p.uni) {
                        case 1: rows_walk_uni<1>(rec, o, live, root, ent, stage, pos); break;
                        case 2: rows_walk_uni<2>(rec, o, live, root, ent, stage, pos); break;
                        case 3: rows_walk_uni<3>(rec, o, live, root, ent, stage, pos); break;
                        case 4: rows_walk_uni<4>(rec, o, live, root, ent, stage, pos); break;
                        default: rows_walk_uni<5>(rec, o, live, root, ent, stage, pos); break;
                    }
                }
                wave_sync();
                // (r05: rounding the copy up to whole 128-byte lines helped
                // plain stores by 1.5 % and non-temporal ones not at all)
                const uint32_t nbytes = total * 2;
                for (uint32_t q2 = lane * 16; q2 < nbytes; q2 += 1024)
                    __builtin_nontemporal_store(*(const AS_LDS u32x4_t *)((const AS_LDS uint8_t *)stage + q2),
                                                (AS_GLOBAL u32x4_t *)(uintptr_t)(treg + 128 + q2));
            } else if constexpr (WALK == WALK_MASK1) {
                rows_walk6(mine, o, live, root, ent, lst, stk,
                           (AS_GLOBAL uint16_t *)reinterpret_cast<uint16_t *>(treg + 128), pos);
            } else {
                rows_walk4(mine, o, live, root, ent, lst, stk, reinterpret_cast<uint16_t *>(treg + 128), pos);
            }
        }
        if (lane == 0) gst(p.tile_counts + t, total | (direct ? 0x80000000u : 0u) | (has_long ? 0x40000000u : 0u));
        wave_sync();  // the slots are reused
    }
}

// tile regions -> CSR: one wave per TPW consecutive tiles (every load of
// the group -- counts, the tile offsets, the first 512 labels of each tile --
// issued before any store, so a wave pays one memory latency for TPW tiles);
// offsets by a wave scan of each tile's counts, labels u16 -> u32.  A direct
// tile (bit 31 of its count: more labels than its region, or a record longer
// than a block) is walked here, one lane per row, from the records in global
// memory straight into the CSR.  Launched before the host knows the total:
// over the capacity it writes no CSR.  The scan is exclusive over the tiles,
// so the batch total is offset + count of the last tile; workgroup 0
// publishes the call's {total, status, sticky bits} (the traversal reset the
// status word; a failed record walk raises it to MBRWT_ERR_DEVICE) and
// clears the traversal's error flags for the next call.
constexpr uint32_t kCompactTpw = 4;
struct CompactParams {
    const uint8_t *temp;
    uint32_t C;
    const uint32_t *tile_counts;
    const uint64_t *tile_offsets;
    uint64_t *offsets;
    uint32_t *cols;
    uint64_t n, cap;
    unsigned long long *scalars;  // the traversal's counters ([2] error flags)
    unsigned long long *status;   // {total, status, sticky}
    const uint64_t *rows;         // the batch (direct tiles)
    const uint32_t *classes;      // record classes (null: none)
    uint32_t class_bits;
    RowsView v;
    const uint32_t *table;        // RWT (direct tiles)
    uint32_t stk_lim;             // walk stack frames (the tree's height; dynamic LDS)
};
__device__ __forceinline__ void publish_status(unsigned long long *status, uint64_t st) {
    atomicMax(&status[1], (unsigned long long)st);
    atomicOr(&status[2], 1ull << st);
}
template <bool WIDE>
__global__ __launch_bounds__(256) void k_compact_tiles(CompactParams p) {
    extern __shared__ uint32_t cstk[];  // the direct walks' stacks: 4 x 128 x stk_lim words (two per lane and frame)
    const uint64_t n = p.n;
    const uint64_t ntiles = (n + 63) / 64;
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t total = gld(p.tile_offsets + ntiles - 1) + (gld(p.tile_counts + ntiles - 1) & 0x3FFFFFFFu);
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        const uint64_t err = p.scalars[2];
        p.scalars[2] = 0;
        p.status[0] = total;
        publish_status(p.status, (err & 1) ? MBRWT_ERR_RANGE : total > p.cap ? MBRWT_ERR_CAPACITY : MBRWT_OK);
    }
    if (total > p.cap) return;
    const uint64_t t0 = (((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6) * kCompactTpw;
    if (t0 >= ntiles) return;
    const uint32_t C = p.C;
    const uint32_t region = 128 + 2 * C;
    uint32_t tc[kCompactTpw], cnt[kCompactTpw], v[kCompactTpw][8];
    uint64_t base[kCompactTpw];
#pragma unroll
    for (uint32_t k = 0; k < kCompactTpw; ++k) {
        const uint64_t t = t0 + k;
        const bool in = t < ntiles;
        const uint8_t *treg = p.temp + (in ? t : 0) * (uint64_t)region;
        const uint64_t r0 = t * 64;
        tc[k] = in ? gld(p.tile_counts + t) : 0x80000000u;
        base[k] = in ? gld(p.tile_offsets + t) : 0;
        cnt[k] = (in && r0 + lane < n) ? (uint32_t)gld(reinterpret_cast<const uint16_t *>(treg) + lane) : 0u;  // (bit 15: long)
        const uint16_t *lab = reinterpret_cast<const uint16_t *>(treg + 128);
#pragma unroll
        for (uint32_t j = 0; j < 8; ++j) v[k][j] = gld(lab + lane + 64 * j);  // (C >= 1024: inside the region)
    }
#pragma unroll
    for (uint32_t k = 0; k < kCompactTpw; ++k) {
        const uint64_t t = t0 + k;
        if (t >= ntiles) break;
        const uint64_t r0 = t * 64;
        const uint32_t nr = (uint32_t)(n - r0 < 64 ? n - r0 : 64);
        const uint32_t c = cnt[k] & 0x7FFFu;
        const uint32_t x = wave_incl_sum(c);
        const uint64_t rbase = base[k] + (x - c);
        if (lane < nr) gst(p.offsets + r0 + lane, rbase);
        if (t == ntiles - 1 && lane == nr - 1) gst(p.offsets + n, base[k] + x);
        const uint32_t tot = tc[k] & 0x3FFFFFFFu;
        const uint64_t tb = base[k];
        base[k] = rbase;  // (the walks below: each row's own offset)
        if (tc[k] >> 31) continue;  // a direct tile: walked below, once the copies' registers are free
        uint32_t *dst = p.cols + tb;
#pragma unroll
        for (uint32_t j = 0; j < 8; ++j) {
            const uint32_t i = lane + 64 * j;
            if (i < tot) gst(dst + i, v[k][j]);
        }
        const uint16_t *lab = reinterpret_cast<const uint16_t *>(p.temp + t * (uint64_t)region + 128);
        for (uint32_t i0 = 512; i0 < tot; i0 += 512) {
            uint32_t w[8];
#pragma unroll
            for (uint32_t j = 0; j < 8; ++j) {
                const uint32_t i = i0 + lane + 64 * j;
                w[j] = i < tot ? (uint32_t)gld(lab + i) : 0u;
            }
#pragma unroll
            for (uint32_t j = 0; j < 8; ++j) {
                const uint32_t i = i0 + lane + 64 * j;
                if (i < tot) gst(dst + i, w[j]);
            }
        }
    }
    // direct tiles and records longer than a block (rare): one lane per row,
    // the record walked from global memory straight into the CSR at the
    // row's offset (base[k] now) -- over the places the copy above filled
    // for a long record, hence the fence
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
#pragma unroll 1
    for (uint32_t k = 0; k < kCompactTpw; ++k) {
        const uint64_t t = t0 + k;
        if (t >= ntiles || !(tc[k] >> 30)) continue;
        const uint64_t r0 = t * 64;
        const uint32_t nr = (uint32_t)(n - r0 < 64 ? n - r0 : 64);
        const bool walk = (tc[k] >> 31) ? (cnt[k] & 0x7FFFu) != 0 : (cnt[k] >> 15) != 0;
        if (lane < nr && walk) {
            uint64_t row = gld(p.rows + r0 + lane);
            if (p.classes) row = class_field(p.classes, p.class_bits, row);
            uint64_t masks;
            uint32_t count;
            rows_locate(p.v, row, masks, count);  // (count = cnt: rows out of range have none)
            uint32_t *dst = p.cols + base[k];
            uint32_t j = 0;
            auto put = [&](uint32_t col) {
                if (j < count) gst(dst + j, col);
                ++j;
            };
            auto byte = [&](uint32_t o) { return (uint32_t)gld_at<uint8_t>(masks + o); };
            const auto mk = rec_masks(byte, p.v.nib);
            // (masks beyond 16 bits: the frames in registers, not packed in
            // LDS; terminal records: no frames)
            const bool ok = p.v.term ? term_walk(p.table, byte, count, put)
                            : WIDE   ? rwt_walk(p.table, mk, put, [](uint32_t) {})
                                     : rwt_walk_lds(p.table, mk, put,
                                                (AS_LDS uint32_t *)cstk + (threadIdx.x >> 6) * 128 * p.stk_lim + lane,
                                                p.stk_lim);
            if (!ok || j != count) publish_status(p.status, MBRWT_ERR_DEVICE);
        }
    }
}

// point queries: the column among the row's labels (BRWT::get, BRWT.cpp:9-24)
__global__ __launch_bounds__(256) void k_rows_get(RowsView v, const uint32_t *table, const uint64_t *rows,
                                                  const uint64_t *qcols, uint64_t n, uint64_t num_cols, uint8_t *out,
                                                  unsigned long long *scalars) {
    const uint64_t gs = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gs) {
        const uint64_t row = gld(rows + i), col = gld(qcols + i);
        if (row >= v.num_rows || col >= num_cols) {
            atomicOr(&scalars[2], 1ull);
            gst(out + i, (uint8_t)0);
            continue;
        }
        uint64_t masks;
        uint32_t count;
        rows_locate(v, row, masks, count);
        uint32_t hit = 0;
        if (count) (void)record_walk(v, table, masks, count, [&](uint32_t c) { hit |= c == col; }, [](uint32_t) {});
        gst(out + i, (uint8_t)hit);
    }
}

// count_labels (annotate_static.cpp:149-162) and the V / L accounting
// (V = 1 + the arities of the internal nodes the descent
// reaches, i.e. of the record's masks)
template <bool WORK>
__global__ __launch_bounds__(256) void k_rows_count(RowsView v, const uint32_t *table, const uint64_t *rows,
                                                    uint64_t n, unsigned long long *counts,
                                                    unsigned long long *scalars, const uint32_t *wt) {
    const uint64_t gs = (uint64_t)gridDim.x * blockDim.x;
    unsigned long long vis = 0, lab = 0;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gs) {
        const uint64_t row = gld(rows + i);
        if (row >= v.num_rows) {
            atomicOr(&scalars[2], 1ull);
            continue;
        }
        uint64_t masks;
        uint32_t count;
        rows_locate(v, row, masks, count);
        vis += 1;
        if (!count) continue;
        if (WORK && v.term) {  // terminal records: V from the terminals' ancestor chains (WT)
            const uint32_t D = wt[0], nT = wt[1];
            const uint32_t *ids = wt + 4, *ars = ids + (size_t)nT * D, *len = ars + (size_t)nT * D, *own = len + nT;
            uint32_t prev = ~0u;
            (void)term_walk(
                table, [&](uint32_t o) { return (uint32_t)gld_at<uint8_t>(masks + o); }, count,
                [&](uint32_t) { ++lab; },
                [&](uint32_t id) {
                    const uint32_t l = len[id];
                    uint32_t k = 0;
                    if (prev != ~0u) {  // (the chain shared with the previous terminal: counted already)
                        const uint32_t lp = len[prev];
                        while (k < l && k < lp && ids[(size_t)id * D + k] == ids[(size_t)prev * D + k]) ++k;
                    }
                    for (; k < l; ++k) vis += ars[(size_t)id * D + k];
                    vis += own[id];
                    prev = id;
                });
            continue;
        }
        (void)record_walk(
            v, table, masks, count,
            [&](uint32_t c) {
                if constexpr (WORK) ++lab;
                else atomicAdd(counts + c, 1ull);
            },
            [&](uint32_t a) {
                if constexpr (WORK) vis += a;
            });
    }
    if constexpr (WORK) {
        for (int off = 32; off > 0; off >>= 1) {
            vis += __shfl_down(vis, off);
            lab += __shfl_down(lab, off);
        }
        if ((threadIdx.x & 63) == 0) {
            atomicAdd(&scalars[3], vis);
            atomicAdd(&scalars[4], lab);
        }
    }
}

// get_column over row records: every row whose record holds the column,
// ascending (a select over the row ids; BRWT::get_column, BRWT.cpp:55-85)
struct RowHasColumn {
    RowsView v;
    const uint32_t *table;
    uint32_t col;
    __device__ bool operator()(const uint64_t &row) const {
        uint64_t masks;
        uint32_t count;
        rows_locate(v, row, masks, count);
        if (!count) return false;
        bool hit = false;
        (void)record_walk(v, table, masks, count, [&](uint32_t c) { hit |= c == col; }, [](uint32_t) {});
        return hit;
    }
};
struct HasColumnCount {
    RowHasColumn f;
    __device__ uint64_t operator()(const uint64_t &row) const { return f(row) ? 1u : 0u; }
};

// the table the one-lane walks read: RWT, or TT for terminal records
const uint32_t *walk_table(const RowsImage &im) { return im.term ? im.d_table3 : im.d_table; }

RowsView view_of(const Ctx &c) {
    RowsView v;
    v.blocks = (uint64_t)(uintptr_t)c.rows.blocks;
    v.spill = (uint64_t)(uintptr_t)c.rows.spill;
    v.magic = c.rows.magic;
    v.num_rows = c.rows.classes ? c.rows.num_classes : c.tree.num_rows;  // (classes: the dictionary's records)
    v.B = c.rows.B;
    v.S = c.rows.S;
    v.nib = c.rows.nib ? 1u : 0u;
    v.term = c.rows.term ? 1u : 0u;
    return v;
}

using RowsFn = void (*)(RowsParams);
constexpr uint32_t kRowsWpb = 8;
// the tree odometer's wide workgroups: a large walk table (the greedy +
// relax shape's 8.8 KB, staged once per workgroup) leaves room for only two
// 8-wave workgroups per CU (16 waves); two of 11 waves fit (22)
constexpr uint32_t kRowsWpbWide = 11;
template <int B, bool NT>
RowsFn rows_fn_b(uint32_t walk, uint32_t wpb, bool nib, bool wide, bool term) {
    if (term) return k_traverse_rows<B, kRowsWpb, NT, WALK_TREE_ODOMETER, VAR_TERM>;  // (terminal records)
    if (nib) return k_traverse_rows<B, kRowsWpb, NT, WALK_ODOMETER, VAR_NIB>;  // (nibble codes: the path odometer)
    if (wide)  // (masks beyond 16 bits: the tree odometer)
        return wpb == kRowsWpbWide ? k_traverse_rows<B, kRowsWpbWide, NT, WALK_TREE_ODOMETER, VAR_WIDE>
                                   : k_traverse_rows<B, kRowsWpb, NT, WALK_TREE_ODOMETER, VAR_WIDE>;
    if (wpb == kRowsWpbWide) return k_traverse_rows<B, kRowsWpbWide, NT, WALK_TREE_ODOMETER>;
    return walk == WALK_ODOMETER        ? k_traverse_rows<B, kRowsWpb, NT, WALK_ODOMETER>
           : walk == WALK_TREE_ODOMETER ? k_traverse_rows<B, kRowsWpb, NT, WALK_TREE_ODOMETER>
           : walk == WALK_MASK1         ? k_traverse_rows<B, kRowsWpb, NT, WALK_MASK1>
                                        : k_traverse_rows<B, kRowsWpb, NT, WALK_GENERAL>;
}
RowsFn rows_fn(const RowsImage &im, uint32_t walk, uint32_t wpb) {
    const bool nt = im.bytes > (1ull << 30);  // non-temporal block reads for images beyond the caches
    const bool wide = im.max_arity > 16, term = im.term;
    if (im.B == 64)
        return nt ? rows_fn_b<64, true>(walk, wpb, im.nib, wide, term)
                  : rows_fn_b<64, false>(walk, wpb, im.nib, wide, term);
    return nt ? rows_fn_b<128, true>(walk, wpb, im.nib, wide, term)
              : rows_fn_b<128, false>(walk, wpb, im.nib, wide, term);
}
// resident waves per CU with workgroups of w waves: the LDS (160 KiB per CU:
// the table once per workgroup + per_wave bytes per wave) within the 24-wave cap
uint32_t rows_waves_per_cu(size_t table_bytes, size_t per_wave, uint32_t w) {
    const size_t lds = table_bytes + w * per_wave;
    const uint32_t wgs = std::min<uint32_t>((uint32_t)((160u << 10) / std::max<size_t>(1, lds)), 24u / w);
    return wgs * w;
}
// per-lane stack slots of the general walks: the current frame is held in
// registers and only a descent pushes, so at most frames - 1 are pending.
// Exact sizing keeps a workgroup of 8 waves within a quarter of the CU's LDS
// at the Kingsford shape (3 frames: 8 x (4096 + 512) B + the table).
uint32_t rows_stack_words(const RowsImage &im) { return std::max(1u, im.frames ? im.frames - 1 : 1u); }

// labels per tile region: room for the tile's mean + 8 sigma
uint32_t rows_tile_labels(const Ctx &c) {
    const double mean = c.tree.num_rows ? (double)c.tree.num_relations / (double)c.tree.num_rows : 0.0;
    const double need = 64.0 * mean + 8.0 * std::sqrt(64.0 * mean + 1.0) + 64.0;
    uint32_t C = 1024;
    while (C < need && C < 4096) C <<= 1;
    return C;
}

struct MaskTile {
    __host__ __device__ __forceinline__ uint64_t operator()(const uint32_t &x) const { return x & 0x3FFFFFFFu; }
};

}  // namespace

// the walk family of a context's get_rows: the odometer on uniform trees,
// the one-byte-mask walk where every mask is one byte, else the general walk
// (MBRWT_OPT_ROWS_WALK = 6 forces the non-odometer walk: tests)
static uint32_t rows_walk_of(const Ctx &c) {
    const RowsImage &im = c.rows;
    if (im.term) return WALK_TREE_ODOMETER;  // (terminal records: their own walk, in the tree odometer's slot)
    if (im.nib) return WALK_ODOMETER;       // (nibble codes: only the path odometer reads them)
    if (im.max_arity > 16) return WALK_TREE_ODOMETER;  // (masks beyond 16 bits: the tree odometer only)
    if (im.uni && c.rows_walk != 6 && c.rows_walk != 4 && c.rows_walk != 3)
        return WALK_ODOMETER;  // (7: without the path table)
    // (A/B: 6 = rows_walk6 where every mask is one byte, 4 = rows_walk4)
    if (c.rows_walk == 6 && im.mask1) return WALK_MASK1;
    if (c.rows_walk == 4) return WALK_GENERAL;
    if (im.frames >= 1 && im.frames <= kRowsOdoLevels) return WALK_TREE_ODOMETER;
    return im.mask1 ? WALK_MASK1 : WALK_GENERAL;
}

int rows_get_rows(Ctx &c, const uint64_t *d_rows, uint64_t n, uint64_t *d_offsets, uint32_t *d_cols, uint64_t cap,
                  uint64_t *needed, hipStream_t s, uint64_t *d_status) {
    const RowsImage &im = c.rows;
    if (n == 0 && d_status) return MBRWT_ERR_UNSUPPORTED;  // (the caller's generic path handles it)
    if (n == 0) {
        MBRWT_HIP(hipMemsetAsync(d_offsets, 0, sizeof(uint64_t), s));
        MBRWT_HIP(hipStreamSynchronize(s));
        if (needed) *needed = 0;
        return MBRWT_OK;
    }
    if (im.var) return var_get_rows(c, d_rows, n, d_offsets, d_cols, cap, needed, s, d_status);
    if (n > 0x7FFFFFF0ull) {
        set_error("batch larger than 2^31 rows");
        return MBRWT_ERR_UNSUPPORTED;
    }
    int rc;
    const uint32_t C = rows_tile_labels(c);
    const uint64_t nt = (n + 63) / 64;
    const uint64_t region = 128 + 2ull * C;
    const uint32_t walk = rows_walk_of(c);
    const uint32_t stk_lim = std::max(1u, std::min(im.height, kRowsMaxHeight));
    // counts workspace: nt+1 tile counts | (8-byte aligned) nt+1 tile offsets
    const uint64_t to_off = ((nt + 1) * sizeof(uint32_t) + 7) / 8 * 8;
    if ((rc = ensure(c.ws_temp, nt * region))) return rc;
    // [tile counts | tile offsets | the kernel's own counters (4 x u64)]
    const uint64_t sc_off = to_off + (nt + 1) * sizeof(uint64_t);
    const bool fresh = c.ws_counts.bytes < sc_off + 32;
    if ((rc = ensure(c.ws_counts, sc_off + 32))) return rc;
    unsigned long long *d_sc = reinterpret_cast<unsigned long long *>(reinterpret_cast<uint8_t *>(c.ws_counts.buf) + sc_off);
    if (fresh || c.rows_sc_dirty || c.rows_sc_at != sc_off) {  // the counters are cleared by k_compact_tiles
        MBRWT_HIP(hipMemsetAsync(d_sc, 0, 32, s));
        c.rows_sc_dirty = false;
        c.rows_sc_at = sc_off;
    }
    uint32_t *d_tc = reinterpret_cast<uint32_t *>(c.ws_counts.buf);
    uint64_t *d_to = reinterpret_cast<uint64_t *>(reinterpret_cast<uint8_t *>(c.ws_counts.buf) + to_off);
    hipcub::TransformInputIterator<uint64_t, MaskTile, const uint32_t *> it(d_tc, MaskTile());
    size_t scan_bytes = 0;
    MBRWT_HIP(hipcub::DeviceScan::ExclusiveSum(nullptr, scan_bytes, it, d_to, nt, s));
    if ((rc = ensure(c.ws_scan, scan_bytes))) return rc;
    // the call's status block: the caller's (asynchronous) or the context's
    unsigned long long *st_blk =
        reinterpret_cast<unsigned long long *>(d_status ? d_status : c.d_scalars);

    RowsParams p{};
    p.rows = d_rows;
    p.n = n;
    p.num_rows = c.tree.num_rows;  // (record classes: mapped inside the traversal)
    p.classes = im.classes;
    p.class_bits = im.class_bits;
    p.blocks = (uint64_t)(uintptr_t)im.blocks;
    p.spill = (uint64_t)(uintptr_t)im.spill;
    p.magic = im.magic;
    p.S = im.S;
    const std::vector<uint32_t> &tab = im.term ? im.table3 : im.table2;  // (terminal records: the TT table)
    p.table_words = (uint32_t)tab.size();
    p.table = im.term ? im.d_table3 : im.d_table2;
    p.C = C;
    p.temp = reinterpret_cast<uint8_t *>(c.ws_temp.buf);
    p.tile_counts = d_tc;
    p.scalars = d_sc;
    p.status = st_blk;
    p.uni = im.uni;
    p.path_walk = (c.rows_walk == 7 && !im.nib) ? 0u : 1u;  // (7: the r03 odometer, A/B)
    p.stk_words = walk >= WALK_ODOMETER ? 0u : rows_stack_words(im);  // (the odometers keep no stack)
    p.frames = im.frames;
    p.mask1 = im.mask1 ? 1u : 0u;

    const size_t table_bytes = ((tab.size() + 3) & ~size_t(3)) * 4;
    const size_t per_wave = 64ull * (im.B + 4) + 256ull * p.stk_words + (walk >= WALK_ODOMETER ? 2ull * C : 0ull);
    const uint32_t wpb = (walk == WALK_TREE_ODOMETER && !im.term && !im.occ_cap &&
                          rows_waves_per_cu(table_bytes, per_wave, kRowsWpbWide) >
                              rows_waves_per_cu(table_bytes, per_wave, kRowsWpb))
                             ? kRowsWpbWide
                             : kRowsWpb;
    const RowsFn kfn = rows_fn(im, walk, wpb);
    // (terminal records: a field's second word may lie past the last wave's stage)
    const size_t lds = table_bytes + wpb * per_wave + (im.term ? 16 : 0);
    const uint32_t threads = 64 * wpb;
    // at most 24 waves (3 workgroups of 8) per CU: more waves make the walk phase
    // slower than the extra loads in flight gain (C4 0.426 ms at 3 against
    // 0.456 at 4, C2 0.068 against 0.073: profiles/r03/v06_rows_occupancy_*);
    // MBRWT_BUILD_ROWS_WGS_PER_CU (when the image is built) overrides
    const int occ_cap = im.occ_cap ? (int)im.occ_cap : (int)std::max(1u, 24u / wpb);
    if (c.rb_fn != reinterpret_cast<const void *>(kfn) || c.rb_lds != lds || c.rb_threads != threads ||
        c.rb_cap != occ_cap) {
        if (lds > 65536)
            MBRWT_HIP(hipFuncSetAttribute(reinterpret_cast<const void *>(kfn),
                                          hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
        int dev_cus = 0, per_cu = 0;
        (void)hipDeviceGetAttribute(&dev_cus, hipDeviceAttributeMultiprocessorCount, c.device);
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, reinterpret_cast<const void *>(kfn), threads, lds) !=
                hipSuccess ||
            per_cu <= 0)
            per_cu = 1;
        per_cu = std::min(per_cu, occ_cap);
        c.rb_cap = occ_cap;
        c.rb_fn = reinterpret_cast<const void *>(kfn);
        c.rb_lds = lds;
        c.rb_threads = threads;
        c.rb_blocks = std::max(1, dev_cus) * per_cu;
    }

    c.rows_sc_dirty = true;  // until k_compact_tiles has run
    hipEvent_t e0 = c.ev0, e1 = c.ev1;
    if (c.timing && d_status) {  // asynchronous calls: one event pair per call, summed by mbrwt_take_timing
        if (c.async_ev.size() <= c.async_used) {
            hipEvent_t ea = nullptr, eb = nullptr;
            MBRWT_HIP(hipEventCreate(&ea));
            MBRWT_HIP(hipEventCreate(&eb));
            c.async_ev.push_back({ea, eb});
        }
        e0 = c.async_ev[c.async_used].first;
        e1 = c.async_ev[c.async_used].second;
        ++c.async_used;
    }
    if (c.timing) MBRWT_HIP(hipEventRecord(e0, s));
    {
        // the odometer: kRowsTilesPerWave tiles per wave, the dispatcher
        // refilling each CU; the other walks keep the persistent grid (the
        // tree odometer's table -- 8.8 KB at the greedy + relax shape -- is
        // staged once per workgroup: one tile per wave took 0.518 against
        // 0.458 ms there, profiles/r05)
        const bool persistent = walk != WALK_ODOMETER && !im.term;  // (terminal records: a small table)
        const uint64_t per_wg = (uint64_t)wpb * kRowsTilesPerWave;
        const uint64_t g = persistent
                               ? std::max<uint64_t>(1, std::min<uint64_t>((nt + wpb - 1) / wpb, (uint64_t)c.rb_blocks))
                               : std::max<uint64_t>(1, std::min<uint64_t>((nt + per_wg - 1) / per_wg, 1ull << 30));
        hipLaunchKernelGGL(kfn, dim3((unsigned)g), dim3(threads), lds, s, p);
        MBRWT_HIP(hipGetLastError());
    }
    if (c.timing) MBRWT_HIP(hipEventRecord(e1, s));
    MBRWT_HIP(hipcub::DeviceScan::ExclusiveSum(c.ws_scan.buf, scan_bytes, it, d_to, nt, s));
    {
        CompactParams cp{};
        cp.temp = p.temp;
        cp.C = C;
        cp.tile_counts = d_tc;
        cp.tile_offsets = d_to;
        cp.offsets = d_offsets;
        cp.cols = d_cols;
        cp.n = n;
        cp.cap = cap;
        cp.scalars = d_sc;
        cp.status = st_blk;
        cp.rows = d_rows;
        cp.classes = im.classes;
        cp.class_bits = im.class_bits;
        cp.v = view_of(c);
        cp.table = im.term ? im.d_table3 : im.d_table;
        const uint64_t waves = (nt + kCompactTpw - 1) / kCompactTpw;
        cp.stk_lim = stk_lim;
        // (MBRWT_OPT_COMPACT_CUS: on the CU-masked stream, between two events)
        hipStream_t sc = s;
        if (c.compact_cus && c.s_compact) {
            MBRWT_HIP(hipEventRecord(c.ev_trav, s));
            MBRWT_HIP(hipStreamWaitEvent(c.s_compact, c.ev_trav, 0));
            sc = c.s_compact;
        }
        if (im.max_arity > 16)
            hipLaunchKernelGGL(k_compact_tiles<true>, dim3((unsigned)((waves + 3) / 4)), dim3(256), 0, sc, cp);
        else
            hipLaunchKernelGGL(k_compact_tiles<false>, dim3((unsigned)((waves + 3) / 4)), dim3(256),
                               (size_t)256 * cp.stk_lim * 8, sc, cp);
        MBRWT_HIP(hipGetLastError());
        if (sc != s) {
            MBRWT_HIP(hipEventRecord(c.ev_comp, sc));
            MBRWT_HIP(hipStreamWaitEvent(s, c.ev_comp, 0));
        }
        c.rows_sc_dirty = false;
    }
    if (d_status) return MBRWT_OK;  // no host synchronisation: the status lands on the stream
    MBRWT_HIP(hipMemcpyAsync(c.h_scalars, c.d_scalars, 2 * sizeof(uint64_t), hipMemcpyDeviceToHost, s));
    MBRWT_HIP(hipStreamSynchronize(s));
    if (c.timing) {
        float ms = 0;
        MBRWT_HIP(hipEventElapsedTime(&ms, c.ev0, c.ev1));
        c.timing_ms += ms;
        c.timing_launches += 1;
    }
    const uint64_t total = c.h_scalars[0], st = c.h_scalars[1];
    if (needed) *needed = total;
    switch (st) {
        case MBRWT_OK: return MBRWT_OK;
        case MBRWT_ERR_RANGE: set_error("row out of range"); return MBRWT_ERR_RANGE;
        case MBRWT_ERR_CAPACITY: set_error("cols_cap too small"); return MBRWT_ERR_CAPACITY;
        default: set_error("row-record walk failed (corrupt image)"); return MBRWT_ERR_DEVICE;
    }
}

namespace {
__global__ void k_set_status(unsigned long long *status, uint64_t need, uint64_t st) {
    status[0] = need;
    status[1] = st;
    status[2] |= 1ull << st;
}
}  // namespace

int rows_set_status(uint64_t *d_status, uint64_t need, int rc, hipStream_t s) {
    hipLaunchKernelGGL(k_set_status, dim3(1), dim3(1), 0, s, reinterpret_cast<unsigned long long *>(d_status), need,
                       (uint64_t)rc);
    MBRWT_HIP(hipGetLastError());
    return MBRWT_OK;
}

static uint64_t simple_grid(uint64_t n) { return std::max<uint64_t>(1, std::min<uint64_t>((n + 255) / 256, 65536)); }

int rows_get_batch(Ctx &c, const uint64_t *d_rows, const uint64_t *d_cols, uint64_t n, uint8_t *d_out, hipStream_t s) {
    if (n == 0) return MBRWT_OK;
    if (c.rows.var) return var_get_batch(c, d_rows, d_cols, n, d_out, s);
    if (c.rows.classes)
        if (int rc = rows_class_map(c, d_rows, n, &d_rows, s)) return rc;
    MBRWT_HIP(hipMemsetAsync(c.d_scalars, 0, 8 * sizeof(uint64_t), s));
    hipLaunchKernelGGL(k_rows_get, dim3((unsigned)simple_grid(n)), dim3(256), 0, s, view_of(c),
                       (const uint32_t *)walk_table(c.rows), d_rows, d_cols, n, c.tree.num_columns, d_out,
                       reinterpret_cast<unsigned long long *>(c.d_scalars));
    MBRWT_HIP(hipGetLastError());
    MBRWT_HIP(hipMemcpyAsync(c.h_scalars, c.d_scalars, 4 * sizeof(uint64_t), hipMemcpyDeviceToHost, s));
    MBRWT_HIP(hipStreamSynchronize(s));
    return (c.h_scalars[2] & 1) ? MBRWT_ERR_RANGE : MBRWT_OK;
}

int rows_count_labels(Ctx &c, const uint64_t *d_rows, uint64_t n, uint64_t *d_counts, hipStream_t s) {
    if (c.rows.var) return var_count(c, d_rows, n, d_counts, nullptr, nullptr, s);
    if (c.rows.classes)
        if (int rc = rows_class_map(c, d_rows, n, &d_rows, s)) return rc;
    if (c.tree.num_columns) MBRWT_HIP(hipMemsetAsync(d_counts, 0, c.tree.num_columns * sizeof(uint64_t), s));
    MBRWT_HIP(hipMemsetAsync(c.d_scalars, 0, 8 * sizeof(uint64_t), s));
    if (n)
        hipLaunchKernelGGL(k_rows_count<false>, dim3((unsigned)simple_grid(n)), dim3(256), 0, s, view_of(c),
                           (const uint32_t *)walk_table(c.rows), d_rows, n, reinterpret_cast<unsigned long long *>(d_counts),
                           reinterpret_cast<unsigned long long *>(c.d_scalars), (const uint32_t *)c.rows.d_table4);
    MBRWT_HIP(hipGetLastError());
    MBRWT_HIP(hipMemcpyAsync(c.h_scalars, c.d_scalars, 4 * sizeof(uint64_t), hipMemcpyDeviceToHost, s));
    MBRWT_HIP(hipStreamSynchronize(s));
    return (c.h_scalars[2] & 1) ? MBRWT_ERR_RANGE : MBRWT_OK;
}

int rows_count_work(Ctx &c, const uint64_t *d_rows, uint64_t n, uint64_t *visits, uint64_t *labels, hipStream_t s) {
    if (c.rows.var) return var_count(c, d_rows, n, nullptr, visits, labels, s);

    if (c.rows.classes)
        if (int rc = rows_class_map(c, d_rows, n, &d_rows, s)) return rc;
    MBRWT_HIP(hipMemsetAsync(c.d_scalars, 0, 8 * sizeof(uint64_t), s));
    if (n)
        hipLaunchKernelGGL(k_rows_count<true>, dim3((unsigned)simple_grid(n)), dim3(256), 0, s, view_of(c),
                           (const uint32_t *)walk_table(c.rows), d_rows, n, nullptr,
                           reinterpret_cast<unsigned long long *>(c.d_scalars), (const uint32_t *)c.rows.d_table4);
    MBRWT_HIP(hipGetLastError());
    MBRWT_HIP(hipMemcpyAsync(c.h_scalars, c.d_scalars, 8 * sizeof(uint64_t), hipMemcpyDeviceToHost, s));
    MBRWT_HIP(hipStreamSynchronize(s));
    if (c.h_scalars[2] & 1) return MBRWT_ERR_RANGE;
    if (visits) *visits = c.h_scalars[3];
    if (labels) *labels = c.h_scalars[4];
    return MBRWT_OK;
}

int rows_get_column(Ctx &c, uint64_t column, uint64_t *d_rows, uint64_t rows_cap, uint64_t *rows_needed,
                    hipStream_t s) {
    if (c.rows.var) return var_get_column(c, column, d_rows, rows_cap, rows_needed, s);
    if (column >= c.tree.num_columns) {
        set_error("column out of range");
        return MBRWT_ERR_RANGE;
    }
    if (c.rows.classes) return rows_class_get_column(c, column, d_rows, rows_cap, rows_needed, s);
    const uint64_t n = c.tree.num_rows;
    const RowHasColumn f{view_of(c), walk_table(c.rows), (uint32_t)column};
    hipcub::CountingInputIterator<uint64_t> rows_it(0);
    // the column's size first (a reduce over the rows), then the rows
    hipcub::TransformInputIterator<uint64_t, HasColumnCount, hipcub::CountingInputIterator<uint64_t>> cnt_it(
        rows_it, HasColumnCount{f});
    int rc;
    size_t red_bytes = 0, sel_bytes = 0;
    uint64_t *d_num = reinterpret_cast<uint64_t *>(c.d_scalars);
    MBRWT_HIP(hipcub::DeviceReduce::Sum(nullptr, red_bytes, cnt_it, d_num, n, s));
    if ((rc = ensure(c.ws_scan, std::max<size_t>(red_bytes, 256)))) return rc;
    MBRWT_HIP(hipcub::DeviceReduce::Sum(c.ws_scan.buf, red_bytes, cnt_it, d_num, n, s));
    MBRWT_HIP(hipMemcpyAsync(c.h_scalars, c.d_scalars, sizeof(uint64_t), hipMemcpyDeviceToHost, s));
    MBRWT_HIP(hipStreamSynchronize(s));
    const uint64_t need = c.h_scalars[0];
    if (rows_needed) *rows_needed = need;
    if (!d_rows || need > rows_cap) {
        if (need > rows_cap) {
            set_error("rows_cap too small");
            return MBRWT_ERR_CAPACITY;
        }
        return MBRWT_OK;
    }
    if (!need) return MBRWT_OK;
    MBRWT_HIP(hipcub::DeviceSelect::If(nullptr, sel_bytes, rows_it, d_rows, d_num, n, f, s));
    if ((rc = ensure(c.ws_scan, sel_bytes))) return rc;
    MBRWT_HIP(hipcub::DeviceSelect::If(c.ws_scan.buf, sel_bytes, rows_it, d_rows, d_num, n, f, s));
    MBRWT_HIP(hipStreamSynchronize(s));
    return MBRWT_OK;
}

}  // namespace mbrwt
