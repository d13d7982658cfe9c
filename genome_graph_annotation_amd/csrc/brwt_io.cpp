// brwt_io.cpp -- the reference's BRWT stream format and the way back from a
// device image to a tree description (include/mbrwt.h "Files").
//
//   mbrwt_tree_parse      BRWT::load (BRWT.cpp:87-111): pre-order nodes of
//                         {RangePartition (utils.cpp:702-725), rrr_vector<63>
//                         index (bit_vector.cpp:906-925), child count,
//                         children}; leaf columns by composing
//                         RangePartition::get (utils.cpp:689-691) up the path
//   mbrwt_tree_serialize  BRWT::serialize (BRWT.cpp:113-128) of a tree
//                         description, partitions in the bottom-up builder's
//                         convention (BRWT_builders.cpp:68-107): the root's
//                         groups list global columns, every other node's
//                         groups are consecutive ranges
//   mbrwt_tree_export     every index column read back from the device image
//                         (PLANE / MASK / PACK / PACK2 / folded root decoders,
//                         the inverses of image.cpp and synth.hip)
// Byte formats: sdsl_format.hpp (sdsl / libmaus2; parity unpinned).
#include <algorithm>
#include <cstring>
#include <memory>
#include <new>
#include <thread>
#include <vector>

#include "mbrwt_internal.hpp"
#include "sdsl_format.hpp"

struct mbrwt_tree {
    uint64_t num_rows = 0, num_columns = 0;
    std::vector<uint32_t> num_children, first_child, leaf_column;
    std::vector<uint64_t> vec_size;
    std::vector<std::vector<uint64_t>> words;
    std::vector<const uint64_t *> word_ptrs;
    mbrwt_tree_desc desc{};

    void finish() {
        const uint32_t N = (uint32_t)num_children.size();
        word_ptrs.assign(N, nullptr);
        for (uint32_t u = 0; u < N; ++u) word_ptrs[u] = words[u].data();
        desc.num_rows = num_rows;
        desc.num_columns = num_columns;
        desc.num_nodes = N;
        desc.num_children = num_children.data();
        desc.first_child = first_child.data();
        desc.leaf_column = leaf_column.data();
        desc.vec_size = vec_size.data();
        desc.vec_words = word_ptrs.data();
    }
};

namespace mbrwt {
namespace {

using fmt::FormatError;

// ---- parse (BRWT::load) ---------------------------------------------------
struct PNode {
    std::vector<std::vector<uint32_t>> partition;
    std::vector<uint64_t> bits;
    uint64_t size = 0;
    std::vector<std::unique_ptr<PNode>> children;
};

std::unique_ptr<PNode> parse_node(fmt::Reader &r, uint32_t depth) {
    if (depth > 4096) throw FormatError("BRWT deeper than 4096 levels");
    auto nd = std::make_unique<PNode>();
    // RangePartition::load (utils.cpp:702-715): #groups, each an int_vector<> (width 32)
    const uint64_t ng = fmt::get_number(r);
    if (ng > r.n - r.pos) throw FormatError("RangePartition: group count larger than the stream");
    uint64_t total = 0;
    nd->partition.resize(ng);
    for (auto &g : nd->partition) {
        const fmt::IntVector v = fmt::get_int_vector(r);
        if (v.len == 0) throw FormatError("RangePartition: empty group");
        g.resize(v.len);
        for (uint64_t i = 0; i < v.len; ++i) {
            const uint64_t x = v.get(i);
            if (x > UINT32_MAX) throw FormatError("RangePartition: value > 2^32");
            g[i] = (uint32_t)x;
        }
        total += v.len;
    }
    // initialize_groups_and_ranks (utils.cpp:651-677): a permutation of [0, total)
    std::vector<uint8_t> seen(total, 0);
    for (const auto &g : nd->partition)
        for (uint32_t x : g) {
            if (x >= total || seen[x]) throw FormatError("RangePartition: not a partition of [0, n)");
            seen[x] = 1;
        }
    nd->bits = fmt::get_rrr(r, &nd->size);
    const uint64_t nc = fmt::get_number(r);
    if (nc && nc != ng) throw FormatError("BRWT: child count != group count");  // BRWT.cpp:107-108
    for (uint64_t i = 0; i < nc; ++i) nd->children.push_back(parse_node(r, depth + 1));
    return nd;
}

// pre-order tree -> BFS description; leaf columns composed up the path
void to_tree(const PNode &root, mbrwt_tree &t) {
    const uint64_t root_cols = [&] {
        uint64_t s = 0;
        for (const auto &g : root.partition) s += g.size();
        return s;
    }();
    if (root.children.empty() && root_cols == 0) {  // BRWT(): no columns
        if (root.size != 0) throw FormatError("BRWT without columns but with rows");
        t.num_rows = t.num_columns = 0;
        return;
    }
    t.num_rows = root.size;
    t.num_columns = root_cols;
    std::vector<const PNode *> bfs{&root};
    std::vector<uint32_t> parent{UINT32_MAX}, cidx{0};
    for (size_t h = 0; h < bfs.size(); ++h) {
        const PNode *n = bfs[h];
        t.num_children.push_back((uint32_t)n->children.size());
        t.first_child.push_back(n->children.empty() ? 0u : (uint32_t)bfs.size());
        for (size_t i = 0; i < n->children.size(); ++i) {
            bfs.push_back(n->children[i].get());
            parent.push_back((uint32_t)h);
            cidx.push_back((uint32_t)i);
        }
    }
    const size_t N = bfs.size();
    t.leaf_column.assign(N, UINT32_MAX);
    t.vec_size.resize(N);
    t.words.resize(N);
    for (size_t u = 0; u < N; ++u) {
        t.vec_size[u] = bfs[u]->size;
        t.words[u] = bfs[u]->bits;
        if (!bfs[u]->children.empty()) continue;
        // a leaf covers one column (BRWT.cpp:35); its local column 0 mapped up
        uint64_t col = 0;
        for (uint32_t v = (uint32_t)u; parent[v] != UINT32_MAX; v = parent[v]) {
            const auto &g = bfs[parent[v]]->partition.at(cidx[v]);
            if (col >= g.size()) throw FormatError("leaf column outside its parent's group");
            col = g[col];
        }
        t.leaf_column[u] = (uint32_t)col;
    }
}

// ---- serialize (BRWT::serialize) ------------------------------------------
void serialize_desc(const mbrwt_tree_desc &d, fmt::Writer &w) {
    const uint32_t N = d.num_nodes;
    if (N == 0) {  // BRWT(): empty partition, empty index, no children
        fmt::put_number(w, 0);
        fmt::put_rrr(w, {}, 0);
        fmt::put_number(w, 0);
        return;
    }
    // leaves below each node in pre-order (global columns)
    std::vector<std::vector<uint32_t>> leaves(N);
    for (uint32_t u = N; u-- > 0;) {
        if (d.num_children[u] == 0) {
            leaves[u] = {d.leaf_column[u]};
            continue;
        }
        for (uint32_t c = 0; c < d.num_children[u]; ++c) {
            const auto &l = leaves[d.first_child[u] + c];
            leaves[u].insert(leaves[u].end(), l.begin(), l.end());
        }
    }
    std::vector<uint32_t> st{0};
    while (!st.empty()) {
        const uint32_t u = st.back();
        st.pop_back();
        const uint32_t a = d.num_children[u];
        // RangePartition::serialize (utils.cpp:717-725)
        if (a == 0) {
            fmt::put_number(w, 1);
            fmt::IntVector g(1, 32);
            g.set(0, 0);
            fmt::put_int_vector(w, g);
        } else {
            fmt::put_number(w, a);
            uint32_t start = 0;
            for (uint32_t c = 0; c < a; ++c) {
                const auto &l = leaves[d.first_child[u] + c];
                fmt::IntVector g(l.size(), 32);
                for (size_t i = 0; i < l.size(); ++i) g.set(i, u == 0 ? l[i] : start + (uint32_t)i);
                start += (uint32_t)l.size();
                fmt::put_int_vector(w, g);
            }
        }
        std::vector<uint64_t> bits(d.vec_words[u], d.vec_words[u] + (d.vec_size[u] + 63) / 64);
        if (d.vec_size[u] & 63) bits.back() &= (1ull << (d.vec_size[u] & 63)) - 1;
        fmt::put_rrr(w, bits, d.vec_size[u]);
        fmt::put_number(w, a);
        for (uint32_t c = a; c-- > 0;) st.push_back(d.first_child[u] + c);
    }
}

// ---- export: device image -> index columns --------------------------------
struct Bits {
    std::vector<uint64_t> w;
    uint64_t n = 0;
    explicit Bits(uint64_t len = 0) : w((len + 63) / 64, 0), n(len) {}
    void set(uint64_t i) { w[i >> 6] |= 1ull << (i & 63); }
    bool get(uint64_t i) const { return (w[i >> 6] >> (i & 63)) & 1; }
    uint64_t ones() const {
        uint64_t s = 0;
        for (uint64_t x : w) s += (uint64_t)__builtin_popcountll(x);
        return s;
    }
};

int copy_down(uint64_t addr, uint64_t bytes, std::vector<uint8_t> &out) {
    out.resize(bytes);
    if (bytes) MBRWT_HIP(hipMemcpy(out.data(), reinterpret_cast<const void *>(addr), bytes, hipMemcpyDeviceToHost));
    return MBRWT_OK;
}

// children columns of an image of kind PLANE or MASK* over L positions
int decode_plain(const DevNode &dn, std::vector<Bits> &ch) {
    const uint32_t a = dn.arity;
    const uint64_t L = dn.length;
    ch.assign(a, Bits(L));
    std::vector<uint8_t> img;
    int rc;
    if (dn.kind == KIND_PLANE) {
        if ((rc = copy_down(dn.base, (L + 31) / 32 * dn.stride, img))) return rc;
        for (uint64_t b = 0; b < (L + 31) / 32; ++b)
            for (uint32_t c = 0; c < a; ++c) {
                uint32_t bits;
                std::memcpy(&bits, &img[b * dn.stride + 8ull * c + 4], 4);
                for (; bits; bits &= bits - 1) {
                    const uint64_t j = b * 32 + (uint64_t)__builtin_ctz(bits);
                    if (j < L) ch[c].set(j);
                }
            }
        return MBRWT_OK;
    }
    const uint32_t wb = mask_bytes(dn.kind);
    if ((rc = copy_down(dn.base, L * wb, img))) return rc;
    for (uint64_t j = 0; j < L; ++j) {
        uint64_t m = 0;
        std::memcpy(&m, &img[j * wb], wb);
        for (; m; m &= m - 1) ch[(uint32_t)__builtin_ctzll(m)].set(j);
    }
    return MBRWT_OK;
}

// KIND_PACK node u: its MASK8 children's columns (length L) and their leaf
// children's columns (length = each child's popcount)
int decode_pack(const Tree &t, uint32_t v, std::vector<Bits> &cols) {
    const DevNode &dn = t.nodes[v];
    const uint32_t a = dn.arity;
    const uint64_t L = dn.length, blocks = (L + kPackSpan - 1) / kPackSpan;
    std::vector<uint8_t> img;
    int rc;
    if ((rc = copy_down(dn.base, blocks * kPackBlock, img))) return rc;
    std::vector<Bits> B(a, Bits(L));
    std::vector<std::vector<uint8_t>> masks(a);
    std::vector<uint8_t> spill;
    for (uint64_t b = 0; b < blocks; ++b) {
        const uint8_t *blk = &img[b * kPackBlock];
        uint32_t pairs = 0;
        uint16_t bits[8] = {0};
        for (uint32_t c = 0; c < a; ++c) {
            std::memcpy(&bits[c], blk + 16 * (c / 2) + 2 * (c % 2), 2);
            pairs += (uint32_t)__builtin_popcount(bits[c]);
        }
        const uint8_t *area = nullptr;
        if (pairs > kPackArea) {
            uint64_t addr = 0;
            for (uint32_t k = 0; k < 8; ++k) addr |= (uint64_t)blk[pack_area_byte(k)] << (8 * k);
            if ((rc = copy_down(addr, pairs, spill))) return rc;
            area = spill.data();
        }
        uint32_t o = 0;
        for (uint32_t c = 0; c < a; ++c)
            for (uint32_t x = bits[c]; x; x &= x - 1) {
                const uint64_t j = b * kPackSpan + (uint64_t)__builtin_ctz(x);
                B[c].set(j);
                masks[c].push_back(area ? area[o] : blk[pack_area_byte(o)]);
                ++o;
            }
    }
    for (uint32_t c = 0; c < a; ++c) {
        const DevNode &bn = t.nodes[dn.first_child + c];
        std::vector<Bits> leaves(bn.arity, Bits(masks[c].size()));
        for (uint64_t k = 0; k < masks[c].size(); ++k)
            for (uint32_t m = masks[c][k]; m; m &= m - 1) leaves[(uint32_t)__builtin_ctz(m)].set(k);
        cols[dn.first_child + c] = std::move(B[c]);
        for (uint32_t e = 0; e < bn.arity; ++e) cols[bn.first_child + e] = std::move(leaves[e]);
    }
    return MBRWT_OK;
}

// KIND_PACK2 node: the columns of its children A, grandchildren B and the
// leaves below, from the records (mbrwt_internal.hpp)
int decode_pack2(const Tree &t, uint32_t v, std::vector<Bits> &cols) {
    const DevNode &dn = t.nodes[v];
    const uint32_t a = dn.arity, S = dn.stride;
    const uint64_t L = dn.length, blocks = (L + S - 1) / S;
    std::vector<uint8_t> img, spill;
    int rc;
    if ((rc = copy_down(dn.base, blocks * kPack2Block, img))) return rc;
    std::vector<Bits> A(a, Bits(L));
    std::vector<std::vector<uint8_t>> m1(a);                    // A's children bits per A position
    std::vector<std::vector<std::vector<uint8_t>>> lm(a);       // leaf masks per (A, B) per B position
    for (uint32_t h = 0; h < a; ++h) lm[h].resize(t.nodes[dn.first_child + h].arity);
    for (uint64_t b = 0; b < blocks; ++b) {
        const uint8_t *blk = &img[b * kPack2Block];
        const uint8_t *rec = blk;
        std::vector<uint32_t> start(S + 1);
        const uint32_t npos = (uint32_t)std::min<uint64_t>(S, L - b * S);
        if (blk[0] == 0) {  // spilled: u16 start[S+1], then the records
            uint64_t addr = 0;
            std::memcpy(&addr, blk + 8, 8);
            std::vector<uint8_t> hdr;
            if ((rc = copy_down(addr, 2ull * (S + 1), hdr))) return rc;
            for (uint32_t k = 0; k <= S; ++k) start[k] = hdr[2 * k] | ((uint32_t)hdr[2 * k + 1] << 8);
            if ((rc = copy_down(addr, start[S], spill))) return rc;
            rec = spill.data();
        } else {
            for (uint32_t k = 0; k < S; ++k) start[k] = blk[k];
        }
        for (uint32_t k = 0; k < npos; ++k) {
            uint32_t o = start[k];
            const uint32_t m2 = rec[o++];
            uint32_t m1v[8] = {0};
            for (uint32_t x = m2; x; x &= x - 1) {
                const uint32_t h = (uint32_t)__builtin_ctz(x);
                A[h].set(b * S + k);
                m1v[h] = rec[o++];
                m1[h].push_back((uint8_t)m1v[h]);
            }
            for (uint32_t x = m2; x; x &= x - 1) {
                const uint32_t h = (uint32_t)__builtin_ctz(x);
                for (uint32_t y = m1v[h]; y; y &= y - 1) lm[h][(uint32_t)__builtin_ctz(y)].push_back(rec[o++]);
            }
        }
    }
    for (uint32_t h = 0; h < a; ++h) {
        const uint32_t an = dn.first_child + h;
        const DevNode &ad = t.nodes[an];
        std::vector<Bits> Bc(ad.arity, Bits(m1[h].size()));
        for (uint64_t k = 0; k < m1[h].size(); ++k)
            for (uint32_t y = m1[h][k]; y; y &= y - 1) Bc[(uint32_t)__builtin_ctz(y)].set(k);
        for (uint32_t e = 0; e < ad.arity; ++e) {
            const uint32_t bn = ad.first_child + e;
            const DevNode &bd = t.nodes[bn];
            std::vector<Bits> leaves(bd.arity, Bits(lm[h][e].size()));
            for (uint64_t k = 0; k < lm[h][e].size(); ++k)
                for (uint32_t m = lm[h][e][k]; m; m &= m - 1) leaves[(uint32_t)__builtin_ctz(m)].set(k);
            for (uint32_t f = 0; f < bd.arity; ++f) cols[bd.first_child + f] = std::move(leaves[f]);
            cols[bn] = std::move(Bc[e]);
        }
        cols[an] = std::move(A[h]);
    }
    return MBRWT_OK;
}

// KIND_PACKT node: the columns of every node below it, from the DFS records
// (mbrwt_internal.hpp): visiting internal node x at its position jx with
// children bits m sets bit jx of each set child's column; an internal child
// is then visited at its own next position (positions ascend with j)
int decode_packt(const Tree &t, uint32_t v, std::vector<Bits> &cols) {
    const DevNode &dn = t.nodes[v];
    const uint32_t S = dn.stride;
    const uint64_t L = dn.length, blocks = (L + S - 1) / S;
    std::vector<uint8_t> img, spill;
    int rc;
    if ((rc = copy_down(dn.base, blocks * kPack2Block, img))) return rc;
    std::vector<uint64_t> next(t.nodes.size(), 0);  // next position of each internal node
    std::vector<uint32_t> inner{v};
    for (size_t h = 0; h < inner.size(); ++h) {
        const DevNode &x = t.nodes[inner[h]];
        for (uint32_t c = 0; c < x.arity; ++c) {
            cols[x.first_child + c] = Bits(x.length);
            if (t.nodes[x.first_child + c].kind != KIND_LEAF) inner.push_back(x.first_child + c);
        }
    }
    struct Frame {
        uint32_t x;
        uint64_t jx;
        uint32_t rem;
    };
    std::vector<Frame> st;
    for (uint64_t b = 0; b < blocks; ++b) {
        const uint8_t *blk = &img[b * kPack2Block];
        const uint8_t *rec = blk;
        std::vector<uint32_t> start(S + 1);
        const uint32_t npos = (uint32_t)std::min<uint64_t>(S, L - b * S);
        if (blk[0] == 0) {  // spilled: u16 start[S+1], then the records
            uint64_t addr = 0;
            std::memcpy(&addr, blk + 8, 8);
            std::vector<uint8_t> hdr;
            if ((rc = copy_down(addr, 2ull * (S + 1), hdr))) return rc;
            for (uint32_t k = 0; k <= S; ++k) start[k] = hdr[2 * k] | ((uint32_t)hdr[2 * k + 1] << 8);
            if ((rc = copy_down(addr, start[S], spill))) return rc;
            rec = spill.data();
        } else {
            for (uint32_t k = 0; k < S; ++k) start[k] = blk[k];
        }
        for (uint32_t k = 0; k < npos; ++k) {
            uint32_t o = start[k] + 1;  // (the record's label count)
            auto mask = [&](uint32_t x) {
                uint32_t m = rec[o++];
                if (packt_mask_bytes(t.nodes[x].arity) == 2) m |= (uint32_t)rec[o++] << 8;
                return m;
            };
            ++next[v];
            st.assign(1, Frame{v, b * S + k, mask(v)});
            while (!st.empty()) {
                Frame &f = st.back();
                if (!f.rem) {
                    st.pop_back();
                    continue;
                }
                const uint32_t c = (uint32_t)__builtin_ctz(f.rem);
                f.rem &= f.rem - 1;
                const uint32_t w = t.nodes[f.x].first_child + c;
                cols[w].set(f.jx);
                if (t.nodes[w].kind == KIND_LEAF) continue;
                const uint64_t jw = next[w]++;
                const uint32_t mw = mask(w);
                st.push_back(Frame{w, jw, mw});
            }
        }
    }
    return MBRWT_OK;
}

// the shape of a context's tree (tree node u = dnode u + 1; the folded
// root's record keeps no arity: its children are dnode 0's)
void fill_shape(const Tree &t, mbrwt_tree &out) {
    const uint32_t N = (uint32_t)t.nodes.size() - 1;
    out.num_children.resize(N);
    out.first_child.resize(N);
    out.leaf_column.assign(N, UINT32_MAX);
    out.vec_size.assign(N, 0);
    out.words.resize(N);
    for (uint32_t u = 0; u < N; ++u) {
        const DevNode &dn = t.nodes[u + 1];
        const bool internal = dn.kind != KIND_LEAF;
        const uint32_t a = dn.kind == KIND_FOLDED ? t.nodes[0].arity : internal ? dn.arity : 0;
        const uint32_t fc = dn.kind == KIND_FOLDED ? t.nodes[0].first_child : dn.first_child;
        out.num_children[u] = a;
        out.first_child[u] = a ? fc - 1 : 0;
        if (!a) out.leaf_column[u] = t.label_perm.empty() ? dn.label : t.label_perm.at(dn.label);
    }
}

int export_tree(const Ctx &c, mbrwt_tree &out) {
    const Tree &t = c.tree;
    out.num_rows = t.num_rows;
    out.num_columns = t.num_columns;
    if (t.nodes.empty()) return MBRWT_OK;
    const uint32_t D = (uint32_t)t.nodes.size();  // dnode u+1 = tree node u
    std::vector<Bits> cols(D);                    // index column of every dnode
    int rc;
    // the root's column, and its children's when the root is folded
    {
        std::vector<Bits> ch;
        if ((rc = decode_plain(t.nodes[0], ch))) return rc;
        if (!t.folded) {
            cols[1] = std::move(ch.at(0));
        } else {
            const DevNode &root = t.nodes[0];
            Bits r(t.num_rows);
            for (uint32_t k = 0; k < root.arity; ++k)
                for (size_t w = 0; w < r.w.size(); ++w) r.w[w] |= ch[k].w[w];
            const uint64_t L = r.ones();
            std::vector<Bits> sub(root.arity, Bits(L));
            uint64_t j = 0;
            for (uint64_t i = 0; i < t.num_rows; ++i) {
                if (!r.get(i)) continue;
                for (uint32_t k = 0; k < root.arity; ++k)
                    if (ch[k].get(i)) sub[k].set(j);
                ++j;
            }
            cols[1] = std::move(r);
            for (uint32_t k = 0; k < root.arity; ++k) cols[root.first_child + k] = std::move(sub[k]);
        }
    }
    for (uint32_t v = 1; v < D; ++v) {
        const DevNode &dn = t.nodes[v];
        if (dn.kind == KIND_LEAF || dn.kind == KIND_FOLDED || dn.base == 0) continue;  // no image of its own
        if (dn.kind == KIND_PACKT) {
            if ((rc = decode_packt(t, v, cols))) return rc;
        } else if (dn.kind == KIND_PACK2) {
            if ((rc = decode_pack2(t, v, cols))) return rc;
        } else if (dn.kind == KIND_PACK) {
            if ((rc = decode_pack(t, v, cols))) return rc;
        } else {
            std::vector<Bits> ch;
            if ((rc = decode_plain(dn, ch))) return rc;
            for (uint32_t k = 0; k < dn.arity; ++k) cols[dn.first_child + k] = std::move(ch[k]);
        }
    }
    fill_shape(t, out);
    for (uint32_t u = 0; u + 1 < D; ++u) {
        out.vec_size[u] = cols[u + 1].n;
        out.words[u] = std::move(cols[u + 1].w);
    }
    return MBRWT_OK;
}

// ---- export of a row-record image (rows.hip, mbrwt_internal.hpp "ROW
// RECORDS"): a row's record is the children mask of every internal node its
// descent reaches, in DFS pre-order, and positions in a node ascend with the
// rows that reach it (rank1 is monotone), so reading the records in row
// order and appending, at every reached node u, bit c of u's mask to child
// c's column rebuilds every index column -- the inverse of k_rows_measure /
// k_rows_write.  A record's label count is 0 exactly when the root's bit is 0
// (a set index bit always has a set child: BRWTBottomUpBuilder's columns are
// the OR of their children's, BRWT_builders.cpp:33-50).  Rows are split over
// host threads; each thread's columns are appended in row order afterwards.
struct BitAppend {
    std::vector<uint64_t> w;
    uint64_t n = 0;
    void push(uint32_t bit) {
        if ((n & 63) == 0) w.push_back(0);
        if (bit) w.back() |= 1ull << (n & 63);
        ++n;
    }
    void append(const BitAppend &o) {  // o's bits after ours
        if (!o.n) return;
        const uint64_t at = n;
        w.resize((at + o.n + 63) / 64, 0);
        for (size_t i = 0; i < o.w.size(); ++i) {
            const uint64_t v = o.w[i], pos = at + 64 * i;
            w[pos >> 6] |= v << (pos & 63);
            if ((pos & 63) && (pos >> 6) + 1 < w.size()) w[(pos >> 6) + 1] |= v >> (64 - (pos & 63));
        }
        n = at + o.n;
    }
};

// Variable-length records (rows_var.hip): a record lists the leaf parents
// ("units") the row reaches and their masks; every node above a reached unit
// is reached, and its mask has the bit of each child with a reached unit
// below.  Those masks are rebuilt per row and then appended exactly as the
// block records' pre-order masks are.
int export_var(const Ctx &c, mbrwt_tree &out) {
    const Tree &t = c.tree;
    const RowsImage &im = c.rows;
    const uint32_t D = (uint32_t)t.nodes.size();
    const uint32_t rootd = t.folded ? 0u : 1u;
    const uint64_t R = t.num_rows;
    const uint32_t W = im.var_W;
    // unit -> dnode, dnode -> (parent, child index)
    std::vector<uint32_t> unit_dnode(im.var_units.size(), 0), parent(D, UINT32_MAX), cidx(D, 0);
    for (uint32_t v = 0; v < D; ++v)
        if (im.var_unit_of[v] != 0xFFFFu) unit_dnode[im.var_unit_of[v]] = v;
    for (uint32_t v = rootd; v < D; ++v) {
        const DevNode &dn = t.nodes[v];
        if (dn.kind == KIND_LEAF || dn.kind == KIND_FOLDED || (v == 0 && !t.folded)) continue;
        for (uint32_t ch = 0; ch < dn.arity; ++ch) {
            parent[dn.first_child + ch] = v;
            cidx[dn.first_child + ch] = ch;
        }
    }
    const unsigned hw = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
    const uint64_t T = R < (1ull << 20) ? 1 : std::min<uint64_t>(hw, (R + (1ull << 20) - 1) >> 20);
    std::vector<uint64_t> cut(T + 1);
    for (uint64_t k = 0; k <= T; ++k) cut[k] = std::min<uint64_t>(R, R * k / T / 13 * 13);
    cut[T] = R;
    std::vector<std::vector<BitAppend>> part(T, std::vector<BitAppend>(D));
    std::vector<int> prc(T, MBRWT_OK);
    // terminal records (r06): every dnode's parent below the root, so a
    // terminal's fields set the children bits of its ancestors
    std::vector<uint32_t> par;
    if (im.term) {
        par.assign(D, ~0u);
        std::vector<uint32_t> q{rootd};
        for (size_t h = 0; h < q.size(); ++h) {
            const DevNode &v = t.nodes[q[h]];
            if (v.kind == KIND_LEAF) continue;
            for (uint32_t c = 0; c < v.arity && v.first_child + c < D; ++c) {
                par[v.first_child + c] = q[h];
                if (t.nodes[v.first_child + c].kind != KIND_LEAF) q.push_back(v.first_child + c);
            }
        }
    }
    auto work = [&](uint64_t k) {
        std::vector<BitAppend> &cols = part[k];
        std::vector<uint32_t> mask_of(D, 0), touched;
        struct Frame {
            uint32_t fc, rem;
        };
        std::vector<Frame> st;
        const uint64_t g0 = cut[k] / 13, g1 = (cut[k + 1] + 12) / 13;
        std::vector<uint8_t> lines, recs;
        for (uint64_t ga = g0; ga < g1;) {
            const uint64_t gb = std::min<uint64_t>(g1, ga + (1u << 16));
            lines.resize((gb - ga) * 64);
            if (hipMemcpy(lines.data(), im.var_lines + ga * 64, lines.size(), hipMemcpyDeviceToHost) != hipSuccess) {
                prc[k] = MBRWT_ERR_DEVICE;
                return;
            }
            for (uint64_t g = ga; g < gb;) {
                // a run of lines whose records are contiguous: one copy
                uint64_t base0 = 0;
                std::memcpy(&base0, &lines[(g - ga) * 64], 8);
                uint64_t end = base0, ge = g;
                while (ge < gb) {
                    uint64_t b = 0;
                    uint32_t span = 0;
                    std::memcpy(&b, &lines[(ge - ga) * 64], 8);
                    std::memcpy(&span, &lines[(ge - ga) * 64 + 8 + 4 * 13], 4);
                    if (b != end || (end - base0) + 4ull * span > (64ull << 20)) {
                        if (ge == g) end = b + 4ull * span, ++ge;  // (a single line always goes)
                        break;
                    }
                    end = b + 4ull * span;
                    ++ge;
                }
                recs.resize(end - base0);
                if (!recs.empty() &&
                    hipMemcpy(recs.data(), reinterpret_cast<const void *>(base0), recs.size(), hipMemcpyDeviceToHost) !=
                        hipSuccess) {
                    prc[k] = MBRWT_ERR_DEVICE;
                    return;
                }
                for (uint64_t gl = g; gl < ge; ++gl) {
                    const uint8_t *L = &lines[(gl - ga) * 64];
                    uint64_t lb = 0;
                    std::memcpy(&lb, L, 8);
                    for (uint32_t tt = 0; tt < 13; ++tt) {
                        const uint64_t r = gl * 13 + tt;
                        if (r < cut[k] || r >= cut[k + 1]) continue;
                        uint32_t e = 0;
                        std::memcpy(&e, L + 8 + 4 * tt, 4);
                        const uint32_t count = e >> 17;
                        cols[1].push(count ? 1u : 0u);
                        if (!count) continue;
                        const uint8_t *rec = &recs[lb - base0 + 4ull * (e & 0x1FFFFu)];
                        uint32_t item = 0;
                        for (uint32_t wi = 0; wi < W; ++wi) {
                            uint32_t w = 0;
                            std::memcpy(&w, rec + 4 * wi, 4);
                            for (; w; w &= w - 1) {
                                const uint32_t u = wi * 32 + (uint32_t)__builtin_ctz(w);
                                uint32_t v = unit_dnode[u];
                                if (!mask_of[v]) touched.push_back(v);
                                mask_of[v] = rec[4 * W + item++];
                                while (v != rootd && parent[v] != UINT32_MAX) {
                                    const uint32_t pv = parent[v], bit = 1u << cidx[v];
                                    if (!mask_of[pv]) touched.push_back(pv);
                                    const bool seen = mask_of[pv] != 0;
                                    mask_of[pv] |= bit;
                                    if (seen) break;  // its ancestors already have their bits
                                    v = pv;
                                }
                            }
                        }
                        // the pre-order visit of the reached nodes (export_rows)
                        auto visit = [&](uint32_t v) {
                            const DevNode &dn = t.nodes[v];
                            const uint32_t m = mask_of[v];
                            for (uint32_t ch = 0; ch < dn.arity; ++ch) cols[dn.first_child + ch].push((m >> ch) & 1u);
                            st.push_back(Frame{dn.first_child, m});
                        };
                        st.clear();
                        visit(rootd);
                        while (!st.empty()) {
                            Frame &f = st.back();
                            if (!f.rem) {
                                st.pop_back();
                                continue;
                            }
                            const uint32_t ch = (uint32_t)__builtin_ctzll(f.rem);
                            f.rem &= f.rem - 1;
                            const uint32_t w = f.fc + ch;
                            if (t.nodes[w].kind != KIND_LEAF) visit(w);
                        }
                        for (uint32_t v : touched) mask_of[v] = 0;
                        touched.clear();
                    }
                }
                g = ge;
            }
            ga = gb;
        }
    };
    if (T == 1) {
        work(0);
    } else {
        std::vector<std::thread> th;
        for (uint64_t k = 0; k < T; ++k)
            th.emplace_back([&, k] {
                (void)hipSetDevice(c.device);
                work(k);
            });
        for (auto &x : th) x.join();
    }
    for (int r : prc)
        if (r) {
            set_error("export: variable-length record image unreadable");
            return r;
        }
    fill_shape(t, out);
    for (uint32_t u = 0; u + 1 < D; ++u) {
        BitAppend &acc = part[0][u + 1];
        for (uint64_t k = 1; k < T; ++k) {
            acc.append(part[k][u + 1]);
            part[k][u + 1] = BitAppend();
        }
        out.vec_size[u] = acc.n;
        out.words[u] = std::move(acc.w);
    }
    return MBRWT_OK;
}

int export_rows(const Ctx &c, mbrwt_tree &out) {
    const Tree &t = c.tree;
    const RowsImage &im = c.rows;
    if (im.var) {
        out.num_rows = t.num_rows;
        out.num_columns = t.num_columns;
        return export_var(c, out);
    }
    out.num_rows = t.num_rows;
    out.num_columns = t.num_columns;
    if (t.nodes.size() < 2) return MBRWT_OK;
    const uint32_t D = (uint32_t)t.nodes.size();
    const uint32_t rootd = t.folded ? 0u : 1u;  // the dnode holding the root's children (arity, first child)
    const uint64_t R = t.num_rows;
    std::vector<uint8_t> spill;
    int rc;
    if ((rc = copy_down((uint64_t)(uintptr_t)im.spill, im.spill_bytes, spill))) return rc;
    std::vector<uint8_t> dict, cidx;  // record classes: the dictionary blocks and the class index
    if (im.classes) {
        if ((rc = copy_down((uint64_t)(uintptr_t)im.blocks, im.num_blocks * im.B, dict))) return rc;
        if ((rc = copy_down((uint64_t)(uintptr_t)im.classes, im.class_index_bytes, cidx))) return rc;
    }
    const unsigned hw = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
    const uint64_t T = R < (1ull << 20) ? 1 : std::min<uint64_t>(hw, (R + (1ull << 20) - 1) >> 20);
    // thread k: rows [a_k, a_{k+1}), block-aligned
    std::vector<uint64_t> cut(T + 1);
    for (uint64_t k = 0; k <= T; ++k) cut[k] = std::min<uint64_t>(R, (R * k / T + im.S - 1) / im.S * im.S);
    cut[T] = R;
    std::vector<std::vector<BitAppend>> part(T, std::vector<BitAppend>(D));
    std::vector<int> prc(T, MBRWT_OK);
    // terminal records (r06): every dnode's parent below the root, so a
    // terminal's fields set the children bits of its ancestors
    std::vector<uint32_t> par;
    if (im.term) {
        par.assign(D, ~0u);
        std::vector<uint32_t> q{rootd};
        for (size_t h = 0; h < q.size(); ++h) {
            const DevNode &v = t.nodes[q[h]];
            if (v.kind == KIND_LEAF) continue;
            for (uint32_t c = 0; c < v.arity && v.first_child + c < D; ++c) {
                par[v.first_child + c] = q[h];
                if (t.nodes[v.first_child + c].kind != KIND_LEAF) q.push_back(v.first_child + c);
            }
        }
    }
    auto work = [&](uint64_t k) {
        std::vector<BitAppend> &cols = part[k];
        std::vector<uint8_t> blk;
        struct Frame {
            uint32_t fc;   // first child (dnode)
            uint64_t rem;  // children still to visit
        };
        std::vector<Frame> st;
        std::vector<uint64_t> mk(im.term ? D : 0, 0);  // terminal records: the row's masks by dnode
        std::vector<uint32_t> touched;
        // one row's record (entry tt of block bp) -> its bits of every index column
        auto row_bits = [&](const uint8_t *bp, uint32_t tt) -> bool {
            const uint32_t e = bp[tt], o = e & 0x7Fu;
            const uint8_t *rec;
            uint32_t count;
            if (e & 0x80u) {
                uint32_t idx = 0;
                std::memcpy(&idx, bp + o + 1, 4);
                if ((uint64_t)idx * 16 + 8 > spill.size()) return false;
                std::memcpy(&count, &spill[(uint64_t)idx * 16], 4);
                rec = &spill[(uint64_t)idx * 16 + 8];
            } else {
                count = bp[o];
                rec = bp + o + 1;
            }
            cols[1].push(count ? 1u : 0u);
            if (!count) return true;
            if (im.term) {  // the terminals' fields -> the masks of every node they reach
                for (const uint32_t u : touched) mk[u] = 0;
                touched.clear();
                const uint32_t w = im.table3[0] & 0xFFu, ib = (im.table3[0] >> 8) & 0xFFu, nT = im.table3[1];
                uint32_t left = count, bit = 0;
                auto set = [&](uint32_t u, uint64_t bits) {
                    if (!mk[u]) touched.push_back(u);
                    mk[u] |= bits;
                };
                while (left) {
                    uint64_t x = 0;
                    for (uint32_t k = 0; 8 * k < (bit & 7) + w; ++k) x |= (uint64_t)rec[(bit >> 3) + k] << (8 * k);
                    const uint32_t f = (uint32_t)(x >> (bit & 7)) & ((1u << w) - 1u);
                    bit += w;
                    const uint32_t id = f & ((1u << ib) - 1u);
                    if (id >= nT || id >= im.term_dnode.size()) return false;
                    const uint32_t e = im.table3[4 + id], u = im.term_dnode[id];
                    const uint32_t m = (e >> 30) == 3u ? f >> ib : 1u;
                    if (!m || u >= D) return false;
                    if ((e >> 30) == 3u) set(u, m);
                    for (uint32_t ch = u; ch != rootd;) {
                        const uint32_t p = par[ch];
                        if (p == ~0u) return false;
                        set(p, 1ull << (ch - t.nodes[p].first_child));
                        ch = p;
                    }
                    left -= std::min<uint32_t>(left, (uint32_t)__builtin_popcount(m));
                }
            }
            uint32_t pos = 0;  // (bytes; nibbles for nibble-coded masks, rows_record.hpp RecMasks)
            auto nibble = [&](uint32_t k) { return (uint32_t)(rec[k >> 1] >> ((k & 1u) * 4u)) & 15u; };
            auto visit = [&](uint32_t v) {  // v reached: read its mask, append its children's bits
                const DevNode &dn = t.nodes[v];
                uint64_t m;
                if (im.term) {
                    m = mk[v];
                } else if (im.nib) {
                    const uint32_t c = nibble(pos);
                    if (c < 8) {
                        m = 1u << c;
                        pos += 1;
                    } else {
                        m = nibble(pos + 1) | nibble(pos + 2) << 4;
                        pos += 3;
                    }
                } else {  // one byte per 8 children (arity <= 64)
                    m = rec[pos++];
                    for (uint32_t k = 8; k < dn.arity; k += 8) m |= (uint64_t)rec[pos++] << k;
                }
                for (uint32_t ch = 0; ch < dn.arity; ++ch) cols[dn.first_child + ch].push((m >> ch) & 1u);
                st.push_back(Frame{dn.first_child, m});
            };
            st.clear();
            visit(rootd);
            while (!st.empty()) {
                Frame &f = st.back();
                if (!f.rem) {
                    st.pop_back();
                    continue;
                }
                const uint32_t ch = (uint32_t)__builtin_ctzll(f.rem);
                f.rem &= f.rem - 1;
                const uint32_t w = f.fc + ch;
                if (t.nodes[w].kind != KIND_LEAF) visit(w);
            }
            return true;
        };
        if (im.classes) {  // record classes: row r's record is block class(r) of the dictionary
            const uint32_t w = im.class_bits;
            for (uint64_t r = cut[k]; r < cut[k + 1]; ++r) {
                const uint64_t bit = r * w;
                uint64_t x = 0;
                std::memcpy(&x, &cidx[(bit >> 5) * 4], 8);
                const uint64_t cls = (x >> (bit & 31)) & ((1ull << w) - 1);
                if (cls >= im.num_classes || !row_bits(&dict[cls * im.B], 0)) {
                    prc[k] = MBRWT_ERR_INVALID;
                    return;
                }
            }
            return;
        }
        const uint64_t chunk_blocks = std::max<uint64_t>(1, (64ull << 20) / im.B);
        for (uint64_t b0 = cut[k] / im.S; b0 * im.S < cut[k + 1]; b0 += chunk_blocks) {
            const uint64_t b1 = std::min<uint64_t>((cut[k + 1] + im.S - 1) / im.S, b0 + chunk_blocks);
            blk.resize((b1 - b0) * im.B);
            if (hipMemcpy(blk.data(), im.blocks + b0 * im.B, blk.size(), hipMemcpyDeviceToHost) != hipSuccess) {
                prc[k] = MBRWT_ERR_DEVICE;
                return;
            }
            for (uint64_t b = b0; b < b1; ++b) {
                const uint8_t *bp = &blk[(b - b0) * im.B];
                for (uint32_t tt = 0; tt < im.S; ++tt) {
                    const uint64_t r = b * im.S + tt;
                    if (r >= cut[k + 1]) break;
                    if (!row_bits(bp, tt)) {
                        prc[k] = MBRWT_ERR_INVALID;
                        return;
                    }
                }
            }
        }
    };
    if (T == 1) {
        work(0);
    } else {
        std::vector<std::thread> th;
        for (uint64_t k = 0; k < T; ++k)
            th.emplace_back([&, k] {
                (void)hipSetDevice(c.device);
                work(k);
            });
        for (auto &x : th) x.join();
    }
    for (int r : prc)
        if (r) {
            set_error("export: row-record image unreadable");
            return r;
        }
    fill_shape(t, out);
    for (uint32_t u = 0; u + 1 < D; ++u) {
        BitAppend &acc = part[0][u + 1];
        for (uint64_t k = 1; k < T; ++k) {
            acc.append(part[k][u + 1]);
            part[k][u + 1] = BitAppend();
        }
        out.vec_size[u] = acc.n;
        out.words[u] = std::move(acc.w);
    }
    return MBRWT_OK;
}

}  // namespace
}  // namespace mbrwt

using namespace mbrwt;

extern "C" {

int mbrwt_tree_parse(const uint8_t *bytes, uint64_t len, uint64_t *consumed, mbrwt_tree **out) {
    if (!out || (!bytes && len)) {
        set_error("null argument");
        return MBRWT_ERR_INVALID;
    }
    *out = nullptr;
    try {
        fmt::Reader r(bytes, len);
        auto root = parse_node(r, 0);
        auto t = std::make_unique<mbrwt_tree>();
        to_tree(*root, *t);
        t->finish();
        if (consumed) *consumed = r.pos;
        *out = t.release();
        return MBRWT_OK;
    } catch (const FormatError &e) {
        set_error(std::string("BRWT stream: ") + e.what());
        return MBRWT_ERR_INVALID;
    } catch (const std::out_of_range &e) {
        set_error(std::string("BRWT stream: ") + e.what());
        return MBRWT_ERR_INVALID;
    } catch (const std::bad_alloc &) {
        set_error("out of host memory");
        return MBRWT_ERR_NOMEM;
    } catch (const std::exception &e) {  // e.g. length_error from a size no stream can back
        set_error(std::string("BRWT stream: ") + e.what());
        return MBRWT_ERR_INVALID;
    } catch (...) {
        set_error("BRWT stream: unexpected exception");
        return MBRWT_ERR_INVALID;
    }
}

int mbrwt_tree_serialize(const mbrwt_tree_desc *desc, uint8_t *buf, uint64_t cap, uint64_t *needed) {
    if (!desc) {
        set_error("null tree description");
        return MBRWT_ERR_INVALID;
    }
    if (desc->num_nodes && (!desc->num_children || !desc->first_child || !desc->leaf_column || !desc->vec_size ||
                            !desc->vec_words)) {
        set_error("null array in tree description");
        return MBRWT_ERR_INVALID;
    }
    try {
        fmt::Writer w;
        serialize_desc(*desc, w);
        if (needed) *needed = w.buf.size();
        if (!buf || cap < w.buf.size()) {
            set_error("buffer too small");
            return MBRWT_ERR_CAPACITY;
        }
        std::memcpy(buf, w.buf.data(), w.buf.size());
        return MBRWT_OK;
    } catch (const std::bad_alloc &) {
        set_error("out of host memory");
        return MBRWT_ERR_NOMEM;
    }
}

int mbrwt_tree_export(mbrwt_ctx *ctx, mbrwt_tree **out) {
    if (!ctx || !out) {
        set_error("null argument");
        return MBRWT_ERR_INVALID;
    }
    *out = nullptr;
    Ctx &c = *reinterpret_cast<Ctx *>(ctx);
    std::lock_guard<std::mutex> lk(c.mu);
    try {
        MBRWT_HIP(hipSetDevice(c.device));
        auto t = std::make_unique<mbrwt_tree>();
        if (c.nodes_freed) {  // row records only: the columns from the records
            if (!c.rows.ready) {
                set_error("export: context without an image");
                return MBRWT_ERR_UNSUPPORTED;
            }
            const int rc = export_rows(c, *t);
            if (rc) return rc;
        } else if (c.shards.empty()) {
            const int rc = export_tree(c, *t);
            if (rc) return rc;
        } else {
            // row shards (shards.hip): every node's column is the concatenation
            // of its columns in the shards, in row order (the inverse of slice_desc)
            for (size_t k = 0; k < c.shards.size(); ++k) {
                mbrwt_tree part;
                const int rc = export_tree(*c.shards[k], part);
                if (rc) return rc;
                if (k == 0) {
                    *t = std::move(part);
                    continue;
                }
                if (part.num_children != t->num_children || part.first_child != t->first_child ||
                    part.leaf_column != t->leaf_column) {
                    set_error("export: row shards with different tree shapes");
                    return MBRWT_ERR_UNSUPPORTED;
                }
                t->num_rows += part.num_rows;
                for (size_t u = 0; u < part.vec_size.size(); ++u) {
                    auto &w = t->words[u];
                    const uint64_t at = t->vec_size[u], len = part.vec_size[u];
                    w.resize((at + len + 63) / 64, 0);
                    for (uint64_t i = 0; i < (len + 63) / 64; ++i) {
                        const uint64_t v = part.words[u][i], pos = at + 64 * i;
                        w[pos >> 6] |= v << (pos & 63);
                        if ((pos & 63) && (pos >> 6) + 1 < w.size()) w[(pos >> 6) + 1] |= v >> (64 - (pos & 63));
                    }
                    t->vec_size[u] = at + len;
                }
            }
            t->num_rows = c.tree.num_rows;
        }
        t->finish();
        *out = t.release();
        return MBRWT_OK;
    } catch (const std::bad_alloc &) {
        set_error("out of host memory");
        return MBRWT_ERR_NOMEM;
    }
}

const mbrwt_tree_desc *mbrwt_tree_get_desc(const mbrwt_tree *t) { return t ? &t->desc : nullptr; }

int mbrwt_load(const uint8_t *bytes, uint64_t len, uint64_t *consumed, int device, mbrwt_ctx **out) {
    if (!out) {
        set_error("null output pointer");
        return MBRWT_ERR_INVALID;
    }
    *out = nullptr;
    mbrwt_tree *t = nullptr;
    int rc = mbrwt_tree_parse(bytes, len, consumed, &t);
    if (rc) return rc;
    rc = mbrwt_create(&t->desc, device, out);
    mbrwt_tree_free(t);
    return rc;
}

void mbrwt_tree_free(mbrwt_tree *t) { delete t; }

}  // extern "C"
