// build.hip -- BRWTBottomUpBuilder::build (BRWT_builders.cpp:119-163) with
// the basic partitioner (BRWT_builders.cpp:20-31) on the device.
//
// Bottom-up, level by level as the reference does: the nodes of a level are
// grouped by `arity` consecutive nodes (a group of one passes through,
// BRWT_builders.cpp:75-77); a group's parent column over the rows is the OR of
// its children's columns (compute_or, :33-50) and each child's index column
// is its row column restricted to the parent's set positions
// (generate_subindex, :52-67) -- a parallel bit extract (pext) of every
// 64-bit word, placed at the exclusive prefix of the parent's popcounts.  The
// root's index column is its row column (:160-162).  The index columns then
// go through build_from_desc (image.cpp) like any tree description, so the
// device image is exactly the one of the equivalent mbrwt_tree_desc.
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "device_access.hpp"
#include "mbrwt_internal.hpp"

namespace mbrwt {
namespace {

// One level of the bottom-up build, batched: every group of >= 2 nodes of the
// level is a parent g; its children are entries [gchild[g], gchild[g+1]) of
// the child tables.
struct LevelArgs {
    const uint64_t *const *child_col;  // [children] the child's row column (W words)
    uint64_t *const *child_out;        // [children] the child's index column (zeroed)
    const uint32_t *child_group;       // [children] its parent g
    const uint32_t *gchild;            // [groups + 1]
    uint64_t *parents;                 // [groups][W] parent row columns
    unsigned long long *popc;          // [groups * W + 1] popcounts of the parents' words
    unsigned long long *pre;           // [groups * W + 1] their exclusive prefix
    uint64_t W;
};

// compute_or (BRWT_builders.cpp:33-50): parent[g][w] = OR of its children's
// words, and the word's popcount (group = y0 + blockIdx.y)
__global__ void k_or(LevelArgs A, uint32_t y0) {
    const uint32_t g = y0 + blockIdx.y;
    const uint32_t c0 = A.gchild[g], c1 = A.gchild[g + 1];
    const uint64_t gstride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t w = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; w < A.W; w += gstride) {
        uint64_t x = 0;
        for (uint32_t c = c0; c < c1; ++c) x |= gld(A.child_col[c] + w);
        A.parents[(uint64_t)g * A.W + w] = x;
        A.popc[(uint64_t)g * A.W + w] = (unsigned long long)__builtin_popcountll(x);
    }
}

// bits of c at the set positions of p, packed from bit 0
__device__ __forceinline__ uint64_t pext64(uint64_t c, uint64_t p) {
    if (p == ~0ull) return c;
    uint64_t r = 0;
    for (uint32_t i = 0; p; ++i, p &= p - 1)
        if (c & (p & (~p + 1))) r |= 1ull << i;
    return r;
}

// generate_subindex (BRWT_builders.cpp:52-67) for every child of the level
// (child = y0 + blockIdx.y): word w of its parent contributes popc(parent[w])
// bits at the parent-relative offset prefix[g][w] - prefix[g][0]
__global__ void k_pext(LevelArgs A, uint32_t y0) {
    const uint32_t c = y0 + blockIdx.y;
    const uint32_t g = A.child_group[c];
    const uint64_t *col = A.child_col[c];
    const uint64_t *par = A.parents + (uint64_t)g * A.W;
    const unsigned long long *pre = A.pre + (uint64_t)g * A.W;
    const unsigned long long base = pre[0];
    unsigned long long *out = reinterpret_cast<unsigned long long *>(A.child_out[c]);
    const uint64_t gstride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t w = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; w < A.W; w += gstride) {
        const uint64_t p = par[w];
        if (!p) continue;
        const uint64_t bits = pext64(gld(col + w), p);
        if (!bits) continue;
        const uint64_t off = pre[w] - base;
        const uint32_t sh = (uint32_t)(off & 63);
        atomicOr(out + (off >> 6), (unsigned long long)(bits << sh));
        if (sh && (bits >> (64 - sh))) atomicOr(out + (off >> 6) + 1, (unsigned long long)(bits >> (64 - sh)));
    }
}

__global__ void k_clear_tails(uint64_t *cols, uint64_t m, uint64_t W, uint64_t keep) {
    const uint64_t gstride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; j < m; j += gstride) cols[j * W + W - 1] &= keep;
}

unsigned grid_of(uint64_t n, uint64_t ys = 1) {  // keep x * y moderate for 2-D grids
    const uint64_t cap = std::max<uint64_t>(1, 65536 / std::max<uint64_t>(1, ys));
    return (unsigned)std::max<uint64_t>(1, std::min<uint64_t>((n + 255) / 256, cap));
}

struct BNode {
    std::vector<uint32_t> children;  // node ids, reference child order
    uint32_t column = UINT32_MAX;    // leaves
    uint64_t *rowcol = nullptr;      // device: the node's column over the rows (W words)
    std::vector<uint64_t> index;     // host: the node's index column
    uint64_t index_len = 0;
};

}  // namespace

int build_from_columns(const mbrwt_columns_desc &cd, int device, Tree &tree, hipStream_t s) {
    MBRWT_HIP(hipSetDevice(device));
    const uint64_t n = cd.num_rows, m = cd.num_columns;
    if (cd.arity < 2 || cd.arity > kMaxArity) {
        set_error("arity must be in [2, 64]");
        return MBRWT_ERR_INVALID;
    }
    if (m && !cd.columns) {
        set_error("null column array");
        return MBRWT_ERR_INVALID;
    }
    if (m > 0xFFFFFFFFull || n > kMaxRows) {
        set_error("num_rows >= 2^32 or num_columns >= 2^32 is not supported by this build");
        return MBRWT_ERR_UNSUPPORTED;
    }
    if (m == 0) {  // BRWTBottomUpBuilder::build of no columns is BRWT() (BRWT_builders.cpp:122-123)
        mbrwt_tree_desc empty{};
        return build_from_desc(empty, device, tree);
    }
    for (uint64_t j = 0; j < m; ++j)
        if (n && !cd.columns[j]) {
            set_error("null column");
            return MBRWT_ERR_INVALID;
        }
    const uint64_t W = (n + 63) / 64;
    std::vector<void *> allocs;
    auto cleanup = [&]() {
        for (void *p : allocs) (void)hipFree(p);
        allocs.clear();
    };
    auto dalloc = [&](size_t bytes) -> void * {
        void *p = nullptr;
        if (hipMalloc(&p, std::max<size_t>(bytes, 8)) != hipSuccess) return nullptr;
        allocs.push_back(p);
        return p;
    };
    auto dfree = [&](void *p) {
        auto it = std::find(allocs.begin(), allocs.end(), p);
        if (it != allocs.end()) {
            (void)hipFree(p);
            allocs.erase(it);
        }
    };
    // the columns, uploaded once (leaves' row columns)
    uint64_t *d_cols = reinterpret_cast<uint64_t *>(dalloc(m * W * sizeof(uint64_t)));
    if (!d_cols) {
        cleanup();
        return hip_fail(hipErrorOutOfMemory, "builder allocation");
    }
    const auto t_start = std::chrono::steady_clock::now();
    // one copy when the caller's columns are back to back, else one per column
    bool contiguous = true;
    for (uint64_t j = 1; j < m && contiguous; ++j) contiguous = cd.columns[j] == cd.columns[0] + j * W;
    if (W) {
        if (contiguous) {
            MBRWT_HIP(hipMemcpyAsync(d_cols, cd.columns[0], m * W * sizeof(uint64_t), hipMemcpyHostToDevice, s));
        } else {
            for (uint64_t j = 0; j < m; ++j)
                MBRWT_HIP(hipMemcpyAsync(d_cols + j * W, cd.columns[j], W * sizeof(uint64_t), hipMemcpyHostToDevice, s));
        }
    }
    // tail bits past num_rows are ignored by the reference's bit vectors: clear them
    if (n & 63) {
        hipLaunchKernelGGL(k_clear_tails, dim3(grid_of(m)), dim3(256), 0, s, d_cols, m, W, (1ull << (n & 63)) - 1);
        MBRWT_HIP(hipGetLastError());
    }

    std::vector<BNode> nodes(m);
    std::vector<uint32_t> level(m);
    for (uint32_t j = 0; j < m; ++j) {
        nodes[j].column = j;
        nodes[j].rowcol = d_cols + (uint64_t)j * W;
        level[j] = j;
    }
    void *prev_parents = nullptr;  // row columns of the previous level's parents
    while (level.size() > 1) {  // BRWT_builders.cpp:134-158
        // groups of the basic partitioner; singletons pass through (:75-77)
        std::vector<uint32_t> next, gchild{0}, child_group, child_node;
        std::vector<size_t> group_slot;  // position in `next` of each parent
        for (size_t g0 = 0; g0 < level.size(); g0 += cd.arity) {
            const size_t g1 = std::min<size_t>(level.size(), g0 + cd.arity);
            if (g1 - g0 == 1) {
                // a passed-through internal node keeps its row column: move it
                // out of the previous level's parent arena, freed below
                BNode &single = nodes[level[g0]];
                if (!single.children.empty() && W) {
                    uint64_t *own = reinterpret_cast<uint64_t *>(dalloc(W * sizeof(uint64_t)));
                    if (!own) {
                        cleanup();
                        return hip_fail(hipErrorOutOfMemory, "builder allocation");
                    }
                    MBRWT_HIP(hipMemcpyAsync(own, single.rowcol, W * sizeof(uint64_t), hipMemcpyDeviceToDevice, s));
                    single.rowcol = own;
                }
                next.push_back(level[g0]);
                continue;
            }
            const uint32_t g = (uint32_t)group_slot.size();
            for (size_t i = g0; i < g1; ++i) {
                child_group.push_back(g);
                child_node.push_back(level[i]);
            }
            gchild.push_back((uint32_t)child_node.size());
            group_slot.push_back(next.size());
            next.push_back(UINT32_MAX);
        }
        const uint32_t G = (uint32_t)group_slot.size(), NC = (uint32_t)child_node.size();
        if ((uint64_t)G * W + 1 > 0x7FFFFFFFull) {  // hipCUB scan item count
            cleanup();
            set_error("matrix too large for the device builder (groups x words >= 2^31)");
            return MBRWT_ERR_UNSUPPORTED;
        }
        // device tables + parent row columns + popcounts/prefixes
        uint64_t *d_par = reinterpret_cast<uint64_t *>(dalloc(G * W * sizeof(uint64_t)));
        unsigned long long *d_popc = reinterpret_cast<unsigned long long *>(dalloc((G * W + 1) * sizeof(uint64_t)));
        unsigned long long *d_pre = reinterpret_cast<unsigned long long *>(dalloc((G * W + 1) * sizeof(uint64_t)));
        const size_t tbytes = NC * (2 * sizeof(uint64_t) + sizeof(uint32_t)) + (G + 1) * sizeof(uint32_t);
        uint8_t *d_tab = reinterpret_cast<uint8_t *>(dalloc(tbytes));
        size_t scan_bytes = 0;
        MBRWT_HIP(hipcub::DeviceScan::ExclusiveSum(nullptr, scan_bytes, d_popc, d_pre, (int)(G * W + 1), s));
        void *d_scan = dalloc(scan_bytes + 16);
        if (!d_par || !d_popc || !d_pre || !d_tab || !d_scan) {
            cleanup();
            return hip_fail(hipErrorOutOfMemory, "builder allocation");
        }
        std::vector<uint8_t> tab(tbytes);
        const uint64_t **h_col = reinterpret_cast<const uint64_t **>(tab.data());
        uint32_t *h_cg = reinterpret_cast<uint32_t *>(tab.data() + NC * 2 * sizeof(uint64_t));
        uint32_t *h_gc = h_cg + NC;
        for (uint32_t c = 0; c < NC; ++c) {
            h_col[c] = nodes[child_node[c]].rowcol;
            h_cg[c] = child_group[c];
        }
        for (uint32_t g = 0; g <= G; ++g) h_gc[g] = gchild[g];
        LevelArgs A{};
        A.child_col = reinterpret_cast<const uint64_t *const *>(d_tab);
        A.child_out = reinterpret_cast<uint64_t *const *>(d_tab + NC * sizeof(uint64_t));
        A.child_group = reinterpret_cast<const uint32_t *>(d_tab + NC * 2 * sizeof(uint64_t));
        A.gchild = A.child_group + NC;
        A.parents = d_par;
        A.popc = d_popc;
        A.pre = d_pre;
        A.W = W;
        MBRWT_HIP(hipMemcpyAsync(d_tab, tab.data(), tbytes, hipMemcpyHostToDevice, s));
        for (uint32_t y0 = 0; W && y0 < G; y0 += 65535) {  // grid y <= 65535
            const uint32_t ny = std::min<uint32_t>(65535, G - y0);
            hipLaunchKernelGGL(k_or, dim3(grid_of(W, ny), ny), dim3(256), 0, s, A, y0);
        }
        MBRWT_HIP(hipGetLastError());
        MBRWT_HIP(hipMemsetAsync(d_popc + G * W, 0, sizeof(uint64_t), s));
        MBRWT_HIP(hipcub::DeviceScan::ExclusiveSum(d_scan, scan_bytes, d_popc, d_pre, (int)(G * W + 1), s));
        // parent popcounts = lengths of the children's index columns
        std::vector<unsigned long long> gpre(G + 1);
        for (uint32_t g = 0; g <= G; ++g)
            MBRWT_HIP(hipMemcpyAsync(&gpre[g], d_pre + (uint64_t)g * W, sizeof(uint64_t), hipMemcpyDeviceToHost, s));
        MBRWT_HIP(hipStreamSynchronize(s));
        // one arena for the level's index columns
        std::vector<uint64_t> out_off(NC + 1, 0);
        for (uint32_t c = 0; c < NC; ++c) {
            const uint64_t len = gpre[child_group[c] + 1] - gpre[child_group[c]];
            out_off[c + 1] = out_off[c] + (len + 63) / 64;
        }
        uint64_t *d_out = reinterpret_cast<uint64_t *>(dalloc(std::max<uint64_t>(1, out_off[NC]) * sizeof(uint64_t)));
        if (!d_out) {
            cleanup();
            return hip_fail(hipErrorOutOfMemory, "builder allocation");
        }
        MBRWT_HIP(hipMemsetAsync(d_out, 0, std::max<uint64_t>(1, out_off[NC]) * sizeof(uint64_t), s));
        uint64_t **h_out = reinterpret_cast<uint64_t **>(tab.data() + NC * sizeof(uint64_t));
        for (uint32_t c = 0; c < NC; ++c) h_out[c] = d_out + out_off[c];
        MBRWT_HIP(hipMemcpyAsync(d_tab + NC * sizeof(uint64_t), h_out, NC * sizeof(uint64_t), hipMemcpyHostToDevice, s));
        for (uint32_t y0 = 0; W && y0 < NC; y0 += 65535) {
            const uint32_t ny = std::min<uint32_t>(65535, NC - y0);
            hipLaunchKernelGGL(k_pext, dim3(grid_of(W, ny), ny), dim3(256), 0, s, A, y0);
        }
        MBRWT_HIP(hipGetLastError());
        std::vector<uint64_t> h_all(std::max<uint64_t>(1, out_off[NC]));
        MBRWT_HIP(hipMemcpyAsync(h_all.data(), d_out, out_off[NC] * sizeof(uint64_t), hipMemcpyDeviceToHost, s));
        MBRWT_HIP(hipStreamSynchronize(s));
        for (uint32_t c = 0; c < NC; ++c) {
            BNode &ch = nodes[child_node[c]];
            ch.index_len = gpre[child_group[c] + 1] - gpre[child_group[c]];
            ch.index.assign(h_all.begin() + out_off[c], h_all.begin() + out_off[c + 1]);
            if (ch.index.empty()) ch.index.push_back(0);
        }
        for (uint32_t g = 0; g < G; ++g) {
            BNode parent;
            parent.children.assign(child_node.begin() + gchild[g], child_node.begin() + gchild[g + 1]);
            parent.rowcol = d_par + (uint64_t)g * W;
            next[group_slot[g]] = (uint32_t)nodes.size();
            nodes.push_back(std::move(parent));
        }
        dfree(d_out);
        dfree(d_tab);
        dfree(d_scan);
        dfree(d_pre);
        dfree(d_popc);
        if (prev_parents) dfree(prev_parents);  // the children's row columns (internal nodes) are done
        prev_parents = d_par;
        level.swap(next);
    }
    // the root's index column is its row column (:160-162)
    BNode &root = nodes[level[0]];
    root.index.assign(std::max<uint64_t>(W, 1), 0);
    root.index_len = n;
    MBRWT_HIP(hipMemcpyAsync(root.index.data(), root.rowcol, W * sizeof(uint64_t), hipMemcpyDeviceToHost, s));
    MBRWT_HIP(hipStreamSynchronize(s));
    cleanup();

    const auto t_index = std::chrono::steady_clock::now();
    // breadth-first numbering (mbrwt_tree_desc)
    std::vector<uint32_t> order{level[0]};
    for (size_t h = 0; h < order.size(); ++h)
        for (uint32_t c : nodes[order[h]].children) order.push_back(c);
    const uint32_t N = (uint32_t)order.size();
    std::vector<uint32_t> bfs(nodes.size());
    for (uint32_t i = 0; i < N; ++i) bfs[order[i]] = i;
    std::vector<uint32_t> num_children(N), first_child(N), leaf_column(N);
    std::vector<uint64_t> vec_size(N);
    std::vector<const uint64_t *> vec_words(N);
    for (uint32_t i = 0; i < N; ++i) {
        const BNode &b = nodes[order[i]];
        num_children[i] = (uint32_t)b.children.size();
        first_child[i] = b.children.empty() ? 0 : bfs[b.children[0]];
        leaf_column[i] = b.children.empty() ? b.column : UINT32_MAX;
        vec_size[i] = b.index_len;
        vec_words[i] = b.index.data();
    }
    mbrwt_tree_desc desc{};
    desc.num_rows = n;
    desc.num_columns = m;
    desc.num_nodes = N;
    desc.num_children = num_children.data();
    desc.first_child = first_child.data();
    desc.leaf_column = leaf_column.data();
    desc.vec_size = vec_size.data();
    desc.vec_words = vec_words.data();
    const int rc = build_from_desc(desc, device, tree);
    if (const char *e = std::getenv("MBRWT_BUILD_TIMING"); e && e[0] == '1') {
        const auto t_end = std::chrono::steady_clock::now();
        std::fprintf(stderr, "[mbrwt build] index columns %.1f ms, image layout %.1f ms\n",
                     std::chrono::duration<double, std::milli>(t_index - t_start).count(),
                     std::chrono::duration<double, std::milli>(t_end - t_index).count());
    }
    return rc;
}

}  // namespace mbrwt
