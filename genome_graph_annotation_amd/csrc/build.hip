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
#include <random>
#include <tuple>
#include <vector>

#include "device_access.hpp"
#include "mbrwt_internal.hpp"

namespace mbrwt {

static thread_local int g_build_partitioner = MBRWT_PARTITIONER_BASIC;
int build_partitioner() { return g_build_partitioner; }
void set_build_partitioner(int partitioner) { g_build_partitioner = partitioner; }

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

// ---- binary_grouping_greedy (partitionings.cpp:148-196) ---------------------
//
// The partitioner of the reference's production build (`transform_anno
// --greedy`, scripts/kingsford/convert.sh:24).  At every level the
// similarity of two columns is their inner product over a fixed row sample
// (random_submatrix, partitionings.cpp:37-58: a fresh mt19937 seeded 1,
// utils::sample_indexes of min(10^6, rows) rows, sorted); the pairs are
// taken greedily by (similarity descending, index distance ascending).  The
// m(m-1)/2 inner products -- the whole cost of the reference's greedy build
// -- are an AND-popcount "GEMM" over the sampled words: k_gather_sample
// compacts the sampled bits of every column, k_similarity computes 64 x 64
// tiles of the lower triangle with both column blocks staged in LDS.  The
// candidate order and the matching stay on the host with the reference's own
// std::sort and comparator: std::sort is not stable, so equal (similarity,
// distance) candidates come out in its order, which only the same algorithm
// reproduces, and that order can decide the matching.

// sampled bits: sub[c][w] bit b = column c at row idx[64 w + b]
__global__ __launch_bounds__(256) void k_gather_sample(const uint64_t *const *cols, const uint64_t *__restrict__ idx,
                                                       uint64_t ns, uint64_t SW, uint64_t *__restrict__ sub) {
    const uint32_t c = blockIdx.y;
    const uint64_t *col = cols[c];
    for (uint64_t w = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; w < SW; w += (uint64_t)gridDim.x * blockDim.x) {
        uint64_t x = 0;
        const uint64_t k0 = 64 * w;
        for (uint32_t b = 0; b < 64 && k0 + b < ns; ++b) {
            const uint64_t r = gld(idx + k0 + b);
            x |= ((gld(col + (r >> 6)) >> (r & 63)) & 1ull) << b;
        }
        sub[(uint64_t)c * SW + w] = x;
    }
}

// inner products of every pair j > k of the m sampled columns (SW words
// each; column c at cols[c]), 64 x 64 tiles of the lower triangle (tile
// (J, K), K <= J, from blockIdx.x), 4 x 4 products per thread, the words in
// chunks of 32 through LDS.  out[j (j - 1) / 2 + k] = <col j, col k>.
constexpr uint32_t kSimTile = 64, kSimChunk = 32;
__global__ __launch_bounds__(256) void k_similarity(const uint64_t *const *cols, uint32_t m, uint64_t SW,
                                                    uint32_t *__restrict__ out) {
    __shared__ uint64_t sa[kSimChunk][kSimTile + 1], sb[kSimChunk][kSimTile + 1];
    // tile index -> (J, K) with K <= J
    uint32_t t = blockIdx.x, J = 0;
    while (t > J) {
        t -= J + 1;
        ++J;
    }
    const uint32_t K = t;
    const uint32_t tx = threadIdx.x & 15, ty = threadIdx.x >> 4;  // 16 x 16 threads, 4 x 4 each
    uint32_t acc[4][4] = {};
    for (uint64_t w0 = 0; w0 < SW; w0 += kSimChunk) {
        for (uint32_t i = threadIdx.x; i < kSimChunk * kSimTile; i += 256) {
            const uint32_t col = i / kSimChunk, w = i % kSimChunk;  // consecutive threads: consecutive words
            const uint32_t ja = J * kSimTile + col, kb = K * kSimTile + col;
            sa[w][col] = (ja < m && w0 + w < SW) ? gld(cols[ja] + w0 + w) : 0ull;
            sb[w][col] = (kb < m && w0 + w < SW) ? gld(cols[kb] + w0 + w) : 0ull;
        }
        __syncthreads();
#pragma unroll 4
        for (uint32_t w = 0; w < kSimChunk; ++w) {
            uint64_t a[4], b[4];
#pragma unroll
            for (uint32_t i = 0; i < 4; ++i) {
                a[i] = sa[w][ty + 16 * i];
                b[i] = sb[w][tx + 16 * i];
            }
#pragma unroll
            for (uint32_t i = 0; i < 4; ++i)
#pragma unroll
                for (uint32_t q = 0; q < 4; ++q) acc[i][q] += (uint32_t)__popcll(a[i] & b[q]);
        }
        __syncthreads();
    }
#pragma unroll
    for (uint32_t i = 0; i < 4; ++i)
#pragma unroll
        for (uint32_t q = 0; q < 4; ++q) {
            const uint32_t j = J * kSimTile + ty + 16 * i, k = K * kSimTile + tx + 16 * q;
            if (j < m && k < j) out[(uint64_t)j * (j - 1) / 2 + k] = acc[i][q];
        }
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

// utils::sample_indexes (utils.cpp:777-816) as random_submatrix calls it
// (partitionings.cpp:37-58): a fresh mt19937 seeded 1, min(10^6, n) rows
// (kNumRowsSampled, partitionings.cpp:5), returned sorted
std::vector<uint64_t> greedy_sample_rows(uint64_t n) {
    std::vector<uint64_t> idx;
    if (!n) return idx;
    std::mt19937 gen;
    gen.seed(1);
    const uint64_t want = std::min<uint64_t>(n, 1000000);
    idx.reserve(3 * want);
    if (want * 10 < n) {
        std::uniform_int_distribution<uint64_t> dis(0, n - 1);
        while (idx.size() < want) {
            idx.clear();
            for (size_t i = 0; i < 1.5 * want; ++i) idx.push_back(dis(gen));
            std::sort(idx.begin(), idx.end());
            idx.erase(std::unique(idx.begin(), idx.end()), idx.end());
        }
    } else {
        std::bernoulli_distribution dis(2.0 * want / n);
        while (idx.size() < want) {
            idx.clear();
            for (uint64_t i = 0; i < n; ++i)
                if (dis(gen)) idx.push_back(i);
        }
    }
    std::shuffle(idx.begin(), idx.end(), gen);
    idx.resize(want);
    std::sort(idx.begin(), idx.end());
    return idx;
}

// the greedy pairs of one level (parallel_binary_grouping_greedy,
// partitionings.cpp:148-196) from the lower-triangle inner products
std::vector<std::vector<size_t>> greedy_groups(const std::vector<uint32_t> &sim, size_t m) {
    std::vector<std::tuple<size_t, size_t, uint64_t>> cand;
    cand.reserve(m * (m - 1) / 2);
    for (size_t j = 1; j < m; ++j)
        for (size_t k = 0; k < j; ++k) cand.emplace_back(j, k, (uint64_t)sim[j * (j - 1) / 2 + k]);
    auto dist = [](size_t a, size_t b) { return a > b ? a - b : b - a; };
    std::sort(cand.begin(), cand.end(), [&](const auto &f, const auto &g) {
        return std::get<2>(f) > std::get<2>(g) ||
               (std::get<2>(f) == std::get<2>(g) &&
                dist(std::get<0>(f), std::get<1>(f)) < dist(std::get<0>(g), std::get<1>(g)));
    });
    std::vector<std::vector<size_t>> groups;
    groups.reserve((m + 1) / 2);
    std::vector<bool> matched(m, false);
    for (const auto &c : cand) {
        const size_t i = std::get<0>(c), j = std::get<1>(c);
        if (!matched[i] && !matched[j]) {
            matched[i] = matched[j] = true;
            groups.push_back({i, j});
        }
    }
    for (size_t i = 0; i < m; ++i)
        if (!matched[i]) groups.push_back({i});
    return groups;
}

// ---- BRWTOptimizer::relax (BRWT_builders.cpp:166-297) ----------------------
//
// reassign (:257-297) moves a pruned node's children up to its parent: a
// grandchild's index column, defined over the pruned node's set positions,
// becomes a column over the pruned node's own positions -- a parallel bit
// deposit (pdep) of the grandchild's bits into the set bits of the pruned
// node's index, word by word at the exclusive prefix of its popcounts.  All
// grandchildren of one pruned node are expanded by one launch (grid y).
struct ExpandArgs {
    const uint64_t *node;              // the pruned node's index column (Wn words)
    const unsigned long long *pre;     // [Wn + 1] exclusive prefix of its word popcounts
    const uint64_t *const *grand;      // [k] grandchild index columns (ceil(ones/64) words)
    uint64_t *const *out;              // [k] expanded columns (Wn words)
    uint64_t Wn, ones;
};

__global__ __launch_bounds__(256) void k_popc_words(const uint64_t *__restrict__ v, uint64_t W,
                                                    unsigned long long *__restrict__ popc) {
    for (uint64_t w = blockIdx.x * 256ull + threadIdx.x; w < W; w += gridDim.x * 256ull) popc[w] = __popcll(v[w]);
}

__global__ __launch_bounds__(256) void k_expand(ExpandArgs A) {
    const uint64_t *g = A.grand[blockIdx.y];
    uint64_t *o = A.out[blockIdx.y];
    const uint64_t gw = (A.ones + 63) / 64;
    for (uint64_t w = blockIdx.x * 256ull + threadIdx.x; w < A.Wn; w += gridDim.x * 256ull) {
        uint64_t bits = A.node[w];
        const uint64_t base = A.pre[w], q = base >> 6, r = base & 63;
        // the grandchild's bits [base, base + popc) from bit 0
        uint64_t src = q < gw ? g[q] >> r : 0;
        if (r && q + 1 < gw) src |= g[q + 1] << (64 - r);
        uint64_t res = 0;
        while (bits) {
            const uint64_t low = bits & (~bits + 1);
            if (src & 1) res |= low;
            src >>= 1;
            bits ^= low;
        }
        o[w] = res;
    }
}

// sizeof(bit_vector_rrr<63>) * 8 in bv_space_taken_rrr (:315-321): sdsl is
// absent, so the struct size is the oracle's estimate (oracle/brwt_oracle.cpp
// kRRRObjectBits; parity unpinned against sdsl, pinned against the oracle --
// it only moves the prune decision, never the query results)
constexpr double kRRRObjectBits = 184 * 8;

double logbinomial(uint64_t n, uint64_t k) {  // :299-303
    return (lgamma(n + 1) - lgamma(k + 1) - lgamma(n - k + 1)) / log(2);
}
double bv_space_taken_rrr63(uint64_t size, uint64_t ones) {  // :315-321, block 63
    return logbinomial(size, ones) + std::ceil(log2(63 + 1) / 63) * size + kRRRObjectBits;
}

uint64_t popcount_words(const std::vector<uint64_t> &v, uint64_t len) {
    uint64_t c = 0;
    for (uint64_t w = 0; w < (len + 63) / 64 && w < v.size(); ++w) c += __builtin_popcountll(v[w]);
    return c;
}

int relax_nodes(std::vector<BNode> &nodes, uint32_t root, uint64_t max_arity, hipStream_t s) {
    std::vector<uint64_t> ones(nodes.size());
    for (size_t u = 0; u < nodes.size(); ++u) ones[u] = popcount_words(nodes[u].index, nodes[u].index_len);
    // pruning_delta (:351-380)
    auto delta = [&](uint32_t u) {
        double d = 0;
        for (uint32_t c : nodes[u].children) {
            d += bv_space_taken_rrr63(nodes[u].index_len, ones[c]);
            d -= bv_space_taken_rrr63(nodes[c].index_len, ones[c]);
        }
        return d - bv_space_taken_rrr63(nodes[u].index_len, ones[u]);
    };
    // reassign (:257-297) on the device
    auto reassign = [&](uint32_t u) -> int {
        BNode &node = nodes[u];
        const uint64_t Wn = (node.index_len + 63) / 64, k = node.children.size();
        if (!Wn) {
            for (uint32_t c : node.children) {
                nodes[c].index.assign(1, 0);
                nodes[c].index_len = 0;
            }
            return MBRWT_OK;
        }
        uint64_t gwords = 0;
        for (uint32_t c : node.children) gwords += std::max<uint64_t>(1, nodes[c].index.size());
        const size_t bytes = (Wn + 2 * (Wn + 1) + gwords + k * Wn + 2 * k) * sizeof(uint64_t);
        void *arena = nullptr;
        if (hipMalloc(&arena, bytes) != hipSuccess) return hip_fail(hipErrorOutOfMemory, "relax allocation");
        uint64_t *d_node = reinterpret_cast<uint64_t *>(arena);
        unsigned long long *d_popc = reinterpret_cast<unsigned long long *>(d_node + Wn);
        unsigned long long *d_pre = d_popc + Wn + 1;
        uint64_t *d_grand = reinterpret_cast<uint64_t *>(d_pre + Wn + 1);
        uint64_t *d_out = d_grand + gwords;
        uint64_t **d_tab = reinterpret_cast<uint64_t **>(d_out + k * Wn);
        std::vector<uint64_t *> tab(2 * k);
        int rc = MBRWT_OK;
        void *d_scan = nullptr;
        do {
            if (hipMemcpyAsync(d_node, node.index.data(), Wn * 8, hipMemcpyHostToDevice, s) != hipSuccess) break;
            uint64_t at = 0;
            for (uint64_t i = 0; i < k; ++i) {
                const auto &gi = nodes[node.children[i]].index;
                tab[i] = d_grand + at;
                tab[k + i] = d_out + i * Wn;
                if (!gi.empty() &&
                    hipMemcpyAsync(d_grand + at, gi.data(), gi.size() * 8, hipMemcpyHostToDevice, s) != hipSuccess)
                    rc = MBRWT_ERR_DEVICE;
                at += std::max<uint64_t>(1, gi.size());
            }
            if (rc) break;
            if (hipMemcpyAsync(d_tab, tab.data(), 2 * k * 8, hipMemcpyHostToDevice, s) != hipSuccess) break;
            hipLaunchKernelGGL(k_popc_words, dim3(grid_of(Wn)), dim3(256), 0, s, d_node, Wn, d_popc);
            if (hipMemsetAsync(d_popc + Wn, 0, 8, s) != hipSuccess) break;
            size_t scan_bytes = 0;
            if (hipcub::DeviceScan::ExclusiveSum(nullptr, scan_bytes, d_popc, d_pre, (int)(Wn + 1), s) != hipSuccess ||
                hipMalloc(&d_scan, scan_bytes + 16) != hipSuccess ||
                hipcub::DeviceScan::ExclusiveSum(d_scan, scan_bytes, d_popc, d_pre, (int)(Wn + 1), s) != hipSuccess)
                break;
            ExpandArgs A{d_node, d_pre, d_tab, d_tab + k, Wn, ones[u]};
            for (uint64_t y0 = 0; y0 < k; y0 += 65535) {
                ExpandArgs B = A;
                B.grand = d_tab + y0;
                B.out = d_tab + k + y0;
                const uint32_t ny = (uint32_t)std::min<uint64_t>(65535, k - y0);
                hipLaunchKernelGGL(k_expand, dim3(grid_of(Wn, ny), ny), dim3(256), 0, s, B);
            }
            if (hipGetLastError() != hipSuccess) break;
            for (uint64_t i = 0; i < k; ++i) {
                BNode &gc = nodes[node.children[i]];
                gc.index.assign(Wn, 0);
                gc.index_len = node.index_len;
                if (hipMemcpyAsync(gc.index.data(), d_out + i * Wn, Wn * 8, hipMemcpyDeviceToHost, s) != hipSuccess)
                    rc = MBRWT_ERR_DEVICE;
            }
            if (rc) break;
            if (hipStreamSynchronize(s) != hipSuccess) break;
            (void)hipFree(d_scan);
            (void)hipFree(arena);
            return MBRWT_OK;
        } while (false);
        (void)hipFree(d_scan);
        (void)hipFree(arena);
        set_error("relax: HIP error while expanding index columns");
        return MBRWT_ERR_DEVICE;
    };
    // parents in BFT order, pushed to the front: leaves' parents first, root last (:171-179)
    std::vector<uint32_t> bft{root};
    for (size_t h = 0; h < bft.size(); ++h)
        for (uint32_t c : nodes[bft[h]].children) bft.push_back(c);
    for (auto it = bft.rbegin(); it != bft.rend(); ++it) {
        BNode &parent = nodes[*it];
        if (parent.children.empty()) continue;
        const std::vector<uint32_t> old = parent.children;
        std::vector<uint32_t> updated;
        const uint64_t nchild = old.size();
        for (uint64_t g = 0; g < nchild; ++g) {
            const uint32_t c = old[g];
            // add_submatrix (:213-255): the arity budget left for this child
            const uint64_t used = updated.size() + nchild - g - 1;
            const uint64_t max_delta = max_arity - std::min<uint64_t>(max_arity, used);
            bool prune = !nodes[c].children.empty();
            if (prune && nodes[c].children.size() > max_delta) prune = false;
            if (!prune || delta(c) > 0) {
                updated.push_back(c);
            } else {
                int rc = reassign(c);
                if (rc) return rc;
                for (uint32_t gc : nodes[c].children) updated.push_back(gc);
                nodes[c].children.clear();
                nodes[c].index.clear();
            }
        }
        nodes[*it].children = std::move(updated);
    }
    return MBRWT_OK;
}

// breadth-first numbering of the node tree (mbrwt_tree_desc) and the image
int desc_from_nodes(const std::vector<BNode> &nodes, uint32_t root, uint64_t n, uint64_t m, const DescSink &emit) {
    std::vector<uint32_t> order{root};
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
    return emit(desc);
}

}  // namespace

int build_from_columns(const mbrwt_columns_desc &cd, int device, Tree &tree, hipStream_t s,
                       uint64_t relax_max_arity) {
    if (cd.num_rows > kMaxRows) {  // (the caller routes these through desc_from_columns + the sharded create)
        set_error("num_rows >= 2^32: build through the row-sharded path");
        return MBRWT_ERR_UNSUPPORTED;
    }
    return desc_from_columns(cd, device, s, relax_max_arity,
                             [&](const mbrwt_tree_desc &d) { return build_from_desc(d, device, tree); });
}

int desc_from_columns(const mbrwt_columns_desc &cd, int device, hipStream_t s, uint64_t relax_max_arity,
                      const DescSink &emit) {
    MBRWT_HIP(hipSetDevice(device));
    const uint64_t n = cd.num_rows, m = cd.num_columns;
    const bool greedy = build_partitioner() == MBRWT_PARTITIONER_GREEDY;
    if (!greedy && (cd.arity < 2 || cd.arity > kMaxArity)) {
        set_error("arity must be in [2, 64]");
        return MBRWT_ERR_INVALID;
    }
    if (m && !cd.columns) {
        set_error("null column array");
        return MBRWT_ERR_INVALID;
    }
    if (m > 0xFFFFFFFFull) {
        set_error("num_columns >= 2^32 is not supported by this build");
        return MBRWT_ERR_UNSUPPORTED;
    }
    if (m == 0) {  // BRWTBottomUpBuilder::build of no columns is BRWT() (BRWT_builders.cpp:122-123)
        mbrwt_tree_desc empty{};
        return emit(empty);
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
    // greedy: the row sample (the same every level: seed 1 each call) and its words
    std::vector<uint64_t> sample;
    uint64_t *d_sample = nullptr;
    const bool sample_all = greedy && n <= 1000000;  // every row, in order: the columns themselves
    if (greedy && !sample_all) {
        sample = greedy_sample_rows(n);
        d_sample = reinterpret_cast<uint64_t *>(dalloc(sample.size() * sizeof(uint64_t)));
        if (!d_sample) {
            cleanup();
            return hip_fail(hipErrorOutOfMemory, "builder allocation");
        }
        MBRWT_HIP(hipMemcpyAsync(d_sample, sample.data(), sample.size() * sizeof(uint64_t), hipMemcpyHostToDevice, s));
    }
    const uint64_t ns = sample_all ? n : sample.size(), SW = (ns + 63) / 64;
    double t_sim_ms = 0, t_sort_ms = 0;
    while (level.size() > 1) {  // BRWT_builders.cpp:134-158
        // the partition of this level: the basic partitioner's consecutive
        // groups (:20-31) or the greedy pairs; singletons pass through (:75-77)
        std::vector<std::vector<size_t>> part;
        if (!greedy) {
            for (size_t g0 = 0; g0 < level.size(); g0 += cd.arity) {
                std::vector<size_t> grp;
                for (size_t i = g0; i < std::min<size_t>(level.size(), g0 + cd.arity); ++i) grp.push_back(i);
                part.push_back(std::move(grp));
            }
        } else {
            const size_t L = level.size();
            if ((uint64_t)L * (L - 1) / 2 > (1ull << 31)) {
                // the reference keeps every pair as a candidate too
                // (partitionings.cpp:154-160): > 2^31 pairs is > 50 GB of host
                // candidates -- refuse instead of exhausting the host
                cleanup();
                set_error("greedy partitioner: more than 65,536 columns on one level");
                return MBRWT_ERR_UNSUPPORTED;
            }
            const auto t0 = std::chrono::steady_clock::now();
            // the level's columns (pointer table), the sampled words, the products
            std::vector<const uint64_t *> hp(L);
            for (size_t i = 0; i < L; ++i) hp[i] = nodes[level[i]].rowcol;
            const uint64_t **d_ptr = reinterpret_cast<const uint64_t **>(dalloc(L * sizeof(void *) * 2));
            uint64_t *d_sub = sample_all ? nullptr : reinterpret_cast<uint64_t *>(dalloc(L * SW * sizeof(uint64_t)));
            const uint64_t npairs = (uint64_t)L * (L - 1) / 2;
            uint32_t *d_sim = reinterpret_cast<uint32_t *>(dalloc(npairs * sizeof(uint32_t)));
            if (!d_ptr || (!sample_all && !d_sub) || !d_sim) {
                cleanup();
                return hip_fail(hipErrorOutOfMemory, "builder allocation");
            }
            MBRWT_HIP(hipMemcpyAsync(d_ptr, hp.data(), L * sizeof(void *), hipMemcpyHostToDevice, s));
            const uint64_t *const *simcols = d_ptr;
            if (!sample_all) {
                for (uint32_t y0 = 0; y0 < L; y0 += 65535) {
                    const uint32_t ny = (uint32_t)std::min<size_t>(65535, L - y0);
                    hipLaunchKernelGGL(k_gather_sample, dim3(grid_of(SW, ny), ny), dim3(256), 0, s, d_ptr + y0,
                                       (const uint64_t *)d_sample, ns, SW, d_sub + (uint64_t)y0 * SW);
                }
                MBRWT_HIP(hipGetLastError());
                std::vector<const uint64_t *> hs(L);
                for (size_t i = 0; i < L; ++i) hs[i] = d_sub + i * SW;
                MBRWT_HIP(hipMemcpyAsync(d_ptr + L, hs.data(), L * sizeof(void *), hipMemcpyHostToDevice, s));
                simcols = d_ptr + L;
            }
            const uint64_t T = (L + kSimTile - 1) / kSimTile, tiles = T * (T + 1) / 2;
            if (tiles > 0x7FFFFFFFull) {
                cleanup();
                set_error("too many columns for the greedy partitioner");
                return MBRWT_ERR_UNSUPPORTED;
            }
            hipLaunchKernelGGL(k_similarity, dim3((unsigned)tiles), dim3(256), 0, s, simcols, (uint32_t)L, SW, d_sim);
            MBRWT_HIP(hipGetLastError());
            std::vector<uint32_t> sim(npairs);
            MBRWT_HIP(hipMemcpyAsync(sim.data(), d_sim, npairs * sizeof(uint32_t), hipMemcpyDeviceToHost, s));
            MBRWT_HIP(hipStreamSynchronize(s));
            const auto t1 = std::chrono::steady_clock::now();
            part = greedy_groups(sim, L);
            const auto t2 = std::chrono::steady_clock::now();
            t_sim_ms += std::chrono::duration<double, std::milli>(t1 - t0).count();
            t_sort_ms += std::chrono::duration<double, std::milli>(t2 - t1).count();
            dfree(d_sim);
            if (d_sub) dfree(d_sub);
            dfree(d_ptr);
        }
        std::vector<uint32_t> next, gchild{0}, child_group, child_node;
        std::vector<size_t> group_slot;  // position in `next` of each parent
        for (const auto &grp : part) {
            const size_t g0 = grp[0];
            if (grp.size() == 1) {
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
            for (const size_t i : grp) {  // (the group's order: the reference's child order)
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

    if (relax_max_arity > 1 && !root.children.empty()) {  // BRWTOptimizer::relax (:166-211)
        const int rr = relax_nodes(nodes, level[0], relax_max_arity, s);
        if (rr) return rr;
    }
    const auto t_index = std::chrono::steady_clock::now();
    const int rc = desc_from_nodes(nodes, level[0], n, m, emit);
    if (const char *e = std::getenv("MBRWT_BUILD_TIMING"); e && e[0] == '1') {
        const auto t_end = std::chrono::steady_clock::now();
        std::fprintf(stderr, "[mbrwt build] index columns %.1f ms (greedy: similarities %.1f ms, sort + matching "
                     "%.1f ms), image layout %.1f ms\n",
                     std::chrono::duration<double, std::milli>(t_index - t_start).count(), t_sim_ms, t_sort_ms,
                     std::chrono::duration<double, std::milli>(t_end - t_index).count());
    }
    return rc;
}

// BRWTOptimizer::relax(brwt, max_arity) (`annograph relax_brwt`,
// main.cpp:746) on a tree description: the BFS tree becomes a node tree, the
// relax above runs, and the relaxed tree becomes the image.
int build_relaxed_from_desc(const mbrwt_tree_desc &desc, uint64_t max_arity, int device, Tree &tree, hipStream_t s) {
    return relaxed_desc(desc, max_arity, device, s,
                        [&](const mbrwt_tree_desc &d) { return build_from_desc(d, device, tree); });
}

int relaxed_desc(const mbrwt_tree_desc &desc, uint64_t max_arity, int device, hipStream_t s, const DescSink &emit) {
    MBRWT_HIP(hipSetDevice(device));
    const uint32_t N = desc.num_nodes;
    if (N && (!desc.num_children || !desc.first_child || !desc.leaf_column || !desc.vec_size || !desc.vec_words)) {
        set_error("null array in the tree description");
        return MBRWT_ERR_INVALID;
    }
    if (!N || max_arity <= 1) return emit(desc);
    std::vector<BNode> nodes(N);
    for (uint32_t u = 0; u < N; ++u) {
        const uint32_t k = desc.num_children[u];
        if (k && ((uint64_t)desc.first_child[u] + k > N || desc.first_child[u] <= u)) {
            set_error("tree description: children out of range");
            return MBRWT_ERR_INVALID;
        }
        for (uint32_t i = 0; i < k; ++i) nodes[u].children.push_back(desc.first_child[u] + i);
        nodes[u].column = k ? UINT32_MAX : desc.leaf_column[u];
        nodes[u].index_len = desc.vec_size[u];
        const uint64_t w = (desc.vec_size[u] + 63) / 64;
        if (w && !desc.vec_words[u]) {
            set_error("tree description: null index column");
            return MBRWT_ERR_INVALID;
        }
        nodes[u].index.assign(std::max<uint64_t>(w, 1), 0);
        if (w) std::copy(desc.vec_words[u], desc.vec_words[u] + w, nodes[u].index.begin());
        if (desc.vec_size[u] & 63) nodes[u].index[w - 1] &= (1ull << (desc.vec_size[u] & 63)) - 1;
    }
    const int rc = relax_nodes(nodes, 0, max_arity, s);
    if (rc) return rc;
    return desc_from_nodes(nodes, 0, desc.num_rows, desc.num_columns, emit);
}

}  // namespace mbrwt
