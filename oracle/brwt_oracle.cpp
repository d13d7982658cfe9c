// brwt_oracle.cpp -- CPU restatement of the reference BRWT / Multi-BRWT path.
//
// TEST INFRASTRUCTURE ONLY: the checker for the HIP product path and the
// CPU baseline of bench.py.  Nothing in genome_graph_annotation_amd/ links it.
//
// Restates (reference paths, read-only at /root/reference):
//   common/bit_vector.{hpp,cpp}       rank1 (inclusive, clamped), select1 (1-based), access
//   common/utils.{hpp,cpp}            RangePartition, sample_indexes
//   annotation/hierarchical_annotation/BRWT.cpp            get / get_row / get_column / stats
//   annotation/hierarchical_annotation/BRWT_builders.cpp   bottom-up build, basic partitioner, relax
//   annotation/hierarchical_annotation/partitionings.cpp   greedy binary grouping
//   experiments/data_generation.cpp, experiments/main.cpp  synthetic matrices and query sampling
// The reference itself cannot be compiled here (sdsl-lite/libmaus2 submodules
// are empty), so this restatement is pinned by the reference's
// own known-answer tests (tests/test_oracle_kats.py).
//
// Parity notes: the sdsl-RRR encoding is replaced by plain bit vectors with
// rank samples -- identical logical rank/select/access results (the reference
// tests only the logical results, tests/test_bit_vector.cpp:19-94).

#include "brwt_oracle.h"

#include <algorithm>
#include <array>
#include <cassert>
#include <cmath>
#include <cstring>
#include <deque>
#include <functional>
#include <limits>
#include <memory>
#include <numeric>
#include <queue>
#include <random>
#include <stdexcept>
#include <tuple>
#include <vector>

#ifdef _OPENMP
#include <omp.h>
#endif

namespace {

inline uint64_t popcnt64(uint64_t x) { return (uint64_t)__builtin_popcountll(x); }

// ------------------------------------------------------------------------
// Plain bit vector with 512-bit rank samples.  Semantics of the reference's
// bit_vector interface (common/bit_vector.hpp:12-45):
//   rank1(id)   = #ones in [0, id], clamped to the total for id >= size
//                 (bit_vector.cpp:857-861)
//   select1(i)  = position of the i-th one, i is 1-based (bit_vector.hpp:19-20)
// ------------------------------------------------------------------------
struct BitVec {
    uint64_t size = 0;
    std::vector<uint64_t> words;  // LSB-first
    std::vector<uint64_t> super;  // ones before each 8-word superblock
    uint64_t ones = 0;

    BitVec() = default;
    explicit BitVec(uint64_t n, bool value = false) : size(n), words((n + 63) / 64, value ? ~0ull : 0ull) {
        clear_tail();
    }

    void clear_tail() {
        if (size & 63) words.back() &= (1ull << (size & 63)) - 1;
    }
    bool get(uint64_t i) const { return (words[i >> 6] >> (i & 63)) & 1; }
    void set(uint64_t i) { words[i >> 6] |= 1ull << (i & 63); }

    void finalize() {
        clear_tail();
        super.assign(words.size() / 8 + 2, 0);
        uint64_t acc = 0;
        for (size_t w = 0; w < words.size(); ++w) {
            if ((w & 7) == 0) super[w >> 3] = acc;
            acc += popcnt64(words[w]);
        }
        super[(words.size() + 7) / 8] = acc;
        ones = acc;
    }

    // inclusive rank, clamped (bit_vector.cpp:857-861)
    uint64_t rank1(uint64_t id) const {
        if (id >= size) return ones;
        uint64_t w = id >> 6;
        uint64_t r = super[w >> 3];
        for (uint64_t k = w & ~7ull; k < w; ++k) r += popcnt64(words[k]);
        uint64_t b = id & 63;
        uint64_t m = (b == 63) ? ~0ull : ((2ull << b) - 1);
        return r + popcnt64(words[w] & m);
    }

    // 1-based select (bit_vector.cpp:863-869); precondition 1 <= i <= ones
    uint64_t select1(uint64_t i) const {
        assert(i >= 1 && i <= ones);
        // binary search the last superblock with super[s] < i
        size_t lo = 0, hi = (words.size() + 7) / 8;  // super[hi] == ones >= i
        while (hi - lo > 1) {
            size_t mid = (lo + hi) / 2;
            if (super[mid] < i) lo = mid; else hi = mid;
        }
        uint64_t need = i - super[lo];
        for (size_t w = lo * 8; w < words.size(); ++w) {
            uint64_t c = popcnt64(words[w]);
            if (need <= c) {
                uint64_t x = words[w];
                for (uint64_t k = 1; k < need; ++k) x &= x - 1;
                return w * 64 + (uint64_t)__builtin_ctzll(x);
            }
            need -= c;
        }
        throw std::logic_error("select1 out of range");
    }

    template <class F>
    void call_ones(F &&f) const {
        for (size_t w = 0; w < words.size(); ++w) {
            uint64_t x = words[w];
            while (x) {
                f(w * 64 + (uint64_t)__builtin_ctzll(x));
                x &= x - 1;
            }
        }
    }
};

// ------------------------------------------------------------------------
// utils::RangePartition (common/utils.hpp:440-479, utils.cpp:621-691)
// ------------------------------------------------------------------------
struct RangePartition {
    std::vector<std::vector<uint32_t>> partition;
    std::vector<uint32_t> groups, ranks;

    RangePartition() = default;
    RangePartition(const std::vector<uint64_t> &arrangement, const std::vector<size_t> &group_sizes) {
        size_t offset = 0;
        for (size_t gs : group_sizes) {
            partition.emplace_back(arrangement.begin() + offset, arrangement.begin() + offset + gs);
            offset += gs;
        }
        if (!initialize()) throw std::logic_error("invalid RangePartition");
    }
    bool initialize() {  // utils.cpp:651-677
        uint64_t n = 0;
        for (auto &g : partition) {
            if (g.empty()) return false;
            n += g.size();
        }
        groups.assign(n, UINT32_MAX);
        ranks.assign(n, UINT32_MAX);
        for (size_t g = 0; g < partition.size(); ++g) {
            for (size_t i = 0; i < partition[g].size(); ++i) {
                uint32_t v = partition[g][i];
                if (v >= n || groups[v] != UINT32_MAX) return false;
                groups[v] = (uint32_t)g;
                ranks[v] = (uint32_t)i;
            }
        }
        return true;
    }
    uint32_t group(uint32_t v) const { return groups[v]; }       // utils.cpp:679-682
    uint32_t rank(uint32_t v) const { return ranks[v]; }         // utils.cpp:684-687
    uint32_t get(uint32_t g, uint32_t r) const { return partition[g][r]; }  // utils.cpp:689-691
    uint64_t num_groups() const { return partition.size(); }
    uint64_t size() const { return ranks.size(); }
};

// ------------------------------------------------------------------------
// sdsl-RRR-like bit vector (the cost model of the reference's
// bit_vector_rrr<63>, common/bit_vector.cpp:857-888 over sdsl::rrr_vector<63>):
// 63-bit blocks stored as {class = popcount (6 bits), the block's number
// among the blocks of its class (ceil(log2 C(63, class)) bits)}, a rank and a
// number-pointer sample every 32 blocks.  operator[] / rank1 walk the classes
// since the sample and decode ONE block by the combinatorial number system --
// the work an sdsl access does.  Only the CPU baseline uses it (timing); its
// answers are checked against the plain vector in the KAT tests.
// ------------------------------------------------------------------------
struct RRRVec {
    static constexpr uint32_t B = 63, K = 32;
    uint64_t size = 0, ones = 0;
    std::vector<uint8_t> cls;
    std::vector<uint64_t> nums, srank, sptr;

    struct Tables {
        uint64_t C[B + 1][B + 1];
        uint8_t space[B + 1];
        Tables() {
            std::memset(C, 0, sizeof(C));
            for (uint32_t n = 0; n <= B; ++n) {
                C[n][0] = 1;
                for (uint32_t k = 1; k <= n; ++k) C[n][k] = C[n - 1][k - 1] + (k < n ? C[n - 1][k] : 0);
            }
            for (uint32_t k = 0; k <= B; ++k)
                space[k] = C[B][k] <= 1 ? 0 : (uint8_t)(64 - __builtin_clzll(C[B][k] - 1));
        }
    };
    static const Tables &T() {
        static const Tables t;
        return t;
    }
    static uint64_t getbits(const std::vector<uint64_t> &w, uint64_t pos, uint32_t len) {
        if (!len) return 0;
        const uint64_t i = pos >> 6, o = pos & 63;
        uint64_t v = w[i] >> o;
        if (o && o + len > 64) v |= w[i + 1] << (64 - o);
        return len == 64 ? v : v & ((1ull << len) - 1);
    }
    static void setbits(std::vector<uint64_t> &w, uint64_t pos, uint32_t len, uint64_t v) {
        if (!len) return;
        const uint64_t i = pos >> 6, o = pos & 63;
        w[i] |= v << o;
        if (o && o + len > 64) w[i + 1] |= v >> (64 - o);
    }

    explicit RRRVec(const BitVec &bv) : size(bv.size), ones(bv.ones) {
        const Tables &t = T();
        const uint64_t nb = (size + B - 1) / B;
        cls.resize(nb);
        std::vector<uint64_t> blk(nb);
        uint64_t bits = 0;
        for (uint64_t b = 0; b < nb; ++b) {
            const uint64_t p = b * B;
            const uint32_t len = (uint32_t)std::min<uint64_t>(B, size - p);
            uint64_t x = bv.words[p >> 6] >> (p & 63);
            if ((p & 63) && (p & 63) + len > 64) x |= bv.words[(p >> 6) + 1] << (64 - (p & 63));
            x &= (len == 64 ? ~0ull : ((1ull << len) - 1));
            blk[b] = x;
            cls[b] = (uint8_t)__builtin_popcountll(x);
            bits += t.space[cls[b]];
        }
        nums.assign(bits / 64 + 2, 0);
        srank.resize(nb / K + 2);
        sptr.resize(nb / K + 2);
        uint64_t pos = 0, r = 0;
        for (uint64_t b = 0; b < nb; ++b) {
            if (b % K == 0) {
                srank[b / K] = r;
                sptr[b / K] = pos;
            }
            // number of the block among the blocks of its class (LSB first)
            uint64_t x = blk[b], nr = 0;
            uint32_t k = cls[b], nn = B;
            while (x) {
                if (x & 1) nr += t.C[nn - 1][k--];
                x >>= 1;
                --nn;
            }
            setbits(nums, pos, t.space[cls[b]], nr);
            pos += t.space[cls[b]];
            r += cls[b];
        }
    }
    // bits [0, o] of block b, decoded from its number (LSB first, stopping
    // after position o as sdsl's decode_bit / decode_popcount do); *rank_before
    // = ones before the block (sample + the classes walked since it)
    uint64_t block_prefix(uint64_t b, uint32_t o, uint64_t *rank_before) const {
        const Tables &t = T();
        const uint64_t s = b / K;
        uint64_t pos = sptr[s], r = srank[s];
        for (uint64_t j = s * K; j < b; ++j) {
            pos += t.space[cls[j]];
            r += cls[j];
        }
        if (rank_before) *rank_before = r;
        uint32_t k = cls[b];
        const uint64_t upto = o == 63 ? ~0ull : ((2ull << o) - 1);
        if (k == 0) return 0;
        if (k == B) return ((1ull << B) - 1) & upto;
        uint64_t nr = getbits(nums, pos, t.space[k]), x = 0;
        for (uint32_t p = 0, nn = B; k && p <= o; ++p, --nn) {
            const uint64_t c = t.C[nn - 1][k];
            if (nr >= c) {
                x |= 1ull << p;
                nr -= c;
                --k;
            }
        }
        return x;
    }
    bool get(uint64_t i) const {
        const uint32_t o = (uint32_t)(i % B);
        return (block_prefix(i / B, o, nullptr) >> o) & 1;
    }
    uint64_t rank1(uint64_t i) const {  // inclusive, clamped (bit_vector.cpp:857-861)
        if (i >= size) return ones;
        uint64_t r = 0;
        const uint64_t x = block_prefix(i / B, (uint32_t)(i % B), &r);
        return r + (uint64_t)__builtin_popcountll(x);
    }
};

// ------------------------------------------------------------------------
// BRWT node (annotation/hierarchical_annotation/BRWT.hpp:18-61)
// ------------------------------------------------------------------------
struct Node {
    RangePartition assignments;
    BitVec nonzero_rows;
    std::unique_ptr<RRRVec> rrr;  // set by to_rrr(): the index held RRR-like (CPU baseline)
    std::vector<std::unique_ptr<Node>> children;

    uint64_t num_columns() const { return assignments.size(); }
    uint64_t num_rows() const { return nonzero_rows.size; }
    bool bit(uint64_t i) const { return rrr ? rrr->get(i) : nonzero_rows.get(i); }
    uint64_t rank(uint64_t i) const { return rrr ? rrr->rank1(i) : nonzero_rows.rank1(i); }

    // BRWT::get (BRWT.cpp:9-24)
    bool get(uint64_t row, uint64_t col) const {
        if (!bit(row)) return false;
        if (children.empty()) return true;
        uint32_t g = assignments.group((uint32_t)col);
        return children[g]->get(rank(row) - 1, assignments.rank((uint32_t)col));
    }

    // BRWT::get_row (BRWT.cpp:26-53), appending to `out` in the reference's
    // order; child-local column ids are remapped in place through
    // assignments_.get(i, col) exactly as BRWT.cpp:48-50 does.
    void get_row(uint64_t row, std::vector<uint32_t> &out, uint64_t &visits) const {
        ++visits;                                  // nonzero_rows_[row], BRWT.cpp:30
        if (!bit(row)) return;
        if (children.empty()) {                    // BRWT.cpp:34-39
            out.push_back(0);
            return;
        }
        uint64_t j = rank(row) - 1;                // BRWT.cpp:43
        for (size_t i = 0; i < children.size(); ++i) {
            size_t start = out.size();
            children[i]->get_row(j, out, visits);
            for (size_t k = start; k < out.size(); ++k)
                out[k] = assignments.get((uint32_t)i, out[k]);
        }
    }

    // BRWT::get_column (BRWT.cpp:55-85)
    std::vector<uint64_t> get_column(uint64_t col) const {
        uint64_t nnz = nonzero_rows.ones;
        if (!nnz) return {};
        if (children.empty()) {
            std::vector<uint64_t> r;
            r.reserve(nnz);
            nonzero_rows.call_ones([&](uint64_t i) { r.push_back(i); });
            return r;
        }
        uint32_t g = assignments.group((uint32_t)col);
        auto rows = children[g]->get_column(assignments.rank((uint32_t)col));
        if (nnz == nonzero_rows.size) return rows;
        for (auto &r : rows) r = nonzero_rows.select1(r + 1);
        return rows;
    }

    // BRWT::num_relations (BRWT.cpp:130-140)
    uint64_t num_relations() const {
        if (children.empty()) return nonzero_rows.ones;
        uint64_t s = 0;
        for (auto &c : children) s += c->num_relations();
        return s;
    }

    // BRWT::BFT (BRWT.cpp:204-220)
    void bft(const std::function<void(const Node &)> &cb) const {
        std::queue<const Node *> q;
        q.push(this);
        while (!q.empty()) {
            const Node *n = q.front();
            q.pop();
            cb(*n);
            for (auto &c : n->children) q.push(c.get());
        }
    }
};

using VectorsPtr = std::vector<std::unique_ptr<BitVec>>;
using Group = std::vector<uint64_t>;
using Partition = std::vector<Group>;
using Partitioner = std::function<Partition(const VectorsPtr &)>;

struct NodeBRWT {  // BRWT_builders.hpp:23-32
    std::vector<uint64_t> column_arrangement;
    std::vector<size_t> group_sizes;
    std::vector<std::unique_ptr<Node>> child_nodes;
};

// BRWTBuilder::initialize (BRWT_builders.cpp:7-18)
std::unique_ptr<Node> initialize(NodeBRWT &&node, BitVec &&nonzero_rows) {
    auto n = std::make_unique<Node>();
    n->assignments = RangePartition(node.column_arrangement, node.group_sizes);
    n->nonzero_rows = std::move(nonzero_rows);
    n->nonzero_rows.finalize();
    n->children = std::move(node.child_nodes);
    return n;
}

// get_basic_partitioner (BRWT_builders.cpp:20-31)
Partitioner basic_partitioner(size_t arity) {
    return [arity](const VectorsPtr &vectors) {
        Partition p((vectors.size() + arity - 1) / arity);
        for (size_t i = 0; i < vectors.size(); ++i) p[i / arity].push_back(i);
        return p;
    };
}

// compute_or (BRWT_builders.cpp:33-49)
BitVec compute_or(const std::vector<BitVec *> &cols) {
    BitVec r(cols.at(0)->size);
    for (auto *c : cols)
        for (size_t w = 0; w < r.words.size(); ++w) r.words[w] |= c->words[w];
    return r;
}

// generate_subindex (BRWT_builders.cpp:51-66)
BitVec generate_subindex(const BitVec &column, const BitVec &reference) {
    uint64_t cnt = 0;
    for (auto w : reference.words) cnt += popcnt64(w);
    BitVec sub(cnt);
    uint64_t j = 0;
    reference.call_ones([&](uint64_t i) {
        if (column.get(i)) sub.set(j);
        ++j;
    });
    return sub;
}

// BRWTBottomUpBuilder::merge (BRWT_builders.cpp:68-107)
std::pair<NodeBRWT, std::unique_ptr<BitVec>> merge(std::vector<NodeBRWT> &&nodes, VectorsPtr &&index) {
    if (nodes.size() == 1) return {std::move(nodes[0]), std::move(index[0])};  // :74-76 pass-through
    NodeBRWT parent;
    std::vector<BitVec *> raw;
    for (auto &p : index) raw.push_back(p.get());
    BitVec parent_index = compute_or(raw);
    for (size_t i = 0; i < nodes.size(); ++i) {
        parent.column_arrangement.insert(parent.column_arrangement.end(),
                                         nodes[i].column_arrangement.begin(),
                                         nodes[i].column_arrangement.end());
        parent.group_sizes.push_back(nodes[i].column_arrangement.size());
        std::iota(nodes[i].column_arrangement.begin(), nodes[i].column_arrangement.end(), 0);
        BitVec shrinked = generate_subindex(*index[i], parent_index);
        index[i].reset();
        parent.child_nodes.emplace_back(initialize(std::move(nodes[i]), std::move(shrinked)));
    }
    return {std::move(parent), std::make_unique<BitVec>(std::move(parent_index))};
}

// BRWTBottomUpBuilder::build (BRWT_builders.cpp:122-163)
std::unique_ptr<Node> build(VectorsPtr &&columns, const Partitioner &partitioner) {
    if (columns.empty()) {
        auto n = std::make_unique<Node>();  // BRWT(): empty root
        n->nonzero_rows.finalize();
        return n;
    }
    std::vector<NodeBRWT> nodes(columns.size());
    for (size_t i = 0; i < columns.size(); ++i) {
        nodes[i].column_arrangement = {i};
        nodes[i].group_sizes = {1};
    }
    while (nodes.size() > 1) {
        auto groups = partitioner(columns);
        std::vector<NodeBRWT> parent_nodes(groups.size());
        VectorsPtr parent_columns(groups.size());
        for (size_t g = 0; g < groups.size(); ++g) {
            std::vector<NodeBRWT> sub_nodes;
            VectorsPtr sub_cols;
            for (auto j : groups[g]) {
                sub_nodes.push_back(std::move(nodes[j]));
                sub_cols.push_back(std::move(columns[j]));
            }
            auto parent = merge(std::move(sub_nodes), std::move(sub_cols));
            parent_nodes[g] = std::move(parent.first);
            parent_columns[g] = std::move(parent.second);
        }
        nodes = std::move(parent_nodes);
        columns = std::move(parent_columns);
    }
    return initialize(std::move(nodes.at(0)), std::move(*columns.at(0)));
}

// ---- greedy binary grouping (partitionings.cpp) ---------------------------

// utils::sample_indexes (utils.cpp:777-816)
std::vector<uint64_t> sample_indexes(uint64_t universe_size, uint64_t sample_size, std::mt19937 &gen) {
    if (!universe_size) return {};
    sample_size = std::min(universe_size, sample_size);
    std::vector<uint64_t> indexes;
    indexes.reserve(3 * sample_size);
    if (sample_size * 10 < universe_size) {
        std::uniform_int_distribution<uint64_t> dis(0, universe_size - 1);
        while (indexes.size() < sample_size) {
            indexes.clear();
            for (size_t i = 0; i < 1.5 * sample_size; ++i) indexes.push_back(dis(gen));
            std::sort(indexes.begin(), indexes.end());
            indexes.erase(std::unique(indexes.begin(), indexes.end()), indexes.end());
        }
    } else {
        std::bernoulli_distribution dis(2.0 * sample_size / universe_size);
        while (indexes.size() < sample_size) {
            indexes.clear();
            for (size_t i = 0; i < universe_size; ++i)
                if (dis(gen)) indexes.push_back(i);
        }
    }
    std::shuffle(indexes.begin(), indexes.end(), gen);
    return std::vector<uint64_t>(indexes.begin(), indexes.begin() + sample_size);
}

// parallel_binary_grouping_greedy (partitionings.cpp:148-196); similarities
// from random_submatrix(..., kNumRowsSampled = 1e6, seed 1) (:5, :37-58, :126-137)
Partition greedy_partitioner(const VectorsPtr &columns) {
    if (columns.empty()) return {};
    const uint64_t n = columns[0]->size;
    std::mt19937 gen;
    gen.seed(1);
    auto idx = sample_indexes(n, std::min<uint64_t>(1000000, n), gen);
    std::sort(idx.begin(), idx.end());
    std::vector<BitVec> sub(columns.size());
    for (size_t i = 0; i < columns.size(); ++i) {  // utils::subvector
        sub[i] = BitVec(idx.size());
        for (size_t k = 0; k < idx.size(); ++k)
            if (columns[i]->get(idx[k])) sub[i].set(k);
    }
    // correlation_similarity (partitionings.cpp:73-94): inner products as double
    std::vector<std::tuple<size_t, size_t, uint64_t>> candidates;
    for (size_t j = 1; j < sub.size(); ++j) {
        for (size_t k = 0; k < j; ++k) {
            uint64_t ip = 0;
            for (size_t w = 0; w < sub[j].words.size(); ++w) ip += popcnt64(sub[j].words[w] & sub[k].words[w]);
            double sim = (double)ip;
            candidates.emplace_back(j, k, (uint64_t)sim);
        }
    }
    auto dist = [](size_t a, size_t b) { return a > b ? a - b : b - a; };
    std::sort(candidates.begin(), candidates.end(), [&](const auto &f, const auto &s) {
        return std::get<2>(f) > std::get<2>(s) ||
               (std::get<2>(f) == std::get<2>(s) && dist(std::get<0>(f), std::get<1>(f)) < dist(std::get<0>(s), std::get<1>(s)));
    });
    Partition partition;
    std::vector<bool> matched(columns.size(), false);
    for (auto &c : candidates) {
        auto i = std::get<0>(c), j = std::get<1>(c);
        if (!matched[i] && !matched[j]) {
            matched[i] = matched[j] = true;
            partition.push_back({i, j});
        }
    }
    for (size_t i = 0; i < columns.size(); ++i)
        if (!matched[i]) partition.push_back({i});
    return partition;
}

// ---- BRWTOptimizer::relax (BRWT_builders.cpp:166-380) ---------------------

// sizeof(bit_vector_rrr<63>) * 8 enters bv_space_taken_rrr (BRWT_builders.cpp:315-321).
// sdsl is absent, so the struct size is an estimate (parity unpinned; it only
// shifts the prune decision, never the query results, which relax preserves).
constexpr double kRRRObjectBits = 184 * 8;

double logbinomial(uint64_t n, uint64_t m) {  // :299-303
    return (lgamma(n + 1) - lgamma(m + 1) - lgamma(n - m + 1)) / log(2);
}
double bv_space_taken_rrr(uint64_t size, uint64_t ones, uint8_t block) {  // :315-321
    return logbinomial(size, ones) + std::ceil(log2(block + 1) / block) * size + kRRRObjectBits;
}
double pruning_delta(const Node &node) {  // :351-380
    double delta = 0;
    for (auto &c : node.children) {
        delta += bv_space_taken_rrr(node.num_rows(), c->nonzero_rows.ones, 63);
        delta -= bv_space_taken_rrr(c->nonzero_rows.size, c->nonzero_rows.ones, 63);
    }
    delta -= bv_space_taken_rrr(node.nonzero_rows.size, node.nonzero_rows.ones, 63);
    return delta;
}

// reassign (BRWT_builders.cpp:257-297)
void reassign(std::unique_ptr<Node> &&node, NodeBRWT *parent) {
    const BitVec &node_index = node->nonzero_rows;
    size_t offset = parent->group_sizes.size();
    parent->group_sizes.resize(offset + node->children.size());
    parent->child_nodes.resize(offset + node->children.size());
    for (size_t i = 0; i < node->children.size(); ++i) {
        auto grand = std::move(node->children[i]);
        BitVec sub(node_index.size);
        uint64_t ci = 0;
        node_index.call_ones([&](uint64_t p) {
            if (grand->nonzero_rows.get(ci)) sub.set(p);
            ++ci;
        });
        sub.finalize();
        grand->nonzero_rows = std::move(sub);
        parent->group_sizes[offset + i] = grand->num_columns();
        parent->child_nodes[offset + i] = std::move(grand);
    }
}

// add_submatrix (BRWT_builders.cpp:213-255)
void add_submatrix(std::unique_ptr<Node> &&sub, NodeBRWT *parent, uint64_t max_delta_arity) {
    bool prune = !sub->children.empty();
    if (prune && sub->children.size() > max_delta_arity) prune = false;
    if (!prune || pruning_delta(*sub) > 0) {
        parent->group_sizes.push_back(sub->num_columns());
        parent->child_nodes.push_back(std::move(sub));
    } else {
        reassign(std::move(sub), parent);
    }
}

void relax(Node *root, uint64_t max_arity) {  // :166-211
    std::deque<Node *> parents;
    root->bft([&](const Node &n) {
        if (!n.children.empty()) parents.push_front(const_cast<Node *>(&n));
    });
    while (!parents.empty()) {
        Node &parent = *parents.front();
        parents.pop_front();
        NodeBRWT updated;
        size_t nchild = parent.children.size();
        for (size_t g = 0; g < nchild; ++g) {
            auto ncols = parent.children[g]->num_columns();
            for (size_t r = 0; r < ncols; ++r)
                updated.column_arrangement.push_back(parent.assignments.get((uint32_t)g, (uint32_t)r));
            uint64_t used = (uint64_t)updated.group_sizes.size() + nchild - g - 1;
            add_submatrix(std::move(parent.children[g]), &updated, max_arity - std::min(max_arity, used));
        }
        BitVec idx = std::move(parent.nonzero_rows);
        auto fresh = initialize(std::move(updated), std::move(idx));
        parent.assignments = std::move(fresh->assignments);
        parent.nonzero_rows = std::move(fresh->nonzero_rows);
        parent.children = std::move(fresh->children);
    }
}

// ---- synthetic top-down generator (DESIGN.md "Synthetic matrices") -------
// Spec shared with the product (genome_graph_annotation_amd/csrc/synth.hip),
// implemented independently on both sides.

inline uint64_t mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
inline uint64_t synth_key(uint64_t seed, uint64_t key) { return mix64(seed ^ ((key + 1) * 0x9E3779B97F4A7C15ull)); }
inline uint64_t synth_draw(uint64_t k, uint64_t pos) { return mix64(k + pos * 0xD1B54A32D192ED03ull); }
constexpr uint64_t kRootKey = 0xFFFFFFFFull;

uint64_t prob_to_threshold(double p) {
    if (!(p > 0.0)) return 0;
    if (p >= 1.0) return UINT64_MAX;
    return (uint64_t)(p * 18446744073709551616.0);
}
inline bool bern(uint64_t x, uint64_t t) { return x < t || t == UINT64_MAX; }

// Inverse-CDF table over the nonzero child masks of a node whose children
// have "subtree nonzero" probabilities q[0..a).  T[k-1] is the threshold of mask k.
std::vector<uint64_t> mask_table(const std::vector<double> &q) {
    const size_t a = q.size();
    const size_t nm = (1ull << a) - 1;
    std::vector<uint64_t> T(nm, UINT64_MAX);
    double prod0 = 1.0;
    for (size_t c = 0; c < a; ++c) prod0 = prod0 * (1.0 - q[c]);
    double Z = 1.0 - prod0;
    if (!(Z > 0.0)) return T;  // unreachable node: always mask 1
    double cum = 0.0;
    for (size_t k = 1; k <= nm; ++k) {
        double p = 1.0;
        for (size_t c = 0; c < a; ++c) p = p * (((k >> c) & 1) ? q[c] : (1.0 - q[c]));
        cum = cum + p / Z;
        T[k - 1] = (k == nm) ? UINT64_MAX : prob_to_threshold(cum);
    }
    return T;
}
// Mask lookup: smallest k in [1, nm] with x < T[k-1] (nm if none).  A guide
// table over the top 12 bits of x gives the first candidate k of the bucket;
// the answer is the same as a binary search over T (the device's form).
struct MaskSampler {
    std::vector<uint64_t> T;
    std::vector<uint32_t> guide;  // 4096 entries
    explicit MaskSampler(std::vector<uint64_t> t) : T(std::move(t)), guide(4096) {
        const uint32_t nm = (uint32_t)T.size();
        uint32_t k = 1;
        for (uint32_t g = 0; g < 4096; ++g) {
            const uint64_t lo = (uint64_t)g << 52;
            while (k < nm && lo >= T[k - 1]) ++k;
            guide[g] = k;
        }
    }
    inline uint32_t operator()(uint64_t x) const {
        const uint32_t nm = (uint32_t)T.size();
        uint32_t k = guide[x >> 52];
        while (k < nm && x >= T[k - 1]) ++k;
        return k;
    }
};

struct ShapeNode {
    std::vector<int> children;  // indices into shape vector
    uint64_t cols = 0;          // leaves below
    uint32_t column = UINT32_MAX;  // leaves: the global column
};

// a tree shape in BFS numbering from arrays (mbrwt_shape_desc's layout);
// cols by a reverse BFS sweep.  Empty on a malformed shape.
std::vector<ShapeNode> shape_from_arrays(uint32_t N, const uint32_t *nc, const uint32_t *fc, const uint32_t *lc) {
    std::vector<ShapeNode> sh(N);
    for (uint32_t u = 0; u < N; ++u) {
        if (nc[u] == 0) {
            sh[u].column = lc[u];
            continue;
        }
        if (fc[u] <= u || (uint64_t)fc[u] + nc[u] > N) return {};
        for (uint32_t c = 0; c < nc[u]; ++c) sh[u].children.push_back((int)(fc[u] + c));
    }
    for (uint32_t u = N; u-- > 0;) {
        if (sh[u].children.empty()) {
            sh[u].cols = 1;
            continue;
        }
        for (int c : sh[u].children) sh[u].cols += sh[c].cols;
    }
    return sh;
}

// Shape of BRWTBottomUpBuilder::build with the basic arity-k partitioner,
// including the pass-through of single-element groups (BRWT_builders.cpp:74-76).
// Returns nodes with node 0 = root in BFS numbering.
std::vector<ShapeNode> basic_shape(uint64_t m, uint32_t arity) {
    std::vector<ShapeNode> all;
    std::vector<int> cur;
    for (uint64_t i = 0; i < m; ++i) {
        all.push_back(ShapeNode{{}, 1, (uint32_t)i});
        cur.push_back((int)i);
    }
    while (cur.size() > 1) {
        std::vector<int> next;
        for (size_t g = 0; g * arity < cur.size(); ++g) {
            size_t b = g * arity, e = std::min<size_t>(cur.size(), b + arity);
            if (e - b == 1) {
                next.push_back(cur[b]);
                continue;
            }
            ShapeNode p;
            for (size_t i = b; i < e; ++i) {
                p.children.push_back(cur[i]);
                p.cols += all[cur[i]].cols;
            }
            all.push_back(p);
            next.push_back((int)all.size() - 1);
        }
        cur = next;
    }
    // BFS renumbering
    std::vector<ShapeNode> bfs;
    std::vector<int> order{cur[0]};
    for (size_t h = 0; h < order.size(); ++h)
        for (int c : all[order[h]].children) order.push_back(c);
    std::vector<int> newid(all.size(), -1);
    for (size_t i = 0; i < order.size(); ++i) newid[order[i]] = (int)i;
    for (int o : order) {
        ShapeNode s = all[o];
        for (auto &c : s.children) c = newid[c];
        bfs.push_back(s);
    }
    return bfs;
}

int resolve_threads(int t) {
#ifdef _OPENMP
    return t > 0 ? t : omp_get_max_threads();
#else
    (void)t;
    return 1;
#endif
}

std::unique_ptr<Node> generate_topdown_shape(uint64_t n, const std::vector<ShapeNode> &shape, double d, uint64_t seed,
                                             int threads);

std::unique_ptr<Node> generate_topdown(uint64_t n, uint64_t m, double d, uint32_t arity, uint64_t seed, int threads) {
    if (m == 0) {
        auto r = std::make_unique<Node>();
        r->nonzero_rows.finalize();
        return r;
    }
    return generate_topdown_shape(n, basic_shape(m, arity), d, seed, threads);
}

// the same law over any shape: node keys are BFS ids, the
// root's partition lists global columns (pre-order leaves per child), every
// other node's partition is consecutive ranges (BRWT_builders.cpp:68-107)
std::unique_ptr<Node> generate_topdown_shape(uint64_t n, const std::vector<ShapeNode> &shape, double d, uint64_t seed,
                                             int threads) {
    const size_t N = shape.size();
    std::vector<double> q(N);
    for (size_t u = 0; u < N; ++u) q[u] = 1.0 - std::pow(1.0 - d, (double)shape[u].cols);

    std::vector<std::unique_ptr<Node>> nodes(N);
    for (auto &p : nodes) p = std::make_unique<Node>();
    threads = resolve_threads(threads);

    // root index vector: Bernoulli(q_root) per row
    {
        BitVec &v = nodes[0]->nonzero_rows;
        v = BitVec(n);
        const uint64_t T = prob_to_threshold(q[0]);
        const uint64_t K = synth_key(seed, kRootKey);
        const int64_t W = (int64_t)v.words.size();
#pragma omp parallel for num_threads(threads) schedule(static)
        for (int64_t w = 0; w < W; ++w) {
            uint64_t word = 0;
            for (uint64_t b = 0; b < 64; ++b) {
                uint64_t r = (uint64_t)w * 64 + b;
                if (r < n && bern(synth_draw(K, r), T)) word |= 1ull << b;
            }
            v.words[w] = word;
        }
        v.finalize();
    }
    // children masks, in BFS order (parents before children)
    for (size_t u = 0; u < N; ++u) {
        auto &sh = shape[u];
        if (sh.children.empty()) continue;
        const uint64_t L = nodes[u]->nonzero_rows.ones;
        const size_t a = sh.children.size();
        std::vector<double> qc(a);
        for (size_t c = 0; c < a; ++c) qc[c] = q[sh.children[c]];
        const MaskSampler T(mask_table(qc));
        const uint64_t K = synth_key(seed, u);
        for (size_t c = 0; c < a; ++c) nodes[sh.children[c]]->nonzero_rows = BitVec(L);
        std::vector<uint64_t *> out(a);
        for (size_t c = 0; c < a; ++c) out[c] = nodes[sh.children[c]]->nonzero_rows.words.data();
        const int64_t W = (int64_t)((L + 63) / 64);
#pragma omp parallel for num_threads(threads) schedule(static)
        for (int64_t w = 0; w < W; ++w) {
            uint64_t acc[64];
            for (size_t c = 0; c < a; ++c) acc[c] = 0;
            for (uint64_t b = 0; b < 64; ++b) {
                uint64_t j = (uint64_t)w * 64 + b;
                if (j >= L) break;
                uint32_t mask = T(synth_draw(K, j));
                for (size_t c = 0; c < a; ++c) acc[c] |= (uint64_t)((mask >> c) & 1) << b;
            }
            for (size_t c = 0; c < a; ++c) out[c][w] = acc[c];
        }
        for (size_t c = 0; c < a; ++c) nodes[sh.children[c]]->nonzero_rows.finalize();
    }
    // assemble the BRWT objects: global columns at the root (pre-order leaves
    // of each child), consecutive ranges below (BRWT_builders.cpp:84-91)
    std::vector<std::vector<uint64_t>> leaves(N);
    for (size_t uu = N; uu-- > 0;) {
        if (shape[uu].children.empty()) {
            leaves[uu] = {shape[uu].column};
            continue;
        }
        for (int c : shape[uu].children) leaves[uu].insert(leaves[uu].end(), leaves[c].begin(), leaves[c].end());
    }
    for (size_t uu = N; uu-- > 0;) {
        auto &sh = shape[uu];
        Node &nd = *nodes[uu];
        if (sh.children.empty()) {
            nd.assignments = RangePartition({0}, {1});
            continue;
        }
        std::vector<uint64_t> arr(sh.cols);
        std::iota(arr.begin(), arr.end(), 0);
        if (uu == 0) arr = leaves[0];
        std::vector<size_t> gs;
        for (int c : sh.children) gs.push_back(shape[c].cols);
        nd.assignments = RangePartition(arr, gs);
        for (int c : sh.children) nd.children.push_back(std::move(nodes[c]));
    }
    return std::move(nodes[0]);
}

// ---- the same top-down tree queried WITHOUT materialising it ---------------
// Every index bit of the synthetic tree is a pure function of (node, position):
// child c of u at position j is bit c of mask(u, j) = T_u(H(K_u, j)), for
// j < popcount(I_u).  BRWT::get_row (BRWT.cpp:26-53) needs, at a visited node,
// the bit and the inclusive rank1 (BRWT.cpp:30,43), i.e. the count of bit c over
// mask(u, 0..j).  So the batch is resolved node by node (depth-first over the
// shape, so only the lists of one root-to-leaf path of nodes are alive): a node
// with queries streams its masks over [0, max queried j] in parallel chunks,
// counting per child, and moves each query down with rank - 1.  Memory is
// O(batch x depth), time O(sum of streamed lengths): the parity check of the
// 1 B-row RefSeq shape (158 GB of plain index bits) needs no host structure.
struct QueryAt {
    uint64_t pos;  // position in the node's children level (rank1 - 1 at the node)
    uint32_t qid;  // index of the query row in the batch
};

// MaskSampler's answer by a branchless binary search (the streamed loops draw
// ~10^11 masks; the guide table's data-dependent scan mispredicts):
// k = 1 + #{i < nm-1 : T[i] <= x}, capped at nm (T is nondecreasing).
struct FlatSampler {
    std::vector<uint64_t> T;  // padded to a power of two with UINT64_MAX
    uint32_t P = 1, nm = 1;
    explicit FlatSampler(const std::vector<uint64_t> &t) : nm((uint32_t)t.size()) {
        while (P < nm) P <<= 1;
        T.assign(P, UINT64_MAX);
        for (uint32_t i = 0; i + 1 < nm; ++i) T[i] = t[i];
    }
    inline uint32_t operator()(uint64_t x) const {
        uint32_t base = 0;
        for (uint32_t step = P >> 1; step; step >>= 1) base += (T[base + step - 1] <= x) ? step : 0;
        base += (T[base] <= x) ? 1 : 0;
        return std::min(base + 1, nm);
    }
};

// byte-lane spread of an 8-bit mask: bit c -> byte c (per-child counters)
static const std::array<uint64_t, 256> kSpread = [] {
    std::array<uint64_t, 256> s{};
    for (uint32_t m = 0; m < 256; ++m)
        for (uint32_t c = 0; c < 8; ++c) s[m] |= (uint64_t)((m >> c) & 1) << (8 * c);
    return s;
}();

struct TopdownQuery {
    const std::vector<ShapeNode> &shape;
    const std::vector<double> &q;
    const std::vector<uint32_t> &leaf_col;
    uint64_t seed;
    int threads;
    std::vector<std::pair<uint32_t, uint32_t>> emitted;  // (qid, column) in DFS order
    uint64_t draws = 0;

    static constexpr uint64_t kChunk = 1ull << 16;

    // Resolve node u's queries (sorted by pos, pos < popcount(I_u)).
    void visit(int u, std::vector<QueryAt> &&qs) {
        const auto &sh = shape[u];
        const size_t a = sh.children.size();
        std::vector<double> qc(a);
        for (size_t c = 0; c < a; ++c) qc[c] = q[sh.children[c]];
        const MaskSampler T(mask_table(qc));
        const uint64_t K = synth_key(seed, (uint64_t)u);
        const uint64_t len = qs.back().pos + 1;
        if (a > 16) throw std::runtime_error("topdown_query: arity > 16");
        const int64_t nchunks = (int64_t)((len + kChunk - 1) / kChunk);
        // per chunk: per-child counts, the index of the chunk's first query
        std::vector<uint64_t> cnt((size_t)nchunks * a, 0);
        std::vector<size_t> qbeg(nchunks + 1);
        {
            size_t i = 0;
            for (int64_t k = 0; k <= nchunks; ++k) {
                const uint64_t lo = (uint64_t)k * kChunk;
                while (i < qs.size() && qs[i].pos < lo) ++i;
                qbeg[k] = i;
            }
        }
        // children's lists per chunk (positions chunk-local until the scan)
        std::vector<std::vector<std::vector<QueryAt>>> down(nchunks, std::vector<std::vector<QueryAt>>(a));
        std::vector<std::vector<std::pair<uint32_t, uint32_t>>> emit(nchunks);
#pragma omp parallel for num_threads(threads) schedule(dynamic, 4)
        for (int64_t k = 0; k < nchunks; ++k) {
            uint64_t local[16] = {0};
            const uint64_t lo = (uint64_t)k * kChunk, hi = std::min(len, lo + kChunk);
            size_t i = qbeg[k];
            const size_t iend = qbeg[k + 1];
            for (uint64_t j = lo; j < hi;) {
                const uint64_t next_q = i < iend ? qs[i].pos : hi;
                if (j < next_q) {
                    // no query in [j, end): count into byte lanes (<= 255 draws), then flush
                    const uint64_t end = std::min(next_q, j + 255);
                    uint64_t acc_lo = 0, acc_hi = 0;
                    for (; j < end; ++j) {
                        const uint32_t mk = T(synth_draw(K, j));
                        acc_lo += kSpread[mk & 255];
                        acc_hi += kSpread[(mk >> 8) & 255];
                    }
                    for (size_t c = 0; c < a; ++c)
                        local[c] += ((c < 8 ? acc_lo >> (8 * c) : acc_hi >> (8 * (c - 8)))) & 255;
                    continue;
                }
                const uint32_t mask = T(synth_draw(K, j));
                for (uint32_t m = mask; m; m &= m - 1) ++local[__builtin_ctz(m)];
                for (; i < iend && qs[i].pos == j; ++i) {
                    for (uint32_t m = mask; m; m &= m - 1) {
                        const int c = __builtin_ctz(m);
                        const int v = sh.children[c];
                        if (shape[v].children.empty())
                            emit[k].push_back({qs[i].qid, leaf_col[v]});
                        else
                            down[k][c].push_back({local[c] - 1, qs[i].qid});
                    }
                }
                ++j;
            }
            for (size_t c = 0; c < a; ++c) cnt[(size_t)k * a + c] = local[c];
        }
        draws += len;
        std::vector<QueryAt>().swap(qs);
        // concatenate the chunks' outputs in chunk order (parallel copies at
        // exclusive prefixes): emissions, and per child the positions rebased by
        // the child's count before the chunk
        std::vector<size_t> eoff(nchunks + 1, 0);
        for (int64_t k = 0; k < nchunks; ++k) eoff[k + 1] = eoff[k] + emit[k].size();
        const size_t e0 = emitted.size();
        emitted.resize(e0 + eoff[nchunks]);
        std::vector<uint64_t> base((size_t)nchunks * a), doff((size_t)(nchunks + 1) * a, 0);
        for (size_t c = 0; c < a; ++c) {
            uint64_t b = 0;
            for (int64_t k = 0; k < nchunks; ++k) {
                base[(size_t)k * a + c] = b;
                b += cnt[(size_t)k * a + c];
                doff[(size_t)(k + 1) * a + c] = doff[(size_t)k * a + c] + down[k][c].size();
            }
        }
        std::vector<std::vector<QueryAt>> lists(a);
        for (size_t c = 0; c < a; ++c) lists[c].resize(doff[(size_t)nchunks * a + c]);
#pragma omp parallel for num_threads(threads) schedule(dynamic, 16)
        for (int64_t k = 0; k < nchunks; ++k) {
            std::copy(emit[k].begin(), emit[k].end(), emitted.begin() + e0 + eoff[k]);
            std::vector<std::pair<uint32_t, uint32_t>>().swap(emit[k]);
            for (size_t c = 0; c < a; ++c) {
                QueryAt *dst = lists[c].data() + doff[(size_t)k * a + c];
                const uint64_t b = base[(size_t)k * a + c];
                for (auto &e : down[k][c]) *dst++ = {e.pos + b, e.qid};
                std::vector<QueryAt>().swap(down[k][c]);
            }
        }
        down.clear();
        // pre-order: children in order, each child's whole subtree before the next
        for (size_t c = 0; c < a; ++c)
            if (!lists[c].empty()) visit(sh.children[c], std::move(lists[c]));
    }
};

// Returns 0, or 2 on an out-of-range row.  Output: the reference's order
// (pre-order of the leaves = ascending columns for the basic partitioner).
int topdown_query_shape(uint64_t n, const std::vector<ShapeNode> &shape, double d, uint64_t seed,
                        const uint64_t *rows, uint64_t nq, int threads, std::vector<uint64_t> &offsets,
                        std::vector<uint32_t> &cols, uint64_t *draws);

int topdown_query(uint64_t n, uint64_t m, double d, uint32_t arity, uint64_t seed, const uint64_t *rows,
                  uint64_t nq, int threads, std::vector<uint64_t> &offsets, std::vector<uint32_t> &cols,
                  uint64_t *draws) {
    if (m == 0) {
        for (uint64_t i = 0; i < nq; ++i)
            if (rows[i] >= n) return 2;
        offsets.assign(nq + 1, 0);
        cols.clear();
        return 0;
    }
    return topdown_query_shape(n, basic_shape(m, arity), d, seed, rows, nq, threads, offsets, cols, draws);
}

int topdown_query_shape(uint64_t n, const std::vector<ShapeNode> &shape, double d, uint64_t seed,
                        const uint64_t *rows, uint64_t nq, int threads, std::vector<uint64_t> &offsets,
                        std::vector<uint32_t> &cols, uint64_t *draws) {
    for (uint64_t i = 0; i < nq; ++i)
        if (rows[i] >= n) return 2;
    offsets.assign(nq + 1, 0);
    cols.clear();
    if (shape.empty() || nq == 0) return 0;
    std::vector<double> q(shape.size());
    for (size_t u = 0; u < shape.size(); ++u) q[u] = 1.0 - std::pow(1.0 - d, (double)shape[u].cols);
    // leaves are emitted by their pre-order rank (sorted per row = the
    // reference's output order, BRWT.cpp:45-51) and mapped to their global
    // columns at the end (RangePartition::get composed, utils.cpp:689-691)
    std::vector<uint32_t> leaf_col(shape.size(), UINT32_MAX);
    {
        uint32_t next = 0;
        std::vector<int> st{0};
        while (!st.empty()) {
            int u = st.back();
            st.pop_back();
            if (shape[u].children.empty()) leaf_col[u] = next++;
            for (size_t c = shape[u].children.size(); c-- > 0;) st.push_back(shape[u].children[c]);
        }
    }
    threads = resolve_threads(threads);
    TopdownQuery tq{shape, q, leaf_col, seed, threads, {}, 0};

    // the root's own index bit: Bernoulli(q_root) per row; its inclusive rank
    // over [0, row] comes from a chunked count of the same draws
    std::vector<QueryAt> root;
    {
        std::vector<std::pair<uint64_t, uint32_t>> sorted(nq);
        for (uint64_t i = 0; i < nq; ++i) sorted[i] = {rows[i], (uint32_t)i};
        std::sort(sorted.begin(), sorted.end());
        const uint64_t Tq = prob_to_threshold(q[0]);
        const uint64_t K = synth_key(seed, kRootKey);
        const uint64_t len = sorted.back().first + 1;
        const uint64_t C = TopdownQuery::kChunk;
        const int64_t nchunks = (int64_t)((len + C - 1) / C);
        std::vector<uint64_t> cnt(nchunks);
        std::vector<size_t> qbeg(nchunks + 1);
        size_t i = 0;
        for (int64_t k = 0; k <= nchunks; ++k) {
            while (i < nq && sorted[i].first < (uint64_t)k * C) ++i;
            qbeg[k] = i;
        }
        std::vector<uint64_t> local_rank(nq, UINT64_MAX);  // by sorted index; MAX = bit unset
#pragma omp parallel for num_threads(threads) schedule(dynamic, 4)
        for (int64_t k = 0; k < nchunks; ++k) {
            const uint64_t lo = (uint64_t)k * C, hi = std::min(len, lo + C);
            uint64_t ones = 0;
            size_t ii = qbeg[k];
            for (uint64_t r = lo; r < hi; ++r) {
                const bool bit = bern(synth_draw(K, r), Tq);
                ones += bit;
                for (; ii < qbeg[k + 1] && sorted[ii].first == r; ++ii) local_rank[ii] = bit ? ones - 1 : UINT64_MAX;
            }
            cnt[k] = ones;
        }
        tq.draws += len;
        uint64_t base = 0;
        for (int64_t k = 0; k < nchunks; ++k) {
            for (size_t s = qbeg[k]; s < qbeg[k + 1]; ++s)
                if (local_rank[s] != UINT64_MAX) root.push_back({local_rank[s] + base, sorted[s].second});
            base += cnt[k];
        }
    }
    if (!root.empty()) {
        if (shape[0].children.empty()) {  // one-column matrix: the root is the leaf (BRWT.cpp:34-39)
            for (auto &e : root) tq.emitted.push_back({e.qid, 0});
        } else {
            tq.visit(0, std::move(root));
        }
    }
    // bucket the emissions by query (parallel, atomic counters) ...
    const int64_t ne = (int64_t)tq.emitted.size();
#pragma omp parallel for num_threads(threads) schedule(static)
    for (int64_t e = 0; e < ne; ++e) __atomic_fetch_add(&offsets[tq.emitted[e].first + 1], 1, __ATOMIC_RELAXED);
    for (uint64_t i = 0; i < nq; ++i) offsets[i + 1] += offsets[i];
    cols.resize(tq.emitted.size());
    {
        std::vector<uint64_t> fill(offsets.begin(), offsets.end() - 1);
#pragma omp parallel for num_threads(threads) schedule(static)
        for (int64_t e = 0; e < ne; ++e)
            cols[__atomic_fetch_add(&fill[tq.emitted[e].first], 1, __ATOMIC_RELAXED)] = tq.emitted[e].second;
    }
    std::vector<std::pair<uint32_t, uint32_t>>().swap(tq.emitted);
    // ... and order each row by leaf_col, which IS the leaves' pre-order rank,
    // i.e. the reference's output order (BRWT.cpp:45-51)
    const int64_t nn = (int64_t)nq;
#pragma omp parallel for num_threads(threads) schedule(dynamic, 1024)
    for (int64_t r = 0; r < nn; ++r) std::sort(cols.begin() + offsets[r], cols.begin() + offsets[r + 1]);
    // pre-order rank -> the leaf's global column
    std::vector<uint32_t> col_of(leaf_col.size());
    for (size_t u = 0; u < shape.size(); ++u)
        if (shape[u].children.empty()) col_of[leaf_col[u]] = shape[u].column;
    const int64_t nc = (int64_t)cols.size();
#pragma omp parallel for num_threads(threads) schedule(static)
    for (int64_t i = 0; i < nc; ++i) cols[i] = col_of[cols[i]];
    if (draws) *draws = tq.draws;
    return 0;
}

// ---- data generation (experiments/data_generation.cpp) -------------------

struct DataGenerator {  // data_generation.hpp:7-79
    std::mt19937 gen;
    DataGenerator() { gen.seed(0); }
    void set_seed(uint32_t s) { gen.seed(s); }
    // generate_random_column_uncompressed (data_generation.cpp:20-29)
    void column(uint64_t n, double d, uint64_t *words) {
        std::bernoulli_distribution dis(d);
        for (uint64_t i = 0; i < n; ++i)
            if (dis(gen)) words[i >> 6] |= 1ull << (i & 63);
    }
};

}  // namespace

// ========================================================================
// C ABI
// ========================================================================

struct OracleTree {
    std::unique_ptr<Node> root;
    // BFS export (lazily built)
    bool exported = false;
    std::vector<const Node *> bfs;
    std::vector<uint32_t> num_children, first_child, leaf_column;
    std::vector<uint64_t> vec_size;

    void do_export() {
        if (exported) return;
        exported = true;
        if (root->num_columns() == 0) return;  // empty matrix: no nodes
        bfs.push_back(root.get());
        std::vector<uint32_t> parent_of{UINT32_MAX}, childidx_of{0};
        for (size_t h = 0; h < bfs.size(); ++h) {
            const Node *n = bfs[h];
            num_children.push_back((uint32_t)n->children.size());
            first_child.push_back(n->children.empty() ? 0u : (uint32_t)bfs.size());
            for (size_t i = 0; i < n->children.size(); ++i) {
                bfs.push_back(n->children[i].get());
                parent_of.push_back((uint32_t)h);
                childidx_of.push_back((uint32_t)i);
            }
            vec_size.push_back(n->nonzero_rows.size);
        }
        // leaf global column: compose RangePartition::get up the path
        leaf_column.assign(bfs.size(), UINT32_MAX);
        for (size_t u = 0; u < bfs.size(); ++u) {
            if (!bfs[u]->children.empty()) continue;
            uint32_t col = 0, v = (uint32_t)u;
            while (parent_of[v] != UINT32_MAX) {
                col = bfs[parent_of[v]]->assignments.get(childidx_of[v], col);
                v = parent_of[v];
            }
            leaf_column[u] = col;
        }
    }
};

struct OracleBitVec {
    BitVec bv;
};

extern "C" {

static VectorsPtr columns_from_words(const uint64_t *col_words, uint64_t n, uint64_t m) {
    const uint64_t W = (n + 63) / 64;
    VectorsPtr cols;
    for (uint64_t j = 0; j < m; ++j) {
        auto bv = std::make_unique<BitVec>(n);
        std::memcpy(bv->words.data(), col_words + j * W, W * 8);
        bv->clear_tail();
        cols.push_back(std::move(bv));
    }
    return cols;
}

static OracleTree *build_tree(VectorsPtr &&cols, int partitioner, uint32_t arity, uint64_t relax_max_arity) {
    auto t = new OracleTree();
    Partitioner p = partitioner == 1 ? Partitioner(greedy_partitioner) : basic_partitioner(arity < 2 ? 2 : arity);
    t->root = build(std::move(cols), p);
    if (relax_max_arity > 1 && !t->root->children.empty()) relax(t->root.get(), relax_max_arity);
    return t;
}

OracleTree *oracle_build_from_columns(const uint64_t *col_words, uint64_t num_rows, uint64_t num_cols,
                                      int partitioner, uint32_t arity, uint64_t relax_max_arity) {
    try {
        return build_tree(columns_from_words(col_words, num_rows, num_cols), partitioner, arity, relax_max_arity);
    } catch (...) {
        return nullptr;
    }
}

void oracle_generate_columns(uint64_t n, uint64_t m, double d, uint32_t seed, uint64_t *col_words) {
    DataGenerator g;
    g.set_seed(seed);
    const uint64_t W = (n + 63) / 64;
    std::memset(col_words, 0, W * m * 8);
    for (uint64_t j = 0; j < m; ++j) g.column(n, d, col_words + j * W);
}

// experiments/main.cpp:232-264 "uniform_rows": `unique` distinct rows drawn
// as columns over `unique` rows (generate_random_columns), each repeated
// n / unique times, the repeated rows shuffled (replicate_shuffle,
// data_generation.cpp:66-86, std::shuffle with the same engine) -- rows of
// the result = n_out = unique * (n / unique).  Column-major words like
// oracle_generate_columns.
uint64_t oracle_generate_uniform_rows(uint64_t n, uint64_t m, double d, uint64_t unique, uint32_t seed,
                                      uint64_t *col_words) {
    if (!unique || unique > n) return 0;
    DataGenerator g;
    g.set_seed(seed);
    const uint64_t Wu = (unique + 63) / 64;
    std::vector<uint64_t> gen((size_t)Wu * m, 0);
    for (uint64_t j = 0; j < m; ++j) g.column(unique, d, gen.data() + j * Wu);  // generate_random_columns
    const uint64_t freq = n / unique, n_out = unique * freq;
    std::vector<uint64_t> src(n_out);  // replicate: row i repeated freq times, in order
    for (uint64_t i = 0; i < n_out; ++i) src[i] = i / freq;
    std::shuffle(src.begin(), src.end(), g.gen);
    if (col_words) {
        const uint64_t W = (n_out + 63) / 64;
        std::memset(col_words, 0, W * m * 8);
        for (uint64_t j = 0; j < m; ++j)
            for (uint64_t r = 0; r < n_out; ++r)
                if ((gen[j * Wu + (src[r] >> 6)] >> (src[r] & 63)) & 1) col_words[j * W + (r >> 6)] |= 1ull << (r & 63);
    }
    return n_out;
}

// experiments/main.cpp:249-264 "uniform_columns": `unique` distinct columns,
// each repeated m / unique times, the repeated columns shuffled; columns of
// the result = unique * (m / unique).
uint64_t oracle_generate_uniform_columns(uint64_t n, uint64_t m, double d, uint64_t unique, uint32_t seed,
                                         uint64_t *col_words) {
    if (!unique || unique > m) return 0;
    DataGenerator g;
    g.set_seed(seed);
    const uint64_t W = (n + 63) / 64;
    std::vector<uint64_t> gen((size_t)W * unique, 0);
    for (uint64_t j = 0; j < unique; ++j) g.column(n, d, gen.data() + j * W);
    const uint64_t freq = m / unique, m_out = unique * freq;
    std::vector<uint64_t> src(m_out);
    for (uint64_t i = 0; i < m_out; ++i) src[i] = i / freq;
    std::shuffle(src.begin(), src.end(), g.gen);
    if (col_words)
        for (uint64_t j = 0; j < m_out; ++j) std::memcpy(col_words + j * W, gen.data() + src[j] * W, W * 8);
    return m_out;
}

// Bytes of every node's index as an sdsl rrr_vector<63> stream
// (sdsl_format.hpp's layout: size, block classes at 6 bits, the blocks'
// numbers, number-pointer and rank samples every 32 blocks, invert bits) --
// the reference's compressed index size (README.md:26-37 reports the files).
uint64_t oracle_rrr_bytes(OracleTree *t) {
    if (!t || !t->root) return 0;
    const auto &T = RRRVec::T();
    auto words = [](uint64_t bits) { return (bits + 63) / 64 * 8; };
    auto width = [](uint64_t v) -> uint64_t { return v ? 64 - __builtin_clzll(v) : 64; };
    uint64_t total = 0;
    std::vector<const Node *> all{t->root.get()};
    for (size_t h = 0; h < all.size(); ++h)
        for (auto &c : all[h]->children) all.push_back(c.get());
    for (const Node *nd : all) {
        const BitVec &bv = nd->nonzero_rows;
        const uint64_t size = bv.size, nb = (size + 63) / 63, ns = (nb + 31) / 32;
        uint64_t btnr = 0;
        for (uint64_t b = 0; b < nb; ++b) {
            const uint64_t p = b * 63;
            if (p >= size) break;
            const uint32_t len = (uint32_t)std::min<uint64_t>(63, size - p);
            uint64_t x = bv.words[p >> 6] >> (p & 63);
            if ((p & 63) && (p & 63) + len > 64) x |= bv.words[(p >> 6) + 1] << (64 - (p & 63));
            x &= (1ull << len) - 1;
            btnr += T.space[__builtin_popcountll(x)];
        }
        total += 8 + (9 + words(nb * 6)) + (8 + words(std::max<uint64_t>(btnr, 64))) + (9 + words(ns * width(btnr))) +
                 (9 + words((ns + 1) * width(bv.ones))) + (8 + words(ns));
    }
    return total;
}

OracleTree *oracle_generate_norepl(uint64_t n, uint64_t m, double d, uint32_t seed, int partitioner,
                                   uint32_t arity, uint64_t relax_max_arity) {
    try {
        std::vector<uint64_t> words(((n + 63) / 64) * m);
        oracle_generate_columns(n, m, d, seed, words.data());
        return oracle_build_from_columns(words.data(), n, m, partitioner, arity, relax_max_arity);
    } catch (...) {
        return nullptr;
    }
}

OracleTree *oracle_generate_topdown(uint64_t n, uint64_t m, double d, uint32_t arity, uint64_t seed, int threads) {
    if (arity < 2 || arity > 12) return nullptr;
    try {
        auto t = new OracleTree();
        t->root = generate_topdown(n, m, d, arity, seed, threads);
        return t;
    } catch (...) {
        return nullptr;
    }
}

void oracle_free(OracleTree *t) { delete t; }

uint64_t oracle_num_rows(const OracleTree *t) { return t->root->num_rows(); }
uint64_t oracle_num_columns(const OracleTree *t) { return t->root->num_columns(); }
uint64_t oracle_num_relations(const OracleTree *t) { return t->root->num_relations(); }
uint64_t oracle_num_nodes(const OracleTree *t) {
    uint64_t c = 0;
    t->root->bft([&](const Node &) { ++c; });
    return c;
}
double oracle_avg_arity(const OracleTree *t) {
    if (t->root->children.empty()) return 0;
    uint64_t nodes = 0, kids = 0;
    t->root->bft([&](const Node &n) {
        if (!n.children.empty()) {
            ++nodes;
            kids += n.children.size();
        }
    });
    return nodes ? (double)kids / nodes : 0;
}
uint64_t oracle_total_column_size(const OracleTree *t) {
    uint64_t s = 0;
    t->root->bft([&](const Node &n) { s += n.nonzero_rows.size; });
    return s;
}
uint64_t oracle_total_num_set_bits(const OracleTree *t) {
    uint64_t s = 0;
    t->root->bft([&](const Node &n) { s += n.nonzero_rows.ones; });
    return s;
}
static uint32_t depth_of(const Node &n) {
    uint32_t d = 0;
    for (auto &c : n.children) d = std::max(d, depth_of(*c));
    return d + 1;
}
uint32_t oracle_depth(const OracleTree *t) { return t->root->num_columns() ? depth_of(*t->root) : 0; }

int oracle_get(const OracleTree *t, uint64_t row, uint64_t col) {
    if (row >= t->root->num_rows() || col >= t->root->num_columns()) return -1;
    return t->root->get(row, col) ? 1 : 0;
}

uint64_t oracle_get_row(const OracleTree *t, uint64_t row, uint32_t *out, uint64_t cap, uint64_t *visits) {
    if (row >= t->root->num_rows()) return UINT64_MAX;
    std::vector<uint32_t> r;
    uint64_t v = 0;
    t->root->get_row(row, r, v);
    if (visits) *visits = v;
    for (uint64_t i = 0; i < r.size() && i < cap; ++i) out[i] = r[i];
    return r.size();
}

int oracle_get_rows(const OracleTree *t, const uint64_t *rows, uint64_t n, uint64_t *offsets, uint32_t *cols,
                    uint64_t cols_cap, uint64_t *cols_needed, uint32_t *visits, int threads) {
    const uint64_t R = t->root->num_rows();
    for (uint64_t i = 0; i < n; ++i)
        if (rows[i] >= R) return 2;
    threads = resolve_threads(threads);
    std::vector<std::vector<uint32_t>> res(n);
    const int64_t nn = (int64_t)n;
#pragma omp parallel for num_threads(threads) schedule(dynamic, 256)
    for (int64_t i = 0; i < nn; ++i) {
        uint64_t v = 0;
        t->root->get_row(rows[i], res[i], v);
        if (visits) visits[i] = (uint32_t)v;
    }
    uint64_t total = 0;
    offsets[0] = 0;
    for (uint64_t i = 0; i < n; ++i) {
        total += res[i].size();
        offsets[i + 1] = total;
    }
    if (cols_needed) *cols_needed = total;
    if (total > cols_cap) return 1;
    for (uint64_t i = 0; i < n; ++i) std::copy(res[i].begin(), res[i].end(), cols + offsets[i]);
    return 0;
}

uint64_t oracle_time_rows(const OracleTree *t, const uint64_t *rows, uint64_t n, int threads) {
    threads = resolve_threads(threads);
    uint64_t total = 0;
    const int64_t nn = (int64_t)n;
#pragma omp parallel num_threads(threads) reduction(+ : total)
    {
        std::vector<uint32_t> buf;
#pragma omp for schedule(dynamic, 64)
        for (int64_t i = 0; i < nn; ++i) {
            buf.clear();
            uint64_t v = 0;
            t->root->get_row(rows[i], buf, v);
            total += buf.size();
        }
    }
    return total;
}

uint64_t oracle_get_column(const OracleTree *t, uint64_t col, uint64_t *out, uint64_t cap) {
    if (col >= t->root->num_columns()) return UINT64_MAX;
    auto r = t->root->get_column(col);
    for (uint64_t i = 0; i < r.size() && i < cap; ++i) out[i] = r[i];
    return r.size();
}

uint32_t oracle_export_num_nodes(const OracleTree *t) {
    const_cast<OracleTree *>(t)->do_export();
    return (uint32_t)t->bfs.size();
}
void oracle_export(const OracleTree *t, uint32_t *num_children, uint32_t *first_child, uint32_t *leaf_column,
                   uint64_t *vec_size) {
    const_cast<OracleTree *>(t)->do_export();
    for (size_t u = 0; u < t->bfs.size(); ++u) {
        num_children[u] = t->num_children[u];
        first_child[u] = t->first_child[u];
        leaf_column[u] = t->leaf_column[u];
        vec_size[u] = t->vec_size[u];
    }
}
const uint64_t *oracle_export_vec_words(const OracleTree *t, uint32_t node) {
    const_cast<OracleTree *>(t)->do_export();
    return t->bfs.at(node)->nonzero_rows.words.data();
}

void oracle_generate_random_ints(uint64_t n, uint64_t begin, uint64_t end, uint32_t seed, uint64_t *out) {
    DataGenerator g;
    g.set_seed(seed);
    std::uniform_int_distribution<> dis(begin, end - 1);  // data_generation.cpp:12 (int!)
    for (uint64_t i = 0; i < n; ++i) out[i] = (uint64_t)dis(g.gen);
}

OracleBitVec *oracle_bv_new(const uint64_t *words, uint64_t size) {
    auto b = new OracleBitVec();
    b->bv = BitVec(size);
    if (size) std::memcpy(b->bv.words.data(), words, ((size + 63) / 64) * 8);
    b->bv.finalize();
    return b;
}
void oracle_bv_free(OracleBitVec *bv) { delete bv; }
uint64_t oracle_bv_rank1(const OracleBitVec *bv, uint64_t id) { return bv->bv.rank1(id); }
uint64_t oracle_bv_select1(const OracleBitVec *bv, uint64_t i) {
    if (i == 0 || i > bv->bv.ones) return UINT64_MAX;  // reference: assert (death test)
    return bv->bv.select1(i);
}
int oracle_bv_get(const OracleBitVec *bv, uint64_t id) { return id < bv->bv.size ? (int)bv->bv.get(id) : -1; }
uint64_t oracle_bv_num_set_bits(const OracleBitVec *bv) { return bv->bv.ones; }

uint64_t oracle_synth_hash(uint64_t seed, uint64_t key, uint64_t pos) { return synth_draw(synth_key(seed, key), pos); }

// Re-encode every node's index RRR-like (RRRVec) and drop the plain words:
// the CPU baseline's sdsl-like leg.  Afterwards only get / get_row /
// time_rows are valid on the tree.
void oracle_to_rrr(OracleTree *t, int threads) {
    std::vector<Node *> all{t->root.get()};
    for (size_t h = 0; h < all.size(); ++h)
        for (auto &c : all[h]->children) all.push_back(c.get());
    threads = resolve_threads(threads);
    const int64_t N = (int64_t)all.size();
#pragma omp parallel for num_threads(threads) schedule(dynamic, 1)
    for (int64_t i = 0; i < N; ++i) {
        Node *nd = all[i];
        nd->rrr = std::make_unique<RRRVec>(nd->nonzero_rows);
        std::vector<uint64_t>().swap(nd->nonzero_rows.words);
        std::vector<uint64_t>().swap(nd->nonzero_rows.super);
    }
}

struct OracleCSR {
    std::vector<uint64_t> offsets;
    std::vector<uint32_t> cols;
    uint64_t draws = 0;
};

OracleCSR *oracle_topdown_get_rows_shaped(uint64_t n, uint32_t num_nodes, const uint32_t *nc, const uint32_t *fc,
                                          const uint32_t *lc, double d, uint64_t seed, const uint64_t *rows, uint64_t nq,
                                          int threads, int *status) {
    auto shape = shape_from_arrays(num_nodes, nc, fc, lc);
    if (shape.empty()) {
        *status = 1;
        return nullptr;
    }
    auto r = new OracleCSR();
    *status = topdown_query_shape(n, shape, d, seed, rows, nq, threads, r->offsets, r->cols, &r->draws);
    if (*status != 0) {
        delete r;
        return nullptr;
    }
    return r;
}

OracleTree *oracle_generate_topdown_shaped(uint64_t n, uint32_t num_nodes, const uint32_t *nc, const uint32_t *fc,
                                           const uint32_t *lc, double d, uint64_t seed, int threads) {
    auto shape = shape_from_arrays(num_nodes, nc, fc, lc);
    if (shape.empty()) return nullptr;
    auto t = new OracleTree();
    t->root = generate_topdown_shape(n, shape, d, seed, resolve_threads(threads));
    return t;
}

OracleCSR *oracle_topdown_get_rows(uint64_t n, uint64_t m, double d, uint32_t arity, uint64_t seed,
                                   const uint64_t *rows, uint64_t nq, int threads, int *status) {
    auto r = new OracleCSR();
    *status = topdown_query(n, m, d, arity, seed, rows, nq, threads, r->offsets, r->cols, &r->draws);
    if (*status != 0) {
        delete r;
        return nullptr;
    }
    return r;
}
uint64_t oracle_csr_num_labels(const OracleCSR *r) { return r->cols.size(); }
uint64_t oracle_csr_draws(const OracleCSR *r) { return r->draws; }
void oracle_csr_copy(const OracleCSR *r, uint64_t *offsets, uint32_t *cols) {
    std::memcpy(offsets, r->offsets.data(), r->offsets.size() * 8);
    if (!r->cols.empty()) std::memcpy(cols, r->cols.data(), r->cols.size() * 4);
}
void oracle_csr_free(OracleCSR *r) { delete r; }

}  // extern "C"
