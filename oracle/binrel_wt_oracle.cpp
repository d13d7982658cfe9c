// binrel_wt_oracle.cpp -- CPU restatement of BinRelWT_sdsl (TEST
// INFRASTRUCTURE ONLY; see binrel_wt_oracle.h).
//
// Reference: annotation/bin_rel_wt/bin_rel_wt_sdsl.cpp (ratschlab/
// genome_graph_annotation).  The string of column ids (rows concatenated in
// generate_rows order) lives in a levelwise wavelet tree with the published
// algorithms of sdsl::wt_int: level l holds bit (L-1-l) of every symbol, the
// symbols ordered stably by their top l bits, so every tree node is one
// interval of its level; rank/select/interval_symbols descend and ascend
// through the node intervals with bit-vector rank/select.  The delimiter
// vector (a 1 before the first row and after every row, a 0 per relation) is
// a plain bit vector with the reference's rank1 (inclusive) / select1 /
// select0 (1-based) semantics (common/bit_vector.hpp:12-45).
#include "binrel_wt_oracle.h"

#include <omp.h>

#include <algorithm>
#include <chrono>
#include <cstring>
#include <vector>

namespace {

inline uint64_t popc(uint64_t x) { return (uint64_t)__builtin_popcountll(x); }

// plain bit vector: exclusive rank (ones in [0, i)), 1-based select
struct Bits {
    uint64_t n = 0;
    std::vector<uint64_t> w;
    std::vector<uint64_t> cum;  // ones before word k
    uint64_t ones = 0;

    void init(uint64_t size) {
        n = size;
        w.assign((size + 63) / 64 + 1, 0);
    }
    void set(uint64_t i) { w[i >> 6] |= 1ull << (i & 63); }
    bool get(uint64_t i) const { return (w[i >> 6] >> (i & 63)) & 1; }
    void finalize() {
        cum.assign(w.size() + 1, 0);
        for (size_t k = 0; k < w.size(); ++k) cum[k + 1] = cum[k] + popc(w[k]);
        ones = cum[(n + 63) / 64];
        if (n & 63) ones = cum[n >> 6] + popc(w[n >> 6] & ((1ull << (n & 63)) - 1));
    }
    uint64_t rank1(uint64_t i) const {  // ones in [0, i)
        if (i >= n) return ones;
        return cum[i >> 6] + ((i & 63) ? popc(w[i >> 6] & ((1ull << (i & 63)) - 1)) : 0);
    }
    uint64_t rank0(uint64_t i) const { return std::min(i, n) - rank1(i); }
    // position of the k-th one / zero (1-based k)
    uint64_t select1(uint64_t k) const {
        uint64_t lo = 0, hi = (n + 63) / 64;  // last word with cum < k
        while (hi - lo > 1) {
            uint64_t mid = (lo + hi) / 2;
            if (cum[mid] < k) lo = mid;
            else hi = mid;
        }
        uint64_t x = w[lo], r = k - cum[lo];
        while (--r) x &= x - 1;
        return lo * 64 + (uint64_t)__builtin_ctzll(x);
    }
    uint64_t select0(uint64_t k) const {
        uint64_t lo = 0, hi = (n + 63) / 64;
        while (hi - lo > 1) {
            uint64_t mid = (lo + hi) / 2;
            if (mid * 64 - cum[mid] < k) lo = mid;
            else hi = mid;
        }
        uint64_t x = ~w[lo], r = k - (lo * 64 - cum[lo]);
        while (--r) x &= x - 1;
        return lo * 64 + (uint64_t)__builtin_ctzll(x);
    }
};

// levelwise wavelet tree over symbols < 2^L (sdsl::wt_int semantics)
struct WaveletTree {
    uint64_t n = 0;
    uint32_t L = 1;
    std::vector<Bits> lev;

    void build(std::vector<uint32_t> seq, uint32_t levels) {
        n = seq.size();
        L = levels;
        lev.assign(L, Bits());
        std::vector<uint32_t> next(n);
        for (uint32_t l = 0; l < L; ++l) {
            const uint32_t sh = L - 1 - l;
            lev[l].init(n);
            for (uint64_t i = 0; i < n; ++i)
                if ((seq[i] >> sh) & 1) lev[l].set(i);
            lev[l].finalize();
            // stable partition inside every node interval (= stable sort by the top l+1 bits)
            uint64_t i = 0;
            while (i < n) {
                const uint32_t prefix = l ? (seq[i] >> (sh + 1)) : 0;
                uint64_t e = i;
                while (e < n && (l ? (seq[e] >> (sh + 1)) : 0) == prefix) ++e;
                uint64_t o = i;
                for (uint64_t k = i; k < e; ++k)
                    if (!((seq[k] >> sh) & 1)) next[o++] = seq[k];
                for (uint64_t k = i; k < e; ++k)
                    if ((seq[k] >> sh) & 1) next[o++] = seq[k];
                i = e;
            }
            seq.swap(next);
        }
    }

    // occurrences of c in [0, i)
    uint64_t rank(uint64_t i, uint32_t c) const {
        if (c >> L) return 0;
        uint64_t s0 = 0, size = n, pos = std::min(i, n);
        for (uint32_t l = 0; l < L; ++l) {
            const Bits &B = lev[l];
            const uint64_t ob = B.rank1(s0), op = B.rank1(s0 + pos) - ob, on = B.rank1(s0 + size) - ob;
            if ((c >> (L - 1 - l)) & 1) {
                s0 += size - on;
                size = on;
                pos = op;
            } else {
                size -= on;
                pos -= op;
            }
        }
        return pos;
    }

    // position of the k-th c (1-based)
    uint64_t select(uint64_t k, uint32_t c) const {
        std::vector<uint64_t> start(L);
        uint64_t s0 = 0, size = n;
        for (uint32_t l = 0; l < L; ++l) {
            start[l] = s0;
            const Bits &B = lev[l];
            const uint64_t ob = B.rank1(s0), on = B.rank1(s0 + size) - ob;
            if ((c >> (L - 1 - l)) & 1) {
                s0 += size - on;
                size = on;
            } else {
                size -= on;
            }
        }
        uint64_t pos = k - 1;  // inside the leaf interval
        for (uint32_t l = L; l-- > 0;) {
            const Bits &B = lev[l];
            if ((c >> (L - 1 - l)) & 1) pos = B.select1(B.rank1(start[l]) + pos + 1) - start[l];
            else pos = B.select0(B.rank0(start[l]) + pos + 1) - start[l];
        }
        return pos;
    }

    // distinct symbols of [i, j), ascending (sdsl wt_int::interval_symbols)
    void interval_symbols(uint64_t i, uint64_t j, std::vector<uint32_t> &out) const {
        rec(0, 0, n, i, j, 0, out);
    }
    void rec(uint32_t l, uint64_t s0, uint64_t size, uint64_t i, uint64_t j, uint32_t prefix,
             std::vector<uint32_t> &out) const {
        if (i >= j) return;
        if (l == L) {
            out.push_back(prefix);
            return;
        }
        const Bits &B = lev[l];
        const uint64_t ob = B.rank1(s0), oi = B.rank1(s0 + i) - ob, oj = B.rank1(s0 + j) - ob,
                       on = B.rank1(s0 + size) - ob;
        rec(l + 1, s0, size - on, i - oi, j - oj, prefix << 1, out);
        rec(l + 1, s0 + size - on, on, oi, oj, (prefix << 1) | 1, out);
    }
};

inline uint64_t mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

uint32_t code_length(uint64_t a) { return a ? 64 - (uint32_t)__builtin_clzll(a) : 1; }  // utils.cpp:276-278

}  // namespace

struct OracleWT {
    uint64_t num_columns = 0;
    WaveletTree wt;
    Bits delim;  // bin_rel_wt_sdsl.cpp:19-34

    uint64_t num_rows() const { return delim.ones - 1; }

    // bin_rel_wt_sdsl.cpp:51-83
    void get_row(uint64_t row, std::vector<uint32_t> &out) const {
        const uint64_t first = delim.select1(row + 1) - row;
        const uint64_t last = delim.select1(row + 2) - (row + 1);
        out.clear();
        wt.interval_symbols(first, last, out);
        out.resize(last - first, 0);  // label_indices is sized (last - first)
    }
};

extern "C" {

OracleWT *wt_oracle_empty(void) {
    OracleWT *t = new OracleWT();
    t->delim.init(1);
    t->delim.set(0);
    t->delim.finalize();
    t->wt.build({}, 1);
    return t;
}

OracleWT *wt_oracle_build(const uint64_t *offsets, const uint32_t *cols, uint64_t num_rows, uint64_t num_columns) {
    const uint64_t nrel = num_rows ? offsets[num_rows] : 0;
    std::vector<uint32_t> flat(nrel);
    for (uint64_t i = 0; i < nrel; ++i) {
        if (cols[i] >= num_columns) return nullptr;
        flat[i] = cols[i];
    }
    OracleWT *t = new OracleWT();
    t->num_columns = num_columns;
    t->delim.init(nrel + num_rows + 1);
    uint64_t pos = 0;
    t->delim.set(pos++);
    for (uint64_t r = 0; r < num_rows; ++r) {
        pos += offsets[r + 1] - offsets[r];
        t->delim.set(pos++);
    }
    t->delim.finalize();
    // sdsl int_vector width code_length(num_columns) (bin_rel_wt_sdsl.cpp:14)
    t->wt.build(std::move(flat), code_length(num_columns));
    return t;
}

void wt_oracle_free(OracleWT *t) { delete t; }

uint64_t wt_oracle_num_rows(const OracleWT *t) { return t->num_rows(); }
uint64_t wt_oracle_num_columns(const OracleWT *t) { return t->num_columns; }
uint64_t wt_oracle_num_relations(const OracleWT *t) { return t->wt.n; }

uint64_t wt_oracle_get_row(const OracleWT *t, uint64_t row, uint32_t *out, uint64_t cap) {
    if (row >= t->num_rows()) return UINT64_MAX;
    std::vector<uint32_t> v;
    t->get_row(row, v);
    for (uint64_t i = 0; i < v.size() && i < cap; ++i) out[i] = v[i];
    return v.size();
}

int wt_oracle_get(const OracleWT *t, uint64_t row, uint64_t col) {
    if (row >= t->num_rows() || col >= t->num_columns) return -1;
    const uint64_t first = t->delim.select1(row + 1) - row;
    const uint64_t last = t->delim.select1(row + 2) - row - 1;
    // sdsl rank is exclusive (bin_rel_wt_sdsl.cpp:105-108)
    return first == 0 ? t->wt.rank(last, (uint32_t)col) != 0
                      : t->wt.rank(first, (uint32_t)col) != t->wt.rank(last, (uint32_t)col);
}

uint64_t wt_oracle_get_column(const OracleWT *t, uint64_t col, uint64_t *out, uint64_t cap) {
    if (col >= t->num_columns) return UINT64_MAX;
    const uint64_t cnt = t->wt.rank(t->wt.n, (uint32_t)col);
    for (uint64_t i = 0; i < cnt; ++i) {
        const uint64_t in_wt = t->wt.select(i + 1, (uint32_t)col);
        const uint64_t in_del = t->delim.select0(in_wt + 1);
        const uint64_t row = (t->delim.rank1(in_del) + (t->delim.get(in_del) ? 1 : 0)) - 1;  // inclusive rank1
        if (i < cap) out[i] = row;
    }
    return cnt;
}

int wt_oracle_get_rows(const OracleWT *t, const uint64_t *rows, uint64_t n, uint64_t *offsets, uint32_t *cols,
                       uint64_t cols_cap, uint64_t *cols_needed, int num_threads) {
    const uint64_t R = t->num_rows();
    for (uint64_t i = 0; i < n; ++i)
        if (rows[i] >= R) return 2;
    offsets[0] = 0;
    for (uint64_t i = 0; i < n; ++i) {
        const uint64_t r = rows[i];
        const uint64_t len = (t->delim.select1(r + 2) - (r + 1)) - (t->delim.select1(r + 1) - r);
        offsets[i + 1] = offsets[i] + len;
    }
    if (cols_needed) *cols_needed = offsets[n];
    if (offsets[n] > cols_cap) return 1;
    if (num_threads <= 0) num_threads = omp_get_max_threads();
#pragma omp parallel num_threads(num_threads)
    {
        std::vector<uint32_t> v;
#pragma omp for schedule(dynamic, 256)
        for (int64_t i = 0; i < (int64_t)n; ++i) {
            t->get_row(rows[i], v);
            std::copy(v.begin(), v.end(), cols + offsets[i]);
        }
    }
    return 0;
}

double wt_oracle_time_rows(const OracleWT *t, const uint64_t *rows, uint64_t n, int num_threads) {
    if (num_threads <= 0) num_threads = omp_get_max_threads();
    uint64_t sink = 0;
    const auto t0 = std::chrono::steady_clock::now();
#pragma omp parallel num_threads(num_threads) reduction(+ : sink)
    {
        std::vector<uint32_t> v;
#pragma omp for schedule(dynamic, 256)
        for (int64_t i = 0; i < (int64_t)n; ++i) {
            t->get_row(rows[i], v);
            sink += v.size();
        }
    }
    const auto t1 = std::chrono::steady_clock::now();
    if (sink == 0xFFFFFFFFFFFFFFFFull) return -1;
    return std::chrono::duration<double>(t1 - t0).count();
}

uint64_t wt_synth_threshold(double density) {
    if (density <= 0) return 0;
    if (density >= 1) return UINT64_MAX;
    return (uint64_t)(density * 18446744073709551616.0);
}

uint64_t wt_synth_row(uint64_t row, uint64_t num_columns, uint64_t threshold, uint64_t seed, uint32_t *out,
                      uint64_t cap) {
    const uint64_t K = mix64(seed ^ ((row + 1) * 0x9E3779B97F4A7C15ull));
    uint64_t cnt = 0;
    for (uint64_t c = 0; c < num_columns; ++c) {
        const uint64_t h = mix64(K + c * 0xD1B54A32D192ED03ull);
        if (threshold == UINT64_MAX || h < threshold) {
            if (cnt < cap) out[cnt] = (uint32_t)c;
            ++cnt;
        }
    }
    return cnt;
}

int wt_synth_rows(uint64_t row0, uint64_t n, uint64_t num_columns, double density, uint64_t seed, uint64_t *offsets,
                  uint32_t *cols, uint64_t cols_cap, uint64_t *cols_needed, int num_threads) {
    const uint64_t T = wt_synth_threshold(density);
    if (num_threads <= 0) num_threads = omp_get_max_threads();
    std::vector<uint64_t> cnt(n);
#pragma omp parallel for num_threads(num_threads) schedule(dynamic, 1024)
    for (int64_t i = 0; i < (int64_t)n; ++i) cnt[i] = wt_synth_row(row0 + i, num_columns, T, seed, nullptr, 0);
    offsets[0] = 0;
    for (uint64_t i = 0; i < n; ++i) offsets[i + 1] = offsets[i] + cnt[i];
    if (cols_needed) *cols_needed = offsets[n];
    if (offsets[n] > cols_cap) return 1;
#pragma omp parallel for num_threads(num_threads) schedule(dynamic, 1024)
    for (int64_t i = 0; i < (int64_t)n; ++i)
        wt_synth_row(row0 + i, num_columns, T, seed, cols + offsets[i], cnt[i]);
    return 0;
}

int wt_synth_rows_at(const uint64_t *rows, uint64_t n, uint64_t num_columns, double density, uint64_t seed,
                     uint64_t *offsets, uint32_t *cols, uint64_t cols_cap, uint64_t *cols_needed,
                     int num_threads) {
    const uint64_t T = wt_synth_threshold(density);
    if (num_threads <= 0) num_threads = omp_get_max_threads();
    std::vector<uint64_t> cnt(n);
#pragma omp parallel for num_threads(num_threads) schedule(dynamic, 1024)
    for (int64_t i = 0; i < (int64_t)n; ++i) cnt[i] = wt_synth_row(rows[i], num_columns, T, seed, nullptr, 0);
    offsets[0] = 0;
    for (uint64_t i = 0; i < n; ++i) offsets[i + 1] = offsets[i] + cnt[i];
    if (cols_needed) *cols_needed = offsets[n];
    if (offsets[n] > cols_cap) return 1;
#pragma omp parallel for num_threads(num_threads) schedule(dynamic, 1024)
    for (int64_t i = 0; i < (int64_t)n; ++i) wt_synth_row(rows[i], num_columns, T, seed, cols + offsets[i], cnt[i]);
    return 0;
}

}  // extern "C"
