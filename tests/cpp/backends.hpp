// backends.hpp -- builds the same BRWT on the CPU oracle (test
// infrastructure) and, when a GPU is requested, on the device through the
// C ABI, behind the mirror's BinaryMatrix interface.
#pragma once
#include <cstring>
#include <memory>
#include <string>
#include <vector>

#include "../../genome_graph_annotation_amd/csrc/annotate_static.hpp"
#include "../../oracle/brwt_oracle.h"

using mbrwt_host::BinaryMatrix;

// dense column-major matrix -> LSB-first words per column
inline std::vector<uint64_t> pack_columns(const std::vector<std::vector<bool>> &cols, uint64_t n) {
    const uint64_t W = (n + 63) / 64;
    std::vector<uint64_t> w(std::max<uint64_t>(1, W * cols.size()), 0);
    for (size_t j = 0; j < cols.size(); ++j)
        for (uint64_t i = 0; i < n; ++i)
            if (cols[j][i]) w[j * W + i / 64] |= 1ull << (i % 64);
    return w;
}

// BinaryMatrix over the oracle (the CPU restatement of the reference BRWT)
class OracleMatrix : public BinaryMatrix {
  public:
    explicit OracleMatrix(OracleTree *t) : t_(t, oracle_free) {}
    uint64_t num_columns() const override { return oracle_num_columns(t_.get()); }
    uint64_t num_rows() const override { return oracle_num_rows(t_.get()); }
    uint64_t num_relations() const override { return oracle_num_relations(t_.get()); }
    bool get(Row r, Column c) const override {
        int v = oracle_get(t_.get(), r, c);
        if (v < 0) throw std::out_of_range("oracle get");
        return v == 1;
    }
    std::vector<Column> get_row(Row r) const override {
        std::vector<uint32_t> buf(std::max<uint64_t>(1, num_columns()));
        uint64_t cnt = oracle_get_row(t_.get(), r, buf.data(), buf.size(), nullptr);
        if (cnt == UINT64_MAX) throw std::out_of_range("oracle get_row");
        return std::vector<Column>(buf.begin(), buf.begin() + cnt);
    }
    std::vector<Row> get_column(Column c) const override {
        std::vector<uint64_t> buf(std::max<uint64_t>(1, num_rows()));
        uint64_t cnt = oracle_get_column(t_.get(), c, buf.data(), buf.size());
        if (cnt == UINT64_MAX) throw std::out_of_range("oracle get_column");
        return std::vector<Row>(buf.begin(), buf.begin() + cnt);
    }
    OracleTree *tree() const { return t_.get(); }

    // the oracle is built from columns, not read from streams
    bool load(std::istream &) override { return false; }
    // BRWT::serialize of the oracle's tree, through libmbrwt's host-side
    // writer (mbrwt_tree_serialize; no device involved)
    void serialize(std::ostream &out) const override;

  private:
    std::shared_ptr<OracleTree> t_;
};

// the oracle's tree as the C-ABI description (arrays held in `st`)
struct DescStorage {
    std::vector<uint32_t> nc, fc, lc;
    std::vector<uint64_t> vs;
    std::vector<const uint64_t *> words;
};
inline mbrwt_tree_desc oracle_desc(const OracleMatrix &m, DescStorage &st) {
    OracleTree *t = m.tree();
    const uint32_t N = oracle_export_num_nodes(t);
    st.nc.resize(N);
    st.fc.resize(N);
    st.lc.resize(N);
    st.vs.resize(N);
    st.words.resize(N);
    if (N) oracle_export(t, st.nc.data(), st.fc.data(), st.lc.data(), st.vs.data());
    for (uint32_t u = 0; u < N; ++u) st.words[u] = oracle_export_vec_words(t, u);
    mbrwt_tree_desc d{};
    d.num_rows = N ? oracle_num_rows(t) : 0;
    d.num_columns = N ? oracle_num_columns(t) : 0;
    d.num_nodes = N;
    d.num_children = st.nc.data();
    d.first_child = st.fc.data();
    d.leaf_column = st.lc.data();
    d.vec_size = st.vs.data();
    d.vec_words = st.words.data();
    return d;
}

inline void OracleMatrix::serialize(std::ostream &out) const {
    DescStorage st;
    const mbrwt_tree_desc d = oracle_desc(*this, st);
    uint64_t need = 0;
    mbrwt_tree_serialize(&d, nullptr, 0, &need);
    std::vector<uint8_t> buf(need);
    mbrwt_host::check_status(mbrwt_tree_serialize(&d, buf.data(), buf.size(), &need), "mbrwt_tree_serialize");
    out.write(reinterpret_cast<const char *>(buf.data()), (std::streamsize)buf.size());
}

// export the oracle's tree into the C-ABI description and build it on the device
inline mbrwt_host::BRWTDevice to_device(const OracleMatrix &m) {
    DescStorage st;
    const mbrwt_tree_desc d = oracle_desc(m, st);
    return mbrwt_host::BRWTDevice(d, 0);
}

inline OracleMatrix build_oracle(const std::vector<std::vector<bool>> &cols, uint64_t n, int partitioner = 0,
                                 uint32_t arity = 2, uint64_t relax = 0) {
    auto w = pack_columns(cols, n);
    return OracleMatrix(oracle_build_from_columns(w.data(), n, cols.size(), partitioner, arity, relax));
}

// the reference's ColumnCompressed label fixture -> (columns, encoder), as
// set_labels/add_labels encode labels in first-seen order
// (annotate_column_compressed.cpp:41-83)
struct LabelFixture {
    std::vector<std::vector<bool>> cols;
    mbrwt_host::LabelEncoder<std::string> enc;
    uint64_t n;
};
inline LabelFixture make_fixture(uint64_t n, const std::vector<std::pair<uint64_t, std::vector<std::string>>> &rows) {
    LabelFixture f;
    f.n = n;
    for (auto &r : rows)
        for (auto &l : r.second) f.enc.insert_and_encode(l);
    f.cols.assign(f.enc.size(), std::vector<bool>(n, false));
    for (auto &r : rows)
        for (auto &l : r.second) f.cols[f.enc.encode(l)][r.first] = true;
    return f;
}
