// tests/test_bin_rel_wt_sdsl.cpp (reference) through the C++ mirror's
// BinaryMatrix interface: the BinRel-WT oracle (CPU restatement of
// BinRelWT_sdsl) or the device engine (argv[1] = oracle | device).
#include <algorithm>
#include <functional>
#include <set>
#include <sstream>

#include "../../genome_graph_annotation_amd/csrc/binrel_wt_device.hpp"
#include "../../oracle/binrel_wt_oracle.h"
#include "minitest.hpp"

using mbrwt_host::BinaryMatrix;

static bool g_device = false;
typedef std::vector<std::vector<bool>> Rows;  // rows[r][c]

class OracleWTMatrix : public BinaryMatrix {
  public:
    OracleWTMatrix(OracleWT *t) : t_(t, wt_oracle_free) {}
    uint64_t num_columns() const override { return wt_oracle_num_columns(t_.get()); }
    uint64_t num_rows() const override { return wt_oracle_num_rows(t_.get()); }
    uint64_t num_relations() const override { return wt_oracle_num_relations(t_.get()); }
    bool load(std::istream &) override { return false; }
    void serialize(std::ostream &) const override { throw std::runtime_error("not supported"); }
    bool get(Row r, Column c) const override {
        int v = wt_oracle_get(t_.get(), r, c);
        if (v < 0) throw std::out_of_range("oracle get");
        return v == 1;
    }
    std::vector<Column> get_row(Row r) const override {
        std::vector<uint32_t> buf(num_columns() + 1);
        uint64_t n = wt_oracle_get_row(t_.get(), r, buf.data(), buf.size());
        if (n == UINT64_MAX) throw std::out_of_range("oracle get_row");
        return std::vector<Column>(buf.begin(), buf.begin() + n);
    }
    std::vector<Row> get_column(Column c) const override {
        std::vector<uint64_t> buf(num_rows() + 1);
        uint64_t n = wt_oracle_get_column(t_.get(), c, buf.data(), buf.size());
        if (n == UINT64_MAX) throw std::out_of_range("oracle get_column");
        return std::vector<Row>(buf.begin(), buf.begin() + n);
    }

  private:
    std::shared_ptr<OracleWT> t_;
};

// BinRelWT_sdsl(generate_rows, num_set_bits, num_columns) on either backend
static std::shared_ptr<BinaryMatrix> build(const Rows &rows, uint64_t num_columns) {
    auto generate = [&](const std::function<void(const std::vector<uint64_t> &)> &callback) {
        for (const auto &row : rows) {
            std::vector<uint64_t> idx;
            for (size_t c = 0; c < row.size(); ++c)
                if (row[c]) idx.push_back(c);
            callback(idx);
        }
    };
    uint64_t nrel = 0;
    for (const auto &row : rows) nrel += std::count(row.begin(), row.end(), true);
    if (g_device) return std::make_shared<mbrwt_host::BinRelWTDevice>(generate, nrel, num_columns);
    std::vector<uint64_t> off{0};
    std::vector<uint32_t> cols;
    generate([&](const std::vector<uint64_t> &idx) {
        for (auto c : idx) cols.push_back((uint32_t)c);
        off.push_back(cols.size());
    });
    cols.push_back(0);
    return std::make_shared<OracleWTMatrix>(wt_oracle_build(off.data(), cols.data(), rows.size(), num_columns));
}

// test_bin_rel_wt_sdsl (test_bin_rel_wt_sdsl.cpp:27-84)
static void check(const BinaryMatrix &m, const Rows &rows, uint64_t num_columns) {
    ASSERT_EQ(rows.size(), m.num_rows());
    if (rows.empty()) {
        ASSERT_EQ(0u, m.num_columns());
        return;
    }
    ASSERT_EQ(num_columns, m.num_columns());
    for (size_t j = 0; j < m.num_rows(); ++j) {
        auto bits = m.get_row(j);
        std::set<uint64_t> s(bits.begin(), bits.end());
        ASSERT_EQ(bits.size(), s.size());
        ASSERT_EQ((size_t)std::count(rows[j].begin(), rows[j].end(), true), bits.size());
        for (auto i : bits) {
            ASSERT_TRUE(i < m.num_columns());
            EXPECT_TRUE(rows[j][i]);
        }
        EXPECT_TRUE(std::is_sorted(bits.begin(), bits.end()));  // interval_symbols order
    }
    for (size_t i = 0; i < m.num_columns(); ++i) {
        auto bits = m.get_column(i);
        std::set<uint64_t> s(bits.begin(), bits.end());
        ASSERT_EQ(bits.size(), s.size());
        for (auto j : bits) {
            ASSERT_TRUE(j < m.num_rows());
            EXPECT_TRUE(rows[j][i]);
        }
        for (size_t j = 0; j < rows.size(); ++j) EXPECT_EQ((bool)rows[j][i], (bool)s.count(j));
    }
    for (size_t i = 0; i < m.num_rows(); ++i)
        for (size_t j = 0; j < m.num_columns(); ++j) EXPECT_EQ((bool)rows[i][j], m.get(i, j));
}

TEST(BinRelWT_sdsl, EmptyConstructor) {  // test_bin_rel_wt_sdsl.cpp:15-25
    auto m = build({}, 0);
    EXPECT_EQ(0u, m->num_columns());
    EXPECT_EQ(0u, m->num_rows());
}
TEST(BinRelWT_sdsl, AllZero) {  // :86-112
    for (size_t nc = 1; nc < 20; ++nc)
        for (size_t nr = 1; nr < 20; ++nr) {
            Rows rows(nr, std::vector<bool>(nc, false));
            check(*build(rows, nc), rows, nc);
        }
}
TEST(BinRelWT_sdsl, AllOne) {  // :114-141
    for (size_t nc = 1; nc < 10; ++nc)
        for (size_t nr = 1; nr < 10; ++nr) {
            Rows rows(nr, std::vector<bool>(nc, true));
            check(*build(rows, nc), rows, nc);
        }
}
TEST(BinRelWT_sdsl, AllMixed) {  // :143-176, first and last columns all zero
    for (size_t nc = 1; nc < 10; ++nc)
        for (size_t nr = 1; nr < 10; ++nr) {
            Rows rows(nr, std::vector<bool>(nc, false));
            for (size_t j = 0; j < nr; ++j)
                for (size_t i = 1; i + 1 < nc; ++i) rows[j][i] = (i + j) % 2;
            check(*build(rows, nc), rows, nc);
        }
}
TEST(BinRelWT_sdsl, OutOfRange) {  // an assert / UB in the reference; the mirror throws
    Rows rows(3, std::vector<bool>(4, true));
    auto m = build(rows, 4);
    EXPECT_THROW(m->get_row(3), std::out_of_range);
    EXPECT_THROW(m->get(0, 4), std::out_of_range);
    EXPECT_THROW(m->get_column(4), std::out_of_range);
}

// test_serialization (test_bin_rel_wt_sdsl.cpp:182-208) on the device mirror
// (the oracle has no stream): dump, a bad stream does not load, the dump
// loads back with the same shape and columns.  Byte layout parity unpinned.
static void check_serialization(const BinaryMatrix &m) {
    std::stringstream good;
    m.serialize(good);
    {
        mbrwt_host::BinRelWTDevice loaded;
        std::stringstream bad("not a BinRelWT stream");
        ASSERT_TRUE(!loaded.load(bad));
    }
    mbrwt_host::BinRelWTDevice loaded;
    ASSERT_TRUE(loaded.load(good));
    ASSERT_TRUE(good.good());
    ASSERT_EQ(m.num_columns(), loaded.num_columns());
    ASSERT_EQ(m.num_rows(), loaded.num_rows());
    for (size_t j = 0; j < loaded.num_columns(); ++j) EXPECT_EQ(m.get_column(j), loaded.get_column(j));
}
TEST(BinRelWT_sdsl, Serialization) {  // :210-272: empty, all zero, all one, mixed
    if (!g_device) return;
    check_serialization(mbrwt_host::BinRelWTDevice());
    for (size_t nc = 1; nc < 8; ++nc)
        for (size_t nr = 1; nr < 8; nr += 2) {
            Rows zero(nr, std::vector<bool>(nc, false)), one(nr, std::vector<bool>(nc, true)), mixed = zero;
            for (size_t j = 0; j < nr; ++j)
                for (size_t i = 1; i + 1 < nc; ++i) mixed[j][i] = (i + j) % 2;
            check_serialization(*build(zero, nc));
            check_serialization(*build(one, nc));
            check_serialization(*build(mixed, nc));
        }
}

int main(int argc, char **argv) {
    g_device = argc > 1 && std::string(argv[1]) == "device";
    return minitest::run_all(argc > 2 ? argv[2] : nullptr);
}
