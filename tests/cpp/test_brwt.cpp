// Grid tests of tests/test_BRWT.cpp:92-212 and tests/test_BRWT_optimizer.cpp
// (reference) through the C++ mirror's BinaryMatrix interface, on the
// backend named by argv[1] (oracle | device).
#include <algorithm>
#include <fstream>
#include <iterator>
#include <set>
#include <sstream>

#include "backends.hpp"
#include "minitest.hpp"

static bool g_device = false;

typedef std::vector<std::vector<bool>> Columns;

static std::shared_ptr<BinaryMatrix> build(const Columns &cols, uint64_t n, uint64_t relax = 0) {
    auto om = std::make_shared<OracleMatrix>(build_oracle(cols, n, 0, 2, relax));
    if (!g_device) return om;
    return std::make_shared<mbrwt_host::BRWTDevice>(to_device(*om));
}

// test_brwt (test_BRWT.cpp:92-150)
static void test_brwt(const BinaryMatrix &m, const Columns &columns, uint64_t n) {
    ASSERT_EQ(columns.size(), m.num_columns());
    if (columns.empty()) {
        ASSERT_EQ(0u, m.num_rows());
        return;
    }
    ASSERT_EQ(n, m.num_rows());
    for (size_t j = 0; j < m.num_columns(); ++j) {  // get_column (test_BRWT.cpp:105-123)
        auto bits = m.get_column(j);
        std::set<uint64_t> s(bits.begin(), bits.end());
        ASSERT_EQ(bits.size(), s.size());
        uint64_t ones = 0;
        for (uint64_t i = 0; i < n; ++i) ones += columns[j][i];
        ASSERT_EQ(ones, bits.size());
        for (auto i : bits) {
            ASSERT_TRUE(i < m.num_rows());
            ASSERT_TRUE(columns[j][i]);
        }
        EXPECT_TRUE(std::is_sorted(bits.begin(), bits.end()));
    }
    std::vector<uint64_t> all(n);
    for (uint64_t i = 0; i < n; ++i) all[i] = i;
    auto rows = m.get_rows(all);
    for (uint64_t i = 0; i < n; ++i) {
        auto &r = rows[i];
        std::set<uint64_t> s(r.begin(), r.end());
        ASSERT_EQ(r.size(), s.size());  // unique
        for (auto j : r) {
            ASSERT_TRUE(j < m.num_columns());
            EXPECT_TRUE(columns[j][i]);
        }
        for (size_t j = 0; j < columns.size(); ++j) EXPECT_EQ((bool)columns[j][i], (bool)s.count(j));
        EXPECT_EQ(r, m.get_row(i));  // batched == single
    }
    for (uint64_t i = 0; i < n; ++i)
        for (size_t j = 0; j < columns.size(); ++j) EXPECT_EQ((bool)columns[j][i], m.get(i, j));
}

static void grid(int kind, uint64_t relax) {
    for (uint64_t n = 1; n < 20; ++n) {
        for (size_t mcols = 1; mcols < 20; ++mcols) {
            Columns cols(mcols, std::vector<bool>(n));
            uint64_t ones = 0;
            for (size_t j = 0; j < mcols; ++j)
                for (uint64_t i = 0; i < n; ++i) {
                    bool b = kind == 0 ? false : kind == 1 ? true : ((i + 2 * j) % 2) != 0;  // test_BRWT.cpp:200
                    cols[j][i] = b;
                    ones += b;
                }
            auto m = build(cols, n, relax);
            EXPECT_EQ(ones, m->num_relations());
            test_brwt(*m, cols, n);
        }
    }
}

// a clone (mbrwt_ctx_clone) answers like its source, before and after the
// source is destroyed (device backend only; the oracle has no clones)
TEST(BRWT, CloneAnswersLikeSource) {
    if (!g_device) return;
    for (int kind = 0; kind < 3; ++kind) {
        const uint64_t n = 19;
        Columns cols(13, std::vector<bool>(n));
        for (size_t j = 0; j < cols.size(); ++j)
            for (uint64_t i = 0; i < n; ++i) cols[j][i] = kind == 0 ? false : kind == 1 ? true : ((i + 2 * j) % 2) != 0;
        auto src = std::make_shared<mbrwt_host::BRWTDevice>(
            to_device(OracleMatrix(build_oracle(cols, n, 0, 2, 0))));
        mbrwt_host::BRWTDevice cl = src->clone();
        test_brwt(cl, cols, n);
        src.reset();  // the image lives on in the clone
        test_brwt(cl, cols, n);
        test_brwt(cl.clone(), cols, n);
    }
}

TEST(BRWT, EmptyConstructor) {  // test_BRWT.cpp:15-25
    auto m = build({}, 0);
    EXPECT_EQ(0u, m->num_columns());
    EXPECT_EQ(0u, m->num_rows());
    EXPECT_THROW(m->get_row(0), std::out_of_range);
}
TEST(BRWT, BuildBottomUPOneColumn) {  // test_BRWT.cpp:27-35
    auto m = build({std::vector<bool>(10, true)}, 10);
    EXPECT_EQ(1u, m->num_columns());
    EXPECT_EQ(10u, m->num_rows());
    EXPECT_EQ(std::vector<uint64_t>({0}), m->get_row(3));
}
TEST(BRWT, OutOfRange) {  // the reference asserts (BRWT.cpp:27); the mirror throws
    auto m = build({std::vector<bool>(10, true)}, 10);
    EXPECT_THROW(m->get_row(10), std::out_of_range);
    EXPECT_THROW(m->get(0, 1), std::out_of_range);
    EXPECT_THROW(m->get_column(1), std::out_of_range);
}
// the same grids built from their columns by the device builder
// (mbrwt_create_from_columns); device backend only
static void grid_device_built(int kind, uint64_t relax = 0, bool greedy = false) {
    if (!g_device) return;
    for (uint64_t n = 1; n < 20; ++n) {
        for (size_t mcols = 1; mcols < 20; ++mcols) {
            Columns cols(mcols, std::vector<bool>(n));
            std::vector<std::vector<uint64_t>> words(mcols, std::vector<uint64_t>((n + 63) / 64, 0));
            uint64_t ones = 0;
            for (size_t j = 0; j < mcols; ++j)
                for (uint64_t i = 0; i < n; ++i) {
                    bool b = kind == 0 ? false : kind == 1 ? true : ((i + 2 * j) % 2) != 0;
                    cols[j][i] = b;
                    ones += b;
                    if (b) words[j][i / 64] |= 1ull << (i % 64);
                }
            auto m = greedy ? mbrwt_host::BRWTDevice::build_greedy(words, n, 0, relax)
                            : mbrwt_host::BRWTDevice::build_bottom_up(words, n, 2, 0, relax);
            EXPECT_EQ(ones, m.num_relations());
            // same shape as the reference builder's tree (the oracle's restatement)
            auto om = OracleMatrix(build_oracle(cols, n, greedy ? 1 : 0, 2, relax));
            EXPECT_EQ(om.num_relations(), m.num_relations());
            EXPECT_EQ(to_device(om).num_nodes(), m.num_nodes());
            test_brwt(m, cols, n);
        }
    }
}
// the grids on two replicas of one device (mbrwt_multi_*: slices of the
// batch on each replica, reassembled into one CSR); device backend only
static void grid_multi(int kind) {
    if (!g_device) return;
    for (uint64_t n = 1; n < 20; ++n) {
        for (size_t mcols = 1; mcols < 20; ++mcols) {
            Columns cols(mcols, std::vector<bool>(n));
            for (size_t j = 0; j < mcols; ++j)
                for (uint64_t i = 0; i < n; ++i) cols[j][i] = kind == 0 ? false : kind == 1 ? true : ((i + 2 * j) % 2) != 0;
            auto om = OracleMatrix(build_oracle(cols, n, 0, 2, 0));
            DescStorage st;
            const mbrwt_tree_desc d = oracle_desc(om, st);
            mbrwt_host::BRWTMultiDevice m(d, {0, 0});
            EXPECT_EQ(2, m.replicas());
            test_brwt(m, cols, n);
            std::vector<uint64_t> rows;
            for (uint64_t i = 0; i < n; ++i) rows.push_back(n - 1 - i);
            const auto got = m.get_rows(rows);
            for (size_t i = 0; i < rows.size(); ++i) EXPECT_TRUE(got[i] == om.get_row(rows[i]));
        }
    }
}
TEST(MultiDevice, AllZero) { grid_multi(0); }
TEST(MultiDevice, AllOne) { grid_multi(1); }
TEST(MultiDevice, AllMixed) { grid_multi(2); }
TEST(BRWT, DeviceBuilderAllZero) { grid_device_built(0); }
TEST(BRWT, DeviceBuilderAllOne) { grid_device_built(1); }
TEST(BRWT, DeviceBuilderAllMixed) { grid_device_built(2); }
TEST(BRWT, BuildBottomUPAllZero) { grid(0, 0); }
TEST(BRWT, BuildBottomUPAllOne) { grid(1, 0); }
TEST(BRWT, BuildBottomUPAllMixed) { grid(2, 0); }
TEST(BRWTOptimizer, BuildBottomUPAllZero) { grid(0, UINT64_MAX); }
TEST(BRWTOptimizer, BuildBottomUPAllOne) { grid(1, UINT64_MAX); }
TEST(BRWTOptimizer, BuildBottomUPAllMixed) { grid(2, UINT64_MAX); }
// binary_grouping_greedy on the device (MBRWT_PARTITIONER_GREEDY) over the
// same grids (test_BRWT.cpp:152-212), against the oracle's greedy tree
TEST(BRWT, DeviceGreedyBuilderAllZero) { grid_device_built(0, 0, true); }
TEST(BRWT, DeviceGreedyBuilderAllOne) { grid_device_built(1, 0, true); }
TEST(BRWT, DeviceGreedyBuilderAllMixed) { grid_device_built(2, 0, true); }
TEST(BRWTOptimizer, DeviceGreedyBuilderAllMixed) { grid_device_built(2, UINT64_MAX, true); }
// BRWTOptimizer::relax on the device (mbrwt_create_from_columns_relaxed)
TEST(BRWTOptimizer, DeviceBuilderAllZero) { grid_device_built(0, UINT64_MAX); }
TEST(BRWTOptimizer, DeviceBuilderAllOne) { grid_device_built(1, UINT64_MAX); }
TEST(BRWTOptimizer, DeviceBuilderAllMixed) { grid_device_built(2, UINT64_MAX); }

// test_serialization (test_BRWT.cpp:214-238) over the grids: the dumped
// matrix loads back (stream still good) with the same shape and every column;
// a bad stream does not load.  The oracle's tree is dumped by the host-side
// writer; oracle backend: the stream parses back to the oracle's own tree;
// device backend: BRWTDevice::load puts it in HBM and is queried, then the
// device matrix is dumped and loaded again.
static void grid_serialization(int kind, uint64_t relax) {
    const std::string good = "/tmp/mbrwt_test_brwt_dump_good", bad = "/tmp/mbrwt_test_brwt_dump_bad_missing";
    for (uint64_t n = 1; n < 20; n += 3) {
        for (size_t mcols = 1; mcols < 20; mcols += 2) {
            Columns cols(mcols, std::vector<bool>(n));
            for (size_t j = 0; j < mcols; ++j)
                for (uint64_t i = 0; i < n; ++i)
                    cols[j][i] = kind == 0 ? false : kind == 1 ? true : ((i + 2 * j) % 2) != 0;
            auto om = OracleMatrix(build_oracle(cols, n, 0, 2, relax));
            {
                std::ofstream out(good, std::ios::binary);
                om.serialize(out);
            }
            if (!g_device) {
                std::ifstream in(good, std::ios::binary);
                std::vector<char> buf((std::istreambuf_iterator<char>(in)), std::istreambuf_iterator<char>());
                mbrwt_tree *t = nullptr;
                uint64_t used = 0;
                ASSERT_EQ(MBRWT_OK, mbrwt_tree_parse(reinterpret_cast<const uint8_t *>(buf.data()), buf.size(),
                                                     &used, &t));
                ASSERT_EQ(buf.size(), used);
                const mbrwt_tree_desc *d = mbrwt_tree_get_desc(t);
                EXPECT_EQ(om.num_rows(), d->num_rows);
                EXPECT_EQ(om.num_columns(), d->num_columns);
                EXPECT_EQ(oracle_export_num_nodes(om.tree()), d->num_nodes);
                mbrwt_tree_free(t);
                continue;
            }
            mbrwt_host::BRWTDevice loaded;
            {
                std::ifstream in(bad, std::ios::binary);
                ASSERT_TRUE(!loaded.load(in));
            }
            {
                std::ifstream in(good, std::ios::binary);
                ASSERT_TRUE(loaded.load(in));
                ASSERT_TRUE(in.good());
            }
            ASSERT_EQ(om.num_columns(), loaded.num_columns());
            ASSERT_EQ(om.num_rows(), loaded.num_rows());
            for (size_t j = 0; j < loaded.num_columns(); ++j) EXPECT_EQ(om.get_column(j), loaded.get_column(j));
            test_brwt(loaded, cols, n);
            // and the device matrix's own dump
            std::stringstream ss;
            loaded.serialize(ss);
            mbrwt_host::BRWTDevice again;
            ASSERT_TRUE(again.load(ss));
            test_brwt(again, cols, n);
        }
    }
}
TEST(BRWT, SerializationAllZero) { grid_serialization(0, 0); }
TEST(BRWT, SerializationAllOne) { grid_serialization(1, 0); }
TEST(BRWT, SerializationAllMixed) { grid_serialization(2, 0); }
TEST(BRWTOptimizer, SerializationAllMixed) { grid_serialization(2, UINT64_MAX); }

int main(int argc, char **argv) {
    g_device = argc > 1 && std::string(argv[1]) == "device";
    return minitest::run_all(argc > 2 ? argv[2] : nullptr);
}
