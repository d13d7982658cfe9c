// Known-answer tests of tests/test_annotation_BRWT.cpp (reference) through
// the C++ mirror StaticBinRelAnnotator, on the backend named by argv[1]:
//   oracle  -- the CPU restatement (runs without a GPU)
//   device  -- BRWTDevice, every query through include/mbrwt.h on the GPU
#include <set>
#include <sstream>

#include "backends.hpp"
#include "minitest.hpp"

using mbrwt_host::StaticBinRelAnnotator;
typedef std::vector<std::string> VS;
typedef std::vector<std::pair<std::string, size_t>> VectorCounts;

static bool g_device = false;

static std::set<std::string> S(const VS &v) { return std::set<std::string>(v.begin(), v.end()); }
static std::set<std::pair<std::string, size_t>> SC(const VectorCounts &v) { return {v.begin(), v.end()}; }

// convert_to_simple_BRWT (annotation_converters.cpp:76-86, grouping arity 2)
static std::shared_ptr<StaticBinRelAnnotator<BinaryMatrix>> annotator(const LabelFixture &f) {
    auto om = std::make_shared<OracleMatrix>(build_oracle(f.cols, f.n, 0, 2));
    std::shared_ptr<BinaryMatrix> m = om;
    if (g_device) m = std::make_shared<mbrwt_host::BRWTDevice>(to_device(*om));
    return std::make_shared<StaticBinRelAnnotator<BinaryMatrix>>(m, f.enc);
}

TEST(BRWTCompressed, GetLabelsAfterConversion) {  // test_annotation_BRWT.cpp:195-218
    auto a = annotator(make_fixture(5, {{0, {"Label0", "Label2", "Label8"}}, {2, {"Label1", "Label2"}}, {4, {"Label8"}}}));
    EXPECT_EQ(S({"Label0", "Label2", "Label8"}), S(a->get_labels(0)));
    EXPECT_EQ(S({}), S(a->get_labels(1)));
    EXPECT_EQ(S({"Label1", "Label2"}), S(a->get_labels(2)));
    EXPECT_EQ(S({}), S(a->get_labels(3)));
    EXPECT_EQ(S({"Label8"}), S(a->get_labels(4)));
    EXPECT_EQ(5u, a->num_objects());
    EXPECT_EQ(4u, a->num_labels());
    EXPECT_EQ(6u, a->num_relations());
}

TEST(BRWTCompressed, has_labels) {  // test_annotation_BRWT.cpp:250-300
    auto a = annotator(make_fixture(5, {{0, {"Label0", "Label2", "Label8"}}, {2, {"Label1", "Label2"}}, {4, {"Label8"}}}));
    EXPECT_FALSE(a->has_labels(0, {"Label0", "Label1", "Label2", "Label4", "Label5", "Label8"}));
    EXPECT_FALSE(a->has_labels(0, {"Label0", "Label2", "Label4", "Label8"}));
    EXPECT_TRUE(a->has_labels(0, {"Label0", "Label2", "Label8"}));
    EXPECT_TRUE(a->has_labels(0, {"Label0", "Label8"}));
    EXPECT_TRUE(a->has_labels(0, {"Label2"}));
    EXPECT_TRUE(a->has_labels(0, {}));
    EXPECT_FALSE(a->has_labels(1, {"Label0", "Label1", "Label2", "Label4", "Label5", "Label8"}));
    EXPECT_FALSE(a->has_labels(1, {"Label0", "Label2", "Label4", "Label8"}));
    EXPECT_FALSE(a->has_labels(1, {"Label0", "Label2", "Label8"}));
    EXPECT_FALSE(a->has_labels(1, {"Label0", "Label8"}));
    EXPECT_FALSE(a->has_labels(1, {"Label2"}));
    EXPECT_TRUE(a->has_labels(1, {}));
    EXPECT_FALSE(a->has_labels(2, {"Label0", "Label1", "Label2", "Label4", "Label5", "Label8"}));
    EXPECT_FALSE(a->has_labels(2, {"Label0", "Label2", "Label4", "Label8"}));
    EXPECT_FALSE(a->has_labels(2, {"Label1", "Label2", "Label8"}));
    EXPECT_FALSE(a->has_labels(2, {"Label1", "Label8"}));
    EXPECT_TRUE(a->has_labels(2, {"Label1", "Label2"}));
    EXPECT_TRUE(a->has_labels(2, {"Label2"}));
    EXPECT_TRUE(a->has_labels(2, {}));
    // has_label (annotate_static.cpp:26-33): unknown labels are false
    EXPECT_TRUE(a->has_label(0, "Label8"));
    EXPECT_FALSE(a->has_label(1, "Label8"));
    EXPECT_FALSE(a->has_label(0, "NoSuchLabel"));
}

TEST(BRWTCompressed, get_top_labels) {  // test_annotation_BRWT.cpp:344-398
    auto a = annotator(make_fixture(5, {{0, {"Label0", "Label2", "Label8"}},
                                        {2, {"Label1", "Label2"}},
                                        {3, {"Label1", "Label2", "Label8"}},
                                        {4, {"Label2", "Label8"}}}));
    EXPECT_EQ(VectorCounts({}), a->get_top_labels({0, 1, 2, 3, 4}, 0));
    EXPECT_EQ(VectorCounts({}), a->get_top_labels({}));
    EXPECT_EQ(VectorCounts({{"Label2", 4}, {"Label8", 3}, {"Label1", 2}, {"Label0", 1}}),
              a->get_top_labels({0, 1, 2, 3, 4}));
    EXPECT_EQ(SC(VectorCounts({{"Label1", 1}, {"Label2", 1}})), SC(a->get_top_labels({2})));
    EXPECT_EQ(VectorCounts({{"Label2", 4}}), a->get_top_labels({0, 1, 2, 3, 4}, 1));
    EXPECT_EQ(VectorCounts({{"Label2", 4}, {"Label8", 3}}), a->get_top_labels({0, 1, 2, 3, 4}, 2));
    EXPECT_EQ(VectorCounts({{"Label2", 4}, {"Label8", 3}, {"Label1", 2}}), a->get_top_labels({0, 1, 2, 3, 4}, 3));
    EXPECT_EQ(VectorCounts({{"Label2", 4}, {"Label8", 3}, {"Label1", 2}, {"Label0", 1}}),
              a->get_top_labels({0, 1, 2, 3, 4}, 4));
    EXPECT_EQ(VectorCounts({{"Label2", 4}, {"Label8", 3}, {"Label1", 2}, {"Label0", 1}}),
              a->get_top_labels({0, 1, 2, 3, 4}, 1000));
}

TEST(BRWTCompressed, get_labels_presence_ratio) {  // test_annotation_BRWT.cpp:400-470
    auto a = annotator(make_fixture(5, {{0, {"Label0", "Label2", "Label8"}},
                                        {2, {"Label1", "Label2"}},
                                        {3, {"Label1", "Label2", "Label8"}},
                                        {4, {"Label2"}}}));
    EXPECT_EQ(VS({}), a->get_labels(std::vector<uint64_t>{}, 1));
    EXPECT_EQ(S({"Label1", "Label2"}), S(a->get_labels({2}, 1)));
    EXPECT_EQ(S({"Label1", "Label2"}), S(a->get_labels({2}, 0)));
    EXPECT_EQ(S({"Label1", "Label2"}), S(a->get_labels({2}, 0.5)));
    EXPECT_EQ(S({"Label2"}), S(a->get_labels({2, 4}, 1)));
    EXPECT_EQ(S({"Label1", "Label2"}), S(a->get_labels({2, 4}, 0)));
    EXPECT_EQ(S({"Label1", "Label2"}), S(a->get_labels({2, 4}, 0.5)));
    EXPECT_EQ(S({"Label2"}), S(a->get_labels({2, 4}, 0.501)));
    EXPECT_EQ(S({}), S(a->get_labels({0, 1, 2, 3, 4}, 1)));
    EXPECT_EQ(S({"Label0", "Label1", "Label2", "Label8"}), S(a->get_labels({0, 1, 2, 3, 4}, 0)));
    EXPECT_EQ(S({"Label0", "Label1", "Label2", "Label8"}), S(a->get_labels({0, 1, 2, 3, 4}, 0.2)));
    EXPECT_EQ(S({"Label1", "Label2", "Label8"}), S(a->get_labels({0, 1, 2, 3, 4}, 0.201)));
    EXPECT_EQ(S({"Label1", "Label2", "Label8"}), S(a->get_labels({0, 1, 2, 3, 4}, 0.4)));
    EXPECT_EQ(S({"Label2"}), S(a->get_labels({0, 1, 2, 3, 4}, 0.401)));
    EXPECT_EQ(S({"Label2"}), S(a->get_labels({0, 1, 2, 3, 4}, 0.8)));
    EXPECT_EQ(S({}), S(a->get_labels({0, 1, 2, 3, 4}, 0.801)));
}

TEST(BRWTCompressed, get_labels_batch_presence_ratio) {  // the vectors above, all reads in one batch
    auto a = annotator(make_fixture(5, {{0, {"Label0", "Label2", "Label8"}},
                                        {2, {"Label1", "Label2"}},
                                        {3, {"Label1", "Label2", "Label8"}},
                                        {4, {"Label2"}}}));
    const std::vector<std::vector<uint64_t>> reads{{}, {2}, {2, 4}, {0, 1, 2, 3, 4}, {4, 4, 2}};
    const std::vector<std::pair<double, std::vector<VS>>> want{
        {0, {{}, {"Label1", "Label2"}, {"Label1", "Label2"}, {"Label0", "Label1", "Label2", "Label8"},
             {"Label1", "Label2"}}},
        {0.2, {{}, {"Label1", "Label2"}, {"Label1", "Label2"}, {"Label0", "Label1", "Label2", "Label8"},
               {"Label1", "Label2"}}},
        {0.201, {{}, {"Label1", "Label2"}, {"Label1", "Label2"}, {"Label1", "Label2", "Label8"}, {"Label1", "Label2"}}},
        {0.401, {{}, {"Label1", "Label2"}, {"Label1", "Label2"}, {"Label2"}, {"Label2"}}},
        {0.8, {{}, {"Label1", "Label2"}, {"Label2"}, {"Label2"}, {"Label2"}}},
        {1, {{}, {"Label1", "Label2"}, {"Label2"}, {}, {"Label2"}}},
    };
    for (const auto &w : want) {
        auto got = a->get_labels_batch(reads, w.first);
        EXPECT_EQ(reads.size(), got.size());
        for (size_t r = 0; r < reads.size(); ++r) {
            EXPECT_EQ(S(w.second[r]), S(got[r]));
            EXPECT_EQ(S(a->get_labels(reads[r], w.first)), S(got[r]));
        }
    }
    EXPECT_EQ(0u, a->get_labels_batch({}, 0.5).size());
}

TEST(BRWTCompressed, get_top_labels_batch) {  // test_annotation_BRWT.cpp:344-398, all reads in one batch
    auto a = annotator(make_fixture(5, {{0, {"Label0", "Label2", "Label8"}},
                                        {2, {"Label1", "Label2"}},
                                        {3, {"Label1", "Label2", "Label8"}},
                                        {4, {"Label2", "Label8"}}}));
    const std::vector<std::vector<uint64_t>> reads{{0, 1, 2, 3, 4}, {}, {2}, {1}, {0, 1, 2, 3, 4}};
    const VectorCounts all{{"Label2", 4}, {"Label8", 3}, {"Label1", 2}, {"Label0", 1}};
    for (size_t k : {0ul, 1ul, 2ul, 3ul, 4ul, 1000ul}) {
        auto got = a->get_top_labels_batch(reads, k);
        EXPECT_EQ(reads.size(), got.size());
        VectorCounts top(all.begin(), all.begin() + std::min(k, all.size()));
        EXPECT_EQ(top, got[0]);
        EXPECT_EQ(top, got[4]);
        EXPECT_EQ(VectorCounts({}), got[1]);
        EXPECT_EQ(VectorCounts({}), got[3]);
        if (k >= 2) EXPECT_EQ(SC(VectorCounts({{"Label1", 1}, {"Label2", 1}})), SC(got[2]));
        if (k == 1) EXPECT_EQ(1u, got[2].size());
    }
    auto got = a->get_top_labels_batch(reads);  // default: all labels
    EXPECT_EQ(all, got[0]);
}

// More columns than the device's batched histograms hold (8,192 for top labels,
// 15,360 for get_labels): the batched calls fall back to the per-read path
// (the reference's get_labels / get_top_labels have no column limit)
TEST(BRWTCompressed, batch_calls_past_the_device_column_limit) {
    std::vector<std::pair<uint64_t, VS>> rows;
    for (uint64_t r = 0; r < 40; ++r) {
        VS l;
        for (uint64_t k = 0; k < 1000; ++k) l.push_back("L" + std::to_string((r * 7919 + k * 104729) % 20000));
        if (r % 3 == 0) l.push_back("L7");
        rows.push_back({r, l});
    }
    auto a = annotator(make_fixture(40, rows));
    EXPECT_TRUE(a->num_labels() > 15360);
    const std::vector<std::vector<uint64_t>> reads{{0, 1, 2, 3}, {}, {5, 6, 9, 12, 39}, {7}};
    auto top = a->get_top_labels_batch(reads, 5);
    auto lab = a->get_labels_batch(reads, 0.5);
    EXPECT_EQ(reads.size(), top.size());
    EXPECT_EQ(reads.size(), lab.size());
    for (size_t r = 0; r < reads.size(); ++r) {
        EXPECT_EQ(a->get_top_labels(reads[r], 5), top[r]);
        EXPECT_EQ(S(a->get_labels(reads[r], 0.5)), S(lab[r]));
    }
}

TEST(LabelEncoder, encode_decode) {  // annotate.cpp:12-31, annotate.hpp:128
    mbrwt_host::LabelEncoder<std::string> e;
    EXPECT_EQ(0u, e.insert_and_encode("a"));
    EXPECT_EQ(1u, e.insert_and_encode("b"));
    EXPECT_EQ(0u, e.insert_and_encode("a"));
    EXPECT_EQ(1u, e.encode("b"));
    EXPECT_EQ(std::string("a"), e.decode(0));
    EXPECT_THROW(e.encode("c"), std::runtime_error);
    EXPECT_THROW(e.decode(5), std::out_of_range);
}

// test_annotation_BRWT.cpp:190-215 (BRWTCompressed, Serialization): the
// annotator is dumped (label encoder + matrix, annotate_static.cpp:96-109)
// and merge_load'ed into a default-constructed annotator
// (annotate_static.cpp:111-130); a missing file does not load.  Oracle
// backend: the label encoder part round-trips and the matrix part parses;
// device backend: the loaded annotator answers from HBM.
TEST(BRWTCompressed, Serialization) {
    const std::string base = "/tmp/mbrwt_test_annotation_dump";
    auto f = make_fixture(5, {{0, {"Label0", "Label2", "Label8"}}, {2, {"Label1", "Label2"}}, {4, {"Label8"}}});
    auto a = annotator(f);
    if (!g_device) {
        std::stringstream ss;
        f.enc.serialize(ss);
        mbrwt_host::LabelEncoder<std::string> e2;
        ASSERT_TRUE(e2.load(ss));
        ASSERT_EQ(f.enc.size(), e2.size());
        for (size_t i = 0; i < e2.size(); ++i) EXPECT_EQ(f.enc.decode(i), e2.decode(i));
        EXPECT_EQ(2u, e2.encode("Label8"));
        return;
    }
    auto m = std::make_shared<mbrwt_host::BRWTDevice>(
        to_device(OracleMatrix(build_oracle(f.cols, f.n, 0, 2))));
    StaticBinRelAnnotator<mbrwt_host::BRWTDevice> dev(m, f.enc);
    dev.serialize(base);  // writes base + ".brwt.annodbg"
    StaticBinRelAnnotator<mbrwt_host::BRWTDevice> annotation;
    EXPECT_TRUE(!annotation.load(base + "_missing"));
    ASSERT_TRUE(annotation.load(base));
    EXPECT_EQ(S({"Label0", "Label2", "Label8"}), S(annotation.get(0)));
    EXPECT_EQ(S({}), S(annotation.get(1)));
    EXPECT_EQ(S({"Label1", "Label2"}), S(annotation.get(2)));
    EXPECT_EQ(S({}), S(annotation.get(3)));
    EXPECT_EQ(S({"Label8"}), S(annotation.get(4)));
    EXPECT_EQ(5u, annotation.num_objects());
    EXPECT_EQ(4u, annotation.num_labels());
    EXPECT_EQ(6u, annotation.num_relations());
    // the dynamic actions of a static annotator throw (annotate_static.cpp:164-168)
    EXPECT_THROW(annotation.add_label(0, "Label1"), std::runtime_error);
}

int main(int argc, char **argv) {
    g_device = argc > 1 && std::string(argv[1]) == "device";
    return minitest::run_all(argc > 2 ? argv[2] : nullptr);
}
