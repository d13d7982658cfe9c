// minitest.hpp -- a minimal test harness for the C++ mirror tests (the
// reference uses GoogleTest, which is not available in this image).
#pragma once
#include <cstdio>
#include <functional>
#include <sstream>
#include <string>
#include <vector>

namespace minitest {
struct Case {
    std::string name;
    std::function<void()> fn;
};
inline std::vector<Case> &registry() {
    static std::vector<Case> r;
    return r;
}
inline int &failures() {
    static int f = 0;
    return f;
}
struct Reg {
    Reg(const char *n, std::function<void()> f) { registry().push_back({n, std::move(f)}); }
};
inline int run_all(const char *filter = nullptr) {
    int ran = 0;
    for (auto &c : registry()) {
        if (filter && c.name.find(filter) == std::string::npos) continue;
        int before = failures();
        c.fn();
        ++ran;
        std::printf("[%s] %s\n", failures() == before ? "  OK  " : " FAIL ", c.name.c_str());
    }
    std::printf("%d tests, %d failed checks\n", ran, failures());
    return failures() ? 1 : 0;
}
}  // namespace minitest

#define MT_CAT2(a, b) a##b
#define MT_CAT(a, b) MT_CAT2(a, b)
#define TEST(suite, name)                                                              \
    static void MT_CAT(test_, MT_CAT(suite, name))();                                  \
    static minitest::Reg MT_CAT(reg_, MT_CAT(suite, name))(#suite "." #name,           \
                                                           MT_CAT(test_, MT_CAT(suite, name))); \
    static void MT_CAT(test_, MT_CAT(suite, name))()
#define EXPECT_TRUE(x)                                                                 \
    do {                                                                               \
        if (!(x)) {                                                                    \
            ++minitest::failures();                                                    \
            std::printf("  %s:%d: EXPECT_TRUE(%s) failed\n", __FILE__, __LINE__, #x);  \
        }                                                                              \
    } while (0)
#define EXPECT_FALSE(x) EXPECT_TRUE(!(x))
#define EXPECT_EQ(a, b)                                                                \
    do {                                                                               \
        if (!((a) == (b))) {                                                           \
            ++minitest::failures();                                                    \
            std::printf("  %s:%d: EXPECT_EQ(%s, %s) failed\n", __FILE__, __LINE__, #a, #b); \
        }                                                                              \
    } while (0)
#define ASSERT_EQ(a, b)                                                                \
    do {                                                                               \
        if (!((a) == (b))) {                                                           \
            ++minitest::failures();                                                    \
            std::printf("  %s:%d: ASSERT_EQ(%s, %s) failed\n", __FILE__, __LINE__, #a, #b); \
            return;                                                                    \
        }                                                                              \
    } while (0)
#define ASSERT_TRUE(x) ASSERT_EQ(!!(x), true)
#define EXPECT_THROW(stmt, exc)                                                        \
    do {                                                                               \
        bool caught = false;                                                           \
        try {                                                                          \
            stmt;                                                                      \
        } catch (const exc &) {                                                        \
            caught = true;                                                             \
        }                                                                              \
        if (!caught) {                                                                 \
            ++minitest::failures();                                                    \
            std::printf("  %s:%d: expected %s\n", __FILE__, __LINE__, #exc);           \
        }                                                                              \
    } while (0)
