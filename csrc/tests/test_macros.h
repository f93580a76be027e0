// Minimal native test macros (the capability of hw1code/test_macros.h:46-94 /
// hw4code/test_macros.h: EXPECT_* that record a failure without aborting,
// PRINT_SUCCESS per test) plus a registry so one driver runs every test and
// exits non-zero on any failure.
#pragma once

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <functional>
#include <string>
#include <vector>

namespace cme::test {

struct Case {
  const char* name;
  std::function<void(bool*)> fn;
};

inline std::vector<Case>& registry() {
  static std::vector<Case> r;
  return r;
}

struct Registrar {
  Registrar(const char* name, std::function<void(bool*)> fn) { registry().push_back({name, std::move(fn)}); }
};

inline bool color() {
  static const bool c = std::getenv("NO_COLOR") == nullptr;
  return c;
}

inline int run_all(const char* filter = nullptr) {
  int failed = 0, ran = 0;
  for (auto& c : registry()) {
    if (filter && std::string(c.name).find(filter) == std::string::npos) continue;
    bool ok = true;
    c.fn(&ok);
    ++ran;
    if (!ok) ++failed;
    std::printf("%s%s%s %s\n", color() ? (ok ? "\033[32m" : "\033[31m") : "", ok ? "[ PASS ]" : "[ FAIL ]",
                color() ? "\033[0m" : "", c.name);
  }
  std::printf("%d tests, %d failed\n", ran, failed);
  return failed ? 1 : 0;
}

}  // namespace cme::test

#define CME_TEST(name)                                                        \
  static void name(bool* success);                                            \
  static ::cme::test::Registrar name##_registrar(#name, name);                \
  static void name(bool* success)

#define EXPECT_TRUE(cond)                                                                  \
  do {                                                                                     \
    if (!(cond)) {                                                                         \
      std::printf("  %s:%d: expected %s\n", __FILE__, __LINE__, #cond);                  \
      *success = false;                                                                    \
    }                                                                                      \
  } while (0)

#define EXPECT_EQ(a, b)                                                                    \
  do {                                                                                     \
    if (!((a) == (b))) {                                                                   \
      std::printf("  %s:%d: %s != %s\n", __FILE__, __LINE__, #a, #b);                     \
      *success = false;                                                                    \
    }                                                                                      \
  } while (0)

#define EXPECT_NEAR(a, b, eps)                                                             \
  do {                                                                                     \
    const double _a = (a), _b = (b);                                                       \
    if (!(std::fabs(_a - _b) <= (eps))) {                                                  \
      std::printf("  %s:%d: |%s - %s| = %g > %g\n", __FILE__, __LINE__, #a, #b,           \
                  std::fabs(_a - _b), (double)(eps));                                      \
      *success = false;                                                                    \
    }                                                                                      \
  } while (0)

#define EXPECT_VECTOR_EQ(a, b)                                                             \
  do {                                                                                     \
    if ((a).size() != (b).size()) {                                                        \
      std::printf("  %s:%d: size %zu != %zu\n", __FILE__, __LINE__, (size_t)(a).size(),    \
                  (size_t)(b).size());                                                     \
      *success = false;                                                                    \
    } else {                                                                               \
      for (size_t _i = 0; _i < (a).size(); ++_i)                                           \
        if (!((a)[_i] == (b)[_i])) {                                                       \
          std::printf("  %s:%d: element %zu differs\n", __FILE__, __LINE__, _i);           \
          *success = false;                                                                \
          break;                                                                           \
        }                                                                                  \
    }                                                                                      \
  } while (0)
