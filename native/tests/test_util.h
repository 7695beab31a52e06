#pragma once
#include <cstdio>
#include <functional>
#include <string>
#include <utility>
#include <vector>

std::vector<std::pair<std::string, std::function<void()>>>& registry();
extern int g_failures;

struct Registrar {
  Registrar(const char* name, std::function<void()> fn) { registry().emplace_back(name, std::move(fn)); }
};

#define TEST(name)                                 \
  static void test_##name();                       \
  static Registrar reg_##name(#name, test_##name); \
  static void test_##name()

#define EXPECT(cond)                                                             \
  do {                                                                           \
    if (!(cond)) {                                                               \
      std::fprintf(stderr, "  %s:%d: EXPECT(%s) failed\n", __FILE__, __LINE__, #cond); \
      ++g_failures;                                                              \
    }                                                                            \
  } while (0)

#define EXPECT_EQ(a, b)                                                                               \
  do {                                                                                                \
    auto _a = (a);                                                                                    \
    auto _b = (b);                                                                                    \
    if (!(_a == _b)) {                                                                                \
      std::fprintf(stderr, "  %s:%d: EXPECT_EQ(%s, %s) failed\n", __FILE__, __LINE__, #a, #b);       \
      ++g_failures;                                                                                   \
    }                                                                                                 \
  } while (0)
