// Unit tests of the native control plane (no framework dependency).  Run: make -C native test
#include <cstdio>
#include <functional>
#include <string>
#include <vector>

#include "detcore/json.h"
#include "detcore/searcher.h"
#include "detcore/sequencer.h"
#include "test_util.h"

std::vector<std::pair<std::string, std::function<void()>>>& registry() {
  static std::vector<std::pair<std::string, std::function<void()>>> r;
  return r;
}
int g_failures = 0;

int main(int argc, char** argv) {
  int ran = 0;
  for (auto& t : registry()) {
    if (argc > 1 && t.first.find(argv[1]) == std::string::npos) continue;
    int before = g_failures;
    try {
      t.second();
    } catch (const std::exception& e) {
      std::fprintf(stderr, "  exception: %s\n", e.what());
      ++g_failures;
    }
    std::printf("%s %s\n", g_failures == before ? "PASS" : "FAIL", t.first.c_str());
    ++ran;
  }
  std::printf("%d tests, %d failures\n", ran, g_failures);
  return g_failures == 0 ? 0 : 1;
}
