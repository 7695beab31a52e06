// LogStore backend mode (the Elasticsearch shipping path, master/internal/trial_logger.go in the
// reference): appends never wait on the backend, failed batches are retried without loss or
// duplication, reads see every appended row at once (memory suffix + backend), and Delete drains.
// Run under TSan/ASan by tests/test_sanitizers.py.
#include <atomic>
#include <chrono>
#include <map>
#include <mutex>
#include <stdexcept>
#include <thread>

#include "detcore/store.h"
#include "test_util.h"

using namespace detcore;

namespace {

// A slow, flaky, eventually-consistent index: Index sleeps, every 3rd call throws, and rows are
// searchable only after Refresh.
class FlakyBackend : public LogBackend {
 public:
  explicit FlakyBackend(int delay_ms) : delay_ms_(delay_ms) {}
  void Index(const std::string& stream, const std::vector<Json>& rows) override {
    std::this_thread::sleep_for(std::chrono::milliseconds(delay_ms_));
    std::lock_guard<std::mutex> g(mu_);
    if (++calls % 3 == 0) {
      ++failures;
      throw std::runtime_error("503");
    }
    for (auto& r : rows) {
      auto& slot = docs[stream][r.get_int("id", 0)];
      if (!slot.is_null()) ++overwrites;
      slot = r.clone();
      unrefreshed[stream].push_back(r.get_int("id", 0));
    }
  }
  void Refresh() override {
    std::lock_guard<std::mutex> g(mu_);
    for (auto& kv : unrefreshed)
      for (int64_t id : kv.second) visible[kv.first][id] = true;
    unrefreshed.clear();
    ++refreshes;
  }
  std::vector<Json> Search(const std::string& stream, int64_t after, int64_t before, int64_t limit, bool desc) override {
    std::lock_guard<std::mutex> g(mu_);
    std::vector<Json> out;
    auto& d = docs[stream];
    if (!desc) {
      for (auto it = d.upper_bound(after); it != d.end() && it->first < before && (int64_t)out.size() < limit; ++it)
        if (visible[stream].count(it->first)) out.push_back(it->second.clone());
    } else {
      for (auto it = d.rbegin(); it != d.rend() && (int64_t)out.size() < limit; ++it)
        if (it->first > after && it->first < before && visible[stream].count(it->first)) out.insert(out.begin(), it->second.clone());
    }
    return out;
  }
  int64_t MaxId(const std::string& stream) override {
    std::lock_guard<std::mutex> g(mu_);
    auto& d = docs[stream];
    return d.empty() ? 0 : d.rbegin()->first;
  }
  void Delete(const std::string& stream) override {
    std::lock_guard<std::mutex> g(mu_);
    docs.erase(stream);
    visible.erase(stream);
  }
  int delay_ms_;
  std::mutex mu_;
  int calls = 0, failures = 0, overwrites = 0, refreshes = 0;
  std::map<std::string, std::map<int64_t, Json>> docs;
  std::map<std::string, std::map<int64_t, bool>> visible;
  std::map<std::string, std::vector<int64_t>> unrefreshed;
};

Json Line(const std::string& msg) {
  Json j = Json::object();
  j["message"] = msg;
  return j;
}

}  // namespace

TEST(logstore_backend_appends_do_not_wait_and_nothing_is_lost) {
  auto* be = new FlakyBackend(400);
  LogStore ls;
  LogShipOptions opt;
  opt.batch_lines = 200;
  opt.max_batch_lines = 500;  // several requests, so the every-3rd failure is hit
  opt.flush_ms = 5;
  opt.refresh_ms = 50;
  ls.SetBackend(std::unique_ptr<LogBackend>(be), opt);
  const int kLines = 3000;
  double worst_ms = 0;
  std::atomic<bool> reading{true};
  std::atomic<int> bad_reads{0};
  std::thread reader([&] {  // a follower: every read is a contiguous prefix 1..k of what was appended
    while (reading.load()) {
      auto rows = ls.Read("trial-1", 0, INT64_MAX);
      for (size_t i = 0; i < rows.size(); ++i)
        if (rows[i].get_int("id", 0) != static_cast<int64_t>(i + 1)) {
          ++bad_reads;
          break;
        }
    }
  });
  for (int i = 0; i < kLines; ++i) {
    auto t0 = std::chrono::steady_clock::now();
    ls.Append(i % 2 ? "trial-1" : "task-7", {Line("l" + std::to_string(i))});
    double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    worst_ms = std::max(worst_ms, ms);
  }
  // read-your-writes before anything is searchable
  EXPECT_EQ(ls.Read("trial-1", 0, INT64_MAX).size(), static_cast<size_t>(kLines / 2));
  EXPECT_EQ(ls.Count("task-7"), kLines / 2);
  auto tail = ls.Read("task-7", 0, 3, nullptr, true);
  EXPECT_EQ(tail.size(), static_cast<size_t>(3));
  EXPECT_EQ(tail.back().get_int("id", 0), kLines / 2);
  EXPECT(ls.Flush(60000));
  reading = false;
  reader.join();
  EXPECT_EQ(bad_reads.load(), 0);
  // never a 400 ms backend call on the appending thread (the bound leaves room for a loaded host and
  // sanitizer builds: the suite runs on parallel workers)
  EXPECT(worst_ms < 200.0);
  Json st = ls.Stats();
  EXPECT(st.get_int("failed_batches", 0) >= 1);
  EXPECT_EQ(st.get_int("shipped_lines", 0), kLines);
  {
    std::lock_guard<std::mutex> g(be->mu_);
    EXPECT_EQ(be->docs["trial-1"].size(), static_cast<size_t>(kLines / 2));
    EXPECT_EQ(be->docs["task-7"].size(), static_cast<size_t>(kLines / 2));
    EXPECT_EQ(be->docs["trial-1"].rbegin()->first, kLines / 2);
    EXPECT(be->failures >= 1);
  }
  // once refreshed, reads come from the backend and still see everything, in order
  std::this_thread::sleep_for(std::chrono::milliseconds(200));
  auto all = ls.Read("trial-1", 10, INT64_MAX);
  EXPECT_EQ(all.size(), static_cast<size_t>(kLines / 2 - 10));
  EXPECT_EQ(all.front().get_int("id", 0), 11);
  EXPECT(ls.Stats().get_int("unrefreshed_lines", -1) == 0);
  // delete while lines are queued
  for (int i = 0; i < 50; ++i) ls.Append("trial-1", {Line("late")});
  ls.Delete("trial-1");
  EXPECT(ls.Flush(60000));
  EXPECT_EQ(ls.Read("trial-1", 0, INT64_MAX).size(), static_cast<size_t>(0));
  {
    std::lock_guard<std::mutex> g(be->mu_);
    EXPECT(be->docs.find("trial-1") == be->docs.end() || be->docs["trial-1"].empty());
  }
}
