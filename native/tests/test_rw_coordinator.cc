#include <vector>

#include "detcore/rw_coordinator.h"
#include "test_util.h"

using detcore::RWCoordinator;

TEST(rw_readers_share_writer_excludes) {
  RWCoordinator c;
  std::vector<std::pair<int64_t, bool>> granted;
  auto g = [&](int64_t t, bool read) { granted.emplace_back(t, read); };
  int64_t r1 = c.Acquire("/cache", true, g);
  int64_t r2 = c.Acquire("/cache", true, g);
  EXPECT_EQ(granted.size(), size_t(2));
  int64_t w = c.Acquire("/cache", false, g);
  EXPECT_EQ(granted.size(), size_t(2));  // writer waits for both readers
  int64_t r3 = c.Acquire("/cache", true, g);
  EXPECT_EQ(granted.size(), size_t(2));  // writer preference: new reader queues behind it
  EXPECT_EQ(c.Inspect("/cache").write_waiting, 1);
  c.Release(r1);
  EXPECT_EQ(granted.size(), size_t(2));
  c.Release(r2);
  EXPECT_EQ(granted.size(), size_t(3));
  EXPECT(granted[2].first == w && !granted[2].second);
  c.Release(w);
  EXPECT_EQ(granted.size(), size_t(4));
  EXPECT(granted[3].first == r3 && granted[3].second);
  c.Release(r3);
  EXPECT_EQ(c.Inspect("/cache").readers, 0);
}

TEST(rw_waiting_writer_disconnect_unblocks_readers) {
  RWCoordinator c;
  int grants = 0;
  auto g = [&](int64_t, bool) { ++grants; };
  int64_t r1 = c.Acquire("a", true, g);
  int64_t w = c.Acquire("a", false, g);
  c.Acquire("a", true, g);
  EXPECT_EQ(grants, 1);
  c.Release(w);  // the waiting writer's socket closed before its grant
  EXPECT_EQ(grants, 2);
  c.Acquire("b", false, g);  // independent resource
  EXPECT_EQ(grants, 3);
  c.Release(r1);
  c.Release(12345);  // unknown ticket is ignored
}
