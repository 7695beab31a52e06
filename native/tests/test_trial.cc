// Counterpart of the reference's master/internal/trial_test.go TestRendezvousInfo: every rank gets
// the same rendezvous addresses in rank order (chief first), differing only in its own rank.
#include <algorithm>

#include "detcore/master_actors.h"
#include "test_util.h"

using namespace detcore;
using namespace detcore::master;

TEST(TestRendezvousInfo) {
  // containers registered out of rank order, on two hosts, with unsorted device lists
  std::vector<RendezvousMember> members = {{1, "10.0.0.2", {5, 4}}, {0, "10.0.0.1", {3, 2}}};
  std::vector<Json> msgs;
  for (const auto& m : members) msgs.push_back(RendezvousInfo(members, m.rank));
  Json rep = msgs[0];
  EXPECT_EQ(rep["addrs"].size(), size_t(2));
  EXPECT_EQ(rep["addrs"][0].as_string(), std::string("10.0.0.1:1736"));  // rank 0 first, lowest device
  EXPECT_EQ(rep["addrs"][1].as_string(), std::string("10.0.0.2:1738"));
  EXPECT_EQ(rep["addrs2"][0].as_string(), std::string("10.0.0.1:1752"));
  for (auto& m : msgs) {  // the same information for all containers, ignoring the rank
    Json a = m, b = rep;
    a["rank"] = 0;
    b["rank"] = 0;
    EXPECT_EQ(a.dump(), b.dump());
  }
  EXPECT_EQ(msgs[0]["rank"].as_int(), int64_t(1));
  EXPECT_EQ(msgs[1]["rank"].as_int(), int64_t(0));
}
