// Scheduler + fitting scenarios (mirrors the reference's resourcemanagers/*_test.go cases with
// in-memory mock agents: fair_share_test.go, priority_test.go, fitting_test.go).
#include <algorithm>
#include <string>

#include "detcore/scheduler.h"
#include "test_util.h"

using namespace detcore::sched;

namespace {
Agent MkAgent(const std::string& id, int slots) {
  Agent a;
  a.id = id;
  for (int i = 0; i < slots; ++i) a.slots.push_back(Slot{i, id + "-" + std::to_string(i), "gpu", true, ""});
  return a;
}
Task MkTask(const std::string& id, const std::string& group, int slots, bool nonpre = false) {
  Task t;
  t.id = id;
  t.group = group;
  t.slots_needed = slots;
  t.non_preemptible = nonpre;
  return t;
}
bool Allocated(const Decision& d, const std::string& id) {
  for (auto& a : d.allocate)
    if (a.first == id) return true;
  return false;
}
bool Released(const Decision& d, const std::string& id) {
  return std::find(d.release.begin(), d.release.end(), id) != d.release.end();
}
void Apply(PoolState& st, const Decision& d) {
  for (auto& a : d.allocate) st.Allocate(a.first, a.second);
}
}  // namespace

TEST(fit_single_agent_best_vs_worst) {
  std::map<std::string, Agent> agents;
  agents["a"] = MkAgent("a", 8);
  agents["b"] = MkAgent("b", 8);
  agents["b"].slots[0].task = "x";  // b has 7 free
  Task t = MkTask("t", "g", 2);
  auto best = FindFits(t, agents, FitMethod::BestFit);
  EXPECT(best && best->size() == 1 && (*best)[0].agent == "b");  // fuller agent
  auto worst = FindFits(t, agents, FitMethod::WorstFit);
  EXPECT(worst && (*worst)[0].agent == "a");
  EXPECT_EQ((*best)[0].devices.size(), size_t(2));
}

TEST(fit_multi_agent_dedicated) {
  std::map<std::string, Agent> agents;
  for (auto id : {"a", "b", "c"}) agents[id] = MkAgent(id, 8);
  Task t = MkTask("t", "g", 16);
  auto f = FindFits(t, agents, FitMethod::BestFit);
  EXPECT(f && f->size() == 2);
  Task bad = MkTask("u", "g", 12);  // 12 % 8 != 0 -> no dedicated fit
  EXPECT(!FindFits(bad, agents, FitMethod::BestFit));
  agents["a"].slots[3].task = "busy";
  agents["b"].slots[3].task = "busy";
  EXPECT(!FindFits(t, agents, FitMethod::BestFit));  // only one idle agent left
}

TEST(fair_share_splits_between_groups_and_preempts) {
  PoolState st;
  st.agents["a"] = MkAgent("a", 8);
  for (int i = 0; i < 8; ++i) st.AddTask(MkTask("e1-" + std::to_string(i), "e1", 1));
  Decision d = Schedule(st, Policy::FairShare, FitMethod::BestFit);
  EXPECT_EQ(d.allocate.size(), size_t(8));
  Apply(st, d);
  // a second experiment arrives: fair share gives it half, so e1 must release 4 tasks
  for (int i = 0; i < 8; ++i) st.AddTask(MkTask("e2-" + std::to_string(i), "e2", 1));
  d = Schedule(st, Policy::FairShare, FitMethod::BestFit);
  EXPECT_EQ(d.release.size(), size_t(4));
  EXPECT(d.allocate.empty());  // cannot start before the releases free slots
  for (auto& r : d.release) st.RemoveTask(r);
  d = Schedule(st, Policy::FairShare, FitMethod::BestFit);
  EXPECT_EQ(d.allocate.size(), size_t(4));
  for (auto& a : d.allocate) EXPECT(a.first.rfind("e2-", 0) == 0);
}

TEST(fair_share_weights) {
  PoolState st;
  st.agents["a"] = MkAgent("a", 9);
  st.groups["heavy"] = Group{"heavy", 2.0, std::nullopt, -1};
  st.groups["light"] = Group{"light", 1.0, std::nullopt, -1};
  for (int i = 0; i < 9; ++i) {
    st.AddTask(MkTask("h" + std::to_string(i), "heavy", 1));
    st.AddTask(MkTask("l" + std::to_string(i), "light", 1));
  }
  Decision d = Schedule(st, Policy::FairShare, FitMethod::BestFit);
  int h = 0, l = 0;
  for (auto& a : d.allocate) (a.first[0] == 'h' ? h : l)++;
  EXPECT_EQ(h, 6);
  EXPECT_EQ(l, 3);
}

TEST(fair_share_non_preemptible_and_zero_slot) {
  PoolState st;
  st.agents["a"] = MkAgent("a", 4);
  st.AddTask(MkTask("np", "g1", 4, true));
  Decision d = Schedule(st, Policy::FairShare, FitMethod::BestFit);
  Apply(st, d);
  st.AddTask(MkTask("other", "g2", 1));
  st.AddTask(MkTask("gc", "g3", 0));  // zero-slot tasks always run (checkpoint GC, commands)
  d = Schedule(st, Policy::FairShare, FitMethod::BestFit);
  EXPECT(!Released(d, "np"));
  EXPECT(Allocated(d, "gc"));
  EXPECT(!Allocated(d, "other"));
}

TEST(fair_share_gang_deadlock_breaker) {
  PoolState st;
  st.agents["a"] = MkAgent("a", 4);
  st.AddTask(MkTask("g1-big", "g1", 4));
  st.AddTask(MkTask("g2-big", "g2", 4));
  // naive equal split offers 2+2 and nobody can start; the breaker disables the newest group
  Decision d = Schedule(st, Policy::FairShare, FitMethod::BestFit);
  EXPECT(Allocated(d, "g1-big"));
  EXPECT(!Allocated(d, "g2-big"));
}

TEST(priority_preempts_lower_priority) {
  PoolState st;
  st.agents["a"] = MkAgent("a", 2);
  st.groups["low"] = Group{"low", 1.0, 50, -1};
  st.groups["high"] = Group{"high", 1.0, 10, -1};
  st.AddTask(MkTask("low1", "low", 2));
  Decision d = Schedule(st, Policy::Priority, FitMethod::BestFit);
  Apply(st, d);
  st.AddTask(MkTask("high1", "high", 1));
  d = Schedule(st, Policy::Priority, FitMethod::BestFit);
  EXPECT(Released(d, "low1"));
  st.RemoveTask("low1");
  d = Schedule(st, Policy::Priority, FitMethod::BestFit);
  EXPECT(Allocated(d, "high1"));
}

TEST(round_robin_interleaves_groups) {
  PoolState st;
  st.agents["a"] = MkAgent("a", 3);
  for (int i = 0; i < 3; ++i) st.AddTask(MkTask("x" + std::to_string(i), "x", 1));
  for (int i = 0; i < 3; ++i) st.AddTask(MkTask("y" + std::to_string(i), "y", 1));
  Decision d = Schedule(st, Policy::RoundRobin, FitMethod::BestFit);
  EXPECT_EQ(d.allocate.size(), size_t(3));
  int x = 0;
  for (auto& a : d.allocate) x += a.first[0] == 'x';
  EXPECT(x == 1 || x == 2);
}

#include "detcore/lttb.h"

TEST(lttb_keeps_endpoints_and_peaks) {
  std::vector<detcore::Point> pts;
  for (int i = 0; i < 1000; ++i) pts.push_back({static_cast<double>(i), i == 500 ? 100.0 : 0.0});
  auto out = detcore::Downsample(pts, 20);
  EXPECT_EQ(out.size(), size_t(20));
  EXPECT_EQ(out.front().x, 0.0);
  EXPECT_EQ(out.back().x, 999.0);
  bool peak = false;
  for (auto& p : out) peak |= p.y == 100.0;
  EXPECT(peak);
  EXPECT_EQ(detcore::Downsample(pts, 2000).size(), size_t(1000));
}

#include "detcore/provisioner.h"

TEST(scale_decider_launch_and_idle_terminate) {
  using namespace detcore::prov;
  ProvisionerConfig cfg;
  cfg.max_instances = 3;
  cfg.slots_per_instance = 2;
  cfg.max_idle_period = std::chrono::milliseconds(1000);
  cfg.max_starting_period = std::chrono::milliseconds(5000);
  ScaleDecider sd(cfg);
  auto t0 = Clock::now();
  auto d = sd.Decide(5, {}, {}, t0);
  EXPECT_EQ(d.launch, 3);  // ceil(5/2) = 3, capped by max 3
  std::vector<Instance> inst = {{"a", "Starting", t0}, {"b", "Starting", t0}, {"c", "Starting", t0}};
  d = sd.Decide(5, {}, inst, t0 + std::chrono::milliseconds(10));
  EXPECT_EQ(d.launch, 0);  // still starting
  std::vector<AgentInfo> agents = {{"a", true}, {"b", true}, {"c", false}};
  d = sd.Decide(0, agents, inst, t0 + std::chrono::milliseconds(100));
  EXPECT(d.terminate.empty());  // idle, but not for long yet
  d = sd.Decide(0, agents, inst, t0 + std::chrono::milliseconds(1500));
  EXPECT_EQ(d.terminate.size(), size_t(2));  // a and b idle > 1s, c busy
  d = sd.Decide(0, {}, {{"z", "Starting", t0}}, t0 + std::chrono::milliseconds(6000));
  EXPECT_EQ(d.terminate.size(), size_t(1));  // never connected within the starting period
}

TEST(scale_decider_idle_connected_capacity_counts) {
  using namespace detcore::prov;
  ProvisionerConfig cfg;
  cfg.max_instances = 2;
  cfg.slots_per_instance = 1;
  cfg.max_idle_period = std::chrono::milliseconds(1500);
  ScaleDecider sd(cfg);
  auto t0 = Clock::now();
  // the launched instance's agent just connected (idle) while the trial's slot is still pending:
  // the scheduler places it there next, so no second instance
  auto d = sd.Decide(1, {{"a", true}}, {{"a", "Running", t0}}, t0 + std::chrono::milliseconds(10));
  EXPECT_EQ(d.launch, 0);
  // demand beyond the idle capacity still launches
  d = sd.Decide(2, {{"a", true}}, {{"a", "Running", t0}}, t0 + std::chrono::milliseconds(20));
  EXPECT_EQ(d.launch, 1);
}
