// Scheduling + fitting (see include/detcore/scheduler.h).
//
// fitting (fitting.go, fitting_methods.go): a shared fit on one agent first — hard constraints
//   slots / zero-slot cap / label, candidates ordered by soft score (BestFit: fuller agents,
//   WorstFit: emptier), then by md5 hash distance task->agent (load-balances equal scores, the
//   reference's exact tie-break), then by address; otherwise a dedicated fit on fully unused agents
//   of one size n dividing the gang (largest n first).
// fair_share (fair_share.go): per agent label, groups' slot demands are offered capacity by
//   progressive filling (max-min fairness, weights, non-preemptible "presubscribed" slots first,
//   deadlock breaker for groups whose smallest pending gang exceeds their offer); groups over their
//   offer release preemptible tasks, groups under it start pending tasks that fit.
// priority (priority.go): per label, zero-slot and slot tasks separately; pending tasks by (group
//   priority, registration); once a priority level leaves a task unplaced no lower level starts;
//   with preemption, a task that does not fit preempts strictly lower-priority tasks (newest first)
//   only if that makes it fit.
// round_robin (round_robin.go): groups by active slots, one task per group per round; a group whose
//   next task does not fit leaves the rotation.
// Within one pass, placements are applied to a working copy of the agents (the reference re-fits at
// allocation time; doing it here means a decision never double-books a device).
#include "detcore/scheduler.h"

#include <algorithm>
#include <cmath>
#include <cstring>
#include <functional>
#include <limits>
#include <set>
#include <stdexcept>

namespace detcore {
namespace sched {

int Agent::NumSlots() const {
  int n = 0;
  for (auto& s : slots)
    if (s.enabled) ++n;
  return n;
}
int Agent::NumEmptySlots() const {
  int n = 0;
  for (auto& s : slots)
    if (s.enabled && s.task.empty()) ++n;
  return n;
}
int Agent::NumUsedSlots() const {
  int n = 0;
  for (auto& s : slots)
    if (!s.task.empty()) ++n;
  return n;
}

Group& PoolState::EnsureGroup(const std::string& id) {
  auto it = groups.find(id);
  if (it != groups.end()) return it->second;
  Group g;
  g.id = id;
  g.registered_seq = next_group_seq++;
  return groups.emplace(id, g).first->second;
}

void PoolState::AddTask(Task t) {
  if (tasks.count(t.id)) return;
  t.registered_seq = next_seq++;
  EnsureGroup(t.group);
  tasks[t.id] = std::move(t);
}

void PoolState::RemoveTask(const std::string& id) {
  auto it = tasks.find(id);
  if (it == tasks.end()) return;
  for (auto& f : it->second.allocation) {
    auto a = agents.find(f.agent);
    if (a == agents.end()) continue;
    if (it->second.slots_needed == 0) a->second.zero_slot_tasks = std::max(0, a->second.zero_slot_tasks - 1);
    for (auto& s : a->second.slots)
      if (s.task == id) s.task.clear();
  }
  tasks.erase(it);
}

void PoolState::Allocate(const std::string& task_id, const std::vector<Fit>& fits) {
  auto it = tasks.find(task_id);
  if (it == tasks.end()) return;
  for (auto& f : fits) {
    auto& a = agents.at(f.agent);
    if (f.devices.empty()) ++a.zero_slot_tasks;
    for (int d : f.devices)
      for (auto& s : a.slots)
        if (s.device_id == d) s.task = task_id;
  }
  it->second.allocation = fits;
}

std::vector<const Task*> PoolState::TasksInOrder() const {
  std::vector<const Task*> out;
  for (auto& kv : tasks) out.push_back(&kv.second);
  std::sort(out.begin(), out.end(), [](const Task* a, const Task* b) { return a->registered_seq < b->registered_seq; });
  return out;
}

int PoolState::Capacity(const std::string& label) const {
  int c = 0;
  for (auto& kv : agents)
    if (kv.second.label == label && kv.second.enabled) c += kv.second.NumSlots();
  return c;
}

// ------------------------------------------------------------------------------------ fitting
namespace {

// MD5 (RFC 1321) of a short string; the low 8 digest bytes little-endian, as stringHashNumber
// (fitting.go:199) reads them.
uint64_t Md5Lo64(const std::string& msg) {
  static const uint32_t K[64] = {
      0xd76aa478, 0xe8c7b756, 0x242070db, 0xc1bdceee, 0xf57c0faf, 0x4787c62a, 0xa8304613, 0xfd469501,
      0x698098d8, 0x8b44f7af, 0xffff5bb1, 0x895cd7be, 0x6b901122, 0xfd987193, 0xa679438e, 0x49b40821,
      0xf61e2562, 0xc040b340, 0x265e5a51, 0xe9b6c7aa, 0xd62f105d, 0x02441453, 0xd8a1e681, 0xe7d3fbc8,
      0x21e1cde6, 0xc33707d6, 0xf4d50d87, 0x455a14ed, 0xa9e3e905, 0xfcefa3f8, 0x676f02d9, 0x8d2a4c8a,
      0xfffa3942, 0x8771f681, 0x6d9d6122, 0xfde5380c, 0xa4beea44, 0x4bdecfa9, 0xf6bb4b60, 0xbebfbc70,
      0x289b7ec6, 0xeaa127fa, 0xd4ef3085, 0x04881d05, 0xd9d4d039, 0xe6db99e5, 0x1fa27cf8, 0xc4ac5665,
      0xf4292244, 0x432aff97, 0xab9423a7, 0xfc93a039, 0x655b59c3, 0x8f0ccc92, 0xffeff47d, 0x85845dd1,
      0x6fa87e4f, 0xfe2ce6e0, 0xa3014314, 0x4e0811a1, 0xf7537e82, 0xbd3af235, 0x2ad7d2bb, 0xeb86d391};
  static const int R[64] = {7, 12, 17, 22, 7, 12, 17, 22, 7, 12, 17, 22, 7, 12, 17, 22,
                            5, 9,  14, 20, 5, 9,  14, 20, 5, 9,  14, 20, 5, 9,  14, 20,
                            4, 11, 16, 23, 4, 11, 16, 23, 4, 11, 16, 23, 4, 11, 16, 23,
                            6, 10, 15, 21, 6, 10, 15, 21, 6, 10, 15, 21, 6, 10, 15, 21};
  std::vector<uint8_t> m(msg.begin(), msg.end());
  const uint64_t bits = static_cast<uint64_t>(msg.size()) * 8;
  m.push_back(0x80);
  while (m.size() % 64 != 56) m.push_back(0);
  for (int i = 0; i < 8; ++i) m.push_back(static_cast<uint8_t>(bits >> (8 * i)));
  uint32_t h0 = 0x67452301, h1 = 0xefcdab89, h2 = 0x98badcfe, h3 = 0x10325476;
  for (size_t off = 0; off < m.size(); off += 64) {
    uint32_t w[16];
    for (int i = 0; i < 16; ++i)
      w[i] = static_cast<uint32_t>(m[off + 4 * i]) | (static_cast<uint32_t>(m[off + 4 * i + 1]) << 8) |
             (static_cast<uint32_t>(m[off + 4 * i + 2]) << 16) | (static_cast<uint32_t>(m[off + 4 * i + 3]) << 24);
    uint32_t a = h0, b = h1, c = h2, d = h3;
    for (int i = 0; i < 64; ++i) {
      uint32_t f;
      int g;
      if (i < 16) { f = (b & c) | (~b & d); g = i; }
      else if (i < 32) { f = (d & b) | (~d & c); g = (5 * i + 1) % 16; }
      else if (i < 48) { f = b ^ c ^ d; g = (3 * i + 5) % 16; }
      else { f = c ^ (b | ~d); g = (7 * i) % 16; }
      const uint32_t t = d;
      d = c;
      c = b;
      const uint32_t x = a + f + K[i] + w[g];
      b = b + ((x << R[i]) | (x >> (32 - R[i])));
      a = t;
    }
    h0 += a; h1 += b; h2 += c; h3 += d;
  }
  return static_cast<uint64_t>(h0) | (static_cast<uint64_t>(h1) << 32);
}

const std::string& Address(const Agent& a) { return a.address.empty() ? a.id : a.address; }

bool LabelOk(const Agent& a, const Task& t) { return a.enabled && a.label == t.label; }

bool ZeroSlotCapOk(const Task& t, const Agent& a) {
  if (t.slots_needed != 0) return true;
  return a.max_zero_slot_tasks > 0 && a.zero_slot_tasks < a.max_zero_slot_tasks;
}

std::vector<int> FreeDevices(const Agent& a, int n) {
  std::vector<int> out;
  for (auto& s : a.slots)
    if (s.enabled && s.task.empty() && static_cast<int>(out.size()) < n) out.push_back(s.device_id);
  return out;
}

struct Candidate {
  const Agent* agent;
  double score;
  uint64_t hash_distance;
};

void SortCandidates(std::vector<Candidate>& c) {
  std::sort(c.begin(), c.end(), [](const Candidate& a, const Candidate& b) {
    if (a.score != b.score) return a.score > b.score;
    if (a.hash_distance != b.hash_distance) return a.hash_distance < b.hash_distance;
    return Address(*a.agent) < Address(*b.agent);
  });
}

}  // namespace

double FitScore(const Task& t, const Agent& a, FitMethod m) {
  const int used = a.NumUsedSlots(), empty = a.NumEmptySlots(), total = a.NumSlots();
  const int maxz = a.max_zero_slot_tasks, zero = a.zero_slot_tasks;
  if (m == FitMethod::BestFit) {
    if (used != 0 || t.slots_needed != 0) return 1.0 / (1.0 + empty);
    if (maxz == 0) return 0.0;
    return 1.0 / (1.0 + (maxz - zero));
  }
  if (used != 0 || t.slots_needed != 0) return total > 0 ? static_cast<double>(empty) / total : 0.0;
  if (maxz == 0) return 0.0;
  return static_cast<double>(maxz - zero) / maxz;
}

std::optional<std::vector<Fit>> FindFits(const Task& t, const std::map<std::string, Agent>& agents, FitMethod m) {
  const uint64_t th = Md5Lo64(t.id);
  // 1) shared fit: one agent holds the whole gang
  std::vector<Candidate> cand;
  for (auto& kv : agents) {
    const Agent& a = kv.second;
    if (!LabelOk(a, t) || a.NumEmptySlots() < t.slots_needed || !ZeroSlotCapOk(t, a)) continue;
    cand.push_back(Candidate{&a, FitScore(t, a, m), th - Md5Lo64(Address(a))});
  }
  if (!cand.empty()) {
    SortCandidates(cand);
    return std::vector<Fit>{Fit{cand[0].agent->id, FreeDevices(*cand[0].agent, t.slots_needed)}};
  }
  if (t.single_agent || t.slots_needed <= 1) return std::nullopt;
  // 2) dedicated multi-agent fit: unused agents grouped by free slots, largest size first
  std::map<int, std::vector<const Agent*>, std::greater<int>> by_size;
  for (auto& kv : agents) {
    const Agent& a = kv.second;
    if (LabelOk(a, t) && a.NumUsedSlots() == 0) by_size[a.NumEmptySlots()].push_back(&a);
  }
  for (auto& kv : by_size) {
    const int n = kv.first;
    if (n == 0 || t.slots_needed % n != 0) continue;
    if (static_cast<int>(kv.second.size()) * n < t.slots_needed) continue;
    std::vector<Candidate> c;
    for (const Agent* a : kv.second) c.push_back(Candidate{a, FitScore(t, *a, m), th - Md5Lo64(Address(*a))});
    SortCandidates(c);
    std::vector<Fit> fits;
    const size_t need = static_cast<size_t>(t.slots_needed / n);
    for (size_t i = 0; i < need; ++i) fits.push_back(Fit{c[i].agent->id, FreeDevices(*c[i].agent, n)});
    return fits;
  }
  return std::nullopt;
}

// ------------------------------------------------------------------------------- schedulers
namespace {

// Working copy of agents so several allocations in one pass see each other's devices.
struct Sim {
  std::map<std::string, Agent> agents;
  void Take(const std::string& task, const std::vector<Fit>& fits) {
    for (auto& f : fits) {
      auto& a = agents.at(f.agent);
      if (f.devices.empty()) ++a.zero_slot_tasks;
      for (int d : f.devices)
        for (auto& s : a.slots)
          if (s.device_id == d) s.task = task;
    }
  }
  void Free(const Task& t) {  // removeTaskFromAgents (priority.go:304)
    for (auto& f : t.allocation) {
      auto it = agents.find(f.agent);
      if (it == agents.end()) continue;
      if (f.devices.empty() && t.slots_needed == 0) it->second.zero_slot_tasks = std::max(0, it->second.zero_slot_tasks - 1);
      for (int d : f.devices)
        for (auto& s : it->second.slots)
          if (s.device_id == d) s.task.clear();
    }
  }
};

struct GroupState {
  const Group* group = nullptr;
  std::vector<const Task*> pending, allocated;
  int demand = 0, active = 0, presubscribed = 0, offered = 0;
  bool disabled = false;
};

// accountForPreoffers (fair_share.go:167), including its sequential-if behaviour: when the offer
// exceeds the remaining pre-offer the pre-offer is cleared without reducing the offer.
void AccountForPreoffers(int& pre, int& offer) {
  if (pre > 0) {
    if (pre == offer) { pre = 0; offer = 0; }
    if (pre > offer) { pre -= offer; offer = 0; }
    if (pre < offer) { pre = 0; }
  }
}

void AllocateSlotOffers(std::vector<GroupState*>& states, int capacity) {
  std::map<GroupState*, int> preoffers;
  for (GroupState* g : states) {
    if (g->presubscribed == 0) continue;
    g->offered = g->presubscribed;
    preoffers[g] = g->presubscribed;
    capacity -= g->presubscribed;
  }
  std::sort(states.begin(), states.end(), [](GroupState* a, GroupState* b) {
    return a->demand != b->demand ? a->demand < b->demand : a->group->registered_seq < b->group->registered_seq;
  });
  // byTime (fair_share.go:219): the reference sorts a copy with a comparator that indexes the
  // ORIGINAL slice, i.e. an insertion sort whose comparisons are fixed by `states`' order
  // (sort.Slice on < 12 elements); reproduced so the deadlock breaker picks the same group.
  std::vector<GroupState*> by_time = states;
  if (by_time.size() < 12) {
    for (size_t i = 1; i < by_time.size(); ++i)
      for (size_t j = i; j > 0 && states[j]->group->registered_seq > states[j - 1]->group->registered_seq; --j)
        std::swap(by_time[j], by_time[j - 1]);
  } else {
    std::stable_sort(by_time.begin(), by_time.end(),
                     [](GroupState* a, GroupState* b) { return a->group->registered_seq > b->group->registered_seq; });
  }
  auto total_weight = [&] {
    double w = 0;
    for (GroupState* g : states)
      if (!g->disabled && g->offered < g->demand) w += g->group->weight;
    return w;
  };
  double tw = total_weight();
  for (int left = static_cast<int>(states.size()); left > 0;) {
    bool progress = false;
    const int start_cap = capacity;
    for (GroupState* g : states) {
      if (g->disabled || g->offered == g->demand) continue;
      // int(NaN) (zero total weight) is the minimum int in Go: the share is then 1
      int share = (tw > 0) ? static_cast<int>(static_cast<double>(start_cap) * g->group->weight / tw) : 0;
      share = std::max(1, share);
      progress = true;
      int offer = std::min({share, capacity, g->demand - g->offered});
      AccountForPreoffers(preoffers[g], offer);
      g->offered += offer;
      capacity -= offer;
      if (g->offered == g->demand) {
        --left;
        tw = total_weight();
      }
    }
    if (capacity == 0) {
      bool adjusted = false;
      for (GroupState* g : by_time) {
        const Task* smallest = nullptr;
        for (const Task* t : g->pending)
          if (!smallest || t->slots_needed < smallest->slots_needed) smallest = t;
        if (!g->disabled && g->offered != g->demand && smallest && smallest->slots_needed > g->offered) {
          capacity += g->offered;
          g->offered = 0;
          g->disabled = true;
          adjusted = true;
          --left;
          tw = total_weight();
          break;
        }
      }
      if (!adjusted) return;
    } else if (!progress) {
      return;
    }
  }
}

void FairShare(PoolState& st, Sim& sim, FitMethod m, Decision& d) {
  for (const Task* t : st.TasksInOrder()) {  // zero-slot tasks start whenever they fit
    if (t->slots_needed != 0 || t->allocated()) continue;
    if (auto fits = FindFits(*t, sim.agents, m)) {
      sim.Take(t->id, *fits);
      d.allocate.emplace_back(t->id, *fits);
    }
  }
  std::map<std::string, int> capacity;
  for (auto& kv : st.agents) capacity[kv.second.label] += kv.second.NumSlots();
  std::map<std::string, std::vector<GroupState*>> by_label;
  std::map<std::string, GroupState> storage;  // key: label + '\0' + group
  for (const Task* t : st.TasksInOrder()) {
    if (t->slots_needed == 0 || t->slots_needed > capacity[t->label]) continue;
    const std::string key = t->label + std::string(1, '\0') + t->group;
    auto it = storage.find(key);
    if (it == storage.end()) {
      it = storage.emplace(key, GroupState{}).first;
      it->second.group = &st.groups.at(t->group);
      by_label[t->label].push_back(&it->second);
    }
    GroupState& g = it->second;
    g.demand += t->slots_needed;
    if (t->allocated()) {
      if (t->non_preemptible) g.presubscribed += t->slots_needed;
      g.allocated.push_back(t);
      g.active += t->slots_needed;
    } else {
      g.pending.push_back(t);
    }
  }
  for (auto& lab : by_label) {
    for (GroupState* g : lab.second)
      if (g->group->max_slots >= 0) g->demand = std::min(g->demand, g->group->max_slots);
    AllocateSlotOffers(lab.second, capacity[lab.first]);
    for (GroupState* g : lab.second) {
      if (g->active > g->offered) {
        for (const Task* t : g->allocated) {
          if (t->non_preemptible) continue;
          d.release.push_back(t->id);
          g->active -= t->slots_needed;
          if (g->active <= g->offered) break;
        }
      } else if (g->active < g->offered) {
        g->offered -= g->active;
        for (const Task* t : g->pending) {
          if (t->slots_needed > g->offered) continue;
          auto fits = FindFits(*t, sim.agents, m);
          if (!fits) continue;
          sim.Take(t->id, *fits);
          d.allocate.emplace_back(t->id, *fits);
          g->offered -= t->slots_needed;
        }
      }
    }
  }
}

int PriorityOf(const PoolState& st, const Task* t) {
  auto it = st.groups.find(t->group);
  if (it == st.groups.end() || !it->second.priority) return kDefaultPriority;
  return *it->second.priority;
}

// prioritySchedulerWithFilter (priority.go:80) for the tasks of one label passing `filter`.
void PriorityPass(PoolState& st, const std::map<std::string, Agent>& label_agents, const std::string& label,
                  FitMethod m, bool zero_slot, Decision& d, std::set<std::string>& released) {
  std::map<int, std::vector<const Task*>> pending, scheduled;
  for (const Task* t : st.TasksInOrder()) {
    if (t->label != label || (t->slots_needed == 0) != zero_slot) continue;
    (t->allocated() ? scheduled : pending)[PriorityOf(st, t)].push_back(t);
  }
  for (auto& kv : scheduled) std::reverse(kv.second.begin(), kv.second.end());  // newest first
  Sim local{label_agents};
  bool start = true;
  std::set<std::string> to_release;
  for (auto& kv : pending) {
    const int prio = kv.first;
    std::vector<const Task*> failed;
    std::vector<std::pair<const Task*, std::vector<Fit>>> ok;
    for (const Task* t : kv.second) {
      auto fits = FindFits(*t, local.agents, m);
      if (!fits) {
        failed.push_back(t);
        continue;
      }
      local.Take(t->id, *fits);
      ok.emplace_back(t, *fits);
    }
    if (start)
      for (auto& a : ok) d.allocate.emplace_back(a.first->id, a.second);
    if (failed.empty()) continue;
    start = false;
    if (!st.preemption) break;
    for (const Task* t : failed) {
      if (auto fits = FindFits(*t, local.agents, m)) {  // fits once already-chosen preemptions land
        local.Take(t->id, *fits);
        continue;
      }
      // trySchedulingTaskViaPreemption (priority.go:162)
      Sim trial = local;
      std::vector<std::string> preempted;
      bool placed = false;
      for (int p = kMaxUserPriority; p > prio && !placed; --p) {
        auto sit = scheduled.find(p);
        if (sit == scheduled.end()) continue;
        for (const Task* c : sit->second) {
          if (c->non_preemptible || to_release.count(c->id) || released.count(c->id)) continue;
          trial.Free(*c);
          preempted.push_back(c->id);
          if (auto fits = FindFits(*t, trial.agents, m)) {
            trial.Take(t->id, *fits);
            placed = true;
            break;
          }
        }
      }
      if (placed) {
        local = trial;
        for (auto& id : preempted) to_release.insert(id);
      }
    }
  }
  for (auto& id : to_release)
    if (released.insert(id).second) d.release.push_back(id);
}

void PrioritySched(PoolState& st, FitMethod m, Decision& d) {
  std::map<std::string, std::map<std::string, Agent>> by_label;
  for (auto& kv : st.agents) by_label[kv.second.label][kv.first] = kv.second;
  std::set<std::string> released;
  for (auto& lab : by_label) {
    PriorityPass(st, lab.second, lab.first, m, true, d, released);
    PriorityPass(st, lab.second, lab.first, m, false, d, released);
  }
}

void RoundRobin(PoolState& st, Sim& sim, FitMethod m, Decision& d) {
  struct RR {
    const Group* group;
    int active = 0;
    std::vector<const Task*> pending;
    size_t next = 0;
  };
  std::vector<RR> states;
  std::map<std::string, size_t> idx;
  for (const Task* t : st.TasksInOrder()) {
    auto it = idx.find(t->group);
    if (it == idx.end()) {
      it = idx.emplace(t->group, states.size()).first;
      states.push_back(RR{&st.groups.at(t->group)});
    }
    RR& g = states[it->second];
    if (t->allocated()) g.active += t->slots_needed;
    else g.pending.push_back(t);
  }
  std::stable_sort(states.begin(), states.end(), [](const RR& a, const RR& b) {
    return a.active != b.active ? a.active < b.active : a.group->registered_seq < b.group->registered_seq;
  });
  std::vector<RR*> live;
  for (auto& s : states) live.push_back(&s);
  while (!live.empty()) {
    std::vector<RR*> keep;
    for (RR* g : live) {
      if (g->next >= g->pending.size()) continue;
      const Task* t = g->pending[g->next];
      auto fits = FindFits(*t, sim.agents, m);
      if (!fits) continue;  // the group leaves the rotation
      sim.Take(t->id, *fits);
      d.allocate.emplace_back(t->id, *fits);
      ++g->next;
      keep.push_back(g);
    }
    live = keep;
  }
}

}  // namespace

Decision Schedule(PoolState& st, Policy p, FitMethod m) {
  Decision d;
  Sim sim{st.agents};
  switch (p) {
    case Policy::FairShare: FairShare(st, sim, m, d); break;
    case Policy::Priority: PrioritySched(st, m, d); break;
    case Policy::RoundRobin: RoundRobin(st, sim, m, d); break;
  }
  return d;
}

Policy ParsePolicy(const std::string& s) {
  if (s == "fair_share" || s.empty()) return Policy::FairShare;
  if (s == "priority") return Policy::Priority;
  if (s == "round_robin") return Policy::RoundRobin;
  throw std::invalid_argument("unknown scheduler type: " + s);
}

FitMethod ParseFitMethod(const std::string& s) {
  if (s == "best" || s.empty()) return FitMethod::BestFit;
  if (s == "worst") return FitMethod::WorstFit;
  throw std::invalid_argument("unknown fitting policy: " + s);
}

}  // namespace sched
}  // namespace detcore
