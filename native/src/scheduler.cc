// Scheduling + fitting (see include/detcore/scheduler.h).
//
// fair_share: max-min progressive filling of slot offers across groups (weights), with
//   non-preemptible "pre-subscribed" slots honoured first and a deadlock breaker for groups whose
//   smallest pending gang cannot fit in its offer; groups holding more than their offer release
//   (preempt) preemptible tasks, groups under their offer start pending tasks that fit
//   (reference fair_share.go:54-307).
// priority: per label, pending tasks by (group priority, registration order); a task that does
//   not fit may preempt allocated tasks of strictly lower priority (priority.go).
// round_robin: groups with the fewest active slots go first, one task per group per round.
// fitting: single agent first (BestFit = prefer fuller agents, WorstFit = emptier), otherwise
//   dedicated idle agents with equal slot counts dividing the gang (fitting.go:70-205).
#include "detcore/scheduler.h"

#include <algorithm>
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

void PoolState::AddTask(Task t) {
  if (tasks.count(t.id)) return;
  t.registered_seq = next_seq++;
  if (!groups.count(t.group)) groups[t.group] = Group{t.group, 1.0, std::nullopt, -1};
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

// Deterministic tie-breaker between equally good agents (the reference uses an md5 distance).
uint64_t Fnv(const std::string& s) {
  uint64_t h = 1469598103934665603ull;
  for (unsigned char c : s) {
    h ^= c;
    h *= 1099511628211ull;
  }
  return h;
}

double Score(const Agent& a, FitMethod m) {
  const double empty = a.NumEmptySlots(), total = std::max(1, a.NumSlots());
  return m == FitMethod::BestFit ? 1.0 / (1.0 + empty) : empty / total;
}

std::vector<int> FreeDevices(const Agent& a, int n) {
  std::vector<int> out;
  for (auto& s : a.slots)
    if (s.enabled && s.task.empty() && static_cast<int>(out.size()) < n) out.push_back(s.device_id);
  return out;
}

bool LabelOk(const Agent& a, const Task& t) { return a.enabled && a.label == t.label; }

}  // namespace

std::optional<std::vector<Fit>> FindFits(const Task& t, const std::map<std::string, Agent>& agents, FitMethod m) {
  // 1) one agent that holds the whole gang
  const Agent* best = nullptr;
  double best_score = -1;
  uint64_t best_tie = 0;
  const uint64_t th = Fnv(t.id);
  for (auto& kv : agents) {
    const Agent& a = kv.second;
    if (!LabelOk(a, t) || a.NumEmptySlots() < t.slots_needed) continue;
    double sc = Score(a, m);
    uint64_t tie = Fnv(a.id) ^ th;
    if (!best || sc > best_score || (sc == best_score && tie < best_tie)) {
      best = &a;
      best_score = sc;
      best_tie = tie;
    }
  }
  if (best) return std::vector<Fit>{Fit{best->id, FreeDevices(*best, t.slots_needed)}};
  if (t.slots_needed <= 1 || t.single_agent) return std::nullopt;
  // 2) dedicated multi-agent fit: fully idle agents with the same slot count n, n | slots_needed,
  //    largest agents first.
  std::map<int, std::vector<const Agent*>, std::greater<int>> by_size;
  for (auto& kv : agents) {
    const Agent& a = kv.second;
    if (LabelOk(a, t) && a.Idle() && a.NumSlots() > 0) by_size[a.NumSlots()].push_back(&a);
  }
  for (auto& kv : by_size) {
    const int n = kv.first;
    if (t.slots_needed % n != 0) continue;
    const size_t need = static_cast<size_t>(t.slots_needed / n);
    if (kv.second.size() < need) continue;
    std::vector<const Agent*> cand = kv.second;
    std::sort(cand.begin(), cand.end(), [&](const Agent* x, const Agent* y) { return (Fnv(x->id) ^ th) < (Fnv(y->id) ^ th); });
    std::vector<Fit> fits;
    for (size_t i = 0; i < need; ++i) fits.push_back(Fit{cand[i]->id, FreeDevices(*cand[i], n)});
    return fits;
  }
  return std::nullopt;
}

// ------------------------------------------------------------------------------- schedulers
namespace {

// Working copy of agents so several allocations in one tick see each other's devices.
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
};

void ScheduleZeroSlot(PoolState& st, Sim& sim, FitMethod m, Decision& d) {
  for (const Task* t : st.TasksInOrder()) {
    if (t->slots_needed != 0 || t->allocated()) continue;
    if (auto fits = FindFits(*t, sim.agents, m)) {
      sim.Take(t->id, *fits);
      d.allocate.emplace_back(t->id, *fits);
    }
  }
}

struct GroupState {
  const Group* group = nullptr;
  int64_t first_seq = 0;
  std::vector<const Task*> reqs, pending, allocated;
  int demand = 0, active = 0, presubscribed = 0, offered = 0;
  bool disabled = false;
};

void FairShare(PoolState& st, Sim& sim, FitMethod m, Decision& d) {
  std::map<std::string, int> capacity;
  for (auto& kv : st.agents)
    if (kv.second.enabled) capacity[kv.second.label] += kv.second.NumSlots();
  // label -> group id -> state
  std::map<std::string, std::map<std::string, GroupState>> by_label;
  for (const Task* t : st.TasksInOrder()) {
    if (t->slots_needed == 0 || t->slots_needed > capacity[t->label]) continue;
    GroupState& g = by_label[t->label][t->group];
    if (!g.group) {
      g.group = &st.groups.at(t->group);
      g.first_seq = t->registered_seq;
    }
    g.reqs.push_back(t);
    g.demand += t->slots_needed;
    if (t->allocated()) {
      g.allocated.push_back(t);
      g.active += t->slots_needed;
      if (t->non_preemptible) g.presubscribed += t->slots_needed;
    } else {
      g.pending.push_back(t);
    }
  }
  for (auto& lab : by_label) {
    std::vector<GroupState*> states;
    for (auto& kv : lab.second) {
      GroupState& g = kv.second;
      if (g.group->max_slots >= 0) g.demand = std::min(g.demand, g.group->max_slots);
      states.push_back(&g);
    }
    int cap = capacity[lab.first];
    // non-preemptible slots are offered first
    std::map<GroupState*, int> preoffer;
    for (GroupState* g : states) {
      if (g->presubscribed == 0) continue;
      g->offered = g->presubscribed;
      preoffer[g] = g->presubscribed;
      cap -= g->presubscribed;
    }
    // progressive filling, smallest demand first (ties: older group first)
    std::sort(states.begin(), states.end(), [](GroupState* a, GroupState* b) {
      return a->demand != b->demand ? a->demand < b->demand : a->first_seq < b->first_seq;
    });
    std::vector<GroupState*> newest_first = states;
    std::sort(newest_first.begin(), newest_first.end(), [](GroupState* a, GroupState* b) { return a->first_seq > b->first_seq; });
    auto total_weight = [&] {
      double w = 0;
      for (GroupState* g : states)
        if (!g->disabled && g->offered < g->demand) w += g->group->weight;
      return w;
    };
    int left = static_cast<int>(states.size());
    double tw = total_weight();
    while (left > 0) {
      bool progress = false;
      const int start_cap = cap;
      for (GroupState* g : states) {
        if (g->disabled || g->offered == g->demand) continue;
        int share = tw > 0 ? static_cast<int>(start_cap * g->group->weight / tw) : 0;
        share = std::max(1, share);
        progress = true;
        int offer = std::min({share, cap, g->demand - g->offered});
        int& pre = preoffer[g];
        if (pre > 0) {  // already-counted presubscribed slots absorb this offer first
          int absorbed = std::min(pre, offer);
          pre -= absorbed;
          offer -= absorbed;
        }
        g->offered += offer;
        cap -= offer;
        if (g->offered == g->demand) {
          --left;
          tw = total_weight();
        }
      }
      if (cap <= 0) {
        // deadlock breaker: the newest group whose smallest pending gang exceeds its offer gives
        // its offer back
        bool adjusted = false;
        for (GroupState* g : newest_first) {
          const Task* smallest = nullptr;
          for (const Task* t : g->pending)
            if (!smallest || t->slots_needed < smallest->slots_needed) smallest = t;
          if (!g->disabled && g->offered != g->demand && smallest && smallest->slots_needed > g->offered) {
            cap += g->offered;
            g->offered = 0;
            g->disabled = true;
            adjusted = true;
            --left;
            tw = total_weight();
            break;
          }
        }
        if (!adjusted) break;
      } else if (!progress) {
        break;
      }
    }
    // decisions
    for (GroupState* g : states) {
      if (g->active > g->offered) {
        for (const Task* t : g->allocated) {
          if (t->non_preemptible) continue;
          d.release.push_back(t->id);
          g->active -= t->slots_needed;
          if (g->active <= g->offered) break;
        }
      } else if (g->active < g->offered) {
        int room = g->offered - g->active;
        for (const Task* t : g->pending) {
          if (t->slots_needed > room) continue;
          auto fits = FindFits(*t, sim.agents, m);
          if (!fits) continue;
          sim.Take(t->id, *fits);
          d.allocate.emplace_back(t->id, *fits);
          room -= t->slots_needed;
        }
      }
    }
  }
}

void PrioritySched(PoolState& st, Sim& sim, FitMethod m, Decision& d) {
  auto prio = [&](const Task* t) {
    auto& g = st.groups.at(t->group);
    return g.priority ? *g.priority : 42;  // reference default priority
  };
  std::vector<const Task*> order = st.TasksInOrder();
  std::stable_sort(order.begin(), order.end(), [&](const Task* a, const Task* b) { return prio(a) < prio(b); });
  std::set<std::string> releasing;
  for (const Task* t : order) {
    if (t->allocated() || t->slots_needed == 0) continue;
    if (auto fits = FindFits(*t, sim.agents, m)) {
      sim.Take(t->id, *fits);
      d.allocate.emplace_back(t->id, *fits);
      continue;
    }
    if (!st.preemption) continue;
    // preempt strictly lower-priority allocated tasks (lowest priority, newest first) until the
    // freed slots could hold the gang; actual start happens on a later tick once released.
    std::vector<const Task*> victims;
    for (const Task* o : order)
      if (o->allocated() && !o->non_preemptible && prio(o) > prio(t) && !releasing.count(o->id) && o->label == t->label)
        victims.push_back(o);
    std::sort(victims.begin(), victims.end(), [&](const Task* a, const Task* b) {
      return prio(a) != prio(b) ? prio(a) > prio(b) : a->registered_seq > b->registered_seq;
    });
    int freed = 0;
    int free_now = 0;
    for (auto& kv : sim.agents)
      if (kv.second.label == t->label) free_now += kv.second.NumEmptySlots();
    for (const Task* v : victims) {
      if (free_now + freed >= t->slots_needed) break;
      releasing.insert(v->id);
      d.release.push_back(v->id);
      freed += v->slots_needed;
    }
  }
}

void RoundRobin(PoolState& st, Sim& sim, FitMethod m, Decision& d) {
  std::map<std::string, int> active;
  std::map<std::string, std::vector<const Task*>> pending;
  for (const Task* t : st.TasksInOrder()) {
    if (t->slots_needed == 0) continue;
    if (t->allocated()) active[t->group] += t->slots_needed;
    else pending[t->group].push_back(t);
  }
  std::vector<std::string> groups;
  for (auto& kv : pending) groups.push_back(kv.first);
  std::stable_sort(groups.begin(), groups.end(), [&](const std::string& a, const std::string& b) { return active[a] < active[b]; });
  std::map<std::string, size_t> cursor;
  bool any = true;
  while (any) {
    any = false;
    for (auto& g : groups) {
      auto& v = pending[g];
      size_t& c = cursor[g];
      while (c < v.size()) {
        const Task* t = v[c++];
        if (auto fits = FindFits(*t, sim.agents, m)) {
          sim.Take(t->id, *fits);
          d.allocate.emplace_back(t->id, *fits);
          any = true;
          break;
        }
      }
    }
  }
}

}  // namespace

Decision Schedule(PoolState& st, Policy p, FitMethod m) {
  Decision d;
  Sim sim{st.agents};
  ScheduleZeroSlot(st, sim, m, d);
  switch (p) {
    case Policy::FairShare: FairShare(st, sim, m, d); break;
    case Policy::Priority: PrioritySched(st, sim, m, d); break;
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
