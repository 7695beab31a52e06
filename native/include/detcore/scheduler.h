// Resource-pool scheduling: gang placement ("fitting") and the fair_share / priority /
// round_robin schedulers (reference master/internal/resourcemanagers/
// {resource_pool,fair_share,priority,round_robin,fitting,fitting_methods}.go).
//
// Pure state + decision functions, no I/O: the master's resource-pool actor owns a PoolState,
// calls Schedule() every tick (500 ms, resource_managers.go:12) and applies the decisions
// (start allocations, ask trials to release = preemption).
#pragma once

#include <cstdint>
#include <map>
#include <optional>
#include <string>
#include <vector>

namespace detcore {
namespace sched {

struct Slot {
  int device_id = 0;
  std::string uuid;
  std::string type = "gpu";  // gpu | cpu | artificial
  bool enabled = true;
  std::string task;  // allocated task id, empty = free
};

struct Agent {
  std::string id;
  std::string label;
  std::string address;  // tie-break identity (reference: the agent actor's address); empty = id
  std::vector<Slot> slots;
  int zero_slot_tasks = 0;
  int max_zero_slot_tasks = 100;  // master max_zero_slot_containers_per_agent
  bool enabled = true;
  int NumSlots() const;
  int NumEmptySlots() const;
  int NumUsedSlots() const;
  bool Idle() const { return NumUsedSlots() == 0 && zero_slot_tasks == 0; }
};

struct Group {
  std::string id;
  double weight = 1.0;
  std::optional<int> priority;  // smaller = more important (priority scheduler)
  int max_slots = -1;           // -1: unlimited
  int64_t registered_seq = 0;   // registration order (the group actor's registration time)
};

constexpr int kDefaultPriority = 42;          // model.DefaultSchedulingPriority
constexpr int kMaxUserPriority = 99;          // model.MaxUserSchedulingPriority

struct Fit {
  std::string agent;
  std::vector<int> devices;  // device ids assigned on that agent
};

struct Task {
  std::string id;
  std::string group;
  std::string label;
  int slots_needed = 0;
  bool non_preemptible = false;
  bool single_agent = false;
  int64_t registered_seq = 0;  // registration order (treeset order in the reference)
  // filled once allocated
  std::vector<Fit> allocation;
  bool allocated() const { return !allocation.empty(); }
};

enum class FitMethod { BestFit, WorstFit };
enum class Policy { FairShare, Priority, RoundRobin };

struct Decision {
  std::vector<std::pair<std::string, std::vector<Fit>>> allocate;  // task id -> fits
  std::vector<std::string> release;                                // preemption requests
};

class PoolState {
 public:
  std::map<std::string, Agent> agents;
  std::map<std::string, Group> groups;
  std::map<std::string, Task> tasks;
  int64_t next_seq = 0;
  int64_t next_group_seq = 0;
  bool preemption = true;  // priority scheduler preemption

  Group& EnsureGroup(const std::string& id);  // creates it (weight 1, registered now) if new
  void AddTask(Task t);
  void RemoveTask(const std::string& id);  // frees its slots
  // Commit an allocation (marks devices busy).
  void Allocate(const std::string& task_id, const std::vector<Fit>& fits);
  std::vector<const Task*> TasksInOrder() const;
  int Capacity(const std::string& label) const;
};

// Gang placement for one task against the current agents (fitting.go:70 findFits): one agent
// holding the whole gang (best score, then md5 hash distance, then address), else fully unused
// agents of one size dividing the gang.
std::optional<std::vector<Fit>> FindFits(const Task& t, const std::map<std::string, Agent>& agents, FitMethod m);
// Soft-constraint score of placing `t` on `a` (fitting_methods.go BestFit / WorstFit).
double FitScore(const Task& t, const Agent& a, FitMethod m);

Decision Schedule(PoolState& st, Policy p, FitMethod m);
Policy ParsePolicy(const std::string& s);
FitMethod ParseFitMethod(const std::string& s);

}  // namespace sched
}  // namespace detcore
