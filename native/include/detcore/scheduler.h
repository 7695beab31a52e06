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
  std::vector<Slot> slots;
  int zero_slot_tasks = 0;
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
};

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
  bool preemption = true;  // priority scheduler preemption

  void AddTask(Task t);
  void RemoveTask(const std::string& id);  // frees its slots
  // Commit an allocation (marks devices busy).
  void Allocate(const std::string& task_id, const std::vector<Fit>& fits);
  std::vector<const Task*> TasksInOrder() const;
  int Capacity(const std::string& label) const;
};

// Gang placement for one task against the current agents (fitting.go:70 findFits).
std::optional<std::vector<Fit>> FindFits(const Task& t, const std::map<std::string, Agent>& agents, FitMethod m);

Decision Schedule(PoolState& st, Policy p, FitMethod m);
Policy ParsePolicy(const std::string& s);
FitMethod ParseFitMethod(const std::string& s);

}  // namespace sched
}  // namespace detcore
