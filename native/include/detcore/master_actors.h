// Actors and messages of det-master (implementation: src/master_actors.cc).
#pragma once

#include <map>
#include <memory>
#include <optional>
#include <set>
#include <string>
#include <vector>

#include "detcore/actor.h"
#include "detcore/master.h"
#include "detcore/provisioner.h"
#include "detcore/scheduler.h"
#include "detcore/searcher.h"
#include "detcore/sequencer.h"
#include "detcore/workload.h"

namespace detcore {
namespace master {

// ------------------------------------------------------------------ resource-pool messages
struct SchedulerTick {};
struct SchedulerKick {};  // event-driven pass between ticks (task added / released, agent joined)
struct AddAgent {
  sched::Agent agent;
};
struct RemoveAgent {
  std::string id;
};
struct AllocateRequest {
  std::string task_id;
  std::string group;
  int slots = 0;
  std::string label;
  bool non_preemptible = false;
  actor::Ref handler;
  std::string name;
};
struct ResourcesAllocated {
  std::string task_id;
  std::vector<sched::Fit> fits;
};
struct ReleaseResources {  // pool -> task: please give the slots back (preemption)
  std::string task_id;
};
struct ResourcesReleased {  // task -> pool: slots are free
  std::string task_id;
};
struct SetGroup {
  std::string group;
  double weight = 1.0;
  std::optional<int> priority;
  int max_slots = -1;
};
struct SetSlotEnabled {
  std::string agent;
  int device = -1;  // -1: whole agent
  bool enabled = true;
};
struct PoolSummary {};

// ------------------------------------------------------------------------- trial messages
struct TrialOps {
  Ops ops;
};
struct TrialRestore {
  Ops ops;
};
struct TrialClose {};
struct TrialKill {};
struct ContainerStateMsg {
  std::string container_id;
  std::string state;  // Assigned | Starting | Running | Terminated
  int exit_code = 0;
  std::string failure;
  std::string address;
};
struct SocketConnected {
  std::string container_id;
  net::WsPtr ws;
};
struct SocketMessage {
  std::string container_id;
  Json msg;
};
struct SocketClosed {
  std::string container_id;
};
struct ExpStateChange {
  std::string state;
  bool kill = false;
};
struct TerminateTimeout {
  int gen = 0;
};
struct WorkloadAck {
  bool best = false;
};

// -------------------------------------------------------------------- experiment messages
struct TrialCreatedMsg {
  Op create;
  int64_t trial_id = 0;
};
struct TrialWorkloadDone {
  int64_t trial_id = 0;
  std::string request_id;
  Json completed;
  double units = 0;
};
struct TrialOpCompleted {
  int64_t trial_id = 0;
  Op op;
  Json metrics;
};
struct TrialExitedMsg {
  int64_t trial_id = 0;
  ExitedReason reason = ExitedReason::Errored;
};
struct SetExperimentState {
  std::string state;
  bool kill = false;
};
struct PatchExperimentConfig {  // det experiment set gc-policy / weight / priority / max-slots
  Json patch;
};
struct ReplayEvents {
  std::vector<Json> events;
};

// --------------------------------------------------------------------------------- actors
class ResourcePoolActor : public actor::Actor {
 public:
  ResourcePoolActor(Master* m, std::string name);
  void Receive(actor::Context& ctx) override;

 private:
  Master* m_;
  std::string name_;
  sched::PoolState st_;
  sched::Policy policy_;
  sched::FitMethod fit_;
  std::map<std::string, actor::Ref> handlers_;
  std::set<std::string> released_;
  bool kick_pending_ = false;
  void Kick(actor::Context& ctx);
  void SchedulePass(actor::Context& ctx);
};

class ExperimentActor : public actor::Actor {
 public:
  ExperimentActor(Master* m, int64_t id, Json config, bool replay);
  void Receive(actor::Context& ctx) override;

 private:
  void ProcessOps(actor::Context& ctx, const Ops& ops);
  void MaybeFinish(actor::Context& ctx);
  void ChildGone(actor::Context& ctx, const actor::Ref& child);
  void Replay(actor::Context& ctx, const std::vector<Json>& events);
  void Event(const std::string& type, Json body);
  void SaveState();
  bool IsBest(double metric);
  static bool IsTerminal(const std::string& s);
  actor::Ref TrialRef(actor::Context& ctx, const RequestID& rid);

  Master* m_;
  int64_t id_;
  Json config_;
  bool replaying_;
  std::unique_ptr<Searcher> searcher_;
  bool smaller_is_better_ = true;
  std::string metric_;
  std::string pool_;
  std::string state_ = "ACTIVE";
  std::string reported_state_;  // last state sent to telemetry
  bool shutdown_ = false, shutdown_failure_ = false, stopping_ = false;
  bool has_best_ = false;
  double best_metric_ = 0;
  Json best_validation_;
  std::map<std::string, Json> latest_ckpt_;  // request id -> latest checkpoint metadata (PBT)
};

// Elastic agent provisioning for one pool: a 1 s tick feeds the pool's demand to
// the ScaleDecider and applies its launch/terminate decisions through the provider.
class ProvisionerActor : public actor::Actor {
 public:
  ProvisionerActor(Master* m, std::string pool, prov::ProvisionerConfig cfg);
  void Receive(actor::Context& ctx) override;

 private:
  Master* m_;
  std::string pool_;
  prov::ProvisionerConfig cfg_;
  prov::ScaleDecider decider_;
  std::unique_ptr<prov::Provider> provider_;
};

// Generic command task (reference master/internal/command/command.go): run an argv
// on an agent with N slots (0 = CPU-only, non-preemptible), stream its logs, report exit status.
struct CommandKill {};
struct ServiceReady {  // a command's HTTP service is listening (POST /commands/:id/ready)
  int port = 0;
};
class CommandActor : public actor::Actor {
 public:
  // secret_env: "K=V" entries (e.g. DET_SHELL_TOKEN) handed to the container's environment only;
  // never written to the store, so no API response can return them.
  CommandActor(Master* m, int64_t id, Json config, Json secret_env = Json::array());
  void Receive(actor::Context& ctx) override;

 private:
  void Save(const std::string& state, int exit_code = 0);
  Master* m_;
  int64_t id_;
  Json config_;
  Json secret_env_;
  std::string pool_;
  std::string task_id_;
  std::string container_;
  std::string agent_;
  std::string address_;  // agent address the container runs at (for the service proxy)
  bool killed_ = false;
};

struct TrialSpec {
  Op create;
  Json warm_start;
  int64_t trial_id = 0;  // non-zero when restored
};

// Rendezvous information every rank of a distributed trial receives (reference trial.go
// pushRendezvous / rendezvousInfoMessage): the chief-first list of "host:port" addresses of each
// container's rendezvous port (1734 + its lowest device id, the slot-offset port the harness
// binds) and the second list 16 ports higher, identical for every rank but the rank itself.
struct RendezvousMember {
  int rank = 0;
  std::string host;
  std::vector<int> devices;
};
Json RendezvousInfo(std::vector<RendezvousMember> members, int rank);

class TrialActor : public actor::Actor {
 public:
  TrialActor(Master* m, actor::Ref exp, int64_t exp_id, Json config, std::string pool, TrialSpec spec,
             std::string exp_state);
  void Receive(actor::Context& ctx) override;

 private:
  struct Container {
    std::string id, agent;
    int rank = 0;
    std::vector<int> devices;
    std::string state = "Assigned";
    std::string address;
    int exit_code = 0;
    std::string failure;
    net::WsPtr ws;
  };
  std::string TaskID() const;
  void Advance(actor::Context& ctx);
  void RequestResources(actor::Context& ctx);
  void OnAllocated(actor::Context& ctx, const ResourcesAllocated& ra);
  void OnContainerState(actor::Context& ctx, const ContainerStateMsg& cs);
  void MaybeRendezvous(actor::Context& ctx);
  void OnSocketMessage(actor::Context& ctx, const SocketMessage& sm);
  void OnWorkloadAck(actor::Context& ctx, bool best);
  void SendNext(actor::Context& ctx);
  void SendWorkload(actor::Context& ctx, const Workload& w);
  void Terminate(actor::Context& ctx);
  void Kill(actor::Context& ctx);
  void SignalContainer(const std::string& cid, const std::string& sig);
  void CheckAllTerminated(actor::Context& ctx);
  void RollBack();
  void RestoreFromStore();
  void SaveWorkloadStart(const Workload& w);
  void SaveWorkloadEnd(const CompletedMessage& cm);

  Master* m_;
  actor::Ref exp_;
  int64_t exp_id_;
  Json config_;
  std::string pool_;
  TrialSpec spec_;
  std::string exp_state_;
  std::unique_ptr<TrialWorkloadSequencer> seq_;
  int64_t trial_id_ = 0;
  int max_restarts_ = 5;
  int slots_ = 1;
  std::string rid_;
  int alloc_gen_ = 0;
  std::string task_id_;
  std::map<std::string, Container> containers_;
  std::vector<std::string> order_;
  bool closing_ = false, canceled_ = false, errored_ = false, exited_early_ = false;
  bool graceful_release_ = false, in_flight_ = false, rendezvous_done_ = false, terminating_ = false;
  bool stopped_ = false;
  int restarts_ = 0;
  Workload current_;
  std::optional<CompletedMessage> pending_;
  actor::Ref self_;
};

}  // namespace master
}  // namespace detcore
