// det-master: the control plane (reference master/internal/*.go).
//
//   REST + WebSocket API (HttpServer)
//     └─ actor system
//          ├─ /pools/<name>            resource pool: agents, gang scheduling tick (fair_share /
//          │                           priority / round_robin + fitting), preemption requests
//          └─ /experiments/<id>        experiment: Searcher, checkpoint policy, state machine
//                └─ /<request-id>      trial: sequencer, allocation, containers, rendezvous,
//                                      workload relay, restarts / rollback, preemption
//   Agents connect over /agents (WebSocket) and run trial processes; trial processes connect
//   over /ws/trial/<e>/<t>/<c>.  All durable state lives in the embedded Store (WAL+snapshot),
//   including the experiment event log replayed on master restart.
#pragma once

#include <chrono>

#include <atomic>
#include <condition_variable>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <set>
#include <string>
#include <vector>

#include "detcore/actor.h"
#include "detcore/config.h"
#include "detcore/json.h"
#include "detcore/kubernetes.h"
#include "detcore/net.h"
#include "detcore/rw_coordinator.h"
#include "detcore/store.h"

namespace detcore {
namespace master {

class Master;

struct AgentConn {
  std::string id;
  std::string pool;
  std::string label;
  std::string host;  // address the agent connected from (trial processes run there)
  net::WsPtr ws;
  std::function<bool(const Json&)> send;  // virtual agents (Kubernetes RM): master -> agent messages
  Json devices;
  std::set<std::string> containers;
};

class Master {
 public:
  explicit Master(MasterConfig cfg);
  ~Master();
  int Start();  // bind + serve; returns the port
  void Stop();
  void Wait();  // until Stop() (signal handler)

  // ---- used by actors / handlers
  Store& store() { return *store_; }
  LogStore& logs() { return *logs_; }
  actor::System& system() { return *sys_; }
  const MasterConfig& config() const { return cfg_; }
  // task_container_defaults (+ TLS trust material) into a task's env / shipped files
  void AddTaskDefaults(Json& env, Json& files) const;
  // The host account {uid, gid, user, group} a task of `username` runs as: the user's linked agent
  // user group, else security.default_agent_user_group, else null (the agent's own account).
  Json AgentUserGroupFor(const std::string& username);
  Json AgentUserGroupForExperiment(int64_t experiment_id);
  bool tls() const { return !tls_cert_pem_.empty(); }
  actor::Ref Pool(const std::string& name);
  bool SendToAgent(const std::string& agent_id, const Json& msg);
  std::string AgentHost(const std::string& agent_id);
  void BindContainer(const std::string& cid, const std::string& agent_id, actor::Ref trial);
  void UnbindContainer(const std::string& cid);
  actor::Ref TrialForContainer(const std::string& cid);
  actor::Ref ExperimentRef(int64_t id);
  std::string master_host() const { return advertised_host_; }
  int port() const { return port_; }
  void AppendTrialLog(int64_t trial_id, const std::string& line, const std::string& stdtype,
                      const std::string& container_id, int rank);
  void RunCheckpointGC(int64_t experiment_id, const Json& exp_config, const Json& to_delete);
  std::string cluster_id() const { return cluster_id_; }
  bool shutting_down() const { return shutting_down_.load(); }
  // Append one telemetry event (reference telemetry/reports.go) when telemetry is configured.
  void ReportTelemetry(const std::string& event, Json properties);

 private:
  void InstallRoutes();
  void InstallApiV1();  // api_v1.cc: the reference's /api/v1 grpc-gateway surface
  void HandleAgentSocket(const net::Request& req, net::WsPtr ws);
 public:
  // agent protocol, shared by WebSocket agents and virtual agents (kubernetes.cc)
  bool RegisterAgent(const std::shared_ptr<AgentConn>& conn, std::string* err);
  void OnAgentMessage(const std::shared_ptr<AgentConn>& conn, const Json& m);
  void AgentGone(const std::shared_ptr<AgentConn>& conn);
  std::string advertised_host() const { return advertised_host_; }

 private:
  void HandleTrialSocket(const net::Request& req, net::WsPtr ws);
  void HandleRWLockSocket(const net::Request& req, net::WsPtr ws);
  void RestoreExperiments();
  void EnsureDefaultUsers();
  std::string UserForRequest(const net::Request& r);
  int64_t CreateExperiment(const Json& body, bool* activate);

  MasterConfig cfg_;
  std::unique_ptr<Store> store_;
  std::mutex state_lat_mu_;  // agent ContainerStateChanged send -> handled (/debug/stats)
  double state_lat_max_ms_ = 0, state_lat_sum_ms_ = 0;
  int64_t state_lat_n_ = 0;
  std::unique_ptr<LogStore> logs_;  // trial-<id> / task-<id> log segments
  std::unique_ptr<actor::System> sys_;
  RWCoordinator rw_coordinator_;  // before http_: socket threads use it until the server stops
  net::HttpServer http_;
  std::map<std::string, actor::Ref> pools_;
  std::mutex mu_;
  std::map<std::string, std::shared_ptr<AgentConn>> agents_;
  std::map<std::string, std::pair<std::string, actor::Ref>> containers_;  // cid -> (agent, trial)
  std::string advertised_host_ = "127.0.0.1";
  std::string cluster_id_;
  int port_ = 0;
  std::mutex stop_mu_;
  std::condition_variable stop_cv_;
  bool stopped_ = false;
  std::atomic<bool> shutting_down_{false};
  std::mutex telemetry_mu_;
  std::unique_ptr<KubernetesRM> kube_;
  std::string tls_cert_pem_;  // security.tls.cert contents, shipped to tasks
  std::chrono::steady_clock::time_point started_ = std::chrono::steady_clock::now();
};

// Helpers shared by the master translation units.
void MasterLog(const std::string& line);  // stderr + the in-memory ring buffer behind GET /logs
Json MasterLogTail(int64_t offset, int64_t limit);
std::string NowRFC3339();
std::string NewUUID();
Json CheckpointsToGC(Store& store, int64_t experiment_id, const Json& exp_config);

}  // namespace master
}  // namespace detcore
