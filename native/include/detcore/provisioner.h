// Elastic agent provisioning (reference master/internal/provisioner/
// {provisioner,scale_decider}.go + resourcemanagers/scaling.go).
//
// ScaleDecider is pure: from the pool's slot demand, the connected/idle agents and the provider's
// instance list it decides how many instances to launch (ceil(pending slots / slots per
// instance), bounded by max_instances) and which to terminate (idle longer than max_idle_period
// beyond min_instances, or started/disconnected longer than max_starting_period without an agent).
// Providers: `local` spawns det-agent processes on this host (artificial or GPU slots) — the
// MI355X-node equivalent of the reference's AWS/GCP instance providers, which need cloud APIs
// that are not reachable here.
#pragma once

#include <chrono>
#include <map>
#include <set>
#include <string>
#include <vector>

#include "detcore/json.h"

namespace detcore {
namespace prov {

using Clock = std::chrono::steady_clock;

struct Instance {
  std::string id;
  std::string state;  // Starting | Running | Stopped
  Clock::time_point launched;
};

struct AgentInfo {
  std::string id;
  bool idle = true;
};

struct ProvisionerConfig {
  int min_instances = 0;
  int max_instances = 0;  // 0: provisioning disabled
  int slots_per_instance = 1;
  std::chrono::milliseconds max_idle_period{300000};
  std::chrono::milliseconds max_starting_period{300000};
  std::string provider = "local";
  std::string agent_binary;        // local provider: det-agent path
  bool artificial = true;          // local provider: --artificial-slots vs GPU detection
  std::string master_host = "127.0.0.1";
  int master_port = 8080;
  std::string python = "python3";
  std::string work_dir = "/tmp/det-provisioned";
  std::string framework_root;      // cloud providers: PYTHONPATH of the provider coprocess
  std::string cluster_id;
  Json raw;                        // the provisioner config as given (cloud provider settings)
  static ProvisionerConfig FromJson(const Json& j);
};

struct Decision {
  int launch = 0;
  std::vector<std::string> terminate;
};

class ScaleDecider {
 public:
  explicit ScaleDecider(ProvisionerConfig cfg) : cfg_(std::move(cfg)) {}
  // pending_slots: slot demand of tasks that have no allocation yet.
  Decision Decide(int pending_slots, const std::vector<AgentInfo>& agents, const std::vector<Instance>& instances,
                  Clock::time_point now);

 private:
  ProvisionerConfig cfg_;
  std::map<std::string, Clock::time_point> idle_since_;
};

class Provider {
 public:
  virtual ~Provider() = default;
  virtual std::vector<Instance> List() = 0;
  virtual void Launch(int n) = 0;
  virtual void Terminate(const std::vector<std::string>& ids) = 0;
};

// det-agent child processes named "<pool>-prov-<n>"; the instance id is the agent id.
class LocalProvider : public Provider {
 public:
  LocalProvider(ProvisionerConfig cfg, std::string pool);
  ~LocalProvider() override;
  std::vector<Instance> List() override;
  void Launch(int n) override;
  void Terminate(const std::vector<std::string>& ids) override;

 private:
  ProvisionerConfig cfg_;
  std::string pool_;
  int next_ = 0;
  std::map<std::string, std::pair<int, Instance>> procs_;  // id -> (pid, instance)
};

// Cloud providers (aws, gcp): determined_1_amd/deploy/cloud_provider.py as a long-lived coprocess
// speaking JSON lines over pipes (the clouds' REST APIs + request signing live there; the master
// has no TLS stack).  Instance ids are the cloud's ids, which the started agents use as agent ids.
class CommandProvider : public Provider {
 public:
  CommandProvider(ProvisionerConfig cfg, std::string pool);
  ~CommandProvider() override;
  std::vector<Instance> List() override;
  void Launch(int n) override;
  void Terminate(const std::vector<std::string>& ids) override;

 private:
  bool Call(const Json& req, Json* resp);
  void Spawn();
  ProvisionerConfig cfg_;
  std::string pool_;
  pid_t pid_ = -1;
  int in_fd_ = -1, out_fd_ = -1;
  std::string rbuf_;
  std::map<std::string, Clock::time_point> launched_;
};

}  // namespace prov
}  // namespace detcore
