// Experiment-config defaults / merge / validation on the master side (SURVEY M26, C-config;
// reference master/pkg/model/{defaults,experiment_config,searcher_config,
// hyperparameters_config}.go) and the master's own config.
//
// Merge order: defaults -> master checkpoint_storage -> template -> user config
// (core_experiment.go:355-416).  Tagged unions (searcher.name, checkpoint_storage.type) replace
// the selected arm wholesale when the tag changes.  The Python side
// (determined_1_amd/config/experiment_config.py) implements the same schema for the CLI and local
// mode; tests pin the two to the same defaults.
#pragma once

#include <string>
#include <vector>

#include "detcore/json.h"

namespace detcore {

Json DefaultExperimentConfig(uint32_t experiment_seed);
Json DeepMerge(const Json& base, const Json& over);
Json MergeExperimentConfig(const Json& user, const Json& master_checkpoint_storage, const Json& tmpl,
                           uint32_t default_seed);
std::vector<std::string> ValidateExperimentConfig(const Json& cfg);

// Master config (reference master/internal/config.go:24-86): port, store dir, scheduler,
// fitting policy, resource pools, checkpoint storage, task defaults.
// "" when g is a valid agent user group {uid, gid, user, group}, else why not.
std::string ValidateAgentUserGroup(const Json& g);

struct MasterConfig {
  std::string listen_host = "0.0.0.0";
  int port = 8080;
  std::string store_dir;  // empty: in-memory
  std::string scheduler = "fair_share";
  std::string fitting_policy = "best";
  bool priority_preemption = true;
  std::vector<std::string> resource_pools{"default"};
  Json checkpoint_storage;  // default for experiments that do not set one
  std::string cluster_name = "determined-mi355x";
  double scheduler_tick_ms = 500;
  std::string python = "python3";
  bool require_auth = false;
  // telemetry.{enabled, file}: reference Segment events (master/internal/telemetry) written as JSON
  // lines to a local file -- there is no egress; disabled unless a file is configured.
  std::string telemetry_file;
  Json kubernetes;   // resource_manager {type: kubernetes, api_server, namespace, max_slots_per_pod, ...}; empty = agents
  Json provisioner;  // {max_instances, min_instances, slots_per_instance, ...}; empty = disabled  // security.authentication: tokens required on the REST API
  // security.tls.{cert,key} (reference master/internal/config.go:118,249-260): PEM files; when both
  // are set the REST/WebSocket API is served over TLS and tasks get DET_USE_TLS/DET_MASTER_CERT_FILE
  std::string tls_cert, tls_key;
  // task_container_defaults (reference master/pkg/model/task_container_defaults.go:19-70)
  int64_t shm_size_bytes = 4294967296;  // 4 GiB, the reference default
  std::string network_mode = "bridge";
  std::string dtrain_network_interface;  // "" = auto-detect
  std::string nccl_port_range, gloo_port_range;  // "MIN:MAX"
  // logging.{type: default | elastic, host, port, index} (reference master/internal/config/elastic.go):
  // with elastic, trial and task logs live in Elasticsearch instead of the local segments
  Json logging;
  // security.default_agent_user_group {uid, gid, user, group}: the host account tasks of users with no
  // linked agent user run as (reference model.AgentUserGroup); null = the agent's own account
  Json default_agent_user_group;
  static MasterConfig FromJson(const Json& j);
  Json ToJson() const;
  std::vector<std::string> Validate() const;
  // config keys DET_* environment variables may set beyond the defaults' leaves
  static std::vector<std::string> EnvPaths();
};

}  // namespace detcore
