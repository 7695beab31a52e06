// Experiment/master config (see include/detcore/config.h).
#include "detcore/config.h"

#include <cctype>
#include <stdexcept>

#include <algorithm>
#include <set>

#include "detcore/searcher.h"

namespace detcore {

Json DefaultExperimentConfig(uint32_t seed) {
  Json c = Json::parse(R"({
    "description": "Experiment",
    "checkpoint_storage": {"type": "shared_fs", "host_path": "/tmp", "save_experiment_best": 0,
                           "save_trial_best": 1, "save_trial_latest": 1},
    "checkpoint_policy": "best",
    "data_layer": {"type": "shared_fs"},
    "hyperparameters": {},
    "searcher": {"smaller_is_better": true},
    "resources": {"slots_per_trial": 1, "weight": 1, "native_parallel": false, "agent_label": "",
                  "resource_pool": ""},
    "optimizations": {"aggregation_frequency": 1, "average_aggregated_gradients": true,
                      "average_training_metrics": false, "gradient_compression": false,
                      "mixed_precision": "O0", "tensor_fusion_threshold": 64,
                      "tensor_fusion_cycle_time": 5, "auto_tune_tensor_fusion": false,
                      "grad_reduction": "fp32_accum", "rccl": {}, "hip_graph": false,
                      "hip_graph_batches": 1},
    "perform_initial_validation": false,
    "min_checkpoint_period": {"batches": 0},
    "min_validation_period": {"batches": 0},
    "records_per_epoch": 0,
    "scheduling_unit": 100,
    "environment": {"image": {"cpu": "determined-mi355x:cpu", "gpu": "determined-mi355x:rocm"}},
    "reproducibility": {},
    "max_restarts": 5,
    "debug": false,
    "internal": null,
    "entrypoint": ""
  })");
  c["reproducibility"]["experiment_seed"] = static_cast<int64_t>(seed);
  return c;
}

static Json SearcherArmDefaults(const std::string& name) {
  if (name == "sync_halving") return Json::parse(R"({"divisor": 4, "train_stragglers": true})");
  if (name == "adaptive") return Json::parse(R"({"divisor": 4, "train_stragglers": true, "mode": "standard", "max_rungs": 5})");
  if (name == "adaptive_simple") return Json::parse(R"({"divisor": 4, "mode": "standard", "max_rungs": 5})");
  if (name == "async_halving") return Json::parse(R"({"divisor": 4, "max_concurrent_trials": 0})");
  if (name == "adaptive_asha")
    return Json::parse(R"({"divisor": 4, "mode": "standard", "max_rungs": 5, "max_concurrent_trials": 0})");
  return Json::object();
}

Json DeepMerge(const Json& base, const Json& over) {
  if (!base.is_object() || !over.is_object()) return over.clone();
  Json out = base.clone();
  for (auto& kv : over.as_object()) {
    const std::string& k = kv.first;
    const Json& v = kv.second;
    static const std::set<std::string> kAtomic = {"hyperparameters", "data", "min_validation_period",
                                                  "min_checkpoint_period", "max_length", "budget",
                                                  "length_per_round"};
    if (v.is_object() && out[k].is_object() && !kAtomic.count(k)) {
      const char* tag = nullptr;
      if (v.has("type") || out[k].has("type")) tag = "type";
      else if (v.has("name")) tag = "name";
      if (tag && v.has(tag) && out[k].has(tag) && !out[k][tag].is_null() && out[k][tag] != v[tag]) {
        Json arm = Json::object();
        for (auto& bk : out[k].as_object())
          if (bk.first.rfind("save_", 0) == 0 || bk.first == "smaller_is_better") arm[bk.first] = bk.second;
        for (auto& ok : v.as_object()) arm[ok.first] = ok.second.clone();
        out[k] = arm;
      } else {
        out[k] = DeepMerge(out[k], v);
      }
    } else {
      out[k] = v.clone();
    }
  }
  return out;
}

Json MergeExperimentConfig(const Json& user, const Json& master_ckpt, const Json& tmpl, uint32_t seed) {
  Json cfg = DefaultExperimentConfig(seed);
  if (master_ckpt.is_object() && !master_ckpt.as_object().empty()) {
    Json o = Json::object();
    o["checkpoint_storage"] = master_ckpt;
    cfg = DeepMerge(cfg, o);
  }
  if (tmpl.is_object()) cfg = DeepMerge(cfg, tmpl);
  cfg = DeepMerge(cfg, user);
  Json& s = cfg["searcher"];
  if (s.has("name")) {
    Json arm = SearcherArmDefaults(s["name"].as_string());
    for (auto& kv : arm.as_object())
      if (!s.has(kv.first)) s[kv.first] = kv.second;
  }
  if (!s.has("smaller_is_better")) s["smaller_is_better"] = true;
  return cfg;
}

static constexpr int kMaxAllowedTrials = 2000;

static bool ParseLen(const Json& v, Length* out) {
  try {
    *out = Length::FromJson(v);
    return true;
  } catch (const std::exception&) {
    return false;
  }
}

std::vector<std::string> ValidateExperimentConfig(const Json& cfg) {
  static const std::set<std::string> kTop = {
      "description", "labels", "data", "checkpoint_storage", "tensorboard_storage", "perform_initial_validation",
      "min_checkpoint_period", "min_validation_period", "checkpoint_policy", "hyperparameters", "searcher",
      "resources", "optimizations", "records_per_epoch", "scheduling_unit", "bind_mounts", "environment",
      "reproducibility", "max_restarts", "security", "debug", "internal", "entrypoint", "data_layer",
      "batches_per_step", "internal_warm_start"};
  static const std::set<std::string> kSearchers = {"single", "random", "grid", "sync_halving", "adaptive",
                                                   "adaptive_simple", "async_halving", "adaptive_asha", "pbt"};
  std::vector<std::string> errs;
  for (auto& kv : cfg.as_object())
    if (!kTop.count(kv.first)) errs.push_back("unknown config key: " + kv.first);
  bool native = cfg["internal"].is_object() && !cfg["internal"]["native"].is_null();
  if (!native && cfg.get_string("entrypoint", "").empty())
    errs.push_back("Must specify an entrypoint that references the trial class.");
  const Json& s = cfg["searcher"];
  std::string name = s.get_string("name", "");
  if (!kSearchers.count(name)) errs.push_back("searcher.name: unknown searcher '" + name + "'");
  if (s.get_string("metric", "").empty()) errs.push_back("searcher.metric must be set");
  bool epochs = false;
  for (const char* f : {"max_length", "budget", "length_per_round"}) {
    if (!s.has(f)) continue;
    Length l;
    if (!ParseLen(s[f], &l)) errs.push_back(std::string("searcher.") + f + ": invalid length");
    else {
      if (l.units <= 0) errs.push_back(std::string(f) + " must be > 0");
      epochs |= l.unit == Unit::Epochs;
    }
  }
  if ((name == "random" || name == "async_halving" || name == "adaptive_simple" || name == "adaptive_asha") &&
      s.get_int("max_trials", 0) <= 0)
    errs.push_back("max_trials must be > 0");
  if ((name == "sync_halving" || name == "async_halving" || name == "adaptive" || name == "adaptive_simple" ||
       name == "adaptive_asha") &&
      !(s.get_double("divisor", 0) > 1.0))
    errs.push_back("divisor must be > 1.0");
  if ((name == "sync_halving" || name == "async_halving") && s.get_int("num_rungs", 0) <= 0)
    errs.push_back("num_rungs must be > 0");
  if (name == "adaptive" || name == "adaptive_simple" || name == "adaptive_asha") {
    std::string mode = s.get_string("mode", "");
    if (mode != "aggressive" && mode != "standard" && mode != "conservative")
      errs.push_back("mode must be one of aggressive, standard, conservative");
    if (s.get_int("max_rungs", 0) <= 0) errs.push_back("max_rungs must be > 0");
  }
  if ((name == "async_halving" || name == "adaptive_asha") && s.get_int("max_concurrent_trials", 0) < 0)
    errs.push_back("max_concurrent_trials must be >= 0");
  if ((name == "adaptive" || name == "sync_halving") && s.has("budget") && s.has("max_length")) {
    Length b, m;
    if (ParseLen(s["budget"], &b) && ParseLen(s["max_length"], &m)) {
      if (b.unit != m.unit)
        errs.push_back("max_length and budget must be specified in terms of the same unit");
      else if (name == "adaptive" && !(b.units > m.units))
        errs.push_back("budget must be greater than max_length");
    }
  }
  if (name == "adaptive_simple" && s.get_int("max_trials", 0) > kMaxAllowedTrials)
    errs.push_back("max_trials must be <= " + std::to_string(kMaxAllowedTrials));
  if (name == "pbt") {
    if (s.get_int("population_size", 0) <= 0) errs.push_back("population_size must be > 0");
    if (s.get_int("num_rounds", 0) <= 0) errs.push_back("num_rounds must be > 0");
    double tf = s["replace_function"].get_double("truncate_fraction", 0.0);
    if (!(tf >= 0.0 && tf <= 0.5)) errs.push_back("truncate_fraction must be in [0, 0.5]");
    double rp = s["explore_function"].get_double("resample_probability", 0.0);
    if (!(rp >= 0.0 && rp <= 1.0)) errs.push_back("resample_probability must be in [0, 1]");
    double pf = s["explore_function"].get_double("perturb_factor", 0.0);
    if (!(pf >= 0.0 && pf <= 1.0)) errs.push_back("perturb_factor must be in [0, 1]");
  }
  for (const char* f : {"min_validation_period", "min_checkpoint_period"}) {
    if (!cfg.has(f)) continue;
    Length l;
    if (!ParseLen(cfg[f], &l)) errs.push_back(std::string(f) + ": invalid length");
    else epochs |= l.unit == Unit::Epochs;
  }
  if (epochs && cfg.get_int("records_per_epoch", 0) <= 0)
    errs.push_back("Must specify records_per_epoch when any configuration is in terms of epochs");
  const Json& hps = cfg["hyperparameters"];
  // global_batch_size (reference hyperparameters_config.go:20-44)
  if (!hps.is_object() || !hps.has("global_batch_size")) {
    errs.push_back("global_batch_size hyperparameter must be specified");
  } else {
    const Json& b = hps["global_batch_size"];
    std::vector<const Json*> vals;
    if (b.is_object() && b.get_string("type", "") == "categorical" && b["vals"].is_array()) {
      for (size_t i = 0; i < b["vals"].size(); ++i) vals.push_back(&b["vals"][i]);
    } else if (b.is_object() && b.get_string("type", "") == "const") {
      vals.push_back(&b["val"]);
    } else if (!b.is_object()) {
      vals.push_back(&b);
    }
    for (auto* v : vals)
      if (!v->is_number()) {
        errs.push_back("global_batch_size hyperparameter must be a numeric value");
        break;
      }
  }
  double n_grid = 1;
  std::vector<std::string> missing;
  if (hps.is_object()) {
    for (auto& kv : hps.as_object()) {
      const Json& hp = kv.second;
      if (!hp.is_object() || !hp.has("type")) continue;
      std::string t = hp["type"].as_string();
      if (t == "const") {
        if (!hp.has("val")) errs.push_back("hyperparameters." + kv.first + ": const needs val");
      } else if (t == "int" || t == "double" || t == "log") {
        double lo = hp.get_double("minval", 0), hi = hp.get_double("maxval", 0);
        if (!(hi > lo)) errs.push_back("hyperparameters." + kv.first + ": minval is greater than maxval");
        if (t == "log" && !(hp.get_double("base", 0) > 0))
          errs.push_back("hyperparameters." + kv.first + ": base must be >= 0");
        bool has_count = hp.has("count") && !hp["count"].is_null();
        if (has_count && hp.get_int("count", 0) <= 0)
          errs.push_back("hyperparameters." + kv.first + ": count must be >= 0");
        if (name == "grid") {
          if (!has_count) {
            missing.push_back(kv.first);
          } else {
            double c = static_cast<double>(hp.get_int("count", 0));
            // int counts clamp to the size of the range (reference grid.go)
            n_grid *= (t == "int" && c > hi - lo) ? hi - lo : c;
          }
        }
      } else if (t == "categorical") {
        if (!hp["vals"].is_array() || hp["vals"].size() == 0)
          errs.push_back("hyperparameters." + kv.first + ": must have at least one category");
        n_grid *= std::max<size_t>(1, hp["vals"].is_array() ? hp["vals"].size() : 0);
      } else {
        errs.push_back("hyperparameters." + kv.first + ": unknown type '" + t + "'");
      }
    }
  }
  if (name == "grid" && !missing.empty()) {
    std::string m = "these hyperparameters must specify counts for grid search: ";
    for (size_t i = 0; i < missing.size(); ++i) m += (i ? ", " : "") + missing[i];
    errs.push_back(m);
  }
  if (name == "grid" && n_grid > kMaxAllowedTrials)
    errs.push_back("number of trials for grid search must be <= " + std::to_string(kMaxAllowedTrials));
  if (cfg.get_int("max_restarts", 0) < 0) errs.push_back("max_restarts must be >= 0");
  for (const char* k : {"save_experiment_best", "save_trial_best", "save_trial_latest"})
    if (cfg["checkpoint_storage"].get_int(k, 0) < 0) errs.push_back(std::string(k) + " must be >= 0");
  std::string ct = cfg["checkpoint_storage"].get_string("type", "shared_fs");
  if (ct != "shared_fs" && ct != "s3" && ct != "gcs" && ct != "hdfs")
    errs.push_back("checkpoint_storage.type: unknown '" + ct + "'");
  std::string cp = cfg.get_string("checkpoint_policy", "best");
  if (cp != "best" && cp != "all" && cp != "none") errs.push_back("checkpoint_policy must be one of best, all, none");
  if (cfg["resources"].get_int("slots_per_trial", 1) < 0) errs.push_back("slots_per_trial must be >= 0");
  if (cfg["optimizations"].get_int("aggregation_frequency", 1) < 1) errs.push_back("aggregation_frequency must be >= 1");
  if (cfg["optimizations"].get_int("hip_graph_batches", 1) < 1)
    errs.push_back("optimizations.hip_graph_batches must be >= 1");
  if (cfg.get_int("scheduling_unit", 100) <= 0) errs.push_back("scheduling_unit must be > 0");
  return errs;
}

MasterConfig MasterConfig::FromJson(const Json& j) {
  MasterConfig c;
  c.listen_host = j.get_string("listen_host", c.listen_host);
  c.port = static_cast<int>(j.get_int("port", c.port));
  c.store_dir = j.get_string("store_dir", c.store_dir);
  if (j["scheduler"].is_object()) {
    c.scheduler = j["scheduler"].get_string("type", c.scheduler);
    c.fitting_policy = j["scheduler"].get_string("fitting_policy", c.fitting_policy);
    c.priority_preemption = j["scheduler"].get_bool("preemption", c.priority_preemption);
  }
  if (j["resource_pools"].is_array()) {
    c.resource_pools.clear();
    for (auto& p : j["resource_pools"].as_array()) c.resource_pools.push_back(p.is_string() ? p.as_string() : p.get_string("pool_name", "default"));
  }
  c.checkpoint_storage = j["checkpoint_storage"];
  c.cluster_name = j.get_string("cluster_name", c.cluster_name);
  c.scheduler_tick_ms = j.get_double("scheduler_tick_ms", c.scheduler_tick_ms);
  c.python = j.get_string("python", c.python);
  c.provisioner = j["provisioner"];
  if (j["resource_manager"].is_object() && j["resource_manager"].get_string("type", "agent") == "kubernetes")
    c.kubernetes = j["resource_manager"];
  if (j["security"].is_object()) c.require_auth = j["security"].get_bool("authentication", c.require_auth);
  if (j["telemetry"].is_object() && j["telemetry"].get_bool("enabled", true))
    c.telemetry_file = j["telemetry"].get_string("file", "");
  if (j["security"]["tls"].is_object()) {
    c.tls_cert = j["security"]["tls"].get_string("cert", "");
    c.tls_key = j["security"]["tls"].get_string("key", "");
  }
  if (j["logging"].is_object()) c.logging = j["logging"];
  if (j["security"]["default_agent_user_group"].is_object())
    c.default_agent_user_group = j["security"]["default_agent_user_group"];
  const Json& tcd = j["task_container_defaults"];
  if (tcd.is_object()) {
    c.shm_size_bytes = tcd.get_int("shm_size_bytes", c.shm_size_bytes);
    c.network_mode = tcd.get_string("network_mode", c.network_mode);
    c.dtrain_network_interface = tcd.get_string("dtrain_network_interface", "");
    c.nccl_port_range = tcd.get_string("nccl_port_range", "");
    c.gloo_port_range = tcd.get_string("gloo_port_range", "");
  }
  auto errs = c.Validate();
  if (!errs.empty()) {
    std::string m = "invalid master config:";
    for (auto& e : errs) m += " " + e + ";";
    throw std::invalid_argument(m);
  }
  return c;
}

static bool ValidPortRange(const std::string& r) {
  if (r.empty()) return true;
  auto colon = r.find(':');
  if (colon == std::string::npos || colon == 0 || colon + 1 == r.size()) return false;
  for (size_t i = 0; i < r.size(); ++i)
    if (i != colon && !std::isdigit(static_cast<unsigned char>(r[i]))) return false;
  const long lo = std::stol(r.substr(0, colon)), hi = std::stol(r.substr(colon + 1));
  return lo <= hi && hi <= 65535;
}

// reference master/internal/user/service.go:28-45 (agentUserGroup.Validate) and
// master/pkg/model/agent_user_group.go:27-47: all four fields set, ids non-negative
std::string ValidateAgentUserGroup(const Json& g) {
  if (!g.is_object()) return "must be an object {uid, gid, user, group}";
  if (!g["uid"].is_number()) return "uid must be set";
  if (!g["gid"].is_number()) return "gid must be set";
  if (g.get_string("user", "").empty()) return "user must be set";
  if (g.get_string("group", "").empty()) return "group must be set";
  if (g.get_int("uid", -1) < 0) return "uid less than zero";
  if (g.get_int("gid", -1) < 0) return "gid less than zero";
  return "";
}

std::vector<std::string> MasterConfig::Validate() const {
  // reference TaskContainerDefaultsConfig.Validate + TLS pairing
  std::vector<std::string> e;
  if (shm_size_bytes < 0) e.push_back("task_container_defaults.shm_size_bytes must be >= 0");
  if (network_mode.empty()) e.push_back("task_container_defaults.network_mode must be set");
  if (!ValidPortRange(nccl_port_range)) e.push_back("task_container_defaults.nccl_port_range must be \"MIN:MAX\"");
  if (!ValidPortRange(gloo_port_range)) e.push_back("task_container_defaults.gloo_port_range must be \"MIN:MAX\"");
  if (tls_cert.empty() != tls_key.empty()) e.push_back("security.tls needs both cert and key");
  if (port <= 0 || port > 65535) e.push_back("port must be in 1..65535");
  if (default_agent_user_group.is_object()) {
    const std::string why = ValidateAgentUserGroup(default_agent_user_group);
    if (!why.empty()) e.push_back("security.default_agent_user_group: " + why);
  }
  if (logging.is_object()) {
    const std::string t = logging.get_string("type", "default");
    if (t != "default" && t != "elastic") e.push_back("logging.type must be default or elastic");
    if (t == "elastic" && logging.get_string("host", "").empty()) e.push_back("logging.host is required for elastic");
    if (t == "elastic" && (logging.get_int("port", 9200) <= 0 || logging.get_int("port", 9200) > 65535))
      e.push_back("logging.port must be in 1..65535");
  }
  return e;
}

std::vector<std::string> MasterConfig::EnvPaths() {
  return {"security.tls.cert", "security.tls.key", "security.authentication", "task_container_defaults.shm_size_bytes",
          "task_container_defaults.network_mode", "task_container_defaults.dtrain_network_interface",
          "task_container_defaults.nccl_port_range", "task_container_defaults.gloo_port_range",
          "checkpoint_storage.type", "checkpoint_storage.host_path", "checkpoint_storage.storage_path",
          "checkpoint_storage.bucket", "checkpoint_storage.save_experiment_best",
          "checkpoint_storage.save_trial_best", "checkpoint_storage.save_trial_latest", "telemetry.file",
          "telemetry.enabled", "logging.type", "logging.host", "logging.port", "scheduler.type", "scheduler.fitting_policy", "resource_pools"};
}

Json MasterConfig::ToJson() const {
  Json j = Json::object();
  j["listen_host"] = listen_host;
  j["port"] = port;
  j["store_dir"] = store_dir;
  Json s = Json::object();
  s["type"] = scheduler;
  s["fitting_policy"] = fitting_policy;
  s["preemption"] = priority_preemption;
  j["scheduler"] = s;
  Json pools = Json::array();
  for (auto& p : resource_pools) pools.push_back(p);
  j["resource_pools"] = pools;
  j["checkpoint_storage"] = checkpoint_storage;
  j["cluster_name"] = cluster_name;
  j["scheduler_tick_ms"] = scheduler_tick_ms;
  j["python"] = python;
  Json sec = Json::object();
  sec["authentication"] = require_auth;
  j["security"] = sec;
  j["provisioner"] = provisioner;
  if (kubernetes.is_object()) j["resource_manager"] = kubernetes;
  Json tel = Json::object();
  tel["enabled"] = !telemetry_file.empty();
  tel["file"] = telemetry_file;
  j["telemetry"] = tel;
  Json tls = Json::object();
  tls["cert"] = tls_cert;
  tls["key"] = tls_key;
  j["security"]["tls"] = tls;
  j["security"]["default_agent_user_group"] = default_agent_user_group;
  Json tcd = Json::object();
  tcd["shm_size_bytes"] = static_cast<long long>(shm_size_bytes);
  tcd["network_mode"] = network_mode;
  tcd["dtrain_network_interface"] = dtrain_network_interface;
  tcd["nccl_port_range"] = nccl_port_range;
  tcd["gloo_port_range"] = gloo_port_range;
  j["task_container_defaults"] = tcd;
  if (logging.is_object()) {
    j["logging"] = logging;
  } else {
    j["logging"]["type"] = "default";
  }
  return j;
}

}  // namespace detcore
