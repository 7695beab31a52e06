// C ABI of libdetcore for Python (ctypes): JSON in, JSON out.  Every entry point catches C++
// exceptions and reports them as {"error": "..."} so a bad config never crashes the caller.
#include <cstdlib>
#include <cstring>
#include <memory>
#include <string>

#include "detcore/config.h"
#include "detcore/json.h"
#include "detcore/scheduler.h"
#include "detcore/searcher.h"

using detcore::Json;

namespace {

char* dup(const std::string& s) {
  char* p = static_cast<char*>(std::malloc(s.size() + 1));
  std::memcpy(p, s.data(), s.size() + 1);
  return p;
}

char* err(const std::exception& e) {
  Json j = Json::object();
  j["error"] = std::string(e.what());
  return dup(j.dump());
}

Json ops_json(const detcore::Ops& ops) {
  Json a = Json::array();
  for (const auto& op : ops) a.push_back(op.ToJson());
  return a;
}

struct SearcherHandle {
  std::unique_ptr<detcore::Searcher> s;
};

detcore::ValidationFn make_valfn(const Json& spec, uint64_t seed) {
  std::string kind = spec.get_string("kind", "constant");
  if (kind == "constant") {
    double v = spec.get_double("value", 1.0);
    return [v](int, int) { return v; };
  }
  if (kind == "random") {
    auto rng = std::make_shared<detcore::NpRand>(static_cast<uint32_t>(seed ^ 0x5bd1e995u));
    return [rng](int, int) { return rng->UnitInterval(); };
  }
  if (kind == "trial_id") {  // metric = trial_id (or -trial_id): deterministic ranking
    double sign = spec.get_double("sign", 1.0);
    return [sign](int tid, int) { return sign * static_cast<double>(tid); };
  }
  if (kind == "trial_id_parity") {  // odd trial ids +id, even -id (pbt_test.go "even_odd")
    return [](int tid, int) { return tid % 2 == 0 ? -static_cast<double>(tid) : static_cast<double>(tid); };
  }
  throw std::invalid_argument("unknown validation function kind " + kind);
}

}  // namespace

extern "C" {

void detcore_free(char* p) { std::free(p); }

int detcore_abi_version() { return 1; }

void* detcore_searcher_new(const char* searcher_cfg, const char* hparams, uint32_t seed, char** error) {
  try {
    Json cfg = Json::parse(searcher_cfg);
    Json hp = Json::parse(hparams && *hparams ? hparams : "{}");
    auto* h = new SearcherHandle;
    h->s = std::make_unique<detcore::Searcher>(seed, detcore::NewSearchMethod(cfg), hp);
    if (error) *error = nullptr;
    return h;
  } catch (const std::exception& e) {
    if (error) *error = dup(e.what());
    return nullptr;
  }
}

void detcore_searcher_free(void* h) { delete static_cast<SearcherHandle*>(h); }

char* detcore_searcher_call(void* handle, const char* method, const char* args) {
  try {
    auto& s = *static_cast<SearcherHandle*>(handle)->s;
    Json a = Json::parse(args && *args ? args : "{}");
    std::string m = method;
    Json out = Json::object();
    if (m == "initial_operations") {
      out["ops"] = ops_json(s.InitialOperations());
    } else if (m == "trial_created") {
      out["ops"] = ops_json(s.TrialCreated(detcore::Op::FromJson(a.at("create")), static_cast<int>(a.at("trial_id").as_int())));
    } else if (m == "operation_completed") {
      out["ops"] = ops_json(s.OperationCompleted(static_cast<int>(a.at("trial_id").as_int()),
                                                 detcore::Op::FromJson(a.at("op")), a["metrics"]));
    } else if (m == "trial_closed") {
      out["ops"] = ops_json(s.TrialClosed(detcore::ParseRequestID(a.at("request_id").as_string())));
    } else if (m == "trial_exited_early") {
      out["ops"] = ops_json(s.TrialExitedEarly(static_cast<int>(a.at("trial_id").as_int()),
                                               detcore::ParseExitedReason(a.get_string("reason", "ERRORED"))));
    } else if (m == "workload_completed") {
      s.WorkloadCompleted(a["msg"], a.get_double("units", 0));
    } else if (m == "progress") {
      out["progress"] = s.Progress();
    } else if (m == "uncommitted_events") {
      Json ev = Json::array();
      for (auto& e : s.UncommittedEvents()) ev.push_back(e);
      out["events"] = ev;
    } else if (m == "state") {
      out["trials_requested"] = s.trials_requested();
      out["trials_closed"] = s.trials_closed();
      out["shutdown"] = s.shutdown();
      out["total_units_completed"] = s.total_units_completed();
    } else {
      throw std::invalid_argument("unknown searcher method " + m);
    }
    return dup(out.dump());
  } catch (const std::exception& e) {
    return err(e);
  }
}

char* detcore_simulate(const char* searcher_cfg, const char* hparams, uint32_t seed, const char* valfn,
                       int random_order, uint64_t sim_seed) {
  try {
    Json cfg = Json::parse(searcher_cfg);
    Json hp = Json::parse(hparams && *hparams ? hparams : "{}");
    detcore::Searcher s(seed, detcore::NewSearchMethod(cfg), hp);
    auto fn = make_valfn(Json::parse(valfn && *valfn ? valfn : "{}"), sim_seed);
    auto res = detcore::Simulate(s, fn, random_order != 0, sim_seed, cfg.get_string("metric", "metric"));
    Json out = Json::object();
    out["results"] = res.Summary();
    out["seed"] = static_cast<int64_t>(sim_seed);
    Json trials = Json::array();
    for (const auto& rid : res.order) {
      Json t = Json::object();
      t["request_id"] = detcore::RequestIDString(rid);
      Json ops = Json::array();
      for (const auto& op : res.results.at(rid)) ops.push_back(op.ToJson());
      t["ops"] = ops;
      trials.push_back(t);
    }
    out["trials"] = trials;
    return dup(out.dump());
  } catch (const std::exception& e) {
    return err(e);
  }
}

// ------------------------------------------------------------------------------------------------
// Scheduler state from a JSON scenario in the shape of the reference's resource-manager test
// fixtures (resourcemanagers/scheduler_test.go mockAgent / mockGroup / mockTask):
//   agents: [{id, label, slots, slots_used, max_zero_slot_containers, zero_slot_containers}]
//   groups: [{id, weight (default 0), max_slots (default none), priority (default none)}]
//   tasks:  [{id, group (default: its own group), slots_needed, label, non_preemptible,
//             allocated_agent, container_started}]
// Groups register first (in order), then each task (and its own implicit group), as the fixtures
// create their actors.  An allocated task whose container has not started holds no devices.
namespace sched_api {
using namespace detcore::sched;

Agent MakeAgent(const Json& j) {
  Agent a;
  a.id = j.at("id").as_string();
  a.label = j.get_string("label", "");
  a.address = j.get_string("address", "/" + a.id);
  a.max_zero_slot_tasks = static_cast<int>(j.get_int("max_zero_slot_containers", 0));
  const int n = static_cast<int>(j.get_int("slots", 0)), used = static_cast<int>(j.get_int("slots_used", 0));
  for (int i = 0; i < n; ++i) a.slots.push_back(Slot{i, a.id + "-" + std::to_string(i), "gpu", true, i < used ? "used" : ""});
  a.zero_slot_tasks = static_cast<int>(j.get_int("zero_slot_containers", 0));
  return a;
}

Task MakeTask(const Json& j) {
  Task t;
  t.id = j.at("id").as_string();
  t.group = j.get_string("group", t.id);
  t.label = j.get_string("label", "");
  t.slots_needed = static_cast<int>(j.get_int("slots_needed", 0));
  t.non_preemptible = j.get_bool("non_preemptible", false);
  t.single_agent = j.get_bool("single_agent", false);
  return t;
}

void AddTasks(PoolState& st, const Json& tasks) {
  for (const auto& j : tasks.as_array()) {
    Task t = MakeTask(j);
    if (!st.groups.count(t.id)) st.EnsureGroup(t.id).weight = 0.0;  // every task actor is also a group
    if (!st.groups.count(t.group)) st.EnsureGroup(t.group).weight = 0.0;
    const std::string agent = j.get_string("allocated_agent", "");
    st.AddTask(t);
    if (agent.empty()) continue;
    Task& tt = st.tasks.at(t.id);
    Fit f{agent, {}};
    if (j.get_bool("container_started", false)) {
      Agent& ag = st.agents.at(agent);
      if (t.slots_needed == 0) ++ag.zero_slot_tasks;
      for (auto& sl : ag.slots)
        if (sl.task.empty() && static_cast<int>(f.devices.size()) < t.slots_needed) {
          sl.task = t.id;
          f.devices.push_back(sl.device_id);
        }
      if (static_cast<int>(f.devices.size()) != t.slots_needed) throw std::invalid_argument("over allocated to agent " + agent);
    }
    tt.allocation = {f};
  }
}

PoolState MakeState(const Json& a) {
  PoolState st;
  st.preemption = a.get_bool("preemption", false);
  if (a["agents"].is_array())
    for (const auto& j : a["agents"].as_array()) {
      Agent ag = MakeAgent(j);
      st.agents[ag.id] = ag;
    }
  if (a["groups"].is_array())
    for (const auto& j : a["groups"].as_array()) {
      Group& g = st.EnsureGroup(j.at("id").as_string());
      g.weight = j.get_double("weight", 0.0);
      g.max_slots = j["max_slots"].is_null() ? -1 : static_cast<int>(j["max_slots"].as_int());
      if (!j["priority"].is_null()) g.priority = static_cast<int>(j["priority"].as_int());
    }
  if (a["tasks"].is_array()) AddTasks(st, a["tasks"]);
  return st;
}

Json FitsJson(const std::vector<Fit>& fits) {
  Json out = Json::array();
  for (auto& f : fits) {
    Json e = Json::array();
    e.push_back(f.agent);
    e.push_back(static_cast<int64_t>(f.devices.size()));
    out.push_back(e);
  }
  return out;
}
}  // namespace sched_api

// Stateful scenario (multi-step tests): "schedule" {policy, fit}; "allocate" {tasks} (fit with
// BestFit on the live agents and commit, the fixtures' AllocateTasks); "add_tasks" {tasks};
// "remove" {task, delete} (free devices; delete=false leaves it pending, RemoveTask); "state".
void* detcore_sched_new(const char* args, char** error) {
  try {
    auto* st = new sched_api::PoolState(sched_api::MakeState(Json::parse(args && *args ? args : "{}")));
    if (error) *error = nullptr;
    return st;
  } catch (const std::exception& e) {
    if (error) *error = dup(e.what());
    return nullptr;
  }
}

void detcore_sched_free(void* h) { delete static_cast<sched_api::PoolState*>(h); }

char* detcore_sched_do(void* h, const char* op, const char* args) {
  try {
    using namespace sched_api;
    PoolState& st = *static_cast<PoolState*>(h);
    Json a = Json::parse(args && *args ? args : "{}");
    std::string o = op;
    Json out = Json::object();
    if (o == "schedule") {
      if (a.has("preemption")) st.preemption = a.get_bool("preemption", false);
      Decision d = Schedule(st, ParsePolicy(a.get_string("policy", "fair_share")), ParseFitMethod(a.get_string("fit", "best")));
      Json alloc = Json::array(), rel = Json::array();
      for (auto& x : d.allocate) alloc.push_back(x.first);
      for (auto& r : d.release) rel.push_back(r);
      out["allocate"] = alloc;
      out["release"] = rel;
    } else if (o == "allocate") {
      for (const auto& id : a.at("tasks").as_array()) {
        const Task& t = st.tasks.at(id.as_string());
        auto fits = FindFits(t, st.agents, FitMethod::BestFit);
        if (!fits) throw std::invalid_argument("no fit for " + t.id);
        st.Allocate(t.id, *fits);
      }
    } else if (o == "add_tasks") {
      AddTasks(st, a.at("tasks"));
    } else if (o == "remove") {
      const std::string id = a.at("task").as_string();
      if (a.get_bool("delete", true)) {
        st.RemoveTask(id);
      } else {
        Task& t = st.tasks.at(id);
        for (auto& f : t.allocation) {
          auto ag = st.agents.find(f.agent);
          if (ag == st.agents.end()) continue;
          if (t.slots_needed == 0 && !f.devices.empty()) continue;
          if (t.slots_needed == 0) ag->second.zero_slot_tasks = std::max(0, ag->second.zero_slot_tasks - 1);
          for (auto& sl : ag->second.slots)
            if (sl.task == id) sl.task.clear();
        }
        t.allocation.clear();
      }
    } else if (o == "state") {
      Json ag = Json::object();
      for (auto& kv : st.agents) ag[kv.first] = kv.second.NumEmptySlots();
      out["empty_slots"] = ag;
      out["num_tasks"] = static_cast<int64_t>(st.tasks.size());
    } else {
      throw std::invalid_argument("unknown scheduler op " + o);
    }
    return dup(out.dump());
  } catch (const std::exception& e) {
    return err(e);
  }
}

char* detcore_sched_call(const char* op, const char* args) {
  try {
    using namespace sched_api;
    Json a = Json::parse(args && *args ? args : "{}");
    std::string o = op;
    const FitMethod fm = ParseFitMethod(a.get_string("fit", "best"));
    if (o == "fit_score") {
      Task t;
      t.slots_needed = static_cast<int>(a.get_int("slots_needed", 0));
      Json out = FitScore(t, MakeAgent(a.at("agent")), fm);
      return dup(out.dump());
    }
    if (o == "find_fits") {
      PoolState st = MakeState(a);
      auto fits = FindFits(MakeTask(a.at("task")), st.agents, fm);
      return dup((fits ? FitsJson(*fits) : Json::array()).dump());
    }
    if (o == "schedule") {
      PoolState st = MakeState(a);
      Decision d = Schedule(st, ParsePolicy(a.get_string("policy", "fair_share")), fm);
      Json out = Json::object();
      Json alloc = Json::array(), fits = Json::object(), rel = Json::array();
      for (auto& x : d.allocate) {
        alloc.push_back(x.first);
        fits[x.first] = FitsJson(x.second);
      }
      for (auto& r : d.release) rel.push_back(r);
      out["allocate"] = alloc;
      out["release"] = rel;
      out["fits"] = fits;
      return dup(out.dump());
    }
    throw std::invalid_argument("unknown scheduler op " + o);
  } catch (const std::exception& e) {
    return err(e);
  }
}

// Searcher helpers pinned by the reference's unit tests: bracket sizing and PBT explore.
char* detcore_searcher_util(const char* name, const char* args) {
  try {
    Json a = Json::parse(args && *args ? args : "{}");
    std::string n = name;
    auto ints = [](const Json& arr) {
      std::vector<int64_t> v;
      for (const auto& x : arr.as_array()) v.push_back(x.as_int());
      return v;
    };
    Json out = Json::array();
    if (n == "bracket_max_trials") {
      for (auto v : detcore::BracketMaxTrials(a.at("max_trials").as_int(), a.at("divisor").as_double(), ints(a.at("brackets"))))
        out.push_back(v);
    } else if (n == "bracket_max_concurrent_trials") {
      for (auto v : detcore::BracketMaxConcurrentTrials(a.at("max_concurrent_trials").as_int(), a.at("divisor").as_double(),
                                                        ints(a.at("bracket_max_trials"))))
        out.push_back(v);
    } else if (n == "adaptive_mode") {
      for (auto v : detcore::AdaptiveModeBrackets(a.at("mode").as_string(), a.at("max_rungs").as_int())) out.push_back(v);
    } else if (n == "hyperparameter_grid") {
      for (auto& v : detcore::HyperparameterGrid(a.at("hyperparameters"))) out.push_back(v);
    } else if (n == "grid_values") {
      for (auto& v : detcore::GridValues(a.at("hyperparameter"))) out.push_back(v);
    } else if (n == "sample_all") {  // {"sample": ..., "next_bits64": RNG state probe after sampling}
      detcore::NpRand r(static_cast<uint32_t>(a.get_int("seed", 0)));
      Json o = Json::object();
      o["sample"] = detcore::SampleAll(a.at("hyperparameters"), r);
      o["next_bits64"] = std::to_string(r.Bits64());
      return dup(o.dump());
    } else if (n == "pbt_explore") {
      detcore::NpRand r(static_cast<uint32_t>(a.get_int("seed", 0)));
      Json hp = a["hyperparameters"];
      detcore::Context ctx{r, hp};
      return dup(detcore::PbtExplore(a.at("config"), ctx, a.at("sample")).dump());
    } else {
      throw std::invalid_argument("unknown searcher util " + n);
    }
    return dup(out.dump());
  } catch (const std::exception& e) {
    return err(e);
  }
}

char* detcore_nprand(uint32_t seed, const char* op, int64_t arg, int64_t n) {
  try {
    detcore::NpRand r(seed);
    std::string o = op;
    Json out = Json::array();
    for (int64_t i = 0; i < n; ++i) {
      if (o == "bits32") out.push_back(static_cast<int64_t>(r.Bits32()));
      else if (o == "unit_interval") out.push_back(r.UnitInterval());
      else if (o == "intn") out.push_back(r.Intn(arg));
      else if (o == "request_id") out.push_back(detcore::RequestIDString(detcore::NewRequestID(r)));
      else throw std::invalid_argument("unknown nprand op " + o);
    }
    return dup(out.dump());
  } catch (const std::exception& e) {
    return err(e);
  }
}

// Master-side experiment-config merge + validation, exposed so tests can pin the Python schema
// (determined_1_amd/config) to the one the master applies.
char* detcore_merge_config(const char* user, const char* master_storage, const char* tmpl, uint32_t seed) {
  try {
    Json u = Json::parse(user && *user ? user : "{}");
    Json ms = master_storage && *master_storage ? Json::parse(master_storage) : Json();
    Json t = tmpl && *tmpl ? Json::parse(tmpl) : Json();
    Json out = Json::object();
    Json merged = detcore::MergeExperimentConfig(u, ms, t, seed);
    Json errs = Json::array();
    for (auto& e : detcore::ValidateExperimentConfig(merged)) errs.push_back(e);
    out["config"] = merged;
    out["errors"] = errs;
    return dup(out.dump());
  } catch (const std::exception& e) {
    return err(e);
  }
}

char* detcore_json_roundtrip(const char* text) {
  try {
    return dup(Json::parse(text).dump());
  } catch (const std::exception& e) {
    return err(e);
  }
}

}  // extern "C"
