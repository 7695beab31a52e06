// det-master process: HTTP/WebSocket API, agent + trial sockets, experiment lifecycle,
// checkpoint GC, restore-on-restart (see include/detcore/master.h).
//
// REST surface (reference master/internal/core.go:518-573 + api_*.go, JSON only):
//   GET    /info                                   cluster id, version
//   POST   /experiments                            {config, model_definition, activate, template}
//   GET    /experiments                            summaries
//   GET    /experiments/:id                        config + trials + state
//   PATCH  /experiments/:id                        {state | archived | description}
//   POST   /experiments/:id/kill                   cancel + kill containers
//   DELETE /experiments/:id                        delete rows + checkpoint GC of everything
//   GET    /experiments/:id/model_def              model definition files
//   GET    /experiments/:id/checkpoints            checkpoints (sorted by the searcher metric)
//   GET    /experiments/:id/metrics                per-trial training/validation metric series
//   GET    /trials/:id                             trial + steps/validations/checkpoints
//   GET    /trials/:id/logs?offset=&limit=         trial logs
//   POST   /trials/:id/kill
//   GET    /checkpoints/:uuid
//   GET    /agents                                 agents + slots (all pools)
//   POST   /agents/:id/slots/:slot/(enable|disable) and /agents/:id/(enable|disable)
//   GET    /resource_pools
//   POST   /searcher/preview                       offline simulation of a searcher config
//   GET|PUT|DELETE /templates[/:name]
//   GET|POST /models[/:name[/versions]]            model registry
//   POST   /trial_logs                             log shipping (agents / harness)
//   WS     /agents?id=&resource_pool=&label=      agent channel
//   WS     /ws/trial/:e/:t/:c                      harness channel (C-ws / C-done)
//   WS     /ws/data-layer/*?read_lock=true|false   readers-writer lock per resource path (M24)
#include "detcore/master.h"

#include <dirent.h>

#include <signal.h>
#include <spawn.h>
#include <sys/socket.h>
#include <sys/stat.h>
#include <sys/wait.h>
#include <unistd.h>

#include <algorithm>
#include <cctype>
#include <cerrno>
#include <chrono>
#include <cstdio>
#include <ctime>
#include <fstream>
#include <deque>
#include <mutex>
#include <random>
#include <sstream>
#include <thread>

#include "detcore/config.h"
#include "detcore/lttb.h"
#include "detcore/master_actors.h"
#include "detcore/searcher.h"

extern char** environ;

namespace detcore {
namespace master {

using actor::Ref;

static const char* kVersion = "0.13.10.dev0+mi355x";

// Master log ring buffer (reference pkg/logger/log_buffer.go: last 25k entries, GET /logs).
namespace {
std::mutex g_log_mu;
std::deque<Json> g_log;
int64_t g_log_seq = 0;
constexpr size_t kLogCap = 25000;
}  // namespace

void MasterLog(const std::string& line) {
  std::fprintf(stderr, "[det-master] %s\n", line.c_str());
  std::lock_guard<std::mutex> g(g_log_mu);
  Json e = Json::object();
  e["id"] = ++g_log_seq;
  e["time"] = NowRFC3339();
  e["message"] = line;
  g_log.push_back(e);
  if (g_log.size() > kLogCap) g_log.pop_front();
}

Json MasterLogTail(int64_t offset, int64_t limit) {
  std::lock_guard<std::mutex> g(g_log_mu);
  Json out = Json::array();
  for (auto& e : g_log) {
    if (e["id"].as_int() <= offset) continue;
    if (static_cast<int64_t>(out.size()) >= limit) break;
    out.push_back(e);
  }
  return out;
}

static void Log(const std::string& s) { MasterLog(s); }

std::string NowRFC3339() {
  auto now = std::chrono::system_clock::now();
  std::time_t t = std::chrono::system_clock::to_time_t(now);
  auto us = std::chrono::duration_cast<std::chrono::microseconds>(now.time_since_epoch()).count() % 1000000;
  std::tm tm{};
  gmtime_r(&t, &tm);
  char buf[64];
  std::strftime(buf, sizeof(buf), "%Y-%m-%dT%H:%M:%S", &tm);
  char out[80];
  std::snprintf(out, sizeof(out), "%s.%06lldZ", buf, static_cast<long long>(us));
  return out;
}

std::string NewUUID() {
  static thread_local std::mt19937_64 rng{std::random_device{}() ^ static_cast<uint64_t>(
                                                std::chrono::steady_clock::now().time_since_epoch().count())};
  uint64_t a = rng(), b = rng();
  a = (a & 0xFFFFFFFFFFFF0FFFull) | 0x0000000000004000ull;
  b = (b & 0x3FFFFFFFFFFFFFFFull) | 0x8000000000000000ull;
  char buf[40];
  std::snprintf(buf, sizeof(buf), "%08x-%04x-%04x-%04x-%012llx", static_cast<unsigned>(a >> 32),
                static_cast<unsigned>((a >> 16) & 0xFFFF), static_cast<unsigned>(a & 0xFFFF),
                static_cast<unsigned>(b >> 48), static_cast<unsigned long long>(b & 0xFFFFFFFFFFFFull));
  return buf;
}

// Checkpoints the retention policy does not keep (reference db/postgres.go:1046-1157): keep the
// experiment's top `save_experiment_best`, each trial's top `save_trial_best` (by the searcher
// metric of the validation at the same step) and each trial's latest `save_trial_latest`.
Json CheckpointsToGC(Store& store, int64_t experiment_id, const Json& cfg) {
  const Json& cs = cfg["checkpoint_storage"];
  int64_t keep_exp = cs.get_int("save_experiment_best", 0), keep_best = cs.get_int("save_trial_best", 1),
          keep_latest = cs.get_int("save_trial_latest", 1);
  const std::string metric = cfg["searcher"].get_string("metric", "");
  const bool smaller = cfg["searcher"].get_bool("smaller_is_better", true);
  struct C {
    Json row;
    bool has_metric = false;
    double metric = 0;
  };
  std::map<int64_t, std::vector<C>> by_trial;
  std::map<int64_t, std::map<int64_t, double>> metric_at;  // trial -> step -> searcher metric
  for (auto& r : store.Where("checkpoints", "experiment_id", Json(experiment_id))) {
    if (r.get_string("state", "") != "COMPLETED") continue;
    const int64_t tid = r["trial_id"].as_int();
    if (!metric_at.count(tid)) {  // one index lookup of the trial's validations
      auto& m = metric_at[tid];
      for (auto& v : store.Where("validations", "trial_id", Json(tid))) {
        if (v.get_string("state", "") != "COMPLETED") continue;
        try {
          m[v.get_int("step_id", -1)] = ValidationMetric(v["metrics"]["validation_metrics"], metric);
        } catch (const std::exception&) {
        }
      }
    }
    C c{r};
    auto& m = metric_at[tid];
    auto it = m.find(r["step_id"].as_int());
    if (it != m.end()) {
      c.metric = it->second;
      c.has_metric = true;
    }
    by_trial[tid].push_back(c);
  }
  auto better = [&](const C& a, const C& b) {
    if (a.has_metric != b.has_metric) return a.has_metric;
    return smaller ? a.metric < b.metric : a.metric > b.metric;
  };
  std::set<std::string> keep;
  std::vector<C> all;
  for (auto& kv : by_trial) {
    auto v = kv.second;
    std::sort(v.begin(), v.end(), [](const C& a, const C& b) { return a.row.get_int("step_id", 0) > b.row.get_int("step_id", 0); });
    for (int64_t i = 0; i < keep_latest && i < static_cast<int64_t>(v.size()); ++i) keep.insert(v[i].row["uuid"].as_string());
    std::stable_sort(v.begin(), v.end(), better);
    for (int64_t i = 0; i < keep_best && i < static_cast<int64_t>(v.size()); ++i)
      if (v[i].has_metric) keep.insert(v[i].row["uuid"].as_string());
    for (auto& c : v) all.push_back(c);
  }
  std::stable_sort(all.begin(), all.end(), better);
  for (int64_t i = 0; i < keep_exp && i < static_cast<int64_t>(all.size()); ++i)
    if (all[i].has_metric) keep.insert(all[i].row["uuid"].as_string());
  // model-registry versions pin their checkpoints
  for (auto& mv : store.Scan("model_versions")) keep.insert(mv.get_string("checkpoint_uuid", ""));
  Json out = Json::array();
  for (auto& c : all)
    if (!keep.count(c.row["uuid"].as_string())) out.push_back(c.row);
  return out;
}

// ---------------------------------------------------------------------------------- Master
Master::Master(MasterConfig cfg) : cfg_(std::move(cfg)) {
  store_ = std::make_unique<Store>(cfg_.store_dir);
  logs_ = std::make_unique<LogStore>(cfg_.store_dir.empty() ? std::string() : cfg_.store_dir + "/logs");
  if (cfg_.logging.is_object() && cfg_.logging.get_string("type", "default") == "elastic")
    logs_->SetBackend(MakeElasticLogBackend(cfg_.logging.get_string("host", ""),
                                            static_cast<int>(cfg_.logging.get_int("port", 9200)),
                                            cfg_.logging.get_string("index", "determined-logs")));
  sys_ = std::make_unique<actor::System>(8);
  Json cid;
  if (store_->Get("cluster_id", 1, &cid)) {
    cluster_id_ = cid["cluster_id"].as_string();
  } else {
    cluster_id_ = NewUUID();
    Json row = Json::object();
    row["cluster_id"] = cluster_id_;
    store_->Put("cluster_id", 1, row);
  }
  if (cfg_.resource_pools.empty()) cfg_.resource_pools.push_back("default");
}

Master::~Master() { Stop(); }

Ref Master::Pool(const std::string& name) {
  std::lock_guard<std::mutex> g(mu_);
  auto it = pools_.find(name);
  if (it != pools_.end()) return it->second;
  return pools_.begin()->second;
}

bool Master::SendToAgent(const std::string& agent_id, const Json& msg) {
  std::shared_ptr<AgentConn> a;
  {
    std::lock_guard<std::mutex> g(mu_);
    auto it = agents_.find(agent_id);
    if (it == agents_.end()) return false;
    a = it->second;
  }
  if (a->send) return a->send(msg);
  return a->ws && a->ws->Send(msg.dump());
}

std::string Master::AgentHost(const std::string& agent_id) {
  std::lock_guard<std::mutex> g(mu_);
  auto it = agents_.find(agent_id);
  return it == agents_.end() ? "127.0.0.1" : it->second->host;
}

void Master::BindContainer(const std::string& cid, const std::string& agent_id, Ref trial) {
  std::lock_guard<std::mutex> g(mu_);
  containers_[cid] = {agent_id, std::move(trial)};
  auto it = agents_.find(agent_id);
  if (it != agents_.end()) it->second->containers.insert(cid);
}

void Master::UnbindContainer(const std::string& cid) {
  std::lock_guard<std::mutex> g(mu_);
  auto it = containers_.find(cid);
  if (it == containers_.end()) return;
  auto a = agents_.find(it->second.first);
  if (a != agents_.end()) a->second->containers.erase(cid);
  containers_.erase(it);
}

Ref Master::TrialForContainer(const std::string& cid) {
  std::lock_guard<std::mutex> g(mu_);
  auto it = containers_.find(cid);
  return it == containers_.end() ? nullptr : it->second.second;
}

Ref Master::ExperimentRef(int64_t id) { return sys_->Get("/experiments/" + std::to_string(id)); }

void Master::AppendTrialLog(int64_t trial_id, const std::string& line, const std::string& stdtype,
                            const std::string& container_id, int rank) {
  Json row = Json::object();
  row["trial_id"] = trial_id;
  row["message"] = line;
  row["stdtype"] = stdtype;
  row["container_id"] = container_id;
  row["rank_id"] = rank;
  row["timestamp"] = NowRFC3339();
  logs_->Append("trial-" + std::to_string(trial_id), {row});
}

void Master::RunCheckpointGC(int64_t experiment_id, const Json& exp_config, const Json& to_delete) {
  // The reference starts a GC container (checkpoint_gc.go); here the GC job is the harness's
  // `determined_1_amd.exec.gc_checkpoints` entrypoint run as a child process of the master,
  // which has the same view of shared_fs / object storage as the trial processes.
  std::string dir = (cfg_.store_dir.empty() ? std::string("/tmp") : cfg_.store_dir) + "/gc";
  ::mkdir(dir.c_str(), 0755);
  std::string path = dir + "/gc-" + std::to_string(experiment_id) + "-" + NewUUID() + ".json";
  Json spec = Json::object();
  spec["experiment_config"] = exp_config;
  spec["checkpoints"] = to_delete;
  {
    std::ofstream f(path);
    f << spec.dump();
  }
  for (auto& c : to_delete.as_array()) {
    Json patch = Json::object();
    patch["state"] = "DELETED";
    store_->Update("checkpoints", c["id"].as_int(), patch);
  }
  std::string py = cfg_.python;
  std::vector<std::string> args = {py, "-m", "determined_1_amd.exec.gc_checkpoints", path};
  std::vector<char*> argv;
  for (auto& a : args) argv.push_back(const_cast<char*>(a.c_str()));
  argv.push_back(nullptr);
  pid_t pid;
  if (posix_spawnp(&pid, py.c_str(), nullptr, nullptr, argv.data(), environ) == 0) {
    std::thread([pid] {
      int st;
      waitpid(pid, &st, 0);
    }).detach();
    Log("checkpoint GC for experiment " + std::to_string(experiment_id) + ": " + std::to_string(to_delete.size()) +
        " checkpoints");
  } else {
    Log("failed to start checkpoint GC");
  }
}

int64_t Master::CreateExperiment(const Json& body, bool* activate) {
  Json user = body["config"];
  if (user.is_string()) user = Json::parse(user.as_string());
  if (!user.is_object()) throw std::invalid_argument("config must be a JSON object");
  Json tmpl;
  if (body.has("template") && body["template"].is_string()) {
    for (auto& t : store_->Where("templates", "name", body["template"]))
      tmpl = t["config"];
    if (tmpl.is_null()) throw std::invalid_argument("template not found: " + body["template"].as_string());
  }
  uint32_t seed = static_cast<uint32_t>(std::chrono::system_clock::now().time_since_epoch().count() & 0xFFFFFFFF);
  Json cfg = MergeExperimentConfig(user, cfg_.checkpoint_storage, tmpl, seed);
  auto errs = ValidateExperimentConfig(cfg);
  if (!errs.empty()) {
    std::string m = "invalid experiment config:";
    for (auto& e : errs) m += "\n  " + e;
    throw std::invalid_argument(m);
  }
  // validates the searcher config by building it
  NewSearchMethod(cfg["searcher"]);
  // warm start (reference experiment.go:112, experiment_utils.go:16-45): every trial of the new
  // experiment starts from the given checkpoint (or the source trial's latest checkpoint)
  const Json& sc = cfg["searcher"];
  if (sc.has("source_checkpoint_uuid") || sc.has("source_trial_id")) {
    Json ck;
    if (sc.has("source_checkpoint_uuid")) {
      for (auto& c : store_->Where("checkpoints", "uuid", sc["source_checkpoint_uuid"])) ck = c;
    } else {
      int64_t best_step = -1;
      for (auto& c : store_->Where("checkpoints", "trial_id", sc["source_trial_id"]))
        if (c.get_string("state", "") == "COMPLETED" && c.get_int("step_id", 0) > best_step) {
          best_step = c.get_int("step_id", 0);
          ck = c;
        }
    }
    if (ck.is_null() || !ck["checkpoint"].is_object()) throw std::invalid_argument("warm-start checkpoint not found");
    cfg["internal_warm_start"] = ck["checkpoint"];
  }
  if (body.get_bool("validate_only", false)) return 0;
  *activate = body.get_bool("activate", true);
  Json row = Json::object();
  row["config"] = cfg;
  row["state"] = *activate ? "ACTIVE" : "PAUSED";
  row["start_time"] = NowRFC3339();
  row["archived"] = false;
  row["progress"] = 0.0;
  row["owner"] = body.get_string("owner", "determined");
  row["parent_id"] = body["parent_id"];
  row["description"] = cfg.get_string("description", "");
  int64_t id = store_->Insert("experiments", row);
  Json md = Json::object();
  md["experiment_id"] = id;
  md["files"] = body["model_definition"].is_array() ? body["model_definition"] : Json::array();
  store_->Put("model_definitions", id, md);
  Json props = Json::object();
  props["id"] = id;
  props["searcher"] = cfg["searcher"];
  props["resources"] = cfg["resources"];
  props["num_hparams"] = static_cast<int64_t>(cfg["hyperparameters"].is_object() ? cfg["hyperparameters"].as_object().size() : 0);
  props["batches_per_step"] = cfg["scheduling_unit"];
  ReportTelemetry("experiment_created", props);
  return id;
}

static net::Response J(int status, const Json& j) { return net::Response::Json(status, j.dump()); }
static net::Response Err(int status, const std::string& m) {
  Json j = Json::object();
  j["error"] = m;
  return J(status, j);
}
static int64_t IntParam(const net::Request& r, const std::string& k) { return std::stoll(r.Param(k)); }

// ------------------------------------------------------------------------- users & sessions
// (reference master/internal/user/service.go): salted SHA-1 password hashes,
// bearer-token sessions, the built-in "admin" and "determined" users with empty passwords.
static std::string Hex(const std::string& raw) {
  static const char* d = "0123456789abcdef";
  std::string o;
  for (unsigned char c : raw) {
    o.push_back(d[c >> 4]);
    o.push_back(d[c & 15]);
  }
  return o;
}

static std::string HashPassword(const std::string& salt, const std::string& pw) { return Hex(net::Sha1(salt + ":" + pw)); }

void Master::EnsureDefaultUsers() {
  for (const char* name : {"admin", "determined"}) {
    if (!store_->Where("users", "username", Json(name)).empty()) continue;
    Json u = Json::object();
    u["username"] = name;
    u["salt"] = NewUUID();
    u["password_hash"] = HashPassword(u["salt"].as_string(), "");
    u["admin"] = std::string(name) == "admin";
    u["active"] = true;
    store_->Insert("users", u);
  }
}

std::string Master::UserForRequest(const net::Request& r) {
  auto it = r.headers.find("authorization");
  if (it == r.headers.end()) return "";
  std::string v = it->second;
  if (v.rfind("Bearer ", 0) == 0) v = v.substr(7);
  for (auto& s : store_->Where("sessions", "token", Json(v))) return s.get_string("username", "");
  return "";
}

void Master::InstallRoutes() {
  EnsureDefaultUsers();
  if (cfg_.require_auth) {
    http_.SetAuth([this](const net::Request& r) {
      if (r.path == "/login" || r.path == "/info" || r.path == "/trial_logs") return true;
      if (r.path == "/" || r.path == "/det" || r.path.rfind("/det/", 0) == 0) return true;  // WebUI shell
      if (r.path == "/api/v1/auth/login" || r.path == "/api/v1/master") return true;
      if (r.path.rfind("/experiments/", 0) == 0 && r.path.size() > 10 &&
          r.path.find("/model_def") != std::string::npos)
        return true;  // agents fetch model definitions
      if (r.path.rfind("/commands/", 0) == 0 && r.path.find("/context") != std::string::npos) return true;
      return !UserForRequest(r).empty();
    });
  }
  http_.Route("POST", "/login", [this](const net::Request& r) {
    Json body = Json::parse(r.body);
    std::string name = body.get_string("username", "");
    for (auto& u : store_->Where("users", "username", Json(name))) {
      if (!u.get_bool("active", true) ||
          HashPassword(u.get_string("salt", ""), body.get_string("password", "")) != u.get_string("password_hash", ""))
        break;
      Json sess = Json::object();
      sess["username"] = name;
      sess["token"] = Hex(net::Sha1(NewUUID() + NewUUID()));
      sess["created"] = NowRFC3339();
      store_->Insert("sessions", sess);
      Json out = Json::object();
      out["token"] = sess["token"];
      out["username"] = name;
      return J(200, out);
    }
    return Err(401, "invalid credentials");
  });
  http_.Route("POST", "/logout", [this](const net::Request& r) {
    auto it = r.headers.find("authorization");
    if (it != r.headers.end()) {
      std::string tok = it->second.rfind("Bearer ", 0) == 0 ? it->second.substr(7) : it->second;
      store_->DeleteWhere("sessions", [&](const Json& s) { return s.get_string("token", "") == tok; });
    }
    return J(200, Json::object());
  });
  http_.Route("GET", "/me", [this](const net::Request& r) {
    std::string u = UserForRequest(r);
    if (u.empty()) return Err(401, "not logged in");
    Json out = Json::object();
    out["username"] = u;
    return J(200, out);
  });
  http_.Route("GET", "/users", [this](const net::Request&) {
    Json out = Json::array();
    for (auto& u : store_->Scan("users")) {
      Json v = Json::object();
      for (const char* k : {"id", "username", "admin", "active"}) v[k] = u[k];
      if (u["agent_user_group"].is_object()) v["agent_user_group"] = u["agent_user_group"];
      out.push_back(v);
    }
    return J(200, out);
  });
  http_.Route("POST", "/users", [this](const net::Request& r) {
    Json body = Json::parse(r.body);
    std::string name = body.get_string("username", "");
    if (name.empty()) return Err(400, "username required");
    if (cfg_.require_auth) {  // with authentication on, only an admin creates users (reference user/service.go postUser)
      bool caller_admin = false;
      for (auto& cu : store_->Where("users", "username", Json(UserForRequest(r)))) caller_admin = cu.get_bool("admin", false);
      if (!caller_admin) return Err(403, "only an admin can create users");
    }
    if (!store_->Where("users", "username", Json(name)).empty()) return Err(409, "user exists");
    Json u = Json::object();
    u["username"] = name;
    u["salt"] = NewUUID();
    u["password_hash"] = HashPassword(u["salt"].as_string(), body.get_string("password", ""));
    u["admin"] = body.get_bool("admin", false);
    u["active"] = true;
    store_->Insert("users", u);
    return J(201, Json::object());
  });
  http_.Route("PATCH", "/users/:name", [this](const net::Request& r) {
    Json body = Json::parse(r.body);
    // with authentication on, only an admin changes another user, admin/active flags or the agent
    // user group (reference user/service.go:248-280, AdminCanBeModifiedBy)
    bool caller_admin = true;
    std::string caller;
    if (cfg_.require_auth) {
      caller = UserForRequest(r);
      caller_admin = false;
      for (auto& cu : store_->Where("users", "username", Json(caller))) caller_admin = cu.get_bool("admin", false);
    }
    const bool privileged = body.has("active") || body.has("admin") || body.has("agent_user_group");
    if (!caller_admin && (privileged || caller != r.Param("name"))) return Err(403, "only an admin can do that");
    for (auto& u : store_->Where("users", "username", Json(r.Param("name")))) {
      Json patch = Json::object();
      if (body.has("password")) patch["password_hash"] = HashPassword(u.get_string("salt", ""), body["password"].as_string());
      if (body.has("active")) patch["active"] = body["active"];
      if (body.has("admin")) patch["admin"] = body["admin"];
      if (body.has("agent_user_group")) {
        const std::string why = ValidateAgentUserGroup(body["agent_user_group"]);
        if (!why.empty()) return Err(400, why);
        Json g = Json::object();
        g["uid"] = body["agent_user_group"].get_int("uid", 0);
        g["gid"] = body["agent_user_group"].get_int("gid", 0);
        g["user"] = body["agent_user_group"].get_string("user", "");
        g["group"] = body["agent_user_group"].get_string("group", "");
        patch["agent_user_group"] = g;
      }
      store_->Update("users", u["id"].as_int(), patch);
      return J(200, Json::object());
    }
    return Err(404, "user not found");
  });

  // ---------------------------------------------------------------- introspection (/debug)
  // The reference exposes Go's pprof (master/internal/core.go:564-568) and actor message tracing
  // (master/pkg/actor/trace.go:17-60).  Here: per-actor mailbox depth / high-water mark, message
  // counts by type, Receive latency (total, max, log2-microsecond histogram) and mailbox wait, the
  // ring of the last processed messages, and process-level stats from /proc.
  http_.Route("GET", "/debug/actors", [this](const net::Request& r) {
    const std::string prefix = r.Query("prefix", "");
    auto stats = sys_->Stats();
    std::sort(stats.begin(), stats.end(), [](const actor::CellStats& a, const actor::CellStats& b) {
      return a.busy_ms > b.busy_ms;
    });
    Json out = Json::array();
    for (auto& st : stats) {
      if (!prefix.empty() && st.address.rfind(prefix, 0) != 0) continue;
      Json a = Json::object();
      a["address"] = st.address;
      a["mailbox"] = static_cast<long long>(st.mailbox);
      a["max_mailbox"] = static_cast<long long>(st.max_mailbox);
      a["processed"] = static_cast<long long>(st.processed);
      a["busy_ms"] = st.busy_ms;
      a["max_ms"] = st.max_ms;
      a["mean_ms"] = st.processed ? st.busy_ms / static_cast<double>(st.processed) : 0.0;
      a["mean_wait_ms"] = st.processed ? st.wait_ms / static_cast<double>(st.processed) : 0.0;
      a["max_wait_ms"] = st.max_wait_ms;
      Json h = Json::object();
      for (int b = 0; b < 16; ++b)
        if (st.hist[b]) h[b == 0 ? std::string("<1us") : "<" + std::to_string(1LL << b) + "us"] = static_cast<long long>(st.hist[b]);
      a["latency_histogram"] = h;
      Json bt = Json::object();
      for (auto& kv : st.by_type) bt[kv.first] = static_cast<long long>(kv.second);
      a["messages"] = bt;
      out.push_back(a);
    }
    return J(200, out);
  });
  http_.Route("GET", "/debug/trace", [this](const net::Request& r) {
    const std::string prefix = r.Query("prefix", "");
    Json out = Json::array();
    for (auto& t : sys_->Trace()) {
      if (!prefix.empty() && t.address.rfind(prefix, 0) != 0) continue;
      Json e = Json::object();
      e["address"] = t.address;
      e["type"] = t.type;
      e["wait_ms"] = t.wait_ms;
      e["run_ms"] = t.run_ms;
      e["at_ms"] = static_cast<long long>(t.at_ms);
      out.push_back(e);
    }
    return J(200, out);
  });
  http_.Route("GET", "/debug/stats", [this](const net::Request&) {
    Json out = Json::object();
    std::ifstream st("/proc/self/status");
    std::string line;
    while (std::getline(st, line)) {
      for (const char* k : {"Threads", "VmRSS", "VmHWM", "VmSize", "voluntary_ctxt_switches", "nonvoluntary_ctxt_switches"}) {
        const std::string key = std::string(k) + ":";
        if (line.rfind(key, 0) == 0) {
          std::string v = line.substr(key.size());
          v.erase(0, v.find_first_not_of(" \t"));
          out[k] = v;
        }
      }
    }
    long fds = 0;
    if (DIR* d = opendir("/proc/self/fd")) {
      while (readdir(d)) ++fds;
      closedir(d);
    }
    out["open_fds"] = static_cast<long long>(fds > 2 ? fds - 2 : fds);
    out["uptime_s"] = std::chrono::duration<double>(std::chrono::steady_clock::now() - started_).count();
    out["actors"] = static_cast<long long>(sys_->Stats().size());
    out["tls"] = tls();
    out["log_shipping"] = logs_->Stats();
    {
      std::lock_guard<std::mutex> g(state_lat_mu_);
      Json lat = Json::object();
      lat["count"] = static_cast<long long>(state_lat_n_);
      lat["max"] = state_lat_max_ms_;
      lat["mean"] = state_lat_n_ ? state_lat_sum_ms_ / static_cast<double>(state_lat_n_) : 0.0;
      out["agent_state_latency_ms"] = lat;
    }
    return J(200, out);
  });
  http_.Route("GET", "/info", [this](const net::Request&) {
    Json j = Json::object();
    j["cluster_id"] = cluster_id_;
    j["cluster_name"] = cfg_.cluster_name;
    j["version"] = kVersion;
    j["master_id"] = cluster_id_;
    return J(200, j);
  });
  http_.Route("GET", "/master/config", [this](const net::Request&) { return J(200, cfg_.ToJson()); });
  http_.Route("GET", "/logs", [](const net::Request& r) {
    return J(200, MasterLogTail(std::stoll(r.Query("offset", "0")), std::stoll(r.Query("limit", "25000"))));
  });

  // ---------------------------------------------------------------------- experiments
  http_.Route("POST", "/experiments", [this](const net::Request& r) {
    Json body = Json::parse(r.body);
    bool activate = true;
    std::string user = UserForRequest(r);
    if (!user.empty()) body["owner"] = user;
    int64_t id = CreateExperiment(body, &activate);
    Json out = Json::object();
    if (id == 0) {
      out["valid"] = true;
      return J(200, out);
    }
    Json row;
    store_->Get("experiments", id, &row);
    sys_->ActorOf("experiments/" + std::to_string(id),
                  std::make_unique<ExperimentActor>(this, id, row["config"], false));
    Log("experiment " + std::to_string(id) + " created (" + row["config"]["searcher"].get_string("name", "") + ")");
    out["id"] = id;
    out["config"] = row["config"];
    net::Response resp = J(201, out);
    resp.headers["Location"] = "/experiments/" + std::to_string(id);
    return resp;
  });
  http_.Route("GET", "/experiments", [this](const net::Request& r) {
    bool all = r.Query("all", "false") == "true";
    Json out = Json::array();
    for (auto& e : store_->Scan("experiments")) {
      if (!all && e.get_bool("archived", false)) continue;
      Json s = Json::object();
      for (const char* k : {"id", "state", "start_time", "end_time", "archived", "progress", "owner", "description"})
        s[k] = e[k];
      s["searcher"] = e["config"]["searcher"].get_string("name", "");
      s["num_trials"] = static_cast<int64_t>(store_->Where("trials", "experiment_id", e["id"]).size());
      s["labels"] = e["config"]["labels"];
      out.push_back(s);
    }
    return J(200, out);
  });
  http_.Route("GET", "/experiments/:id", [this](const net::Request& r) {
    int64_t id = IntParam(r, "id");
    Json e;
    if (!store_->Get("experiments", id, &e)) return Err(404, "experiment not found");
    Json trials = Json::array();
    for (auto& t : store_->Where("trials", "experiment_id", Json(id))) {
      Json tj = t;
      int64_t tid = t["id"].as_int();
      int64_t batches = 0;
      for (auto& s : store_->Where("steps", "trial_id", Json(tid)))
        if (s.get_string("state", "") == "COMPLETED") batches = std::max(batches, s.get_int("prior_batches_processed", 0) + s.get_int("num_batches", 0));
      tj["total_batches_processed"] = batches;
      Json best;
      const std::string metric = e["config"]["searcher"].get_string("metric", "");
      const bool smaller = e["config"]["searcher"].get_bool("smaller_is_better", true);
      for (auto& v : store_->Where("validations", "trial_id", Json(tid))) {
        if (v.get_string("state", "") != "COMPLETED") continue;
        try {
          double m = ValidationMetric(v["metrics"]["validation_metrics"], metric);
          if (best.is_null() || (smaller ? m < best.as_double() : m > best.as_double())) best = m;
        } catch (const std::exception&) {
        }
      }
      tj["best_validation_metric"] = best;
      trials.push_back(tj);
    }
    e["trials"] = trials;
    return J(200, e);
  });
  http_.Route("PATCH", "/experiments/:id", [this](const net::Request& r) {
    int64_t id = IntParam(r, "id");
    Json e;
    if (!store_->Get("experiments", id, &e)) return Err(404, "experiment not found");
    Json body = Json::parse(r.body);
    Json patch = Json::object();
    if (body.has("archived")) patch["archived"] = body["archived"];
    if (body.has("description")) patch["description"] = body["description"];
    if (body.has("labels")) patch["labels"] = body["labels"];
    // reference `det experiment set {weight,priority,max-slots,gc-policy}`: config changes that take
    // effect now -- the pool's group weights/limits and an immediate checkpoint GC pass
    Json cfg_patch = Json::object();
    if (body["resources"].is_object()) {
      for (const char* k : {"weight", "priority", "max_slots"})
        if (body["resources"].has(k)) cfg_patch["resources"][k] = body["resources"][k];
    }
    if (body["checkpoint_storage"].is_object()) {
      for (const char* k : {"save_experiment_best", "save_trial_best", "save_trial_latest"})
        if (body["checkpoint_storage"].has(k)) cfg_patch["checkpoint_storage"][k] = body["checkpoint_storage"][k];
    }
    if (cfg_patch.size() > 0) {
      Json cfg = DeepMerge(e["config"], cfg_patch);
      patch["config"] = cfg;
      if (Ref ex = ExperimentRef(id)) ex->AskSync(PatchExperimentConfig{cfg_patch});
      if (cfg_patch.has("resources")) {
        std::string pool = cfg["resources"].get_string("resource_pool", "");
        Pool(pool.empty() ? cfg_.resource_pools[0] : pool)
            ->Tell(SetGroup{std::to_string(id), cfg["resources"].get_double("weight", 1.0),
                            cfg["resources"].has("priority") && !cfg["resources"]["priority"].is_null()
                                ? std::optional<int>(static_cast<int>(cfg["resources"]["priority"].as_int()))
                                : std::nullopt,
                            static_cast<int>(cfg["resources"].get_int("max_slots", -1))});
      }
    }
    if (patch.size() > 0) store_->Update("experiments", id, patch);
    if (cfg_patch.has("checkpoint_storage")) {
      Json gc = CheckpointsToGC(*store_, id, patch["config"]);
      if (gc.size() > 0) RunCheckpointGC(id, patch["config"], gc);
    }
    if (body.has("state")) {
      Ref ex = ExperimentRef(id);
      if (!ex) return Err(409, "experiment is not running (state " + e.get_string("state", "") + ")");
      actor::Message m = ex->AskSync(SetExperimentState{body["state"].as_string(), false});
      std::string err = m.has_value() ? std::any_cast<std::string>(m) : "no response";
      if (!err.empty()) return Err(409, err);
    }
    store_->Get("experiments", id, &e);
    return J(200, e);
  });
  http_.Route("POST", "/experiments/:id/kill", [this](const net::Request& r) {
    int64_t id = IntParam(r, "id");
    Ref ex = ExperimentRef(id);
    if (!ex) return Err(409, "experiment is not running");
    ex->AskSync(SetExperimentState{"STOPPING_CANCELED", true});
    return J(200, Json::object());
  });
  http_.Route("DELETE", "/experiments/:id", [this](const net::Request& r) {
    int64_t id = IntParam(r, "id");
    Json e;
    if (!store_->Get("experiments", id, &e)) return Err(404, "experiment not found");
    if (ExperimentRef(id)) return Err(409, "experiment is still running; kill it first");
    Json all = Json::array();
    for (auto& c : store_->Scan("checkpoints", [&](const Json& c) {
           return c.get_int("experiment_id", -1) == id && c.get_string("state", "") == "COMPLETED";
         }))
      all.push_back(c);
    if (all.size() > 0) RunCheckpointGC(id, e["config"], all);
    std::vector<int64_t> trial_ids;
    for (auto& t : store_->Where("trials", "experiment_id", Json(id))) trial_ids.push_back(t["id"].as_int());
    for (int64_t tid : trial_ids) {
      store_->DeleteWhereEq("steps", "trial_id", Json(tid));
      store_->DeleteWhereEq("validations", "trial_id", Json(tid));
      store_->DeleteWhereEq("checkpoints", "trial_id", Json(tid));
      logs_->Delete("trial-" + std::to_string(tid));
      store_->Delete("trials", tid);
    }
    store_->Delete("model_definitions", id);
    store_->Delete("experiments", id);
    return J(200, Json::object());
  });
  http_.Route("GET", "/experiments/:id/model_def", [this](const net::Request& r) {
    Json md;
    if (!store_->Get("model_definitions", IntParam(r, "id"), &md)) return Err(404, "not found");
    return J(200, md);
  });
  http_.Route("GET", "/experiments/:id/checkpoints", [this](const net::Request& r) {
    int64_t id = IntParam(r, "id");
    Json e;
    if (!store_->Get("experiments", id, &e)) return Err(404, "experiment not found");
    const std::string metric = e["config"]["searcher"].get_string("metric", "");
    const bool smaller = e["config"]["searcher"].get_bool("smaller_is_better", true);
    std::vector<Json> out;
    for (auto& c : store_->Scan("checkpoints", [&](const Json& c) {
           return c.get_int("experiment_id", -1) == id && c.get_string("state", "") == "COMPLETED";
         })) {
      Json cj = c;
      for (auto& v : store_->Scan("validations", [&](const Json& v) {
             return v.get_int("trial_id", -1) == c["trial_id"].as_int() && v.get_int("step_id", -1) == c["step_id"].as_int();
           })) {
        cj["validation_metrics"] = v["metrics"]["validation_metrics"];
        try {
          cj["searcher_metric"] = ValidationMetric(v["metrics"]["validation_metrics"], metric);
        } catch (const std::exception&) {
        }
      }
      out.push_back(cj);
    }
    std::stable_sort(out.begin(), out.end(), [&](const Json& a, const Json& b) {
      bool ha = a.has("searcher_metric"), hb = b.has("searcher_metric");
      if (ha != hb) return ha;
      if (!ha) return false;
      return smaller ? a["searcher_metric"].as_double() < b["searcher_metric"].as_double()
                     : a["searcher_metric"].as_double() > b["searcher_metric"].as_double();
    });
    Json arr = Json::array();
    for (auto& c : out) arr.push_back(c);
    return J(200, arr);
  });
  http_.Route("GET", "/experiments/:id/metrics", [this](const net::Request& r) {
    int64_t id = IntParam(r, "id");
    Json out = Json::array();
    for (auto& t : store_->Where("trials", "experiment_id", Json(id))) {
      Json tj = Json::object();
      int64_t tid = t["id"].as_int();
      tj["trial_id"] = tid;
      Json tr = Json::array(), va = Json::array();
      for (auto& s : store_->Where("steps", "trial_id", Json(tid))) {
        if (s.get_string("state", "") != "COMPLETED") continue;
        Json p = Json::object();
        p["step_id"] = s["step_id"];
        p["total_batches"] = s.get_int("prior_batches_processed", 0) + s.get_int("num_batches", 0);
        p["metrics"] = s["metrics"]["avg_metrics"];
        tr.push_back(p);
      }
      for (auto& v : store_->Where("validations", "trial_id", Json(tid))) {
        if (v.get_string("state", "") != "COMPLETED") continue;
        Json p = Json::object();
        p["step_id"] = v["step_id"];
        p["total_batches"] = v.get_int("prior_batches_processed", 0);
        p["metrics"] = v["metrics"]["validation_metrics"];
        va.push_back(p);
      }
      // ?downsample=N: LTTB over (total_batches, metric) per metric name (reference TrialsSample)
      size_t ds = static_cast<size_t>(std::stoll(r.Query("downsample", "0")));
      const std::string mname = r.Query("metric", "");
      if (ds >= 3 && !mname.empty()) {
        auto sample = [&](const Json& series) {
          std::vector<Point> pts;
          for (auto& p : series.as_array())
            if (p["metrics"].is_object() && p["metrics"][mname].is_number())
              pts.push_back({static_cast<double>(p.get_int("total_batches", 0)), p["metrics"][mname].as_double()});
          std::sort(pts.begin(), pts.end(), [](const Point& a, const Point& b) { return a.x < b.x; });
          Json arr = Json::array();
          for (auto& p : Downsample(pts, ds)) {
            Json j = Json::object();
            j["total_batches"] = static_cast<int64_t>(p.x);
            j["value"] = p.y;
            arr.push_back(j);
          }
          return arr;
        };
        tj["training"] = sample(tr);
        tj["validation"] = sample(va);
      } else {
        tj["training"] = tr;
        tj["validation"] = va;
      }
      out.push_back(tj);
    }
    return J(200, out);
  });

  // --------------------------------------------------------------------------- trials
  http_.Route("GET", "/trials/:id", [this](const net::Request& r) {
    int64_t id = IntParam(r, "id");
    Json t;
    if (!store_->Get("trials", id, &t)) return Err(404, "trial not found");
    Json steps = Json::array(), vals = Json::array(), ckpts = Json::array();
    for (auto& s : store_->Where("steps", "trial_id", Json(id))) steps.push_back(s);
    for (auto& s : store_->Where("validations", "trial_id", Json(id))) vals.push_back(s);
    for (auto& s : store_->Where("checkpoints", "trial_id", Json(id))) ckpts.push_back(s);
    t["steps"] = steps;
    t["validations"] = vals;
    t["checkpoints"] = ckpts;
    return J(200, t);
  });
  http_.Route("GET", "/trials/:id/logs", [this](const net::Request& r) {
    // filters as the reference TrialLogsRequest: rank_id, stdtype, container_id, agent (via
    // container), substring match, head/tail limits
    int64_t id = IntParam(r, "id");
    int64_t offset = std::stoll(r.Query("offset", "0"));
    int64_t limit = std::stoll(r.Query("limit", "100000"));
    const std::string rank = r.Query("rank_id", ""), stdtype = r.Query("stdtype", ""),
                      cid = r.Query("container_id", ""), grep = r.Query("contains", "");
    const bool tail = r.Query("tail", "false") == "true";
    auto pred = [&](const Json& l) {
      if (!rank.empty() && std::to_string(l.get_int("rank_id", 0)) != rank) return false;
      if (!stdtype.empty() && l.get_string("stdtype", "") != stdtype) return false;
      if (!cid.empty() && l.get_string("container_id", "") != cid) return false;
      if (!grep.empty() && l.get_string("message", "").find(grep) == std::string::npos) return false;
      return true;
    };
    Json out = Json::array();
    for (auto& l : logs_->Read("trial-" + std::to_string(id), offset, std::max<int64_t>(0, limit), pred, tail))
      out.push_back(l);
    return J(200, out);
  });
  http_.Route("POST", "/trials/:id/kill", [this](const net::Request& r) {
    int64_t id = IntParam(r, "id");
    Json t;
    if (!store_->Get("trials", id, &t)) return Err(404, "trial not found");
    Ref tr = sys_->Get("/experiments/" + std::to_string(t["experiment_id"].as_int()) + "/" + t["request_id"].as_string());
    if (!tr) return Err(409, "trial is not running");
    tr->Tell(TrialKill{});
    return J(200, Json::object());
  });
  http_.Route("POST", "/trial_logs", [this](const net::Request& r) {
    Json body = Json::parse(r.body);
    Json items = body.is_array() ? body : Json(Json::Array{body});
    std::map<int64_t, std::vector<Json>> by_trial;  // one segment append per trial per request
    const std::string now = NowRFC3339();
    for (auto& l : items.as_array()) {
      Json row = Json::object();
      row["trial_id"] = l.get_int("trial_id", 0);
      row["message"] = l.get_string("message", l.get_string("log", ""));
      row["stdtype"] = l.get_string("stdtype", "stdout");
      row["container_id"] = l.get_string("container_id", "");
      row["rank_id"] = l.get_int("rank_id", 0);
      row["timestamp"] = now;
      by_trial[row["trial_id"].as_int()].push_back(row);
    }
    for (auto& kv : by_trial) logs_->Append("trial-" + std::to_string(kv.first), std::move(kv.second));
    return J(200, Json::object());
  });
  http_.Route("GET", "/checkpoints/:uuid", [this](const net::Request& r) {
    for (auto& c : store_->Where("checkpoints", "uuid", Json(r.Param("uuid")))) {
      Json t;
      if (store_->Get("trials", c["trial_id"].as_int(), &t)) {
        c["hparams"] = t["hparams"];
        Json e;
        if (store_->Get("experiments", t["experiment_id"].as_int(), &e)) c["experiment_config"] = e["config"];
      }
      for (auto& v : store_->Scan("validations", [&](const Json& v) {
             return v.get_int("trial_id", -1) == c["trial_id"].as_int() && v.get_int("step_id", -1) == c["step_id"].as_int();
           }))
        c["validation_metrics"] = v["metrics"]["validation_metrics"];
      return J(200, c);
    }
    return Err(404, "checkpoint not found");
  });

  // --------------------------------------------------------------------- agents/pools
  auto agents_json = [this]() {
    Json out = Json::array();
    std::vector<std::string> pools;
    {
      std::lock_guard<std::mutex> g(mu_);
      for (auto& p : pools_) pools.push_back(p.first);
    }
    for (auto& p : pools) {
      actor::Message m = Pool(p)->AskSync(PoolSummary{});
      if (!m.has_value()) continue;
      Json s = std::any_cast<Json>(m);
      for (auto& a : s["agents"].as_array()) {
        Json aj = a;
        aj["resource_pool"] = p;
        out.push_back(aj);
      }
    }
    return out;
  };
  http_.Route("GET", "/agents", [agents_json](const net::Request&) { return J(200, agents_json()); });
  auto slot_toggle = [this](const net::Request& r, int device, bool enable) {
    std::string agent = r.Param("id");
    std::string pool;
    {
      std::lock_guard<std::mutex> g(mu_);
      auto it = agents_.find(agent);
      if (it == agents_.end()) return Err(404, "agent not found");
      pool = it->second->pool;
    }
    actor::Message m = Pool(pool)->AskSync(SetSlotEnabled{agent, device, enable});
    bool ok = m.has_value() && std::any_cast<bool>(m);
    return ok ? J(200, Json::object()) : Err(404, "slot not found");
  };
  http_.Route("POST", "/agents/:id/slots/:slot/enable",
              [slot_toggle](const net::Request& r) { return slot_toggle(r, std::stoi(r.Param("slot")), true); });
  http_.Route("POST", "/agents/:id/slots/:slot/disable",
              [slot_toggle](const net::Request& r) { return slot_toggle(r, std::stoi(r.Param("slot")), false); });
  http_.Route("POST", "/agents/:id/enable", [slot_toggle](const net::Request& r) { return slot_toggle(r, -1, true); });
  http_.Route("POST", "/agents/:id/disable", [slot_toggle](const net::Request& r) { return slot_toggle(r, -1, false); });
  http_.Route("GET", "/resource_pools", [this](const net::Request&) {
    Json out = Json::array();
    std::vector<std::string> pools;
    {
      std::lock_guard<std::mutex> g(mu_);
      for (auto& p : pools_) pools.push_back(p.first);
    }
    for (auto& p : pools) {
      actor::Message m = Pool(p)->AskSync(PoolSummary{});
      if (m.has_value()) {
        Json s = std::any_cast<Json>(m);
        s.as_object().erase("agents");
        out.push_back(s);
      }
    }
    return J(200, out);
  });

  // ------------------------------------------------------------------------- commands
  http_.Route("POST", "/commands", [this](const net::Request& r) {
    Json body = Json::parse(r.body);
    Json cfg = body["config"];
    if (!cfg["entrypoint"].is_array() || cfg["entrypoint"].size() == 0)
      throw std::invalid_argument("command config needs entrypoint: [argv...]");
    Json row = Json::object();
    row["config"] = cfg;
    row["state"] = "PENDING";
    row["start_time"] = NowRFC3339();
    row["description"] = cfg.get_string("description", "");
    row["type"] = cfg.get_string("type", "command");
    row["owner"] = UserForRequest(r).empty() ? std::string("determined") : UserForRequest(r);
    int64_t id = store_->Insert("commands", row);
    Json ctxrow = Json::object();
    ctxrow["files"] = body["context"].is_array() ? body["context"] : Json::array();
    store_->Put("command_contexts", id, ctxrow);
    // Secrets (task auth tokens) travel beside the config, not in it: the stored row -- and with it
    // every GET /commands and /api/v1/{shells,notebooks,...} response -- never holds them.
    Json secret = body["secret_environment"].is_array() ? body["secret_environment"] : Json::array();
    sys_->ActorOf("commands/" + std::to_string(id), std::make_unique<CommandActor>(this, id, cfg, secret));
    Json out = Json::object();
    out["id"] = id;
    return J(201, out);
  });
  http_.Route("GET", "/commands", [this](const net::Request& r) {
    Json out = Json::array();
    std::string type = r.Query("type", "");
    for (auto& c : store_->Scan("commands"))
      if (type.empty() || c.get_string("type", "command") == type) out.push_back(c);
    return J(200, out);
  });
  http_.Route("POST", "/commands/:id/ready", [this](const net::Request& r) {
    Json body = Json::parse(r.body.empty() ? "{}" : r.body);
    Ref ref = sys_->Get("/commands/" + r.Param("id"));
    if (!ref) return Err(404, "command not running");
    ServiceReady sr;
    sr.port = static_cast<int>(body.get_int("port", 0));
    if (sr.port <= 0) return Err(400, "ready needs a port");
    auto f = ref->Ask(sr);
    if (f.wait_for(std::chrono::seconds(10)) != std::future_status::ready) return Err(504, "command did not answer");
    return J(200, Json::object());
  });
  // Service proxy (reference /proxy/:service/*, master/internal/proxy): forwards to a ready
  // command's HTTP service, e.g. `det tensorboard start` -> /proxy/cmd-<id>/
  auto proxy = [this](const net::Request& r) {
    std::string task = r.Param("task");
    int64_t id = 0;
    try {
      id = std::stoll(task.rfind("cmd-", 0) == 0 ? task.substr(4) : task);
    } catch (const std::exception&) {
      return Err(404, "unknown service " + task);
    }
    Json c;
    if (!store_->Get("commands", id, &c) || c.get_string("service_address", "").empty())
      return Err(404, "service " + task + " is not ready");
    if (c.get_string("state", "") == "TERMINATED") return Err(404, "service " + task + " has exited");
    std::string addr = c.get_string("service_address", "");
    auto colon = addr.rfind(':');
    std::string path = "/" + r.Param("*");
    std::string qs;
    for (auto& kv : r.query) qs += (qs.empty() ? "?" : "&") + net::UrlEncode(kv.first) + "=" + net::UrlEncode(kv.second);
    auto it = r.headers.find("content-type");
    auto resp = net::HttpCall(addr.substr(0, colon), std::stoi(addr.substr(colon + 1)), r.method, path + qs, r.body,
                              30000, it == r.headers.end() ? "application/json" : it->second);
    if (!resp.error.empty()) return Err(502, "proxy: " + resp.error);
    net::Response out;
    out.status = resp.status;
    out.body = resp.body;
    out.content_type = resp.content_type.empty() ? "application/octet-stream" : resp.content_type;
    return out;
  };
  for (const char* m : {"GET", "POST", "PUT", "DELETE"}) {
    http_.Route(m, "/proxy/:task/*", proxy);
    http_.Route(m, "/proxy/:task", proxy);
  }
  // TCP tunnel (reference cli/determined_cli/tunnel.py over master/internal/proxy's WebSocket
  // upgrade): a WebSocket upgrade on /proxy/<task>/ is spliced onto a raw TCP connection to the
  // service, binary frames both ways, so any TCP protocol (not just HTTP) reaches the task;
  // `det tunnel` is the client.
  auto tunnel = [this](const net::Request& r, net::WsPtr ws) {
    std::string task = r.Param("task");
    int64_t id = 0;
    try {
      id = std::stoll(task.rfind("cmd-", 0) == 0 ? task.substr(4) : task);
    } catch (const std::exception&) {
      ws->Close();
      return;
    }
    Json c;
    if (!store_->Get("commands", id, &c) || c.get_string("service_address", "").empty() ||
        c.get_string("state", "") == "TERMINATED") {
      ws->Close();
      return;
    }
    std::string addr = c.get_string("service_address", "");
    auto colon = addr.rfind(':');
    std::string err;
    int fd = net::ConnectTcp(addr.substr(0, colon), std::stoi(addr.substr(colon + 1)), 10000, &err);
    if (fd < 0) {
      ws->Close();
      return;
    }
    std::thread up([fd, ws] {  // service -> client
      std::string buf(65536, '\0');
      for (;;) {
        ssize_t n = ::recv(fd, &buf[0], buf.size(), 0);
        if (n < 0 && errno == EINTR) continue;
        if (n <= 0 || !ws->SendBinary(buf.substr(0, static_cast<size_t>(n)))) break;
      }
      ws->Close();
    });
    ws->ReadLoop([fd](const std::string& m) {  // client -> service; an empty frame = client EOF
      if (m.empty()) {
        ::shutdown(fd, SHUT_WR);  // half-close: the service sees EOF and can still answer
        return;
      }
      size_t off = 0;
      while (off < m.size()) {
        ssize_t n = ::send(fd, m.data() + off, m.size() - off, MSG_NOSIGNAL);
        if (n < 0 && errno == EINTR) continue;
        if (n <= 0) return;
        off += static_cast<size_t>(n);
      }
    });
    ::shutdown(fd, SHUT_RDWR);
    up.join();
    ::close(fd);
  };
  // a raw TCP stream into a task's service: gated by the same session check as /proxy
  http_.RouteWs("/proxy/:task/*", tunnel, /*require_auth=*/true);
  http_.RouteWs("/proxy/:task", tunnel, /*require_auth=*/true);
  http_.Route("GET", "/commands/:id", [this](const net::Request& r) {
    Json c;
    if (!store_->Get("commands", IntParam(r, "id"), &c)) return Err(404, "command not found");
    return J(200, c);
  });
  http_.Route("GET", "/commands/:id/context", [this](const net::Request& r) {
    Json c;
    if (!store_->Get("command_contexts", IntParam(r, "id"), &c)) return Err(404, "not found");
    return J(200, c);
  });
  http_.Route("GET", "/commands/:id/logs", [this](const net::Request& r) {
    std::string task = "cmd-" + r.Param("id");
    int64_t offset = std::stoll(r.Query("offset", "0"));
    Json out = Json::array();
    for (auto& l : logs_->Read("task-" + task, offset, INT64_MAX)) out.push_back(l);
    return J(200, out);
  });
  http_.Route("POST", "/commands/:id/kill", [this](const net::Request& r) {
    Ref c = sys_->Get("/commands/" + r.Param("id"));
    if (!c) return Err(409, "command is not running");
    c->Tell(CommandKill{});
    return J(200, Json::object());
  });

  // --------------------------------------------------------------- searcher preview
  http_.Route("POST", "/searcher/preview", [this](const net::Request& r) {
    Json body = Json::parse(r.body);
    Json user = body["config"].is_string() ? Json::parse(body["config"].as_string()) : body["config"];
    Json cfg = MergeExperimentConfig(user, cfg_.checkpoint_storage, Json(), 0);
    uint32_t seed = static_cast<uint32_t>(body.has("seed") && body["seed"].is_number()
                                              ? body["seed"].as_int()
                                              : cfg["reproducibility"].get_int("experiment_seed", 0));
    Searcher s(seed, NewSearchMethod(cfg["searcher"]), cfg["hyperparameters"]);
    std::mt19937_64 rng(seed);
    std::uniform_real_distribution<double> U(0.0, 1.0);
    auto res = Simulate(s, [&](int, int) { return U(rng); }, true, seed, cfg["searcher"].get_string("metric", "metric"));
    Json out = Json::object();
    out["results"] = res.Summary();
    out["trials"] = res.TrialSimulations();
    out["seed"] = static_cast<int64_t>(seed);
    out["config"] = cfg;
    out["num_trials"] = static_cast<int64_t>(res.order.size());
    return J(200, out);
  });

  // ------------------------------------------------------------------------ templates
  http_.Route("GET", "/templates", [this](const net::Request&) {
    Json out = Json::array();
    for (auto& t : store_->Scan("templates")) out.push_back(t);
    return J(200, out);
  });
  http_.Route("GET", "/templates/:name", [this](const net::Request& r) {
    for (auto& t : store_->Where("templates", "name", Json(r.Param("name")))) return J(200, t);
    return Err(404, "template not found");
  });
  http_.Route("PUT", "/templates/:name", [this](const net::Request& r) {
    Json body = Json::parse(r.body);
    Json cfg = body.has("config") ? body["config"] : body;
    if (cfg.is_string()) cfg = Json::parse(cfg.as_string());
    store_->DeleteWhere("templates", [&](const Json& t) { return t.get_string("name", "") == r.Param("name"); });
    Json row = Json::object();
    row["name"] = r.Param("name");
    row["config"] = cfg;
    store_->Insert("templates", row);
    return J(200, row);
  });
  http_.Route("DELETE", "/templates/:name", [this](const net::Request& r) {
    store_->DeleteWhere("templates", [&](const Json& t) { return t.get_string("name", "") == r.Param("name"); });
    return J(200, Json::object());
  });

  // ------------------------------------------------------------------- model registry
  http_.Route("GET", "/models", [this](const net::Request&) {
    Json out = Json::array();
    for (auto& m : store_->Scan("models")) out.push_back(m);
    return J(200, out);
  });
  http_.Route("POST", "/models/:name", [this](const net::Request& r) {
    if (!store_->Where("models", "name", Json(r.Param("name"))).empty()) return Err(409, "model exists");
    Json body = r.body.empty() ? Json::object() : Json::parse(r.body);
    Json row = Json::object();
    row["name"] = r.Param("name");
    row["description"] = body.get_string("description", "");
    row["metadata"] = body["metadata"];
    row["creation_time"] = NowRFC3339();
    store_->Insert("models", row);
    return J(201, row);
  });
  http_.Route("GET", "/models/:name", [this](const net::Request& r) {
    for (auto& m : store_->Where("models", "name", Json(r.Param("name")))) {
      Json vs = Json::array();
      for (auto& v : store_->Where("model_versions", "model_name", Json(r.Param("name")))) vs.push_back(v);
      m["versions"] = vs;
      return J(200, m);
    }
    return Err(404, "model not found");
  });
  http_.Route("GET", "/models/:name/versions", [this](const net::Request& r) {
    Json vs = Json::array();
    for (auto& v : store_->Where("model_versions", "model_name", Json(r.Param("name")))) vs.push_back(v);
    return J(200, vs);
  });
  http_.Route("POST", "/models/:name/versions", [this](const net::Request& r) {
    if (store_->Where("models", "name", Json(r.Param("name"))).empty()) return Err(404, "model not found");
    Json body = Json::parse(r.body);
    std::string uuid = body.get_string("checkpoint_uuid", "");
    if (store_->Where("checkpoints", "uuid", Json(uuid)).empty()) return Err(404, "checkpoint not found");
    int64_t ver = static_cast<int64_t>(store_->Where("model_versions", "model_name", Json(r.Param("name"))).size()) + 1;
    Json row = Json::object();
    row["model_name"] = r.Param("name");
    row["version"] = ver;
    row["checkpoint_uuid"] = uuid;
    row["creation_time"] = NowRFC3339();
    store_->Insert("model_versions", row);
    return J(201, row);
  });

  // ----------------------------------------------------------------------- websockets
  http_.RouteWs("/agents", [this](const net::Request& r, net::WsPtr ws) { HandleAgentSocket(r, ws); });
  http_.RouteWs("/ws/trial/:e/:t/:c", [this](const net::Request& r, net::WsPtr ws) { HandleTrialSocket(r, ws); });
  http_.RouteWs("/ws/data-layer/*", [this](const net::Request& r, net::WsPtr ws) { HandleRWLockSocket(r, ws); });
  InstallApiV1();

  // WebUI (determined_1_amd/webui/index.html): a single-file app over /api/v1, served as-is
  auto webui = [](const net::Request&) {
    char buf[4096];
    ssize_t n = readlink("/proc/self/exe", buf, sizeof(buf) - 1);
    std::string self = n > 0 ? std::string(buf, static_cast<size_t>(n)) : "det-master";
    std::ifstream f(self.substr(0, self.rfind('/')) + "/../webui/index.html", std::ios::binary);
    if (!f) return net::Response::Text(404, "webui not installed");
    std::stringstream ss;
    ss << f.rdbuf();
    net::Response r;
    r.status = 200;
    r.content_type = "text/html; charset=utf-8";
    r.body = ss.str();
    return r;
  };
  http_.Route("GET", "/det", webui);
  http_.Route("GET", "/det/*", webui);
  http_.Route("GET", "/", [](const net::Request&) {
    net::Response r;
    r.status = 302;
    r.headers["Location"] = "/det/";
    return r;
  });
}

// One socket = one lock request; the lock is held until the socket closes (reference
// core.go:253-289).  The resource is the full request path, as in the reference.
void Master::HandleRWLockSocket(const net::Request& r, net::WsPtr ws) {
  std::string mode = r.Query("read_lock", "");
  for (auto& ch : mode) ch = static_cast<char>(std::tolower(static_cast<unsigned char>(ch)));
  if (mode != "true" && mode != "false") {
    ws->Send("error: read_lock must be true or false");
    ws->Close();
    return;
  }
  const bool read = mode == "true";
  std::weak_ptr<net::WsConn> weak = ws;
  int64_t ticket = rw_coordinator_.Acquire(r.path, read, [weak](int64_t, bool granted_read) {
    if (auto s = weak.lock()) s->Send(granted_read ? "read_lock_granted" : "write_lock_granted");
  });
  ws->ReadLoop([](const std::string&) {});
  rw_coordinator_.Release(ticket);
}

void Master::ReportTelemetry(const std::string& event, Json properties) {
  if (cfg_.telemetry_file.empty()) return;
  Json line = Json::object();
  line["event"] = event;
  line["timestamp"] = NowRFC3339();
  line["cluster_id"] = cluster_id_;
  line["properties"] = std::move(properties);
  std::lock_guard<std::mutex> g(telemetry_mu_);
  std::ofstream f(cfg_.telemetry_file, std::ios::app);
  f << line.dump() << "\n";
}

bool Master::RegisterAgent(const std::shared_ptr<AgentConn>& conn, std::string* err) {
  std::lock_guard<std::mutex> g(mu_);
  if (conn->pool.empty() || !pools_.count(conn->pool)) conn->pool = pools_.begin()->first;
  if (agents_.count(conn->id)) {
    *err = "agent id already connected: " + conn->id;
    return false;
  }
  agents_[conn->id] = conn;
  return true;
}

void Master::HandleAgentSocket(const net::Request& r, net::WsPtr ws) {
  auto conn = std::make_shared<AgentConn>();
  conn->id = r.Query("id", "agent-" + NewUUID().substr(0, 8));
  conn->pool = r.Query("resource_pool", "");
  conn->label = r.Query("label", "");
  conn->host = r.Query("host", r.remote_addr);
  conn->ws = ws;
  std::string err;
  if (!RegisterAgent(conn, &err)) {
    Json m = Json::object();
    m["type"] = "Error";
    m["error"] = err;
    ws->Send(m.dump());
    return;
  }
  Json opts = Json::object();
  opts["type"] = "MasterSetAgentOptions";
  opts["master_host"] = advertised_host_;
  opts["master_port"] = port_;
  opts["cluster_id"] = cluster_id_;
  ws->Send(opts.dump());
  ws->ReadLoop([&](const std::string& text) {
    Json m;
    try {
      m = Json::parse(text);
    } catch (const std::exception&) {
      return;
    }
    OnAgentMessage(conn, m);
  });
  AgentGone(conn);
}

// One agent -> master message (a real agent's WebSocket, or a virtual agent such as the
// Kubernetes resource manager's).
void Master::OnAgentMessage(const std::shared_ptr<AgentConn>& conn, const Json& m) {
  const std::string t = m.get_string("type", "");
  if (t == "AgentStarted") {
    sched::Agent a;
    a.id = conn->id;
    a.label = m.get_string("label", conn->label);
    conn->devices = m["devices"];
    {
      Json props = Json::object();
      props["uuid"] = conn->id;
      props["devices"] = conn->devices;
      ReportTelemetry("agent_connected", props);
    }
    for (auto& d : m["devices"].as_array()) {
      sched::Slot s;
      s.device_id = static_cast<int>(d.get_int("id", 0));
      s.uuid = d.get_string("uuid", "");
      s.type = d.get_string("type", "gpu");
      a.slots.push_back(s);
    }
    Pool(conn->pool)->Tell(AddAgent{a});
  } else if (t == "ContainerStateChanged") {
    if (m.get_int("sent_us", 0) > 0) {
      const double ms = (std::chrono::duration_cast<std::chrono::microseconds>(
                             std::chrono::system_clock::now().time_since_epoch()).count() -
                         m.get_int("sent_us", 0)) / 1000.0;
      std::lock_guard<std::mutex> g(state_lat_mu_);
      state_lat_max_ms_ = std::max(state_lat_max_ms_, ms);
      state_lat_sum_ms_ += ms;
      ++state_lat_n_;
    }
    std::string cid = m.get_string("container_id", "");
    Ref tr = TrialForContainer(cid);
    if (tr)
      tr->Tell(ContainerStateMsg{cid, m.get_string("state", ""), static_cast<int>(m.get_int("exit_code", 0)),
                                 m.get_string("failure", ""), m.get_string("address", "")});
  } else if (t == "ContainerLog" && !m.get_string("task_id", "").empty()) {
    Json row = Json::object();
    row["task_id"] = m["task_id"];
    row["message"] = m["log"];
    row["stdtype"] = m["stdtype"];
    row["timestamp"] = NowRFC3339();
    logs_->Append("task-" + m.get_string("task_id", ""), {row});
  } else if (t == "ContainerLog") {
    AppendTrialLog(m.get_int("trial_id", 0), m.get_string("log", ""), m.get_string("stdtype", "stdout"),
                   m.get_string("container_id", ""), static_cast<int>(m.get_int("rank", 0)));
  }
}

void Master::AgentGone(const std::shared_ptr<AgentConn>& conn) {
  // every container on the agent is gone (reference agent.go:114-126)
  std::vector<std::string> cids;
  {
    std::lock_guard<std::mutex> g(mu_);
    cids.assign(conn->containers.begin(), conn->containers.end());
    agents_.erase(conn->id);
  }
  {
    Json props = Json::object();  // telemetry file I/O outside mu_
    props["uuid"] = conn->id;
    ReportTelemetry("agent_disconnected", props);
  }
  Pool(conn->pool)->Tell(RemoveAgent{conn->id});
  for (auto& cid : cids) {
    Ref tr = TrialForContainer(cid);
    if (tr) tr->Tell(ContainerStateMsg{cid, "Terminated", -1, "agent failed while container was running", ""});
  }
  Log("agent " + conn->id + " disconnected");
}

void Master::HandleTrialSocket(const net::Request& r, net::WsPtr ws) {
  std::string cid = r.Param("c");
  Ref tr = TrialForContainer(cid);
  if (!tr) return;
  tr->Tell(SocketConnected{cid, ws});
  ws->ReadLoop([&](const std::string& text) {
    try {
      tr->Tell(SocketMessage{cid, Json::parse(text)});
    } catch (const std::exception&) {
    }
  });
  tr->Tell(SocketClosed{cid});
}

void Master::RestoreExperiments() {
  // Non-terminal experiments are rebuilt from the event log (experiment.go:238-294).
  for (auto& e : store_->Scan("experiments")) {
    std::string st = e.get_string("state", "");
    if (st == "COMPLETED" || st == "CANCELED" || st == "ERROR") continue;
    int64_t id = e["id"].as_int();
    std::vector<Json> events = store_->Where("searcher_events", "experiment_id", Json(id));
    std::sort(events.begin(), events.end(), [](const Json& a, const Json& b) { return a["id"].as_int() < b["id"].as_int(); });
    if (st.rfind("STOPPING_", 0) == 0) {
      // nothing left running: finish the stop
      Json patch = Json::object();
      patch["state"] = st == "STOPPING_CANCELED" ? "CANCELED" : st == "STOPPING_ERROR" ? "ERROR" : "COMPLETED";
      patch["end_time"] = NowRFC3339();
      store_->Update("experiments", id, patch);
      continue;
    }
    Ref ex = sys_->ActorOf("experiments/" + std::to_string(id), std::make_unique<ExperimentActor>(this, id, e["config"], true));
    ex->Tell(ReplayEvents{events});
    Log("restoring experiment " + std::to_string(id) + " from " + std::to_string(events.size()) + " events");
  }
}

Json Master::AgentUserGroupFor(const std::string& username) {
  if (!username.empty())
    for (auto& u : store_->Where("users", "username", Json(username)))
      if (u["agent_user_group"].is_object()) return u["agent_user_group"].clone();
  return cfg_.default_agent_user_group.is_object() ? cfg_.default_agent_user_group.clone() : Json();
}

Json Master::AgentUserGroupForExperiment(int64_t experiment_id) {
  Json e;
  if (!store_->Get("experiments", experiment_id, &e)) return AgentUserGroupFor("");
  return AgentUserGroupFor(e.get_string("owner", ""));
}

void Master::AddTaskDefaults(Json& env, Json& files) const {
  // task_container_defaults -> container env (reference master/pkg/tasks/task.go:224-248).  The agent
  // runs tasks as process groups, not Docker containers: shm size and network mode are advisory here
  // and exported for the task (and any container runtime wrapping the agent) to honour.
  env["DET_TRIAL_RUNNER_NETWORK_INTERFACE"] =
      cfg_.dtrain_network_interface.empty() ? "DET_AUTO_DETECT_NETWORK_INTERFACE" : cfg_.dtrain_network_interface;
  if (!cfg_.dtrain_network_interface.empty()) {
    env["NCCL_SOCKET_IFNAME"] = cfg_.dtrain_network_interface;  // RCCL bootstrap / socket transport
    env["GLOO_SOCKET_IFNAME"] = cfg_.dtrain_network_interface;  // the gloo control plane
  }
  if (!cfg_.nccl_port_range.empty()) env["NCCL_PORT_RANGE"] = cfg_.nccl_port_range;
  if (!cfg_.gloo_port_range.empty()) env["GLOO_PORT_RANGE"] = cfg_.gloo_port_range;
  env["DET_SHM_SIZE_BYTES"] = std::to_string(cfg_.shm_size_bytes);
  env["DET_NETWORK_MODE"] = cfg_.network_mode;
  if (!tls_cert_pem_.empty()) {  // reference addTLSVars: tasks talk TLS to the master
    env["DET_USE_TLS"] = "true";
    env["DET_MASTER_CERT_FILE"] = ".det/master.crt";
    Json f = Json::object();
    f["path"] = ".det/master.crt";
    f["content"] = net::Base64Encode(tls_cert_pem_);
    files.push_back(f);
  }
}

int Master::Start() {
  for (auto& p : cfg_.resource_pools) pools_[p] = sys_->ActorOf("pools/" + p, std::make_unique<ResourcePoolActor>(this, p));
  if (!cfg_.tls_cert.empty()) {
    std::string err;
    if (!http_.EnableTls(cfg_.tls_cert, cfg_.tls_key, &err)) throw std::runtime_error(err);
    std::ifstream f(cfg_.tls_cert);
    std::stringstream ss;
    ss << f.rdbuf();
    tls_cert_pem_ = ss.str();
    Log("serving the API over TLS (" + cfg_.tls_cert + ")");
  }
  InstallRoutes();
  port_ = http_.Listen(cfg_.listen_host, cfg_.port);
  if (port_ < 0) throw std::runtime_error("cannot bind port " + std::to_string(cfg_.port));
  if (cfg_.listen_host != "0.0.0.0" && !cfg_.listen_host.empty()) advertised_host_ = cfg_.listen_host;
  http_.Start();
  if (cfg_.provisioner.is_object() && cfg_.provisioner.get_int("max_instances", 0) > 0) {
    prov::ProvisionerConfig pc = prov::ProvisionerConfig::FromJson(cfg_.provisioner);
    pc.master_host = advertised_host_;
    pc.master_port = port_;
    pc.python = cfg_.python;
    pc.cluster_id = cluster_id_;
    if (pc.framework_root.empty()) {
      char buf[4096];
      ssize_t n = readlink("/proc/self/exe", buf, sizeof(buf) - 1);
      std::string self = n > 0 ? std::string(buf, static_cast<size_t>(n)) : "det-master";
      pc.framework_root = self.substr(0, self.rfind('/')) + "/../..";  // <root>/determined_1_amd/_native/
    }
    if (pc.agent_binary.empty()) {
      char buf[4096];
      ssize_t n = readlink("/proc/self/exe", buf, sizeof(buf) - 1);
      std::string self = n > 0 ? std::string(buf, static_cast<size_t>(n)) : "det-master";
      pc.agent_binary = self.substr(0, self.rfind('/')) + "/det-agent";
    }
    for (auto& p : cfg_.resource_pools)
      sys_->ActorOf("provisioners/" + p, std::make_unique<ProvisionerActor>(this, p, pc));
    Log("provisioner enabled: max " + std::to_string(pc.max_instances) + " agents per pool");
  }
  if (cfg_.kubernetes.is_object()) {
    kube_ = std::make_unique<KubernetesRM>(this, KubeConfig::FromJson(cfg_.kubernetes));
    kube_->Start();
  }
  RestoreExperiments();
  Log(std::string("listening on ") + cfg_.listen_host + ":" + std::to_string(port_) + " scheduler=" + cfg_.scheduler);
  return port_;
}

void Master::Stop() {
  {
    std::lock_guard<std::mutex> g(stop_mu_);
    if (stopped_) return;
    stopped_ = true;
  }
  shutting_down_ = true;
  if (kube_) kube_->Stop();
  http_.Stop();
  {
    std::lock_guard<std::mutex> g(mu_);
    for (auto& a : agents_)
      if (a.second->ws) a.second->ws->Close();
  }
  sys_->Shutdown();
  store_->Flush();
  stop_cv_.notify_all();
}

void Master::Wait() {
  std::unique_lock<std::mutex> l(stop_mu_);
  stop_cv_.wait(l, [&] { return stopped_; });
}

}  // namespace master
}  // namespace detcore
