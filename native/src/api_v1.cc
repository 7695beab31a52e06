// /api/v1: the reference's public API surface (proto/src/determined/api/v1/api.proto:73-785,
// served by grpc-gateway in master/internal/grpc/api.go) on the master's own HTTP server.
//
// Shape rules kept from the gateway so reference clients keep working:
//   * JSON field names are lowerCamelCase (runtime.JSONPb without OrigName), enums are the proto
//     names ("STATE_ACTIVE"), google.protobuf.Struct payloads (hparams, configs, metrics,
//     metadata) pass through untouched;
//   * query parameters are accepted in snake_case or lowerCamelCase; repeated fields as repeated
//     keys or comma-separated values;
//   * server-streaming RPCs (TrialLogs, TrialLogsFields, MasterLogs, MetricNames, MetricBatches,
//     TrialsSnapshot, TrialsSample, NotebookLogs) are HTTP/1.1 chunked responses carrying one
//     `{"result": ...}` JSON object per line, with the reference's follow/poll semantics
//     (api_experiment.go:539-960, api_trials.go:51-130);
//   * errors are `{"error": msg, "code": <grpc code>, "message": msg}` with the mapped status.
//
// Unary RPCs reuse the legacy REST handlers in-process (HttpServer::Dispatch) and reshape their
// JSON; the streams read the Store / LogStore directly.  There is no gRPC wire protocol: no
// protobuf runtime exists in this image, and the gateway's HTTP/JSON surface is what the CLI,
// SDK and WebUI use.
#include <algorithm>
#include <chrono>
#include <cmath>
#include <map>
#include <set>
#include <sstream>
#include <string>
#include <thread>
#include <vector>

#include "detcore/lttb.h"
#include "detcore/master.h"
#include "detcore/master_actors.h"
#include "detcore/searcher.h"

namespace detcore {
namespace master {

namespace {

using Writer = net::Response::Writer;

int GrpcCode(int http) {
  switch (http) {
    case 400: return 3;   // INVALID_ARGUMENT
    case 401: return 16;  // UNAUTHENTICATED
    case 403: return 7;   // PERMISSION_DENIED
    case 404: return 5;   // NOT_FOUND
    case 409: return 9;   // FAILED_PRECONDITION
    case 504: return 4;   // DEADLINE_EXCEEDED
    default: return http >= 500 ? 13 : 2;
  }
}

net::Response JV(int status, const Json& j) { return net::Response::Json(status, j.dump()); }

net::Response ErrV(int status, const std::string& msg) {
  Json j = Json::object();
  j["error"] = msg;
  j["code"] = GrpcCode(status);
  j["message"] = msg;
  j["details"] = Json::array();
  return JV(status, j);
}

std::string Camel(const std::string& k) {
  std::string out;
  bool up = false;
  for (char c : k) {
    if (c == '_') {
      up = !out.empty();
      continue;
    }
    out.push_back(up ? static_cast<char>(std::toupper(static_cast<unsigned char>(c))) : c);
    up = false;
  }
  return out;
}

std::string Snake(const std::string& k) {
  std::string out;
  for (char c : k) {
    if (std::isupper(static_cast<unsigned char>(c))) {
      out.push_back('_');
      out.push_back(static_cast<char>(std::tolower(static_cast<unsigned char>(c))));
    } else {
      out.push_back(c);
    }
  }
  return out;
}

// google.protobuf.Struct / free-form payloads: copied verbatim
const std::set<std::string>& OpaqueKeys() {
  static const std::set<std::string> k = {"hparams", "config", "metrics", "metadata", "validation_metrics",
                                          "avg_metrics", "batch_metrics", "experiment_config", "resources",
                                          "checkpoint", "files", "warm_start_checkpoint", "labels"};
  return k;
}

bool IsEnumState(const std::string& s) {
  if (s.empty() || s.rfind("STATE_", 0) == 0) return false;
  for (char c : s)
    if (!(std::isupper(static_cast<unsigned char>(c)) || c == '_')) return false;
  return true;
}

Json ToApi(const Json& j) {
  if (j.is_array()) {
    Json out = Json::array();
    for (auto& v : j.as_array()) out.push_back(ToApi(v));
    return out;
  }
  if (!j.is_object()) return j;
  Json out = Json::object();
  for (auto& kv : j.as_object()) {
    const std::string key = Camel(kv.first);
    if (OpaqueKeys().count(kv.first)) {
      out[key] = kv.second;
    } else if (kv.first == "state" && kv.second.is_string() && IsEnumState(kv.second.as_string())) {
      out[key] = "STATE_" + kv.second.as_string();
    } else {
      out[key] = ToApi(kv.second);
    }
  }
  return out;
}

// request-body keys: accept camelCase, hand snake_case to legacy handlers
Json FromApi(const Json& j) {
  if (j.is_array()) {
    Json out = Json::array();
    for (auto& v : j.as_array()) out.push_back(FromApi(v));
    return out;
  }
  if (!j.is_object()) return j;
  Json out = Json::object();
  for (auto& kv : j.as_object()) {
    const std::string key = Snake(kv.first);
    out[key] = OpaqueKeys().count(key) ? kv.second : FromApi(kv.second);
  }
  return out;
}

std::string Q(const net::Request& r, const std::string& snake, const std::string& dflt = "") {
  std::string v = r.Query(snake, "");
  if (v.empty()) v = r.Query(Camel(snake), "");
  return v.empty() ? dflt : v;
}

int64_t QInt(const net::Request& r, const std::string& snake, int64_t dflt) {
  std::string v = Q(r, snake);
  if (v.empty()) return dflt;
  try {
    return std::stoll(v);
  } catch (const std::exception&) {
    throw std::invalid_argument("query parameter " + snake + " must be an integer");
  }
}

bool QBool(const net::Request& r, const std::string& snake) {
  std::string v = Q(r, snake);
  return v == "true" || v == "1";
}

std::vector<std::string> QList(const net::Request& r, const std::string& snake) {
  std::vector<std::string> out;
  std::string v = Q(r, snake);
  std::stringstream ss(v);
  std::string item;
  while (std::getline(ss, item, ','))
    if (!item.empty()) out.push_back(item);
  return out;
}

bool Terminal(const std::string& s) {
  return s == "COMPLETED" || s == "CANCELED" || s == "ERROR" || s == "DELETED";
}

std::string StripState(const std::string& s) { return s.rfind("STATE_", 0) == 0 ? s.substr(6) : s; }

double PeriodSeconds(const net::Request& r, double dflt) {
  std::string v = Q(r, "period_seconds");
  if (v.empty()) return dflt;
  double d = std::stod(v);
  return d > 0 ? d : dflt;
}

// Sleep in small slices so a stopping server or a gone client ends the stream promptly.
bool StreamPause(const Writer& w, double seconds) {
  auto start = std::chrono::steady_clock::now();
  auto until = start + std::chrono::milliseconds(static_cast<int64_t>(seconds * 1000));
  auto probe = start;
  while (std::chrono::steady_clock::now() < until) {
    std::this_thread::sleep_for(std::chrono::milliseconds(50));
    if (!w("")) return false;  // server stopping
    auto now = std::chrono::steady_clock::now();
    if (now - probe >= std::chrono::seconds(1)) {
      probe = now;
      // whitespace between JSON lines is valid; a failed write means the client is gone
      if (!w(" ")) return false;
    }
  }
  return true;
}

bool SendResult(const Writer& w, const Json& result) {
  Json m = Json::object();
  m["result"] = result;
  return w(m.dump() + "\n");
}

net::Response Stream(std::function<void(const Writer&)> f) {
  net::Response r;
  r.stream = std::move(f);
  return r;
}

Json Pagination(int64_t offset, int64_t limit, int64_t total) {
  Json p = Json::object();
  int64_t start = std::min(offset, total);
  int64_t end = limit > 0 ? std::min(total, start + limit) : total;
  p["offset"] = offset;
  p["limit"] = limit;
  p["startIndex"] = start;
  p["endIndex"] = end;
  p["total"] = total;
  return p;
}

std::string MetricTypeOf(const net::Request& r) {
  std::string t = Q(r, "metric_type");
  if (t == "METRIC_TYPE_TRAINING" || t == "training" || t == "1") return "training";
  if (t == "METRIC_TYPE_VALIDATION" || t == "validation" || t == "2") return "validation";
  throw std::invalid_argument("must specify a metric type");
}

struct SeriesPoint {
  int64_t batches;
  double value;
};

}  // namespace

void Master::InstallApiV1() {
  // Legacy handler reuse: same headers (auth), new path/body.
  auto call = [this](const net::Request& orig, const std::string& method, const std::string& path,
                     const std::string& body = "") {
    net::Request r;
    r.method = method;
    r.headers = orig.headers;
    r.remote_addr = orig.remote_addr;
    auto q = path.find('?');
    r.path = path.substr(0, q);
    if (q != std::string::npos) {
      std::stringstream ss(path.substr(q + 1));
      std::string kv;
      while (std::getline(ss, kv, '&')) {
        auto eq = kv.find('=');
        r.query[net::UrlDecode(kv.substr(0, eq))] = eq == std::string::npos ? "" : net::UrlDecode(kv.substr(eq + 1));
      }
    }
    r.body = body;
    return http_.Dispatch(r);
  };
  // Legacy JSON reply -> (status, Json), passing errors through in the gateway shape.
  auto unwrap = [](const net::Response& r, Json* out) -> bool {
    if (r.status >= 400) return false;
    *out = r.body.empty() ? Json::object() : Json::parse(r.body);
    return true;
  };
  auto relay_err = [](const net::Response& r) {
    std::string msg = r.body;
    try {
      Json j = Json::parse(r.body);
      msg = j.get_string("error", r.body);
    } catch (const std::exception&) {
    }
    return ErrV(r.status, msg);
  };
  auto exp_api = [this](const Json& e) {
    Json o = Json::object();
    o["id"] = e["id"];
    o["description"] = e.get_string("description", "");
    o["labels"] = e["labels"].is_array() ? e["labels"] : (e["config"]["labels"].is_array() ? e["config"]["labels"] : Json::array());
    o["startTime"] = e["start_time"];
    o["endTime"] = e["end_time"];
    o["state"] = "STATE_" + e.get_string("state", "ACTIVE");
    o["archived"] = e.get_bool("archived", false);
    o["numTrials"] = static_cast<int64_t>(store_->Where("trials", "experiment_id", e["id"]).size());
    o["progress"] = e["progress"];
    o["username"] = e.get_string("owner", "determined");
    o["resourcePool"] = e["config"]["resources"].get_string("resource_pool", "");
    o["searcherType"] = e["config"]["searcher"].get_string("name", "");
    o["notes"] = e.get_string("notes", "");
    o["parentId"] = e["parent_id"];
    return o;
  };
  auto trial_api = [this](int64_t tid) {
    Json t;
    if (!store_->Get("trials", tid, &t)) return Json();
    Json e;
    store_->Get("experiments", t["experiment_id"].as_int(), &e);
    const std::string metric = e["config"]["searcher"].get_string("metric", "");
    const bool smaller = e["config"]["searcher"].get_bool("smaller_is_better", true);
    Json o = Json::object();
    o["id"] = tid;
    o["experimentId"] = t["experiment_id"];
    o["startTime"] = t["start_time"];
    o["endTime"] = t["end_time"];
    o["state"] = "STATE_" + t.get_string("state", "ACTIVE");
    o["hparams"] = t["hparams"];
    o["restarts"] = t.get_int("restarts", 0);
    int64_t batches = 0;
    for (auto& s : store_->Where("steps", "trial_id", Json(tid)))
      if (s.get_string("state", "") == "COMPLETED")
        batches = std::max(batches, s.get_int("prior_batches_processed", 0) + s.get_int("num_batches", 0));
    o["totalBatchesProcessed"] = batches;
    Json best, latest;
    for (auto& v : store_->Where("validations", "trial_id", Json(tid))) {
      if (v.get_string("state", "") != "COMPLETED") continue;
      Json vj = Json::object();
      vj["totalBatches"] = v.get_int("prior_batches_processed", 0);
      vj["metrics"] = v["metrics"]["validation_metrics"];
      vj["endTime"] = v["end_time"];
      try {
        double m = ValidationMetric(v["metrics"]["validation_metrics"], metric);
        vj["searcherMetric"] = m;
        if (best.is_null() || (smaller ? m < best["searcherMetric"].as_double() : m > best["searcherMetric"].as_double()))
          best = vj;
      } catch (const std::exception&) {
      }
      if (latest.is_null() || vj.get_int("totalBatches", 0) >= latest.get_int("totalBatches", 0)) latest = vj;
    }
    o["bestValidation"] = best;
    o["latestValidation"] = latest;
    Json bestck;
    int64_t best_step = -1;
    for (auto& c : store_->Where("checkpoints", "trial_id", Json(tid)))
      if (c.get_string("state", "") == "COMPLETED" && c.get_int("step_id", 0) > best_step) {
        best_step = c.get_int("step_id", 0);
        bestck = ToApi(c);
      }
    o["latestCheckpoint"] = bestck;
    return o;
  };

  // ------------------------------------------------------------------------------ auth/users
  http_.Route("POST", "/api/v1/auth/login", [=](const net::Request& r) {
    auto res = call(r, "POST", "/login", r.body);
    Json j;
    if (!unwrap(res, &j)) return relay_err(res);
    Json out = Json::object();
    out["token"] = j["token"];
    Json u = Json::object();
    u["username"] = j["username"];
    u["active"] = true;
    for (auto& row : store_->Where("users", "username", j["username"])) {
      u["id"] = row["id"];
      u["admin"] = row.get_bool("admin", false);
    }
    out["user"] = u;
    return JV(200, out);
  });
  http_.Route("GET", "/api/v1/auth/user", [=](const net::Request& r) {
    std::string name = UserForRequest(r);
    if (name.empty() && !cfg_.require_auth) name = "determined";
    for (auto& row : store_->Where("users", "username", Json(name))) {
      Json u = Json::object();
      for (const char* k : {"id", "username", "admin", "active"}) u[k] = row[k];
      if (row["agent_user_group"].is_object()) {
        Json g = Json::object();
        g["agentUid"] = row["agent_user_group"]["uid"];
        g["agentGid"] = row["agent_user_group"]["gid"];
        g["agentUser"] = row["agent_user_group"]["user"];
        g["agentGroup"] = row["agent_user_group"]["group"];
        u["agentUserGroup"] = g;
      }
      Json out = Json::object();
      out["user"] = u;
      return JV(200, out);
    }
    return ErrV(401, "not logged in");
  });
  http_.Route("POST", "/api/v1/auth/logout", [=](const net::Request& r) {
    auto res = call(r, "POST", "/logout");
    return res.status < 400 ? JV(200, Json::object()) : relay_err(res);
  });
  http_.Route("GET", "/api/v1/users", [=](const net::Request& r) {
    auto res = call(r, "GET", "/users");
    Json j;
    if (!unwrap(res, &j)) return relay_err(res);
    Json out = Json::object();
    out["users"] = j;
    return JV(200, out);
  });
  http_.Route("GET", "/api/v1/users/:username", [=](const net::Request& r) {
    for (auto& row : store_->Where("users", "username", Json(r.Param("username")))) {
      Json u = Json::object();
      for (const char* k : {"id", "username", "admin", "active"}) u[k] = row[k];
      if (row["agent_user_group"].is_object()) {
        Json g = Json::object();
        g["agentUid"] = row["agent_user_group"]["uid"];
        g["agentGid"] = row["agent_user_group"]["gid"];
        g["agentUser"] = row["agent_user_group"]["user"];
        g["agentGroup"] = row["agent_user_group"]["group"];
        u["agentUserGroup"] = g;
      }
      Json out = Json::object();
      out["user"] = u;
      return JV(200, out);
    }
    return ErrV(404, "user not found");
  });
  http_.Route("POST", "/api/v1/users", [=](const net::Request& r) {
    Json body = Json::parse(r.body.empty() ? "{}" : r.body);
    Json legacy = Json::object();
    legacy["username"] = body["user"].get_string("username", body.get_string("username", ""));
    legacy["admin"] = body["user"].get_bool("admin", false);
    legacy["password"] = body.get_string("password", "");
    auto res = call(r, "POST", "/users", legacy.dump());
    if (res.status >= 400) return relay_err(res);
    Json out = Json::object();
    for (auto& row : store_->Where("users", "username", legacy["username"])) {
      Json u = Json::object();
      for (const char* k : {"id", "username", "admin", "active"}) u[k] = row[k];
      out["user"] = u;
    }
    return JV(200, out);
  });
  http_.Route("POST", "/api/v1/users/:username/password", [=](const net::Request& r) {
    Json body = Json::parse(r.body.empty() ? "{}" : r.body);
    Json legacy = Json::object();
    legacy["password"] = body.is_string() ? body : Json(body.get_string("password", ""));
    auto res = call(r, "PATCH", "/users/" + net::UrlEncode(r.Param("username")), legacy.dump());
    return res.status < 400 ? JV(200, Json::object()) : relay_err(res);
  });

  // --------------------------------------------------------------------------------- master
  http_.Route("GET", "/api/v1/master", [=](const net::Request& r) {
    auto res = call(r, "GET", "/info");
    Json j;
    if (!unwrap(res, &j)) return relay_err(res);
    Json out = ToApi(j);
    out["telemetryEnabled"] = !cfg_.telemetry_file.empty();
    return JV(200, out);
  });
  http_.Route("GET", "/api/v1/master/config", [=](const net::Request&) {
    Json out = Json::object();
    out["config"] = cfg_.ToJson();
    return JV(200, out);
  });
  http_.Route("GET", "/api/v1/master/telemetry", [=](const net::Request&) {
    Json out = Json::object();
    out["enabled"] = !cfg_.telemetry_file.empty();
    out["segmentKey"] = "";
    return JV(200, out);
  });
  http_.Route("GET", "/api/v1/master/logs", [=](const net::Request& r) {
    int64_t offset = QInt(r, "offset", 0), limit = QInt(r, "limit", 0);
    bool follow = QBool(r, "follow");
    return Stream([=](const Writer& w) {
      int64_t after = offset;
      int64_t sent = 0;
      while (true) {
        Json batch = MasterLogTail(after, limit > 0 ? limit - sent : 1000);
        for (auto& e : batch.as_array()) {
          Json le = Json::object();
          Json entry = Json::object();
          entry["id"] = e["id"];
          entry["message"] = e.get_string("message", e.get_string("log", ""));
          le["logEntry"] = entry;
          if (!SendResult(w, le)) return;
          after = e["id"].as_int();
          ++sent;
        }
        if (limit > 0 && sent >= limit) return;
        if (!follow && batch.size() == 0) return;
        if (batch.size() == 0 && !StreamPause(w, 0.25)) return;
      }
    });
  });

  // --------------------------------------------------------------------------------- agents
  auto agents_api = [=](const net::Request& r) {
    auto res = call(r, "GET", "/agents");
    Json j;
    if (!unwrap(res, &j)) return Json::array();
    Json out = Json::array();
    for (auto& a : j.as_array()) {
      Json o = ToApi(a);
      Json slots = Json::object();
      if (a["slots"].is_array())
        for (auto& s : a["slots"].as_array()) slots[std::to_string(s.get_int("id", 0))] = ToApi(s);
      o["slots"] = slots;
      out.push_back(o);
    }
    return out;
  };
  http_.Route("GET", "/api/v1/agents", [=](const net::Request& r) {
    Json out = Json::object();
    Json agents = agents_api(r);
    std::string label = Q(r, "label");
    if (!label.empty()) {
      Json f = Json::array();
      for (auto& a : agents.as_array())
        if (a.get_string("label", "") == label) f.push_back(a);
      agents = f;
    }
    out["agents"] = agents;
    out["pagination"] = Pagination(0, 0, static_cast<int64_t>(agents.size()));
    return JV(200, out);
  });
  http_.Route("GET", "/api/v1/agents/:agent_id", [=](const net::Request& r) {
    Json all_agents = agents_api(r);
    for (auto& a : all_agents.as_array())
      if (a.get_string("id", "") == r.Param("agent_id")) {
        Json out = Json::object();
        out["agent"] = a;
        return JV(200, out);
      }
    return ErrV(404, "agent not found");
  });
  http_.Route("GET", "/api/v1/agents/:agent_id/slots", [=](const net::Request& r) {
    Json all_agents = agents_api(r);
    for (auto& a : all_agents.as_array())
      if (a.get_string("id", "") == r.Param("agent_id")) {
        Json slots = Json::array();
        for (auto& kv : a["slots"].as_object()) slots.push_back(kv.second);
        Json out = Json::object();
        out["slots"] = slots;
        return JV(200, out);
      }
    return ErrV(404, "agent not found");
  });
  http_.Route("GET", "/api/v1/agents/:agent_id/slots/:slot_id", [=](const net::Request& r) {
    Json all_agents = agents_api(r);
    for (auto& a : all_agents.as_array())
      if (a.get_string("id", "") == r.Param("agent_id") && a["slots"].has(r.Param("slot_id"))) {
        Json out = Json::object();
        out["slot"] = a["slots"][r.Param("slot_id")];
        return JV(200, out);
      }
    return ErrV(404, "slot not found");
  });
  for (const char* verb : {"enable", "disable"}) {
    std::string v = verb;
    http_.Route("POST", "/api/v1/agents/:agent_id/" + v, [=](const net::Request& r) {
      auto res = call(r, "POST", "/agents/" + r.Param("agent_id") + "/" + v);
      return res.status < 400 ? JV(200, Json::object()) : relay_err(res);
    });
    http_.Route("POST", "/api/v1/agents/:agent_id/slots/:slot_id/" + v, [=](const net::Request& r) {
      auto res = call(r, "POST", "/agents/" + r.Param("agent_id") + "/slots/" + r.Param("slot_id") + "/" + v);
      return res.status < 400 ? JV(200, Json::object()) : relay_err(res);
    });
  }

  // ---------------------------------------------------------------------------- experiments
  http_.Route("POST", "/api/v1/experiments", [=](const net::Request& r) {
    Json body = Json::parse(r.body.empty() ? "{}" : r.body);
    Json legacy = Json::object();
    legacy["config"] = body["config"];  // a YAML/JSON string or an object; the legacy handler parses both
    Json files = Json::array();
    for (auto& f : (body.has("modelDefinition") ? body["modelDefinition"] : body["model_definition"]).as_array()) {
      Json lf = Json::object();
      lf["path"] = f.get_string("path", "");
      lf["content"] = f.get_string("content", "");
      lf["type"] = f.get_string("type", "file");
      files.push_back(lf);
    }
    legacy["model_definition"] = files;
    legacy["validate_only"] = body.get_bool("validateOnly", body.get_bool("validate_only", false));
    if (body.has("parentId") || body.has("parent_id")) legacy["parent_id"] = body.has("parentId") ? body["parentId"] : body["parent_id"];
    legacy["activate"] = body.get_bool("activate", true);
    auto res = call(r, "POST", "/experiments", legacy.dump());
    Json j;
    if (!unwrap(res, &j)) return relay_err(res);
    Json out = Json::object();
    if (!j.has("id")) return JV(200, out);  // validate_only
    Json e;
    store_->Get("experiments", j["id"].as_int(), &e);
    out["experiment"] = exp_api(e);
    out["config"] = e["config"];
    return JV(200, out);
  });
  http_.Route("GET", "/api/v1/experiments", [=](const net::Request& r) {
    const std::string desc = Q(r, "description");
    auto states = QList(r, "states");
    auto users = QList(r, "users");
    auto labels = QList(r, "labels");
    const std::string archived = Q(r, "archived");
    const std::string sort_by = Q(r, "sort_by", "SORT_BY_ID");
    const bool desc_order = Q(r, "order_by", "ORDER_BY_ASC") == "ORDER_BY_DESC";
    int64_t offset = QInt(r, "offset", 0), limit = QInt(r, "limit", 0);
    std::vector<Json> rows;
    for (auto& e : store_->Scan("experiments")) {
      Json o = exp_api(e);
      if (!desc.empty() && o.get_string("description", "").find(desc) == std::string::npos) continue;
      if (!archived.empty() && o.get_bool("archived", false) != (archived == "true")) continue;
      if (!states.empty() && std::find(states.begin(), states.end(), o.get_string("state", "")) == states.end() &&
          std::find(states.begin(), states.end(), StripState(o.get_string("state", ""))) == states.end())
        continue;
      if (!users.empty() && std::find(users.begin(), users.end(), o.get_string("username", "")) == users.end()) continue;
      bool ok = true;
      for (auto& l : labels) {
        bool has = false;
        for (auto& x : o["labels"].as_array()) has = has || (x.is_string() && x.as_string() == l);
        ok = ok && has;
      }
      if (!ok) continue;
      rows.push_back(o);
    }
    auto key = [&](const Json& o) -> Json {
      if (sort_by == "SORT_BY_DESCRIPTION") return o["description"];
      if (sort_by == "SORT_BY_START_TIME") return o["startTime"];
      if (sort_by == "SORT_BY_END_TIME") return o["endTime"];
      if (sort_by == "SORT_BY_STATE") return o["state"];
      if (sort_by == "SORT_BY_NUM_TRIALS") return o["numTrials"];
      if (sort_by == "SORT_BY_PROGRESS") return o["progress"];
      if (sort_by == "SORT_BY_USER") return o["username"];
      return o["id"];
    };
    std::stable_sort(rows.begin(), rows.end(), [&](const Json& a, const Json& b) {
      Json ka = key(a), kb = key(b);
      bool lt = ka.is_number() && kb.is_number() ? ka.as_double() < kb.as_double() : ka.dump() < kb.dump();
      bool gt = ka.is_number() && kb.is_number() ? ka.as_double() > kb.as_double() : ka.dump() > kb.dump();
      return desc_order ? gt : lt;
    });
    Json out = Json::object();
    Json list = Json::array();
    int64_t total = static_cast<int64_t>(rows.size());
    for (int64_t i = std::min(offset, total); i < total && (limit <= 0 || i < offset + limit); ++i) list.push_back(rows[i]);
    out["experiments"] = list;
    out["pagination"] = Pagination(offset, limit, total);
    return JV(200, out);
  });
  http_.Route("GET", "/api/v1/experiment/labels", [=](const net::Request&) {
    std::map<std::string, int> counts;
    for (auto& e : store_->Scan("experiments")) {
      Json ls = e["labels"].is_array() ? e["labels"] : e["config"]["labels"];
      if (ls.is_array())
        for (auto& l : ls.as_array())
          if (l.is_string()) counts[l.as_string()]++;
    }
    std::vector<std::pair<std::string, int>> v(counts.begin(), counts.end());
    std::stable_sort(v.begin(), v.end(), [](const auto& a, const auto& b) { return a.second > b.second; });
    Json out = Json::object();
    Json labels = Json::array();
    for (auto& kv : v) labels.push_back(kv.first);
    out["labels"] = labels;
    return JV(200, out);
  });
  http_.Route("GET", "/api/v1/experiments/:experiment_id", [=](const net::Request& r) {
    Json e;
    if (!store_->Get("experiments", std::stoll(r.Param("experiment_id")), &e)) return ErrV(404, "experiment not found");
    Json out = Json::object();
    out["experiment"] = exp_api(e);
    out["config"] = e["config"];
    return JV(200, out);
  });
  http_.Route("GET", "/api/v1/experiments/:experiment_id/validation-history", [=](const net::Request& r) {
    int64_t id = std::stoll(r.Param("experiment_id"));
    Json e;
    if (!store_->Get("experiments", id, &e)) return ErrV(404, "experiment not found");
    const std::string metric = e["config"]["searcher"].get_string("metric", "");
    const bool smaller = e["config"]["searcher"].get_bool("smaller_is_better", true);
    std::vector<Json> vals;
    for (auto& t : store_->Where("trials", "experiment_id", Json(id)))
      for (auto& v : store_->Where("validations", "trial_id", t["id"]))
        if (v.get_string("state", "") == "COMPLETED") vals.push_back(v);
    std::stable_sort(vals.begin(), vals.end(), [](const Json& a, const Json& b) {
      return a.get_string("end_time", "") < b.get_string("end_time", "");
    });
    Json hist = Json::array();
    bool have = false;
    double best = 0;
    for (auto& v : vals) {
      double m;
      try {
        m = ValidationMetric(v["metrics"]["validation_metrics"], metric);
      } catch (const std::exception&) {
        continue;
      }
      if (have && !(smaller ? m < best : m > best)) continue;
      have = true;
      best = m;
      Json h = Json::object();
      h["trialId"] = v["trial_id"];
      h["endTime"] = v["end_time"];
      h["searcherMetric"] = m;
      hist.push_back(h);
    }
    Json out = Json::object();
    out["validationHistory"] = hist;
    return JV(200, out);
  });
  struct StateVerb {
    const char* verb;
    const char* state;
  };
  for (StateVerb sv : {StateVerb{"activate", "ACTIVE"}, StateVerb{"pause", "PAUSED"},
                       StateVerb{"cancel", "STOPPING_CANCELED"}}) {
    std::string st = sv.state;
    http_.Route("POST", std::string("/api/v1/experiments/:id/") + sv.verb, [=](const net::Request& r) {
      Json body = Json::object();
      body["state"] = st;
      auto res = call(r, "PATCH", "/experiments/" + r.Param("id"), body.dump());
      return res.status < 400 ? JV(200, Json::object()) : relay_err(res);
    });
  }
  http_.Route("POST", "/api/v1/experiments/:id/kill", [=](const net::Request& r) {
    auto res = call(r, "POST", "/experiments/" + r.Param("id") + "/kill");
    return res.status < 400 ? JV(200, Json::object()) : relay_err(res);
  });
  for (const char* verb : {"archive", "unarchive"}) {
    bool arch = std::string(verb) == "archive";
    http_.Route("POST", std::string("/api/v1/experiments/:id/") + verb, [=](const net::Request& r) {
      Json e;
      if (!store_->Get("experiments", std::stoll(r.Param("id")), &e)) return ErrV(404, "experiment not found");
      if (arch && !Terminal(e.get_string("state", ""))) return ErrV(409, "experiment is not in a terminal state");
      Json body = Json::object();
      body["archived"] = arch;
      auto res = call(r, "PATCH", "/experiments/" + r.Param("id"), body.dump());
      return res.status < 400 ? JV(200, Json::object()) : relay_err(res);
    });
  }
  http_.Route("PATCH", "/api/v1/experiments/:id", [=](const net::Request& r) {
    int64_t id = std::stoll(r.Param("id"));
    Json body = Json::parse(r.body.empty() ? "{}" : r.body);
    Json exp = body.has("experiment") ? body["experiment"] : body;
    Json patch = Json::object();
    for (const char* k : {"description", "labels", "notes"})
      if (exp.has(k)) patch[k] = exp[k];
    Json e;
    if (!store_->Get("experiments", id, &e)) return ErrV(404, "experiment not found");
    if (patch.size() > 0) store_->Update("experiments", id, patch);
    store_->Get("experiments", id, &e);
    Json out = Json::object();
    out["experiment"] = exp_api(e);
    return JV(200, out);
  });
  http_.Route("GET", "/api/v1/experiments/:id/checkpoints", [=](const net::Request& r) {
    auto res = call(r, "GET", "/experiments/" + r.Param("id") + "/checkpoints");
    Json j;
    if (!unwrap(res, &j)) return relay_err(res);
    auto states = QList(r, "states");
    Json list = Json::array();
    for (auto& c : j.as_array()) {
      Json o = ToApi(c);
      if (!states.empty() && std::find(states.begin(), states.end(), o.get_string("state", "")) == states.end()) continue;
      list.push_back(o);
    }
    int64_t offset = QInt(r, "offset", 0), limit = QInt(r, "limit", 0);
    Json page = Json::array();
    int64_t total = static_cast<int64_t>(list.size());
    for (int64_t i = std::min(offset, total); i < total && (limit <= 0 || i < offset + limit); ++i) page.push_back(list[static_cast<size_t>(i)]);
    Json out = Json::object();
    out["checkpoints"] = page;
    out["pagination"] = Pagination(offset, limit, total);
    return JV(200, out);
  });
  http_.Route("POST", "/api/v1/preview-hp-search", [=](const net::Request& r) {
    Json body = Json::parse(r.body.empty() ? "{}" : r.body);
    Json legacy = Json::object();
    legacy["config"] = body["config"];
    if (body.has("seed")) legacy["seed"] = body["seed"];
    auto res = call(r, "POST", "/searcher/preview", legacy.dump());
    Json j;
    if (!unwrap(res, &j)) return relay_err(res);
    Json sim = Json::object();
    Json results = Json::array();
    for (auto& kv : j["results"].as_object()) {
      Json one = Json::object();
      one["units"] = kv.first;
      one["count"] = kv.second;
      results.push_back(one);
    }
    sim["results"] = results;  // det-master extension: {units, count} per distinct sequence
    sim["trials"] = j["trials"];
    sim["config"] = j["config"];
    sim["seed"] = j["seed"];
    Json out = Json::object();
    out["simulation"] = sim;
    return JV(200, out);
  });
  http_.Route("GET", "/api/v1/experiments/:experiment_id/trials", [=](const net::Request& r) {
    int64_t id = std::stoll(r.Param("experiment_id"));
    Json e;
    if (!store_->Get("experiments", id, &e)) return ErrV(404, "experiment not found");
    auto states = QList(r, "states");
    std::vector<Json> rows;
    for (auto& t : store_->Where("trials", "experiment_id", Json(id))) {
      Json o = trial_api(t["id"].as_int());
      if (!states.empty() && std::find(states.begin(), states.end(), o.get_string("state", "")) == states.end()) continue;
      rows.push_back(o);
    }
    std::stable_sort(rows.begin(), rows.end(), [](const Json& a, const Json& b) { return a["id"].as_int() < b["id"].as_int(); });
    if (Q(r, "order_by") == "ORDER_BY_DESC") std::reverse(rows.begin(), rows.end());
    int64_t offset = QInt(r, "offset", 0), limit = QInt(r, "limit", 0);
    Json list = Json::array();
    int64_t total = static_cast<int64_t>(rows.size());
    for (int64_t i = std::min(offset, total); i < total && (limit <= 0 || i < offset + limit); ++i) list.push_back(rows[i]);
    Json out = Json::object();
    out["trials"] = list;
    out["pagination"] = Pagination(offset, limit, total);
    return JV(200, out);
  });

  // --------------------------------------------------------------------------------- trials
  http_.Route("GET", "/api/v1/trials/:trial_id", [=](const net::Request& r) {
    int64_t tid = std::stoll(r.Param("trial_id"));
    Json t = trial_api(tid);
    if (t.is_null()) return ErrV(404, "trial not found");
    Json workloads = Json::array();
    for (auto& s : store_->Where("steps", "trial_id", Json(tid))) {
      Json w = Json::object();
      w["training"] = ToApi(s);
      workloads.push_back(w);
    }
    for (auto& v : store_->Where("validations", "trial_id", Json(tid))) {
      Json w = Json::object();
      w["validation"] = ToApi(v);
      workloads.push_back(w);
    }
    for (auto& c : store_->Where("checkpoints", "trial_id", Json(tid))) {
      Json w = Json::object();
      w["checkpoint"] = ToApi(c);
      workloads.push_back(w);
    }
    Json out = Json::object();
    out["trial"] = t;
    out["workloads"] = workloads;
    return JV(200, out);
  });
  http_.Route("POST", "/api/v1/trials/:id/kill", [=](const net::Request& r) {
    auto res = call(r, "POST", "/trials/" + r.Param("id") + "/kill");
    return res.status < 400 ? JV(200, Json::object()) : relay_err(res);
  });
  http_.Route("GET", "/api/v1/trials/:id/checkpoints", [=](const net::Request& r) {
    int64_t tid = std::stoll(r.Param("id"));
    auto states = QList(r, "states");
    Json list = Json::array();
    for (auto& c : store_->Where("checkpoints", "trial_id", Json(tid))) {
      Json o = ToApi(c);
      if (!states.empty() && std::find(states.begin(), states.end(), o.get_string("state", "")) == states.end()) continue;
      list.push_back(o);
    }
    Json out = Json::object();
    out["checkpoints"] = list;
    out["pagination"] = Pagination(0, 0, static_cast<int64_t>(list.size()));
    return JV(200, out);
  });
  // TrialLogs: reference api_trials.go:51 -- offset (negative: from the end), limit, follow
  // until the trial is terminal and drained, filters on container/rank/stdtype.
  http_.Route("GET", "/api/v1/trials/:trial_id/logs", [=](const net::Request& r) {
    int64_t tid = std::stoll(r.Param("trial_id"));
    Json t;
    if (!store_->Get("trials", tid, &t)) return ErrV(404, "trial not found");
    int64_t offset = QInt(r, "offset", 0), limit = QInt(r, "limit", 0);
    if (limit < 0) return ErrV(400, "limit must be >= 0");
    const bool follow = QBool(r, "follow");
    if (follow && limit > 0) return ErrV(400, "follow and limit are mutually exclusive");
    auto ranks = QList(r, "rank_ids"), cids = QList(r, "container_ids"), stdtypes = QList(r, "stdtypes");
    auto pred = [=](const Json& l) {
      if (!ranks.empty() && std::find(ranks.begin(), ranks.end(), std::to_string(l.get_int("rank_id", 0))) == ranks.end())
        return false;
      if (!cids.empty() && std::find(cids.begin(), cids.end(), l.get_string("container_id", "")) == cids.end()) return false;
      if (!stdtypes.empty() && std::find(stdtypes.begin(), stdtypes.end(), l.get_string("stdtype", "")) == stdtypes.end())
        return false;
      return true;
    };
    const std::string stream = "trial-" + std::to_string(tid);
    return Stream([=](const Writer& w) {
      int64_t after = 0;
      if (offset < 0) {  // the last -offset matching lines
        auto tail = logs_->Read(stream, 0, -offset, pred, true);
        if (!tail.empty()) after = tail.front()["id"].as_int() - 1;
      } else {
        after = offset;
      }
      int64_t sent = 0;
      int idle_after_terminal = 0;
      while (true) {
        int64_t want = limit > 0 ? limit - sent : 1000;
        auto rows = logs_->Read(stream, after, want, pred, false);
        for (auto& l : rows) {
          Json o = Json::object();
          o["id"] = l["id"].as_int() - 1;  // the WebUI expects 0-indexed ids
          o["trialId"] = tid;
          o["message"] = l.get_string("message", "");
          o["timestamp"] = l["timestamp"];
          o["containerId"] = l.get_string("container_id", "");
          o["rankId"] = l.get_int("rank_id", 0);
          o["stdtype"] = l.get_string("stdtype", "");
          o["level"] = "LOG_LEVEL_INFO";
          if (!SendResult(w, o)) return;
          after = l["id"].as_int();
          ++sent;
        }
        if (limit > 0 && sent >= limit) return;
        if (!follow) {
          if (rows.empty()) return;
          continue;
        }
        if (!rows.empty()) continue;
        Json cur;
        if (!store_->Get("trials", tid, &cur)) return;
        if (Terminal(cur.get_string("state", "")) && ++idle_after_terminal >= 4) return;  // ~1 s drain
        if (!StreamPause(w, 0.25)) return;
      }
    });
  });
  http_.Route("GET", "/api/v1/trials/:trial_id/logs/fields", [=](const net::Request& r) {
    int64_t tid = std::stoll(r.Param("trial_id"));
    const bool follow = QBool(r, "follow");
    const std::string stream = "trial-" + std::to_string(tid);
    return Stream([=](const Writer& w) {
      std::set<std::string> cids, ranks, stdtypes;
      int64_t after = 0;
      while (true) {
        auto rows = logs_->Read(stream, after, 100000, nullptr, false);
        bool changed = false;
        for (auto& l : rows) {
          changed |= cids.insert(l.get_string("container_id", "")).second;
          changed |= ranks.insert(std::to_string(l.get_int("rank_id", 0))).second;
          changed |= stdtypes.insert(l.get_string("stdtype", "")).second;
          after = l["id"].as_int();
        }
        if (changed || (!follow)) {
          Json o = Json::object();
          Json a = Json::array(), b = Json::array(), c = Json::array();
          for (auto& x : cids) a.push_back(x);
          for (auto& x : ranks) b.push_back(std::stoll(x));
          for (auto& x : stdtypes) c.push_back(x);
          o["containerIds"] = a;
          o["rankIds"] = b;
          o["stdtypes"] = c;
          o["sources"] = Json(Json::Array{Json("SOURCE_TRIAL")});
          o["levels"] = Json(Json::Array{Json("LOG_LEVEL_INFO")});
          if (!SendResult(w, o)) return;
        }
        if (!follow) return;
        Json cur;
        if (!store_->Get("trials", tid, &cur) || Terminal(cur.get_string("state", ""))) return;
        if (!StreamPause(w, 1.0)) return;
      }
    });
  });

  // ------------------------------------------------------------------------ metric streams
  // Training points: completed steps (batches = prior + num); validation points: completed
  // validations (batches = prior).  Shared by MetricNames/MetricBatches/TrialsSnapshot/TrialsSample.
  auto series = [this](int64_t tid, const std::string& type, const std::string& name) {
    std::vector<SeriesPoint> out;
    if (type == "training") {
      for (auto& s : store_->Where("steps", "trial_id", Json(tid))) {
        if (s.get_string("state", "") != "COMPLETED") continue;
        const Json& m = s["metrics"]["avg_metrics"];
        if (m.is_object() && m[name].is_number())
          out.push_back({s.get_int("prior_batches_processed", 0) + s.get_int("num_batches", 0), m[name].as_double()});
      }
    } else {
      for (auto& v : store_->Where("validations", "trial_id", Json(tid))) {
        if (v.get_string("state", "") != "COMPLETED") continue;
        const Json& m = v["metrics"]["validation_metrics"];
        if (m.is_object() && m[name].is_number()) out.push_back({v.get_int("prior_batches_processed", 0), m[name].as_double()});
      }
    }
    std::sort(out.begin(), out.end(), [](const SeriesPoint& a, const SeriesPoint& b) { return a.batches < b.batches; });
    return out;
  };
  auto exp_state = [this](int64_t id) {
    Json e;
    return store_->Get("experiments", id, &e) ? e.get_string("state", "DELETED") : std::string("DELETED");
  };
  http_.Route("GET", "/api/v1/experiments/:experiment_id/metrics-stream/metric-names", [=](const net::Request& r) {
    int64_t id = std::stoll(r.Param("experiment_id"));
    Json e;
    if (!store_->Get("experiments", id, &e)) return ErrV(404, "experiment not found");
    double period = PeriodSeconds(r, 30.0);
    const std::string searcher_metric = e["config"]["searcher"].get_string("metric", "");
    return Stream([=](const Writer& w) {
      std::set<std::string> seen_t, seen_v;
      while (true) {
        Json out = Json::object();
        out["searcherMetric"] = searcher_metric;
        Json tr = Json::array(), va = Json::array();
        for (auto& t : store_->Where("trials", "experiment_id", Json(id))) {
          for (auto& s : store_->Where("steps", "trial_id", t["id"]))
            if (s["metrics"]["avg_metrics"].is_object())
              for (auto& kv : s["metrics"]["avg_metrics"].as_object())
                if (seen_t.insert(kv.first).second) tr.push_back(kv.first);
          for (auto& v : store_->Where("validations", "trial_id", t["id"]))
            if (v["metrics"]["validation_metrics"].is_object())
              for (auto& kv : v["metrics"]["validation_metrics"].as_object())
                if (seen_v.insert(kv.first).second) va.push_back(kv.first);
        }
        out["trainingMetrics"] = tr;
        out["validationMetrics"] = va;
        if (!SendResult(w, out)) return;
        if (Terminal(exp_state(id))) return;
        if (!StreamPause(w, period)) return;
      }
    });
  });
  http_.Route("GET", "/api/v1/experiments/:experiment_id/metrics-stream/batches", [=](const net::Request& r) {
    int64_t id = std::stoll(r.Param("experiment_id"));
    Json e;
    if (!store_->Get("experiments", id, &e)) return ErrV(404, "experiment not found");
    const std::string name = Q(r, "metric_name");
    if (name.empty()) return ErrV(400, "must specify a metric name");
    const std::string type = MetricTypeOf(r);
    double period = PeriodSeconds(r, 30.0);
    return Stream([=](const Writer& w) {
      std::set<int64_t> seen;
      while (true) {
        std::vector<int64_t> fresh;
        for (auto& t : store_->Where("trials", "experiment_id", Json(id)))
          for (auto& p : series(t["id"].as_int(), type, name))
            if (seen.insert(p.batches).second) fresh.push_back(p.batches);
        std::sort(fresh.begin(), fresh.end());
        Json out = Json::object();
        Json b = Json::array();
        for (int64_t x : fresh) b.push_back(x);
        out["batches"] = b;
        if (!SendResult(w, out)) return;
        if (Terminal(exp_state(id))) return;
        if (!StreamPause(w, period)) return;
      }
    });
  });
  http_.Route("GET", "/api/v1/experiments/:experiment_id/metrics-stream/trials-snapshot", [=](const net::Request& r) {
    int64_t id = std::stoll(r.Param("experiment_id"));
    Json e;
    if (!store_->Get("experiments", id, &e)) return ErrV(404, "experiment not found");
    const std::string name = Q(r, "metric_name");
    if (name.empty()) return ErrV(400, "must specify a metric name");
    const std::string type = MetricTypeOf(r);
    const int64_t at = QInt(r, "batches_processed", 0);
    double period = PeriodSeconds(r, 30.0);
    return Stream([=](const Writer& w) {
      std::set<int64_t> sent;
      while (true) {
        Json trials = Json::array();
        for (auto& t : store_->Where("trials", "experiment_id", Json(id))) {
          int64_t tid = t["id"].as_int();
          if (sent.count(tid)) continue;
          for (auto& p : series(tid, type, name))
            if (p.batches == at) {
              Json o = Json::object();
              o["trialId"] = tid;
              o["hparams"] = t["hparams"];
              o["metric"] = p.value;
              trials.push_back(o);
              sent.insert(tid);
              break;
            }
        }
        Json out = Json::object();
        out["trials"] = trials;
        if (!SendResult(w, out)) return;
        if (Terminal(exp_state(id))) return;
        if (!StreamPause(w, period)) return;
      }
    });
  });
  // TrialsSample (api_experiment.go:839): top trials by training length (adaptive/ASHA/SHA
  // searchers) or by best metric (random/grid), LTTB-downsampled first sight, then only new
  // points; promoted/demoted trial ids when the top set changes.
  http_.Route("GET", "/api/v1/experiments/:experiment_id/metrics-stream/trials-sample", [=](const net::Request& r) {
    int64_t id = std::stoll(r.Param("experiment_id"));
    Json e;
    if (!store_->Get("experiments", id, &e)) return ErrV(404, "experiment not found");
    const std::string name = Q(r, "metric_name");
    const std::string type = MetricTypeOf(r);
    if (name.empty()) return ErrV(400, "must specify a metric name");
    const std::string searcher = e["config"]["searcher"].get_string("name", "");
    if (searcher == "single") return ErrV(400, "single-trial experiments are not supported for trial sampling");
    if (searcher == "pbt") return ErrV(400, "population-based training not supported for trial sampling");
    const bool by_metric = searcher == "random" || searcher == "grid";
    const std::string smetric = e["config"]["searcher"].get_string("metric", "");
    const bool smaller = e["config"]["searcher"].get_bool("smaller_is_better", true);
    const int64_t max_trials = QInt(r, "max_trials", 25) > 0 ? QInt(r, "max_trials", 25) : 25;
    const int64_t max_points = QInt(r, "max_datapoints", 1000) > 0 ? QInt(r, "max_datapoints", 1000) : 1000;
    const int64_t start_b = QInt(r, "start_batches", 0);
    const int64_t end_b = QInt(r, "end_batches", 0) > 0 ? QInt(r, "end_batches", 0) : INT64_MAX;
    double period = PeriodSeconds(r, 30.0);
    return Stream([=](const Writer& w) {
      std::map<int64_t, int64_t> cursor;  // trial -> last batches sent
      std::set<int64_t> current;
      while (true) {
        // rank trials
        std::vector<std::pair<double, int64_t>> ranked;
        for (auto& t : store_->Where("trials", "experiment_id", Json(id))) {
          int64_t tid = t["id"].as_int();
          double key;
          if (by_metric) {
            bool have = false;
            double best = 0;
            for (auto& p : series(tid, "validation", smetric))
              if (!have || (smaller ? p.value < best : p.value > best)) {
                best = p.value;
                have = true;
              }
            if (!have) continue;
            key = smaller ? best : -best;
          } else {
            int64_t len = 0;
            for (auto& s : store_->Where("steps", "trial_id", Json(tid)))
              if (s.get_string("state", "") == "COMPLETED")
                len = std::max(len, s.get_int("prior_batches_processed", 0) + s.get_int("num_batches", 0));
            key = -static_cast<double>(len);
          }
          ranked.push_back({key, tid});
        }
        std::stable_sort(ranked.begin(), ranked.end());
        if (static_cast<int64_t>(ranked.size()) > max_trials) ranked.resize(static_cast<size_t>(max_trials));
        Json trials = Json::array(), promoted = Json::array(), demoted = Json::array();
        std::set<int64_t> now;
        for (auto& kv : ranked) {
          int64_t tid = kv.second;
          now.insert(tid);
          Json tr = Json::object();
          tr["trialId"] = tid;
          bool fresh = !current.count(tid);
          if (fresh) {
            Json t;
            store_->Get("trials", tid, &t);
            tr["hparams"] = t["hparams"];
            promoted.push_back(tid);
            current.insert(tid);
          }
          std::vector<Point> pts;
          int64_t last = cursor.count(tid) ? cursor[tid] : -1;
          for (auto& p : series(tid, type, name))
            if (p.batches >= start_b && p.batches <= end_b && p.batches > last)
              pts.push_back({static_cast<double>(p.batches), p.value});
          if (fresh) pts = Downsample(pts, static_cast<size_t>(max_points));
          Json data = Json::array();
          for (auto& p : pts) {
            Json d = Json::object();
            d["batches"] = static_cast<int64_t>(p.x);
            d["value"] = p.y;
            data.push_back(d);
            cursor[tid] = std::max(cursor[tid], static_cast<int64_t>(p.x));
          }
          tr["data"] = data;
          trials.push_back(tr);
        }
        for (auto it = current.begin(); it != current.end();) {
          if (!now.count(*it)) {
            demoted.push_back(*it);
            cursor.erase(*it);
            it = current.erase(it);
          } else {
            ++it;
          }
        }
        Json out = Json::object();
        out["trials"] = trials;
        out["promotedTrials"] = promoted;
        out["demotedTrials"] = demoted;
        if (!SendResult(w, out)) return;
        if (Terminal(exp_state(id))) return;
        if (!StreamPause(w, period)) return;
      }
    });
  });

  // ------------------------------------------------------------------------------ templates
  http_.Route("GET", "/api/v1/templates", [=](const net::Request& r) {
    auto res = call(r, "GET", "/templates");
    Json j;
    if (!unwrap(res, &j)) return relay_err(res);
    Json out = Json::object();
    out["templates"] = j;
    out["pagination"] = Pagination(0, 0, static_cast<int64_t>(j.size()));
    return JV(200, out);
  });
  http_.Route("GET", "/api/v1/templates/:template_name", [=](const net::Request& r) {
    auto res = call(r, "GET", "/templates/" + net::UrlEncode(r.Param("template_name")));
    Json j;
    if (!unwrap(res, &j)) return relay_err(res);
    Json out = Json::object();
    out["template"] = j;
    return JV(200, out);
  });
  http_.Route("PUT", "/api/v1/templates/:template_name", [=](const net::Request& r) {
    Json body = Json::parse(r.body.empty() ? "{}" : r.body);
    Json cfg = body.has("template") ? body["template"]["config"] : body["config"];
    Json legacy = Json::object();
    legacy["config"] = cfg;
    auto res = call(r, "PUT", "/templates/" + net::UrlEncode(r.Param("template_name")), legacy.dump());
    Json j;
    if (!unwrap(res, &j)) return relay_err(res);
    Json out = Json::object();
    out["template"] = j;
    return JV(200, out);
  });
  http_.Route("DELETE", "/api/v1/templates/:template_name", [=](const net::Request& r) {
    auto res = call(r, "DELETE", "/templates/" + net::UrlEncode(r.Param("template_name")));
    return res.status < 400 ? JV(200, Json::object()) : relay_err(res);
  });

  // ------------------------------------------------------------------ models / checkpoints
  http_.Route("GET", "/api/v1/models", [=](const net::Request& r) {
    auto res = call(r, "GET", "/models");
    Json j;
    if (!unwrap(res, &j)) return relay_err(res);
    const std::string name = Q(r, "name"), desc = Q(r, "description");
    Json list = Json::array();
    for (auto& m : j.as_array()) {
      if (!name.empty() && m.get_string("name", "").find(name) == std::string::npos) continue;
      if (!desc.empty() && m.get_string("description", "").find(desc) == std::string::npos) continue;
      list.push_back(ToApi(m));
    }
    Json out = Json::object();
    out["models"] = list;
    out["pagination"] = Pagination(0, 0, static_cast<int64_t>(list.size()));
    return JV(200, out);
  });
  http_.Route("GET", "/api/v1/models/:model_name", [=](const net::Request& r) {
    auto res = call(r, "GET", "/models/" + net::UrlEncode(r.Param("model_name")));
    Json j;
    if (!unwrap(res, &j)) return relay_err(res);
    Json out = Json::object();
    out["model"] = ToApi(j);
    return JV(200, out);
  });
  http_.Route("POST", "/api/v1/models/:model_name", [=](const net::Request& r) {
    Json body = Json::parse(r.body.empty() ? "{}" : r.body);
    Json m = body.has("model") ? body["model"] : body;
    auto res = call(r, "POST", "/models/" + net::UrlEncode(r.Param("model_name")), FromApi(m).dump());
    Json j;
    if (!unwrap(res, &j)) return relay_err(res);
    Json out = Json::object();
    out["model"] = ToApi(j);
    return JV(200, out);
  });
  http_.Route("PATCH", "/api/v1/models/:model_name", [=](const net::Request& r) {
    Json body = Json::parse(r.body.empty() ? "{}" : r.body);
    Json m = body.has("model") ? body["model"] : body;
    for (auto& row : store_->Where("models", "name", Json(r.Param("model_name")))) {
      Json patch = Json::object();
      if (m.has("description")) patch["description"] = m["description"];
      if (m.has("metadata")) patch["metadata"] = m["metadata"];
      patch["last_updated_time"] = NowRFC3339();
      store_->Update("models", row["id"].as_int(), patch);
      Json cur;
      store_->Get("models", row["id"].as_int(), &cur);
      Json out = Json::object();
      out["model"] = ToApi(cur);
      return JV(200, out);
    }
    return ErrV(404, "model not found");
  });
  http_.Route("GET", "/api/v1/models/:model_name/versions", [=](const net::Request& r) {
    auto mres = call(r, "GET", "/models/" + net::UrlEncode(r.Param("model_name")));
    Json mj;
    if (!unwrap(mres, &mj)) return relay_err(mres);
    Json versions = Json::array();
    for (auto& v : mj["versions"].as_array()) {
      Json o = ToApi(v);
      auto cres = call(r, "GET", "/checkpoints/" + v.get_string("checkpoint_uuid", ""));
      Json cj;
      if (unwrap(cres, &cj)) o["checkpoint"] = ToApi(cj);
      versions.push_back(o);
    }
    mj.as_object().erase("versions");
    Json out = Json::object();
    out["model"] = ToApi(mj);
    out["modelVersions"] = versions;
    return JV(200, out);
  });
  http_.Route("GET", "/api/v1/models/:model_name/versions/:model_version", [=](const net::Request& r) {
    for (auto& v : store_->Where("model_versions", "model_name", Json(r.Param("model_name"))))
      if (std::to_string(v.get_int("version", 0)) == r.Param("model_version")) {
        Json o = ToApi(v);
        auto cres = call(r, "GET", "/checkpoints/" + v.get_string("checkpoint_uuid", ""));
        Json cj;
        if (unwrap(cres, &cj)) o["checkpoint"] = ToApi(cj);
        Json out = Json::object();
        out["modelVersion"] = o;
        return JV(200, out);
      }
    return ErrV(404, "model version not found");
  });
  http_.Route("POST", "/api/v1/models/:model_name/versions", [=](const net::Request& r) {
    Json body = Json::parse(r.body.empty() ? "{}" : r.body);
    Json legacy = Json::object();
    legacy["checkpoint_uuid"] = body.get_string("checkpointUuid", body.get_string("checkpoint_uuid", ""));
    auto res = call(r, "POST", "/models/" + net::UrlEncode(r.Param("model_name")) + "/versions", legacy.dump());
    Json j;
    if (!unwrap(res, &j)) return relay_err(res);
    Json out = Json::object();
    out["modelVersion"] = ToApi(j);
    return JV(200, out);
  });
  http_.Route("GET", "/api/v1/checkpoints/:checkpoint_uuid", [=](const net::Request& r) {
    auto res = call(r, "GET", "/checkpoints/" + r.Param("checkpoint_uuid"));
    Json j;
    if (!unwrap(res, &j)) return relay_err(res);
    Json out = Json::object();
    out["checkpoint"] = ToApi(j);
    return JV(200, out);
  });
  http_.Route("POST", "/api/v1/checkpoints/:checkpoint_uuid/metadata", [=](const net::Request& r) {
    Json body = Json::parse(r.body.empty() ? "{}" : r.body);
    Json md = body["checkpoint"]["metadata"];
    for (auto& c : store_->Where("checkpoints", "uuid", Json(r.Param("checkpoint_uuid")))) {
      Json patch = Json::object();
      patch["metadata"] = md.is_object() ? md : Json::object();
      store_->Update("checkpoints", c["id"].as_int(), patch);
      Json out = Json::object();
      out["checkpoint"] = ToApi(c);
      out["checkpoint"]["metadata"] = patch["metadata"];
      return JV(200, out);
    }
    return ErrV(404, "checkpoint not found");
  });

  // ------------------------------------------------- commands / notebooks / shells / tensorboards
  struct TaskKind {
    const char* plural;  // URL collection
    const char* type;    // commands.type
    const char* one;     // response key for a single task
  };
  for (TaskKind k : {TaskKind{"commands", "command", "command"}, TaskKind{"notebooks", "notebook", "notebook"},
                     TaskKind{"shells", "shell", "shell"}, TaskKind{"tensorboards", "tensorboard", "tensorboard"}}) {
    const std::string plural = k.plural, type = k.type, one = k.one;
    const std::string id_param = std::string(k.one) + "_id";
    auto task_api = [=](const Json& c) {
      Json o = Json::object();
      o["id"] = std::to_string(c["id"].as_int());
      o["description"] = c.get_string("description", "");
      o["state"] = "STATE_" + c.get_string("state", "PENDING");
      o["container"] = Json::object();
      o["container"]["state"] = "STATE_" + c.get_string("state", "PENDING");
      o["username"] = c.get_string("owner", "determined");
      o["startTime"] = c["start_time"];
      o["exitStatus"] = c["exit_code"];
      o["serviceAddress"] = c.get_string("service_address", "").empty() ? Json() : Json("/proxy/cmd-" + std::to_string(c["id"].as_int()) + "/");
      o["config"] = c["config"];
      return o;
    };
    http_.Route("GET", "/api/v1/" + plural, [=](const net::Request& r) {
      auto res = call(r, "GET", "/commands?type=" + type);
      Json j;
      if (!unwrap(res, &j)) return relay_err(res);
      Json list = Json::array();
      for (auto& c : j.as_array()) list.push_back(task_api(c));
      Json out = Json::object();
      out[plural] = list;
      return JV(200, out);
    });
    http_.Route("GET", "/api/v1/" + plural + "/:" + id_param, [=](const net::Request& r) {
      auto res = call(r, "GET", "/commands/" + r.Param(id_param));
      Json j;
      if (!unwrap(res, &j)) return relay_err(res);
      if (j.get_string("type", "command") != type) return ErrV(404, one + " not found");
      Json out = Json::object();
      out[one] = task_api(j);
      out["config"] = j["config"];
      return JV(200, out);
    });
    http_.Route("POST", "/api/v1/" + plural + "/:" + id_param + "/kill", [=](const net::Request& r) {
      auto res = call(r, "POST", "/commands/" + r.Param(id_param) + "/kill");
      Json c;
      store_->Get("commands", std::stoll(r.Param(id_param)), &c);
      Json out = Json::object();
      out[one] = task_api(c);
      return res.status < 400 || res.status == 409 ? JV(200, out) : relay_err(res);
    });
    http_.Route("POST", "/api/v1/" + plural, [=](const net::Request& r) {
      Json body = Json::parse(r.body.empty() ? "{}" : r.body);
      Json cfg = body["config"].is_object() ? body["config"] : Json::object();
      cfg["type"] = type;
      if (!cfg["entrypoint"].is_array() || cfg["entrypoint"].size() == 0) {
        // notebooks / shells / tensorboards run the framework's own task servers
        const std::string mod = type == "notebook" ? "determined_1_amd.exec.notebook"
                                : type == "shell"  ? "determined_1_amd.exec.shell"
                                                   : "determined_1_amd.tensorboard.serve";
        if (type == "command") return ErrV(400, "command config needs entrypoint: [argv...]");
        cfg["entrypoint"] = Json(Json::Array{Json("python3"), Json("-m"), Json(mod)});
      }
      Json legacy = Json::object();
      legacy["config"] = cfg;
      legacy["context"] = body.has("files") ? body["files"] : Json::array();
      if (body["secretEnvironment"].is_array()) legacy["secret_environment"] = body["secretEnvironment"];
      auto res = call(r, "POST", "/commands", legacy.dump());
      Json j;
      if (!unwrap(res, &j)) return relay_err(res);
      Json c;
      store_->Get("commands", j["id"].as_int(), &c);
      Json out = Json::object();
      out[one] = task_api(c);
      out["config"] = c["config"];
      return JV(200, out);
    });
    if (type == "notebook") {
      http_.Route("GET", "/api/v1/notebooks/:notebook_id/logs", [=](const net::Request& r) {
        const std::string id = r.Param("notebook_id");
        const bool follow = QBool(r, "follow");
        int64_t offset = QInt(r, "offset", 0);
        return Stream([=](const Writer& w) {
          int64_t after = offset;
          while (true) {
            auto rows = logs_->Read("task-cmd-" + id, after, 1000, nullptr, false);
            for (auto& l : rows) {
              Json le = Json::object();
              Json entry = Json::object();
              entry["id"] = l["id"];
              entry["message"] = l.get_string("message", "");
              le["logEntry"] = entry;
              if (!SendResult(w, le)) return;
              after = l["id"].as_int();
            }
            if (!rows.empty()) continue;
            Json c;
            if (!follow || !store_->Get("commands", std::stoll(id), &c) || c.get_string("state", "") == "TERMINATED") return;
            if (!StreamPause(w, 0.25)) return;
          }
        });
      });
    }
  }
}

}  // namespace master
}  // namespace detcore
