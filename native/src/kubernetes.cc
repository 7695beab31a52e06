// Kubernetes resource manager: virtual agents backed by pods.  See detcore/kubernetes.h.
#include "detcore/kubernetes.h"

#include <sys/socket.h>
#include <sys/time.h>
#include <unistd.h>

#include <algorithm>
#include <cctype>
#include <chrono>
#include <cstring>
#include <set>
#include <sstream>

#include "detcore/master.h"
#include "detcore/net.h"

namespace detcore {
namespace master {

namespace {

std::string DnsName(std::string s) {
  std::string out;
  for (char c : s) {
    char l = static_cast<char>(std::tolower(static_cast<unsigned char>(c)));
    out.push_back(std::isalnum(static_cast<unsigned char>(l)) || l == '-' ? l : '-');
  }
  while (!out.empty() && out.back() == '-') out.pop_back();
  if (out.size() > 63) out = out.substr(0, 63);
  while (!out.empty() && out.back() == '-') out.pop_back();
  return out;
}

// Streaming GET (pod log follow): calls on_line per line until EOF, stop, or on_line false.
void StreamLines(const std::string& host, int port, const std::string& path, const std::atomic<bool>& stop,
                 const std::function<bool(const std::string&)>& on_line) {
  std::string err;
  int fd = net::ConnectTcp(host, port, 5000, &err);
  if (fd < 0) return;
  timeval tv{1, 0};
  setsockopt(fd, SOL_SOCKET, SO_RCVTIMEO, &tv, sizeof(tv));
  std::string req = "GET " + path + " HTTP/1.1\r\nHost: " + host + "\r\nConnection: close\r\n\r\n";
  if (send(fd, req.data(), req.size(), MSG_NOSIGNAL) < 0) {
    close(fd);
    return;
  }
  std::string buf, body, line;
  bool headers_done = false, chunked = false, ok = true;
  char tmp[8192];
  auto emit = [&](const std::string& data) {
    for (char c : data) {
      if (c == '\n') {
        if (!line.empty() && line.back() == '\r') line.pop_back();
        if (!on_line(line)) ok = false;
        line.clear();
      } else {
        line.push_back(c);
      }
    }
  };
  while (ok && !stop.load()) {
    ssize_t n = recv(fd, tmp, sizeof(tmp), 0);
    if (n < 0 && (errno == EAGAIN || errno == EWOULDBLOCK || errno == EINTR)) continue;
    if (n <= 0) break;
    buf.append(tmp, static_cast<size_t>(n));
    if (!headers_done) {
      auto he = buf.find("\r\n\r\n");
      if (he == std::string::npos) continue;
      std::string head = buf.substr(0, he);
      for (auto& c : head) c = static_cast<char>(std::tolower(static_cast<unsigned char>(c)));
      chunked = head.find("transfer-encoding: chunked") != std::string::npos;
      if (head.rfind("http/1.1 200", 0) != 0 && head.rfind("http/1.0 200", 0) != 0) break;
      buf.erase(0, he + 4);
      headers_done = true;
    }
    if (!chunked) {
      emit(buf);
      buf.clear();
      continue;
    }
    while (true) {  // decode as many complete chunks as buffered
      auto le = buf.find("\r\n");
      if (le == std::string::npos) break;
      size_t len = std::strtoul(buf.substr(0, le).c_str(), nullptr, 16);
      if (len == 0) {
        ok = false;
        break;
      }
      if (buf.size() < le + 2 + len + 2) break;
      emit(buf.substr(le + 2, len));
      buf.erase(0, le + 2 + len + 2);
    }
  }
  if (!line.empty()) on_line(line);
  close(fd);
}

}  // namespace

KubeConfig KubeConfig::FromJson(const Json& j) {
  KubeConfig c;
  std::string api = j.get_string("api_server", "127.0.0.1:8001");
  if (api.rfind("http://", 0) == 0) api = api.substr(7);
  auto colon = api.rfind(':');
  c.host = colon == std::string::npos ? api : api.substr(0, colon);
  c.port = colon == std::string::npos ? 80 : std::stoi(api.substr(colon + 1));
  c.ns = j.get_string("namespace", c.ns);
  c.max_slots_per_pod = static_cast<int>(j.get_int("max_slots_per_pod", c.max_slots_per_pod));
  c.slot_type = j.get_string("slot_type", c.slot_type);
  c.slot_resource = j.get_string("slot_resource", c.slot_resource);
  c.cpu_slots_per_node = static_cast<int>(j.get_int("cpu_slots_per_node", c.cpu_slots_per_node));
  c.image = j.get_string("image", c.image);
  c.python = j.get_string("python", c.python);
  c.pool = j.get_string("resource_pool", c.pool);
  c.master_host = j.get_string("master_service_host", c.master_host);
  c.master_port = static_cast<int>(j.get_int("master_service_port", c.master_port));
  c.poll_ms = static_cast<int>(j.get_int("poll_ms", c.poll_ms));
  if (c.max_slots_per_pod < 1) throw std::invalid_argument("kubernetes.max_slots_per_pod must be >= 1");
  return c;
}

KubernetesRM::KubernetesRM(Master* m, KubeConfig cfg) : m_(m), cfg_(std::move(cfg)) {}

KubernetesRM::~KubernetesRM() { Stop(); }

std::string KubernetesRM::Path(const std::string& kind, const std::string& name) const {
  std::string p = "/api/v1/namespaces/" + cfg_.ns + "/" + kind;
  return name.empty() ? p : p + "/" + name;
}

void KubernetesRM::Start() {
  if (cfg_.master_host.empty()) cfg_.master_host = m_->advertised_host();
  if (cfg_.master_port <= 0) cfg_.master_port = m_->port();
  auto r = net::HttpCall(cfg_.host, cfg_.port, "GET", "/api/v1/nodes", "", 10000);
  if (!r.error.empty() || r.status != 200)
    throw std::runtime_error("kubernetes: cannot list nodes at " + cfg_.host + ":" + std::to_string(cfg_.port) +
                             ": " + (r.error.empty() ? std::to_string(r.status) + " " + r.body.substr(0, 200) : r.error));
  Json nodes = Json::parse(r.body);
  for (auto& n : nodes["items"].as_array()) {
    const std::string node = n["metadata"].get_string("name", "node");
    if (n["spec"].get_bool("unschedulable", false)) continue;
    int slots = 0;
    if (cfg_.slot_type == "gpu") {
      const Json& q = n["status"]["allocatable"][cfg_.slot_resource];
      slots = q.is_string() ? std::atoi(q.as_string().c_str()) : q.is_number() ? static_cast<int>(q.as_int()) : 0;
    } else {
      slots = cfg_.cpu_slots_per_node;
    }
    for (int g = 0, left = slots; left > 0; ++g) {
      int n_slots = std::min(left, cfg_.max_slots_per_pod);
      left -= n_slots;
      auto conn = std::make_shared<AgentConn>();
      conn->id = "k8s-" + DnsName(node) + "-" + std::to_string(g);
      conn->pool = cfg_.pool;
      conn->label = "";
      conn->host = cfg_.master_host;
      const std::string agent = conn->id;
      conn->send = [this, agent](const Json& msg) { return FromMaster(agent, msg); };
      std::string err;
      if (!m_->RegisterAgent(conn, &err)) throw std::runtime_error("kubernetes: " + err);
      Json started = Json::object();
      started["type"] = "AgentStarted";
      Json devices = Json::array();
      for (int i = 0; i < n_slots; ++i) {
        Json d = Json::object();
        d["id"] = i;
        d["type"] = cfg_.slot_type;
        d["brand"] = cfg_.slot_type == "gpu" ? "AMD Instinct (" + cfg_.slot_resource + ")" : "CPU";
        d["uuid"] = node + "-" + std::to_string(g) + "-" + std::to_string(i);
        devices.push_back(d);
      }
      started["devices"] = devices;
      conn->devices = devices;
      conn->containers.clear();
      {
        std::lock_guard<std::mutex> l(mu_);
        agents_.push_back(conn);
      }
      // remember which node this virtual agent lives on (nodeSelector)
      conn->label = "";
      m_->OnAgentMessage(conn, started);
      MasterLog("kubernetes: node " + node + " group " + std::to_string(g) + " -> virtual agent " + agent + " (" +
                std::to_string(n_slots) + " " + cfg_.slot_type + " slots)");
    }
  }
  watcher_ = std::thread([this] { WatchLoop(); });
}

void KubernetesRM::Stop() {
  if (stop_.exchange(true)) return;
  if (watcher_.joinable()) watcher_.join();
  std::vector<std::shared_ptr<std::thread>> logs;
  {
    std::lock_guard<std::mutex> l(mu_);
    for (auto& kv : pods_)
      if (kv.second.logs) logs.push_back(kv.second.logs);
  }
  for (auto& t : logs)
    if (t->joinable()) t->join();
}

Json KubernetesRM::Summary() const {
  std::lock_guard<std::mutex> l(mu_);
  Json out = Json::object();
  Json pods = Json::array();
  for (auto& kv : pods_) {
    Json p = Json::object();
    p["container_id"] = kv.first;
    p["pod"] = kv.second.name;
    p["agent"] = kv.second.agent;
    p["state"] = kv.second.reported;
    pods.push_back(p);
  }
  out["pods"] = pods;
  out["namespace"] = cfg_.ns;
  out["agents"] = static_cast<int64_t>(agents_.size());
  return out;
}

void KubernetesRM::Report(const std::string& agent, const Json& msg) {
  std::shared_ptr<AgentConn> conn;
  {
    std::lock_guard<std::mutex> l(mu_);
    for (auto& a : agents_)
      if (a->id == agent) conn = a;
  }
  if (conn) m_->OnAgentMessage(conn, msg);
}

bool KubernetesRM::FromMaster(const std::string& agent, const Json& msg) {
  const std::string t = msg.get_string("type", "");
  if (t == "StartContainer") {
    std::thread([this, agent, msg] { CreatePod(agent, msg); }).detach();
    return true;
  }
  if (t == "SignalContainer") {
    const std::string sig = msg.get_string("signal", "SIGKILL");
    std::string cid = msg.get_string("container_id", "");
    std::thread([this, cid, sig] { DeletePod(cid, sig == "SIGKILL" ? 0 : 30); }).detach();
    return true;
  }
  return true;  // other master -> agent messages have no pod counterpart
}

void KubernetesRM::CreatePod(const std::string& agent, const Json& msg) {
  const std::string cid = msg.get_string("container_id", "");
  const Json& spec = msg["spec"];
  auto state = [&](const std::string& s, int code, const std::string& failure) {
    Json m = Json::object();
    m["type"] = "ContainerStateChanged";
    m["container_id"] = cid;
    m["state"] = s;
    m["exit_code"] = code;
    if (!failure.empty()) m["failure"] = failure;
    Report(agent, m);
  };
  const int64_t exp_id = spec.get_int("experiment_id", 0), trial_id = spec.get_int("trial_id", 0);
  const int rank = static_cast<int>(spec.get_int("rank", 0));
  const std::string task_id = spec.get_string("task_id", "");
  std::string name = trial_id > 0 ? "exp-" + std::to_string(exp_id) + "-trial-" + std::to_string(trial_id) + "-rank-" +
                                        std::to_string(rank) + "-" + cid.substr(0, 8)
                                  : "task-" + (task_id.empty() ? std::string("x") : task_id) + "-" + cid.substr(0, 8);
  name = DnsName(name);
  // node of the virtual agent: "k8s-<node>-<group>"
  std::string node = agent.substr(4, agent.rfind('-') - 4);
  const int n_slots = static_cast<int>(msg["devices"].size());

  Json cm = Json::object();
  cm["apiVersion"] = "v1";
  cm["kind"] = "ConfigMap";
  cm["metadata"]["name"] = name;
  cm["metadata"]["labels"]["determined"] = cid;
  cm["metadata"]["labels"]["determined-cluster"] = DnsName(m_->cluster_id());
  cm["data"]["spec.json"] = spec.dump();
  auto r = net::HttpCall(cfg_.host, cfg_.port, "POST", Path("configmaps"), cm.dump(), 10000);
  if (!r.error.empty() || r.status >= 300) {
    state("Terminated", 1, "kubernetes: cannot create configmap: " + (r.error.empty() ? r.body.substr(0, 200) : r.error));
    return;
  }

  Json env = Json::array();
  std::map<std::string, std::string> kv;
  for (auto& e : spec["env"].as_object()) kv[e.first] = e.second.is_string() ? e.second.as_string() : e.second.dump();
  Json slot_ids = Json::array();
  for (int i = 0; i < n_slots; ++i) slot_ids.push_back(i);
  kv["DET_CLUSTER_ID"] = m_->cluster_id();
  kv["DET_MASTER"] = cfg_.master_host + ":" + std::to_string(cfg_.master_port);
  kv["DET_MASTER_HOST"] = cfg_.master_host;
  kv["DET_MASTER_ADDR"] = cfg_.master_host;
  kv["DET_MASTER_PORT"] = std::to_string(cfg_.master_port);
  kv["DET_AGENT_ID"] = agent;
  kv["DET_CONTAINER_ID"] = cid;
  kv["DET_SLOT_IDS"] = slot_ids.dump();
  kv["DET_USE_GPU"] = cfg_.slot_type == "gpu" ? "true" : "false";
  if (cfg_.slot_type != "gpu") kv["DET_NUM_CPU_SLOTS"] = std::to_string(n_slots);
  kv["DET_SPEC_FILE"] = "/run/determined/spec/spec.json";
  kv["HSA_ENABLE_IPC_MODE_LEGACY"] = "0";
  for (auto& e : kv) {
    Json v = Json::object();
    v["name"] = e.first;
    v["value"] = e.second;
    env.push_back(v);
  }
  Json cmd = Json::array();
  cmd.push_back(cfg_.python);
  cmd.push_back("-m");
  cmd.push_back("determined_1_amd.exec.pod_entrypoint");
  cmd.push_back("--");
  if (spec["cmd"].is_array() && spec["cmd"].size() > 0) {
    for (auto& a : spec["cmd"].as_array()) cmd.push_back(a);
  } else {
    cmd.push_back(cfg_.python);
    cmd.push_back("-m");
    cmd.push_back("determined_1_amd.exec.harness");
  }
  Json container = Json::object();
  container["name"] = "determined-container";
  container["image"] = spec.get_string("image", cfg_.image);
  container["command"] = cmd;
  container["env"] = env;
  container["workingDir"] = "/run/determined/workdir";
  if (spec["user"].is_object()) {  // the task owner's agent user group (reference kubernetes/spec.go)
    container["securityContext"]["runAsUser"] = spec["user"].get_int("uid", 0);
    container["securityContext"]["runAsGroup"] = spec["user"].get_int("gid", 0);
  }
  Json mounts = Json::array();
  Json mount = Json::object();
  mount["name"] = "det-spec";
  mount["mountPath"] = "/run/determined/spec";
  mounts.push_back(mount);
  container["volumeMounts"] = mounts;
  if (cfg_.slot_type == "gpu" && n_slots > 0) {
    container["resources"]["limits"][cfg_.slot_resource] = std::to_string(n_slots);
    container["resources"]["requests"][cfg_.slot_resource] = std::to_string(n_slots);
  }
  Json pod = Json::object();
  pod["apiVersion"] = "v1";
  pod["kind"] = "Pod";
  pod["metadata"]["name"] = name;
  pod["metadata"]["labels"]["determined"] = cid;
  pod["metadata"]["labels"]["determined-cluster"] = DnsName(m_->cluster_id());
  pod["spec"]["restartPolicy"] = "Never";
  pod["spec"]["nodeSelector"]["kubernetes.io/hostname"] = node;
  pod["spec"]["containers"] = Json(Json::Array{container});
  Json vols = Json::array();
  Json vol = Json::object();
  vol["name"] = "det-spec";
  vol["configMap"]["name"] = name;
  vols.push_back(vol);
  pod["spec"]["volumes"] = vols;
  {
    std::lock_guard<std::mutex> l(mu_);
    Pod p;
    p.cid = cid;
    p.name = name;
    p.agent = agent;
    p.trial_id = trial_id;
    p.rank = rank;
    p.task_id = task_id;
    pods_[cid] = p;
  }
  r = net::HttpCall(cfg_.host, cfg_.port, "POST", Path("pods"), pod.dump(), 10000);
  if (!r.error.empty() || r.status >= 300) {
    {
      std::lock_guard<std::mutex> l(mu_);
      pods_.erase(cid);
    }
    net::HttpCall(cfg_.host, cfg_.port, "DELETE", Path("configmaps", name), "", 10000);
    state("Terminated", 1, "kubernetes: cannot create pod: " + (r.error.empty() ? r.body.substr(0, 200) : r.error));
    return;
  }
  MasterLog("kubernetes: created pod " + name + " for container " + cid);
}

void KubernetesRM::DeletePod(const std::string& cid, int grace_seconds) {
  std::string name;
  {
    std::lock_guard<std::mutex> l(mu_);
    auto it = pods_.find(cid);
    if (it == pods_.end()) return;
    it->second.deleting = true;
    name = it->second.name;
  }
  Json body = Json::object();
  body["gracePeriodSeconds"] = grace_seconds;
  net::HttpCall(cfg_.host, cfg_.port, "DELETE", Path("pods", name), body.dump(), 10000);
}

void KubernetesRM::FollowLogs(Pod p, std::shared_ptr<std::atomic<bool>> done) {
  StreamLines(cfg_.host, cfg_.port, Path("pods", p.name) + "/log?follow=true", stop_, [&](const std::string& line) {
    Json m = Json::object();
    m["type"] = "ContainerLog";
    m["container_id"] = p.cid;
    m["trial_id"] = p.trial_id;
    if (!p.task_id.empty()) m["task_id"] = p.task_id;
    m["rank"] = p.rank;
    m["stdtype"] = "stdout";
    m["log"] = line;
    Report(p.agent, m);
    return true;
  });
  done->store(true);
}

void KubernetesRM::WatchLoop() {
  const std::string selector = "determined-cluster%3D" + net::UrlEncode(DnsName(m_->cluster_id()));
  while (!stop_.load()) {
    std::this_thread::sleep_for(std::chrono::milliseconds(cfg_.poll_ms));
    bool any;
    {
      std::lock_guard<std::mutex> l(mu_);
      any = !pods_.empty();
    }
    if (!any) continue;
    auto r = net::HttpCall(cfg_.host, cfg_.port, "GET", Path("pods") + "?labelSelector=" + selector, "", 10000);
    if (!r.error.empty() || r.status != 200) continue;
    Json list;
    try {
      list = Json::parse(r.body);
    } catch (const std::exception&) {
      continue;
    }
    std::map<std::string, Json> by_cid;
    for (auto& item : list["items"].as_array()) by_cid[item["metadata"]["labels"].get_string("determined", "")] = item;
    std::vector<std::pair<std::string, Json>> reports;  // (agent, msg), sent without mu_
    std::vector<std::string> cleanup;                   // pod names to delete (pod + configmap)
    std::vector<std::shared_ptr<std::thread>> joins;
    {
      std::lock_guard<std::mutex> l(mu_);
      for (auto it = pods_.begin(); it != pods_.end();) {
        Pod& p = it->second;
        auto found = by_cid.find(p.cid);
        std::string phase = found == by_cid.end() ? "Gone" : found->second["status"].get_string("phase", "Pending");
        auto state_msg = [&](const std::string& s) {
          Json m = Json::object();
          m["type"] = "ContainerStateChanged";
          m["container_id"] = p.cid;
          m["state"] = s;
          return m;
        };
        if (phase == "Pending" && p.reported.empty()) {
          p.reported = "Starting";
          reports.push_back({p.agent, state_msg("Starting")});
        } else if (phase == "Running" && p.reported != "Running") {
          if (p.reported.empty()) reports.push_back({p.agent, state_msg("Starting")});
          p.reported = "Running";
          Json m = state_msg("Running");
          m["address"] = found->second["status"].get_string("podIP", cfg_.master_host);
          reports.push_back({p.agent, m});
          p.logs_done = std::make_shared<std::atomic<bool>>(false);
          p.logs = std::make_shared<std::thread>(&KubernetesRM::FollowLogs, this, p, p.logs_done);
        } else if (phase == "Succeeded" || phase == "Failed" || phase == "Gone") {
          if (p.logs && p.logs_done && !p.logs_done->load() && phase != "Gone") {
            ++it;  // let the log follower drain the container's output first
            continue;
          }
          int code = phase == "Succeeded" ? 0 : 1;
          std::string failure;
          if (phase != "Gone") {
            for (auto& cs : found->second["status"]["containerStatuses"].as_array()) {
              const Json& term = cs["state"]["terminated"];
              if (term.is_object()) {
                code = static_cast<int>(term.get_int("exitCode", code));
                failure = term.get_string("reason", "");
              }
            }
          } else {
            code = p.deleting ? 137 : -1;
            failure = p.deleting ? "pod deleted" : "pod vanished";
          }
          Json m = state_msg("Terminated");
          m["exit_code"] = code;
          if (code != 0) m["failure"] = failure.empty() ? "container exited with code " + std::to_string(code) : failure;
          if (p.reported.empty()) reports.push_back({p.agent, state_msg("Starting")});
          reports.push_back({p.agent, m});
          if (p.logs) joins.push_back(p.logs);
          if (phase != "Gone") cleanup.push_back(p.name);
          else cleanup.push_back("-" + p.name);  // configmap only
          it = pods_.erase(it);
          continue;
        }
        ++it;
      }
    }
    for (auto& t : joins)
      if (t->joinable()) t->join();
    for (auto& rep : reports) Report(rep.first, rep.second);
    for (auto& name : cleanup) {
      bool cm_only = !name.empty() && name[0] == '-';
      std::string n = cm_only ? name.substr(1) : name;
      if (!cm_only) net::HttpCall(cfg_.host, cfg_.port, "DELETE", Path("pods", n), "", 10000);
      net::HttpCall(cfg_.host, cfg_.port, "DELETE", Path("configmaps", n), "", 10000);
    }
  }
}

}  // namespace master
}  // namespace detcore
