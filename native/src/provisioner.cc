// Elastic provisioning (see include/detcore/provisioner.h).
#include "detcore/provisioner.h"

#include <signal.h>
#include <spawn.h>
#include <sys/wait.h>

#include <algorithm>
#include <cstdio>

extern char** environ;

namespace detcore {
namespace prov {

ProvisionerConfig ProvisionerConfig::FromJson(const Json& j) {
  ProvisionerConfig c;
  c.min_instances = static_cast<int>(j.get_int("min_instances", 0));
  c.max_instances = static_cast<int>(j.get_int("max_instances", 0));
  c.slots_per_instance = static_cast<int>(j.get_int("slots_per_instance", 1));
  c.max_idle_period = std::chrono::milliseconds(j.get_int("max_idle_agent_period_ms", 300000));
  c.max_starting_period = std::chrono::milliseconds(j.get_int("max_agent_starting_period_ms", 300000));
  c.provider = j.get_string("provider", "local");
  c.agent_binary = j.get_string("agent_binary", "");
  c.artificial = j.get_bool("artificial_slots", true);
  c.work_dir = j.get_string("work_dir", c.work_dir);
  c.raw = j;
  return c;
}

Decision ScaleDecider::Decide(int pending_slots, const std::vector<AgentInfo>& agents,
                              const std::vector<Instance>& instances, Clock::time_point now) {
  Decision d;
  std::map<std::string, bool> connected_idle;
  for (auto& a : agents) connected_idle[a.id] = a.idle;
  int live = 0;
  std::vector<const Instance*> idle_candidates;
  for (auto& inst : instances) {
    if (inst.state == "Stopped") continue;
    ++live;
    auto it = connected_idle.find(inst.id);
    if (it == connected_idle.end()) {
      // no agent yet: starting, or stuck / disconnected
      idle_since_.erase(inst.id);
      if (now - inst.launched > cfg_.max_starting_period) d.terminate.push_back(inst.id);
      continue;
    }
    if (!it->second) {
      idle_since_.erase(inst.id);
      continue;
    }
    auto ins = idle_since_.emplace(inst.id, now).first;
    if (now - ins->second > cfg_.max_idle_period) idle_candidates.push_back(&inst);
  }
  // keep min_instances alive; terminate the longest-idle first
  std::sort(idle_candidates.begin(), idle_candidates.end(),
            [&](const Instance* a, const Instance* b) { return idle_since_[a->id] < idle_since_[b->id]; });
  int removable = live - static_cast<int>(d.terminate.size()) - cfg_.min_instances;
  if (pending_slots > 0) removable = 0;  // demand exists: don't shrink
  for (const Instance* inst : idle_candidates) {
    if (removable <= 0) break;
    d.terminate.push_back(inst->id);
    idle_since_.erase(inst->id);
    --removable;
  }
  // launch for unmet demand: instances still starting count as capacity on the way, and so do the
  // slots of connected idle instances that are kept (the scheduler places pending work on them at its
  // next pass; without this an agent that connects between a scheduling pass and this decision
  // looks like missing capacity and a second instance is launched)
  int starting = 0, idle_kept = 0;
  for (auto& inst : instances) {
    if (inst.state == "Stopped") continue;
    auto it = connected_idle.find(inst.id);
    if (it == connected_idle.end()) ++starting;
    else if (it->second && std::find(d.terminate.begin(), d.terminate.end(), inst.id) == d.terminate.end()) ++idle_kept;
  }
  int spi = std::max(1, cfg_.slots_per_instance);
  const int unmet = std::max(0, pending_slots - idle_kept * spi);
  int want = (unmet + spi - 1) / spi - starting;
  int room = cfg_.max_instances - (live - static_cast<int>(d.terminate.size()));
  d.launch = std::max(0, std::min(want, room));
  if (live - static_cast<int>(d.terminate.size()) + d.launch < cfg_.min_instances)
    d.launch = cfg_.min_instances - (live - static_cast<int>(d.terminate.size()));
  return d;
}

LocalProvider::LocalProvider(ProvisionerConfig cfg, std::string pool) : cfg_(std::move(cfg)), pool_(std::move(pool)) {}

LocalProvider::~LocalProvider() {
  std::vector<std::string> ids;
  for (auto& kv : procs_) ids.push_back(kv.first);
  Terminate(ids);
}

std::vector<Instance> LocalProvider::List() {
  std::vector<Instance> out;
  for (auto it = procs_.begin(); it != procs_.end();) {
    int st;
    if (waitpid(it->second.first, &st, WNOHANG) == it->second.first) {
      it = procs_.erase(it);
      continue;
    }
    out.push_back(it->second.second);
    ++it;
  }
  return out;
}

void LocalProvider::Launch(int n) {
  for (int i = 0; i < n; ++i) {
    std::string id = pool_ + "-prov-" + std::to_string(next_++);
    std::vector<std::string> args = {cfg_.agent_binary, "--master-host", cfg_.master_host, "--master-port",
                                     std::to_string(cfg_.master_port), "--agent-id", id, "--resource-pool", pool_,
                                     "--python", cfg_.python, "--work-dir", cfg_.work_dir + "/" + id};
    if (cfg_.artificial) {
      args.push_back("--artificial-slots");
      args.push_back(std::to_string(cfg_.slots_per_instance));
    }
    std::vector<char*> argv;
    for (auto& a : args) argv.push_back(const_cast<char*>(a.c_str()));
    argv.push_back(nullptr);
    pid_t pid;
    if (posix_spawn(&pid, cfg_.agent_binary.c_str(), nullptr, nullptr, argv.data(), environ) != 0) {
      std::fprintf(stderr, "[det-master] provisioner: failed to launch %s\n", cfg_.agent_binary.c_str());
      continue;
    }
    procs_[id] = {pid, Instance{id, "Starting", Clock::now()}};
    std::fprintf(stderr, "[det-master] provisioner: launched agent %s (pid %d)\n", id.c_str(), pid);
  }
}

void LocalProvider::Terminate(const std::vector<std::string>& ids) {
  for (auto& id : ids) {
    auto it = procs_.find(id);
    if (it == procs_.end()) continue;
    ::kill(it->second.first, SIGTERM);
    int st;
    waitpid(it->second.first, &st, 0);
    procs_.erase(it);
    std::fprintf(stderr, "[det-master] provisioner: terminated agent %s\n", id.c_str());
  }
}

CommandProvider::CommandProvider(ProvisionerConfig cfg, std::string pool) : cfg_(std::move(cfg)), pool_(std::move(pool)) {
  Spawn();
}

CommandProvider::~CommandProvider() {
  if (in_fd_ >= 0) close(in_fd_);
  if (out_fd_ >= 0) close(out_fd_);
  if (pid_ > 0) {
    ::kill(pid_, SIGTERM);
    int st;
    waitpid(pid_, &st, 0);
  }
}

void CommandProvider::Spawn() {
  int to_child[2], from_child[2];
  if (pipe(to_child) != 0 || pipe(from_child) != 0) return;
  Json raw = cfg_.raw;
  raw["cluster_id"] = cfg_.cluster_id;
  std::string conf = raw.dump();
  std::vector<std::string> args = {cfg_.python, "-m", "determined_1_amd.deploy.cloud_provider", "--config", conf,
                                   "--pool", pool_, "--master-host", cfg_.master_host, "--master-port",
                                   std::to_string(cfg_.master_port)};
  pid_t pid = fork();
  if (pid == 0) {
    dup2(to_child[0], 0);
    dup2(from_child[1], 1);
    close(to_child[1]);
    close(from_child[0]);
    if (!cfg_.framework_root.empty()) {
      const char* old = getenv("PYTHONPATH");
      std::string pp = cfg_.framework_root + (old && *old ? std::string(":") + old : "");
      setenv("PYTHONPATH", pp.c_str(), 1);
    }
    std::vector<char*> argv;
    for (auto& a : args) argv.push_back(const_cast<char*>(a.c_str()));
    argv.push_back(nullptr);
    execvp(argv[0], argv.data());
    _exit(127);
  }
  close(to_child[0]);
  close(from_child[1]);
  pid_ = pid;
  in_fd_ = to_child[1];
  out_fd_ = from_child[0];
}

bool CommandProvider::Call(const Json& req, Json* resp) {
  if (in_fd_ < 0) return false;
  std::string line = req.dump() + "\n";
  if (write(in_fd_, line.data(), line.size()) != static_cast<ssize_t>(line.size())) return false;
  while (true) {
    auto nl = rbuf_.find('\n');
    if (nl != std::string::npos) {
      std::string out = rbuf_.substr(0, nl);
      rbuf_.erase(0, nl + 1);
      try {
        *resp = Json::parse(out);
      } catch (const std::exception&) {
        return false;
      }
      if (resp->has("error")) {
        std::fprintf(stderr, "[det-master] provisioner (%s): %s\n", cfg_.provider.c_str(),
                     resp->get_string("error", "").c_str());
        return false;
      }
      return true;
    }
    char buf[4096];
    ssize_t n = read(out_fd_, buf, sizeof(buf));
    if (n <= 0) return false;
    rbuf_.append(buf, static_cast<size_t>(n));
  }
}

std::vector<Instance> CommandProvider::List() {
  std::vector<Instance> out;
  Json req = Json::object(), resp;
  req["op"] = "list";
  if (!Call(req, &resp)) return out;
  for (auto& it : resp["instances"].as_array()) {
    Instance inst;
    inst.id = it.get_string("id", "");
    inst.state = it.get_string("state", "Starting");
    auto l = launched_.find(inst.id);
    inst.launched = l == launched_.end() ? Clock::now() : l->second;
    if (l == launched_.end()) launched_[inst.id] = inst.launched;
    if (inst.state != "Stopped") out.push_back(inst);
  }
  return out;
}

void CommandProvider::Launch(int n) {
  Json req = Json::object(), resp;
  req["op"] = "launch";
  req["n"] = n;
  if (!Call(req, &resp)) return;
  for (auto& id : resp["launched"].as_array()) {
    launched_[id.as_string()] = Clock::now();
    std::fprintf(stderr, "[det-master] provisioner (%s): launched instance %s\n", cfg_.provider.c_str(),
                 id.as_string().c_str());
  }
}

void CommandProvider::Terminate(const std::vector<std::string>& ids) {
  Json req = Json::object(), resp;
  req["op"] = "terminate";
  Json arr = Json::array();
  for (auto& i : ids) arr.push_back(i);
  req["ids"] = arr;
  if (!Call(req, &resp)) return;
  for (auto& i : ids) {
    launched_.erase(i);
    std::fprintf(stderr, "[det-master] provisioner (%s): terminated instance %s\n", cfg_.provider.c_str(), i.c_str());
  }
}

}  // namespace prov
}  // namespace detcore
