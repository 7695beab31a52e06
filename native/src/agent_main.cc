// det-agent: one per node (reference agent/internal/{agent,detect,containers,
// container,fluent}.go).
//
//   * device detection: AMD GPUs from the KFD topology (/sys/class/kfd/kfd/topology/nodes/*,
//     no GPU context is created), `--artificial-slots N` fake devices for CPU-only clusters/tests,
//     `--slot-type none` for zero-slot agents;
//   * WebSocket to the master (/agents?id=..), AgentStarted{devices};
//   * StartContainer -> a "container" is a process group: a fresh work dir holding the model
//     definition (fetched from the master) and the spec's files, env = C-env contract +
//     DET_SLOT_IDS / DET_USE_GPU / HIP_VISIBLE_DEVICES, stdout/stderr shipped to the master as
//     ContainerLog lines (the reference's Fluent Bit path);
//   * container state machine Assigned -> Starting -> Running -> Terminated(exit code);
//   * SignalContainer -> kill(-pgid); master disconnect -> kill everything, reconnect w/ backoff.
//   * harness containers are forked from a warm zygote (determined_1_amd/exec/zygote.py) that has
//     torch + the harness imported but no GPU context, instead of a cold `python -m` exec; the
//     zygote reports the child's pid and exit status over its unix socket.  Without a zygote
//     (`--no-zygote`, or it is not up) containers are fork/exec'd as before.
#include <dirent.h>
#include <fcntl.h>
#include <signal.h>
#include <sys/socket.h>
#include <sys/stat.h>
#include <sys/types.h>
#include <sys/un.h>
#include <sys/wait.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <ftw.h>
#include <grp.h>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <map>
#include <memory>
#include <mutex>
#include <sstream>
#include <string>
#include <utility>
#include <thread>
#include <vector>

#include "detcore/json.h"
#include "detcore/net.h"

extern char** environ;

using detcore::Json;
namespace net = detcore::net;

namespace {

struct Options {
  std::string master_host = "127.0.0.1";
  int master_port = 8080;
  // TLS to the master (reference agent --security-tls-*): verify its cert against this PEM
  bool master_tls = false;
  std::string master_cert_file, master_cert_name;
  std::string id;
  std::string pool;
  std::string label;
  int artificial_slots = 0;
  std::string slot_type = "auto";  // auto | gpu | cpu | none
  std::string visible_gpus;        // comma list filter
  std::string python = "python3";
  std::string work_dir = "/tmp/det-agent";
  std::string framework_root;
  std::string advertise_host;
  bool zygote = true;  // serve harness containers from a warm pre-imported Python (exec/zygote.py)
};

void Log(const std::string& s) { std::fprintf(stderr, "[det-agent] %s\n", s.c_str()); }

std::string ReadFile(const std::string& p) {
  std::ifstream f(p);
  std::stringstream ss;
  ss << f.rdbuf();
  return ss.str();
}

// KFD topology: GPU nodes have simd_count > 0.  The order of GPU nodes is the HIP device order.
Json DetectAmdGpus(const std::string& visible) {
  Json out = Json::array();
  const std::string base = "/sys/class/kfd/kfd/topology/nodes";
  DIR* d = opendir(base.c_str());
  if (!d) return out;
  std::vector<int> nodes;
  while (dirent* e = readdir(d)) {
    if (e->d_name[0] == '.') continue;
    nodes.push_back(std::atoi(e->d_name));
  }
  closedir(d);
  std::sort(nodes.begin(), nodes.end());
  int idx = 0;
  std::vector<std::string> allow;
  {
    std::stringstream ss(visible);
    std::string t;
    while (std::getline(ss, t, ',')) allow.push_back(t);
  }
  for (int n : nodes) {
    std::string props = ReadFile(base + "/" + std::to_string(n) + "/properties");
    long simd = 0;
    unsigned long long uid = 0;
    std::stringstream ps(props);
    std::string k;
    long long v;
    while (ps >> k >> v) {
      if (k == "simd_count") simd = static_cast<long>(v);
      if (k == "unique_id") uid = static_cast<unsigned long long>(v);
    }
    if (simd <= 0) continue;
    int dev = idx++;
    if (!allow.empty() && std::find(allow.begin(), allow.end(), std::to_string(dev)) == allow.end()) continue;
    std::string name = ReadFile(base + "/" + std::to_string(n) + "/name");
    while (!name.empty() && (name.back() == '\n' || name.back() == ' ')) name.pop_back();
    Json g = Json::object();
    g["id"] = dev;
    g["type"] = "gpu";
    g["brand"] = name.empty() ? "AMD Instinct" : name;
    char buf[32];
    std::snprintf(buf, sizeof(buf), "GPU-%016llx", uid);
    g["uuid"] = std::string(buf);
    out.push_back(g);
  }
  return out;
}

Json DetectDevices(const Options& o) {
  Json out = Json::array();
  if (o.slot_type == "none") return out;
  if (o.artificial_slots > 0) {
    for (int i = 0; i < o.artificial_slots; ++i) {
      Json d = Json::object();
      d["id"] = i;
      d["type"] = "cpu";
      d["brand"] = "Artificial";
      d["uuid"] = o.id + "-artificial-" + std::to_string(i);
      out.push_back(d);
    }
    return out;
  }
  if (o.slot_type == "auto" || o.slot_type == "gpu") out = DetectAmdGpus(o.visible_gpus);
  if (out.size() == 0 && (o.slot_type == "auto" || o.slot_type == "cpu")) {
    Json d = Json::object();
    d["id"] = 0;
    d["type"] = "cpu";
    d["brand"] = "CPU";
    d["uuid"] = o.id + "-cpu";
    out.push_back(d);
  }
  return out;
}

void MkdirP(const std::string& path) {
  std::string cur;
  std::stringstream ss(path);
  std::string part;
  if (!path.empty() && path[0] == '/') cur = "/";
  while (std::getline(ss, part, '/')) {
    if (part.empty()) continue;
    cur += part + "/";
    ::mkdir(cur.c_str(), 0755);
  }
}

struct Proc {
  std::string cid;
  pid_t pid = -1;
  int64_t trial_id = 0;
  int rank = 0;
};

class Agent {
 public:
  explicit Agent(Options o) : o_(std::move(o)) {}

  int Run() {
    devices_ = DetectDevices(o_);
    if (o_.zygote) StartZygote();
    Log("detected " + std::to_string(devices_.size()) + " slots: " + devices_.dump());
    int backoff_ms = 500;
    while (!stop_.load()) {
      std::string err;
      std::string path = "/agents?id=" + o_.id + "&resource_pool=" + o_.pool + "&label=" + o_.label;
      if (!o_.advertise_host.empty()) path += "&host=" + o_.advertise_host;
      ws_ = net::WsConnect(o_.master_host, o_.master_port, path, &err);
      if (!ws_) {
        Log("cannot reach master " + o_.master_host + ":" + std::to_string(o_.master_port) + ": " + err);
        std::this_thread::sleep_for(std::chrono::milliseconds(backoff_ms));
        backoff_ms = std::min(backoff_ms * 2, 10000);
        continue;
      }
      backoff_ms = 500;
      Json started = Json::object();
      started["type"] = "AgentStarted";
      started["version"] = "0.13.10.dev0+mi355x";
      started["label"] = o_.label;
      started["devices"] = devices_;
      ws_->Send(started.dump());
      Log("connected to master as " + o_.id);
      ws_->ReadLoop([&](const std::string& text) { Handle(text); });
      Log("master connection lost; killing containers");
      KillAll();
      if (o_.master_port <= 0) break;
      std::this_thread::sleep_for(std::chrono::milliseconds(backoff_ms));
    }
    KillAll();
    StopZygote();
    return 0;
  }

  void Stop() {
    stop_ = true;
    if (ws_) ws_->Close();
  }

  void StopZygote() {
    if (zygote_pid_ > 0) {
      ::kill(zygote_pid_, SIGTERM);
      int st = 0;
      for (int i = 0; i < 50 && waitpid(zygote_pid_, &st, WNOHANG) == 0; ++i)
        std::this_thread::sleep_for(std::chrono::milliseconds(20));
      ::kill(zygote_pid_, SIGKILL);
      waitpid(zygote_pid_, &st, WNOHANG);
      zygote_pid_ = -1;
    }
  }

 private:
  // The zygote is a child of the agent (it exits when the agent goes away); its stderr is the
  // agent's.  Startup is asynchronous: until its socket accepts, containers are fork/exec'd.
  void StartZygote() {
    zygote_sock_ = o_.work_dir + "/zygote-" + std::to_string(getpid()) + ".sock";
    std::string pp = o_.framework_root;
    const char* old = getenv("PYTHONPATH");
    if (old && *old) pp += std::string(":") + old;
    pid_t pid = fork();
    if (pid == 0) {
      setenv("PYTHONPATH", pp.c_str(), 1);
      setenv("HSA_ENABLE_IPC_MODE_LEGACY", "0", 1);
      execlp(o_.python.c_str(), o_.python.c_str(), "-m", "determined_1_amd.exec.zygote", "--socket",
             zygote_sock_.c_str(), static_cast<char*>(nullptr));
      _exit(127);
    }
    if (pid <= 0) return;
    zygote_pid_ = pid;
    // wait for the socket before registering slots with the master, so the first containers are
    // served warm; give up (cold fork/exec for every container) if the zygote exits or stalls
    for (int i = 0; i < 600; ++i) {
      struct stat st;
      if (::stat(zygote_sock_.c_str(), &st) == 0) return;
      int status = 0;
      if (waitpid(pid, &status, WNOHANG) == pid) {
        Log("zygote exited during preload; containers will be fork/exec'd");
        zygote_pid_ = -1;
        return;
      }
      std::this_thread::sleep_for(std::chrono::milliseconds(50));
    }
    Log("zygote not ready after 30 s; containers will be fork/exec'd until it is");
  }

  // Ask the zygote to fork a harness child with the container's stdout/stderr pipes, env and cwd.
  // Returns the connected socket (the exit status arrives on it later) and sets *child; -1 when the
  // zygote is unavailable or refused, in which case the caller fork/execs.
  int ZygoteSpawn(const std::vector<std::string>& args, const std::map<std::string, std::string>& env,
                  const std::string& cwd, int out_fd, int err_fd, pid_t* child, int uid = -1, int gid = -1) {
    if (zygote_pid_ <= 0 || args.size() < 3 || args[1] != "-m") return -1;
    int fd = socket(AF_UNIX, SOCK_STREAM | SOCK_CLOEXEC, 0);
    if (fd < 0) return -1;
    sockaddr_un addr{};
    addr.sun_family = AF_UNIX;
    if (zygote_sock_.size() >= sizeof(addr.sun_path)) {
      close(fd);
      return -1;
    }
    std::strncpy(addr.sun_path, zygote_sock_.c_str(), sizeof(addr.sun_path) - 1);
    if (connect(fd, reinterpret_cast<sockaddr*>(&addr), sizeof(addr)) != 0) {
      close(fd);
      return -1;
    }
    Json req = Json::object();
    Json argv = Json::array();
    for (size_t i = 1; i < args.size(); ++i) argv.push_back(args[i]);
    req["argv"] = argv;
    Json je = Json::object();
    for (auto& kv : env) je[kv.first] = kv.second;
    req["env"] = je;
    req["cwd"] = cwd;
    if (uid >= 0) {  // the zygote child switches to the task owner's account after fork
      req["uid"] = uid;
      req["gid"] = gid;
    }
    std::string body = req.dump();
    std::string msg(4, '\0');
    uint32_t n = static_cast<uint32_t>(body.size());
    msg[0] = static_cast<char>((n >> 24) & 0xff);
    msg[1] = static_cast<char>((n >> 16) & 0xff);
    msg[2] = static_cast<char>((n >> 8) & 0xff);
    msg[3] = static_cast<char>(n & 0xff);
    msg += body;
    int fds[2] = {out_fd, err_fd};
    char cbuf[CMSG_SPACE(sizeof(fds))];
    std::memset(cbuf, 0, sizeof(cbuf));
    iovec iov{const_cast<char*>(msg.data()), msg.size()};
    msghdr mh{};
    mh.msg_iov = &iov;
    mh.msg_iovlen = 1;
    mh.msg_control = cbuf;
    mh.msg_controllen = sizeof(cbuf);
    cmsghdr* cm = CMSG_FIRSTHDR(&mh);
    cm->cmsg_level = SOL_SOCKET;
    cm->cmsg_type = SCM_RIGHTS;
    cm->cmsg_len = CMSG_LEN(sizeof(fds));
    std::memcpy(CMSG_DATA(cm), fds, sizeof(fds));
    ssize_t sent = sendmsg(fd, &mh, MSG_NOSIGNAL);
    if (sent < 0) {
      close(fd);
      return -1;
    }
    size_t off = static_cast<size_t>(sent);
    while (off < msg.size()) {
      ssize_t w = send(fd, msg.data() + off, msg.size() - off, MSG_NOSIGNAL);
      if (w <= 0) {
        close(fd);
        return -1;
      }
      off += static_cast<size_t>(w);
    }
    std::string line = ReadLine(fd);
    if (line.rfind("pid ", 0) != 0) {
      close(fd);
      return -1;
    }
    *child = static_cast<pid_t>(std::atol(line.c_str() + 4));
    return *child > 0 ? fd : (close(fd), -1);
  }

  // chown -R (no symlink following): the task's work dir belongs to the account it runs as
  static void ChownTree(const std::string& root, uid_t uid, gid_t gid) {
    static uid_t s_uid;
    static gid_t s_gid;
    static std::mutex mu;
    std::lock_guard<std::mutex> g(mu);
    s_uid = uid;
    s_gid = gid;
    nftw(root.c_str(), [](const char* p, const struct stat*, int, struct FTW*) -> int {
      if (lchown(p, s_uid, s_gid) != 0) return 0;  // best effort per entry
      return 0;
    }, 32, FTW_PHYS);
  }

  static std::string ReadLine(int fd) {
    std::string out;
    char c;
    while (true) {
      ssize_t r = read(fd, &c, 1);
      if (r <= 0 || c == '\n') break;
      out.push_back(c);
    }
    return out;
  }

  void Send(const Json& m) {
    auto ws = ws_;
    if (ws) ws->Send(m.dump());
  }
  // wall-clock send time of a state change: the master reports how long state changes wait
  // behind other traffic on this socket (/debug/stats agent_state_latency_ms)
  static long long NowUs() {
    return std::chrono::duration_cast<std::chrono::microseconds>(std::chrono::system_clock::now().time_since_epoch())
        .count();
  }

  void State(const std::string& cid, const std::string& state, int exit_code = 0, const std::string& failure = "") {
    Json m = Json::object();
    m["type"] = "ContainerStateChanged";
    m["container_id"] = cid;
    m["state"] = state;
    m["sent_us"] = NowUs();
    m["exit_code"] = exit_code;
    if (!failure.empty()) m["failure"] = failure;
    Send(m);
  }

  void Handle(const std::string& text) {
    Json m;
    try {
      m = Json::parse(text);
    } catch (const std::exception&) {
      return;
    }
    const std::string t = m.get_string("type", "");
    if (t == "MasterSetAgentOptions") {
      if (o_.advertise_host.empty()) o_.advertise_host = net::LocalIPForPeer(o_.master_host, o_.master_port);
    } else if (t == "StartContainer") {
      std::thread([this, m] { Start(m); }).detach();
    } else if (t == "SignalContainer") {
      Signal(m.get_string("container_id", ""), m.get_string("signal", "SIGKILL"));
    } else if (t == "Error") {
      Log("master error: " + m.get_string("error", ""));
    }
  }

  void Start(const Json& m) {
    const std::string cid = m.get_string("container_id", "");
    const Json& spec = m["spec"];
    State(cid, "Starting");
    std::string dir = o_.work_dir + "/" + cid;
    MkdirP(dir);
    // model definition (trials) or command context from the master
    int64_t exp_id = spec.get_int("experiment_id", 0);
    std::string ctx_url = spec.get_string("context_url", "/experiments/" + std::to_string(exp_id) + "/model_def");
    auto r = net::HttpCall(o_.master_host, o_.master_port, "GET", ctx_url);
    if (r.status != 200) {
      State(cid, "Terminated", 1, "cannot fetch model definition: " + r.error + " " + r.body.substr(0, 200));
      return;
    }
    try {
      Json md = Json::parse(r.body);
      for (auto& f : md["files"].as_array()) {
        std::string rel = f.get_string("path", "");
        if (rel.empty() || rel.find("..") != std::string::npos) continue;
        std::string full = dir + "/" + rel;
        if (f.get_string("type", "file") == "dir" || (!rel.empty() && rel.back() == '/')) {
          MkdirP(full);
          continue;
        }
        MkdirP(full.substr(0, full.rfind('/')));
        std::ofstream out(full, std::ios::binary);
        out << net::Base64Decode(f.get_string("content", ""));
      }
      for (auto& f : spec["files"].as_array()) {
        std::string full = dir + "/" + f.get_string("path", "");
        MkdirP(full.substr(0, full.rfind('/')));
        std::ofstream out(full, std::ios::binary);
        out << net::Base64Decode(f.get_string("content", ""));
      }
    } catch (const std::exception& e) {
      State(cid, "Terminated", 1, std::string("bad container spec: ") + e.what());
      return;
    }
    // env: agent env + C-env + device mask
    std::map<std::string, std::string> env;
    for (char** e = environ; *e; ++e) {
      std::string kv = *e;
      auto eq = kv.find('=');
      if (eq != std::string::npos) env[kv.substr(0, eq)] = kv.substr(eq + 1);
    }
    for (auto& kv : spec["env"].as_object()) env[kv.first] = kv.second.is_string() ? kv.second.as_string() : kv.second.dump();
    if (env.count("DET_LATEST_CHECKPOINT") && !env["DET_LATEST_CHECKPOINT"].empty() && env["DET_LATEST_CHECKPOINT"][0] != '/')
      env["DET_LATEST_CHECKPOINT"] = dir + "/" + env["DET_LATEST_CHECKPOINT"];
    Json slot_ids = Json::array();
    std::string hip;
    bool gpu = false;
    for (auto& d : m["devices"].as_array()) {
      int id = static_cast<int>(d.as_int());
      slot_ids.push_back(id);
      for (const auto& dev : std::as_const(devices_).as_array())  // const: no COW detach (Start runs per container thread)
        if (dev.get_int("id", -1) == id && dev.get_string("type", "") == "gpu") {
          gpu = true;
          hip += (hip.empty() ? "" : ",") + std::to_string(id);
        }
    }
    env["DET_SLOT_IDS"] = slot_ids.dump();
    env["DET_USE_GPU"] = gpu ? "true" : "false";
    env["DET_AGENT_ID"] = o_.id;
    env["DET_CONTAINER_ID"] = cid;
    if (gpu) {
      env["HIP_VISIBLE_DEVICES"] = hip;
      env["DET_CONTAINER_GPUS"] = hip;
    } else {
      env["HIP_VISIBLE_DEVICES"] = "";
      env["DET_NUM_CPU_SLOTS"] = std::to_string(slot_ids.size());
    }
    std::string pp = o_.framework_root + ":" + dir;
    if (env.count("PYTHONPATH") && !env["PYTHONPATH"].empty()) pp += ":" + env["PYTHONPATH"];
    env["PYTHONPATH"] = pp;
    env["HSA_ENABLE_IPC_MODE_LEGACY"] = "0";
    // the task owner's host account (reference master/pkg/tasks/task.go:60-100 getUser +
    // injectUserArchive): passwd/group/shadow entries for it, the work dir handed over to it, and
    // the process started as uid:gid (setgroups/setgid/setuid after fork, here or in the zygote)
    int run_uid = -1, run_gid = -1;
    if (spec["user"].is_object()) {
      const Json& u = spec["user"];
      run_uid = static_cast<int>(u.get_int("uid", -1));
      run_gid = static_cast<int>(u.get_int("gid", -1));
      const std::string uname = u.get_string("user", ""), gname = u.get_string("group", "");
      if (run_uid < 0 || run_gid < 0 || uname.empty() || gname.empty()) {
        State(cid, "Terminated", 1, "invalid agent user group in the container spec");
        return;
      }
      if (geteuid() != 0 && static_cast<uid_t>(run_uid) != geteuid()) {
        State(cid, "Terminated", 1, "det-agent runs as uid " + std::to_string(geteuid()) +
                                        ", not root: cannot start a task as uid " + std::to_string(run_uid));
        return;
      }
      const std::string etc = dir + "/.det/etc";
      MkdirP(etc);
      std::ofstream(etc + "/passwd") << uname << ":x:" << run_uid << ":" << run_gid << "::" << dir << ":/bin/sh\n";
      std::ofstream(etc + "/group") << gname << ":x:" << run_gid << ":\n";
      std::ofstream(etc + "/shadow") << uname << ":!!:::::::\n";
      ::chmod((etc + "/shadow").c_str(), 0600);
      env["USER"] = env["LOGNAME"] = uname;
      env["HOME"] = dir;
      env["DET_AGENT_USER"] = uname;
      env["DET_AGENT_GROUP"] = gname;
      env["DET_TASK_ETC"] = etc;
      if (geteuid() == 0) {
        ChownTree(dir, static_cast<uid_t>(run_uid), static_cast<gid_t>(run_gid));
        // the task dir is its owner's alone: the +x added to the parents below only lets an
        // account traverse to its own dir, never list or read another task's
        ::chmod(dir.c_str(), 0700);
        // the task account must be able to reach its own work dir through the agent's
        for (const std::string& d : {o_.work_dir, dir.substr(0, dir.rfind('/'))}) {
          struct stat st {};
          if (::stat(d.c_str(), &st) == 0) ::chmod(d.c_str(), (st.st_mode & 07777) | 0111);
        }
      }
    }
    std::vector<std::string> envs;
    for (auto& kv : env) envs.push_back(kv.first + "=" + kv.second);
    std::vector<char*> envp;
    for (auto& s : envs) envp.push_back(const_cast<char*>(s.c_str()));
    envp.push_back(nullptr);
    std::vector<std::string> args = {o_.python, "-m", "determined_1_amd.exec.harness"};
    if (spec["cmd"].is_array() && spec["cmd"].size() > 0) {
      args.clear();
      for (auto& a : spec["cmd"].as_array()) args.push_back(a.as_string());
    }
    std::vector<char*> argv;
    for (auto& a : args) argv.push_back(const_cast<char*>(a.c_str()));
    argv.push_back(nullptr);

    int out_pipe[2], err_pipe[2];
    if (pipe(out_pipe) != 0 || pipe(err_pipe) != 0) {
      State(cid, "Terminated", 1, "pipe failed");
      return;
    }
    // the child's failure messages are formatted here, before fork(): after it this multithreaded
    // process may only make async-signal-safe calls (no stdio locks, no strerror)
    char msg_uid[160], msg_dir[512];
    std::snprintf(msg_uid, sizeof msg_uid, "det-agent: cannot switch to uid %d gid %d\n", run_uid, run_gid);
    std::snprintf(msg_dir, sizeof msg_dir, "det-agent: cannot enter the work dir %s\n", dir.c_str());
    const size_t msg_uid_len = std::strlen(msg_uid), msg_dir_len = std::strlen(msg_dir);
    pid_t pid = -1;
    int zfd = spec["cmd"].is_array() && spec["cmd"].size() > 0
                  ? -1
                  : ZygoteSpawn(args, env, dir, out_pipe[1], err_pipe[1], &pid, run_uid, run_gid);
    if (zfd < 0) pid = fork();
    if (pid == 0) {
      setpgid(0, 0);
      dup2(out_pipe[1], 1);
      dup2(err_pipe[1], 2);
      close(out_pipe[0]);
      close(err_pipe[0]);
      if (run_uid >= 0 && static_cast<uid_t>(run_uid) != geteuid()) {
        const gid_t g = static_cast<gid_t>(run_gid);
        if (setgroups(1, &g) != 0 || setgid(g) != 0 || setuid(static_cast<uid_t>(run_uid)) != 0) {
          ssize_t w = ::write(2, msg_uid, msg_uid_len);
          (void)w;
          _exit(126);
        }
      }
      if (chdir(dir.c_str()) != 0) {
        ssize_t w = ::write(2, msg_dir, msg_dir_len);
        (void)w;
        _exit(127);
      }
      execvpe(argv[0], argv.data(), envp.data());
      _exit(127);
    }
    close(out_pipe[1]);
    close(err_pipe[1]);
    if (pid < 0) {
      State(cid, "Terminated", 1, "fork failed");
      return;
    }
    if (zfd < 0) setpgid(pid, pid);
    {
      std::lock_guard<std::mutex> g(mu_);
      Proc p;
      p.cid = cid;
      p.pid = pid;
      p.trial_id = spec.get_int("trial_id", 0);
      p.rank = static_cast<int>(spec.get_int("rank", 0));
      procs_[cid] = p;
    }
    Json running = Json::object();
    running["type"] = "ContainerStateChanged";
    running["container_id"] = cid;
    running["sent_us"] = NowUs();
    running["state"] = "Running";
    running["address"] = o_.advertise_host;
    Send(running);
    int64_t trial_id = spec.get_int("trial_id", 0);
    int rank = static_cast<int>(spec.get_int("rank", 0));
    std::string task_id = spec.get_string("task_id", "");
    std::thread t_out([=] { Pump(out_pipe[0], cid, trial_id, rank, "stdout", dir + "/stdout.log", task_id); });
    std::thread t_err([=] { Pump(err_pipe[0], cid, trial_id, rank, "stderr", dir + "/stderr.log", task_id); });
    int code = 1;
    if (zfd >= 0) {
      // the zygote owns (and reaps) the child; it sends "exit <code>" when it ends
      std::string line = ReadLine(zfd);
      close(zfd);
      if (line.rfind("exit ", 0) == 0) {
        code = std::atoi(line.c_str() + 5);
      } else {  // zygote gone: wait for the orphaned child by polling
        while (::kill(pid, 0) == 0) std::this_thread::sleep_for(std::chrono::milliseconds(200));
      }
    } else {
      int status = 0;
      waitpid(pid, &status, 0);
      code = WIFEXITED(status) ? WEXITSTATUS(status) : 128 + WTERMSIG(status);
    }
    t_out.join();
    t_err.join();
    {
      std::lock_guard<std::mutex> g(mu_);
      procs_.erase(cid);
    }
    State(cid, "Terminated", code, code == 0 ? "" : "container exited with code " + std::to_string(code));
  }

  void Pump(int fd, const std::string& cid, int64_t trial_id, int rank, const std::string& stdtype,
            const std::string& logfile, const std::string& task_id) {
    FILE* in = fdopen(fd, "r");
    std::ofstream lf(logfile, std::ios::app);
    char* line = nullptr;
    size_t cap = 0;
    ssize_t n;
    while ((n = getline(&line, &cap, in)) > 0) {
      std::string s(line, static_cast<size_t>(n));
      lf << s;
      lf.flush();
      while (!s.empty() && (s.back() == '\n' || s.back() == '\r')) s.pop_back();
      Json m = Json::object();
      m["type"] = "ContainerLog";
      m["container_id"] = cid;
      m["trial_id"] = trial_id;
      if (!task_id.empty()) m["task_id"] = task_id;
      m["rank"] = rank;
      m["stdtype"] = stdtype;
      m["log"] = s;
      Send(m);
    }
    free(line);
    fclose(in);
  }

  void Signal(const std::string& cid, const std::string& sig) {
    std::lock_guard<std::mutex> g(mu_);
    auto it = procs_.find(cid);
    if (it == procs_.end()) return;
    int s = sig == "SIGTERM" ? SIGTERM : sig == "SIGINT" ? SIGINT : SIGKILL;
    ::kill(-it->second.pid, s);
  }

  void KillAll() {
    std::lock_guard<std::mutex> g(mu_);
    for (auto& kv : procs_) ::kill(-kv.second.pid, SIGKILL);
  }

  Options o_;
  Json devices_;
  net::WsPtr ws_;
  std::mutex mu_;
  std::map<std::string, Proc> procs_;
  std::atomic<bool> stop_{false};
  pid_t zygote_pid_ = -1;
  std::string zygote_sock_;
};

Agent* g_agent = nullptr;
void OnSignal(int) {
  if (g_agent) std::thread([] { g_agent->Stop(); }).detach();
}

std::string SelfDir() {
  char buf[4096];
  ssize_t n = readlink("/proc/self/exe", buf, sizeof(buf) - 1);
  if (n <= 0) return ".";
  buf[n] = 0;
  std::string p = buf;
  return p.substr(0, p.rfind('/'));
}

}  // namespace

int main(int argc, char** argv) {
  Options o;
  char host[256] = {0};
  gethostname(host, sizeof(host) - 1);
  o.id = host;
  // framework root: <root>/determined_1_amd/_native/det-agent
  std::string self = SelfDir();
  o.framework_root = self + "/../..";
  for (int i = 1; i < argc; ++i) {
    std::string a = argv[i];
    auto next = [&]() -> std::string { return i + 1 < argc ? argv[++i] : ""; };
    if (a == "--master-host") o.master_host = next();
    else if (a == "--master-port") o.master_port = std::stoi(next());
    else if (a == "--agent-id") o.id = next();
    else if (a == "--resource-pool") o.pool = next();
    else if (a == "--label") o.label = next();
    else if (a == "--artificial-slots") o.artificial_slots = std::stoi(next());
    else if (a == "--slot-type") o.slot_type = next();
    else if (a == "--visible-gpus") o.visible_gpus = next();
    else if (a == "--python") o.python = next();
    else if (a == "--work-dir") o.work_dir = next();
    else if (a == "--framework-root") o.framework_root = next();
    else if (a == "--advertise-host") o.advertise_host = next();
    else if (a == "--master-cert-file") o.master_cert_file = next();
    else if (a == "--master-cert-name") o.master_cert_name = next();
    else if (a == "--master-tls") o.master_tls = true;
    else if (a == "--no-zygote") o.zygote = false;
    else if (a == "--detect-only") {
      std::printf("%s\n", DetectDevices(o).dump().c_str());
      return 0;
    } else {
      std::fprintf(stderr,
                   "usage: det-agent --master-host H --master-port P [--agent-id ID] [--resource-pool P]\n"
                   "                 [--label L] [--artificial-slots N] [--slot-type auto|gpu|cpu|none]\n"
                   "                 [--visible-gpus 0,1] [--python PY] [--work-dir DIR] [--no-zygote] [--detect-only]\n"
                   "                 [--master-tls] [--master-cert-file PEM] [--master-cert-name NAME]\n");
      return a == "-h" || a == "--help" ? 0 : 2;
    }
  }
  MkdirP(o.work_dir);
  signal(SIGPIPE, SIG_IGN);
  if (o.master_tls || !o.master_cert_file.empty()) {
    std::string err;
    if (!net::RegisterTlsEndpoint(o.master_host, o.master_port, o.master_cert_file, o.master_cert_name, &err)) {
      std::fprintf(stderr, "det-agent: %s\n", err.c_str());
      return 2;
    }
  }
  Agent agent(o);
  g_agent = &agent;
  signal(SIGINT, OnSignal);
  signal(SIGTERM, OnSignal);
  return agent.Run();
}
