// det-master entrypoint (reference master/cmd/determined-master/root.go + master/internal/config.go):
// layered config, lowest to highest precedence:
//   built-in defaults < config file (--config-file FILE.yaml|json, else /etc/determined/master.yaml
//   when present, or $DET_MASTER_CONFIG_FILE) < DET_* environment (viper-style: security.tls.cert ->
//   DET_SECURITY_TLS_CERT) < command-line flags.
#include <signal.h>
#include <unistd.h>

#include <cstdio>
#include <cstring>
#include <fstream>
#include <map>
#include <sstream>
#include <string>

#include "detcore/config.h"
#include "detcore/master.h"
#include "detcore/yaml.h"

extern char** environ;

static detcore::master::Master* g_master = nullptr;

static void OnSignal(int) {
  // Stop() is not async-signal-safe; hand it to a thread.
  static bool once = false;
  if (once) return;
  once = true;
  std::thread([] {
    if (g_master) g_master->Stop();
  }).detach();
}

static void Usage() {
  std::fprintf(stderr,
               "usage: det-master [--config-file FILE.yaml|FILE.json] [--host H] [--port P] [--store-dir DIR]\n"
               "                  [--tls-cert PEM --tls-key PEM]\n"
               "                  [--scheduler fair_share|priority|round_robin] [--fitting-policy best|worst]\n"
               "                  [--resource-pools a,b] [--checkpoint-host-path DIR] [--python PY]\n"
               "                  [--kubernetes-api HOST:PORT [--kubernetes-namespace NS]\n"
               "                   [--kubernetes-max-slots-per-pod N] [--kubernetes-slot-type gpu|cpu]\n"
               "                   [--kubernetes-cpu-slots-per-node N] [--kubernetes-master-host H]]\n");
}

static detcore::Json LoadConfigFile(const std::string& path) {
  std::ifstream f(path);
  if (!f) {
    std::fprintf(stderr, "cannot read config file %s\n", path.c_str());
    std::exit(2);
  }
  std::stringstream ss;
  ss << f.rdbuf();
  const std::string text = ss.str();
  size_t b = text.find_first_not_of(" \t\r\n");
  try {
    if (b != std::string::npos && text[b] == '{') return detcore::Json::parse(text);
    detcore::Json j = detcore::ParseYaml(text);
    return j.is_object() ? j : detcore::Json::object();
  } catch (const std::exception& e) {
    std::fprintf(stderr, "config file %s: %s\n", path.c_str(), e.what());
    std::exit(2);
  }
}

int main(int argc, char** argv) {
  detcore::Json cfgj = detcore::Json::object();  // command-line flags (highest precedence)
  std::string config_file;
  for (int i = 1; i < argc; ++i) {
    std::string a = argv[i];
    auto next = [&]() -> std::string {
      if (i + 1 >= argc) {
        Usage();
        std::exit(2);
      }
      return argv[++i];
    };
    if (a == "--config-file") {
      config_file = next();
    } else if (a == "--tls-cert") {
      cfgj["security"]["tls"]["cert"] = next();
    } else if (a == "--tls-key") {
      cfgj["security"]["tls"]["key"] = next();
    } else if (a == "--host") {
      cfgj["listen_host"] = next();
    } else if (a == "--port") {
      cfgj["port"] = std::stoi(next());
    } else if (a == "--store-dir") {
      cfgj["store_dir"] = next();
    } else if (a == "--scheduler") {
      cfgj["scheduler"]["type"] = next();
    } else if (a == "--fitting-policy") {
      cfgj["scheduler"]["fitting_policy"] = next();
    } else if (a == "--resource-pools") {
      detcore::Json pools = detcore::Json::array();
      std::stringstream ss(next());
      std::string p;
      while (std::getline(ss, p, ',')) pools.push_back(p);
      cfgj["resource_pools"] = pools;
    } else if (a == "--checkpoint-host-path") {
      detcore::Json cs = detcore::Json::object();
      cs["type"] = "shared_fs";
      cs["host_path"] = next();
      cfgj["checkpoint_storage"] = cs;
    } else if (a == "--python") {
      cfgj["python"] = next();
    } else if (a == "--provision-max") {
      cfgj["provisioner"]["max_instances"] = std::stoi(next());
    } else if (a == "--provision-slots") {
      cfgj["provisioner"]["slots_per_instance"] = std::stoi(next());
    } else if (a == "--provision-idle-ms") {
      cfgj["provisioner"]["max_idle_agent_period_ms"] = std::stoi(next());
    } else if (a == "--kubernetes-api") {
      cfgj["resource_manager"]["type"] = "kubernetes";
      cfgj["resource_manager"]["api_server"] = next();
    } else if (a == "--kubernetes-namespace") {
      cfgj["resource_manager"]["namespace"] = next();
    } else if (a == "--kubernetes-max-slots-per-pod") {
      cfgj["resource_manager"]["max_slots_per_pod"] = std::stoi(next());
    } else if (a == "--kubernetes-slot-type") {
      cfgj["resource_manager"]["slot_type"] = next();
    } else if (a == "--kubernetes-cpu-slots-per-node") {
      cfgj["resource_manager"]["cpu_slots_per_node"] = std::stoi(next());
    } else if (a == "--kubernetes-python") {
      cfgj["resource_manager"]["python"] = next();
    } else if (a == "--kubernetes-master-host") {
      cfgj["resource_manager"]["master_service_host"] = next();
    } else if (a == "--telemetry-file") {
      cfgj["telemetry"]["file"] = next();
      cfgj["telemetry"]["enabled"] = true;
    } else if (a == "--require-auth") {
      cfgj["security"]["authentication"] = true;
    } else if (a == "--scheduler-tick-ms") {
      cfgj["scheduler_tick_ms"] = std::stod(next());
    } else if (a == "-h" || a == "--help") {
      Usage();
      return 0;
    } else {
      std::fprintf(stderr, "unknown flag %s\n", a.c_str());
      Usage();
      return 2;
    }
  }
  if (config_file.empty()) {
    const char* e = std::getenv("DET_MASTER_CONFIG_FILE");
    if (e && *e) config_file = e;
    else if (access("/etc/determined/master.yaml", R_OK) == 0) config_file = "/etc/determined/master.yaml";
  }
  detcore::Json file = config_file.empty() ? detcore::Json::object() : LoadConfigFile(config_file);
  std::map<std::string, std::string> env;
  for (char** e = environ; e && *e; ++e) {
    std::string kv = *e;
    auto eq = kv.find('=');
    if (eq != std::string::npos && kv.compare(0, 4, "DET_") == 0) env[kv.substr(0, eq)] = kv.substr(eq + 1);
  }
  const detcore::Json defaults = detcore::MasterConfig().ToJson();
  const detcore::Json base = detcore::DeepMerge(defaults, file);
  const detcore::Json envj = detcore::EnvOverlay(base, detcore::MasterConfig::EnvPaths(), env);
  cfgj = detcore::DeepMerge(detcore::DeepMerge(base, envj), cfgj);
  signal(SIGPIPE, SIG_IGN);
  detcore::master::Master m(detcore::MasterConfig::FromJson(cfgj));
  g_master = &m;
  signal(SIGINT, OnSignal);
  signal(SIGTERM, OnSignal);
  int port = m.Start();
  std::printf("det-master listening on port %d\n", port);
  std::fflush(stdout);
  m.Wait();
  return 0;
}
