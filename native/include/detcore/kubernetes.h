// Kubernetes resource manager (reference master/internal/resourcemanagers/
// kubernetes_resource_manager.go, master/internal/kubernetes/{pods,pod,spec,informer,log}.go).
//
// MI355X-first shape: the cluster's AMD GPUs (node allocatable `amd.com/gpu`, the ROCm device
// plugin's resource) are exposed to the master's ordinary scheduler as *virtual agents* -- one per
// node and per `max_slots_per_pod` group of that node's GPUs -- so fair-share / priority /
// round-robin and gang fitting work unchanged, and a trial that needs more GPUs than one pod may
// hold is split into one pod per group exactly like the reference's `max_slots_per_pod`.  The
// master -> agent protocol of a virtual agent is translated into Kubernetes REST calls:
//
//   StartContainer  -> ConfigMap (the container spec) + Pod (requests/limits amd.com/gpu: n,
//                      pinned to the node via nodeSelector, command = pod_entrypoint + harness)
//   SignalContainer -> DELETE pod (grace 0 for SIGKILL)
//   pod phase       -> ContainerStateChanged (Pending=Starting, Running (+podIP)=Running,
//                      Succeeded/Failed (+exit code) or vanished = Terminated)
//   pod log follow  -> ContainerLog lines (the reference's Fluent Bit / pod log path)
//
// Talks plain HTTP to the API server (`kubectl proxy` or an in-cluster sidecar); no client-go.
#pragma once

#include <atomic>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "detcore/json.h"

namespace detcore {
namespace master {

class Master;
struct AgentConn;

struct KubeConfig {
  std::string host = "127.0.0.1";  // API server (kubectl proxy) host:port
  int port = 8001;
  std::string ns = "default";
  int max_slots_per_pod = 8;
  std::string slot_type = "gpu";           // gpu | cpu
  std::string slot_resource = "amd.com/gpu";
  int cpu_slots_per_node = 1;              // slot_type=cpu: slots advertised per node
  std::string image = "determined-mi355x:rocm";
  std::string python = "python3";
  std::string pool;                        // resource pool the virtual agents join ("" = default)
  std::string master_host;                 // address pods use to reach the master
  int master_port = 0;
  int poll_ms = 250;
  static KubeConfig FromJson(const Json& j);
};

class KubernetesRM {
 public:
  KubernetesRM(Master* m, KubeConfig cfg);
  ~KubernetesRM();
  // Reads node capacity, registers the virtual agents and starts the pod watcher.
  void Start();
  void Stop();
  Json Summary() const;

 private:
  struct Pod {
    std::string cid, name, agent, task_id;
    int64_t trial_id = 0;
    int rank = 0;
    std::string reported;  // last state sent to the master
    bool deleting = false;
    std::shared_ptr<std::thread> logs;
    std::shared_ptr<std::atomic<bool>> logs_done;
  };
  bool FromMaster(const std::string& agent, const Json& msg);
  void CreatePod(const std::string& agent, const Json& msg);
  void DeletePod(const std::string& cid, int grace_seconds);
  void WatchLoop();
  void FollowLogs(Pod p, std::shared_ptr<std::atomic<bool>> done);
  void Report(const std::string& agent, const Json& msg);
  std::string Path(const std::string& kind, const std::string& name = "") const;

  Master* m_;
  KubeConfig cfg_;
  std::vector<std::shared_ptr<AgentConn>> agents_;
  mutable std::mutex mu_;
  std::map<std::string, Pod> pods_;  // by container id
  std::atomic<bool> stop_{false};
  std::thread watcher_;
};

}  // namespace master
}  // namespace detcore
