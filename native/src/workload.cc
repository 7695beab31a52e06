#include "detcore/workload.h"

#include <stdexcept>
#include <tuple>

namespace detcore {

const char* WorkloadKindName(Workload::Kind k) {
  switch (k) {
    case Workload::Kind::RunStep: return "RUN_STEP";
    case Workload::Kind::ComputeValidationMetrics: return "COMPUTE_VALIDATION_METRICS";
    case Workload::Kind::CheckpointModel: return "CHECKPOINT_MODEL";
    case Workload::Kind::Terminate: return "TERMINATE";
  }
  return "RUN_STEP";
}

static Workload::Kind ParseKind(const std::string& s) {
  if (s == "RUN_STEP") return Workload::Kind::RunStep;
  if (s == "COMPUTE_VALIDATION_METRICS") return Workload::Kind::ComputeValidationMetrics;
  if (s == "CHECKPOINT_MODEL") return Workload::Kind::CheckpointModel;
  if (s == "TERMINATE") return Workload::Kind::Terminate;
  throw std::invalid_argument("unknown workload kind " + s);
}

bool Workload::operator<(const Workload& o) const {
  return std::make_tuple(static_cast<int>(kind), experiment_id, trial_id, step_id, num_batches, total_batches_processed) <
         std::make_tuple(static_cast<int>(o.kind), o.experiment_id, o.trial_id, o.step_id, o.num_batches,
                         o.total_batches_processed);
}

Json Workload::ToJson() const {
  Json j = Json::object();
  j["kind"] = WorkloadKindName(kind);
  j["experiment_id"] = experiment_id;
  j["trial_id"] = trial_id;
  j["step_id"] = step_id;
  j["num_batches"] = num_batches;
  j["total_batches_processed"] = total_batches_processed;
  return j;
}

Workload Workload::FromJson(const Json& j) {
  Workload w;
  w.kind = ParseKind(j.at("kind").as_string());
  w.experiment_id = j.get_int("experiment_id", 0);
  w.trial_id = j.get_int("trial_id", 0);
  w.step_id = j.get_int("step_id", 0);
  w.num_batches = j.get_int("num_batches", 0);
  w.total_batches_processed = j.get_int("total_batches_processed", 0);
  return w;
}

std::string Workload::String() const {
  std::string nb = kind == Kind::RunStep ? " (" + std::to_string(num_batches) + " Batches)" : "";
  return std::string("<") + WorkloadKindName(kind) + nb + ": (" + std::to_string(experiment_id) + "," +
         std::to_string(trial_id) + "," + std::to_string(step_id) + ")>";
}

Json CompletedMessage::ToJson() const {
  Json j = Json::object();
  j["type"] = "WORKLOAD_COMPLETED";
  j["workload"] = workload.ToJson();
  j["start_time"] = start_time;
  j["end_time"] = end_time;
  j["metrics"] = metrics;
  if (exited_reason) j["exited_reason"] = ExitedReasonName(*exited_reason);
  return j;
}

CompletedMessage CompletedMessage::FromJson(const Json& j) {
  CompletedMessage m;
  m.workload = Workload::FromJson(j.at("workload"));
  m.start_time = j.get_string("start_time", "");
  m.end_time = j.get_string("end_time", "");
  m.metrics = j["metrics"];
  if (j["exited_reason"].is_string()) m.exited_reason = ParseExitedReason(j["exited_reason"].as_string());
  return m;
}

}  // namespace detcore
