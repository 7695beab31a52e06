// Master<->harness workload protocol value types (SURVEY §2.6 C-ws / C-done;
// reference master/pkg/workload/{workload,completed_message}.go).
#pragma once

#include <cstdint>
#include <optional>
#include <string>

#include "detcore/json.h"
#include "detcore/searcher.h"

namespace detcore {

struct Workload {
  enum class Kind { RunStep = 1, ComputeValidationMetrics = 2, CheckpointModel = 3, Terminate = 4 };
  Kind kind = Kind::RunStep;
  int64_t experiment_id = 0;
  int64_t trial_id = 0;
  int64_t step_id = 0;
  int64_t num_batches = 0;
  int64_t total_batches_processed = 0;

  bool operator==(const Workload& o) const {
    return kind == o.kind && experiment_id == o.experiment_id && trial_id == o.trial_id && step_id == o.step_id &&
           num_batches == o.num_batches && total_batches_processed == o.total_batches_processed;
  }
  bool operator!=(const Workload& o) const { return !(*this == o); }
  bool operator<(const Workload& o) const;
  Json ToJson() const;
  static Workload FromJson(const Json& j);
  std::string String() const;
};

const char* WorkloadKindName(Workload::Kind k);

struct CompletedMessage {
  Workload workload;
  std::string start_time, end_time;
  Json metrics;  // RUN_STEP: {batch_metrics, avg_metrics, num_inputs}; VALIDATION: {num_inputs,
                 // validation_metrics}; CHECKPOINT: {uuid, resources, framework, format}
  std::optional<ExitedReason> exited_reason;
  Json ToJson() const;
  static CompletedMessage FromJson(const Json& j);
};

}  // namespace detcore
