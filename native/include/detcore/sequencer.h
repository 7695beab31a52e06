// Trial workload sequencer: turns searcher Runnable ops (Train/Validate/Checkpoint) into harness
// workloads with the reference's priorities (reference
// master/internal/trial_workload_sequencer.go):
//   initial validation -> post-graceful-stop checkpoint -> post-validation checkpoint (policy) ->
//   min_validation_period -> min_checkpoint_period -> the current op
// A Validate op is preceded by a checkpoint if batches are un-checkpointed; a train step is
// min(left, until-val, until-ckpt, scheduling_unit) batches.  State is snapshotted at every
// checkpoint so a failed trial rolls back to exactly its last checkpoint.
#pragma once

#include <map>
#include <optional>
#include <string>
#include <vector>

#include "detcore/json.h"
#include "detcore/searcher.h"
#include "detcore/workload.h"

namespace detcore {

struct SequencerConfig {
  int64_t experiment_id = 0;
  bool perform_initial_validation = false;
  std::string checkpoint_policy = "best";  // best | all | none
  Length min_validation_period;             // units == 0: disabled
  Length min_checkpoint_period;
  Unit default_unit = Unit::Batches;
  int64_t global_batch_size = 1;
  int64_t records_per_epoch = 0;
  int64_t scheduling_unit = 100;
  static SequencerConfig FromExperimentConfig(const Json& cfg, int64_t experiment_id, int64_t global_batch_size);
};

class TrialWorkloadSequencer {
 public:
  TrialWorkloadSequencer(SequencerConfig cfg, Json first_checkpoint = Json());

  void SetTrialID(int64_t trial_id) {
    trial_id_ = trial_id;
    trial_id_valid_ = true;
  }
  void OperationRequested(const Op& op);  // Train / Validate / Checkpoint
  bool UpToDate() const;
  Workload NextWorkload() const;  // throws if UpToDate()
  // Returns the searcher op that completed (if any) and its metrics.
  struct Completion {
    std::optional<Op> op;
    Json metrics;
  };
  Completion WorkloadCompleted(const CompletedMessage& msg, bool is_best_validation);
  Completion CompleteCachedCheckpoints();
  std::optional<Workload> PrecloseCheckpointWorkload() const;
  Workload TerminateWorkload() const;
  int64_t RollBack();  // to the last checkpoint snapshot; returns the step id
  const Json& LatestCheckpoint() const { return st_.latest_checkpoint; }
  int64_t TotalBatchesProcessed() const { return st_.total_batches; }
  int64_t CurStepID() const { return st_.cur_step_id; }
  size_t NumOps() const { return ops_.size(); }
  size_t CurOpIndex() const { return st_.cur_op_idx; }
  Json DebugState() const;

 private:
  struct State {
    int64_t batches_towards_op = 0, batches_since_val = 0, batches_since_ckpt = 0, total_batches = 0;
    bool need_initial_validation = false, need_post_validation_ckpt = false, exiting_early = false,
         graceful_stop = false;
    size_t cur_op_idx = 0;
    int64_t cur_step_id = 0;
    Json latest_checkpoint;
    std::map<Workload, CompletedMessage> cached_checkpoints;
  };
  Completion RunStepCompleted(const CompletedMessage& msg);
  Completion ValidationCompleted(const CompletedMessage& msg, bool is_best);
  Completion CheckpointCompleted(const CompletedMessage& msg);
  Workload Train(int64_t n) const;
  Workload Validate() const;
  Workload Checkpoint() const;
  bool MinValidationNeeded() const;
  bool MinCheckpointNeeded() const;
  int64_t BatchesUntilValNeeded() const;
  int64_t BatchesUntilCkptNeeded() const;
  bool PostGracefulStopCheckpointNeeded() const { return st_.graceful_stop && st_.batches_since_ckpt != 0; }
  bool PostValidationCheckpointNeeded() const { return st_.need_post_validation_ckpt && st_.batches_since_ckpt != 0; }
  UnitContext ctx() const;

  SequencerConfig cfg_;
  std::vector<Op> ops_;
  State st_;
  State snapshot_;
  int64_t trial_id_ = 0;
  bool trial_id_valid_ = false;
};

}  // namespace detcore
