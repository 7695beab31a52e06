#include "detcore/sequencer.h"

#include <algorithm>
#include <climits>
#include <stdexcept>

namespace detcore {

SequencerConfig SequencerConfig::FromExperimentConfig(const Json& cfg, int64_t experiment_id,
                                                      int64_t global_batch_size) {
  SequencerConfig c;
  c.experiment_id = experiment_id;
  c.perform_initial_validation = cfg.get_bool("perform_initial_validation", false);
  c.checkpoint_policy = cfg.get_string("checkpoint_policy", "best");
  if (cfg["min_validation_period"].is_object() && cfg["min_validation_period"].size() == 1)
    c.min_validation_period = Length::FromJson(cfg["min_validation_period"]);
  if (cfg["min_checkpoint_period"].is_object() && cfg["min_checkpoint_period"].size() == 1)
    c.min_checkpoint_period = Length::FromJson(cfg["min_checkpoint_period"]);
  const Json& s = cfg["searcher"];
  for (const char* k : {"max_length", "length_per_round", "budget"}) {
    if (s.has(k)) {
      c.default_unit = Length::FromJson(s[k]).unit;
      break;
    }
  }
  c.global_batch_size = std::max<int64_t>(1, global_batch_size);
  c.records_per_epoch = cfg.get_int("records_per_epoch", 0);
  c.scheduling_unit = cfg.get_int("scheduling_unit", 100);
  return c;
}

TrialWorkloadSequencer::TrialWorkloadSequencer(SequencerConfig cfg, Json first_checkpoint) : cfg_(std::move(cfg)) {
  st_.need_initial_validation = cfg_.perform_initial_validation;
  st_.latest_checkpoint = std::move(first_checkpoint);
  snapshot_ = st_;
}

UnitContext TrialWorkloadSequencer::ctx() const {
  return UnitContext{cfg_.default_unit, cfg_.global_batch_size, cfg_.records_per_epoch};
}

void TrialWorkloadSequencer::OperationRequested(const Op& op) {
  if (!op.runnable()) throw std::invalid_argument("illegal workload for trialWorkloadSequencer: " + op.String());
  ops_.push_back(op);
}

bool TrialWorkloadSequencer::UpToDate() const {
  return ops_.size() == st_.cur_op_idx || (st_.exiting_early && !PostGracefulStopCheckpointNeeded());
}

Workload TrialWorkloadSequencer::Train(int64_t n) const {
  Workload w;
  w.kind = Workload::Kind::RunStep;
  w.experiment_id = cfg_.experiment_id;
  w.trial_id = trial_id_;
  w.step_id = st_.cur_step_id + 1;
  w.num_batches = n;
  w.total_batches_processed = st_.total_batches;
  return w;
}

Workload TrialWorkloadSequencer::Validate() const {
  Workload w;
  w.kind = Workload::Kind::ComputeValidationMetrics;
  w.experiment_id = cfg_.experiment_id;
  w.trial_id = trial_id_;
  w.step_id = st_.cur_step_id;
  w.total_batches_processed = st_.total_batches;
  return w;
}

Workload TrialWorkloadSequencer::Checkpoint() const {
  Workload w = Validate();
  w.kind = Workload::Kind::CheckpointModel;
  return w;
}

Workload TrialWorkloadSequencer::TerminateWorkload() const {
  Workload w;
  w.kind = Workload::Kind::Terminate;
  w.experiment_id = cfg_.experiment_id;
  w.trial_id = trial_id_;
  w.step_id = st_.cur_step_id;
  return w;
}

bool TrialWorkloadSequencer::MinValidationNeeded() const {
  if (cfg_.min_validation_period.units == 0) return false;
  return EqualWithinBatch(cfg_.min_validation_period, st_.batches_since_val, ctx());
}

bool TrialWorkloadSequencer::MinCheckpointNeeded() const {
  if (cfg_.min_checkpoint_period.units == 0) return false;
  return EqualWithinBatch(cfg_.min_checkpoint_period, st_.batches_since_ckpt, ctx());
}

int64_t TrialWorkloadSequencer::BatchesUntilValNeeded() const {
  if (cfg_.min_validation_period.units == 0) return INT32_MAX;
  return ToNearestBatch(cfg_.min_validation_period, ctx()) - st_.batches_since_val;
}

int64_t TrialWorkloadSequencer::BatchesUntilCkptNeeded() const {
  if (cfg_.min_checkpoint_period.units == 0) return INT32_MAX;
  return ToNearestBatch(cfg_.min_checkpoint_period, ctx()) - st_.batches_since_ckpt;
}

Workload TrialWorkloadSequencer::NextWorkload() const {
  if (UpToDate()) throw std::logic_error("cannot call NextWorkload() when UpToDate()");
  if (!trial_id_valid_) throw std::logic_error("cannot call NextWorkload() before SetTrialID()");
  if (st_.need_initial_validation) return Validate();
  if (PostGracefulStopCheckpointNeeded()) return Checkpoint();
  if (PostValidationCheckpointNeeded()) return Checkpoint();
  if (MinValidationNeeded()) return Validate();
  if (MinCheckpointNeeded()) return Checkpoint();
  const Op& op = ops_[st_.cur_op_idx];
  switch (op.kind) {
    case Op::Kind::Validate:
      if (st_.batches_since_ckpt != 0) return Checkpoint();
      return Validate();
    case Op::Kind::Checkpoint:
      return Checkpoint();
    case Op::Kind::Train: {
      int64_t left = ToNearestBatch(op.length, ctx()) - st_.batches_towards_op;
      int64_t n = std::min({left, BatchesUntilValNeeded(), BatchesUntilCkptNeeded(), cfg_.scheduling_unit});
      return Train(std::max<int64_t>(n, 1));
    }
    default:
      throw std::logic_error("unexpected op type determining workload");
  }
}

std::optional<Workload> TrialWorkloadSequencer::PrecloseCheckpointWorkload() const {
  if (st_.batches_since_ckpt == 0 || !trial_id_valid_) return std::nullopt;
  return Checkpoint();
}

int64_t TrialWorkloadSequencer::RollBack() {
  st_ = snapshot_;
  return st_.cur_step_id;
}

TrialWorkloadSequencer::Completion TrialWorkloadSequencer::CompleteCachedCheckpoints() {
  if (UpToDate()) return {};
  Workload w = NextWorkload();
  auto it = st_.cached_checkpoints.find(w);
  if (it == st_.cached_checkpoints.end()) return {};
  CompletedMessage msg = it->second;
  st_.cached_checkpoints.erase(it);
  return WorkloadCompleted(msg, false);
}

TrialWorkloadSequencer::Completion TrialWorkloadSequencer::WorkloadCompleted(const CompletedMessage& msg,
                                                                             bool is_best_validation) {
  if (UpToDate()) {
    if (msg.workload.kind != Workload::Kind::CheckpointModel)
      throw std::logic_error("illegal non-checkpoint workload completed message received: " + msg.workload.String());
  } else {
    Workload w = NextWorkload();
    if (msg.workload != w && msg.workload.kind != Workload::Kind::CheckpointModel)
      throw std::logic_error("illegal completed message received: expected checkpoint or " + w.String() + ", got " +
                             msg.workload.String());
  }
  if (msg.exited_reason) {
    st_.exiting_early = true;
    if (*msg.exited_reason == ExitedReason::UserCanceled || *msg.exited_reason == ExitedReason::InvalidHP)
      st_.graceful_stop = true;
    else
      return {};
  }
  switch (msg.workload.kind) {
    case Workload::Kind::RunStep: return RunStepCompleted(msg);
    case Workload::Kind::CheckpointModel: return CheckpointCompleted(msg);
    case Workload::Kind::ComputeValidationMetrics: return ValidationCompleted(msg, is_best_validation);
    default: throw std::logic_error("invalid operation for trialWorkloadSequencer");
  }
}

TrialWorkloadSequencer::Completion TrialWorkloadSequencer::RunStepCompleted(const CompletedMessage& msg) {
  st_.cur_step_id++;
  int64_t n = msg.workload.num_batches;
  st_.total_batches += n;
  st_.batches_towards_op += n;
  st_.batches_since_val += n;
  st_.batches_since_ckpt += n;
  const Op& op = ops_[st_.cur_op_idx];
  if (op.kind == Op::Kind::Train && EqualWithinBatch(op.length, st_.batches_towards_op, ctx())) {
    st_.cur_op_idx++;
    st_.batches_towards_op = 0;
    return Completion{op, Json::object()};
  }
  return {};
}

TrialWorkloadSequencer::Completion TrialWorkloadSequencer::ValidationCompleted(const CompletedMessage& msg,
                                                                               bool is_best) {
  st_.batches_since_val = 0;
  st_.need_initial_validation = false;
  if (st_.batches_since_ckpt != 0) {
    if (cfg_.checkpoint_policy == "all") st_.need_post_validation_ckpt = true;
    else if (cfg_.checkpoint_policy == "best" && is_best) st_.need_post_validation_ckpt = true;
  }
  if (st_.cur_op_idx < ops_.size() && ops_[st_.cur_op_idx].kind == Op::Kind::Validate) {
    Op op = ops_[st_.cur_op_idx];
    st_.cur_op_idx++;
    if (st_.batches_since_ckpt == 0) snapshot_ = st_;
    return Completion{op, msg.metrics};
  }
  if (st_.batches_since_ckpt == 0) snapshot_ = st_;
  return {};
}

TrialWorkloadSequencer::Completion TrialWorkloadSequencer::CheckpointCompleted(const CompletedMessage& msg) {
  st_.batches_since_ckpt = 0;
  st_.need_post_validation_ckpt = false;
  st_.latest_checkpoint = msg.metrics;
  Completion out;
  if (!UpToDate() && ops_[st_.cur_op_idx].kind == Op::Kind::Checkpoint) {
    out = Completion{ops_[st_.cur_op_idx], msg.metrics};
    st_.cur_op_idx++;
  } else {
    st_.cached_checkpoints[msg.workload] = msg;
  }
  snapshot_ = st_;  // deferred snapshot in the reference
  return out;
}

Json TrialWorkloadSequencer::DebugState() const {
  Json j = Json::object();
  j["batches_towards_op"] = st_.batches_towards_op;
  j["batches_since_val"] = st_.batches_since_val;
  j["batches_since_ckpt"] = st_.batches_since_ckpt;
  j["total_batches"] = st_.total_batches;
  j["cur_op_idx"] = static_cast<int64_t>(st_.cur_op_idx);
  j["cur_step_id"] = st_.cur_step_id;
  j["num_ops"] = static_cast<int64_t>(ops_.size());
  j["exiting_early"] = st_.exiting_early;
  j["graceful_stop"] = st_.graceful_stop;
  return j;
}

}  // namespace detcore
