// Sequencer scenarios (cf. reference master/internal/trial_workload_sequencer_test.go).
#include "detcore/sequencer.h"
#include "test_util.h"

using namespace detcore;

namespace {

SequencerConfig cfg(int64_t min_val, int64_t min_ckpt, const char* policy = "none", int64_t unit = 100) {
  SequencerConfig c;
  c.experiment_id = 1;
  c.checkpoint_policy = policy;
  c.min_validation_period = Length(Unit::Batches, min_val);
  c.min_checkpoint_period = Length(Unit::Batches, min_ckpt);
  c.global_batch_size = 64;
  c.scheduling_unit = unit;
  return c;
}

CompletedMessage done(const Workload& w, Json metrics = Json::object()) {
  CompletedMessage m;
  m.workload = w;
  m.metrics = std::move(metrics);
  return m;
}

Json ckpt_metrics(const char* uuid) {
  Json j = Json::object();
  j["uuid"] = uuid;
  return j;
}

}  // namespace

TEST(sequencer_min_periods_and_scheduling_unit) {
  NpRand rand(0);
  Op create = Op::Create(rand, Json::object());
  TrialWorkloadSequencer s(cfg(200, 400));
  s.SetTrialID(1);
  s.OperationRequested(Op::Train(create.request_id, Length(Unit::Batches, 500)));
  s.OperationRequested(Op::Validate(create.request_id));
  s.OperationRequested(Op::Checkpoint(create.request_id));
  // two 100-batch steps, then the min-validation validation
  Workload w = s.NextWorkload();
  EXPECT(w.kind == Workload::Kind::RunStep && w.num_batches == 100 && w.step_id == 1 && w.total_batches_processed == 0);
  EXPECT(!s.WorkloadCompleted(done(w), false).op);
  w = s.NextWorkload();
  EXPECT(w.kind == Workload::Kind::RunStep && w.step_id == 2 && w.total_batches_processed == 100);
  s.WorkloadCompleted(done(w), false);
  w = s.NextWorkload();
  EXPECT(w.kind == Workload::Kind::ComputeValidationMetrics && w.step_id == 2);
  s.WorkloadCompleted(done(w), false);
  // steps 3,4 -> min checkpoint at 400
  for (int i = 3; i <= 4; ++i) {
    w = s.NextWorkload();
    EXPECT(w.kind == Workload::Kind::RunStep && w.step_id == i);
    s.WorkloadCompleted(done(w), false);
  }
  w = s.NextWorkload();
  EXPECT(w.kind == Workload::Kind::ComputeValidationMetrics);  // 200 since last val
  s.WorkloadCompleted(done(w), false);
  w = s.NextWorkload();
  EXPECT(w.kind == Workload::Kind::CheckpointModel && w.step_id == 4);
  s.WorkloadCompleted(done(w, ckpt_metrics("c4")), false);
  // last train step completes the Train op
  w = s.NextWorkload();
  EXPECT(w.kind == Workload::Kind::RunStep && w.step_id == 5 && w.num_batches == 100);
  auto c = s.WorkloadCompleted(done(w), false);
  EXPECT(c.op && c.op->kind == Op::Kind::Train);
  // Validate op: un-checkpointed batches -> checkpoint first
  w = s.NextWorkload();
  EXPECT(w.kind == Workload::Kind::CheckpointModel && w.step_id == 5);
  s.WorkloadCompleted(done(w, ckpt_metrics("c5")), false);
  w = s.NextWorkload();
  EXPECT(w.kind == Workload::Kind::ComputeValidationMetrics);
  c = s.WorkloadCompleted(done(w), false);
  EXPECT(c.op && c.op->kind == Op::Kind::Validate);
  // Checkpoint op: the cached step-5 checkpoint completes it without a new workload
  EXPECT(!s.UpToDate());
  c = s.CompleteCachedCheckpoints();
  EXPECT(c.op && c.op->kind == Op::Kind::Checkpoint);
  EXPECT(s.UpToDate());
  EXPECT_EQ(s.LatestCheckpoint()["uuid"].as_string(), std::string("c5"));
}

TEST(sequencer_rollback_to_last_checkpoint) {
  NpRand rand(0);
  Op create = Op::Create(rand, Json::object());
  TrialWorkloadSequencer s(cfg(0, 0, "none", 10));
  s.SetTrialID(7);
  s.OperationRequested(Op::Train(create.request_id, Length(Unit::Batches, 30)));
  s.OperationRequested(Op::Checkpoint(create.request_id));
  Workload w = s.NextWorkload();
  s.WorkloadCompleted(done(w), false);
  auto pc = s.PrecloseCheckpointWorkload();
  EXPECT(pc.has_value() && pc->step_id == 1 && pc->total_batches_processed == 10);
  s.WorkloadCompleted(done(*pc, ckpt_metrics("a")), false);
  w = s.NextWorkload();
  s.WorkloadCompleted(done(w), false);
  EXPECT_EQ(s.TotalBatchesProcessed(), 20);
  int64_t step = s.RollBack();
  EXPECT_EQ(step, 1);
  EXPECT_EQ(s.TotalBatchesProcessed(), 10);
  w = s.NextWorkload();
  EXPECT(w.kind == Workload::Kind::RunStep && w.step_id == 2 && w.total_batches_processed == 10 && w.num_batches == 10);
}

TEST(sequencer_best_policy_post_validation_checkpoint) {
  NpRand rand(0);
  Op create = Op::Create(rand, Json::object());
  TrialWorkloadSequencer s(cfg(5, 0, "best", 5));
  s.SetTrialID(1);
  s.OperationRequested(Op::Train(create.request_id, Length(Unit::Batches, 10)));
  Workload w = s.NextWorkload();
  s.WorkloadCompleted(done(w), false);
  w = s.NextWorkload();
  EXPECT(w.kind == Workload::Kind::ComputeValidationMetrics);
  s.WorkloadCompleted(done(w), /*is_best=*/true);
  w = s.NextWorkload();
  EXPECT(w.kind == Workload::Kind::CheckpointModel);
}

TEST(sequencer_graceful_stop_checkpoints_then_up_to_date) {
  NpRand rand(0);
  Op create = Op::Create(rand, Json::object());
  TrialWorkloadSequencer s(cfg(0, 0, "none", 5));
  s.SetTrialID(1);
  s.OperationRequested(Op::Train(create.request_id, Length(Unit::Batches, 100)));
  Workload w = s.NextWorkload();
  CompletedMessage m = done(w);
  m.exited_reason = ExitedReason::UserCanceled;
  s.WorkloadCompleted(m, false);
  EXPECT(!s.UpToDate());
  w = s.NextWorkload();
  EXPECT(w.kind == Workload::Kind::CheckpointModel);
  s.WorkloadCompleted(done(w, ckpt_metrics("g")), false);
  EXPECT(s.UpToDate());
}

TEST(json_roundtrip_and_ordering) {
  Json j = Json::parse(R"({"b": [1, 2.5, "x"], "a": {"z": null, "y": true}, "c": -0.000001})");
  EXPECT_EQ(j.dump(), std::string(R"({"a":{"y":true,"z":null},"b":[1,2.5,"x"],"c":-0.000001})"));
  Json k = j;
  k["a"]["y"] = false;  // copy-on-write: j unchanged
  EXPECT(j["a"]["y"].as_bool());
  EXPECT_EQ(Json::parse("1e21").dump(), std::string("1e+21"));
}

TEST(length_conversions) {
  UnitContext c{Unit::Records, 64, 6400};
  EXPECT_EQ(ToNearestBatch(Length(Unit::Records, 640), c), 10);
  EXPECT_EQ(ToNearestBatch(Length(Unit::Epochs, 2), c), 200);
  EXPECT(EqualWithinBatch(Length(Unit::Records, 650), 10, c));
  EXPECT(!EqualWithinBatch(Length(Unit::Records, 704), 10, c));
}

// ---- named counterparts of master/internal/trial_workload_sequencer_test.go ----------------
namespace {
Workload W(Workload::Kind k, int64_t step, int64_t nb, int64_t total) {
  Workload w;
  w.kind = k;
  w.experiment_id = 1;
  w.trial_id = 1;
  w.step_id = step;
  w.num_batches = nb;
  w.total_batches_processed = total;
  return w;
}
bool Same(const Workload& a, const Workload& b) {
  return a.kind == b.kind && a.experiment_id == b.experiment_id && a.trial_id == b.trial_id && a.step_id == b.step_id &&
         a.num_batches == b.num_batches && a.total_batches_processed == b.total_batches_processed;
}
}  // namespace

TEST(TestTrialWorkloadSequencer) {
  const int64_t su = 100;  // DefaultExperimentConfig().SchedulingUnit
  using K = Workload::Kind;
  Workload train1 = W(K::RunStep, 1, su, 0), train2 = W(K::RunStep, 2, su, su), train3 = W(K::RunStep, 3, su, 2 * su),
           train4 = W(K::RunStep, 4, su, 3 * su), train5 = W(K::RunStep, 5, su, 4 * su);
  Workload ckpt1 = W(K::CheckpointModel, 1, 0, su), ckpt2 = W(K::CheckpointModel, 2, 0, 2 * su),
           ckpt4 = W(K::CheckpointModel, 4, 0, 4 * su), ckpt5 = W(K::CheckpointModel, 5, 0, 5 * su);
  Workload val2 = W(K::ComputeValidationMetrics, 2, 0, 2 * su), val4 = W(K::ComputeValidationMetrics, 4, 0, 4 * su),
           val5 = W(K::ComputeValidationMetrics, 5, 0, 5 * su);
  NpRand rand(0);
  Json hp = Json::object();
  hp["global_batch_size"] = 64;
  Op create = Op::Create(rand, hp);
  Op train = Op::Train(create.request_id, Length(Unit::Batches, 500));
  Op validate = Op::Validate(create.request_id), checkpoint = Op::Checkpoint(create.request_id);
  TrialWorkloadSequencer s(cfg(200, 400, "none", su));
  EXPECT(s.UpToDate());
  s.OperationRequested(train);
  EXPECT(!s.UpToDate());
  s.OperationRequested(validate);
  s.OperationRequested(checkpoint);
  bool threw = false;
  try { s.NextWorkload(); } catch (const std::logic_error&) { threw = true; }
  EXPECT(threw);  // before SetTrialID
  s.SetTrialID(1);
  EXPECT(Same(s.NextWorkload(), train1));
  EXPECT(!s.PrecloseCheckpointWorkload());  // nothing trained yet
  EXPECT(!s.WorkloadCompleted(done(train1), false).op);
  EXPECT(Same(s.NextWorkload(), train2));
  EXPECT(Same(*s.PrecloseCheckpointWorkload(), ckpt1));
  EXPECT(!s.WorkloadCompleted(done(train2), false).op);
  EXPECT(Same(s.NextWorkload(), val2));
  EXPECT(Same(*s.PrecloseCheckpointWorkload(), ckpt2));
  EXPECT(!s.WorkloadCompleted(done(val2), false).op);
  EXPECT(Same(s.NextWorkload(), train3));
  EXPECT(!s.WorkloadCompleted(done(train3), false).op);
  EXPECT(Same(s.NextWorkload(), train4));
  EXPECT(!s.WorkloadCompleted(done(train4), false).op);
  EXPECT(Same(s.NextWorkload(), val4));
  EXPECT(!s.WorkloadCompleted(done(val4), false).op);
  EXPECT(Same(s.NextWorkload(), ckpt4));
  EXPECT(!s.WorkloadCompleted(done(ckpt4, ckpt_metrics("c4")), false).op);
  EXPECT(!s.PrecloseCheckpointWorkload());
  auto c = s.WorkloadCompleted(done(train5), false);
  EXPECT(c.op && c.op->kind == Op::Kind::Train && c.op->request_id == train.request_id);
  EXPECT(Same(s.NextWorkload(), ckpt5));
  EXPECT_EQ(s.RollBack(), 4);  // back to the step-4 checkpoint
  EXPECT(Same(s.NextWorkload(), train5));
  c = s.WorkloadCompleted(done(train5), false);  // replay
  EXPECT(c.op && c.op->kind == Op::Kind::Train);
  EXPECT(Same(s.NextWorkload(), ckpt5));
  EXPECT(!s.WorkloadCompleted(done(ckpt5, ckpt_metrics("c5")), false).op);
  EXPECT(Same(s.NextWorkload(), val5));
  c = s.WorkloadCompleted(done(val5), false);
  EXPECT(c.op && c.op->kind == Op::Kind::Validate);
  EXPECT(!s.PrecloseCheckpointWorkload());
  c = s.CompleteCachedCheckpoints();
  EXPECT(c.op && c.op->kind == Op::Kind::Checkpoint);
  EXPECT(s.UpToDate());
  threw = false;
  try { s.NextWorkload(); } catch (const std::logic_error&) { threw = true; }
  EXPECT(threw);  // up to date
}

TEST(TestTrialWorkloadSequencerFailedWorkloads) {
  NpRand rand(0);
  Op create = Op::Create(rand, Json::object());
  TrialWorkloadSequencer s(cfg(0, 100, "best", 100));
  s.SetTrialID(1);
  s.OperationRequested(Op::Train(create.request_id, Length(Unit::Batches, 500)));
  s.WorkloadCompleted(done(W(Workload::Kind::RunStep, 1, 100, 0)), false);
  CompletedMessage m = done(W(Workload::Kind::CheckpointModel, 1, 0, 100), Json());
  m.exited_reason = ExitedReason::Errored;  // "not ok": a failed checkpoint, no metrics
  auto c = s.WorkloadCompleted(m, false);
  EXPECT(!c.op);
  EXPECT(s.DebugState()["exiting_early"].as_bool());
}

TEST(TestTrialWorkloadSequencerOperationLessThanBatchSize) {
  NpRand rand(0);
  Op create = Op::Create(rand, Json::object());
  SequencerConfig c0 = cfg(0, 0, "best", 100);
  c0.default_unit = Unit::Records;
  TrialWorkloadSequencer s(c0);
  s.SetTrialID(1);
  Op train = Op::Train(create.request_id, Length(Unit::Records, 24));  // < one 64-record batch
  s.OperationRequested(train);
  auto c = s.WorkloadCompleted(done(W(Workload::Kind::RunStep, 1, 1, 0)), false);
  EXPECT(c.op && c.op->kind == Op::Kind::Train && c.op->request_id == train.request_id);
}
