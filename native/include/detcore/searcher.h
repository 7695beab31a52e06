// Hyperparameter search: bit-reproducible numpy-MT19937 RNG, search operations, the nine search
// methods (single, random, grid, sync_halving, adaptive, adaptive_simple, async_halving,
// adaptive_asha, pbt), the event-logging Searcher wrapper and the offline Simulate driver.
//
// Behavioural reference: master/pkg/searcher/*.go and master/pkg/nprand/nprand.go of the
// reference.  Same seed + same config => same request IDs, trial seeds, hparam samples and
// operation sequences as the reference (checked against its test vectors in native/tests and
// tests/test_searcher.py).
#pragma once

#include <array>
#include <cstdint>
#include <functional>
#include <map>
#include <memory>
#include <set>
#include <string>
#include <vector>

#include "detcore/json.h"

namespace detcore {

// ---------------------------------------------------------------------------------------------
// numpy RandomState-compatible Mersenne Twister (RandomKit rk_random / rk_interval / rk_double)
// ---------------------------------------------------------------------------------------------
class NpRand {
 public:
  explicit NpRand(uint32_t seed = 0) { Seed(seed); }
  void Seed(uint32_t seed);
  uint32_t Bits32();
  uint64_t Bits64();
  void Read(uint8_t* p, size_t n);  // little-endian bytes of successive Bits32()
  int64_t Int64(int64_t low, int64_t high);  // [low, high)
  int64_t Int64n(int64_t n);                 // [0, n)
  int64_t Intn(int64_t n) { return Int64n(n); }
  double UnitInterval();                     // [0, 1) with 53 random bits
  double Uniform(double low, double high);

 private:
  uint64_t BitsLimit(uint64_t limit);
  std::array<uint32_t, 624> key_{};
  int pos_ = 624;
};

// ---------------------------------------------------------------------------------------------
enum class Unit { Records, Batches, Epochs };
const char* UnitName(Unit u);  // "records" / "batches" / "epochs"

struct Length {
  Unit unit = Unit::Batches;
  int64_t units = 0;
  Length() = default;
  Length(Unit u, int64_t n) : unit(u), units(n) {}
  static Length FromJson(const Json& j);
  Json ToJson() const;
  bool operator==(const Length& o) const { return unit == o.unit && units == o.units; }
  bool operator!=(const Length& o) const { return !(*this == o); }
  std::string ShortString() const;  // "64000R" / "5B" / "2E"
};

// Unit conversions (master/pkg/model/length.go).
struct UnitContext {
  Unit default_unit = Unit::Batches;
  int64_t global_batch_size = 1;
  int64_t records_per_epoch = 0;
};
int64_t ToNearestBatch(const Length& l, const UnitContext& c);
bool EqualWithinBatch(const Length& l, int64_t batches, const UnitContext& c);
double UnitsFromBatches(int64_t batches, const UnitContext& c);

using RequestID = std::array<uint8_t, 16>;
std::string RequestIDString(const RequestID& r);
RequestID ParseRequestID(const std::string& s);
RequestID NewRequestID(NpRand& rand);

enum class ExitedReason { Errored, UserCanceled, InvalidHP };
const char* ExitedReasonName(ExitedReason r);
ExitedReason ParseExitedReason(const std::string& s);

struct Op {
  enum class Kind { Create, Train, Validate, Checkpoint, Close, Shutdown };
  Kind kind = Kind::Shutdown;
  RequestID request_id{};
  // Create
  uint32_t trial_seed = 0;
  Json hparams;
  bool has_checkpoint = false;
  RequestID checkpoint_request_id{};
  // Train
  Length length;
  // Shutdown
  bool failure = false;

  static Op Create(NpRand& rand, Json hparams);
  static Op CreateFromCheckpoint(NpRand& rand, Json hparams, const RequestID& ckpt);
  static Op Train(const RequestID& r, Length l);
  static Op Validate(const RequestID& r);
  static Op Checkpoint(const RequestID& r);
  static Op Close(const RequestID& r);
  static Op Shutdown(bool failure = false);
  bool runnable() const { return kind == Kind::Train || kind == Kind::Validate || kind == Kind::Checkpoint; }
  Json ToJson() const;
  static Op FromJson(const Json& j);
  std::string String() const;
};
using Ops = std::vector<Op>;

// Hyperparameter sampling (hyperparameters.go): sorted-name order, int upper bound exclusive.
Json SampleAll(const Json& hparams, NpRand& rand);
Json SampleOne(const Json& hp, NpRand& rand);
std::vector<Json> GridValues(const Json& hp);
std::vector<Json> HyperparameterGrid(const Json& hparams);

struct Context {
  NpRand& rand;
  const Json& hparams;
};

class SearchMethod {
 public:
  virtual ~SearchMethod() = default;
  virtual Ops InitialOperations(Context& ctx) = 0;
  virtual Ops TrialCreated(Context&, const RequestID&) { return {}; }
  virtual Ops TrainCompleted(Context&, const RequestID&, const Op&) { return {}; }
  virtual Ops CheckpointCompleted(Context&, const RequestID&, const Op&, const Json&) { return {}; }
  virtual Ops ValidationCompleted(Context&, const RequestID&, const Op&, const Json&) { return {}; }
  virtual Ops TrialClosed(Context&, const RequestID&) { return {}; }
  virtual Ops TrialExitedEarly(Context&, const RequestID&, ExitedReason) { return {Op::Shutdown(true)}; }
  virtual double Progress(double units_completed) = 0;
  virtual Unit unit() const = 0;
};

// Build a search method from a (defaulted) searcher config object.  Besides the nine searcher
// names, {"name": "tournament", "subs": [cfg, ...]} runs sub-searchers side by side
// (tournament.go newTournamentSearch, which adaptive/adaptive_simple/adaptive_asha build on).
std::unique_ptr<SearchMethod> NewSearchMethod(const Json& searcher_config);

// Bracket rung counts of an adaptive mode (adaptive.go conservativeMode/standardMode/aggressiveMode).
std::vector<int64_t> AdaptiveModeBrackets(const std::string& mode, int64_t max_rungs);
// adaptive_asha bracket sizing (adaptive_asha.go getBracketMaxTrials / getBracketMaxConcurrentTrials).
std::vector<int64_t> BracketMaxTrials(int64_t max_trials, double divisor, const std::vector<int64_t>& brackets);
std::vector<int64_t> BracketMaxConcurrentTrials(int64_t max_concurrent, double divisor,
                                                const std::vector<int64_t>& bracket_max_trials);
// PBT exploreParams of `sample` under a pbt searcher config (pbt.go).
Json PbtExplore(const Json& pbt_searcher_config, Context& ctx, const Json& sample);

// Extract a scalar validation metric (ValidationMetrics.Metric): throws if missing/non-float.
double ValidationMetric(const Json& validation_metrics, const std::string& name);

class Searcher {
 public:
  Searcher(uint32_t seed, std::unique_ptr<SearchMethod> method, Json hparams);
  Ops InitialOperations();
  Ops TrialCreated(const Op& create, int trial_id);
  Ops TrialExitedEarly(int trial_id, ExitedReason reason);
  void WorkloadCompleted(const Json& completed_msg, double units_completed);
  Ops OperationCompleted(int trial_id, const Op& op, const Json& metrics);
  Ops TrialClosed(const RequestID& request_id);
  double Progress() const;
  bool TrialID(const RequestID& r, int* out) const;
  bool RequestIDOf(int trial_id, RequestID* out) const;
  std::vector<Json> UncommittedEvents();
  // event-log counters
  int trials_requested() const { return trials_requested_; }
  int trials_closed() const { return trials_closed_; }
  bool shutdown() const { return shutdown_; }
  double total_units_completed() const { return total_units_; }
  SearchMethod& method() { return *method_; }

 private:
  void OperationsCreated(const Ops& ops);
  Context ctx() { return Context{rand_, hparams_}; }
  NpRand rand_;
  Json hparams_;
  std::unique_ptr<SearchMethod> method_;
  std::vector<Json> uncommitted_;
  std::set<RequestID> early_exits_;
  double total_units_ = 0;
  bool shutdown_ = false;
  int trials_requested_ = 0;
  int trials_closed_ = 0;
  std::map<RequestID, int> trial_ids_;
  std::map<int, RequestID> request_ids_;
};

// Offline simulation (simulate.go).  valfn(trial_id, op_index) gives the validation metric.
struct SimulationResult {
  std::map<RequestID, std::vector<Op>> results;  // runnable ops per trial
  std::vector<RequestID> order;                  // creation order
  Json Summary() const;                          // {"64000R V 128000R V": count, ...}
  // reference experimentv1.ExperimentSimulation.trials: [{operations: [{type, length: {unit,
  // count}}], occurrences}] in first-seen order (api_experiment.go:182-260)
  Json TrialSimulations() const;
};
using ValidationFn = std::function<double(int trial_id, int op_index)>;
// random_order: pick trials uniformly among those with pending ops (seeded by sim_seed);
// otherwise always the first-created trial with pending ops.
SimulationResult Simulate(Searcher& s, const ValidationFn& valfn, bool random_order, uint64_t sim_seed,
                          const std::string& metric_name);

}  // namespace detcore
