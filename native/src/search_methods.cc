// The search methods: random/single, grid, sync halving (SHA), adaptive (tournament of SHA),
// adaptive_simple, async halving (ASHA), adaptive_asha (tournament of ASHA), PBT.
// Behavioural reference: master/pkg/searcher/{random,grid,sha,adaptive,adaptive_simple,asha,
// adaptive_asha,tournament,pbt}.go.  Integer truncations and rung/promotion arithmetic follow the
// reference exactly because the published test vectors depend on them.
#include <algorithm>
#include <cfloat>
#include <cmath>
#include <stdexcept>

#include "detcore/searcher.h"

namespace detcore {

namespace {

constexpr double kExitedMetric = DBL_MAX;

int64_t imax(int64_t a, int64_t b) { return a > b ? a : b; }
int64_t imin(int64_t a, int64_t b) { return a < b ? a : b; }

struct TrialMetric {
  RequestID request_id{};
  double metric = 0;
  bool promoted = false;
};

struct Rung {
  Length units_needed;
  std::vector<TrialMetric> metrics;
  int64_t start_trials = 0;
  int64_t promote_trials = 0;
  int64_t outstanding_trials = 0;

  size_t insert_index(double metric) const {
    // sort.Search(len, metrics[i].metric > metric) == first element strictly greater
    size_t lo = 0, hi = metrics.size();
    while (lo < hi) {
      size_t mid = (lo + hi) / 2;
      if (metrics[mid].metric > metric) hi = mid;
      else lo = mid + 1;
    }
    return lo;
  }

  std::vector<RequestID> PromotionsSync(const RequestID& rid, double metric) {
    size_t idx = insert_index(metric);
    metrics.insert(metrics.begin() + static_cast<long>(idx), TrialMetric{rid, metric, false});
    int64_t curr = static_cast<int64_t>(metrics.size()) + promote_trials - start_trials;
    if (curr <= 0) return {};
    if (static_cast<int64_t>(idx) < curr) return {rid};
    return {metrics[static_cast<size_t>(curr - 1)].request_id};
  }

  std::vector<RequestID> PromotionsAsync(const RequestID& rid, double metric, double divisor) {
    int64_t old_num = static_cast<int64_t>(static_cast<double>(metrics.size()) / divisor);
    int64_t num = static_cast<int64_t>(static_cast<double>(metrics.size() + 1) / divisor);
    size_t idx = insert_index(metric);
    bool now = static_cast<int64_t>(idx) < num;
    metrics.insert(metrics.begin() + static_cast<long>(idx), TrialMetric{rid, metric, now});
    if (now) return {rid};
    if (num != old_num && !metrics[static_cast<size_t>(old_num)].promoted) {
      metrics[static_cast<size_t>(old_num)].promoted = true;
      return {metrics[static_cast<size_t>(old_num)].request_id};
    }
    return {};
  }
};

// ----------------------------------------------------------------------------------------------
class RandomSearch : public SearchMethod {
 public:
  RandomSearch(int64_t max_trials, Length max_length) : max_trials_(max_trials), max_length_(max_length) {}
  Ops InitialOperations(Context& ctx) override {
    Ops ops;
    for (int64_t t = 0; t < max_trials_; ++t) {
      Op c = Op::Create(ctx.rand, SampleAll(ctx.hparams, ctx.rand));
      ops.push_back(c);
      ops.push_back(Op::Train(c.request_id, max_length_));
      ops.push_back(Op::Validate(c.request_id));
      ops.push_back(Op::Close(c.request_id));
    }
    return ops;
  }
  double Progress(double u) override { return u / static_cast<double>(max_length_.units * max_trials_); }
  Ops TrialExitedEarly(Context&, const RequestID&, ExitedReason) override { return {}; }
  Unit unit() const override { return max_length_.unit; }

 private:
  int64_t max_trials_;
  Length max_length_;
};

class GridSearch : public SearchMethod {
 public:
  explicit GridSearch(Length max_length) : max_length_(max_length) {}
  Ops InitialOperations(Context& ctx) override {
    Ops ops;
    auto grid = HyperparameterGrid(ctx.hparams);
    trials_ = static_cast<int64_t>(grid.size());
    for (auto& params : grid) {
      Op c = Op::Create(ctx.rand, params);
      ops.push_back(c);
      ops.push_back(Op::Train(c.request_id, max_length_));
      ops.push_back(Op::Validate(c.request_id));
      ops.push_back(Op::Close(c.request_id));
    }
    return ops;
  }
  double Progress(double u) override { return u / static_cast<double>(max_length_.units * trials_); }
  Ops TrialExitedEarly(Context&, const RequestID&, ExitedReason) override { return {}; }
  Unit unit() const override { return max_length_.unit; }

 private:
  Length max_length_;
  int64_t trials_ = 0;
};

// ----------------------------------------------------------------------------------------------
struct ShaConfig {
  std::string metric;
  bool smaller_is_better = true;
  int64_t num_rungs = 0;
  Length max_length;
  Length budget;
  double divisor = 4;
  bool train_stragglers = true;
};

class SyncHalvingSearch : public SearchMethod {
 public:
  // standard constructor (sha.go newSyncHalvingSearch)
  explicit SyncHalvingSearch(const ShaConfig& c) : cfg_(c) {
    int64_t expected = 0;
    for (int64_t id = 0; id < c.num_rungs; ++id) {
      double compound = std::pow(c.divisor, static_cast<double>(c.num_rungs - id - 1));
      Rung r;
      r.units_needed = Length(c.max_length.unit,
                              imax(static_cast<int64_t>(static_cast<double>(c.max_length.units) / compound), 1));
      r.start_trials = imax(static_cast<int64_t>(compound), 1);
      if (id == 0) expected += r.units_needed.units * r.start_trials;
      else expected += (r.units_needed.units - rungs_[static_cast<size_t>(id - 1)].units_needed.units) * r.start_trials;
      rungs_.push_back(r);
    }
    double mult = static_cast<double>(c.budget.units) / static_cast<double>(expected);
    expected = 0;
    for (size_t id = 0; id < rungs_.size(); ++id) {
      Rung& cur = rungs_[id];
      cur.start_trials = static_cast<int64_t>(mult * static_cast<double>(cur.start_trials));
      if (id == 0) {
        expected += cur.units_needed.units * cur.start_trials;
      } else {
        Rung& prev = rungs_[id - 1];
        cur.units_needed = Length(c.max_length.unit, imax(cur.units_needed.units, prev.units_needed.units));
        cur.start_trials = imax(imin(cur.start_trials, prev.start_trials), 1);
        prev.promote_trials = cur.start_trials;
        expected += (cur.units_needed.units - prev.units_needed.units) * cur.start_trials;
      }
    }
    expected_units_ = expected;
  }
  // adaptive_simple constructor (adaptive_simple.go newSyncHalvingSimpleSearch)
  SyncHalvingSearch(const ShaConfig& c, int64_t trials, bool /*simple*/) : cfg_(c) {
    int64_t expected = 0;
    for (int64_t id = 0; id < c.num_rungs; ++id) {
      int64_t units = imax(static_cast<int64_t>(static_cast<double>(c.max_length.units) /
                                                std::pow(c.divisor, static_cast<double>(c.num_rungs - id - 1))),
                           1);
      int64_t start = imax(static_cast<int64_t>(static_cast<double>(trials) / std::pow(c.divisor, static_cast<double>(id))), 1);
      if (id != 0) {
        Rung& prev = rungs_[static_cast<size_t>(id - 1)];
        units = imax(units, prev.units_needed.units);
        start = imax(start, prev.promote_trials);
        prev.promote_trials = start;
        expected += (units - prev.units_needed.units) * start;
      } else {
        expected += units * start;
      }
      Rung r;
      r.units_needed = Length(c.max_length.unit, units);
      r.start_trials = start;
      rungs_.push_back(r);
    }
    cfg_.budget = Length(c.max_length.unit, expected);
    expected_units_ = expected;
  }

  Ops InitialOperations(Context& ctx) override {
    Ops ops;
    for (int64_t t = 0; t < rungs_[0].start_trials; ++t) {
      Op c = Op::Create(ctx.rand, SampleAll(ctx.hparams, ctx.rand));
      ops.push_back(c);
      ops.push_back(Op::Train(c.request_id, rungs_[0].units_needed));
      ops.push_back(Op::Validate(c.request_id));
    }
    return ops;
  }
  Ops ValidationCompleted(Context& ctx, const RequestID& rid, const Op&, const Json& metrics) override {
    double m = ValidationMetric(metrics, cfg_.metric);
    if (!cfg_.smaller_is_better) m *= -1;
    return PromoteSync(ctx, rid, m);
  }
  Ops TrialExitedEarly(Context& ctx, const RequestID& rid, ExitedReason) override {
    early_exit_[rid] = true;
    return PromoteSync(ctx, rid, kExitedMetric);
  }
  double Progress(double u) override { return std::min(1.0, u / static_cast<double>(expected_units_)); }
  Unit unit() const override { return cfg_.max_length.unit; }

 private:
  Ops PromoteSync(Context& ctx, const RequestID& rid, double metric) {
    int64_t ri = trial_rungs_[rid];
    Rung& rung = rungs_[static_cast<size_t>(ri)];
    if (ri == cfg_.num_rungs - 1) {
      ++trials_completed_;
      if (!early_exit_[rid]) return {Op::Close(rid)};
      return {};
    }
    Ops ops;
    auto to_promote = rung.PromotionsSync(rid, metric);
    if (!to_promote.empty()) {
      for (const auto& pid : to_promote) {
        trial_rungs_[pid] = ri + 1;
        if (!early_exit_[pid]) {
          int64_t units = imax(rungs_[static_cast<size_t>(ri + 1)].units_needed.units - rung.units_needed.units, 1);
          ops.push_back(Op::Train(pid, Length(unit(), units)));
          ops.push_back(Op::Validate(pid));
        } else {
          return PromoteSync(ctx, pid, kExitedMetric);
        }
      }
      if (rung.start_trials < static_cast<int64_t>(rung.metrics.size()))
        throw std::runtime_error("number of trials exceeded initial trials for rung");
      if (static_cast<int64_t>(rung.metrics.size()) == rung.start_trials) {
        for (size_t i = static_cast<size_t>(rung.promote_trials); i < rung.metrics.size(); ++i) {
          ++trials_completed_;
          if (!early_exit_[rung.metrics[i].request_id]) ops.push_back(Op::Close(rung.metrics[i].request_id));
        }
      }
    }
    return ops;
  }

  ShaConfig cfg_;
  std::vector<Rung> rungs_;
  std::map<RequestID, int64_t> trial_rungs_;
  std::map<RequestID, bool> early_exit_;
  int64_t trials_completed_ = 0;
  int64_t expected_units_ = 0;
};

// ----------------------------------------------------------------------------------------------
struct AshaConfig {
  std::string metric;
  bool smaller_is_better = true;
  int64_t num_rungs = 0;
  Length max_length;
  int64_t max_trials = 0;
  double divisor = 4;
  int64_t max_concurrent_trials = 0;
};

class AsyncHalvingSearch : public SearchMethod {
 public:
  explicit AsyncHalvingSearch(const AshaConfig& c) : cfg_(c) {
    for (int64_t id = 0; id < c.num_rungs; ++id) {
      double rate = std::pow(c.divisor, static_cast<double>(c.num_rungs - id - 1));
      Rung r;
      r.units_needed = Length(c.max_length.unit, imax(static_cast<int64_t>(static_cast<double>(c.max_length.units) / rate), 1));
      rungs_.push_back(r);
    }
  }
  Ops InitialOperations(Context& ctx) override {
    int64_t conc;
    if (cfg_.max_concurrent_trials > 0) conc = imin(cfg_.max_concurrent_trials, cfg_.max_trials);
    else conc = imax(imin(static_cast<int64_t>(std::pow(cfg_.divisor, static_cast<double>(cfg_.num_rungs - 1))), cfg_.max_trials), 1);
    Ops ops;
    for (int64_t t = 0; t < conc; ++t) {
      Op c = Op::Create(ctx.rand, SampleAll(ctx.hparams, ctx.rand));
      trial_rungs_[c.request_id] = 0;
      ops.push_back(c);
      ops.push_back(Op::Train(c.request_id, rungs_[0].units_needed));
      ops.push_back(Op::Validate(c.request_id));
    }
    return ops;
  }
  Ops TrialCreated(Context&, const RequestID& rid) override {
    rungs_[0].outstanding_trials++;
    trial_rungs_[rid] = 0;
    return {};
  }
  Ops TrialClosed(Context&, const RequestID& rid) override {
    ++trials_completed_;
    closed_[rid] = true;
    return {};
  }
  Ops ValidationCompleted(Context& ctx, const RequestID& rid, const Op&, const Json& metrics) override {
    double m = ValidationMetric(metrics, cfg_.metric);
    if (!cfg_.smaller_is_better) m *= -1;
    return PromoteAsync(ctx, rid, m);
  }
  Ops TrialExitedEarly(Context& ctx, const RequestID& rid, ExitedReason) override {
    early_exit_[rid] = true;
    closed_[rid] = true;
    return PromoteAsync(ctx, rid, kExitedMetric);
  }
  double Progress(double) override {
    double all = static_cast<double>(rungs_[0].metrics.size());
    double p = all / (1.2 * static_cast<double>(cfg_.max_trials));
    if (static_cast<int64_t>(rungs_[0].metrics.size()) == cfg_.max_trials)
      p = std::max(static_cast<double>(trials_completed_) / static_cast<double>(cfg_.max_trials), p);
    return p;
  }
  Unit unit() const override { return cfg_.max_length.unit; }

 private:
  Ops PromoteAsync(Context& ctx, const RequestID& rid, double metric) {
    int64_t ri = trial_rungs_[rid];
    Rung& rung = rungs_[static_cast<size_t>(ri)];
    rung.outstanding_trials--;
    bool added_train = false;
    Ops ops;
    if (ri == cfg_.num_rungs - 1) {
      rung.metrics.push_back(TrialMetric{rid, metric, false});
      if (!early_exit_[rid]) {
        ops.push_back(Op::Close(rid));
        closed_[rid] = true;
      }
    } else {
      Rung& next = rungs_[static_cast<size_t>(ri + 1)];
      for (const auto& pid : rung.PromotionsAsync(rid, metric, cfg_.divisor)) {
        trial_rungs_[pid] = ri + 1;
        next.outstanding_trials++;
        if (!early_exit_[pid]) {
          int64_t units = imax(next.units_needed.units - rung.units_needed.units, 1);
          ops.push_back(Op::Train(pid, Length(unit(), units)));
          ops.push_back(Op::Validate(pid));
          added_train = true;
        } else {
          return PromoteAsync(ctx, pid, kExitedMetric);
        }
      }
    }
    int64_t all = static_cast<int64_t>(trial_rungs_.size());
    if (!added_train && all < cfg_.max_trials) {
      Op c = Op::Create(ctx.rand, SampleAll(ctx.hparams, ctx.rand));
      trial_rungs_[c.request_id] = 0;
      ops.push_back(c);
      ops.push_back(Op::Train(c.request_id, rungs_[0].units_needed));
      ops.push_back(Op::Validate(c.request_id));
    }
    if (static_cast<int64_t>(rungs_[0].metrics.size()) == cfg_.max_trials) {
      Ops more = CloseOutRungs();
      ops.insert(ops.end(), more.begin(), more.end());
    }
    return ops;
  }
  Ops CloseOutRungs() {
    Ops ops;
    for (auto& rung : rungs_) {
      if (rung.outstanding_trials > 0) break;
      for (const auto& tm : rung.metrics) {
        if (!tm.promoted && !closed_[tm.request_id]) {
          if (!early_exit_[tm.request_id]) {
            ops.push_back(Op::Close(tm.request_id));
            closed_[tm.request_id] = true;
          }
        }
      }
    }
    return ops;
  }

  AshaConfig cfg_;
  std::vector<Rung> rungs_;
  std::map<RequestID, int64_t> trial_rungs_;
  std::map<RequestID, bool> early_exit_;
  std::map<RequestID, bool> closed_;
  int64_t trials_completed_ = 0;
};

// ----------------------------------------------------------------------------------------------
class TournamentSearch : public SearchMethod {
 public:
  explicit TournamentSearch(std::vector<std::unique_ptr<SearchMethod>> subs) : subs_(std::move(subs)) {
    units_.assign(subs_.size(), 0.0);
  }
  Ops InitialOperations(Context& ctx) override {
    Ops all;
    for (size_t i = 0; i < subs_.size(); ++i) {
      Ops ops = subs_[i]->InitialOperations(ctx);
      Mark(i, ops);
      all.insert(all.end(), ops.begin(), ops.end());
    }
    return all;
  }
  Ops TrialCreated(Context& ctx, const RequestID& r) override {
    size_t i = table_.at(r);
    return Mark(i, subs_[i]->TrialCreated(ctx, r));
  }
  Ops TrainCompleted(Context& ctx, const RequestID& r, const Op& t) override {
    size_t i = table_.at(r);
    units_[i] += static_cast<double>(t.length.units);
    return Mark(i, subs_[i]->TrainCompleted(ctx, r, t));
  }
  Ops CheckpointCompleted(Context& ctx, const RequestID& r, const Op& c, const Json& m) override {
    size_t i = table_.at(r);
    return Mark(i, subs_[i]->CheckpointCompleted(ctx, r, c, m));
  }
  Ops ValidationCompleted(Context& ctx, const RequestID& r, const Op& v, const Json& m) override {
    size_t i = table_.at(r);
    return Mark(i, subs_[i]->ValidationCompleted(ctx, r, v, m));
  }
  Ops TrialClosed(Context& ctx, const RequestID& r) override {
    size_t i = table_.at(r);
    return Mark(i, subs_[i]->TrialClosed(ctx, r));
  }
  Ops TrialExitedEarly(Context& ctx, const RequestID& r, ExitedReason e) override {
    size_t i = table_.at(r);
    return Mark(i, subs_[i]->TrialExitedEarly(ctx, r, e));
  }
  double Progress(double) override {
    double s = 0;
    for (size_t i = 0; i < subs_.size(); ++i) s += subs_[i]->Progress(units_[i]);
    return s / static_cast<double>(subs_.size());
  }
  Unit unit() const override { return subs_[0]->unit(); }

 private:
  Ops Mark(size_t i, Ops ops) {
    for (const auto& op : ops)
      if (op.kind == Op::Kind::Create) table_[op.request_id] = i;
    return ops;
  }
  std::vector<std::unique_ptr<SearchMethod>> subs_;
  std::vector<double> units_;
  std::map<RequestID, size_t> table_;
};

// ----------------------------------------------------------------------------------------------
struct PbtConfig {
  std::string metric;
  bool smaller_is_better = true;
  int64_t population_size = 0;
  int64_t num_rounds = 0;
  Length length_per_round;
  double truncate_fraction = 0;
  double resample_probability = 0;
  double perturb_factor = 0;
};

class PBTSearch : public SearchMethod {
 public:
  explicit PBTSearch(const PbtConfig& c) : cfg_(c) {}
  Ops InitialOperations(Context& ctx) override {
    Ops ops;
    for (int64_t t = 0; t < cfg_.population_size; ++t) {
      Op c = Op::Create(ctx.rand, SampleAll(ctx.hparams, ctx.rand));
      params_[c.request_id] = c.hparams;
      ops.push_back(c);
      ops.push_back(Op::Train(c.request_id, cfg_.length_per_round));
      ops.push_back(Op::Validate(c.request_id));
    }
    return ops;
  }
  Ops ValidationCompleted(Context& ctx, const RequestID& rid, const Op&, const Json& metrics) override {
    double m = ValidationMetric(metrics, cfg_.metric);
    metrics_[rid] = m * (cfg_.smaller_is_better ? 1.0 : -1.0);
    return RunNewTrials(ctx, rid);
  }
  Ops CheckpointCompleted(Context&, const RequestID& rid, const Op&, const Json&) override {
    auto it = waiting_.find(rid);
    if (it == waiting_.end()) return {};
    Ops ops = it->second;
    waiting_.erase(it);
    return ops;
  }
  Ops TrialExitedEarly(Context& ctx, const RequestID& rid, ExitedReason) override {
    early_exit_[rid] = true;
    metrics_[rid] = kExitedMetric;
    return RunNewTrials(ctx, rid);
  }
  double Progress(double u) override {
    return u / static_cast<double>(cfg_.length_per_round.units * cfg_.population_size * cfg_.num_rounds);
  }
  Unit unit() const override { return cfg_.length_per_round.unit; }

  // exploreParams (pbt.go): resample each hyperparameter with resample_probability, else perturb
  // numeric ones by (1 +- perturb_factor) clamped to their range; sorted-name RNG order.
  Json Explore(Context& ctx, const Json& old) {
    Json out = Json::object();
    if (!ctx.hparams.is_object()) return out;
    for (const auto& kv : ctx.hparams.as_object()) {
      const std::string& name = kv.first;
      const Json& hp = kv.second;
      if (ctx.rand.UnitInterval() < cfg_.resample_probability) {
        out[name] = SampleOne(hp, ctx.rand);
        continue;
      }
      Json val = old[name];
      bool decrease = ctx.rand.UnitInterval() < .5;
      double mult = decrease ? 1 - cfg_.perturb_factor : 1 + cfg_.perturb_factor;
      std::string t = hp.is_object() ? hp.get_string("type", "") : "";
      if (t == "int") {
        double v = static_cast<double>(val.as_int()) * mult;
        int64_t iv = static_cast<int64_t>(decrease ? std::floor(v) : std::ceil(v));
        iv = std::min(std::max(iv, hp.at("minval").as_int()), hp.at("maxval").as_int());
        val = Json(iv);
      } else if (t == "double") {
        double v = val.as_double() * mult;
        v = std::min(std::max(v, hp.at("minval").as_double()), hp.at("maxval").as_double());
        val = Json(v);
      } else if (t == "log") {
        double base = hp.at("base").as_double();
        double lo = std::pow(base, hp.at("minval").as_double()), hi = std::pow(base, hp.at("maxval").as_double());
        double v = std::min(std::max(val.as_double() * mult, lo), hi);
        val = Json(v);
      }
      out[name] = val;
    }
    return out;
  }

 private:
  Ops RunNewTrials(Context& ctx, const RequestID& rid) {
    Ops ops;
    rounds_of_[rid]++;
    if (static_cast<int64_t>(metrics_.size()) < cfg_.population_size) return ops;
    ++rounds_completed_;
    if (rounds_completed_ >= cfg_.num_rounds) {
      for (const auto& kv : metrics_)  // reference iterates a Go map (random order); we use id order
        if (!early_exit_[kv.first]) ops.push_back(Op::Close(kv.first));
      return ops;
    }
    int64_t ntrunc = static_cast<int64_t>(cfg_.truncate_fraction * static_cast<double>(cfg_.population_size));
    std::vector<RequestID> ids;
    for (const auto& kv : metrics_) ids.push_back(kv.first);
    std::stable_sort(ids.begin(), ids.end(), [&](const RequestID& a, const RequestID& b) {
      double ma = metrics_[a], mb = metrics_[b];
      if (ma != mb) return ma < mb;
      return a < b;
    });
    metrics_.clear();
    int64_t n = static_cast<int64_t>(ids.size());
    for (int64_t i = n - ntrunc; i < n; ++i)
      if (!early_exit_[ids[static_cast<size_t>(i)]]) ops.push_back(Op::Close(ids[static_cast<size_t>(i)]));
    for (int64_t i = 0; i < ntrunc; ++i) {
      const RequestID& r = ids[static_cast<size_t>(i)];
      if (early_exit_[r]) continue;
      Op ck = Op::Checkpoint(r);
      ops.push_back(ck);
      Json np = Explore(ctx, params_[r]);
      Op c = Op::CreateFromCheckpoint(ctx.rand, np, r);
      params_[c.request_id] = np;
      waiting_[r] = {c, Op::Train(c.request_id, cfg_.length_per_round), Op::Validate(c.request_id)};
    }
    for (int64_t i = 0; i < n - ntrunc; ++i) {
      const RequestID& r = ids[static_cast<size_t>(i)];
      if (!early_exit_[r]) {
        ops.push_back(Op::Train(r, cfg_.length_per_round));
        ops.push_back(Op::Validate(r));
      } else {
        metrics_[r] = kExitedMetric;
      }
    }
    return ops;
  }

  PbtConfig cfg_;
  int64_t rounds_completed_ = 0;
  std::map<RequestID, double> metrics_;
  std::map<RequestID, int64_t> rounds_of_;
  std::map<RequestID, Json> params_;
  std::map<RequestID, Ops> waiting_;  // keyed by the checkpointed trial
  std::map<RequestID, bool> early_exit_;
};

// ----------------------------------------------------------------------------------------------
std::vector<int64_t> adaptive_brackets(const std::string& mode, int64_t max_rungs) {
  std::vector<int64_t> b;
  if (mode == "conservative") {
    for (int64_t i = 1; i <= max_rungs; ++i) b.push_back(i);
  } else if (mode == "standard") {
    for (int64_t i = (max_rungs - 1) / 2 + 1; i <= max_rungs; ++i) b.push_back(i);
  } else if (mode == "aggressive") {
    b.push_back(max_rungs);
  } else {
    throw std::invalid_argument("unexpected adaptive mode: " + mode);
  }
  return b;
}

std::vector<int64_t> brackets_from(const Json& c, int64_t max_rungs) {
  std::vector<int64_t> b;
  if (c["bracket_rungs"].is_array() && c["bracket_rungs"].size() > 0) {
    for (const auto& v : c["bracket_rungs"].as_array()) b.push_back(v.as_int());
  } else {
    b = adaptive_brackets(c.get_string("mode", "standard"), max_rungs);
  }
  std::sort(b.begin(), b.end(), std::greater<int64_t>());
  return b;
}

ShaConfig sha_config(const Json& c) {
  ShaConfig s;
  s.metric = c.get_string("metric", "");
  s.smaller_is_better = c.get_bool("smaller_is_better", true);
  s.num_rungs = c.get_int("num_rungs", 0);
  s.max_length = Length::FromJson(c.at("max_length"));
  if (c.has("budget")) s.budget = Length::FromJson(c["budget"]);
  s.divisor = c.get_double("divisor", 4);
  s.train_stragglers = c.get_bool("train_stragglers", true);
  return s;
}

std::vector<int64_t> bracket_max_trials(int64_t max_trials, double divisor, const std::vector<int64_t>& brackets) {
  std::vector<double> w;
  double total = 0;
  for (auto nr : brackets) {
    w.push_back(std::pow(divisor, static_cast<double>(nr - 1)) / static_cast<double>(nr));
    total += w.back();
  }
  std::vector<int64_t> t;
  int64_t alloc = 0;
  for (size_t i = 0; i < brackets.size(); ++i) {
    t.push_back(imax(static_cast<int64_t>(w[i] / total * static_cast<double>(max_trials)), 1));
    alloc += t.back();
  }
  t[0] += imax(max_trials - alloc, 0);
  return t;
}

std::vector<int64_t> bracket_max_concurrent(int64_t max_conc, double divisor, const std::vector<int64_t>& max_trials) {
  int64_t nb = static_cast<int64_t>(max_trials.size());
  int64_t min_trials, rem = 0;
  if (max_conc == 0) {
    min_trials = imax(max_trials.back(), static_cast<int64_t>(divisor));
  } else {
    max_conc = imax(max_conc, nb);
    min_trials = max_conc / nb;
    rem = max_conc % nb;
  }
  std::vector<int64_t> out(static_cast<size_t>(nb), min_trials);
  for (int64_t i = 0; i < rem; ++i) out[static_cast<size_t>(i)]++;
  return out;
}

PbtConfig pbt_config(const Json& c) {
  PbtConfig p;
  p.metric = c.get_string("metric", "");
  p.smaller_is_better = c.get_bool("smaller_is_better", true);
  p.population_size = c.at("population_size").as_int();
  p.num_rounds = c.at("num_rounds").as_int();
  p.length_per_round = Length::FromJson(c.at("length_per_round"));
  p.truncate_fraction = c["replace_function"].get_double("truncate_fraction", 0);
  p.resample_probability = c["explore_function"].get_double("resample_probability", 0);
  p.perturb_factor = c["explore_function"].get_double("perturb_factor", 0);
  return p;
}

}  // namespace

std::vector<int64_t> AdaptiveModeBrackets(const std::string& mode, int64_t max_rungs) {
  return adaptive_brackets(mode, max_rungs);
}

std::vector<int64_t> BracketMaxTrials(int64_t max_trials, double divisor, const std::vector<int64_t>& brackets) {
  return bracket_max_trials(max_trials, divisor, brackets);
}

std::vector<int64_t> BracketMaxConcurrentTrials(int64_t max_concurrent, double divisor,
                                                const std::vector<int64_t>& bracket_max_trials) {
  return bracket_max_concurrent(max_concurrent, divisor, bracket_max_trials);
}

Json PbtExplore(const Json& pbt_searcher_config, Context& ctx, const Json& sample) {
  PBTSearch p(pbt_config(pbt_searcher_config));
  return p.Explore(ctx, sample);
}

std::unique_ptr<SearchMethod> NewSearchMethod(const Json& c) {
  const std::string name = c.get_string("name", "");
  if (name == "tournament") {  // newTournamentSearch(subs...): arbitrary sub-searchers side by side
    std::vector<std::unique_ptr<SearchMethod>> subs;
    for (const auto& sc : c.at("subs").as_array()) subs.push_back(NewSearchMethod(sc));
    if (subs.empty()) throw std::invalid_argument("tournament needs at least one sub-searcher");
    return std::make_unique<TournamentSearch>(std::move(subs));
  }
  if (name == "single") return std::make_unique<RandomSearch>(1, Length::FromJson(c.at("max_length")));
  if (name == "random")
    return std::make_unique<RandomSearch>(c.at("max_trials").as_int(), Length::FromJson(c.at("max_length")));
  if (name == "grid") return std::make_unique<GridSearch>(Length::FromJson(c.at("max_length")));
  if (name == "sync_halving") return std::make_unique<SyncHalvingSearch>(sha_config(c));
  if (name == "adaptive") {
    auto brackets = brackets_from(c, c.get_int("max_rungs", 5));
    std::vector<std::unique_ptr<SearchMethod>> subs;
    Length budget = Length::FromJson(c.at("budget"));
    for (auto nr : brackets) {
      ShaConfig s = sha_config(c);
      s.num_rungs = nr;
      s.budget = Length(budget.unit, budget.units / static_cast<int64_t>(brackets.size()));
      subs.push_back(std::make_unique<SyncHalvingSearch>(s));
    }
    return std::make_unique<TournamentSearch>(std::move(subs));
  }
  if (name == "adaptive_simple") {
    auto brackets = adaptive_brackets(c.get_string("mode", "standard"), c.get_int("max_rungs", 5));
    std::sort(brackets.begin(), brackets.end(), std::greater<int64_t>());
    std::vector<std::unique_ptr<SearchMethod>> subs;
    int64_t mt = c.at("max_trials").as_int();
    int64_t nb = static_cast<int64_t>(brackets.size());
    for (size_t i = 0; i < brackets.size(); ++i) {
      ShaConfig s = sha_config(c);
      s.num_rungs = brackets[i];
      s.train_stragglers = true;
      int64_t count = mt / nb + ((static_cast<int64_t>(i) < mt % nb) ? 1 : 0);
      subs.push_back(std::make_unique<SyncHalvingSearch>(s, imax(count, 1), true));
    }
    return std::make_unique<TournamentSearch>(std::move(subs));
  }
  if (name == "async_halving") {
    AshaConfig a;
    a.metric = c.get_string("metric", "");
    a.smaller_is_better = c.get_bool("smaller_is_better", true);
    a.num_rungs = c.at("num_rungs").as_int();
    a.max_length = Length::FromJson(c.at("max_length"));
    a.max_trials = c.at("max_trials").as_int();
    a.divisor = c.get_double("divisor", 4);
    a.max_concurrent_trials = c.get_int("max_concurrent_trials", 0);
    return std::make_unique<AsyncHalvingSearch>(a);
  }
  if (name == "adaptive_asha") {
    Length ml = Length::FromJson(c.at("max_length"));
    int64_t max_trials = c.at("max_trials").as_int();
    double divisor = c.get_double("divisor", 4);
    int64_t max_rungs = c.get_int("max_rungs", 5);
    std::vector<int64_t> brackets;
    if (c["bracket_rungs"].is_array() && c["bracket_rungs"].size() > 0) {
      for (const auto& v : c["bracket_rungs"].as_array()) brackets.push_back(v.as_int());
    } else {
      max_rungs = imin(max_rungs, static_cast<int64_t>(std::log(static_cast<double>(ml.units)) / std::log(divisor)) + 1);
      max_rungs = imin(max_rungs, static_cast<int64_t>(std::log(static_cast<double>(max_trials)) / std::log(divisor)) + 1);
      brackets = adaptive_brackets(c.get_string("mode", "standard"), max_rungs);
    }
    std::sort(brackets.begin(), brackets.end(), std::greater<int64_t>());
    auto bmt = bracket_max_trials(max_trials, divisor, brackets);
    auto bmc = bracket_max_concurrent(c.get_int("max_concurrent_trials", 0), divisor, bmt);
    std::vector<std::unique_ptr<SearchMethod>> subs;
    for (size_t i = 0; i < brackets.size(); ++i) {
      AshaConfig a;
      a.metric = c.get_string("metric", "");
      a.smaller_is_better = c.get_bool("smaller_is_better", true);
      a.num_rungs = brackets[i];
      a.max_length = ml;
      a.max_trials = bmt[i];
      a.divisor = divisor;
      a.max_concurrent_trials = bmc[i];
      subs.push_back(std::make_unique<AsyncHalvingSearch>(a));
    }
    return std::make_unique<TournamentSearch>(std::move(subs));
  }
  if (name == "pbt") return std::make_unique<PBTSearch>(pbt_config(c));
  throw std::invalid_argument("no searcher type specified (searcher.name=" + name + ")");
}

}  // namespace detcore
