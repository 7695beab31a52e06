// NpRand, Length, RequestID, Op, hyperparameter sampling, Searcher (event log) and Simulate.
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <sstream>
#include <stdexcept>

#include "detcore/searcher.h"

namespace detcore {

// ------------------------------------------------------------------------------------------
// NpRand: MT19937 exactly as numpy's RandomState / the reference's nprand package.
// ------------------------------------------------------------------------------------------
namespace {
constexpr int kN = 624;
constexpr int kM = 397;
constexpr uint32_t kMatrixA = 0x9908b0dfu;
constexpr uint32_t kUpper = 0x80000000u;
constexpr uint32_t kLower = 0x7fffffffu;
}  // namespace

void NpRand::Seed(uint32_t seed) {
  for (int pos = 0; pos < kN; ++pos) {
    key_[pos] = seed;
    seed = 1812433253u * (seed ^ (seed >> 30)) + static_cast<uint32_t>(pos) + 1u;
  }
  pos_ = kN;
}

uint32_t NpRand::Bits32() {
  uint32_t y;
  if (pos_ == kN) {
    int i = 0;
    for (; i < kN - kM; ++i) {
      y = (key_[i] & kUpper) | (key_[i + 1] & kLower);
      key_[i] = key_[i + kM] ^ (y >> 1) ^ (static_cast<uint32_t>(-static_cast<int32_t>(y & 1)) & kMatrixA);
    }
    for (; i < kN - 1; ++i) {
      y = (key_[i] & kUpper) | (key_[i + 1] & kLower);
      key_[i] = key_[i + (kM - kN)] ^ (y >> 1) ^ (static_cast<uint32_t>(-static_cast<int32_t>(y & 1)) & kMatrixA);
    }
    y = (key_[kN - 1] & kUpper) | (key_[0] & kLower);
    key_[kN - 1] = key_[kM - 1] ^ (y >> 1) ^ (static_cast<uint32_t>(-static_cast<int32_t>(y & 1)) & kMatrixA);
    pos_ = 0;
  }
  y = key_[pos_++];
  y ^= y >> 11;
  y ^= (y << 7) & 0x9d2c5680u;
  y ^= (y << 15) & 0xefc60000u;
  y ^= y >> 18;
  return y;
}

uint64_t NpRand::Bits64() {
  uint64_t hi = static_cast<uint64_t>(Bits32()) << 32;
  return hi | Bits32();
}

void NpRand::Read(uint8_t* p, size_t n) {
  int left = 0;
  uint32_t val = 0;
  for (size_t i = 0; i < n; ++i) {
    if (left == 0) {
      val = Bits32();
      left = 4;
    }
    p[i] = static_cast<uint8_t>(val);
    val >>= 8;
    --left;
  }
}

uint64_t NpRand::BitsLimit(uint64_t limit) {
  if (limit == 0) return 0;
  uint64_t mask = limit;
  mask |= mask >> 1;
  mask |= mask >> 2;
  mask |= mask >> 4;
  mask |= mask >> 8;
  mask |= mask >> 16;
  mask |= mask >> 32;
  if (limit <= 0xffffffffull) {
    for (;;) {
      uint64_t v = static_cast<uint64_t>(Bits32()) & mask;
      if (v <= limit) return v;
    }
  }
  for (;;) {
    uint64_t v = Bits64() & mask;
    if (v <= limit) return v;
  }
}

int64_t NpRand::Int64(int64_t low, int64_t high) {
  if (high <= low) throw std::invalid_argument("nprand Int64: high <= low");
  return low + static_cast<int64_t>(BitsLimit(static_cast<uint64_t>(high) - static_cast<uint64_t>(low) - 1));
}

int64_t NpRand::Int64n(int64_t n) {
  if (n < 0) throw std::invalid_argument("nprand Int64n: n < 0");
  return static_cast<int64_t>(BitsLimit(static_cast<uint64_t>(n) - 1));
}

double NpRand::UnitInterval() {
  double a = static_cast<double>(Bits32() >> 5);
  double b = static_cast<double>(Bits32() >> 6);
  return (a * 67108864.0 + b) / 9007199254740992.0;
}

double NpRand::Uniform(double low, double high) {
  if (high <= low) throw std::invalid_argument("nprand Uniform: high <= low");
  return low + (high - low) * UnitInterval();
}

// ------------------------------------------------------------------------------------------
const char* UnitName(Unit u) {
  switch (u) {
    case Unit::Records: return "records";
    case Unit::Batches: return "batches";
    case Unit::Epochs: return "epochs";
  }
  return "batches";
}

Length Length::FromJson(const Json& j) {
  if (!j.is_object() || j.size() != 1) throw std::invalid_argument("invalid length: " + j.dump());
  if (j.has("records")) return Length(Unit::Records, j["records"].as_int());
  if (j.has("batches")) return Length(Unit::Batches, j["batches"].as_int());
  if (j.has("epochs")) return Length(Unit::Epochs, j["epochs"].as_int());
  throw std::invalid_argument("invalid length: " + j.dump());
}

Json Length::ToJson() const {
  Json j = Json::object();
  j[UnitName(unit)] = units;
  return j;
}

std::string Length::ShortString() const {
  const char* suffix = unit == Unit::Records ? "R" : unit == Unit::Batches ? "B" : "E";
  return std::to_string(units) + suffix;
}

int64_t ToNearestBatch(const Length& l, const UnitContext& c) {
  switch (l.unit) {
    case Unit::Records: return l.units / c.global_batch_size;
    case Unit::Batches: return l.units;
    case Unit::Epochs: return (l.units * c.records_per_epoch) / c.global_batch_size;
  }
  return l.units;
}

bool EqualWithinBatch(const Length& l, int64_t batches, const UnitContext& c) {
  switch (l.unit) {
    case Unit::Records: return std::llabs(l.units - batches * c.global_batch_size) < c.global_batch_size;
    case Unit::Batches: return l.units == batches;
    case Unit::Epochs:
      return std::llabs(l.units * c.records_per_epoch - batches * c.global_batch_size) < c.global_batch_size;
  }
  return false;
}

double UnitsFromBatches(int64_t batches, const UnitContext& c) {
  switch (c.default_unit) {
    case Unit::Records: return static_cast<double>(batches * c.global_batch_size);
    case Unit::Batches: return static_cast<double>(batches);
    case Unit::Epochs:
      return static_cast<double>(batches * c.global_batch_size) / static_cast<double>(c.records_per_epoch);
  }
  return static_cast<double>(batches);
}

std::string RequestIDString(const RequestID& r) {
  char buf[37];
  std::snprintf(buf, sizeof(buf), "%02x%02x%02x%02x-%02x%02x-%02x%02x-%02x%02x-%02x%02x%02x%02x%02x%02x", r[0], r[1],
                r[2], r[3], r[4], r[5], r[6], r[7], r[8], r[9], r[10], r[11], r[12], r[13], r[14], r[15]);
  return buf;
}

RequestID ParseRequestID(const std::string& s) {
  RequestID r{};
  int n = 0;
  for (size_t i = 0; i < s.size() && n < 32; ++i) {
    char c = s[i];
    if (c == '-') continue;
    int v;
    if (c >= '0' && c <= '9') v = c - '0';
    else if (c >= 'a' && c <= 'f') v = c - 'a' + 10;
    else if (c >= 'A' && c <= 'F') v = c - 'A' + 10;
    else throw std::invalid_argument("bad request id " + s);
    if (n % 2 == 0) r[n / 2] = static_cast<uint8_t>(v << 4);
    else r[n / 2] |= static_cast<uint8_t>(v);
    ++n;
  }
  if (n != 32) throw std::invalid_argument("bad request id " + s);
  return r;
}

RequestID NewRequestID(NpRand& rand) {
  RequestID u{};
  rand.Read(u.data(), u.size());
  u[6] = static_cast<uint8_t>((u[6] & 0x0f) | 0x40);  // version 4
  u[8] = static_cast<uint8_t>((u[8] & 0x3f) | 0x80);  // variant 10
  return u;
}

const char* ExitedReasonName(ExitedReason r) {
  switch (r) {
    case ExitedReason::Errored: return "ERRORED";
    case ExitedReason::UserCanceled: return "USER_CANCELED";
    case ExitedReason::InvalidHP: return "INVALID_HP";
  }
  return "ERRORED";
}

ExitedReason ParseExitedReason(const std::string& s) {
  if (s == "USER_CANCELED") return ExitedReason::UserCanceled;
  if (s == "INVALID_HP") return ExitedReason::InvalidHP;
  return ExitedReason::Errored;
}

// ------------------------------------------------------------------------------------------
Op Op::Create(NpRand& rand, Json hparams) {
  Op o;
  o.kind = Kind::Create;
  o.request_id = NewRequestID(rand);
  o.trial_seed = static_cast<uint32_t>(rand.Int64n(int64_t(1) << 31));
  o.hparams = std::move(hparams);
  return o;
}
Op Op::CreateFromCheckpoint(NpRand& rand, Json hparams, const RequestID& ckpt) {
  Op o = Create(rand, std::move(hparams));
  o.has_checkpoint = true;
  o.checkpoint_request_id = ckpt;
  return o;
}
Op Op::Train(const RequestID& r, Length l) {
  Op o;
  o.kind = Kind::Train;
  o.request_id = r;
  o.length = l;
  return o;
}
Op Op::Validate(const RequestID& r) {
  Op o;
  o.kind = Kind::Validate;
  o.request_id = r;
  return o;
}
Op Op::Checkpoint(const RequestID& r) {
  Op o;
  o.kind = Kind::Checkpoint;
  o.request_id = r;
  return o;
}
Op Op::Close(const RequestID& r) {
  Op o;
  o.kind = Kind::Close;
  o.request_id = r;
  return o;
}
Op Op::Shutdown(bool failure) {
  Op o;
  o.kind = Kind::Shutdown;
  o.failure = failure;
  return o;
}

Json Op::ToJson() const {
  Json j = Json::object();
  switch (kind) {
    case Kind::Create:
      j["type"] = "Create";
      j["request_id"] = RequestIDString(request_id);
      j["trial_seed"] = static_cast<int64_t>(trial_seed);
      j["hparams"] = hparams;
      if (has_checkpoint) {
        Json c = Json::object();
        c["request_id"] = RequestIDString(checkpoint_request_id);
        j["checkpoint"] = c;
      } else {
        j["checkpoint"] = Json();
      }
      j["workload_sequencer_type"] = "TRIAL_WORKLOAD_SEQUENCER";
      break;
    case Kind::Train:
      j["type"] = "Train";
      j["request_id"] = RequestIDString(request_id);
      j["length"] = length.ToJson();
      break;
    case Kind::Validate:
      j["type"] = "Validate";
      j["request_id"] = RequestIDString(request_id);
      break;
    case Kind::Checkpoint:
      j["type"] = "Checkpoint";
      j["request_id"] = RequestIDString(request_id);
      break;
    case Kind::Close:
      j["type"] = "Close";
      j["request_id"] = RequestIDString(request_id);
      break;
    case Kind::Shutdown:
      j["type"] = "Shutdown";
      j["failure"] = failure;
      break;
  }
  return j;
}

Op Op::FromJson(const Json& j) {
  const std::string t = j.at("type").as_string();
  Op o;
  if (t == "Shutdown") return Shutdown(j.get_bool("failure", false));
  o.request_id = ParseRequestID(j.at("request_id").as_string());
  if (t == "Create") {
    o.kind = Kind::Create;
    o.trial_seed = static_cast<uint32_t>(j.at("trial_seed").as_int());
    o.hparams = j["hparams"];
    if (j["checkpoint"].is_object()) {
      o.has_checkpoint = true;
      o.checkpoint_request_id = ParseRequestID(j["checkpoint"].at("request_id").as_string());
    }
  } else if (t == "Train") {
    o.kind = Kind::Train;
    o.length = Length::FromJson(j.at("length"));
  } else if (t == "Validate") {
    o.kind = Kind::Validate;
  } else if (t == "Checkpoint") {
    o.kind = Kind::Checkpoint;
  } else if (t == "Close") {
    o.kind = Kind::Close;
  } else {
    throw std::invalid_argument("unknown op type " + t);
  }
  return o;
}

std::string Op::String() const {
  switch (kind) {
    case Kind::Create: return "{Create " + RequestIDString(request_id) + ", seed " + std::to_string(trial_seed) + "}";
    case Kind::Train: return "{Train " + RequestIDString(request_id) + ", " + length.ShortString() + "}";
    case Kind::Validate: return "{Validate " + RequestIDString(request_id) + "}";
    case Kind::Checkpoint: return "{Checkpoint " + RequestIDString(request_id) + "}";
    case Kind::Close: return "{Close " + RequestIDString(request_id) + "}";
    case Kind::Shutdown: return "{Shutdown}";
  }
  return "{?}";
}

// ------------------------------------------------------------------------------------------
// hyperparameters
// ------------------------------------------------------------------------------------------
namespace {
std::string hp_type(const Json& hp) {
  if (hp.is_object() && hp["type"].is_string()) return hp["type"].as_string();
  return "const_bare";
}
}  // namespace

Json SampleOne(const Json& hp, NpRand& rand) {
  const std::string t = hp_type(hp);
  if (t == "const_bare") return hp;
  if (t == "const") return hp["val"];
  if (t == "int") {
    int64_t lo = hp.at("minval").as_int(), hi = hp.at("maxval").as_int();
    return Json(lo + rand.Intn(hi - lo));
  }
  if (t == "double") return Json(rand.Uniform(hp.at("minval").as_double(), hp.at("maxval").as_double()));
  if (t == "log") {
    double v = rand.Uniform(hp.at("minval").as_double(), hp.at("maxval").as_double());
    return Json(std::pow(hp.at("base").as_double(), v));
  }
  if (t == "categorical") {
    const auto& vals = hp.at("vals").as_array();
    return vals.at(static_cast<size_t>(rand.Intn(static_cast<int64_t>(vals.size()))));
  }
  throw std::invalid_argument("unexpected hyperparameter type: " + t);
}

Json SampleAll(const Json& hparams, NpRand& rand) {
  Json out = Json::object();
  if (!hparams.is_object()) return out;
  for (const auto& kv : hparams.as_object()) out[kv.first] = SampleOne(kv.second, rand);
  return out;
}

std::vector<Json> GridValues(const Json& hp) {
  const std::string t = hp_type(hp);
  std::vector<Json> vals;
  if (t == "const_bare") return {hp};
  if (t == "const") return {hp["val"]};
  if (t == "categorical") return hp.at("vals").as_array();
  int64_t count = hp.at("count").as_int();
  if (t == "int") {
    int64_t lo = hp.at("minval").as_int(), hi = hp.at("maxval").as_int();
    count = std::min<int64_t>(count, hi - lo + 1);
    if (count == 1) return {Json(static_cast<int64_t>(std::round(static_cast<double>(lo + hi) / 2.0)))};
    for (int64_t i = 0; i < count; ++i)
      vals.emplace_back(static_cast<int64_t>(
          std::round(static_cast<double>(lo) + static_cast<double>(i * (hi - lo)) / static_cast<double>(count - 1))));
    return vals;
  }
  double lo = hp.at("minval").as_double(), hi = hp.at("maxval").as_double();
  if (t == "double") {
    if (count == 1) return {Json((lo + hi) / 2.0)};
    for (int64_t i = 0; i < count; ++i)
      vals.emplace_back(lo + static_cast<double>(i) * (hi - lo) / static_cast<double>(count - 1));
    return vals;
  }
  if (t == "log") {
    double base = hp.at("base").as_double();
    if (count == 1) return {Json(std::pow(base, (lo + hi) / 2.0))};
    for (int64_t i = 0; i < count; ++i)
      vals.emplace_back(std::pow(base, lo + static_cast<double>(i) * (hi - lo) / static_cast<double>(count - 1)));
    return vals;
  }
  throw std::invalid_argument("unexpected hyperparameter type " + t);
}

namespace {
std::vector<Json> cartesian(const std::vector<std::string>& names, const std::vector<std::vector<Json>>& sets,
                            size_t from) {
  std::vector<Json> out;
  if (from >= names.size()) return out;
  if (from + 1 == names.size()) {
    for (const auto& v : sets[from]) {
      Json s = Json::object();
      s[names[from]] = v;
      out.push_back(s);
    }
    return out;
  }
  auto right = cartesian(names, sets, from + 1);
  for (const auto& l : sets[from]) {
    for (const auto& r : right) {
      Json d = r.clone();
      d[names[from]] = l;
      out.push_back(d);
    }
  }
  return out;
}
}  // namespace

std::vector<Json> HyperparameterGrid(const Json& hparams) {
  std::vector<std::string> names;
  std::vector<std::vector<Json>> sets;
  if (hparams.is_object()) {
    for (const auto& kv : hparams.as_object()) {
      names.push_back(kv.first);
      sets.push_back(GridValues(kv.second));
    }
  }
  return cartesian(names, sets, 0);
}

double ValidationMetric(const Json& vm, const std::string& name) {
  const Json& m = vm.is_object() && vm.has("validation_metrics") ? vm["validation_metrics"] : vm;
  if (!m.has(name)) throw std::invalid_argument("'" + name + "' could not be found in validation metrics");
  const Json& v = m[name];
  if (!v.is_number()) throw std::invalid_argument("'" + name + "' is not a scalar float value");
  return v.as_double();
}

// ------------------------------------------------------------------------------------------
// Searcher
// ------------------------------------------------------------------------------------------
Searcher::Searcher(uint32_t seed, std::unique_ptr<SearchMethod> method, Json hparams)
    : rand_(seed), hparams_(std::move(hparams)), method_(std::move(method)) {}

void Searcher::OperationsCreated(const Ops& ops) {
  for (const auto& op : ops) {
    if (op.kind == Op::Kind::Create) ++trials_requested_;
    if (op.kind == Op::Kind::Shutdown) shutdown_ = true;
  }
}

Ops Searcher::InitialOperations() {
  Context c = ctx();
  Ops ops = method_->InitialOperations(c);
  OperationsCreated(ops);
  return ops;
}

Ops Searcher::TrialCreated(const Op& create, int trial_id) {
  Json ev = Json::object();
  ev["type"] = "TrialCreated";
  ev["create"] = create.ToJson();
  ev["trial_id"] = trial_id;
  uncommitted_.push_back(ev);
  trial_ids_[create.request_id] = trial_id;
  request_ids_[trial_id] = create.request_id;
  Context c = ctx();
  Ops ops = method_->TrialCreated(c, create.request_id);
  OperationsCreated(ops);
  return ops;
}

Ops Searcher::TrialExitedEarly(int trial_id, ExitedReason reason) {
  auto it = request_ids_.find(trial_id);
  if (it == request_ids_.end()) throw std::invalid_argument("unexpected trial ID sent to searcher: " + std::to_string(trial_id));
  early_exits_.insert(it->second);
  Context c = ctx();
  Ops ops = method_->TrialExitedEarly(c, it->second, reason);
  OperationsCreated(ops);
  return ops;
}

void Searcher::WorkloadCompleted(const Json& msg, double units) {
  total_units_ += units;
  Json ev = Json::object();
  ev["type"] = "WorkloadCompleted";
  ev["msg"] = msg;
  ev["units"] = units;
  uncommitted_.push_back(ev);
}

Ops Searcher::OperationCompleted(int trial_id, const Op& op, const Json& metrics) {
  auto it = request_ids_.find(trial_id);
  if (it == request_ids_.end()) throw std::invalid_argument("unexpected trial ID sent to searcher: " + std::to_string(trial_id));
  Context c = ctx();
  Ops ops;
  switch (op.kind) {
    case Op::Kind::Train: ops = method_->TrainCompleted(c, it->second, op); break;
    case Op::Kind::Checkpoint: ops = method_->CheckpointCompleted(c, it->second, op, metrics); break;
    case Op::Kind::Validate: ops = method_->ValidationCompleted(c, it->second, op, metrics); break;
    default: throw std::invalid_argument("unexpected op: " + op.String());
  }
  OperationsCreated(ops);
  return ops;
}

Ops Searcher::TrialClosed(const RequestID& rid) {
  Json ev = Json::object();
  ev["type"] = "TrialClosed";
  ev["request_id"] = RequestIDString(rid);
  uncommitted_.push_back(ev);
  ++trials_closed_;
  Context c = ctx();
  Ops ops = method_->TrialClosed(c, rid);
  OperationsCreated(ops);
  if (trials_requested_ == trials_closed_) {
    Op sd = Op::Shutdown(static_cast<int>(early_exits_.size()) >= trials_requested_);
    OperationsCreated({sd});
    ops.push_back(sd);
  }
  return ops;
}

double Searcher::Progress() const {
  double p = method_->Progress(total_units_);
  if (std::isnan(p) || std::isinf(p)) return 0.0;
  return p;
}

bool Searcher::TrialID(const RequestID& r, int* out) const {
  auto it = trial_ids_.find(r);
  if (it == trial_ids_.end()) return false;
  *out = it->second;
  return true;
}

bool Searcher::RequestIDOf(int trial_id, RequestID* out) const {
  auto it = request_ids_.find(trial_id);
  if (it == request_ids_.end()) return false;
  *out = it->second;
  return true;
}

std::vector<Json> Searcher::UncommittedEvents() {
  std::vector<Json> out;
  out.swap(uncommitted_);
  return out;
}

// ------------------------------------------------------------------------------------------
// Simulate
// ------------------------------------------------------------------------------------------
Json SimulationResult::Summary() const {
  std::map<std::string, int64_t> counts;
  for (const auto& kv : results) {
    std::string key;
    for (const auto& op : kv.second) {
      if (!key.empty()) key += " ";
      if (op.kind == Op::Kind::Train) key += op.length.ShortString();
      else if (op.kind == Op::Kind::Validate) key += "V";
      else if (op.kind == Op::Kind::Checkpoint) key += "C";
    }
    counts[key]++;
  }
  Json j = Json::object();
  for (const auto& kv : counts) j[kv.first] = kv.second;
  return j;
}

Json SimulationResult::TrialSimulations() const {
  Json trials = Json::array();
  std::map<std::string, size_t> index;
  for (const auto& id : order) {
    auto it = results.find(id);
    if (it == results.end()) continue;
    std::string key;
    Json ops = Json::array();
    for (const auto& op : it->second) {
      Json o = Json::object();
      if (op.kind == Op::Kind::Train) {
        key += op.length.ShortString() + " ";
        o["type"] = "RUNNABLE_TYPE_TRAIN";
        Json len = Json::object();
        len["unit"] = op.length.unit == Unit::Records ? "UNIT_RECORDS"
                      : op.length.unit == Unit::Epochs ? "UNIT_EPOCHS" : "UNIT_BATCHES";
        len["count"] = op.length.units;
        o["length"] = len;
      } else if (op.kind == Op::Kind::Validate) {
        key += "V ";
        o["type"] = "RUNNABLE_TYPE_VALIDATE";
      } else if (op.kind == Op::Kind::Checkpoint) {
        key += "C ";
        o["type"] = "RUNNABLE_TYPE_CHECKPOINT";
      } else {
        continue;
      }
      ops.push_back(o);
    }
    auto f = index.find(key);
    if (f != index.end()) {
      Json& t = trials.as_array()[f->second];
      t["occurrences"] = t["occurrences"].as_int() + 1;
      continue;
    }
    index[key] = trials.size();
    Json t = Json::object();
    t["operations"] = ops;
    t["occurrences"] = static_cast<int64_t>(1);
    trials.push_back(t);
  }
  return trials;
}

SimulationResult Simulate(Searcher& s, const ValidationFn& valfn, bool random_order, uint64_t sim_seed,
                          const std::string& metric_name) {
  SimulationResult sim;
  NpRand random(static_cast<uint32_t>(sim_seed));
  std::map<RequestID, std::vector<Op>> pending;
  std::map<RequestID, int> trial_ids;
  std::map<RequestID, int> op_idx;
  auto handle = [&](const Ops& ops) {
    for (const auto& op : ops) {
      if (op.kind == Op::Kind::Create) {
        sim.order.push_back(op.request_id);
        pending[op.request_id] = {op};
      } else if (op.kind == Op::Kind::Shutdown) {
        return true;
      } else {
        pending[op.request_id].push_back(op);
      }
    }
    return false;
  };
  Ops ops = s.InitialOperations();
  double last = s.Progress();
  if (last != 0.0) throw std::runtime_error("initial searcher progress started at " + std::to_string(last));
  bool shutdown = handle(ops);
  int next_trial = 1;
  while (!shutdown) {
    RequestID rid{};
    bool found = false;
    if (!random_order) {
      for (const auto& r : sim.order) {
        auto it = pending.find(r);
        if (it != pending.end() && !it->second.empty()) {
          rid = r;
          found = true;
          break;
        }
      }
    } else {
      std::vector<RequestID> cands;
      for (const auto& kv : pending)
        if (!kv.second.empty()) cands.push_back(kv.first);  // std::map: already sorted by bytes
      if (!cands.empty()) {
        rid = cands[static_cast<size_t>(random.Intn(static_cast<int64_t>(cands.size())))];
        found = true;
      }
    }
    if (!found) throw std::runtime_error("tried to pick a trial when no trial had pending operations");
    Op op = pending[rid].front();
    pending[rid].erase(pending[rid].begin());
    if (op.kind == Op::Kind::Create) {
      sim.results[rid] = {};
      trial_ids[rid] = next_trial;
      op_idx[rid] = 0;
      shutdown = handle(s.TrialCreated(op, next_trial));
      ++next_trial;
    } else if (op.runnable()) {
      Json metrics = Json::object();
      if (op.kind == Op::Kind::Validate) {
        Json vm = Json::object();
        vm[metric_name] = valfn(trial_ids[rid], op_idx[rid]);
        metrics["num_inputs"] = 1;
        metrics["validation_metrics"] = vm;
      } else if (op.kind == Op::Kind::Checkpoint) {
        RequestID u{};
        random.Read(u.data(), u.size());
        metrics["uuid"] = RequestIDString(u);
        metrics["resources"] = Json::object();
      }
      sim.results[rid].push_back(op);
      if (op.kind == Op::Kind::Train) {
        Json msg = Json::object();
        msg["trial_id"] = trial_ids[rid];
        msg["step_id"] = op_idx[rid];
        s.WorkloadCompleted(msg, static_cast<double>(op.length.units));
      }
      Ops next = s.OperationCompleted(trial_ids[rid], op, metrics);
      op_idx[rid]++;
      shutdown = handle(next);
    } else if (op.kind == Op::Kind::Close) {
      pending.erase(rid);
      shutdown = handle(s.TrialClosed(rid));
    } else {
      throw std::runtime_error("unexpected searcher operation " + op.String());
    }
    if (shutdown) {
      if (!pending.empty()) throw std::runtime_error("searcher shutdown prematurely");
      break;
    }
    double p = s.Progress();
    if (p < last - 1e-12) throw std::runtime_error("searcher progress dropped");
    last = p;
  }
  last = s.Progress();
  if (std::fabs(last - 1.0) > 1e-9)
    throw std::runtime_error("searcher progress did not end at 100%: " + std::to_string(last * 100));
  if (sim.results.size() != sim.order.size()) throw std::runtime_error("more trials created than completed");
  return sim;
}

}  // namespace detcore
