// Resource-pool, experiment and trial actors of det-master (see include/detcore/master.h).
//
// Reference behaviour: master/internal/resourcemanagers/resource_pool.go (scheduler tick,
// allocate/release), master/internal/experiment.go (searcher ops -> trials, state machine,
// best-validation tracking, checkpoint GC on completion), master/internal/trial.go (allocation,
// per-rank container specs, rendezvous, workload relay, restarts with rollback, preemption via a
// pre-close checkpoint, terminate timeout) and trial_workload_sequencer.go (native/src/sequencer.cc).
#include "detcore/master_actors.h"

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <random>
#include <sstream>

#include "detcore/sequencer.h"
#include "detcore/workload.h"

namespace detcore {
namespace master {

using actor::Context;
using actor::Ref;

static void Log(const std::string& s) { MasterLog(s); }

// =========================================================================== resource pool
ResourcePoolActor::ResourcePoolActor(Master* m, std::string name)
    : m_(m), name_(std::move(name)) {
  policy_ = sched::ParsePolicy(m->config().scheduler);
  fit_ = sched::ParseFitMethod(m->config().fitting_policy);
  st_.preemption = m->config().priority_preemption;
}

// The reference only schedules on its periodic tick (resource_pool.go); with short HP-search
// trials the tick latency is paid twice per trial (release, then allocate), so state changes also
// queue one coalesced pass.  The tick remains for time-based policies and as a safety net.
void ResourcePoolActor::Kick(Context& ctx) {
  if (kick_pending_) return;
  kick_pending_ = true;
  ctx.Self()->Tell(SchedulerKick{}, ctx.Self());
}

void ResourcePoolActor::SchedulePass(Context& ctx) {
  sched::Decision d = sched::Schedule(st_, policy_, fit_);
  for (auto& a : d.allocate) {
    st_.Allocate(a.first, a.second);
    auto h = handlers_.find(a.first);
    if (h != handlers_.end()) h->second->Tell(ResourcesAllocated{a.first, a.second}, ctx.Self());
  }
  for (auto& id : d.release) {
    if (released_.count(id)) continue;
    released_.insert(id);
    auto h = handlers_.find(id);
    if (h != handlers_.end()) h->second->Tell(ReleaseResources{id}, ctx.Self());
  }
}

void ResourcePoolActor::Receive(Context& ctx) {
  if (ctx.Is<actor::PreStart>()) {
    ctx.system().NotifyAfter(ctx.Self(), std::chrono::milliseconds(static_cast<int>(m_->config().scheduler_tick_ms)),
                             SchedulerTick{});
  } else if (auto a = ctx.As<AddAgent>()) {
    st_.agents[a->agent.id] = a->agent;
    Kick(ctx);
    Log("pool " + name_ + ": agent " + a->agent.id + " joined with " + std::to_string(a->agent.NumSlots()) + " slots");
  } else if (auto r = ctx.As<RemoveAgent>()) {
    st_.agents.erase(r->id);
  } else if (auto req = ctx.As<AllocateRequest>()) {
    sched::Task t;
    t.id = req->task_id;
    t.group = req->group;
    t.label = req->label;
    t.slots_needed = req->slots;
    t.non_preemptible = req->non_preemptible;
    st_.AddTask(t);
    handlers_[req->task_id] = req->handler;
    released_.erase(req->task_id);
    Kick(ctx);
  } else if (auto rel = ctx.As<ResourcesReleased>()) {
    st_.RemoveTask(rel->task_id);
    handlers_.erase(rel->task_id);
    released_.erase(rel->task_id);
    Kick(ctx);
  } else if (auto g = ctx.As<SetGroup>()) {
    sched::Group& grp = st_.EnsureGroup(g->group);
    grp.weight = g->weight;
    grp.priority = g->priority;
    grp.max_slots = g->max_slots;
    Kick(ctx);
  } else if (auto se = ctx.As<SetSlotEnabled>()) {
    auto it = st_.agents.find(se->agent);
    bool ok = false;
    if (it != st_.agents.end()) {
      for (auto& s : it->second.slots)
        if (se->device < 0 || s.device_id == se->device) {
          s.enabled = se->enabled;
          ok = true;
        }
      if (se->device < 0) it->second.enabled = se->enabled;
    }
    ctx.Respond(ok);
  } else if (ctx.Is<SchedulerTick>()) {
    SchedulePass(ctx);
    ctx.system().NotifyAfter(ctx.Self(), std::chrono::milliseconds(static_cast<int>(m_->config().scheduler_tick_ms)),
                             SchedulerTick{});
  } else if (ctx.Is<SchedulerKick>()) {
    kick_pending_ = false;
    SchedulePass(ctx);
  } else if (ctx.Is<PoolSummary>()) {
    Json out = Json::object();
    out["name"] = name_;
    Json agents = Json::array();
    int slots = 0, used = 0;
    for (auto& kv : st_.agents) {
      Json a = Json::object();
      a["id"] = kv.first;
      a["label"] = kv.second.label;
      a["enabled"] = kv.second.enabled;
      Json sl = Json::array();
      for (auto& s : kv.second.slots) {
        Json j = Json::object();
        j["id"] = s.device_id;
        j["uuid"] = s.uuid;
        j["type"] = s.type;
        j["enabled"] = s.enabled;
        j["task"] = s.task;
        sl.push_back(j);
        ++slots;
        used += !s.task.empty();
      }
      a["slots"] = sl;
      a["idle"] = kv.second.Idle();
      agents.push_back(a);
    }
    out["agents"] = agents;
    out["num_slots"] = slots;
    out["slots_used"] = used;
    out["num_tasks"] = static_cast<int64_t>(st_.tasks.size());
    int pending = 0, pending_slots = 0;
    for (auto& kv : st_.tasks)
      if (!kv.second.allocated()) {
        ++pending;
        pending_slots += kv.second.slots_needed;
      }
    out["tasks_pending"] = pending;
    out["pending_slots"] = pending_slots;
    out["scheduler"] = m_->config().scheduler;
    ctx.Respond(out);
  }
}

// ================================================================================ experiment
ExperimentActor::ExperimentActor(Master* m, int64_t id, Json config, bool replay)
    : m_(m), id_(id), config_(std::move(config)), replaying_(replay) {
  uint32_t seed = static_cast<uint32_t>(config_["reproducibility"].get_int("experiment_seed", 0));
  searcher_ = std::make_unique<Searcher>(seed, NewSearchMethod(config_["searcher"]), config_["hyperparameters"]);
  smaller_is_better_ = config_["searcher"].get_bool("smaller_is_better", true);
  metric_ = config_["searcher"].get_string("metric", "");
  pool_ = config_["resources"].get_string("resource_pool", "");
  if (pool_.empty()) pool_ = m_->config().resource_pools.empty() ? "default" : m_->config().resource_pools[0];
  if (replay) {
    // a restored experiment already reported its current state before the master restarted
    Json row;
    if (m_->store().Get("experiments", id_, &row)) reported_state_ = row.get_string("state", "");
  }
}

void ExperimentActor::Event(const std::string& type, Json body) {
  if (replaying_ || m_->shutting_down()) return;
  body["type"] = type;
  body["experiment_id"] = id_;
  m_->store().Insert("searcher_events", body);
}

void ExperimentActor::SaveState() {
  if (m_->shutting_down()) return;
  Json patch = Json::object();
  patch["state"] = state_;
  patch["progress"] = searcher_->Progress();
  if (IsTerminal(state_)) patch["end_time"] = NowRFC3339();
  if (!best_validation_.is_null()) patch["best_validation"] = best_validation_;
  m_->store().Update("experiments", id_, patch);
  if (state_ != reported_state_) {
    reported_state_ = state_;
    Json props = Json::object();
    props["id"] = id_;
    props["state"] = state_;
    if (IsTerminal(state_)) props["num_trials"] = static_cast<int64_t>(m_->store().Where("trials", "experiment_id", Json(id_)).size());
    m_->ReportTelemetry("experiment_state_changed", props);
  }
}

bool ExperimentActor::IsTerminal(const std::string& s) {
  return s == "COMPLETED" || s == "CANCELED" || s == "ERROR";
}

Ref ExperimentActor::TrialRef(Context& ctx, const RequestID& rid) { return ctx.Child(RequestIDString(rid)); }

void ExperimentActor::ProcessOps(Context& ctx, const Ops& ops) {
  std::map<std::string, Ops> per_trial;
  std::vector<std::string> order;
  for (const Op& op : ops) {
    switch (op.kind) {
      case Op::Kind::Create: {
        std::string rid = RequestIDString(op.request_id);
        if (ctx.Child(rid)) break;
        Json warm = config_["internal_warm_start"];
        if (op.has_checkpoint) {
          // PBT: warm start from the checkpoint of the parent trial's latest checkpoint
          auto it = latest_ckpt_.find(RequestIDString(op.checkpoint_request_id));
          if (it != latest_ckpt_.end()) warm = it->second;
        }
        TrialSpec spec{op, warm, 0};
        ctx.ActorOf(rid, std::make_unique<TrialActor>(m_, ctx.Self(), id_, config_, pool_, spec, state_));
        break;
      }
      case Op::Kind::Train:
      case Op::Kind::Validate:
      case Op::Kind::Checkpoint:
      case Op::Kind::Close: {
        std::string rid = RequestIDString(op.request_id);
        if (!per_trial.count(rid)) order.push_back(rid);
        per_trial[rid].push_back(op);
        break;
      }
      case Op::Kind::Shutdown:
        shutdown_ = true;
        shutdown_failure_ = op.failure;
        break;
    }
  }
  for (auto& rid : order) {
    Ref t = ctx.Child(rid);
    if (t) t->Tell(TrialOps{per_trial[rid]}, ctx.Self());
  }
  MaybeFinish(ctx);
}

void ExperimentActor::MaybeFinish(Context& ctx) {
  if (!shutdown_ && !(stopping_ && ctx.Children().empty())) return;
  if (!ctx.Children().empty()) {
    if (shutdown_)
      for (auto& c : ctx.Children()) c->Tell(TrialClose{}, ctx.Self());
    return;
  }
  if (IsTerminal(state_)) return;
  if (state_ == "STOPPING_CANCELED") state_ = "CANCELED";
  else if (state_ == "STOPPING_ERROR" || shutdown_failure_) state_ = "ERROR";
  else state_ = "COMPLETED";
  SaveState();
  Log("experiment " + std::to_string(id_) + " -> " + state_);
  // checkpoint GC of everything the retention policy does not keep (experiment.go:418-425)
  Json to_delete = CheckpointsToGC(m_->store(), id_, config_);
  if (to_delete.size() > 0) m_->RunCheckpointGC(id_, config_, to_delete);
  m_->store().DeleteWhere("searcher_events", [&](const Json& r) { return r.get_int("experiment_id", -1) == id_; });
  m_->store().Flush();
  ctx.Self()->Stop();
}

bool ExperimentActor::IsBest(double metric) {
  bool best = !has_best_ || (smaller_is_better_ ? metric < best_metric_ : metric > best_metric_);
  if (best) {
    has_best_ = true;
    best_metric_ = metric;
    best_validation_ = metric;
  }
  return best;
}

void ExperimentActor::Receive(Context& ctx) {
  if (ctx.Is<actor::PreStart>()) {
    m_->Pool(pool_)->Tell(SetGroup{std::to_string(id_), config_["resources"].get_double("weight", 1.0),
                                   config_["resources"].has("priority")
                                       ? std::optional<int>(static_cast<int>(config_["resources"]["priority"].as_int()))
                                       : std::nullopt,
                                   static_cast<int>(config_["resources"].get_int("max_slots", -1))});
    Json row;
    if (m_->store().Get("experiments", id_, &row)) state_ = row.get_string("state", "ACTIVE");
    if (IsTerminal(state_)) {
      ctx.Self()->Stop();
      return;
    }
    if (!replaying_) {
      Ops ops = searcher_->InitialOperations();
      Event("InitialOperations", Json::object());
      ProcessOps(ctx, ops);
    }
  } else if (auto rp = ctx.As<ReplayEvents>()) {
    Replay(ctx, rp->events);
  } else if (auto tc = ctx.As<TrialCreatedMsg>()) {
    Json ev = Json::object();
    ev["create"] = tc->create.ToJson();
    ev["trial_id"] = tc->trial_id;
    Event("TrialCreated", ev);
    ProcessOps(ctx, searcher_->TrialCreated(tc->create, static_cast<int>(tc->trial_id)));
  } else if (auto wd = ctx.As<TrialWorkloadDone>()) {
    bool best = false;
    const Json& msg = wd->completed;
    if (msg["workload"].get_string("kind", "") == "COMPUTE_VALIDATION_METRICS" && msg["metrics"].is_object() &&
        msg["metrics"]["validation_metrics"].is_object()) {
      try {
        best = IsBest(ValidationMetric(msg["metrics"]["validation_metrics"], metric_));
      } catch (const std::exception&) {
      }
    }
    searcher_->WorkloadCompleted(msg, wd->units);
    searcher_->UncommittedEvents();
    Json ev = Json::object();
    ev["units"] = wd->units;
    Event("WorkloadCompleted", ev);
    Json patch = Json::object();
    patch["progress"] = searcher_->Progress();
    m_->store().Update("experiments", id_, patch);
    if (!msg["metrics"].is_null() && msg["workload"].get_string("kind", "") == "CHECKPOINT_MODEL")
      latest_ckpt_[wd->request_id] = msg["metrics"];
    if (ctx.Sender()) ctx.Sender()->Tell(WorkloadAck{best}, ctx.Self());
  } else if (auto oc = ctx.As<TrialOpCompleted>()) {
    Json ev = Json::object();
    ev["trial_id"] = oc->trial_id;
    ev["op"] = oc->op.ToJson();
    ev["metrics"] = oc->metrics;
    Event("OperationCompleted", ev);
    ProcessOps(ctx, searcher_->OperationCompleted(static_cast<int>(oc->trial_id), oc->op, oc->metrics));
  } else if (auto te = ctx.As<TrialExitedMsg>()) {
    Json ev = Json::object();
    ev["trial_id"] = te->trial_id;
    ev["reason"] = ExitedReasonName(te->reason);
    Event("TrialExitedEarly", ev);
    ProcessOps(ctx, searcher_->TrialExitedEarly(static_cast<int>(te->trial_id), te->reason));
  } else if (auto cs = ctx.As<actor::ChildStopped>()) {
    ChildGone(ctx, cs->child);
  } else if (auto cf = ctx.As<actor::ChildFailed>()) {
    Log("trial actor failed: " + cf->error);
    ChildGone(ctx, cf->child);
  } else if (auto pc = ctx.As<PatchExperimentConfig>()) {
    config_ = DeepMerge(config_, pc->patch);
    ctx.Respond(true);
  } else if (auto st = ctx.As<SetExperimentState>()) {
    const std::string& want = st->state;
    std::string err;
    if (IsTerminal(state_)) err = "experiment is in a terminal state";
    else if (want == "ACTIVE" || want == "PAUSED") {
      if (state_ == "ACTIVE" || state_ == "PAUSED") state_ = want;
      else err = "cannot change state from " + state_;
    } else if (want == "STOPPING_CANCELED" || want == "STOPPING_COMPLETED" || want == "STOPPING_ERROR") {
      state_ = want;
      stopping_ = true;
      if (want == "STOPPING_COMPLETED") shutdown_ = true;
    } else {
      err = "invalid state " + want;
    }
    if (err.empty()) {
      SaveState();
      for (auto& c : ctx.Children()) c->Tell(ExpStateChange{state_, st->kill}, ctx.Self());
      MaybeFinish(ctx);
    }
    ctx.Respond(err);
  } else if (ctx.Is<actor::PostStop>()) {
    m_->Pool(pool_)->Tell(ResourcesReleased{"__group__" + std::to_string(id_)});
  }
}

void ExperimentActor::ChildGone(Context& ctx, const Ref& child) {
  if (m_->shutting_down()) return;  // master restart: trials are restored, not closed
  RequestID rid;
  try {
    rid = ParseRequestID(child->id());
  } catch (const std::exception&) {
    return;
  }
  Json ev = Json::object();
  ev["request_id"] = child->id();
  Event("TrialClosed", ev);
  if (!stopping_ || shutdown_) ProcessOps(ctx, searcher_->TrialClosed(rid));
  SaveState();
  MaybeFinish(ctx);
}

void ExperimentActor::Replay(Context& ctx, const std::vector<Json>& events) {
  // Re-feed the recorded searcher calls to a fresh Searcher with the same seed: the search
  // methods are deterministic, so this reproduces its state (experiment.go:170-236 replay).
  std::map<std::string, Ops> trial_ops;     // runnable ops per trial, in order
  std::map<std::string, Op> creates;
  std::map<int64_t, std::string> trial_rid;
  std::set<std::string> closed_trials, close_requested;
  auto absorb = [&](const Ops& ops) {
    for (const Op& op : ops) {
      std::string rid = RequestIDString(op.request_id);
      if (op.kind == Op::Kind::Create) creates[rid] = op;
      else if (op.kind == Op::Kind::Close) close_requested.insert(rid);
      else if (op.kind == Op::Kind::Shutdown) {
        shutdown_ = true;
        shutdown_failure_ = op.failure;
      } else trial_ops[rid].push_back(op);
    }
  };
  for (const Json& e : events) {
    const std::string t = e.get_string("type", "");
    if (t == "InitialOperations") absorb(searcher_->InitialOperations());
    else if (t == "TrialCreated") {
      Op c = Op::FromJson(e["create"]);
      trial_rid[e["trial_id"].as_int()] = RequestIDString(c.request_id);
      absorb(searcher_->TrialCreated(c, static_cast<int>(e["trial_id"].as_int())));
    } else if (t == "WorkloadCompleted") {
      searcher_->WorkloadCompleted(Json::object(), e.get_double("units", 0));
      searcher_->UncommittedEvents();
    } else if (t == "OperationCompleted") {
      absorb(searcher_->OperationCompleted(static_cast<int>(e["trial_id"].as_int()), Op::FromJson(e["op"]), e["metrics"]));
    } else if (t == "TrialExitedEarly") {
      absorb(searcher_->TrialExitedEarly(static_cast<int>(e["trial_id"].as_int()), ParseExitedReason(e["reason"].as_string())));
    } else if (t == "TrialClosed") {
      closed_trials.insert(e["request_id"].as_string());
      absorb(searcher_->TrialClosed(ParseRequestID(e["request_id"].as_string())));
    }
  }
  replaying_ = false;
  // best validation so far
  for (auto& kv : trial_rid) {
    for (auto& v : m_->store().Where("validations", "trial_id", Json(kv.first))) {
      try {
        IsBest(ValidationMetric(v["metrics"]["validation_metrics"], metric_));
      } catch (const std::exception&) {
      }
    }
  }
  // recreate the live trials, rolled back to their last checkpoint
  for (auto& kv : creates) {
    const std::string& rid = kv.first;
    if (closed_trials.count(rid)) continue;
    int64_t trial_id = 0;
    for (auto& tr : trial_rid)
      if (tr.second == rid) trial_id = tr.first;
    TrialSpec spec{kv.second, Json(), trial_id};
    Ref t = ctx.ActorOf(rid, std::make_unique<TrialActor>(m_, ctx.Self(), id_, config_, pool_, spec, state_));
    Ops ops = trial_ops[rid];
    if (close_requested.count(rid)) ops.push_back(Op::Close(kv.second.request_id));
    t->Tell(TrialRestore{ops}, ctx.Self());
  }
  Log("experiment " + std::to_string(id_) + " restored: " + std::to_string(ctx.Children().size()) + " live trials");
  MaybeFinish(ctx);
}

// ===================================================================================== trial
TrialActor::TrialActor(Master* m, Ref exp, int64_t exp_id, Json config, std::string pool, TrialSpec spec,
                       std::string exp_state)
    : m_(m), exp_(std::move(exp)), exp_id_(exp_id), config_(std::move(config)), pool_(std::move(pool)),
      spec_(std::move(spec)), exp_state_(std::move(exp_state)) {
  int64_t gbs = 1;
  const Json& hp = spec_.create.hparams;
  if (hp.has("global_batch_size")) gbs = hp["global_batch_size"].as_int();
  Json first_ckpt = spec_.warm_start;
  seq_ = std::make_unique<TrialWorkloadSequencer>(SequencerConfig::FromExperimentConfig(config_, exp_id_, gbs), first_ckpt);
  trial_id_ = spec_.trial_id;
  if (trial_id_) seq_->SetTrialID(trial_id_);
  max_restarts_ = static_cast<int>(config_.get_int("max_restarts", 5));
  slots_ = static_cast<int>(config_["resources"].get_int("slots_per_trial", 1));
  rid_ = RequestIDString(spec_.create.request_id);
}

std::string TrialActor::TaskID() const { return "trial-" + std::to_string(exp_id_) + "-" + rid_ + "-" + std::to_string(alloc_gen_); }

void TrialActor::Receive(Context& ctx) {
  self_ = ctx.Self();
  if (auto ops = ctx.As<TrialOps>()) {
    for (const Op& op : ops->ops) {
      if (op.kind == Op::Kind::Close) closing_ = true;
      else seq_->OperationRequested(op);
    }
    Advance(ctx);
  } else if (auto rs = ctx.As<TrialRestore>()) {
    // restore after master restart: re-request the searcher ops, then roll back to the last
    // checkpoint recorded in the store (trial.go:1008-1033 restore)
    for (const Op& op : rs->ops) {
      if (op.kind == Op::Kind::Close) closing_ = true;
      else seq_->OperationRequested(op);
    }
    RestoreFromStore();
    Advance(ctx);
  } else if (ctx.Is<TrialClose>()) {
    closing_ = true;
    Advance(ctx);
  } else if (auto ra = ctx.As<ResourcesAllocated>()) {
    OnAllocated(ctx, *ra);
  } else if (auto rel = ctx.As<ReleaseResources>()) {
    if (rel->task_id == task_id_) {
      Log("trial " + std::to_string(trial_id_) + ": preempted by the scheduler");
      graceful_release_ = true;
      if (!in_flight_) SendNext(ctx);
    }
  } else if (auto cs = ctx.As<ContainerStateMsg>()) {
    OnContainerState(ctx, *cs);
  } else if (auto sc = ctx.As<SocketConnected>()) {
    auto it = containers_.find(sc->container_id);
    if (it == containers_.end()) {
      sc->ws->Close();
      return;
    }
    it->second.ws = sc->ws;
    MaybeRendezvous(ctx);
  } else if (auto sm = ctx.As<SocketMessage>()) {
    OnSocketMessage(ctx, *sm);
  } else if (auto ack = ctx.As<WorkloadAck>()) {
    OnWorkloadAck(ctx, ack->best);
  } else if (auto sd = ctx.As<SocketClosed>()) {
    auto it = containers_.find(sd->container_id);
    if (it != containers_.end()) it->second.ws = nullptr;
  } else if (auto ec = ctx.As<ExpStateChange>()) {
    exp_state_ = ec->state;
    if (ec->state == "PAUSED") {
      graceful_release_ = true;
      if (!in_flight_) SendNext(ctx);
    } else if (ec->state == "ACTIVE") {
      Advance(ctx);
    } else if (ec->state == "STOPPING_CANCELED" || ec->state == "STOPPING_ERROR") {
      canceled_ = true;
      if (ec->kill || containers_.empty()) Kill(ctx);
      else {
        graceful_release_ = true;
        if (!in_flight_) SendNext(ctx);
      }
    } else if (ec->state == "STOPPING_COMPLETED") {
      closing_ = true;
      Advance(ctx);
    }
  } else if (ctx.Is<TrialKill>()) {
    canceled_ = true;
    Kill(ctx);
  } else if (auto tt = ctx.As<TerminateTimeout>()) {
    if (tt->gen == alloc_gen_ && !containers_.empty()) {
      Log("trial " + std::to_string(trial_id_) + ": terminate timeout, killing containers");
      Kill(ctx);
    }
  } else if (ctx.Is<actor::PostStop>()) {
    if (!task_id_.empty()) m_->Pool(pool_)->Tell(ResourcesReleased{task_id_});
    for (auto& c : containers_) m_->UnbindContainer(c.first);
    if (trial_id_ && !m_->shutting_down()) {
      Json patch = Json::object();
      patch["state"] = errored_ ? "ERROR" : (canceled_ ? "CANCELED" : "COMPLETED");
      patch["end_time"] = NowRFC3339();
      m_->store().Update("trials", trial_id_, patch);
    }
  }
}

void TrialActor::Advance(Context& ctx) {
  if (stopped_) return;
  if (!containers_.empty()) {
    if (!in_flight_ && rendezvous_done_) SendNext(ctx);
    return;
  }
  if (task_id_.empty()) {
    if (canceled_ || (closing_ && seq_->UpToDate() && !seq_->PrecloseCheckpointWorkload())) {
      stopped_ = true;
      ctx.Self()->Stop();
      return;
    }
    if (exp_state_ == "ACTIVE" && !seq_->UpToDate()) RequestResources(ctx);
  }
}

void TrialActor::RequestResources(Context& ctx) {
  ++alloc_gen_;
  task_id_ = TaskID();
  // scheduling events (scripts/bench_asha.py splits idle slot time into "no runnable trial" and
  // "a trial waits for resources or its container": the control plane's share)
  Log("[sched] event=requested request=" + rid_ + " trial=" + std::to_string(trial_id_) + " task=" + task_id_);
  AllocateRequest req;
  req.task_id = task_id_;
  req.group = std::to_string(exp_id_);
  req.slots = slots_;
  req.label = config_["resources"].get_string("agent_label", "");
  req.handler = ctx.Self();
  req.name = "Trial " + std::to_string(trial_id_) + " (Experiment " + std::to_string(exp_id_) + ")";
  m_->Pool(pool_)->Tell(req);
}

void TrialActor::OnAllocated(Context& ctx, const ResourcesAllocated& ra) {
  if (ra.task_id != task_id_ || !containers_.empty()) return;
  Log("[sched] event=allocated request=" + rid_ + " trial=" + std::to_string(trial_id_) + " task=" + task_id_);
  if (exp_state_ != "ACTIVE" || seq_->UpToDate() || canceled_) {
    m_->Pool(pool_)->Tell(ResourcesReleased{task_id_});
    task_id_.clear();
    Advance(ctx);
    return;
  }
  if (trial_id_ == 0) {
    Json row = Json::object();
    row["experiment_id"] = exp_id_;
    row["request_id"] = rid_;
    row["seed"] = static_cast<int64_t>(spec_.create.trial_seed);
    row["hparams"] = spec_.create.hparams;
    row["state"] = "ACTIVE";
    row["start_time"] = NowRFC3339();
    row["restarts"] = 0;
    if (!spec_.warm_start.is_null()) row["warm_start_checkpoint"] = spec_.warm_start;
    trial_id_ = m_->store().Insert("trials", row);
    seq_->SetTrialID(trial_id_);
    exp_->Tell(TrialCreatedMsg{spec_.create, trial_id_}, ctx.Self());
  }
  Workload w = seq_->NextWorkload();
  SaveWorkloadStart(w);
  current_ = w;
  in_flight_ = true;
  rendezvous_done_ = false;
  int rank = 0;
  int total = 0;
  for (auto& f : ra.fits) total += static_cast<int>(std::max<size_t>(1, f.devices.size()));
  std::string ckpt_path;
  for (auto& f : ra.fits) {
    Container c;
    c.id = NewUUID();
    c.agent = f.agent;
    c.rank = rank++;
    c.devices = f.devices;
    containers_[c.id] = c;
    order_.push_back(c.id);
    m_->BindContainer(c.id, f.agent, ctx.Self());
  }
  for (auto& cid : order_) {
    Container& c = containers_[cid];
    Json env = Json::object();
    env["DET_MASTER_ADDR"] = m_->master_host();
    env["DET_MASTER_PORT"] = std::to_string(m_->port());
    env["DET_MASTER"] = m_->master_host() + ":" + std::to_string(m_->port());
    env["DET_CLUSTER_ID"] = m_->cluster_id();
    env["DET_AGENT_ID"] = c.agent;
    env["DET_CONTAINER_ID"] = cid;
    env["DET_EXPERIMENT_ID"] = std::to_string(exp_id_);
    env["DET_TRIAL_ID"] = std::to_string(trial_id_);
    env["DET_TRIAL_SEED"] = std::to_string(spec_.create.trial_seed);
    env["DET_EXPERIMENT_CONFIG"] = config_.dump();
    env["DET_HPARAMS"] = spec_.create.hparams.dump();
    env["DET_INITIAL_WORKLOAD"] = w.ToJson().dump();
    env["DET_WORKLOAD_MANAGER_TYPE"] = "TRIAL_WORKLOAD_MANAGER";
    int offset = c.devices.empty() ? 0 : *std::min_element(c.devices.begin(), c.devices.end());
    env["DET_TRIAL_UNIQUE_PORT_OFFSET"] = std::to_string(offset);
    env["DET_RENDEZVOUS_PORTS"] = std::to_string(1734 + offset) + "," + std::to_string(1734 + offset + 16);
    env["DET_NUM_CONTAINERS"] = std::to_string(order_.size());
    env["DET_CONTAINER_RANK"] = std::to_string(c.rank);
    env["DET_TOTAL_SLOTS"] = std::to_string(total);
    // user environment (environment.environment_variables: ["K=V"] or {cpu: [...], gpu: [...]})
    const Json& ev = config_["environment"]["environment_variables"];
    auto add_env = [&](const Json& list) {
      if (!list.is_array()) return;
      for (auto& kv : list.as_array()) {
        if (!kv.is_string()) continue;
        const std::string& s = kv.as_string();
        auto eq = s.find('=');
        if (eq != std::string::npos) env[s.substr(0, eq)] = s.substr(eq + 1);
      }
    };
    Json files = Json::array();
    m_->AddTaskDefaults(env, files);  // task_container_defaults first: the user's env wins
    if (ev.is_array()) add_env(ev);
    else if (ev.is_object()) add_env(ev[c.devices.empty() ? "cpu" : "gpu"]);
    const Json& latest = seq_->LatestCheckpoint();
    if (!latest.is_null() && latest.is_object() && latest.has("uuid")) {
      Json f = Json::object();
      f["path"] = "checkpoint.json";
      f["content"] = net::Base64Encode(latest.dump());
      files.push_back(f);
      env["DET_LATEST_CHECKPOINT"] = "checkpoint.json";
    } else {
      env["DET_LATEST_CHECKPOINT"] = "";
    }
    Json spec = Json::object();
    spec["env"] = env;
    spec["files"] = files;
    spec["experiment_id"] = exp_id_;
    spec["trial_id"] = trial_id_;
    spec["rank"] = c.rank;
    // the owner's host account (reference tasks/task.go:60-100: passwd/group files + run as uid:gid)
    Json aug = m_->AgentUserGroupForExperiment(exp_id_);
    if (aug.is_object()) spec["user"] = aug;
    Json dev = Json::array();
    for (int d : c.devices) dev.push_back(d);
    Json msg = Json::object();
    msg["type"] = "StartContainer";
    msg["container_id"] = cid;
    msg["devices"] = dev;
    msg["spec"] = spec;
    if (!m_->SendToAgent(c.agent, msg)) {
      Log("trial " + std::to_string(trial_id_) + ": agent " + c.agent + " unreachable");
      c.state = "Terminated";
      c.failure = "agent unreachable";
    }
  }
  CheckAllTerminated(ctx);
}

void TrialActor::OnContainerState(Context& ctx, const ContainerStateMsg& cs) {
  auto it = containers_.find(cs.container_id);
  if (it == containers_.end()) return;
  Container& c = it->second;
  c.state = cs.state;
  if (!cs.address.empty()) c.address = cs.address;
  if (cs.state == "Running") {
    MaybeRendezvous(ctx);
  } else if (cs.state == "Terminated") {
    c.exit_code = cs.exit_code;
    c.failure = cs.failure;
    if (c.ws) c.ws->Close();
    c.ws = nullptr;
    // a gang member died: take the rest down (trial.go:924-955)
    if (!terminating_ && (cs.exit_code != 0 || !cs.failure.empty())) {
      for (auto& o : containers_)
        if (o.second.state != "Terminated") SignalContainer(o.first, "SIGKILL");
    }
    CheckAllTerminated(ctx);
  }
}

Json RendezvousInfo(std::vector<RendezvousMember> members, int rank) {
  std::stable_sort(members.begin(), members.end(),
                   [](const RendezvousMember& a, const RendezvousMember& b) { return a.rank < b.rank; });
  Json addrs = Json::array(), addrs2 = Json::array();
  for (const auto& m : members) {
    const int offset = m.devices.empty() ? 0 : *std::min_element(m.devices.begin(), m.devices.end());
    addrs.push_back(m.host + ":" + std::to_string(1734 + offset));
    addrs2.push_back(m.host + ":" + std::to_string(1734 + offset + 16));
  }
  Json msg = Json::object();
  msg["type"] = "RENDEZVOUS_INFO";
  msg["addrs"] = addrs;
  msg["addrs2"] = addrs2;
  msg["rank"] = rank;
  return msg;
}

void TrialActor::MaybeRendezvous(Context& ctx) {
  if (rendezvous_done_ || containers_.empty()) return;
  std::vector<RendezvousMember> members;
  for (auto& cid : order_) {
    const Container& c = containers_[cid];
    if (c.state != "Running" || !c.ws) return;
    members.push_back(RendezvousMember{c.rank, c.address.empty() ? m_->AgentHost(c.agent) : c.address, c.devices});
  }
  for (auto& cid : order_) {
    const Container& c = containers_[cid];
    c.ws->Send(RendezvousInfo(members, c.rank).dump());
  }
  rendezvous_done_ = true;
  // the initial workload travels in DET_INITIAL_WORKLOAD; the harness answers it first
}

void TrialActor::OnSocketMessage(Context& ctx, const SocketMessage& sm) {
  const Json& msg = sm.msg;
  if (msg.get_string("type", "") != "WORKLOAD_COMPLETED") return;
  auto it = containers_.find(sm.container_id);
  if (it == containers_.end() || it->second.rank != 0) return;  // chief answers for the gang
  CompletedMessage cm;
  try {
    cm = CompletedMessage::FromJson(msg);
  } catch (const std::exception& e) {
    Log(std::string("bad WORKLOAD_COMPLETED: ") + e.what());
    return;
  }
  if (cm.workload != current_) {
    Log("trial " + std::to_string(trial_id_) + ": ignoring completion of unexpected workload " + cm.workload.String());
    return;
  }
  in_flight_ = false;
  SaveWorkloadEnd(cm);
  double units = 0;
  if (cm.workload.kind == Workload::Kind::RunStep) {
    UnitContext uc{Unit::Batches, 1, config_.get_int("records_per_epoch", 0)};
    const Json& hp = spec_.create.hparams;
    uc.global_batch_size = hp.has("global_batch_size") ? hp["global_batch_size"].as_int() : 1;
    for (const char* k : {"max_length", "length_per_round", "budget"})
      if (config_["searcher"].has(k)) {
        uc.default_unit = Length::FromJson(config_["searcher"][k]).unit;
        break;
      }
    units = UnitsFromBatches(cm.workload.num_batches, uc);
  }
  if (cm.workload.kind == Workload::Kind::Terminate) {
    return;  // the containers exit on their own
  }
  // the experiment decides "best validation" and feeds the searcher; continue on its ack
  pending_ = cm;
  exp_->Tell(TrialWorkloadDone{trial_id_, rid_, msg, units}, ctx.Self());
}

void TrialActor::OnWorkloadAck(Context& ctx, bool best) {
  if (!pending_) return;
  CompletedMessage cm = *pending_;
  pending_.reset();
  if (cm.exited_reason) {
    ExitedReason why = *cm.exited_reason;
    if (why == ExitedReason::Errored || why == ExitedReason::InvalidHP) {
      errored_ = why == ExitedReason::Errored;
      exp_->Tell(TrialExitedMsg{trial_id_, why}, ctx.Self());
      closing_ = true;
      canceled_ = true;
      exited_early_ = true;
      Terminate(ctx);
      return;
    }
  }
  TrialWorkloadSequencer::Completion comp;
  try {
    comp = seq_->WorkloadCompleted(cm, best);
  } catch (const std::exception& e) {
    Log(std::string("sequencer rejected completion: ") + e.what());
  }
  if (comp.op) exp_->Tell(TrialOpCompleted{trial_id_, *comp.op, comp.metrics}, ctx.Self());
  if (cm.exited_reason && *cm.exited_reason == ExitedReason::UserCanceled) {
    exp_->Tell(TrialExitedMsg{trial_id_, ExitedReason::UserCanceled}, ctx.Self());
    closing_ = true;
  }
  SendNext(ctx);
}

void TrialActor::SendNext(Context& ctx) {
  if (containers_.empty() || in_flight_ || terminating_) return;
  bool stop = graceful_release_ || canceled_ || seq_->UpToDate();
  if (stop) {
    if (!canceled_ || !exited_early_) {
      if (auto pre = seq_->PrecloseCheckpointWorkload()) {
        if (!canceled_ || graceful_release_) {
          SendWorkload(ctx, *pre);
          return;
        }
      }
    }
    Terminate(ctx);
    return;
  }
  SendWorkload(ctx, seq_->NextWorkload());
}

void TrialActor::SendWorkload(Context& ctx, const Workload& w) {
  current_ = w;
  in_flight_ = true;
  SaveWorkloadStart(w);
  Json msg = Json::object();
  msg["type"] = "RUN_WORKLOAD";
  msg["workload"] = w.ToJson();
  std::string s = msg.dump();
  for (auto& kv : containers_)
    if (kv.second.ws) kv.second.ws->Send(s);
}

void TrialActor::Terminate(Context& ctx) {
  if (terminating_) return;
  terminating_ = true;
  Workload w = seq_->TerminateWorkload();
  current_ = w;
  Json msg = Json::object();
  msg["type"] = "RUN_WORKLOAD";
  msg["workload"] = w.ToJson();
  std::string s = msg.dump();
  bool any = false;
  for (auto& kv : containers_)
    if (kv.second.ws) {
      kv.second.ws->Send(s);
      any = true;
    }
  if (!any) Kill(ctx);
  else ctx.system().NotifyAfter(ctx.Self(), std::chrono::milliseconds(60000), TerminateTimeout{alloc_gen_});
}

void TrialActor::Kill(Context& ctx) {
  terminating_ = true;
  if (containers_.empty()) {
    Advance(ctx);
    return;
  }
  for (auto& kv : containers_)
    if (kv.second.state != "Terminated") SignalContainer(kv.first, "SIGKILL");
}

void TrialActor::SignalContainer(const std::string& cid, const std::string& sig) {
  auto it = containers_.find(cid);
  if (it == containers_.end()) return;
  Json msg = Json::object();
  msg["type"] = "SignalContainer";
  msg["container_id"] = cid;
  msg["signal"] = sig;
  m_->SendToAgent(it->second.agent, msg);
}

void TrialActor::CheckAllTerminated(Context& ctx) {
  if (containers_.empty()) return;
  for (auto& kv : containers_)
    if (kv.second.state != "Terminated") return;
  bool failed = false;
  std::string why;
  for (auto& kv : containers_) {
    if (kv.second.exit_code != 0 || !kv.second.failure.empty()) {
      failed = true;
      why = kv.second.failure.empty() ? "exit code " + std::to_string(kv.second.exit_code) : kv.second.failure;
    }
    m_->UnbindContainer(kv.first);
  }
  bool expected = terminating_ && !in_flight_;
  if (terminating_ && canceled_) expected = true;  // we killed it
  containers_.clear();
  order_.clear();
  m_->Pool(pool_)->Tell(ResourcesReleased{task_id_});
  task_id_.clear();
  const bool was_graceful = graceful_release_;
  terminating_ = false;
  graceful_release_ = false;
  rendezvous_done_ = false;
  if (!expected || (failed && !terminating_ && !canceled_ && !was_graceful && !expected)) {
    ++restarts_;
    in_flight_ = false;
    Log("trial " + std::to_string(trial_id_) + " failed (" + why + "), restart " + std::to_string(restarts_) + "/" +
        std::to_string(max_restarts_));
    if (trial_id_) {
      Json patch = Json::object();
      patch["restarts"] = restarts_;
      m_->store().Update("trials", trial_id_, patch);
    }
    if (restarts_ > max_restarts_) {
      errored_ = true;
      exited_early_ = true;
      canceled_ = true;
      exp_->Tell(TrialExitedMsg{trial_id_, ExitedReason::Errored}, ctx.Self());
      stopped_ = true;
      ctx.Self()->Stop();
      return;
    }
    RollBack();
  }
  in_flight_ = false;
  Advance(ctx);
}

void TrialActor::RollBack() {
  int64_t step = seq_->RollBack();
  if (!trial_id_) return;
  auto newer = [&](const Json& r) { return r.get_int("trial_id", -1) == trial_id_ && r.get_int("step_id", 0) > step; };
  m_->store().DeleteWhere("steps", newer);
  m_->store().DeleteWhere("validations", newer);
  m_->store().DeleteWhere("checkpoints", [&](const Json& r) {
    return newer(r) && r.get_string("state", "") != "COMPLETED";
  });
}

void TrialActor::RestoreFromStore() {
  // Replay this trial's completed workloads (in step order) into the sequencer, then roll back
  // to the last checkpoint: exactly the state a restarted container would resume from.
  if (!trial_id_) return;
  struct Row {
    int64_t step;
    int order;
    Json row;
    Workload::Kind kind;
  };
  std::vector<Row> rows;
  for (auto& r : m_->store().Where("steps", "trial_id", Json(trial_id_)))
    if (r.get_string("state", "") == "COMPLETED") rows.push_back({r["step_id"].as_int(), 0, r, Workload::Kind::RunStep});
  for (auto& r : m_->store().Where("validations", "trial_id", Json(trial_id_)))
    if (r.get_string("state", "") == "COMPLETED") rows.push_back({r["step_id"].as_int(), 1, r, Workload::Kind::ComputeValidationMetrics});
  for (auto& r : m_->store().Where("checkpoints", "trial_id", Json(trial_id_)))
    if (r.get_string("state", "") == "COMPLETED") rows.push_back({r["step_id"].as_int(), 2, r, Workload::Kind::CheckpointModel});
  std::sort(rows.begin(), rows.end(), [](const Row& a, const Row& b) {
    return a.row.get_int("seq", 0) != b.row.get_int("seq", 0) ? a.row.get_int("seq", 0) < b.row.get_int("seq", 0)
                                                                : a.order < b.order;
  });
  for (auto& r : rows) {
    if (seq_->UpToDate()) break;
    Workload w = seq_->NextWorkload();
    if (w.kind != r.kind) break;
    CompletedMessage cm;
    cm.workload = w;
    cm.metrics = r.row["metrics"];
    if (r.kind == Workload::Kind::CheckpointModel) cm.metrics = r.row["checkpoint"];
    seq_->WorkloadCompleted(cm, false);
  }
  Json row;
  if (m_->store().Get("trials", trial_id_, &row)) restarts_ = static_cast<int>(row.get_int("restarts", 0));
  RollBack();
}

void TrialActor::SaveWorkloadStart(const Workload& w) {
  if (!trial_id_ || w.kind == Workload::Kind::Terminate) return;
  const char* table = w.kind == Workload::Kind::RunStep ? "steps"
                      : w.kind == Workload::Kind::ComputeValidationMetrics ? "validations"
                                                                           : "checkpoints";
  // replace an earlier attempt at the same (trial, step) (after a restart)
  m_->store().DeleteWhere(table, [&](const Json& r) {
    return r.get_int("trial_id", -1) == trial_id_ && r.get_int("step_id", -1) == w.step_id &&
           r.get_string("state", "") != "COMPLETED";
  });
  Json row = Json::object();
  row["trial_id"] = trial_id_;
  row["experiment_id"] = exp_id_;
  row["step_id"] = w.step_id;
  row["state"] = "ACTIVE";
  row["start_time"] = NowRFC3339();
  row["num_batches"] = w.num_batches;
  row["prior_batches_processed"] = w.total_batches_processed;
  row["seq"] = m_->store().NextID("workload_seq");
  m_->store().Insert(table, row);
}

void TrialActor::SaveWorkloadEnd(const CompletedMessage& cm) {
  const Workload& w = cm.workload;
  if (!trial_id_ || w.kind == Workload::Kind::Terminate) return;
  const char* table = w.kind == Workload::Kind::RunStep ? "steps"
                      : w.kind == Workload::Kind::ComputeValidationMetrics ? "validations"
                                                                           : "checkpoints";
  for (auto& r : m_->store().Scan(table, [&](const Json& r) {
         return r.get_int("trial_id", -1) == trial_id_ && r.get_int("step_id", -1) == w.step_id &&
                r.get_string("state", "") == "ACTIVE";
       })) {
    Json patch = Json::object();
    patch["state"] = cm.exited_reason ? "ERROR" : "COMPLETED";
    patch["end_time"] = NowRFC3339();
    if (w.kind == Workload::Kind::CheckpointModel) {
      patch["checkpoint"] = cm.metrics;
      patch["uuid"] = cm.metrics["uuid"];
      patch["resources"] = cm.metrics["resources"];
      patch["framework"] = cm.metrics["framework"];
      patch["format"] = cm.metrics["format"];
      patch["total_batches_processed"] = w.total_batches_processed;
    } else {
      patch["metrics"] = cm.metrics;
    }
    m_->store().Update(table, r["id"].as_int(), patch);
  }
}

// =============================================================================== provisioner
ProvisionerActor::ProvisionerActor(Master* m, std::string pool, prov::ProvisionerConfig cfg)
    : m_(m), pool_(std::move(pool)), cfg_(cfg), decider_(cfg) {
  if (cfg.provider == "local")
    provider_ = std::make_unique<prov::LocalProvider>(cfg, pool_);
  else
    provider_ = std::make_unique<prov::CommandProvider>(cfg, pool_);
}

void ProvisionerActor::Receive(Context& ctx) {
  if (ctx.Is<actor::PreStart>() || ctx.Is<SchedulerTick>()) {
    if (ctx.Is<SchedulerTick>()) {
      actor::Message msum = m_->Pool(pool_)->AskSync(PoolSummary{}, std::chrono::milliseconds(5000));
      if (msum.has_value()) {
        Json s = std::any_cast<Json>(msum);
        std::vector<prov::AgentInfo> agents;
        for (auto& a : s["agents"].as_array()) agents.push_back({a.get_string("id", ""), a.get_bool("idle", true)});
        auto d = decider_.Decide(static_cast<int>(s.get_int("pending_slots", 0)), agents, provider_->List(),
                                 prov::Clock::now());
        if (!d.terminate.empty()) provider_->Terminate(d.terminate);
        if (d.launch > 0) provider_->Launch(d.launch);
      }
    }
    ctx.system().NotifyAfter(ctx.Self(), std::chrono::milliseconds(1000), SchedulerTick{});
  } else if (ctx.Is<actor::PostStop>()) {
    provider_.reset();
  }
}

// =================================================================================== command
CommandActor::CommandActor(Master* m, int64_t id, Json config, Json secret_env)
    : m_(m), id_(id), config_(std::move(config)), secret_env_(std::move(secret_env)) {
  pool_ = config_["resources"].get_string("resource_pool", "");
  if (pool_.empty()) pool_ = m_->config().resource_pools.empty() ? "default" : m_->config().resource_pools[0];
}

void CommandActor::Save(const std::string& state, int exit_code) {
  Json patch = Json::object();
  patch["state"] = state;
  if (state == "TERMINATED") {
    patch["exit_code"] = exit_code;
    patch["end_time"] = NowRFC3339();
  }
  if (!agent_.empty()) patch["agent"] = agent_;
  m_->store().Update("commands", id_, patch);
}

void CommandActor::Receive(Context& ctx) {
  if (ctx.Is<actor::PreStart>()) {
    task_id_ = "cmd-" + std::to_string(id_);
    AllocateRequest req;
    req.task_id = task_id_;
    req.group = task_id_;
    req.slots = static_cast<int>(config_["resources"].get_int("slots", 0));
    req.label = config_["resources"].get_string("agent_label", "");
    req.non_preemptible = true;  // commands are not checkpointable
    req.handler = ctx.Self();
    req.name = "Command " + std::to_string(id_);
    m_->Pool(pool_)->Tell(req);
    Save("PENDING");
  } else if (auto ra = ctx.As<ResourcesAllocated>()) {
    if (ra->task_id != task_id_ || !container_.empty() || killed_) return;
    const sched::Fit& f = ra->fits.front();
    container_ = NewUUID();
    agent_ = f.agent;
    m_->BindContainer(container_, f.agent, ctx.Self());
    Json env = Json::object();
    env["DET_TASK_ID"] = task_id_;
    env["DET_MASTER"] = m_->master_host() + ":" + std::to_string(m_->port());
    Json files = Json::array();
    m_->AddTaskDefaults(env, files);
    for (const Json* ev : {&config_["environment"]["environment_variables"], &secret_env_})
      if (ev->is_array())
        for (auto& kv : ev->as_array()) {
          const std::string& str = kv.as_string();
          auto eq = str.find('=');
          if (eq != std::string::npos) env[str.substr(0, eq)] = str.substr(eq + 1);
        }
    Json spec = Json::object();
    spec["env"] = env;
    spec["files"] = files;
    spec["cmd"] = config_["entrypoint"];
    {
      Json row;
      Json aug = m_->AgentUserGroupFor(m_->store().Get("commands", id_, &row) ? row.get_string("owner", "") : "");
      if (aug.is_object()) spec["user"] = aug;
    }
    spec["task_id"] = task_id_;
    spec["context_url"] = "/commands/" + std::to_string(id_) + "/context";
    Json dev = Json::array();
    for (int d : f.devices) dev.push_back(d);
    Json msg = Json::object();
    msg["type"] = "StartContainer";
    msg["container_id"] = container_;
    msg["devices"] = dev;
    msg["spec"] = spec;
    if (!m_->SendToAgent(f.agent, msg)) {
      Save("TERMINATED", -1);
      ctx.Self()->Stop();
      return;
    }
    Save("ASSIGNED");
  } else if (auto cs = ctx.As<ContainerStateMsg>()) {
    if (cs->container_id != container_) return;
    if (cs->state == "Running") {
      address_ = cs->address.empty() ? "127.0.0.1" : cs->address;
      Save("RUNNING");
    }
    if (cs->state == "Terminated") {
      Save("TERMINATED", cs->exit_code);
      ctx.Self()->Stop();
    }
  } else if (auto sr = ctx.As<ServiceReady>()) {
    // reference readiness: log-pattern checks (master/internal/command); here the service reports
    // its bound port, and /proxy/<task>/ forwards to it
    Json patch = Json::object();
    patch["service_address"] = (address_.empty() ? std::string("127.0.0.1") : address_) + ":" + std::to_string(sr->port);
    patch["ready"] = true;
    m_->store().Update("commands", id_, patch);
    ctx.Respond(true);
  } else if (ctx.Is<ReleaseResources>() || ctx.Is<CommandKill>()) {
    killed_ = true;
    if (container_.empty()) {
      Save("TERMINATED", -1);
      ctx.Self()->Stop();
    } else {
      Json msg = Json::object();
      msg["type"] = "SignalContainer";
      msg["container_id"] = container_;
      msg["signal"] = "SIGKILL";
      m_->SendToAgent(agent_, msg);
    }
  } else if (ctx.Is<actor::PostStop>()) {
    m_->Pool(pool_)->Tell(ResourcesReleased{task_id_});
    if (!container_.empty()) m_->UnbindContainer(container_);
  }
}

}  // namespace master
}  // namespace detcore
