// Actor runtime (see include/detcore/actor.h).
#include "detcore/actor.h"

#include <cxxabi.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>

#include <algorithm>
#include <exception>
#include <stdexcept>

namespace detcore {
namespace actor {

namespace {
constexpr int kBatch = 64;
}

// ------------------------------------------------------------------------------------- Context
Ref Context::Self() const { return self_->shared_from_this(); }
System& Context::system() const { return *self_->sys_; }

void Context::Respond(Message m) {
  if (env_->reply && !responded_) {
    responded_ = true;
    env_->reply->set_value(std::move(m));
  }
}

Ref Context::ActorOf(const std::string& id, std::unique_ptr<Actor> a) {
  auto it = self_->children_.find(id);
  if (it != self_->children_.end()) return it->second;
  Ref child = self_->sys_->Spawn(self_->address_ + "/" + id, std::move(a), Self());
  self_->children_[id] = child;
  return child;
}

Ref Context::Child(const std::string& id) const {
  auto it = self_->children_.find(id);
  return it == self_->children_.end() ? nullptr : it->second;
}

std::vector<Ref> Context::Children() const {
  std::vector<Ref> out;
  for (auto& kv : self_->children_) out.push_back(kv.second);
  return out;
}

void Context::Tell(const Ref& to, Message m) const {
  if (to) to->Tell(std::move(m), Self());
}

std::future<Message> Context::Ask(const Ref& to, Message m) const {
  if (!to) {
    std::promise<Message> p;
    p.set_value(Message());
    return p.get_future();
  }
  return to->Ask(std::move(m), Self());
}

// ---------------------------------------------------------------------------------------- Cell
Cell::Cell(System* sys, std::string address, std::unique_ptr<Actor> actor, std::weak_ptr<Cell> parent)
    : sys_(sys), address_(std::move(address)), actor_(std::move(actor)), parent_(std::move(parent)) {}

Cell::~Cell() = default;

std::string Cell::id() const {
  auto p = address_.rfind('/');
  return p == std::string::npos ? address_ : address_.substr(p + 1);
}

bool Cell::stopped() const {
  std::lock_guard<std::mutex> g(mu_);
  return state_ == State::Stopped;
}

std::string Cell::error() const {
  std::lock_guard<std::mutex> g(mu_);
  return error_;
}

std::string MessageTypeName(const Message& m) {
  const char* n = m.type().name();
  int st = 0;
  char* d = abi::__cxa_demangle(n, nullptr, nullptr, &st);
  std::string out = (st == 0 && d) ? d : n;
  std::free(d);
  for (const char* pre : {"detcore::master::", "detcore::actor::", "detcore::"})
    if (out.rfind(pre, 0) == 0) out = out.substr(std::strlen(pre));
  return out;
}

void Cell::Post(Envelope e) {
  bool schedule = false;
  e.enq = std::chrono::steady_clock::now();
  {
    std::lock_guard<std::mutex> g(mu_);
    if (state_ == State::Stopped) {
      if (e.reply) e.reply->set_value(Message());
      return;
    }
    inbox_.push_back(std::move(e));
    if (inbox_.size() > stats_.max_mailbox) stats_.max_mailbox = inbox_.size();
    if (!scheduled_) {
      scheduled_ = true;
      schedule = true;
    }
  }
  if (schedule) sys_->Schedule(shared_from_this());
}

void Cell::Tell(Message m, Ref sender) {
  Envelope e;
  e.msg = std::move(m);
  e.sender = std::move(sender);
  Post(std::move(e));
}

std::future<Message> Cell::Ask(Message m, Ref sender) {
  Envelope e;
  e.msg = std::move(m);
  e.sender = std::move(sender);
  e.reply = std::make_shared<std::promise<Message>>();
  auto fut = e.reply->get_future();
  Post(std::move(e));
  return fut;
}

Message Cell::AskSync(Message m, std::chrono::milliseconds timeout) {
  auto fut = Ask(std::move(m));
  if (fut.wait_for(timeout) != std::future_status::ready) return Message();
  return fut.get();
}

void Cell::Stop() {
  Envelope e;
  e.stop = true;
  Post(std::move(e));
}

bool Cell::AwaitTermination(std::chrono::milliseconds timeout) {
  std::unique_lock<std::mutex> l(mu_);
  auto pred = [&] { return state_ == State::Stopped; };
  if (timeout.count() < 0) {
    cv_.wait(l, pred);
    return true;
  }
  return cv_.wait_for(l, timeout, pred);
}

void Cell::RunBatch() {
  for (int i = 0; i < kBatch; ++i) {
    Envelope e;
    {
      std::lock_guard<std::mutex> g(mu_);
      if (inbox_.empty() || state_ == State::Stopped) {
        scheduled_ = false;
        // resolve asks that raced with the stop
        if (state_ == State::Stopped) {
          for (auto& pending : inbox_)
            if (pending.reply) pending.reply->set_value(Message());
          inbox_.clear();
        }
        return;
      }
      e = std::move(inbox_.front());
      inbox_.pop_front();
    }
    const auto t0 = std::chrono::steady_clock::now();
    std::string type = e.stop ? "Stop" : MessageTypeName(e.msg);
    Process(e);
    const auto t1 = std::chrono::steady_clock::now();
    const double run = std::chrono::duration<double, std::milli>(t1 - t0).count();
    const double wait = e.enq.time_since_epoch().count() ? std::chrono::duration<double, std::milli>(t0 - e.enq).count() : 0.0;
    {
      std::lock_guard<std::mutex> g(mu_);
      CellStats& st = stats_;
      ++st.processed;
      st.busy_ms += run;
      st.max_ms = std::max(st.max_ms, run);
      st.wait_ms += wait;
      st.max_wait_ms = std::max(st.max_wait_ms, wait);
      int b = 0;
      for (double us = run * 1000.0; us >= 1.0 && b < 15; us /= 2) ++b;
      ++st.hist[b];
      ++st.by_type[type];
    }
    TraceRecord tr;
    tr.address = address_;
    tr.type = std::move(type);
    tr.wait_ms = wait;
    tr.run_ms = run;
    tr.at_ms = std::chrono::duration_cast<std::chrono::milliseconds>(std::chrono::system_clock::now().time_since_epoch()).count();
    sys_->Record(std::move(tr));
  }
  bool again;
  {
    std::lock_guard<std::mutex> g(mu_);
    again = !inbox_.empty() && state_ != State::Stopped;
    if (!again) scheduled_ = false;
  }
  if (again) sys_->Schedule(shared_from_this());
}

void Cell::Process(Envelope& e) {
  if (e.stop) {
    if (state_ == State::Running) BeginStop("");
    if (e.reply) e.reply->set_value(Message());
    return;
  }
  if (const ChildStopped* cs = std::any_cast<ChildStopped>(&e.msg)) {
    if (cs->child) children_.erase(cs->child->id());
  } else if (const ChildFailed* cf = std::any_cast<ChildFailed>(&e.msg)) {
    if (cf->child) children_.erase(cf->child->id());
  }
  Context ctx(this, &e);
  try {
    actor_->Receive(ctx);
  } catch (const std::exception& ex) {
    if (e.reply && !ctx.responded_) {
      ctx.responded_ = true;
      e.reply->set_value(Message());
    }
    if (state_ == State::Running) BeginStop(std::string("actor ") + address_ + " failed: " + ex.what());
    return;
  } catch (...) {
    if (e.reply && !ctx.responded_) {
      ctx.responded_ = true;
      e.reply->set_value(Message());
    }
    if (state_ == State::Running) BeginStop("actor " + address_ + " failed: unknown exception");
    return;
  }
  if (e.reply && !ctx.responded_) e.reply->set_value(Message());  // errNoResponse
  if (state_ == State::Stopping && children_.empty()) FinishStop();
}

void Cell::BeginStop(const std::string& error) {
  {
    std::lock_guard<std::mutex> g(mu_);
    state_ = State::Stopping;
    if (!error.empty()) error_ = error;
  }
  for (auto& kv : children_) kv.second->Stop();
  if (children_.empty()) FinishStop();
}

void Cell::FinishStop() {
  Envelope pe;
  pe.msg = PostStop{};
  Context ctx(this, &pe);
  try {
    actor_->Receive(ctx);
  } catch (...) {
  }
  std::string err;
  {
    std::lock_guard<std::mutex> g(mu_);
    state_ = State::Stopped;
    err = error_;
    for (auto& pending : inbox_)
      if (pending.reply) pending.reply->set_value(Message());
    inbox_.clear();
  }
  cv_.notify_all();
  sys_->Unregister(address_);
  Ref self = shared_from_this();
  if (Ref p = parent_.lock()) {
    if (err.empty()) p->Tell(ChildStopped{self}, self);
    else p->Tell(ChildFailed{self, err}, self);
  }
}

// -------------------------------------------------------------------------------------- System
System::System(int threads) {
  if (threads < 1) threads = 1;
  for (int i = 0; i < threads; ++i) workers_.emplace_back([this] { WorkerLoop(); });
  timer_thread_ = std::thread([this] { TimerLoop(); });
}

System::~System() { Shutdown(); }

Ref System::Spawn(const std::string& address, std::unique_ptr<Actor> a, const Ref& parent) {
  auto cell = std::make_shared<Cell>(this, address, std::move(a), parent);
  {
    std::lock_guard<std::mutex> g(mu_);
    registry_[address] = cell;
  }
  cell->Tell(PreStart{});
  return cell;
}

Ref System::ActorOf(const std::string& path, std::unique_ptr<Actor> a) {
  std::string addr = path.empty() || path[0] != '/' ? "/" + path : path;
  {
    std::lock_guard<std::mutex> g(mu_);
    auto it = roots_.find(addr);
    if (it != roots_.end() && !it->second->stopped()) return it->second;
  }
  Ref r = Spawn(addr, std::move(a), nullptr);
  std::lock_guard<std::mutex> g(mu_);
  roots_[addr] = r;
  return r;
}

Ref System::Get(const std::string& address) const {
  std::lock_guard<std::mutex> g(mu_);
  auto it = registry_.find(address);
  if (it == registry_.end()) return nullptr;
  return it->second.lock();
}

void System::Unregister(const std::string& address) {
  std::lock_guard<std::mutex> g(mu_);
  registry_.erase(address);
  roots_.erase(address);
}

void System::Schedule(Ref cell) {
  {
    std::lock_guard<std::mutex> g(mu_);
    ready_.push_back(std::move(cell));
  }
  cv_.notify_one();
}

void System::WorkerLoop() {
  for (;;) {
    Ref cell;
    {
      std::unique_lock<std::mutex> l(mu_);
      cv_.wait(l, [&] { return shutdown_ || !ready_.empty(); });
      if (ready_.empty()) return;  // shutdown and drained
      cell = std::move(ready_.front());
      ready_.pop_front();
    }
    cell->RunBatch();
  }
}

void System::NotifyAfter(const Ref& ref, std::chrono::milliseconds delay, Message msg) {
  {
    std::lock_guard<std::mutex> g(tmu_);
    timers_.push_back(Timer{std::chrono::steady_clock::now() + delay, tseq_++, ref, std::move(msg)});
    std::push_heap(timers_.begin(), timers_.end());
  }
  tcv_.notify_one();
}

void System::TimerLoop() {
  std::unique_lock<std::mutex> l(tmu_);
  for (;;) {
    if (shutdown_) return;
    if (timers_.empty()) {
      tcv_.wait(l);
      continue;
    }
    auto at = timers_.front().at;
    if (std::chrono::steady_clock::now() < at) {
      tcv_.wait_until(l, at);
      continue;
    }
    std::pop_heap(timers_.begin(), timers_.end());
    Timer t = std::move(timers_.back());
    timers_.pop_back();
    l.unlock();
    if (Ref r = t.ref.lock()) r->Tell(std::move(t.msg));
    l.lock();
  }
}

void System::Shutdown() {
  std::vector<Ref> roots;
  {
    std::lock_guard<std::mutex> g(mu_);
    if (shutdown_ && workers_.empty()) return;
    for (auto& kv : roots_) roots.push_back(kv.second);
  }
  for (auto& r : roots) r->Stop();
  for (auto& r : roots) r->AwaitTermination(std::chrono::milliseconds(10000));
  {
    std::lock_guard<std::mutex> g(mu_);
    shutdown_ = true;
  }
  {
    std::lock_guard<std::mutex> g(tmu_);
  }
  cv_.notify_all();
  tcv_.notify_all();
  for (auto& w : workers_)
    if (w.joinable()) w.join();
  workers_.clear();
  if (timer_thread_.joinable()) timer_thread_.join();
}

void System::Record(TraceRecord r) {
  std::lock_guard<std::mutex> g(trace_mu_);
  if (trace_.size() < kTraceRing) {
    trace_.push_back(std::move(r));
  } else {
    trace_[trace_next_] = std::move(r);
  }
  trace_next_ = (trace_next_ + 1) % kTraceRing;
}

std::vector<TraceRecord> System::Trace() const {
  std::lock_guard<std::mutex> g(trace_mu_);
  if (trace_.size() < kTraceRing) return trace_;
  std::vector<TraceRecord> out(trace_.begin() + static_cast<long>(trace_next_), trace_.end());
  out.insert(out.end(), trace_.begin(), trace_.begin() + static_cast<long>(trace_next_));
  return out;
}

std::vector<CellStats> System::Stats() const {
  std::vector<Ref> cells;
  {
    std::lock_guard<std::mutex> g(mu_);
    for (auto& kv : registry_)
      if (auto c = kv.second.lock()) cells.push_back(c);
  }
  std::vector<CellStats> out;
  for (auto& c : cells) {
    std::lock_guard<std::mutex> g(c->mu_);
    CellStats s = c->stats_;
    s.address = c->address_;
    s.mailbox = c->inbox_.size();
    out.push_back(std::move(s));
  }
  return out;
}

}  // namespace actor
}  // namespace detcore
