// Hierarchical actor runtime for the control plane (reference master/pkg/actor/*.go).
//
// Semantics kept from the reference:
//   * each actor processes one message at a time (no locks needed inside Receive);
//   * Tell is fire-and-forget, Ask returns a future that resolves to an EMPTY std::any when the
//     receiver never calls Respond (the reference's errNoResponse);
//   * lifecycle messages PreStart / PostStop / ChildStopped / ChildFailed;
//   * an exception escaping Receive stops the actor and its parent gets ChildFailed;
//   * stopping an actor first stops and awaits all children;
//   * addresses are paths ("/experiments/12/<request-id>").
// Design differences: actors are multiplexed over a fixed worker pool (not one OS thread each),
// a cell is scheduled on at most one worker at a time, and timers run on one timer thread.
#pragma once

#include <any>
#include <chrono>
#include <atomic>
#include <condition_variable>
#include <deque>
#include <functional>
#include <future>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

namespace detcore {
namespace actor {

using Message = std::any;
class Cell;
class System;
using Ref = std::shared_ptr<Cell>;

// Lifecycle messages.
struct PreStart {};
struct PostStop {};
struct ChildStopped {
  Ref child;
};
struct ChildFailed {
  Ref child;
  std::string error;
};

class Context;

class Actor {
 public:
  virtual ~Actor() = default;
  virtual void Receive(Context& ctx) = 0;
};

// Wrap a lambda as an actor.
class FuncActor : public Actor {
 public:
  explicit FuncActor(std::function<void(Context&)> f) : f_(std::move(f)) {}
  void Receive(Context& ctx) override { f_(ctx); }

 private:
  std::function<void(Context&)> f_;
};

struct Envelope {
  Message msg;
  Ref sender;
  std::shared_ptr<std::promise<Message>> reply;
  bool stop = false;
  std::chrono::steady_clock::time_point enq{};  // Post time (mailbox latency)
};

// Introspection (reference pprof + master/pkg/actor/trace.go): per-actor mailbox and processing
// statistics, and a ring of the most recent processed messages across the system.
struct CellStats {
  std::string address;
  size_t mailbox = 0;       // current depth
  size_t max_mailbox = 0;   // high-water mark
  uint64_t processed = 0;
  double busy_ms = 0;       // total time inside Receive
  double max_ms = 0;        // slowest Receive
  double wait_ms = 0;       // total time messages sat in the mailbox
  double max_wait_ms = 0;
  uint64_t hist[16] = {0};  // Receive latency histogram: bucket b = [2^(b-1), 2^b) microseconds
  std::map<std::string, uint64_t> by_type;
};
struct TraceRecord {
  std::string address, type;
  double wait_ms = 0, run_ms = 0;
  int64_t at_ms = 0;  // unix ms when processing finished
};
std::string MessageTypeName(const Message& m);

class Context {
 public:
  const Message& message() const { return env_->msg; }
  template <class T>
  const T* As() const {
    return std::any_cast<T>(&env_->msg);
  }
  template <class T>
  bool Is() const {
    return env_->msg.type() == typeid(T);
  }
  Ref Self() const;
  const Ref& Sender() const { return env_->sender; }
  System& system() const;
  bool ExpectingResponse() const { return env_->reply != nullptr && !responded_; }
  void Respond(Message m);
  Ref ActorOf(const std::string& id, std::unique_ptr<Actor> a);
  Ref Child(const std::string& id) const;
  std::vector<Ref> Children() const;
  void Tell(const Ref& to, Message m) const;
  std::future<Message> Ask(const Ref& to, Message m) const;

 private:
  friend class Cell;
  Context(Cell* self, Envelope* env) : self_(self), env_(env) {}
  Cell* self_;
  Envelope* env_;
  bool responded_ = false;
};

class Cell : public std::enable_shared_from_this<Cell> {
 public:
  Cell(System* sys, std::string address, std::unique_ptr<Actor> actor, std::weak_ptr<Cell> parent);
  ~Cell();
  const std::string& address() const { return address_; }
  std::string id() const;
  void Tell(Message m, Ref sender = nullptr);
  std::future<Message> Ask(Message m, Ref sender = nullptr);
  // Ask with a deadline: returns an empty any on timeout or no response.
  Message AskSync(Message m, std::chrono::milliseconds timeout = std::chrono::milliseconds(30000));
  void Stop();
  bool AwaitTermination(std::chrono::milliseconds timeout = std::chrono::milliseconds(-1));
  bool stopped() const;
  Ref parent() const { return parent_.lock(); }
  std::string error() const;

 private:
  friend class System;
  friend class Context;
  void Post(Envelope e);
  void RunBatch();  // executed by a pool worker
  void Process(Envelope& e);
  void BeginStop(const std::string& error);
  void FinishStop();
  enum class State { Running, Stopping, Stopped };

  System* sys_;
  std::string address_;
  std::unique_ptr<Actor> actor_;
  std::weak_ptr<Cell> parent_;
  mutable std::mutex mu_;
  std::condition_variable cv_;
  std::deque<Envelope> inbox_;
  bool scheduled_ = false;
  State state_ = State::Running;  // guarded by mu_ for readers; mutated by the worker
  std::map<std::string, Ref> children_;  // worker-only
  std::string error_;
  CellStats stats_;  // guarded by mu_
};

class System {
 public:
  explicit System(int threads = 4);
  ~System();
  Ref ActorOf(const std::string& path, std::unique_ptr<Actor> a);  // top-level under "/"
  Ref Get(const std::string& address) const;
  // Deliver msg to ref after delay (reference actors.NotifyAfter).
  void NotifyAfter(const Ref& ref, std::chrono::milliseconds delay, Message msg);
  void Shutdown();  // stop every top-level actor, then the workers
  std::vector<CellStats> Stats() const;       // every live actor
  std::vector<TraceRecord> Trace() const;     // most recent processed messages, oldest first
  static constexpr size_t kTraceRing = 512;

 private:
  friend class Cell;
  friend class Context;
  Ref Spawn(const std::string& address, std::unique_ptr<Actor> a, const Ref& parent);
  void Schedule(Ref cell);
  void Unregister(const std::string& address);
  void WorkerLoop();
  void TimerLoop();

  mutable std::mutex mu_;
  std::condition_variable cv_;
  std::deque<Ref> ready_;
  std::map<std::string, std::weak_ptr<Cell>> registry_;
  std::map<std::string, Ref> roots_;
  std::vector<std::thread> workers_;
  std::atomic<bool> shutdown_{false};  // written under mu_, read under tmu_ by TimerLoop

  struct Timer {
    std::chrono::steady_clock::time_point at;
    uint64_t seq;
    std::weak_ptr<Cell> ref;
    Message msg;
    bool operator<(const Timer& o) const { return at != o.at ? at > o.at : seq > o.seq; }
  };
  mutable std::mutex trace_mu_;
  std::vector<TraceRecord> trace_;  // ring of kTraceRing
  size_t trace_next_ = 0;
  void Record(TraceRecord r);
  std::mutex tmu_;
  std::condition_variable tcv_;
  std::vector<Timer> timers_;  // heap
  uint64_t tseq_ = 0;
  std::thread timer_thread_;
};

}  // namespace actor
}  // namespace detcore
