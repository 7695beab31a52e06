// Distributed readers-writer lock service (reference master/internal/rw_coordinator.go:27-174,
// served at WS /ws/data-layer/*resource?read_lock=true|false, core.go:253-289,561).
//
// Each lock holder is one WebSocket connection: the master calls Acquire() when the socket opens
// and Release() when it closes; a grant is delivered by the Grant callback ("read_lock_granted" /
// "write_lock_granted" text frames on the socket).  Differences from the reference, on purpose:
//   * waiters are served in arrival order (deques), not Go map order, so no waiter starves;
//   * a writer is granted only when there is neither a writer nor any reader owner (the reference's
//     `writeLockOwner != nil && len(readLockOwners) != 0` test lets a writer in beside readers);
//   * writers are preferred: once a writer waits, new readers queue behind it.
#pragma once
#include <cstdint>
#include <deque>
#include <functional>
#include <map>
#include <mutex>
#include <set>
#include <string>

namespace detcore {

class RWCoordinator {
 public:
  // Called (outside the coordinator's lock) when `ticket` is granted its lock.
  using Grant = std::function<void(int64_t ticket, bool read_lock)>;

  // Queue a request on `resource`; returns the ticket that names it.  `grant` may run before
  // Acquire returns (immediate grant) and is invoked at most once per ticket.
  int64_t Acquire(const std::string& resource, bool read_lock, Grant grant);
  // Drop a ticket (owner or waiter) and grant whatever became eligible.
  void Release(int64_t ticket);

  struct Status {
    int readers = 0;
    bool writer = false;
    int read_waiting = 0;
    int write_waiting = 0;
  };
  Status Inspect(const std::string& resource) const;

 private:
  struct Waiter {
    int64_t ticket;
    bool read;
    Grant grant;
  };
  struct Resource {
    std::set<int64_t> readers;
    int64_t writer = 0;  // 0 = none
    std::deque<Waiter> waiting;
  };
  using Ready = std::deque<std::pair<Waiter, bool>>;
  void Schedule(Resource* r, Ready* ready);

  mutable std::mutex mu_;
  int64_t next_ticket_ = 1;
  std::map<std::string, Resource> resources_;
  std::map<int64_t, std::string> ticket_resource_;
};

}  // namespace detcore
