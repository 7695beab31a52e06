// Readers-writer lock coordinator for the data-layer cache (see include/detcore/rw_coordinator.h;
// reference master/internal/rw_coordinator.go).
#include "detcore/rw_coordinator.h"

#include <algorithm>

namespace detcore {

void RWCoordinator::Schedule(Resource* r, Ready* ready) {
  // Grant from the head of the queue: one writer when the resource is idle, otherwise the run of
  // readers up to the first waiting writer (writer preference keeps writers from starving).
  while (!r->waiting.empty()) {
    Waiter& w = r->waiting.front();
    if (!w.read) {
      if (r->writer != 0 || !r->readers.empty()) return;
      r->writer = w.ticket;
      ready->emplace_back(std::move(w), false);
      r->waiting.pop_front();
      return;
    }
    if (r->writer != 0) return;
    r->readers.insert(w.ticket);
    ready->emplace_back(std::move(w), true);
    r->waiting.pop_front();
  }
}

int64_t RWCoordinator::Acquire(const std::string& resource, bool read_lock, Grant grant) {
  Ready ready;
  int64_t ticket;
  {
    std::lock_guard<std::mutex> g(mu_);
    ticket = next_ticket_++;
    Resource& r = resources_[resource];
    r.waiting.push_back(Waiter{ticket, read_lock, std::move(grant)});
    ticket_resource_[ticket] = resource;
    Schedule(&r, &ready);
  }
  for (auto& p : ready)
    if (p.first.grant) p.first.grant(p.first.ticket, p.second);
  return ticket;
}

void RWCoordinator::Release(int64_t ticket) {
  Ready ready;
  {
    std::lock_guard<std::mutex> g(mu_);
    auto it = ticket_resource_.find(ticket);
    if (it == ticket_resource_.end()) return;
    auto rit = resources_.find(it->second);
    ticket_resource_.erase(it);
    if (rit == resources_.end()) return;
    Resource& r = rit->second;
    if (r.writer == ticket) r.writer = 0;
    r.readers.erase(ticket);
    r.waiting.erase(std::remove_if(r.waiting.begin(), r.waiting.end(),
                                   [ticket](const Waiter& w) { return w.ticket == ticket; }),
                    r.waiting.end());
    Schedule(&r, &ready);
    if (r.writer == 0 && r.readers.empty() && r.waiting.empty()) resources_.erase(rit);
  }
  for (auto& p : ready)
    if (p.first.grant) p.first.grant(p.first.ticket, p.second);
}

RWCoordinator::Status RWCoordinator::Inspect(const std::string& resource) const {
  std::lock_guard<std::mutex> g(mu_);
  Status s;
  auto it = resources_.find(resource);
  if (it == resources_.end()) return s;
  s.readers = static_cast<int>(it->second.readers.size());
  s.writer = it->second.writer != 0;
  for (const auto& w : it->second.waiting) (w.read ? s.read_waiting : s.write_waiting)++;
  return s;
}

}  // namespace detcore
