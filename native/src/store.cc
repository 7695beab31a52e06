// Embedded durable store (see include/detcore/store.h).
#include "detcore/store.h"

#include <sys/stat.h>
#include <unistd.h>

#include <dirent.h>

#include <algorithm>
#include <climits>
#include <iterator>
#include <fstream>
#include <sstream>
#include <stdexcept>

namespace detcore {

namespace {
// Columns the master looks rows up by (Where()): indexed in every table that has them.
const char* const kIndexed[] = {"experiment_id", "trial_id", "uuid", "name", "model_name", "username",
                                "token", "task_id", "checkpoint_uuid"};
}  // namespace

void Store::IndexRow(const std::string& table, int64_t id, const Json& row, bool add) {
  if (!row.is_object()) return;
  for (const char* f : kIndexed) {
    if (!row.has(f)) continue;
    auto& bucket = index_[table][f][row[f].dump()];
    if (add) bucket.insert(id);
    else bucket.erase(id);
  }
}

Store::Store(std::string dir, size_t compact_every) : dir_(std::move(dir)), compact_every_(compact_every) {
  if (!dir_.empty()) {
    ::mkdir(dir_.c_str(), 0755);
    Load();
    wal_ = std::fopen((dir_ + "/wal.jsonl").c_str(), "a");
    if (!wal_) throw std::runtime_error("cannot open WAL in " + dir_);
  }
}

Store::~Store() {
  std::lock_guard<std::mutex> g(mu_);
  if (wal_) {
    std::fflush(wal_);
    ::fsync(fileno(wal_));
    std::fclose(wal_);
    wal_ = nullptr;
  }
}

void Store::Load() {
  std::ifstream snap(dir_ + "/snapshot.json");
  if (snap) {
    std::stringstream ss;
    ss << snap.rdbuf();
    Json j = Json::parse(ss.str());
    for (auto& t : j["tables"].as_object())
      for (auto& r : t.second.as_object()) tables_[t.first][std::stoll(r.first)] = r.second;
    for (auto& s : j["seq"].as_object()) seq_[s.first] = s.second.as_int();
  }
  std::ifstream wal(dir_ + "/wal.jsonl");
  std::string line;
  while (std::getline(wal, line)) {
    if (line.empty()) continue;
    Json e;
    try {
      e = Json::parse(line);
    } catch (const std::exception&) {
      break;  // torn final line from a crash: everything before it is committed
    }
    const std::string& t = e["t"].as_string();
    int64_t k = e["k"].as_int();
    if (e.get_bool("d", false)) tables_[t].erase(k);
    else tables_[t][k] = e["v"];
    if (k > seq_[t]) seq_[t] = k;
    ++wal_entries_;
  }
  for (auto& t : tables_)
    for (auto& r : t.second) IndexRow(t.first, r.first, r.second, true);
}

void Store::Log(const Json& entry) {
  if (!wal_) return;
  std::string line = entry.dump();
  line.push_back('\n');
  std::fwrite(line.data(), 1, line.size(), wal_);
  std::fflush(wal_);
  if (++wal_entries_ >= compact_every_) CompactLocked();
}

int64_t Store::NextID(const std::string& table) {
  std::lock_guard<std::mutex> g(mu_);
  return ++seq_[table];
}

int64_t Store::Insert(const std::string& table, Json row) {
  std::lock_guard<std::mutex> g(mu_);
  int64_t id = ++seq_[table];
  row["id"] = id;
  tables_[table][id] = row;
  IndexRow(table, id, row, true);
  Json e = Json::object();
  e["t"] = table;
  e["k"] = id;
  e["v"] = row;
  Log(e);
  return id;
}

void Store::Put(const std::string& table, int64_t id, Json row) {
  std::lock_guard<std::mutex> g(mu_);
  row["id"] = id;
  auto& tab = tables_[table];
  auto old = tab.find(id);
  if (old != tab.end()) IndexRow(table, id, old->second, false);
  tab[id] = row;
  IndexRow(table, id, row, true);
  if (id > seq_[table]) seq_[table] = id;
  Json e = Json::object();
  e["t"] = table;
  e["k"] = id;
  e["v"] = row;
  Log(e);
}

bool Store::Get(const std::string& table, int64_t id, Json* out) const {
  std::lock_guard<std::mutex> g(mu_);
  auto t = tables_.find(table);
  if (t == tables_.end()) return false;
  auto r = t->second.find(id);
  if (r == t->second.end()) return false;
  *out = r->second;
  return true;
}

bool Store::Delete(const std::string& table, int64_t id) {
  std::lock_guard<std::mutex> g(mu_);
  auto t = tables_.find(table);
  if (t == tables_.end()) return false;
  auto r = t->second.find(id);
  if (r == t->second.end()) return false;
  IndexRow(table, id, r->second, false);
  t->second.erase(r);
  Json e = Json::object();
  e["t"] = table;
  e["k"] = id;
  e["d"] = true;
  Log(e);
  return true;
}

bool Store::Update(const std::string& table, int64_t id, const Json& patch) {
  std::lock_guard<std::mutex> g(mu_);
  auto t = tables_.find(table);
  if (t == tables_.end()) return false;
  auto r = t->second.find(id);
  if (r == t->second.end()) return false;
  Json row = r->second;
  for (auto& kv : patch.as_object()) row[kv.first] = kv.second;
  IndexRow(table, id, r->second, false);
  r->second = row;
  IndexRow(table, id, row, true);
  Json e = Json::object();
  e["t"] = table;
  e["k"] = id;
  e["v"] = row;
  Log(e);
  return true;
}

std::vector<Json> Store::Scan(const std::string& table, const std::function<bool(const Json&)>& pred) const {
  std::lock_guard<std::mutex> g(mu_);
  return ScanLocked(table, pred);
}

std::vector<Json> Store::ScanLocked(const std::string& table, const std::function<bool(const Json&)>& pred) const {
  std::vector<Json> out;
  auto t = tables_.find(table);
  if (t == tables_.end()) return out;
  for (auto& kv : t->second)
    if (!pred || pred(kv.second)) out.push_back(kv.second);
  return out;
}

std::vector<Json> Store::Where(const std::string& table, const std::string& field, const Json& value) const {
  std::lock_guard<std::mutex> g(mu_);
  if (std::find_if(std::begin(kIndexed), std::end(kIndexed), [&](const char* f) { return field == f; }) ==
      std::end(kIndexed))
    return ScanLocked(table, [&](const Json& r) { return r[field] == value; });
  std::vector<Json> out;
  auto ti = index_.find(table);
  auto t = tables_.find(table);
  if (ti == index_.end() || t == tables_.end()) return out;
  auto fi = ti->second.find(field);
  if (fi == ti->second.end()) return out;
  auto b = fi->second.find(value.dump());
  if (b == fi->second.end()) return out;
  for (int64_t id : b->second) {  // ascending id, as a scan would return them
    auto r = t->second.find(id);
    if (r != t->second.end() && r->second[field] == value) out.push_back(r->second);
  }
  return out;
}

size_t Store::Count(const std::string& table) const {
  std::lock_guard<std::mutex> g(mu_);
  auto t = tables_.find(table);
  return t == tables_.end() ? 0 : t->second.size();
}

void Store::DeleteWhere(const std::string& table, const std::function<bool(const Json&)>& pred) {  // NOLINT
  std::vector<int64_t> ids;
  for (auto& r : Scan(table, pred)) ids.push_back(r["id"].as_int());
  for (int64_t id : ids) Delete(table, id);
}

void Store::DeleteWhereEq(const std::string& table, const std::string& field, const Json& value) {
  std::vector<int64_t> ids;
  for (auto& r : Where(table, field, value)) ids.push_back(r["id"].as_int());
  for (int64_t id : ids) Delete(table, id);
}

void Store::Flush() {
  std::lock_guard<std::mutex> g(mu_);
  if (wal_) {
    std::fflush(wal_);
    ::fsync(fileno(wal_));
  }
}

void Store::Compact() {
  std::lock_guard<std::mutex> g(mu_);
  CompactLocked();
}

void Store::CompactLocked() {
  if (dir_.empty()) return;
  Json snap = Json::object();
  Json tables = Json::object();
  for (auto& t : tables_) {
    Json rows = Json::object();
    for (auto& r : t.second) rows[std::to_string(r.first)] = r.second;
    tables[t.first] = rows;
  }
  Json seq = Json::object();
  for (auto& s : seq_) seq[s.first] = s.second;
  snap["tables"] = tables;
  snap["seq"] = seq;
  std::string tmp = dir_ + "/snapshot.json.tmp";
  {
    std::ofstream f(tmp, std::ios::trunc);
    f << snap.dump();
    f.flush();
  }
  ::rename(tmp.c_str(), (dir_ + "/snapshot.json").c_str());
  if (wal_) std::fclose(wal_);
  wal_ = std::fopen((dir_ + "/wal.jsonl").c_str(), "w");
  wal_entries_ = 0;
}

// ---------------------------------------------------------------------------------- LogStore
LogStore::LogStore(std::string dir) : dir_(std::move(dir)) {
  if (dir_.empty()) return;
  ::mkdir(dir_.c_str(), 0755);
}

LogStore::~LogStore() {
  if (!shipper_.joinable()) return;
  if (Flush(5000)) {  // best effort: ship what is queued while the backend answers ...
    try {
      backend_->Refresh();  // ... and make it searchable for whoever reads the index next
    } catch (const std::exception&) {
    }
  }
  {
    std::lock_guard<std::mutex> g(mu_);
    stop_ = true;
  }
  ship_cv_.notify_all();
  shipper_.join();
}

void LogStore::SetBackend(std::unique_ptr<LogBackend> b, LogShipOptions opt) {
  backend_ = std::move(b);
  opt_ = opt;
  if (backend_ && !shipper_.joinable()) shipper_ = std::thread([this] { ShipLoop(); });
}

std::string LogStore::Path(const std::string& stream) const { return dir_ + "/" + stream + ".jsonl"; }

LogStore::Stream& LogStore::Open(const std::string& stream) {
  auto it = streams_.find(stream);
  if (it != streams_.end()) return it->second;
  Stream& s = streams_[stream];
  if (dir_.empty()) return s;
  std::ifstream f(Path(stream), std::ios::binary);
  std::string line;
  uint64_t off = 0;
  while (std::getline(f, line)) {
    if (f.eof() && line.empty()) break;
    s.offsets.push_back(off);
    off += line.size() + 1;
  }
  s.size = off;
  return s;
}

// The stream's state with its next id known: the first touch of a stream (per master lifetime)
// reads the highest id already in the backend, without holding the lock across the request.
LogStore::Remote& LogStore::RemoteLocked(std::unique_lock<std::mutex>& lk, const std::string& stream) {
  Remote* r = &remote_[stream];
  if (r->next > 0) return *r;
  lk.unlock();
  int64_t mx = 0;
  for (int attempt = 0;; ++attempt) {
    try {
      mx = backend_->MaxId(stream);
      break;
    } catch (const std::exception&) {
      if (attempt >= 4) {
        lk.lock();
        throw;
      }
      std::this_thread::sleep_for(std::chrono::milliseconds(50 << attempt));
    }
  }
  lk.lock();
  r = &remote_[stream];  // (map nodes are stable, but the entry may have been erased meanwhile)
  if (r->next == 0) r->next = mx + 1;
  return *r;
}

int64_t LogStore::Append(const std::string& stream, std::vector<Json> rows) {
  if (backend_) {
    std::unique_lock<std::mutex> lk(mu_);
    Remote& r = RemoteLocked(lk, stream);
    if (pending_total_ + static_cast<int64_t>(rows.size()) > opt_.max_pending_lines) {
      if (dropped_ == 0) std::fprintf(stderr, "log shipping: %lld lines queued, dropping new lines\n",
                                      static_cast<long long>(pending_total_));
      dropped_ += static_cast<int64_t>(rows.size());
      return r.next - 1;
    }
    if (pending_total_ == 0) oldest_pending_ = std::chrono::steady_clock::now();
    for (auto& row : rows) {
      row["id"] = r.next++;
      r.pending.push_back(std::move(row));
    }
    pending_total_ += static_cast<int64_t>(rows.size());
    const int64_t last = r.next - 1;
    lk.unlock();
    ship_cv_.notify_one();  // the shipper times the 20 ms flush from the oldest queued line
    return last;
  }
  std::lock_guard<std::mutex> g(mu_);
  Stream& s = Open(stream);
  std::string buf;
  for (auto& r : rows) {
    r["id"] = static_cast<int64_t>(s.offsets.size() + 1);
    std::string line = r.dump();
    s.offsets.push_back(s.size + buf.size());
    if (dir_.empty()) s.mem.push_back(line);
    buf += line;
    buf.push_back('\n');
  }
  if (!dir_.empty() && !buf.empty()) {
    FILE* f = std::fopen(Path(stream).c_str(), "ab");
    if (!f) throw std::runtime_error("cannot append to log segment " + Path(stream));
    std::fwrite(buf.data(), 1, buf.size(), f);
    std::fclose(f);
  }
  s.size += buf.size();
  return static_cast<int64_t>(s.offsets.size());
}

void LogStore::ShipLoop() {
  using clock = std::chrono::steady_clock;
  int backoff_ms = 0;
  auto last_refresh = clock::now();
  std::unique_lock<std::mutex> lk(mu_);
  for (;;) {
    // wait for a batch: batch_lines queued, the oldest line flush_ms old, or a refresh due
    for (;;) {
      if (stop_ && pending_total_ == 0) return;
      const auto now = clock::now();
      const bool refresh_due = acked_total_ > 0 && now - last_refresh >= std::chrono::milliseconds(opt_.refresh_ms);
      if (refresh_due || stop_) break;
      if (pending_total_ > 0 &&
          (pending_total_ >= opt_.batch_lines || now - oldest_pending_ >= std::chrono::milliseconds(opt_.flush_ms)))
        break;
      auto until = now + std::chrono::milliseconds(pending_total_ > 0 ? opt_.flush_ms : opt_.refresh_ms);
      if (pending_total_ > 0) until = oldest_pending_ + std::chrono::milliseconds(opt_.flush_ms);
      if (acked_total_ > 0) until = std::min(until, last_refresh + std::chrono::milliseconds(opt_.refresh_ms));
      ship_cv_.wait_until(lk, until);
    }
    if (acked_total_ > 0 && clock::now() - last_refresh >= std::chrono::milliseconds(opt_.refresh_ms)) {
      // retire acknowledged rows: after a refresh that started later than their ack they are
      // searchable, so readers no longer need the in-memory copies
      const int64_t upto = ack_seq_;
      lk.unlock();
      bool ok = true;
      try {
        backend_->Refresh();
      } catch (const std::exception& e) {
        ok = false;
        lk.lock();
        last_error_ = e.what();
        lk.unlock();
      }
      lk.lock();
      last_refresh = clock::now();
      if (ok) {
        ++refreshes_;
        for (auto& kv : remote_) {
          auto& a = kv.second.acked;
          while (!a.empty() && a.front().first <= upto) {
            a.pop_front();
            --acked_total_;
          }
        }
      }
    }
    if (pending_total_ == 0) continue;
    // take up to max_batch_lines rows, stream by stream
    std::vector<std::pair<std::string, std::vector<Json>>> batch;
    int64_t n = 0;
    for (auto& kv : remote_) {
      Remote& r = kv.second;
      if (r.pending.empty() || !r.inflight.empty() || r.deleting) continue;
      std::vector<Json> rows;
      while (!r.pending.empty() && n < opt_.max_batch_lines) {
        rows.push_back(r.pending.front());  // the queued copy stays readable via inflight
        r.pending.pop_front();
        ++n;
      }
      r.inflight = rows;
      batch.emplace_back(kv.first, std::move(rows));
      if (n >= opt_.max_batch_lines) break;
    }
    if (n == 0) {  // (only streams being deleted hold lines)
      ship_cv_.wait_for(lk, std::chrono::milliseconds(opt_.flush_ms));
      continue;
    }
    pending_total_ -= n;
    inflight_total_ += n;
    lk.unlock();
    std::vector<bool> ok(batch.size(), false);
    std::string err;
    for (size_t i = 0; i < batch.size(); ++i) {
      try {
        backend_->Index(batch[i].first, batch[i].second);
        ok[i] = true;
      } catch (const std::exception& e) {
        err = e.what();
      }
    }
    lk.lock();
    bool any_fail = false;
    for (size_t i = 0; i < batch.size(); ++i) {
      auto it = remote_.find(batch[i].first);
      const int64_t k = static_cast<int64_t>(batch[i].second.size());
      inflight_total_ -= k;
      if (it == remote_.end()) continue;
      Remote& r = it->second;
      r.inflight.clear();
      if (ok[i]) {
        const int64_t seq = ++ack_seq_;
        for (auto& row : batch[i].second) r.acked.emplace_back(seq, std::move(row));
        acked_total_ += k;
        shipped_ += k;
      } else if (!r.deleting) {
        // back to the front of the queue, in order: the next attempt re-sends the same ids
        for (auto row = batch[i].second.rbegin(); row != batch[i].second.rend(); ++row) r.pending.push_front(*row);
        pending_total_ += k;
        any_fail = true;
      }
    }
    ++batches_;
    idle_cv_.notify_all();
    if (any_fail) {
      ++failures_;
      last_error_ = err;
      oldest_pending_ = clock::now() - std::chrono::milliseconds(opt_.flush_ms);  // retry without waiting for more
      backoff_ms = backoff_ms == 0 ? 50 : std::min(backoff_ms * 2, opt_.max_backoff_ms);
      ship_cv_.wait_for(lk, std::chrono::milliseconds(backoff_ms), [this] { return stop_; });
      if (stop_) return;  // shutting down with the backend failing: Flush already gave up
    } else {
      backoff_ms = 0;
    }
  }
}

bool LogStore::Flush(int timeout_ms) {
  if (!backend_) return true;
  std::unique_lock<std::mutex> lk(mu_);
  ship_cv_.notify_all();
  return idle_cv_.wait_for(lk, std::chrono::milliseconds(timeout_ms),
                           [this] { return pending_total_ == 0 && inflight_total_ == 0; });
}

Json LogStore::Stats() const {
  std::lock_guard<std::mutex> g(mu_);
  Json out = Json::object();
  out["backend"] = backend_ != nullptr;
  out["pending_lines"] = static_cast<long long>(pending_total_);
  out["inflight_lines"] = static_cast<long long>(inflight_total_);
  out["unrefreshed_lines"] = static_cast<long long>(acked_total_);
  out["shipped_lines"] = static_cast<long long>(shipped_);
  out["batches"] = static_cast<long long>(batches_);
  out["failed_batches"] = static_cast<long long>(failures_);
  out["dropped_lines"] = static_cast<long long>(dropped_);
  out["refreshes"] = static_cast<long long>(refreshes_);
  out["last_error"] = last_error_;
  return out;
}

std::vector<Json> LogStore::Read(const std::string& stream, int64_t after_id, int64_t limit,
                                 const std::function<bool(const Json&)>& pred, bool tail) {
  std::vector<Json> out;
  if (backend_) {
    if (after_id < 0) after_id = 0;
    if (limit <= 0) return out;
    // the in-memory suffix of the stream (acknowledged-but-unrefreshed, in flight, queued: ids
    // ascending and contiguous) and the backend below it
    std::vector<Json> mem;
    int64_t mem_min = INT64_MAX;
    {
      std::unique_lock<std::mutex> lk(mu_);
      Remote& r = RemoteLocked(lk, stream);
      auto take = [&](const Json& row) {
        const int64_t id = row.get_int("id", 0);
        mem_min = std::min(mem_min, id);
        if (id > after_id) mem.push_back(row.clone());
      };
      for (auto& a : r.acked) take(a.second);
      for (auto& row : r.inflight) take(row);
      for (auto& row : r.pending) take(row);
    }
    const int64_t page = std::min<int64_t>(std::max<int64_t>(limit, 256), 5000);
    if (!tail) {  // ascending pages from after_id (below the memory suffix), then the suffix
      if (after_id + 1 < mem_min) {
        for (int64_t cur = after_id;;) {
          auto rows = backend_->Search(stream, cur, mem_min, page, false);
          for (auto& row : rows) {
            cur = row.get_int("id", cur);
            if (pred && !pred(row)) continue;
            out.push_back(std::move(row));
            if (static_cast<int64_t>(out.size()) >= limit) return out;
          }
          if (static_cast<int64_t>(rows.size()) < page) break;
        }
      }
      for (auto& row : mem) {
        if (pred && !pred(row)) continue;
        out.push_back(std::move(row));
        if (static_cast<int64_t>(out.size()) >= limit) break;
      }
      return out;
    }
    // tail: the memory suffix from its end, then descending backend pages below it
    std::vector<Json> rev;
    for (auto it = mem.rbegin(); it != mem.rend() && static_cast<int64_t>(rev.size()) < limit; ++it)
      if (!pred || pred(*it)) rev.push_back(std::move(*it));
    for (int64_t before = mem_min; static_cast<int64_t>(rev.size()) < limit && after_id + 1 < before;) {
      auto rows = backend_->Search(stream, after_id, before, page, true);
      for (auto it = rows.rbegin(); it != rows.rend(); ++it) {
        before = it->get_int("id", before);
        if (pred && !pred(*it)) continue;
        rev.push_back(std::move(*it));
        if (static_cast<int64_t>(rev.size()) >= limit) break;
      }
      if (static_cast<int64_t>(rows.size()) < page) break;
    }
    out.assign(std::make_move_iterator(rev.rbegin()), std::make_move_iterator(rev.rend()));
    return out;
  }
  std::lock_guard<std::mutex> g(mu_);
  Stream& s = Open(stream);
  const int64_t n = static_cast<int64_t>(s.offsets.size());
  if (after_id < 0) after_id = 0;
  if (after_id >= n || limit <= 0) return out;
  std::ifstream f;
  if (!dir_.empty()) {
    f.open(Path(stream), std::ios::binary);
    f.seekg(static_cast<std::streamoff>(s.offsets[static_cast<size_t>(after_id)]));
  }
  std::string line;
  for (int64_t i = after_id; i < n; ++i) {
    if (dir_.empty()) line = s.mem[static_cast<size_t>(i)];
    else if (!std::getline(f, line)) break;
    Json row;
    try {
      row = Json::parse(line);
    } catch (const std::exception&) {
      continue;
    }
    if (pred && !pred(row)) continue;
    out.push_back(std::move(row));
    if (!tail && static_cast<int64_t>(out.size()) >= limit) break;
  }
  if (tail && static_cast<int64_t>(out.size()) > limit) out.erase(out.begin(), out.end() - limit);
  return out;
}

int64_t LogStore::Count(const std::string& stream) {
  std::unique_lock<std::mutex> lk(mu_);
  if (backend_) return RemoteLocked(lk, stream).next - 1;
  auto it = streams_.find(stream);
  if (it != streams_.end()) return static_cast<int64_t>(it->second.offsets.size());
  return Open(stream).offsets.size();
}

void LogStore::Delete(const std::string& stream) {
  std::unique_lock<std::mutex> lk(mu_);
  if (backend_) {
    Remote& r = remote_[stream];
    r.deleting = true;
    pending_total_ -= static_cast<int64_t>(r.pending.size());
    acked_total_ -= static_cast<int64_t>(r.acked.size());
    r.pending.clear();
    r.acked.clear();
    idle_cv_.wait(lk, [&] { return remote_[stream].inflight.empty(); });  // a request in flight lands first
    lk.unlock();
    std::exception_ptr err;
    try {
      backend_->Delete(stream);
    } catch (...) {
      err = std::current_exception();
    }
    lk.lock();
    remote_.erase(stream);
    if (err) std::rethrow_exception(err);
    return;
  }
  streams_.erase(stream);
  if (!dir_.empty()) ::unlink(Path(stream).c_str());
}

}  // namespace detcore
