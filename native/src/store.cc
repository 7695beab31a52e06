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

LogStore::~LogStore() = default;

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

int64_t LogStore::RemoteMax(const std::string& stream) {
  auto it = remote_next_.find(stream);
  if (it == remote_next_.end()) it = remote_next_.emplace(stream, backend_->MaxId(stream) + 1).first;
  return it->second - 1;
}

int64_t LogStore::Append(const std::string& stream, std::vector<Json> rows) {
  std::lock_guard<std::mutex> g(mu_);
  if (backend_) {
    int64_t id = RemoteMax(stream);
    for (auto& r : rows) r["id"] = ++id;
    backend_->Index(stream, rows);
    remote_next_[stream] = id + 1;
    return id;
  }
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

std::vector<Json> LogStore::Read(const std::string& stream, int64_t after_id, int64_t limit,
                                 const std::function<bool(const Json&)>& pred, bool tail) {
  std::lock_guard<std::mutex> g(mu_);
  std::vector<Json> out;
  if (backend_) {
    if (after_id < 0) after_id = 0;
    if (limit <= 0) return out;
    const int64_t page = std::min<int64_t>(std::max<int64_t>(limit, 256), 5000);
    if (!tail) {  // ascending pages from after_id until `limit` rows pass the filter
      for (int64_t cur = after_id;;) {
        auto rows = backend_->Search(stream, cur, INT64_MAX, page, false);
        for (auto& r : rows) {
          cur = r.get_int("id", cur);
          if (pred && !pred(r)) continue;
          out.push_back(std::move(r));
          if (static_cast<int64_t>(out.size()) >= limit) return out;
        }
        if (static_cast<int64_t>(rows.size()) < page) return out;
      }
    }
    // tail: descending pages from the end until `limit` rows pass the filter
    std::vector<Json> rev;
    for (int64_t before = INT64_MAX;;) {
      auto rows = backend_->Search(stream, after_id, before, page, true);
      for (auto it = rows.rbegin(); it != rows.rend(); ++it) {
        before = it->get_int("id", before);
        if (pred && !pred(*it)) continue;
        rev.push_back(std::move(*it));
        if (static_cast<int64_t>(rev.size()) >= limit) break;
      }
      if (static_cast<int64_t>(rev.size()) >= limit || static_cast<int64_t>(rows.size()) < page) break;
    }
    out.assign(std::make_move_iterator(rev.rbegin()), std::make_move_iterator(rev.rend()));
    return out;
  }
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

int64_t LogStore::Count(const std::string& stream) const {
  std::lock_guard<std::mutex> g(mu_);
  if (backend_) return const_cast<LogStore*>(this)->RemoteMax(stream);
  auto it = streams_.find(stream);
  if (it != streams_.end()) return static_cast<int64_t>(it->second.offsets.size());
  return const_cast<LogStore*>(this)->Open(stream).offsets.size();
}

void LogStore::Delete(const std::string& stream) {
  std::lock_guard<std::mutex> g(mu_);
  if (backend_) {
    backend_->Delete(stream);
    remote_next_.erase(stream);
    return;
  }
  streams_.erase(stream);
  if (!dir_.empty()) ::unlink(Path(stream).c_str());
}

}  // namespace detcore
