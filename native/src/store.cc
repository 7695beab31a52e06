// Embedded durable store (see include/detcore/store.h).
#include "detcore/store.h"

#include <sys/stat.h>
#include <unistd.h>

#include <fstream>
#include <sstream>
#include <stdexcept>

namespace detcore {

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
  tables_[table][id] = row;
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
  if (t == tables_.end() || !t->second.erase(id)) return false;
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
  r->second = row;
  Json e = Json::object();
  e["t"] = table;
  e["k"] = id;
  e["v"] = row;
  Log(e);
  return true;
}

std::vector<Json> Store::Scan(const std::string& table, const std::function<bool(const Json&)>& pred) const {
  std::lock_guard<std::mutex> g(mu_);
  std::vector<Json> out;
  auto t = tables_.find(table);
  if (t == tables_.end()) return out;
  for (auto& kv : t->second)
    if (!pred || pred(kv.second)) out.push_back(kv.second);
  return out;
}

std::vector<Json> Store::Where(const std::string& table, const std::string& field, const Json& value) const {
  return Scan(table, [&](const Json& r) { return r[field] == value; });
}

size_t Store::Count(const std::string& table) const {
  std::lock_guard<std::mutex> g(mu_);
  auto t = tables_.find(table);
  return t == tables_.end() ? 0 : t->second.size();
}

void Store::DeleteWhere(const std::string& table, const std::function<bool(const Json&)>& pred) {
  std::vector<int64_t> ids;
  for (auto& r : Scan(table, pred)) ids.push_back(r["id"].as_int());
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

}  // namespace detcore
