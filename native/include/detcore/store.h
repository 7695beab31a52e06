// Embedded durable store for the master (replaces the reference's Postgres).
//
// Tables are id-keyed JSON rows held in memory and made durable by an append-only write-ahead
// log (one JSON line per mutation, fsync'd in batches) plus periodic snapshot compaction:
//   <dir>/snapshot.json   {"tables": {name: {id: row}}, "seq": {name: last_id}}
//   <dir>/wal.jsonl       {"t": table, "k": id, "v": row} | {"t": table, "k": id, "d": true}
// Opening replays snapshot + WAL, so a restarted master sees every committed row (experiments,
// trials, steps, validations, checkpoints, searcher_events, trial_logs, templates, models, ...).
// All methods are thread-safe.
#pragma once

#include <cstdint>
#include <cstdio>
#include <functional>
#include <map>
#include <mutex>
#include <string>
#include <vector>

#include "detcore/json.h"

namespace detcore {

class Store {
 public:
  // dir empty => memory only (tests).
  explicit Store(std::string dir = "", size_t compact_every = 20000);
  ~Store();

  int64_t NextID(const std::string& table);
  // Insert with a fresh id (row["id"] is set); returns the id.
  int64_t Insert(const std::string& table, Json row);
  void Put(const std::string& table, int64_t id, Json row);
  bool Get(const std::string& table, int64_t id, Json* out) const;
  bool Delete(const std::string& table, int64_t id);
  // Merge top-level fields of `patch` into the row (no-op if missing); returns false if missing.
  bool Update(const std::string& table, int64_t id, const Json& patch);
  std::vector<Json> Scan(const std::string& table, const std::function<bool(const Json&)>& pred = nullptr) const;
  std::vector<Json> Where(const std::string& table, const std::string& field, const Json& value) const;
  size_t Count(const std::string& table) const;
  void DeleteWhere(const std::string& table, const std::function<bool(const Json&)>& pred);
  void Flush();     // fsync the WAL
  void Compact();   // snapshot + truncate WAL
  const std::string& dir() const { return dir_; }

 private:
  void Load();
  void Log(const Json& entry);
  void CompactLocked();
  std::string dir_;
  size_t compact_every_;
  size_t wal_entries_ = 0;
  mutable std::mutex mu_;
  std::map<std::string, std::map<int64_t, Json>> tables_;
  std::map<std::string, int64_t> seq_;
  FILE* wal_ = nullptr;
};

}  // namespace detcore
