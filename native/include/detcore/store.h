// Embedded durable store for the master (replaces the reference's Postgres).
//
// Tables are id-keyed JSON rows held in memory and made durable by an append-only write-ahead
// log (one JSON line per mutation, fsync'd in batches) plus periodic snapshot compaction:
//   <dir>/snapshot.json   {"tables": {name: {id: row}}, "seq": {name: last_id}}
//   <dir>/wal.jsonl       {"t": table, "k": id, "v": row} | {"t": table, "k": id, "d": true}
// Opening replays snapshot + WAL, so a restarted master sees every committed row (experiments,
// trials, steps, validations, checkpoints, searcher_events, trial_logs, templates, models, ...).
// Secondary indexes on the foreign-key / lookup columns (experiment_id, trial_id, uuid, name, ...)
// make Where() a hash lookup instead of a table scan.  High-volume append-only streams (trial and
// task logs) do not live here: see LogStore.
// All methods are thread-safe.
#pragma once

#include <cstdint>
#include <cstdio>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <set>
#include <string>
#include <unordered_map>
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
  // Delete every row whose indexed `field` equals `value` (index lookup, no scan).
  void DeleteWhereEq(const std::string& table, const std::string& field, const Json& value);
  void Flush();     // fsync the WAL
  void Compact();   // snapshot + truncate WAL
  const std::string& dir() const { return dir_; }

 private:
  void Load();
  void Log(const Json& entry);
  void CompactLocked();
  void IndexRow(const std::string& table, int64_t id, const Json& row, bool add);
  std::vector<Json> ScanLocked(const std::string& table, const std::function<bool(const Json&)>& pred) const;
  // table -> field -> value key -> row ids
  std::map<std::string, std::map<std::string, std::unordered_map<std::string, std::set<int64_t>>>> index_;
  std::string dir_;
  size_t compact_every_;
  size_t wal_entries_ = 0;
  mutable std::mutex mu_;
  std::map<std::string, std::map<int64_t, Json>> tables_;
  std::map<std::string, int64_t> seq_;
  FILE* wal_ = nullptr;
};

// Append-only, per-stream log segments (trial / task logs): <dir>/logs/<stream>.jsonl, one JSON
// line per entry, with only the byte offset of each line kept in memory (8 B/line), so a long
// HP search with millions of log lines costs disk, not master RSS.  Entry ids are 1-based line
// numbers per stream (the cursor clients follow).  Memory-only when dir is empty (tests).
// Remote log index behind a LogStore (reference master/internal/elastic/elastic_trial_logs.go:
// trial logs in Elasticsearch instead of the database).  Rows carry the LogStore's per-stream id.
class LogBackend {
 public:
  virtual ~LogBackend() = default;
  virtual void Index(const std::string& stream, const std::vector<Json>& rows) = 0;
  // Rows with after_id < id < before_id, `limit` of them from the low end (or the high end when
  // desc), returned in ascending id order.
  virtual std::vector<Json> Search(const std::string& stream, int64_t after_id, int64_t before_id, int64_t limit,
                                   bool desc) = 0;
  virtual int64_t MaxId(const std::string& stream) = 0;  // 0 for an empty / unknown stream
  virtual void Delete(const std::string& stream) = 0;
};
// Elasticsearch backend over its REST API (_bulk / _search / _delete_by_query on one index).
std::unique_ptr<LogBackend> MakeElasticLogBackend(const std::string& host, int port, const std::string& index);

class LogStore {
 public:
  explicit LogStore(std::string dir = "");
  ~LogStore();
  // Route every stream to `b` (local segments are then not written).
  void SetBackend(std::unique_ptr<LogBackend> b) { backend_ = std::move(b); }
  // Appends rows to `stream`, setting row["id"]; returns the last id.
  int64_t Append(const std::string& stream, std::vector<Json> rows);
  // Entries with id > after_id passing `pred`, at most `limit` (the last `limit` when tail).
  std::vector<Json> Read(const std::string& stream, int64_t after_id, int64_t limit,
                         const std::function<bool(const Json&)>& pred = nullptr, bool tail = false);
  int64_t Count(const std::string& stream) const;
  void Delete(const std::string& stream);

 private:
  struct Stream {
    std::vector<uint64_t> offsets;  // byte offset of every line
    uint64_t size = 0;
    std::vector<std::string> mem;   // memory-only mode
  };
  std::string Path(const std::string& stream) const;
  Stream& Open(const std::string& stream);  // loads the offsets of an existing segment
  std::string dir_;
  mutable std::mutex mu_;
  std::map<std::string, Stream> streams_;
  std::unique_ptr<LogBackend> backend_;
  std::map<std::string, int64_t> remote_next_;  // next id per stream on the backend
  int64_t RemoteMax(const std::string& stream);
};

}  // namespace detcore
