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

#include <chrono>
#include <condition_variable>
#include <cstdint>
#include <cstdio>
#include <functional>
#include <deque>
#include <map>
#include <memory>
#include <mutex>
#include <set>
#include <string>
#include <thread>
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
// Called from the LogStore's shipper thread (Index, Refresh) and from readers (Search, MaxId,
// Delete) concurrently: implementations are thread-safe.
class LogBackend {
 public:
  virtual ~LogBackend() = default;
  // Index rows (idempotent per (stream, id): a retried batch overwrites, never duplicates).  Throws
  // on any failure, including per-item errors.
  virtual void Index(const std::string& stream, const std::vector<Json>& rows) = 0;
  // Make everything indexed so far searchable (Elasticsearch _refresh); a no-op by default.
  virtual void Refresh() {}
  // Rows with after_id < id < before_id, `limit` of them from the low end (or the high end when
  // desc), returned in ascending id order.
  virtual std::vector<Json> Search(const std::string& stream, int64_t after_id, int64_t before_id, int64_t limit,
                                   bool desc) = 0;
  virtual int64_t MaxId(const std::string& stream) = 0;  // 0 for an empty / unknown stream
  virtual void Delete(const std::string& stream) = 0;
};
// Elasticsearch backend over its REST API (_bulk / _search / _delete_by_query / _refresh on one
// index, created with a keyword mapping for the stream name).
std::unique_ptr<LogBackend> MakeElasticLogBackend(const std::string& host, int port, const std::string& index);

// Backend-mode shipping (reference master/internal/trial_logger.go:11-19: a logger actor buffers
// up to 1000 lines or 20 ms): Append assigns ids and queues rows in memory -- no network I/O on the
// caller's thread (the agent socket) -- and a shipper thread sends them in batches, retrying with
// backoff while the backend fails (no line is lost; idempotent ids).  Rows stay readable from
// memory until a backend refresh has made them searchable, so a follower never skips an id.
struct LogShipOptions {
  int batch_lines = 1000;         // ship as soon as this many lines are queued
  int flush_ms = 20;              // ... or when the oldest queued line is this old
  int max_batch_lines = 5000;     // rows per shipping request
  int refresh_ms = 1000;          // min interval between backend refreshes that retire acked rows
  int max_backoff_ms = 5000;
  int64_t max_pending_lines = 4000000;  // beyond this, new lines are dropped (counted, logged)
};

class LogStore {
 public:
  explicit LogStore(std::string dir = "");
  ~LogStore();
  // Route every stream to `b` (local segments are then not written) through the shipper thread.
  void SetBackend(std::unique_ptr<LogBackend> b, LogShipOptions opt = LogShipOptions());
  // Appends rows to `stream`, setting row["id"]; returns the last id.
  int64_t Append(const std::string& stream, std::vector<Json> rows);
  // Entries with id > after_id passing `pred`, at most `limit` (the last `limit` when tail).
  std::vector<Json> Read(const std::string& stream, int64_t after_id, int64_t limit,
                         const std::function<bool(const Json&)>& pred = nullptr, bool tail = false);
  int64_t Count(const std::string& stream);
  void Delete(const std::string& stream);
  // Backend mode: wait until every queued line is acknowledged (false on timeout).
  bool Flush(int timeout_ms);
  // Shipper counters: pending / inflight / unrefreshed lines, shipped, batches, failures, dropped.
  Json Stats() const;

 private:
  struct Stream {
    std::vector<uint64_t> offsets;  // byte offset of every line
    uint64_t size = 0;
    std::vector<std::string> mem;   // memory-only mode
  };
  struct Remote {
    int64_t next = 0;          // next id to assign; 0 = not read from the backend yet
    std::deque<Json> pending;  // ids assigned, not sent
    std::vector<Json> inflight;  // in a shipping request
    std::deque<std::pair<int64_t, Json>> acked;  // (ack sequence, row): acknowledged, maybe not searchable yet
    bool deleting = false;
  };
  std::string Path(const std::string& stream) const;
  Stream& Open(const std::string& stream);  // loads the offsets of an existing segment
  Remote& RemoteLocked(std::unique_lock<std::mutex>& lk, const std::string& stream);  // next id known
  void ShipLoop();
  std::string dir_;
  mutable std::mutex mu_;
  std::map<std::string, Stream> streams_;
  std::unique_ptr<LogBackend> backend_;
  LogShipOptions opt_;
  std::map<std::string, Remote> remote_;
  std::condition_variable ship_cv_, idle_cv_;
  std::thread shipper_;
  bool stop_ = false;
  int64_t pending_total_ = 0, inflight_total_ = 0, acked_total_ = 0;
  std::chrono::steady_clock::time_point oldest_pending_{};
  int64_t ack_seq_ = 0;
  int64_t shipped_ = 0, batches_ = 0, failures_ = 0, dropped_ = 0, refreshes_ = 0;
  std::string last_error_;
};

}  // namespace detcore
