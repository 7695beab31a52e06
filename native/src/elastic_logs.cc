// Elasticsearch trial/task log backend for LogStore.
//
// Reference: master/internal/elastic/elastic_trial_logs.go:38-95 (AddTrialLogs = one _bulk request,
// TrialLogs = filtered search ordered by a tiebreak key with search_after paging, TrialLogCount,
// DeleteTrialLogs = _delete_by_query) and master/internal/config/elastic.go (logging.type: elastic,
// host, port).  Here every document carries the LogStore stream name ("trial-<id>", "task-<id>") and
// the per-stream id the master assigns, so paging is a range filter on `id` and the same cursors
// clients follow against the local segments keep working unchanged.
#include <algorithm>
#include <climits>
#include <stdexcept>

#include "detcore/net.h"
#include "detcore/store.h"

namespace detcore {

namespace {

class ElasticLogBackend : public LogBackend {
 public:
  ElasticLogBackend(std::string host, int port, std::string index)
      : host_(std::move(host)), port_(port), index_(std::move(index)) {}

  void Index(const std::string& stream, const std::vector<Json>& rows) override {
    if (rows.empty()) return;
    std::string body;
    for (const auto& r : rows) {
      Json meta = Json::object();
      meta["index"]["_index"] = index_;
      meta["index"]["_id"] = stream + ":" + std::to_string(r.get_int("id", 0));
      Json doc = r.clone();
      doc["stream"] = stream;
      body += meta.dump();
      body.push_back('\n');
      body += doc.dump();
      body.push_back('\n');
    }
    // refresh=wait_for: a log line is searchable when the shipping request returns, so a client
    // following the stream never skips an id that is still being indexed.
    Json resp = Call("POST", "/_bulk?refresh=wait_for", body, "application/x-ndjson");
    if (resp.get_bool("errors", false)) throw std::runtime_error("elasticsearch _bulk reported item errors");
  }

  std::vector<Json> Search(const std::string& stream, int64_t after_id, int64_t before_id, int64_t limit,
                           bool desc) override {
    Json q = Json::object();
    q["size"] = static_cast<long long>(limit);
    Json filters = Json::array();
    Json term = Json::object();
    term["term"]["stream"] = stream;
    filters.push_back(term);
    Json range = Json::object();
    range["range"]["id"]["gt"] = static_cast<long long>(after_id);
    if (before_id != INT64_MAX) range["range"]["id"]["lt"] = static_cast<long long>(before_id);
    filters.push_back(range);
    q["query"]["bool"]["filter"] = filters;
    Json sort = Json::array();
    Json key = Json::object();
    key["id"] = desc ? "desc" : "asc";
    sort.push_back(key);
    q["sort"] = sort;
    std::vector<Json> out;
    Json resp = Call("POST", "/" + index_ + "/_search", q.dump(), "application/json", /*missing_ok=*/true);
    const Json& hits = resp["hits"]["hits"];
    if (hits.is_array())
      for (const auto& h : hits.as_array()) {
        Json src = h["_source"].clone();
        if (src.is_object()) src.as_object().erase("stream");
        out.push_back(std::move(src));
      }
    if (desc) std::reverse(out.begin(), out.end());
    return out;
  }

  int64_t MaxId(const std::string& stream) override {
    auto rows = Search(stream, 0, INT64_MAX, 1, true);
    return rows.empty() ? 0 : rows.back().get_int("id", 0);
  }

  void Delete(const std::string& stream) override {
    Json q = Json::object();
    q["query"]["term"]["stream"] = stream;
    Call("POST", "/" + index_ + "/_delete_by_query?refresh=true", q.dump(), "application/json", true);
  }

 private:
  Json Call(const std::string& method, const std::string& path, const std::string& body, const std::string& ctype,
            bool missing_ok = false) {
    auto r = net::HttpCall(host_, port_, method, path, body, 30000, ctype);
    if (!r.error.empty()) throw std::runtime_error("elasticsearch " + path + ": " + r.error);
    if (r.status == 404 && missing_ok) return Json::object();  // index not created yet
    if (r.status < 200 || r.status >= 300)
      throw std::runtime_error("elasticsearch " + path + ": HTTP " + std::to_string(r.status) + " " + r.body);
    return r.body.empty() ? Json::object() : Json::parse(r.body);
  }

  std::string host_;
  int port_;
  std::string index_;
};

}  // namespace

std::unique_ptr<LogBackend> MakeElasticLogBackend(const std::string& host, int port, const std::string& index) {
  return std::make_unique<ElasticLogBackend>(host, port, index);
}

}  // namespace detcore
