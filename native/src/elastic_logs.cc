// Elasticsearch trial/task log backend for LogStore.
//
// Shipping runs on the LogStore's shipper thread (batched, retried, never on the agent socket);
// _bulk does not wait for a refresh -- LogStore keeps acknowledged rows readable in memory until
// its periodic Refresh() has made them searchable.  The stream name is filtered as a keyword: the
// index is created with an explicit mapping (stream: keyword, id: long), and an index that already
// exists with Elasticsearch's dynamic mapping (stream: text + stream.keyword) is queried on
// stream.keyword -- a term query on the analysed text field would match nothing ("trial-7" is
// indexed as the tokens "trial" and "7"; reference elastic_trial_logs.go filters on .keyword too).
//
// Reference: master/internal/elastic/elastic_trial_logs.go:38-95 (AddTrialLogs = one _bulk request,
// TrialLogs = filtered search ordered by a tiebreak key with search_after paging, TrialLogCount,
// DeleteTrialLogs = _delete_by_query) and master/internal/config/elastic.go (logging.type: elastic,
// host, port).  Here every document carries the LogStore stream name ("trial-<id>", "task-<id>") and
// the per-stream id the master assigns, so paging is a range filter on `id` and the same cursors
// clients follow against the local segments keep working unchanged.
#include <algorithm>
#include <climits>
#include <mutex>
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
    EnsureIndex();
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
    Json resp = Call("POST", "/_bulk", body, "application/x-ndjson");
    if (resp.get_bool("errors", false)) throw std::runtime_error("elasticsearch _bulk reported item errors");
  }

  void Refresh() override { Call("POST", "/" + index_ + "/_refresh", "", "application/json", /*missing_ok=*/true); }

  std::vector<Json> Search(const std::string& stream, int64_t after_id, int64_t before_id, int64_t limit,
                           bool desc) override {
    const std::string field = StreamField();
    Json q = Json::object();
    q["size"] = static_cast<long long>(limit);
    Json filters = Json::array();
    Json term = Json::object();
    term["term"][field] = stream;
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
    q["query"]["term"][StreamField()] = stream;
    Call("POST", "/" + index_ + "/_delete_by_query?refresh=true", q.dump(), "application/json", true);
  }

 private:
  // Create the index with a keyword mapping, or learn how an existing one maps `stream`.
  void EnsureIndex() {
    std::lock_guard<std::mutex> g(mu_);
    if (!field_.empty()) return;
    auto r = net::HttpCall(host_, port_, "GET", "/" + index_ + "/_mapping", "", 30000, "application/json");
    if (!r.error.empty()) throw std::runtime_error("elasticsearch _mapping: " + r.error);
    if (r.status == 404) {
      Json m = Json::object();
      m["mappings"]["properties"]["stream"]["type"] = "keyword";
      m["mappings"]["properties"]["id"]["type"] = "long";
      auto c = net::HttpCall(host_, port_, "PUT", "/" + index_, m.dump(), 30000, "application/json");
      if (!c.error.empty()) throw std::runtime_error("elasticsearch create index: " + c.error);
      // 400 resource_already_exists: another master created it between the two calls
      if ((c.status < 200 || c.status >= 300) && c.body.find("resource_already_exists") == std::string::npos)
        throw std::runtime_error("elasticsearch create index: HTTP " + std::to_string(c.status) + " " + c.body);
      if (c.status >= 200 && c.status < 300) {
        field_ = "stream";
        return;
      }
      r = net::HttpCall(host_, port_, "GET", "/" + index_ + "/_mapping", "", 30000, "application/json");
    }
    if (r.status < 200 || r.status >= 300)
      throw std::runtime_error("elasticsearch _mapping: HTTP " + std::to_string(r.status) + " " + r.body);
    Json body = Json::parse(r.body);
    const Json* props = nullptr;
    if (body.is_object())
      for (auto& kv : body.as_object()) {  // {"<index or its alias target>": {"mappings": {"properties": ...}}}
        props = &kv.second["mappings"]["properties"];
        break;
      }
    const Json* st = props && props->is_object() && props->as_object().count("stream") ? &(*props)["stream"] : nullptr;
    if (!st || st->get_string("type", "") == "keyword") {
      field_ = "stream";  // keyword (or not mapped yet: the template / first document decides)
    } else if ((*st)["fields"]["keyword"].get_string("type", "") == "keyword") {
      field_ = "stream.keyword";
    } else {
      throw std::runtime_error("elasticsearch index " + index_ + " maps `stream` as " + st->get_string("type", "?") +
                               " without a keyword sub-field: log queries cannot filter on it");
    }
  }

  std::string StreamField() {
    EnsureIndex();
    std::lock_guard<std::mutex> g(mu_);
    return field_;
  }

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
  std::mutex mu_;
  std::string field_;  // "stream" or "stream.keyword", once the index is known
};

}  // namespace

std::unique_ptr<LogBackend> MakeElasticLogBackend(const std::string& host, int port, const std::string& index) {
  return std::make_unique<ElasticLogBackend>(host, port, index);
}

}  // namespace detcore
