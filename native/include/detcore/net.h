// Minimal HTTP/1.1 + WebSocket (RFC 6455) server and client over POSIX sockets for the control
// plane (master REST API, master<->harness and master<->agent WebSockets).
// Optional TLS (OpenSSL): HttpServer::EnableTls serves HTTPS/WSS; clients speak TLS to the
// endpoints registered with RegisterTlsEndpoint (the agent -> master link).  JSON bodies.  One thread per connection: the control plane carries tens of
// connections, not thousands.
#pragma once

#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

namespace detcore {
namespace net {

std::string Base64Encode(const std::string& in);
std::string Base64Decode(const std::string& in);
std::string Sha1(const std::string& in);  // 20 raw bytes
std::string UrlDecode(const std::string& s);
std::string UrlEncode(const std::string& s);

struct Request {
  std::string method;
  std::string path;                            // without query string
  std::map<std::string, std::string> query;    // decoded
  std::map<std::string, std::string> headers;  // lower-case keys
  std::map<std::string, std::string> params;   // route ":name" captures
  std::string body;
  std::string remote_addr;
  std::string Query(const std::string& k, const std::string& dflt = "") const {
    auto it = query.find(k);
    return it == query.end() ? dflt : it->second;
  }
  std::string Param(const std::string& k) const {
    auto it = params.find(k);
    return it == params.end() ? "" : it->second;
  }
};

struct Response {
  int status = 200;
  std::string content_type = "application/json";
  std::map<std::string, std::string> headers;
  std::string body;
  // Streaming body (grpc-gateway server streams): when set, the server sends the headers with
  // chunked transfer encoding and calls stream(write); each write(chunk) sends one chunk and
  // returns false once the client is gone or the server is stopping.
  using Writer = std::function<bool(const std::string&)>;
  std::function<void(const Writer&)> stream;
  static Response Json(int status, const std::string& body) {
    Response r;
    r.status = status;
    r.body = body;
    return r;
  }
  static Response Text(int status, const std::string& body) {
    Response r;
    r.status = status;
    r.content_type = "text/plain";
    r.body = body;
    return r;
  }
};

// A WebSocket connection (either side).  Send is thread-safe.
class WsConn : public std::enable_shared_from_this<WsConn> {
 public:
  WsConn(int fd, bool client_side, std::string peer, std::string initial = "");
  ~WsConn();
  bool Send(const std::string& text);
  bool SendBinary(const std::string& data);  // opcode 2 (byte streams: the TCP tunnel)
  void Close();
  bool closed() const { return closed_.load(); }
  const std::string& peer() const { return peer_; }
  // Blocking read loop: calls on_message for each text/binary message; returns on close/error.
  void ReadLoop(const std::function<void(const std::string&)>& on_message);
  // Blocking read of one message; false on close.
  bool Recv(std::string* out);

 private:
  bool SendFrame(int opcode, const std::string& payload);
  int fd_;
  bool client_;
  std::string peer_;
  std::mutex send_mu_;
  std::atomic<bool> closed_{false};
  std::string rbuf_;
};
using WsPtr = std::shared_ptr<WsConn>;

using Handler = std::function<Response(const Request&)>;
// Called on the connection's thread after the upgrade; should run ws->ReadLoop(...).
using WsHandler = std::function<void(const Request&, WsPtr ws)>;

class HttpServer {
 public:
  HttpServer() = default;
  ~HttpServer();
  // Pattern segments starting with ':' capture; a trailing "*" matches the rest.
  void Route(const std::string& method, const std::string& pattern, Handler h);
  // require_auth: the auth hook (SetAuth) also gates the upgrade (401 before switching protocols);
  // used for user-facing sockets (the TCP tunnel), not for agent / trial sockets.
  void RouteWs(const std::string& pattern, WsHandler h, bool require_auth = false);
  // Optional authorisation hook for plain HTTP routes (and auth-gated WebSocket routes): false -> 401.
  void SetAuth(std::function<bool(const Request&)> auth) { auth_ = std::move(auth); }
  // Serve every connection over TLS with this PEM certificate chain and key (call before Start).
  bool EnableTls(const std::string& cert_file, const std::string& key_file, std::string* error);
  bool tls() const { return tls_ctx_ != nullptr; }
  // Binds host:port (port 0 = ephemeral); returns the bound port.
  int Listen(const std::string& host, int port);
  void Start();  // accept loop on a background thread
  void Stop();
  // Route a request in-process (no auth hook, plain HTTP routes only): lets one API surface be
  // layered on another, e.g. /api/v1/* over the legacy REST handlers.
  Response Dispatch(Request req) const;
  bool running() const { return running_.load(); }
  int port() const { return port_; }

 private:
  struct RouteEntry {
    std::string method;
    std::vector<std::string> segs;
    Handler h;
    WsHandler ws;
    bool ws_auth = false;
  };
  bool Match(const RouteEntry& r, const std::vector<std::string>& segs, std::map<std::string, std::string>* params) const;
  const RouteEntry* Find(Request* req, bool want_ws, bool* path_hit) const;
  void Serve(int fd, std::string peer);
  std::vector<RouteEntry> routes_;
  std::function<bool(const Request&)> auth_;
  int listen_fd_ = -1;
  int port_ = 0;
  std::atomic<bool> running_{false};
  std::thread accept_thread_;
  std::mutex conns_mu_;
  std::condition_variable conns_cv_;
  std::vector<int> conn_fds_;
  int active_conns_ = 0;
  void* tls_ctx_ = nullptr;  // SSL_CTX*
};

// Client helpers.
struct ClientResponse {
  int status = 0;
  std::string body;
  std::string content_type;
  std::string error;  // non-empty on transport failure
};
ClientResponse HttpCall(const std::string& host, int port, const std::string& method, const std::string& path,
                        const std::string& body = "", int timeout_ms = 30000,
                        const std::string& content_type = "application/json");
WsPtr WsConnect(const std::string& host, int port, const std::string& path, std::string* error = nullptr);

int ConnectTcp(const std::string& host, int port, int timeout_ms, std::string* error);
// Client-side TLS for one endpoint: HttpCall / WsConnect to host:port then handshake TLS, verifying
// the server against ca_file (a PEM bundle; the master's self-signed cert works), and the name
// server_name when non-empty.
bool RegisterTlsEndpoint(const std::string& host, int port, const std::string& ca_file, const std::string& server_name,
                         std::string* error);
std::string LocalIPForPeer(const std::string& host, int port);

}  // namespace net
}  // namespace detcore
