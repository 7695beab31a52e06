// HTTP/1.1 + WebSocket transport (see include/detcore/net.h).
#include "detcore/net.h"

#include <arpa/inet.h>
#include <fcntl.h>
#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <poll.h>
#include <sys/socket.h>
#include <sys/types.h>
#include <unistd.h>

#include <algorithm>
#include <cctype>
#include <cerrno>
#include <cstring>
#include <random>
#include <sstream>
#include <unordered_map>

#include <openssl/err.h>
#include <openssl/ssl.h>

namespace detcore {
namespace net {

// ------------------------------------------------------------------------------ encodings / sha1
static const char kB64[] = "ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789+/";

std::string Base64Encode(const std::string& in) {
  std::string out;
  out.reserve((in.size() + 2) / 3 * 4);
  size_t i = 0;
  const unsigned char* p = reinterpret_cast<const unsigned char*>(in.data());
  for (; i + 2 < in.size(); i += 3) {
    uint32_t v = (p[i] << 16) | (p[i + 1] << 8) | p[i + 2];
    out += kB64[(v >> 18) & 63];
    out += kB64[(v >> 12) & 63];
    out += kB64[(v >> 6) & 63];
    out += kB64[v & 63];
  }
  if (i + 1 == in.size()) {
    uint32_t v = p[i] << 16;
    out += kB64[(v >> 18) & 63];
    out += kB64[(v >> 12) & 63];
    out += "==";
  } else if (i + 2 == in.size()) {
    uint32_t v = (p[i] << 16) | (p[i + 1] << 8);
    out += kB64[(v >> 18) & 63];
    out += kB64[(v >> 12) & 63];
    out += kB64[(v >> 6) & 63];
    out += '=';
  }
  return out;
}

std::string Base64Decode(const std::string& in) {
  int T[256];
  std::fill(T, T + 256, -1);
  for (int i = 0; i < 64; ++i) T[static_cast<unsigned char>(kB64[i])] = i;
  T[static_cast<unsigned char>('-')] = 62;  // url-safe alphabet too
  T[static_cast<unsigned char>('_')] = 63;
  std::string out;
  uint32_t val = 0;
  int bits = -8;
  for (unsigned char c : in) {
    if (T[c] < 0) continue;
    val = (val << 6) | T[c];
    bits += 6;
    if (bits >= 0) {
      out.push_back(static_cast<char>((val >> bits) & 0xFF));
      bits -= 8;
    }
  }
  return out;
}

std::string Sha1(const std::string& msg) {
  uint32_t h0 = 0x67452301, h1 = 0xEFCDAB89, h2 = 0x98BADCFE, h3 = 0x10325476, h4 = 0xC3D2E1F0;
  std::string m = msg;
  uint64_t ml = static_cast<uint64_t>(msg.size()) * 8;
  m.push_back(static_cast<char>(0x80));
  while (m.size() % 64 != 56) m.push_back(0);
  for (int i = 7; i >= 0; --i) m.push_back(static_cast<char>((ml >> (8 * i)) & 0xFF));
  auto rol = [](uint32_t v, int s) { return (v << s) | (v >> (32 - s)); };
  for (size_t chunk = 0; chunk < m.size(); chunk += 64) {
    uint32_t w[80];
    for (int i = 0; i < 16; ++i) {
      const unsigned char* p = reinterpret_cast<const unsigned char*>(m.data() + chunk + 4 * i);
      w[i] = (p[0] << 24) | (p[1] << 16) | (p[2] << 8) | p[3];
    }
    for (int i = 16; i < 80; ++i) w[i] = rol(w[i - 3] ^ w[i - 8] ^ w[i - 14] ^ w[i - 16], 1);
    uint32_t a = h0, b = h1, c = h2, d = h3, e = h4;
    for (int i = 0; i < 80; ++i) {
      uint32_t f, k;
      if (i < 20) { f = (b & c) | (~b & d); k = 0x5A827999; }
      else if (i < 40) { f = b ^ c ^ d; k = 0x6ED9EBA1; }
      else if (i < 60) { f = (b & c) | (b & d) | (c & d); k = 0x8F1BBCDC; }
      else { f = b ^ c ^ d; k = 0xCA62C1D6; }
      uint32_t t = rol(a, 5) + f + e + k + w[i];
      e = d; d = c; c = rol(b, 30); b = a; a = t;
    }
    h0 += a; h1 += b; h2 += c; h3 += d; h4 += e;
  }
  std::string out;
  for (uint32_t h : {h0, h1, h2, h3, h4})
    for (int i = 3; i >= 0; --i) out.push_back(static_cast<char>((h >> (8 * i)) & 0xFF));
  return out;
}

std::string UrlDecode(const std::string& s) {
  std::string out;
  for (size_t i = 0; i < s.size(); ++i) {
    if (s[i] == '%' && i + 2 < s.size() && isxdigit(s[i + 1]) && isxdigit(s[i + 2])) {
      out.push_back(static_cast<char>(std::stoi(s.substr(i + 1, 2), nullptr, 16)));
      i += 2;
    } else if (s[i] == '+') {
      out.push_back(' ');
    } else {
      out.push_back(s[i]);
    }
  }
  return out;
}

// ---------------------------------------------------------------------------------------- TLS
// TLS (reference master security.tls, master/internal/config.go:118,249-260): OpenSSL on the same
// fd-based I/O.  A connection fd that carries TLS is registered here with its SSL object; the
// socket is switched to non-blocking and every SSL call runs under the connection's mutex (an
// SSL object must not be used from two threads at once, and a WebSocket is read on one thread
// while other threads send), waiting in poll() -- never inside the lock -- for WANT_READ /
// WANT_WRITE.  Plain fds take the old blocking send/recv paths untouched.
namespace {
// The SSL object lives as long as the last reference to its TlsConn: a thread that looked the
// connection up before another thread closed the fd (a WebSocket ReadLoop woken by the shutdown()
// of WsConn::Close) still holds a valid SSL*, and sees `closed` instead of a freed pointer.
struct TlsConn {
  SSL* ssl = nullptr;
  bool closed = false;
  std::mutex mu;
  int rcv_timeout_ms = -1;  // emulates SO_RCVTIMEO for client calls
  ~TlsConn() {
    if (ssl) SSL_free(ssl);
  }
};
std::mutex g_tls_mu;
std::unordered_map<int, std::shared_ptr<TlsConn>> g_tls;
struct TlsEndpoint {
  SSL_CTX* ctx = nullptr;
  std::string server_name;
};
std::mutex g_ep_mu;
std::map<std::string, TlsEndpoint> g_endpoints;  // "host:port" -> client context

std::shared_ptr<TlsConn> TlsOf(int fd) {
  std::lock_guard<std::mutex> g(g_tls_mu);
  auto it = g_tls.find(fd);
  return it == g_tls.end() ? nullptr : it->second;
}

std::string SslErrors() {
  std::string out;
  unsigned long e;
  char buf[256];
  while ((e = ERR_get_error()) != 0) {
    ERR_error_string_n(e, buf, sizeof(buf));
    if (!out.empty()) out += "; ";
    out += buf;
  }
  return out.empty() ? "tls error" : out;
}

// Run an SSL operation to completion on a non-blocking fd; >0 result, 0 = clean close, -1 = error
// or timeout.
template <typename F>
int TlsCall(TlsConn* t, int fd, F op, int timeout_ms) {
  for (;;) {
    int r, err;
    {
      std::lock_guard<std::mutex> g(t->mu);
      if (t->closed || !t->ssl) return -1;  // closed by another thread
      ERR_clear_error();
      r = op(t->ssl);
      if (r > 0) return r;
      err = SSL_get_error(t->ssl, r);
    }
    short ev;
    if (err == SSL_ERROR_WANT_READ) ev = POLLIN;
    else if (err == SSL_ERROR_WANT_WRITE) ev = POLLOUT;
    else if (err == SSL_ERROR_ZERO_RETURN) return 0;
    else return -1;
    pollfd p{fd, ev, 0};
    int pr = poll(&p, 1, timeout_ms < 0 ? 1000 : timeout_ms);
    if (pr < 0 && errno == EINTR) continue;
    if (pr == 0 && timeout_ms >= 0) return -1;
    if (pr > 0 && (p.revents & (POLLERR | POLLNVAL))) return -1;
  }
}

bool AttachTls(int fd, SSL_CTX* ctx, bool server, const std::string& server_name, int timeout_ms, std::string* error) {
  SSL* ssl = SSL_new(ctx);
  if (!ssl) {
    if (error) *error = SslErrors();
    return false;
  }
  SSL_set_fd(ssl, fd);
  if (!server && !server_name.empty()) {
    // SNI for names only; the certificate must match the name (or the literal IP) that was dialed
    in6_addr a6;
    in_addr a4;
    const bool is_ip = inet_pton(AF_INET, server_name.c_str(), &a4) == 1 || inet_pton(AF_INET6, server_name.c_str(), &a6) == 1;
    if (!is_ip) SSL_set_tlsext_host_name(ssl, server_name.c_str());
    X509_VERIFY_PARAM* vp = SSL_get0_param(ssl);
    if (is_ip) X509_VERIFY_PARAM_set1_ip_asc(vp, server_name.c_str());
    else SSL_set1_host(ssl, server_name.c_str());
  }
  fcntl(fd, F_SETFL, fcntl(fd, F_GETFL, 0) | O_NONBLOCK);
  auto t = std::make_shared<TlsConn>();
  t->ssl = ssl;
  int r = TlsCall(t.get(), fd, [server](SSL* s) { return server ? SSL_accept(s) : SSL_connect(s); }, timeout_ms);
  if (r <= 0) {
    if (error) *error = "tls handshake failed: " + SslErrors();
    return false;  // ~TlsConn frees the SSL
  }
  std::lock_guard<std::mutex> g(g_tls_mu);
  g_tls[fd] = t;
  return true;
}
}  // namespace

static void CloseFd(int fd) {
  std::shared_ptr<TlsConn> t;
  {
    std::lock_guard<std::mutex> g(g_tls_mu);
    auto it = g_tls.find(fd);
    if (it != g_tls.end()) {
      t = it->second;
      g_tls.erase(it);
    }
  }
  if (t) {
    std::lock_guard<std::mutex> g(t->mu);
    if (!t->closed && t->ssl) SSL_shutdown(t->ssl);  // best effort close_notify; non-blocking
    t->closed = true;  // the SSL itself is freed with the last TlsConn reference
  }
  ::close(fd);
}

bool RegisterTlsEndpoint(const std::string& host, int port, const std::string& ca_file, const std::string& server_name,
                         std::string* error) {
  SSL_CTX* ctx = SSL_CTX_new(TLS_client_method());
  if (!ctx) {
    if (error) *error = SslErrors();
    return false;
  }
  SSL_CTX_set_min_proto_version(ctx, TLS1_2_VERSION);
  if (!ca_file.empty()) {
    if (SSL_CTX_load_verify_locations(ctx, ca_file.c_str(), nullptr) != 1) {
      if (error) *error = "cannot load CA file " + ca_file + ": " + SslErrors();
      SSL_CTX_free(ctx);
      return false;
    }
    SSL_CTX_set_verify(ctx, SSL_VERIFY_PEER, nullptr);
  } else {
    SSL_CTX_set_default_verify_paths(ctx);
    SSL_CTX_set_verify(ctx, SSL_VERIFY_PEER, nullptr);
  }
  std::lock_guard<std::mutex> g(g_ep_mu);
  TlsEndpoint& ep = g_endpoints[(host == "localhost" ? "127.0.0.1" : host) + ":" + std::to_string(port)];
  if (ep.ctx) SSL_CTX_free(ep.ctx);
  ep.ctx = ctx;
  ep.server_name = server_name;
  return true;
}

static SSL_CTX* EndpointCtx(const std::string& host, int port, std::string* name) {
  std::lock_guard<std::mutex> g(g_ep_mu);
  auto it = g_endpoints.find((host == "localhost" ? "127.0.0.1" : host) + ":" + std::to_string(port));
  if (it == g_endpoints.end()) return nullptr;
  *name = it->second.server_name;
  return it->second.ctx;
}

// -------------------------------------------------------------------------------- socket utils
static bool WriteAll(int fd, const char* p, size_t n) {
  if (auto t = TlsOf(fd)) {
    while (n > 0) {
      const int chunk = static_cast<int>(std::min<size_t>(n, 1 << 20));
      int w = TlsCall(t.get(), fd, [p, chunk](SSL* s) { return SSL_write(s, p, chunk); }, 30000);
      if (w <= 0) return false;
      p += w;
      n -= static_cast<size_t>(w);
    }
    return true;
  }
  while (n > 0) {
    ssize_t w = ::send(fd, p, n, MSG_NOSIGNAL);
    if (w < 0) {
      if (errno == EINTR) continue;
      return false;
    }
    p += w;
    n -= static_cast<size_t>(w);
  }
  return true;
}

// one read of at most n bytes: >0 bytes, 0 EOF, <0 error (recv semantics)
static ssize_t RecvSome(int fd, char* buf, size_t n) {
  if (auto t = TlsOf(fd)) {
    const int want = static_cast<int>(std::min<size_t>(n, 1 << 20));
    int r = TlsCall(t.get(), fd, [buf, want](SSL* s) { return SSL_read(s, buf, want); }, t->rcv_timeout_ms);
    return r;
  }
  return ::recv(fd, buf, n, 0);
}

// Read into buf until it contains `delim`; returns false on EOF/error.
static bool ReadUntil(int fd, std::string& buf, const std::string& delim, size_t max_bytes = 1 << 20) {
  char tmp[8192];
  while (buf.find(delim) == std::string::npos) {
    if (buf.size() > max_bytes) return false;
    ssize_t r = RecvSome(fd, tmp, sizeof(tmp));
    if (r < 0 && errno == EINTR) continue;
    if (r <= 0) return false;
    buf.append(tmp, static_cast<size_t>(r));
  }
  return true;
}

static bool ReadN(int fd, std::string& buf, size_t n) {
  char tmp[65536];
  while (buf.size() < n) {
    size_t want = std::min(sizeof(tmp), n - buf.size());
    ssize_t r = RecvSome(fd, tmp, want);
    if (r < 0 && errno == EINTR) continue;
    if (r <= 0) return false;
    buf.append(tmp, static_cast<size_t>(r));
  }
  return true;
}

// Client connect: TCP, plus TLS when host:port was registered with RegisterTlsEndpoint.
static int ConnectMaybeTls(const std::string& host, int port, int timeout_ms, std::string* error) {
  int fd = ConnectTcp(host, port, timeout_ms, error);
  if (fd < 0) return fd;
  std::string name;
  if (SSL_CTX* ctx = EndpointCtx(host, port, &name)) {
    // the peer certificate is checked against --master-cert-name when given, else against the
    // host that was dialed (a chain-only check accepted any trusted certificate)
    if (!AttachTls(fd, ctx, false, name.empty() ? host : name, timeout_ms, error)) {
      ::close(fd);
      return -1;
    }
  }
  return fd;
}

static std::string Lower(std::string s) {
  for (auto& c : s) c = static_cast<char>(tolower(static_cast<unsigned char>(c)));
  return s;
}

static std::string Trim(const std::string& s) {
  size_t a = s.find_first_not_of(" \t\r\n"), b = s.find_last_not_of(" \t\r\n");
  return a == std::string::npos ? "" : s.substr(a, b - a + 1);
}

static std::vector<std::string> SplitPath(const std::string& p) {
  std::vector<std::string> out;
  std::string cur;
  for (char c : p) {
    if (c == '/') {
      if (!cur.empty()) out.push_back(cur);
      cur.clear();
    } else {
      cur.push_back(c);
    }
  }
  if (!cur.empty()) out.push_back(cur);
  return out;
}

static const char* StatusText(int s) {
  switch (s) {
    case 101: return "Switching Protocols";
    case 200: return "OK";
    case 201: return "Created";
    case 204: return "No Content";
    case 302: return "Found";
    case 403: return "Forbidden";
    case 400: return "Bad Request";
    case 401: return "Unauthorized";
    case 404: return "Not Found";
    case 405: return "Method Not Allowed";
    case 409: return "Conflict";
    case 502: return "Bad Gateway";
    case 504: return "Gateway Timeout";
    case 500: return "Internal Server Error";
    default: return "Status";
  }
}

int ConnectTcp(const std::string& host, int port, int timeout_ms, std::string* error) {
  addrinfo hints{};
  hints.ai_family = AF_INET;
  hints.ai_socktype = SOCK_STREAM;
  addrinfo* res = nullptr;
  std::string h = host == "localhost" ? "127.0.0.1" : host;
  if (getaddrinfo(h.c_str(), std::to_string(port).c_str(), &hints, &res) != 0 || !res) {
    if (error) *error = "resolve failed: " + host;
    return -1;
  }
  int fd = ::socket(res->ai_family, res->ai_socktype, res->ai_protocol);
  if (fd < 0) {
    freeaddrinfo(res);
    if (error) *error = "socket failed";
    return -1;
  }
  int fl = fcntl(fd, F_GETFL, 0);
  fcntl(fd, F_SETFL, fl | O_NONBLOCK);
  int rc = ::connect(fd, res->ai_addr, res->ai_addrlen);
  freeaddrinfo(res);
  if (rc < 0 && errno != EINPROGRESS) {
    ::close(fd);
    if (error) *error = std::string("connect failed: ") + strerror(errno);
    return -1;
  }
  if (rc < 0) {
    pollfd p{fd, POLLOUT, 0};
    if (poll(&p, 1, timeout_ms) <= 0) {
      ::close(fd);
      if (error) *error = "connect timeout";
      return -1;
    }
    int err = 0;
    socklen_t len = sizeof(err);
    getsockopt(fd, SOL_SOCKET, SO_ERROR, &err, &len);
    if (err != 0) {
      ::close(fd);
      if (error) *error = std::string("connect failed: ") + strerror(err);
      return -1;
    }
  }
  fcntl(fd, F_SETFL, fl);
  int one = 1;
  setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
  return fd;
}

std::string LocalIPForPeer(const std::string& host, int port) {
  std::string err;
  int fd = ConnectTcp(host, port, 2000, &err);
  if (fd < 0) return "127.0.0.1";
  sockaddr_in a{};
  socklen_t l = sizeof(a);
  getsockname(fd, reinterpret_cast<sockaddr*>(&a), &l);
  char buf[64];
  inet_ntop(AF_INET, &a.sin_addr, buf, sizeof(buf));
  ::close(fd);
  return buf;
}

// ------------------------------------------------------------------------------------- WsConn
WsConn::WsConn(int fd, bool client_side, std::string peer, std::string initial)
    : fd_(fd), client_(client_side), peer_(std::move(peer)), rbuf_(std::move(initial)) {}

WsConn::~WsConn() {
  Close();
}

bool WsConn::SendFrame(int opcode, const std::string& payload) {
  std::lock_guard<std::mutex> g(send_mu_);
  if (closed_.load()) return false;
  std::string hdr;
  hdr.push_back(static_cast<char>(0x80 | opcode));
  const uint8_t mask_bit = client_ ? 0x80 : 0;
  size_t n = payload.size();
  if (n < 126) {
    hdr.push_back(static_cast<char>(mask_bit | n));
  } else if (n < 65536) {
    hdr.push_back(static_cast<char>(mask_bit | 126));
    hdr.push_back(static_cast<char>((n >> 8) & 0xFF));
    hdr.push_back(static_cast<char>(n & 0xFF));
  } else {
    hdr.push_back(static_cast<char>(mask_bit | 127));
    for (int i = 7; i >= 0; --i) hdr.push_back(static_cast<char>((static_cast<uint64_t>(n) >> (8 * i)) & 0xFF));
  }
  if (client_) {
    static thread_local std::mt19937 rng{std::random_device{}()};
    uint32_t m = rng();
    char mk[4] = {static_cast<char>(m), static_cast<char>(m >> 8), static_cast<char>(m >> 16), static_cast<char>(m >> 24)};
    hdr.append(mk, 4);
    std::string masked = payload;
    for (size_t i = 0; i < masked.size(); ++i) masked[i] ^= mk[i & 3];
    return WriteAll(fd_, hdr.data(), hdr.size()) && WriteAll(fd_, masked.data(), masked.size());
  }
  return WriteAll(fd_, hdr.data(), hdr.size()) && WriteAll(fd_, payload.data(), payload.size());
}

bool WsConn::Send(const std::string& text) { return SendFrame(0x1, text); }
bool WsConn::SendBinary(const std::string& data) { return SendFrame(0x2, data); }

void WsConn::Close() {
  bool was = closed_.exchange(true);
  if (!was) {
    {
      std::lock_guard<std::mutex> g(send_mu_);
      std::string f;
      f.push_back(static_cast<char>(0x88));
      f.push_back(static_cast<char>(client_ ? 0x80 : 0));
      if (client_) f.append(4, '\0');
      WriteAll(fd_, f.data(), f.size());
    }
    ::shutdown(fd_, SHUT_RDWR);
    CloseFd(fd_);
  }
}

bool WsConn::Recv(std::string* out) {
  std::string message;
  for (;;) {
    if (!ReadN(fd_, rbuf_, 2)) return false;
    uint8_t b0 = static_cast<uint8_t>(rbuf_[0]), b1 = static_cast<uint8_t>(rbuf_[1]);
    bool fin = b0 & 0x80;
    int opcode = b0 & 0x0F;
    bool masked = b1 & 0x80;
    uint64_t len = b1 & 0x7F;
    size_t hl = 2;
    if (len == 126) {
      if (!ReadN(fd_, rbuf_, 4)) return false;
      len = (static_cast<uint8_t>(rbuf_[2]) << 8) | static_cast<uint8_t>(rbuf_[3]);
      hl = 4;
    } else if (len == 127) {
      if (!ReadN(fd_, rbuf_, 10)) return false;
      len = 0;
      for (int i = 0; i < 8; ++i) len = (len << 8) | static_cast<uint8_t>(rbuf_[2 + i]);
      hl = 10;
    }
    if (len > (1ull << 31)) return false;
    size_t ml = masked ? 4 : 0;
    if (!ReadN(fd_, rbuf_, hl + ml + len)) return false;
    std::string payload = rbuf_.substr(hl + ml, len);
    if (masked) {
      const char* mk = rbuf_.data() + hl;
      for (size_t i = 0; i < payload.size(); ++i) payload[i] ^= mk[i & 3];
    }
    rbuf_.erase(0, hl + ml + len);
    if (opcode == 0x8) {  // close
      Close();
      return false;
    }
    if (opcode == 0x9) {  // ping -> pong
      SendFrame(0xA, payload);
      continue;
    }
    if (opcode == 0xA) continue;
    message += payload;
    if (fin) {
      *out = std::move(message);
      return true;
    }
  }
}

void WsConn::ReadLoop(const std::function<void(const std::string&)>& on_message) {
  std::string m;
  while (!closed_.load() && Recv(&m)) on_message(m);
  Close();
}

// ---------------------------------------------------------------------------------- HttpServer
HttpServer::~HttpServer() { Stop(); }

void HttpServer::Route(const std::string& method, const std::string& pattern, Handler h) {
  routes_.push_back(RouteEntry{method, SplitPath(pattern), std::move(h), nullptr});
}

void HttpServer::RouteWs(const std::string& pattern, WsHandler h, bool require_auth) {
  routes_.push_back(RouteEntry{"GET", SplitPath(pattern), nullptr, std::move(h), require_auth});
}

bool HttpServer::Match(const RouteEntry& r, const std::vector<std::string>& segs,
                       std::map<std::string, std::string>* params) const {
  size_t i = 0;
  for (; i < r.segs.size(); ++i) {
    if (r.segs[i] == "*") {
      std::string rest;
      for (size_t j = i; j < segs.size(); ++j) rest += (j > i ? "/" : "") + segs[j];
      (*params)["*"] = rest;
      return true;
    }
    if (i >= segs.size()) return false;
    if (!r.segs[i].empty() && r.segs[i][0] == ':') (*params)[r.segs[i].substr(1)] = UrlDecode(segs[i]);
    else if (r.segs[i] != segs[i]) return false;
  }
  return i == segs.size();
}

int HttpServer::Listen(const std::string& host, int port) {
  listen_fd_ = ::socket(AF_INET, SOCK_STREAM, 0);
  int one = 1;
  setsockopt(listen_fd_, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
  sockaddr_in a{};
  a.sin_family = AF_INET;
  a.sin_port = htons(static_cast<uint16_t>(port));
  inet_pton(AF_INET, host.empty() ? "0.0.0.0" : host.c_str(), &a.sin_addr);
  if (::bind(listen_fd_, reinterpret_cast<sockaddr*>(&a), sizeof(a)) < 0) {
    ::close(listen_fd_);
    listen_fd_ = -1;
    return -1;
  }
  ::listen(listen_fd_, 128);
  socklen_t l = sizeof(a);
  getsockname(listen_fd_, reinterpret_cast<sockaddr*>(&a), &l);
  port_ = ntohs(a.sin_port);
  return port_;
}

void HttpServer::Start() {
  running_ = true;
  accept_thread_ = std::thread([this] {
    while (running_.load()) {
      pollfd p{listen_fd_, POLLIN, 0};
      int pr = poll(&p, 1, 200);
      if (pr <= 0) continue;
      sockaddr_in ca{};
      socklen_t cl = sizeof(ca);
      int fd = ::accept(listen_fd_, reinterpret_cast<sockaddr*>(&ca), &cl);
      if (fd < 0) continue;
      int one = 1;
      setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
      char buf[64];
      inet_ntop(AF_INET, &ca.sin_addr, buf, sizeof(buf));
      {
        std::lock_guard<std::mutex> g(conns_mu_);
        conn_fds_.push_back(fd);
        ++active_conns_;
      }
      std::thread([this, fd, peer = std::string(buf)] {
        Serve(fd, peer);
        std::lock_guard<std::mutex> g(conns_mu_);
        conn_fds_.erase(std::remove(conn_fds_.begin(), conn_fds_.end(), fd), conn_fds_.end());
        --active_conns_;
        conns_cv_.notify_all();
      }).detach();
    }
  });
}

void HttpServer::Stop() {
  if (!running_.exchange(false)) return;
  if (accept_thread_.joinable()) accept_thread_.join();
  if (listen_fd_ >= 0) ::close(listen_fd_);
  listen_fd_ = -1;
  std::unique_lock<std::mutex> l(conns_mu_);
  for (int fd : conn_fds_) ::shutdown(fd, SHUT_RDWR);
  conns_cv_.wait_for(l, std::chrono::seconds(5), [&] { return active_conns_ == 0; });
}

const HttpServer::RouteEntry* HttpServer::Find(Request* req, bool want_ws, bool* path_hit) const {
  auto segs = SplitPath(req->path);
  for (auto& r : routes_) {
    std::map<std::string, std::string> params;
    if (!Match(r, segs, &params)) continue;
    if ((r.ws != nullptr) != want_ws) continue;
    *path_hit = true;
    if (r.method != req->method) continue;
    req->params = std::move(params);
    return &r;
  }
  return nullptr;
}

Response HttpServer::Dispatch(Request req) const {
  bool path_hit = false;
  const RouteEntry* hit = Find(&req, false, &path_hit);
  if (!hit) return Response::Json(path_hit ? 405 : 404, R"({"error":"not found"})");
  return hit->h(req);
}

void HttpServer::Serve(int fd, std::string peer) {
  if (tls_ctx_) {
    std::string err;
    if (!AttachTls(fd, static_cast<SSL_CTX*>(tls_ctx_), true, "", 10000, &err)) {
      ::shutdown(fd, SHUT_RDWR);
      ::close(fd);
      return;
    }
  }
  std::string buf;
  for (;;) {
    if (!ReadUntil(fd, buf, "\r\n\r\n")) break;
    size_t he = buf.find("\r\n\r\n");
    std::string head = buf.substr(0, he);
    buf.erase(0, he + 4);
    Request req;
    req.remote_addr = peer;
    std::istringstream hs(head);
    std::string line;
    std::getline(hs, line);
    {
      std::istringstream ls(line);
      std::string target, ver;
      ls >> req.method >> target >> ver;
      auto q = target.find('?');
      req.path = UrlDecode(target.substr(0, q));
      if (q != std::string::npos) {
        std::string qs = target.substr(q + 1);
        size_t s = 0;
        while (s <= qs.size()) {
          size_t e = qs.find('&', s);
          if (e == std::string::npos) e = qs.size();
          std::string kv = qs.substr(s, e - s);
          auto eq = kv.find('=');
          if (!kv.empty()) req.query[UrlDecode(kv.substr(0, eq))] = eq == std::string::npos ? "" : UrlDecode(kv.substr(eq + 1));
          s = e + 1;
        }
      }
    }
    while (std::getline(hs, line)) {
      auto c = line.find(':');
      if (c == std::string::npos) continue;
      req.headers[Lower(Trim(line.substr(0, c)))] = Trim(line.substr(c + 1));
    }
    size_t cl = 0;
    if (req.headers.count("content-length")) cl = std::stoul(req.headers["content-length"]);
    if (cl > 0) {
      if (!ReadN(fd, buf, cl)) break;
      req.body = buf.substr(0, cl);
      buf.erase(0, cl);
    }
    bool path_hit = false;
    bool want_ws = Lower(req.headers["upgrade"]) == "websocket";
    const RouteEntry* hit = Find(&req, want_ws, &path_hit);
    if (hit && hit->ws && hit->ws_auth && auth_ && !auth_(req)) {
      const std::string body = R"({"error":"unauthenticated: log in with POST /login"})";
      std::string resp = "HTTP/1.1 401 Unauthorized\r\nContent-Type: application/json\r\nContent-Length: " +
                         std::to_string(body.size()) + "\r\nConnection: close\r\n\r\n" + body;
      WriteAll(fd, resp.data(), resp.size());
      break;
    }
    if (hit && hit->ws) {
      std::string key = req.headers["sec-websocket-key"];
      std::string accept = Base64Encode(Sha1(key + "258EAFA5-E914-47DA-95CA-C5AB0DC85B11"));
      std::string resp = "HTTP/1.1 101 Switching Protocols\r\nUpgrade: websocket\r\nConnection: Upgrade\r\n"
                         "Sec-WebSocket-Accept: " + accept + "\r\n\r\n";
      if (!WriteAll(fd, resp.data(), resp.size())) break;
      auto ws = std::make_shared<WsConn>(fd, false, peer, buf);
      hit->ws(req, ws);
      ws->Close();  // closes fd
      return;
    }
    Response res;
    if (!hit) {
      res = Response::Json(path_hit ? 405 : 404, R"({"error":"not found"})");
    } else if (auth_ && !auth_(req)) {
      res = Response::Json(401, R"({"error":"unauthenticated: log in with POST /login"})");
    } else {
      try {
        res = hit->h(req);
      } catch (const std::exception& e) {
        std::string msg = e.what();
        std::string esc;
        for (char ch : msg) {
          if (ch == '"' || ch == '\\') esc.push_back('\\');
          if (ch == '\n') { esc += "\\n"; continue; }
          esc.push_back(ch);
        }
        res = Response::Json(400, "{\"error\":\"" + esc + "\"}");
      }
    }
    bool close_after = Lower(req.headers["connection"]) == "close";
    if (res.stream) {
      std::ostringstream hs;
      hs << "HTTP/1.1 " << res.status << " " << StatusText(res.status) << "\r\n"
         << "Content-Type: " << res.content_type << "\r\n"
         << "Transfer-Encoding: chunked\r\n";
      for (auto& kv : res.headers) hs << kv.first << ": " << kv.second << "\r\n";
      hs << (close_after ? "Connection: close\r\n" : "Connection: keep-alive\r\n") << "\r\n";
      std::string h = hs.str();
      bool ok = WriteAll(fd, h.data(), h.size());
      if (ok) {
        res.stream([&](const std::string& chunk) {
          if (!ok || !running_.load()) return false;
          if (chunk.empty()) return true;  // an empty chunk would end the body
          char len[32];
          std::snprintf(len, sizeof(len), "%zx\r\n", chunk.size());
          std::string frame = std::string(len) + chunk + "\r\n";
          ok = WriteAll(fd, frame.data(), frame.size());
          return ok;
        });
        ok = ok && WriteAll(fd, "0\r\n\r\n", 5);
      }
      if (!ok || close_after) break;
      continue;
    }
    std::ostringstream os;
    os << "HTTP/1.1 " << res.status << " " << StatusText(res.status) << "\r\n"
       << "Content-Type: " << res.content_type << "\r\n"
       << "Content-Length: " << res.body.size() << "\r\n";
    for (auto& kv : res.headers) os << kv.first << ": " << kv.second << "\r\n";
    os << (close_after ? "Connection: close\r\n" : "Connection: keep-alive\r\n") << "\r\n";
    std::string out = os.str() + res.body;
    if (!WriteAll(fd, out.data(), out.size()) || close_after) break;
  }
  ::shutdown(fd, SHUT_RDWR);
  CloseFd(fd);
}

bool HttpServer::EnableTls(const std::string& cert_file, const std::string& key_file, std::string* error) {
  SSL_CTX* ctx = SSL_CTX_new(TLS_server_method());
  if (!ctx) {
    if (error) *error = SslErrors();
    return false;
  }
  SSL_CTX_set_min_proto_version(ctx, TLS1_2_VERSION);
  if (SSL_CTX_use_certificate_chain_file(ctx, cert_file.c_str()) != 1 ||
      SSL_CTX_use_PrivateKey_file(ctx, key_file.c_str(), SSL_FILETYPE_PEM) != 1 || SSL_CTX_check_private_key(ctx) != 1) {
    if (error) *error = "cannot load TLS cert/key: " + SslErrors();
    SSL_CTX_free(ctx);
    return false;
  }
  tls_ctx_ = ctx;
  return true;
}

// ------------------------------------------------------------------------------------- clients
std::string UrlEncode(const std::string& s) {
  static const char* hex = "0123456789ABCDEF";
  std::string out;
  for (unsigned char c : s) {
    if (std::isalnum(c) || c == '-' || c == '_' || c == '.' || c == '~') {
      out += static_cast<char>(c);
    } else {
      out += '%';
      out += hex[c >> 4];
      out += hex[c & 15];
    }
  }
  return out;
}

ClientResponse HttpCall(const std::string& host, int port, const std::string& method, const std::string& path,
                        const std::string& body, int timeout_ms, const std::string& content_type) {
  ClientResponse out;
  int fd = ConnectMaybeTls(host, port, timeout_ms, &out.error);
  if (fd < 0) return out;
  timeval tv{timeout_ms / 1000, (timeout_ms % 1000) * 1000};
  setsockopt(fd, SOL_SOCKET, SO_RCVTIMEO, &tv, sizeof(tv));
  if (auto t = TlsOf(fd)) t->rcv_timeout_ms = timeout_ms;
  std::ostringstream os;
  os << method << " " << path << " HTTP/1.1\r\nHost: " << host << ":" << port
     << "\r\nConnection: close\r\nContent-Type: " << content_type << "\r\nContent-Length: " << body.size() << "\r\n\r\n"
     << body;
  std::string req = os.str();
  if (!WriteAll(fd, req.data(), req.size())) {
    CloseFd(fd);
    out.error = "write failed";
    return out;
  }
  std::string buf;
  if (!ReadUntil(fd, buf, "\r\n\r\n")) {
    CloseFd(fd);
    out.error = "no response";
    return out;
  }
  size_t he = buf.find("\r\n\r\n");
  std::string head = buf.substr(0, he);
  buf.erase(0, he + 4);
  std::istringstream hs(head);
  std::string ver;
  hs >> ver >> out.status;
  size_t cl = std::string::npos;
  std::string line;
  while (std::getline(hs, line)) {
    auto c = line.find(':');
    if (c == std::string::npos) continue;
    const std::string key = Lower(Trim(line.substr(0, c)));
    if (key == "content-length") cl = std::stoul(Trim(line.substr(c + 1)));
    else if (key == "content-type") out.content_type = Trim(line.substr(c + 1));
  }
  if (cl != std::string::npos) ReadN(fd, buf, cl);
  else {
    char tmp[8192];
    ssize_t r;
    while ((r = RecvSome(fd, tmp, sizeof(tmp))) > 0) buf.append(tmp, static_cast<size_t>(r));
  }
  out.body = buf;
  CloseFd(fd);
  return out;
}

WsPtr WsConnect(const std::string& host, int port, const std::string& path, std::string* error) {
  int fd = ConnectMaybeTls(host, port, 10000, error);
  if (fd < 0) return nullptr;
  std::string key = Base64Encode(std::to_string(std::random_device{}()) + "detcore-ws-key!!");
  std::ostringstream os;
  os << "GET " << path << " HTTP/1.1\r\nHost: " << host << ":" << port
     << "\r\nUpgrade: websocket\r\nConnection: Upgrade\r\nSec-WebSocket-Version: 13\r\nSec-WebSocket-Key: " << key
     << "\r\n\r\n";
  std::string req = os.str();
  std::string buf;
  if (!WriteAll(fd, req.data(), req.size()) || !ReadUntil(fd, buf, "\r\n\r\n") || buf.find(" 101 ") == std::string::npos) {
    if (error) *error = "websocket upgrade failed: " + buf.substr(0, 64);
    CloseFd(fd);
    return nullptr;
  }
  size_t he = buf.find("\r\n\r\n");
  return std::make_shared<WsConn>(fd, true, host, buf.substr(he + 4));
}

}  // namespace net
}  // namespace detcore
