#include "http.h"

#include <openssl/err.h>
#include <openssl/pem.h>

#include <arpa/inet.h>
#include <fcntl.h>
#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <openssl/err.h>
#include <openssl/x509v3.h>
#include <poll.h>
#include <sys/socket.h>
#include <unistd.h>

#include <algorithm>
#include <cctype>
#include <cerrno>
#include <cstdlib>
#include <chrono>
#include <cstring>
#include <memory>

namespace mi355x::http {

namespace {

// scheme://host[:port][/prefix]: *authority gets "host[:port]" as written (the Host
// header, as Go's net/http sends it), *prefix the path without its trailing '/'
// (requests go below it, e.g. an apiserver behind a proxy at /k8s/clusters/c-1)
bool parse_url(const std::string& url, bool* tls, std::string* host, int* port, std::string* authority = nullptr,
               std::string* prefix = nullptr) {
  std::string rest;
  if (url.rfind("https://", 0) == 0) {
    *tls = true;
    rest = url.substr(8);
  } else if (url.rfind("http://", 0) == 0) {
    *tls = false;
    rest = url.substr(7);
  } else {
    return false;
  }
  const size_t slash = rest.find_first_of("/?#");
  std::string path;
  if (slash != std::string::npos) {
    path = rest.substr(slash);
    rest = rest.substr(0, slash);
  }
  if (path.find_first_of("?#") != std::string::npos) return false;  // a query or fragment is no API root
  while (!path.empty() && path.back() == '/') path.pop_back();
  if (authority) *authority = rest;
  if (prefix) *prefix = path;
  *port = *tls ? 443 : 80;
  if (!rest.empty() && rest[0] == '[') {  // [v6]:port
    const size_t close = rest.find(']');
    if (close == std::string::npos) return false;
    *host = rest.substr(1, close - 1);
    if (close + 1 < rest.size() && rest[close + 1] == ':') *port = std::atoi(rest.c_str() + close + 2);
  } else {
    const size_t colon = rest.rfind(':');
    *host = rest.substr(0, colon);
    if (colon != std::string::npos) *port = std::atoi(rest.c_str() + colon + 1);
  }
  return !host->empty() && *port > 0 && *port < 65536;
}

std::string ssl_error() {
  const unsigned long e = ERR_get_error();
  if (!e) return "TLS error";
  char b[256];
  ERR_error_string_n(e, b, sizeof(b));
  return b;
}

bool is_ip(const std::string& h) {
  in6_addr a6{};
  in_addr a4{};
  return inet_pton(AF_INET, h.c_str(), &a4) == 1 || inet_pton(AF_INET6, h.c_str(), &a6) == 1;
}

std::string lower(std::string s) {
  for (auto& c : s) c = static_cast<char>(std::tolower(static_cast<unsigned char>(c)));
  return s;
}

// TCP connection to host:port within tmo_ms (every resolved address tried); "" or an error
std::string connect_tcp(const std::string& host, int port, int tmo_ms, int* out) {
  addrinfo hints{};
  hints.ai_family = AF_UNSPEC;
  hints.ai_socktype = SOCK_STREAM;
  addrinfo* res = nullptr;
  const int gai = getaddrinfo(host.c_str(), std::to_string(port).c_str(), &hints, &res);
  if (gai != 0) return std::string("resolve ") + host + ": " + gai_strerror(gai);
  std::string err = "no address for " + host;
  for (addrinfo* a = res; a; a = a->ai_next) {
    const int fd = ::socket(a->ai_family, a->ai_socktype | SOCK_CLOEXEC | SOCK_NONBLOCK, a->ai_protocol);
    if (fd < 0) continue;
    int rc = ::connect(fd, a->ai_addr, a->ai_addrlen);
    if (rc != 0 && errno == EINPROGRESS) {
      pollfd p{fd, POLLOUT, 0};
      rc = ::poll(&p, 1, tmo_ms) == 1 ? 0 : -1;
      int so = 0;
      socklen_t sl = sizeof(so);
      if (rc == 0 && (getsockopt(fd, SOL_SOCKET, SO_ERROR, &so, &sl) != 0 || so != 0)) {
        errno = so ? so : errno;
        rc = -1;
      } else if (rc != 0) {
        errno = ETIMEDOUT;
      }
    }
    if (rc == 0) {
      ::fcntl(fd, F_SETFL, ::fcntl(fd, F_GETFL) & ~O_NONBLOCK);
      const int one = 1;
      setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
      *out = fd;
      freeaddrinfo(res);
      return "";
    }
    err = "connect " + host + ":" + std::to_string(port) + ": " + std::strerror(errno);
    ::close(fd);
  }
  freeaddrinfo(res);
  return err;
}

std::string b64(const std::string& in) {
  static const char* tbl = "ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789+/";
  std::string out;
  size_t i = 0;
  for (; i + 2 < in.size(); i += 3) {
    const uint32_t v = (uint8_t(in[i]) << 16) | (uint8_t(in[i + 1]) << 8) | uint8_t(in[i + 2]);
    for (int k = 18; k >= 0; k -= 6) out.push_back(tbl[(v >> k) & 63]);
  }
  if (i < in.size()) {
    const uint32_t v = (uint8_t(in[i]) << 16) | (i + 1 < in.size() ? uint8_t(in[i + 1]) << 8 : 0);
    out.push_back(tbl[(v >> 18) & 63]);
    out.push_back(tbl[(v >> 12) & 63]);
    out.push_back(i + 1 < in.size() ? tbl[(v >> 6) & 63] : '=');
    out.push_back('=');
  }
  return out;
}

std::string pct_decode(const std::string& s) {
  std::string out;
  for (size_t i = 0; i < s.size(); ++i) {
    if (s[i] == '%' && i + 2 < s.size() && std::isxdigit(static_cast<unsigned char>(s[i + 1])) &&
        std::isxdigit(static_cast<unsigned char>(s[i + 2]))) {
      out.push_back(static_cast<char>(std::stoi(s.substr(i + 1, 2), nullptr, 16)));
      i += 2;
    } else {
      out.push_back(s[i]);
    }
  }
  return out;
}

bool ip_in_cidr(const std::string& ip, const std::string& cidr) {
  const size_t slash = cidr.find('/');
  if (slash == std::string::npos) return false;
  const std::string net = cidr.substr(0, slash);
  char* end = nullptr;
  const long bits = std::strtol(cidr.c_str() + slash + 1, &end, 10);
  if (*end) return false;
  unsigned char a[16] = {}, b[16] = {};
  int len = 0;
  if (inet_pton(AF_INET, ip.c_str(), a) == 1 && inet_pton(AF_INET, net.c_str(), b) == 1) len = 4;
  else if (inet_pton(AF_INET6, ip.c_str(), a) == 1 && inet_pton(AF_INET6, net.c_str(), b) == 1) len = 16;
  if (!len || bits < 0 || bits > len * 8) return false;
  for (long k = 0; k < bits; ++k)
    if (((a[k / 8] ^ b[k / 8]) >> (7 - k % 8)) & 1) return false;
  return true;
}

}  // namespace

bool no_proxy_match(const std::string& no_proxy, const std::string& host_in, int port) {
  const std::string host = lower(host_in);
  size_t pos = 0;
  while (pos <= no_proxy.size()) {
    size_t c = no_proxy.find(',', pos);
    if (c == std::string::npos) c = no_proxy.size();
    std::string e = lower(no_proxy.substr(pos, c - pos));
    pos = c + 1;
    while (!e.empty() && std::isspace(static_cast<unsigned char>(e.front()))) e.erase(0, 1);
    while (!e.empty() && std::isspace(static_cast<unsigned char>(e.back()))) e.pop_back();
    if (e.empty()) continue;
    if (e == "*") return true;
    if (e.find('/') != std::string::npos) {  // a CIDR block
      if (is_ip(host) && ip_in_cidr(host, e)) return true;
      continue;
    }
    std::string h = e, p;  // host[:port], [v6]:port
    if (!e.empty() && e[0] == '[') {
      const size_t close = e.find(']');
      if (close == std::string::npos) continue;
      h = e.substr(1, close - 1);
      if (close + 1 < e.size() && e[close + 1] == ':') p = e.substr(close + 2);
    } else if (std::count(e.begin(), e.end(), ':') == 1) {
      h = e.substr(0, e.find(':'));
      p = e.substr(e.find(':') + 1);
    }
    if (h.empty()) continue;
    if (!p.empty() && p != std::to_string(port)) continue;
    if (is_ip(h)) {
      unsigned char x[16] = {}, y[16] = {};
      const int af = h.find(':') != std::string::npos ? AF_INET6 : AF_INET;
      if (inet_pton(af, h.c_str(), x) == 1 && inet_pton(af, host.c_str(), y) == 1 &&
          std::memcmp(x, y, af == AF_INET ? 4 : 16) == 0)
        return true;
      continue;
    }
    if (h.rfind("*.", 0) == 0) h.erase(0, 1);
    const bool exact_too = h[0] != '.';  // "foo.com" matches foo.com and its subdomains, ".foo.com" only these
    if (exact_too) h = "." + h;
    if ((host.size() > h.size() && host.compare(host.size() - h.size(), h.size(), h) == 0) ||
        (exact_too && host == h.substr(1)))
      return true;
  }
  return false;
}

std::string env_proxy(bool tls, const std::string& host, int port) {
  auto env = [](const char* a, const char* b) {
    const char* v = std::getenv(a);
    if (!v || !*v) v = std::getenv(b);
    return std::string(v ? v : "");
  };
  const std::string proxy = tls ? env("HTTPS_PROXY", "https_proxy") : env("HTTP_PROXY", "http_proxy");
  if (proxy.empty()) return "";
  // never for the local host (Go's httpproxy), nor what NO_PROXY names
  in6_addr a6{};
  in_addr a4{};
  if (lower(host) == "localhost" || (inet_pton(AF_INET, host.c_str(), &a4) == 1 && (ntohl(a4.s_addr) >> 24) == 127) ||
      (inet_pton(AF_INET6, host.c_str(), &a6) == 1 && IN6_IS_ADDR_LOOPBACK(&a6)))
    return "";
  if (no_proxy_match(env("NO_PROXY", "no_proxy"), host, port)) return "";
  return proxy.find("://") == std::string::npos ? "http://" + proxy : proxy;
}

Conn::~Conn() { close(); }

void Conn::close() {
  if (ssl_) {
    SSL_free(ssl_);
    ssl_ = nullptr;
  }
  if (ctx_) {
    SSL_CTX_free(ctx_);
    ctx_ = nullptr;
  }
  if (fd_ >= 0) {
    ::close(fd_);
    fd_ = -1;
  }
}

std::string Conn::open(const Config& cfg) {
  close();
  bool tls = false;
  int port = 0;
  if (!parse_url(cfg.server, &tls, &host_, &port, &authority_, &prefix_)) return "bad server URL " + cfg.server;
  const int tmo_ms = static_cast<int>(cfg.timeout_s * 1000);
  absolute_form_ = false;
  proxy_auth_.clear();
  const std::string proxy = !cfg.proxy_url.empty() ? cfg.proxy_url : cfg.proxy_from_env ? env_proxy(tls, host_, port) : "";
  if (proxy.empty()) {
    std::string err = connect_tcp(host_, port, tmo_ms, &fd_);
    if (!err.empty()) return err;
  } else {
    // an HTTP proxy (kubeconfig proxy-url, else $HTTPS_PROXY / $HTTP_PROXY as Go reads them):
    // CONNECT for an https server, absolute-form requests for an http one
    bool ptls = false;
    int pport = 0;
    std::string phost, pauth_url;
    std::string purl = proxy;
    const size_t at = purl.find('@'), scheme = purl.find("://");
    if (at != std::string::npos && scheme != std::string::npos && at > scheme) {
      pauth_url = pct_decode(purl.substr(scheme + 3, at - scheme - 3));
      purl.erase(scheme + 3, at - scheme - 2);
    }
    if (purl.rfind("http://", 0) != 0) return "proxy " + purl + ": only http:// proxies are supported";
    if (!parse_url(purl, &ptls, &phost, &pport)) return "bad proxy URL " + purl;
    if (!pauth_url.empty()) proxy_auth_ = "Basic " + b64(pauth_url);
    std::string err = connect_tcp(phost, pport, tmo_ms, &fd_);
    if (!err.empty()) return "proxy " + err;
    if (!tls) {
      absolute_form_ = true;
    } else {
      const std::string target = (host_.find(':') != std::string::npos ? "[" + host_ + "]" : host_) + ":" +
                                 std::to_string(port);
      std::string req = "CONNECT " + target + " HTTP/1.1\r\nHost: " + target + "\r\n";
      if (!proxy_auth_.empty()) req += "Proxy-Authorization: " + proxy_auth_ + "\r\n";
      req += "\r\n";
      if (!write_all(req)) return "proxy CONNECT: send failed";
      std::string head;  // byte by byte: what follows the head is the server's TLS
      while (head.size() < 8192 && head.find("\r\n\r\n") == std::string::npos) {
        char ch;
        const long n = read_some(&ch, 1, tmo_ms);
        if (n <= 0) return "proxy CONNECT: no answer";
        head.push_back(ch);
      }
      const size_t sp = head.find(' ');
      if (head.rfind("HTTP/1.", 0) != 0 || sp == std::string::npos || std::atoi(head.c_str() + sp + 1) != 200)
        return "proxy CONNECT " + target + ": " + head.substr(0, head.find("\r\n"));
    }
  }
  // a blocking read never outlives the request deadline (TLS records can arrive in pieces)
  timeval tv{static_cast<time_t>(cfg.timeout_s), static_cast<suseconds_t>((cfg.timeout_s - static_cast<long>(cfg.timeout_s)) * 1e6)};
  setsockopt(fd_, SOL_SOCKET, SO_RCVTIMEO, &tv, sizeof(tv));
  setsockopt(fd_, SOL_SOCKET, SO_SNDTIMEO, &tv, sizeof(tv));
  if (!tls) return "";
  ctx_ = SSL_CTX_new(TLS_client_method());
  if (!ctx_) return ssl_error();
  SSL_CTX_set_min_proto_version(ctx_, TLS1_2_VERSION);
  if (!cfg.insecure) {
    SSL_CTX_set_verify(ctx_, SSL_VERIFY_PEER, nullptr);
    if (!cfg.ca_pem.empty()) {
      X509_STORE* store = SSL_CTX_get_cert_store(ctx_);
      BIO* bio = BIO_new_mem_buf(cfg.ca_pem.data(), static_cast<int>(cfg.ca_pem.size()));
      int n = 0;
      while (X509* x = PEM_read_bio_X509(bio, nullptr, nullptr, nullptr)) {
        X509_STORE_add_cert(store, x);
        X509_free(x);
        ++n;
      }
      BIO_free(bio);
      ERR_clear_error();
      if (n == 0) return "CA data: no PEM certificate";
    } else {
      const int ok = cfg.ca_file.empty() ? SSL_CTX_set_default_verify_paths(ctx_)
                                         : SSL_CTX_load_verify_locations(ctx_, cfg.ca_file.c_str(), nullptr);
      if (ok != 1) return "CA " + cfg.ca_file + ": " + ssl_error();
    }
  }
  // client certificate (kubeconfig client-certificate / -data, client-key / -data)
  if (!cfg.cert_file.empty() || !cfg.cert_pem.empty()) {
    bool ok;
    if (!cfg.cert_pem.empty()) {
      BIO* bio = BIO_new_mem_buf(cfg.cert_pem.data(), static_cast<int>(cfg.cert_pem.size()));
      X509* x = PEM_read_bio_X509(bio, nullptr, nullptr, nullptr);
      ok = x && SSL_CTX_use_certificate(ctx_, x) == 1;
      while (ok) {  // the rest of the chain
        X509* extra = PEM_read_bio_X509(bio, nullptr, nullptr, nullptr);
        if (!extra) break;
        if (SSL_CTX_add_extra_chain_cert(ctx_, extra) != 1) X509_free(extra);
      }
      ERR_clear_error();
      if (x) X509_free(x);
      BIO_free(bio);
    } else {
      ok = SSL_CTX_use_certificate_chain_file(ctx_, cfg.cert_file.c_str()) == 1;
    }
    if (!ok) return "client certificate: " + ssl_error();
    if (!cfg.key_pem.empty()) {
      BIO* bio = BIO_new_mem_buf(cfg.key_pem.data(), static_cast<int>(cfg.key_pem.size()));
      EVP_PKEY* k = PEM_read_bio_PrivateKey(bio, nullptr, nullptr, nullptr);
      ok = k && SSL_CTX_use_PrivateKey(ctx_, k) == 1;
      if (k) EVP_PKEY_free(k);
      BIO_free(bio);
    } else {
      ok = !cfg.key_file.empty() && SSL_CTX_use_PrivateKey_file(ctx_, cfg.key_file.c_str(), SSL_FILETYPE_PEM) == 1;
    }
    if (!ok || SSL_CTX_check_private_key(ctx_) != 1) return "client key: " + ssl_error();
  }
  ssl_ = SSL_new(ctx_);
  if (!ssl_) return ssl_error();
  const std::string& name = cfg.tls_server_name.empty() ? host_ : cfg.tls_server_name;
  if (is_ip(name)) {
    X509_VERIFY_PARAM_set1_ip_asc(SSL_get0_param(ssl_), name.c_str());
  } else {
    SSL_set_tlsext_host_name(ssl_, name.c_str());
    SSL_set1_host(ssl_, name.c_str());
  }
  SSL_set_fd(ssl_, fd_);
  if (SSL_connect(ssl_) != 1) {
    const long vr = SSL_get_verify_result(ssl_);
    std::string e = vr != X509_V_OK ? std::string("certificate verify failed: ") + X509_verify_cert_error_string(vr)
                                    : ssl_error();
    close();
    return "TLS handshake with " + cfg.server + ": " + e;
  }
  return "";
}

bool Conn::write_all(const std::string& data) {
  size_t off = 0;
  while (off < data.size()) {
    long n;
    if (ssl_) {
      n = SSL_write(ssl_, data.data() + off, static_cast<int>(data.size() - off));
    } else {
      n = ::send(fd_, data.data() + off, data.size() - off, MSG_NOSIGNAL);
      if (n < 0 && errno == EINTR) continue;
    }
    if (n <= 0) return false;
    off += static_cast<size_t>(n);
  }
  return true;
}

long Conn::read_some(char* buf, size_t n, int timeout_ms, int wake_fd) {
  if (fd_ < 0) return -1;
  if (!(ssl_ && SSL_pending(ssl_) > 0)) {
    pollfd p[2] = {{fd_, POLLIN, 0}, {wake_fd, POLLIN, 0}};
    int r;
    do {
      r = ::poll(p, wake_fd >= 0 ? 2 : 1, timeout_ms);
    } while (r < 0 && errno == EINTR && wake_fd < 0);
    if (r < 0) return wake_fd >= 0 ? -3 : -1;
    if (r == 0) return -2;
    if (wake_fd >= 0 && (p[1].revents & POLLIN)) return -3;
  }
  if (ssl_) {
    const int k = SSL_read(ssl_, buf, static_cast<int>(n));
    if (k > 0) return k;
    const int e = SSL_get_error(ssl_, k);
    if (e == SSL_ERROR_ZERO_RETURN) return 0;
    if (e == SSL_ERROR_SYSCALL && ERR_peek_error() == 0) return 0;  // peer closed without close_notify
    return -1;
  }
  long k;
  do {
    k = ::recv(fd_, buf, n, 0);
  } while (k < 0 && errno == EINTR);
  return k < 0 ? -1 : k;
}

long Body::fill(int timeout_ms, int wake_fd) {
  char b[16384];
  const long n = c_->read_some(b, sizeof(b), timeout_ms, wake_fd);
  if (n > 0) raw_.append(b, static_cast<size_t>(n));
  return n;
}

long Body::read(std::string* out, int timeout_ms, int wake_fd) {
  for (;;) {
    if (done_) return 0;
    if (!chunked_) {
      if (left_ == 0) {
        done_ = true;
        return 0;
      }
      if (!raw_.empty()) {
        size_t take = raw_.size();
        if (left_ > 0 && static_cast<long long>(take) > left_) take = static_cast<size_t>(left_);
        out->append(raw_, 0, take);
        raw_.erase(0, take);
        if (left_ > 0) left_ -= static_cast<long long>(take);
        return static_cast<long>(take);
      }
      const long n = fill(timeout_ms, wake_fd);
      if (n == 0) {
        done_ = true;
        return left_ > 0 ? -1 : 0;  // EOF before Content-Length is a truncated body
      }
      if (n < 0) return n;
      continue;
    }
    if (!in_chunk_) {
      const size_t eol = raw_.find("\r\n");
      if (eol == std::string::npos) {
        if (raw_.size() > 4096) return -1;
        const long n = fill(timeout_ms, wake_fd);
        if (n <= 0) return n == 0 ? -1 : n;
        continue;
      }
      char* end = nullptr;
      const long long sz = std::strtoll(raw_.c_str(), &end, 16);
      if (end == raw_.c_str() || sz < 0) return -1;
      raw_.erase(0, eol + 2);
      if (sz == 0) {
        done_ = true;  // trailers, if any, are ignored (Connection: close)
        return 0;
      }
      left_ = sz;
      in_chunk_ = true;
    }
    if (left_ > 0 && !raw_.empty()) {
      size_t take = raw_.size();
      if (static_cast<long long>(take) > left_) take = static_cast<size_t>(left_);
      out->append(raw_, 0, take);
      raw_.erase(0, take);
      left_ -= static_cast<long long>(take);
      return static_cast<long>(take);
    }
    if (left_ == 0) {  // chunk data done: its CRLF
      if (raw_.size() < 2) {
        const long n = fill(timeout_ms, wake_fd);
        if (n <= 0) return n == 0 ? -1 : n;
        continue;
      }
      if (raw_.compare(0, 2, "\r\n") != 0) return -1;
      raw_.erase(0, 2);
      in_chunk_ = false;
      continue;
    }
    const long n = fill(timeout_ms, wake_fd);
    if (n <= 0) return n == 0 ? -1 : n;
  }
}

std::string start(Conn* c, const Config& cfg, const std::string& method, const std::string& path,
                  const Headers& headers, const std::string& body, Head* head, std::string* raw_rest,
                  int timeout_ms, int wake_fd) {
  std::string err = c->open(cfg);
  if (!err.empty()) return err;
  const std::string target = (c->absolute_form() ? "http://" + c->authority() : "") + c->prefix() + path;
  std::string req = method + " " + target + " HTTP/1.1\r\nHost: " + c->authority() + "\r\nConnection: close\r\n";
  if (c->absolute_form() && !c->proxy_auth().empty()) req += "Proxy-Authorization: " + c->proxy_auth() + "\r\n";
  for (const auto& [k, v] : headers) req += k + ": " + v + "\r\n";
  if (!body.empty() || method == "PATCH" || method == "PUT" || method == "POST")
    req += "Content-Length: " + std::to_string(body.size()) + "\r\n";
  req += "\r\n" + body;
  if (!c->write_all(req)) return "send failed";
  std::string raw;
  size_t hend;
  const auto deadline = std::chrono::steady_clock::now() + std::chrono::milliseconds(timeout_ms);
  while ((hend = raw.find("\r\n\r\n")) == std::string::npos) {
    if (raw.size() > 65536) return "response head too large";
    const int left = static_cast<int>(
        std::chrono::duration_cast<std::chrono::milliseconds>(deadline - std::chrono::steady_clock::now()).count());
    if (left <= 0) return "timed out waiting for the response";
    char b[4096];
    const long n = c->read_some(b, sizeof(b), left, wake_fd);
    if (n == -3) return "interrupted";
    if (n == -2) return "timed out waiting for the response";
    if (n <= 0) return "connection closed before the response";
    raw.append(b, static_cast<size_t>(n));
  }
  const std::string h = raw.substr(0, hend);
  *raw_rest = raw.substr(hend + 4);
  // "HTTP/1.1 200 OK"
  const size_t sp = h.find(' ');
  if (h.rfind("HTTP/1.", 0) != 0 || sp == std::string::npos) return "bad status line";
  head->status = std::atoi(h.c_str() + sp + 1);
  size_t pos = h.find("\r\n");
  while (pos != std::string::npos) {
    const size_t next = h.find("\r\n", pos + 2);
    const std::string line = h.substr(pos + 2, next == std::string::npos ? std::string::npos : next - pos - 2);
    const size_t colon = line.find(':');
    if (colon != std::string::npos) {
      const std::string k = lower(line.substr(0, colon));
      std::string v = line.substr(colon + 1);
      while (!v.empty() && (v[0] == ' ' || v[0] == '\t')) v.erase(0, 1);
      if (k == "transfer-encoding" && lower(v).find("chunked") != std::string::npos) head->chunked = true;
      if (k == "content-length") head->length = std::atoll(v.c_str());
    }
    pos = next;
  }
  if (head->chunked) head->length = -1;
  return "";
}

Response request(const Config& cfg, const std::string& method, const std::string& path, const Headers& headers,
                 const std::string& body, int wake_fd) {
  Response r;
  Conn c;
  Head h;
  std::string rest;
  const int tmo = static_cast<int>(cfg.timeout_s * 1000);
  r.error = start(&c, cfg, method, path, headers, body, &h, &rest, tmo, wake_fd);
  if (!r.error.empty()) return r;
  Body b(&c, h.chunked, h.length, std::move(rest));
  const auto deadline = std::chrono::steady_clock::now() + std::chrono::milliseconds(tmo);
  for (;;) {
    const int left = static_cast<int>(
        std::chrono::duration_cast<std::chrono::milliseconds>(deadline - std::chrono::steady_clock::now()).count());
    if (left <= 0) {
      r.error = "timed out reading the response body";
      return r;
    }
    if (r.body.size() > (64u << 20)) {
      r.error = "response body too large";
      return r;
    }
    const long n = b.read(&r.body, left, wake_fd);
    if (n == 0) break;
    if (n < 0) {
      r.error = n == -2 ? "timed out reading the response body" : n == -3 ? "interrupted" : "truncated response body";
      return r;
    }
  }
  r.status = h.status;
  return r;
}

std::string Stream::open(const Config& cfg, const std::string& path, const Headers& headers, int* status,
                         std::string* error_body, int timeout_ms, int wake_fd) {
  buf_.clear();
  body_.reset();
  std::string rest;
  head_ = Head{};
  std::string err = start(&conn_, cfg, "GET", path, headers, "", &head_, &rest, timeout_ms, wake_fd);
  if (!err.empty()) return err;
  *status = head_.status;
  body_ = std::make_unique<Body>(&conn_, head_.chunked, head_.length, std::move(rest));
  if (head_.status != 200) {  // the error Status object, for the caller's message
    while (error_body->size() < 4096 && body_->read(error_body, timeout_ms, wake_fd) > 0) {
    }
  }
  return "";
}

int Stream::next_line(std::string* line, int timeout_ms, int wake_fd) {
  for (;;) {
    const size_t nl = buf_.find('\n');
    if (nl != std::string::npos) {
      *line = buf_.substr(0, nl);
      buf_.erase(0, nl + 1);
      return 1;
    }
    if (!body_) return -1;
    if (buf_.size() > (16u << 20)) return -1;  // one event larger than any Node
    const long n = body_->read(&buf_, timeout_ms, wake_fd);
    if (n == 0) {
      if (buf_.empty()) return 0;
      *line = std::move(buf_);  // last event without a trailing newline
      buf_.clear();
      return 1;
    }
    if (n < 0) return static_cast<int>(n);
  }
}

}  // namespace mi355x::http
