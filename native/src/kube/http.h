// HTTP/1.1 client for the native node labeller: the handful of apiserver
// calls it makes (GET / PATCH / PUT a Node, a streamed watch), over TCP with
// OpenSSL TLS (CA verification, hostname or IP check) or plain HTTP (tests).
// One connection per request ("Connection: close"); a watch keeps its own.
#pragma once

#include <openssl/ssl.h>

#include <memory>
#include <string>
#include <utility>
#include <vector>

namespace mi355x::http {

struct Config {
  std::string server;   // https://host:port or http://host:port
  std::string ca_file;  // empty: system trust store (unless ca_pem)
  std::string ca_pem;   // CA bundle in memory (kubeconfig certificate-authority-data)
  // client certificate auth (kubeconfig users[].user): files or PEM in memory
  std::string cert_file, key_file, cert_pem, key_pem;
  bool insecure = false;
  std::string tls_server_name;  // kubeconfig tls-server-name: SNI and the name the certificate must carry
  // an HTTP proxy (kubeconfig proxy-url); else, with proxy_from_env, $HTTPS_PROXY / $HTTP_PROXY
  // and $NO_PROXY as Go's net/http reads them (never for localhost / loopback)
  std::string proxy_url;
  bool proxy_from_env = true;
  double timeout_s = 15.0;
};

struct Response {
  int status = 0;       // 0 = transport error (see error)
  std::string body;
  std::string error;
};

using Headers = std::vector<std::pair<std::string, std::string>>;

class Conn {
 public:
  Conn() = default;
  Conn(const Conn&) = delete;
  Conn& operator=(const Conn&) = delete;
  ~Conn();

  std::string open(const Config& cfg);  // "" on success
  bool write_all(const std::string& data);
  // >0 bytes read, 0 end of stream, -1 error, -2 timeout, -3 wake_fd readable
  long read_some(char* buf, size_t n, int timeout_ms, int wake_fd = -1);
  void close();
  const std::string& host() const { return host_; }
  const std::string& authority() const { return authority_; }  // host[:port] as the server URL writes it
  const std::string& prefix() const { return prefix_; }        // the server URL's path, below which requests go
  bool absolute_form() const { return absolute_form_; }        // through an HTTP proxy to an http:// server
  const std::string& proxy_auth() const { return proxy_auth_; }

 private:
  int fd_ = -1;
  SSL_CTX* ctx_ = nullptr;
  SSL* ssl_ = nullptr;
  std::string host_, authority_, prefix_, proxy_auth_;
  bool absolute_form_ = false;
};

// $NO_PROXY matching as Go's httpproxy does it: "*", IPs, CIDR blocks, host[:port],
// "foo.com" (itself and its subdomains), ".foo.com" / "*.foo.com" (subdomains only)
bool no_proxy_match(const std::string& no_proxy, const std::string& host, int port);
// the proxy URL the environment gives for a request to host:port ("" = direct)
std::string env_proxy(bool tls, const std::string& host, int port);

// A response body read incrementally (Content-Length, chunked, or to EOF).
class Body {
 public:
  // prefix: body bytes already received together with the response head
  Body(Conn* c, bool chunked, long long length, std::string prefix = "")
      : c_(c), chunked_(chunked), left_(chunked ? 0 : length), raw_(std::move(prefix)) {}
  // appends decoded bytes; same return codes as Conn::read_some (0 = body complete)
  long read(std::string* out, int timeout_ms, int wake_fd = -1);

 private:
  long fill(int timeout_ms, int wake_fd);
  Conn* c_;
  bool chunked_;
  long long left_;         // bytes left in the body (length mode) / in the chunk (chunked)
  std::string raw_;        // received, not yet decoded
  bool in_chunk_ = false;
  bool done_ = false;
};

struct Head {
  int status = 0;
  bool chunked = false;
  long long length = -1;   // -1: until EOF
};

// Sends one request and reads the status line + headers; raw_rest gets the bytes after them.
std::string start(Conn* c, const Config& cfg, const std::string& method, const std::string& path,
                  const Headers& headers, const std::string& body, Head* head, std::string* raw_rest,
                  int timeout_ms, int wake_fd = -1);

Response request(const Config& cfg, const std::string& method, const std::string& path, const Headers& headers,
                 const std::string& body = "", int wake_fd = -1);

// A body reader that first consumes bytes already received with the head.
class Stream {
 public:
  Stream() = default;
  std::string open(const Config& cfg, const std::string& path, const Headers& headers, int* status,
                   std::string* error_body, int timeout_ms, int wake_fd);
  // next newline-terminated line (without the newline). Return codes: 1 line, 0 end, -1 error,
  // -2 timeout, -3 woken
  int next_line(std::string* line, int timeout_ms, int wake_fd);
  void close() { conn_.close(); }

 private:
  Conn conn_;
  Head head_;
  std::unique_ptr<Body> body_;
  std::string buf_;
};

}  // namespace mi355x::http
