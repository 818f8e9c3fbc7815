// Minimal HTTP/1.1 client for the Kubernetes REST API: one keep-alive TCP
// connection (optionally TLS through OpenSSL), Content-Length and chunked
// bodies, and a line reader over a streaming (watch) response.
//
// The scheduler's service mode (control/remote.py) used Python's http.client
// for every binding and a Python informer per watched kind; with this client
// the bindings, patches and the LIST/WATCH mirror run on native threads with
// no interpreter lock on the path (rest/kube.h).
#pragma once

#include <sys/types.h>

#include <cstdint>
#include <memory>
#include <string>
#include <string_view>
#include <vector>

namespace xsched::rest {

// client-go rest.TLSClientConfig: cluster CA (file or PEM), optional client
// certificate and key (file or PEM), insecure-skip-tls-verify.
struct TlsOptions {
  bool enabled = false;
  std::string ca_file, ca_pem;
  std::string cert_file, key_file, cert_pem, key_pem;
  bool insecure = false;
};

struct Endpoint {
  std::string host = "127.0.0.1";
  int port = 80;
  std::string token;  // bearer token ("" = none)
  TlsOptions tls;
  int timeout_ms = 30'000;  // connect and per-request I/O (not watch streams)
  // client-go's token bucket (KubeSchedulerConfiguration clientConnection):
  // at most `qps` requests per second with bursts of `burst`; 0 = unlimited.
  double qps = 0;
  int burst = 0;
};

struct Response {
  int status = 0;
  std::string body;
};

class TlsContext;  // shared OpenSSL context (rest/http.cc)

class HttpConn {
 public:
  // Connects (and handshakes); throws std::runtime_error on failure.
  HttpConn(const Endpoint& ep, std::shared_ptr<TlsContext> tls, bool streaming = false);
  ~HttpConn();
  HttpConn(const HttpConn&) = delete;
  HttpConn& operator=(const HttpConn&) = delete;

  // One request and its full response. Throws std::runtime_error on I/O
  // errors (the connection is then unusable).
  Response roundtrip(std::string_view method, std::string_view path, std::string_view body = {},
                     std::string_view content_type = "application/json");
  // Streaming GET: sends the request and reads the status line and headers;
  // the body is then read line by line with next_line().
  int open_stream(std::string_view path);
  // Next newline-terminated line of the stream body (without the newline);
  // false at the end of the stream or on an error.
  bool next_line(std::string& line);
  // The server asked to close, or an error happened: do not reuse.
  bool reusable() const { return reusable_; }
  // The last roundtrip failed the way a keep-alive connection the server
  // closed while idle fails: EOF or a reset before any response byte, never
  // a receive timeout. Only then may a pooled request be sent again.
  bool failed_stale() const { return (fail_ == Fail::kEof || fail_ == Fail::kReset) && rx_bytes_ == 0; }
  // Unblocks a reader blocked in next_line() (from another thread).
  void shutdown();

 private:
  void send_request(std::string_view method, std::string_view path, std::string_view body,
                    std::string_view content_type);
  int read_head(bool* chunked, int64_t* content_length);
  bool fill();  // reads more bytes into buf_; false on EOF/error
  bool read_line_raw(std::string& out);  // one CRLF/LF-terminated line of the raw stream
  bool read_exact(size_t n, std::string& out);
  bool read_chunked_body(std::string& out);
  bool next_chunk();  // streaming: loads the next chunk's bytes into pending_

  Endpoint ep_;
  std::shared_ptr<TlsContext> tls_;
  int fd_ = -1;
  void* ssl_ = nullptr;  // SSL*
  std::string buf_;      // received, not yet consumed
  size_t pos_ = 0;
  bool reusable_ = true;
  enum class Fail { kNone, kEof, kReset, kTimeout, kOther };
  Fail fail_ = Fail::kNone;
  size_t rx_bytes_ = 0;  // bytes received since the current request was sent
  void note_io_failure(ssize_t n);
  // streaming state
  bool stream_chunked_ = false;
  int64_t stream_left_ = -1;  // Content-Length stream: bytes left (-1: until close)
  std::string pending_;       // decoded body bytes not yet returned as lines
};

// Shared TLS configuration (one SSL_CTX per endpoint).
std::shared_ptr<TlsContext> make_tls_context(const TlsOptions& o);

// Percent-encodes one URL path segment.
std::string url_segment(std::string_view s);

}  // namespace xsched::rest
