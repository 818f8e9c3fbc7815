#include "rest/http.h"

#include <arpa/inet.h>
#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <openssl/err.h>
#include <openssl/pem.h>
#include <openssl/ssl.h>
#include <openssl/x509v3.h>
#include <sys/socket.h>
#include <sys/time.h>
#include <unistd.h>

#include <cctype>
#include <cerrno>
#include <cstring>
#include <stdexcept>

namespace xsched::rest {

namespace {

constexpr int kWatchRecvTimeoutS = 330;  // > the watches' timeoutSeconds=300

std::string ssl_error(const std::string& what) {
  unsigned long e = ERR_get_error();
  char buf[256];
  ERR_error_string_n(e, buf, sizeof(buf));
  return what + ": " + buf;
}

bool is_ip_literal(const std::string& h) {
  in6_addr a6;
  in_addr a4;
  return inet_pton(AF_INET, h.c_str(), &a4) == 1 || inet_pton(AF_INET6, h.c_str(), &a6) == 1;
}

bool ieq(std::string_view a, std::string_view b) {
  if (a.size() != b.size()) return false;
  for (size_t i = 0; i < a.size(); ++i)
    if (std::tolower(static_cast<unsigned char>(a[i])) != std::tolower(static_cast<unsigned char>(b[i]))) return false;
  return true;
}

std::string_view trim(std::string_view s) {
  while (!s.empty() && (s.front() == ' ' || s.front() == '\t')) s.remove_prefix(1);
  while (!s.empty() && (s.back() == ' ' || s.back() == '\t' || s.back() == '\r')) s.remove_suffix(1);
  return s;
}

}  // namespace

class TlsContext {
 public:
  explicit TlsContext(const TlsOptions& o) : insecure(o.insecure) {
    ctx = SSL_CTX_new(TLS_client_method());
    if (!ctx) throw std::runtime_error(ssl_error("SSL_CTX_new"));
    SSL_CTX_set_min_proto_version(ctx, TLS1_2_VERSION);
    if (!o.ca_file.empty()) {
      if (SSL_CTX_load_verify_locations(ctx, o.ca_file.c_str(), nullptr) != 1)
        throw std::runtime_error(ssl_error("loading CA file"));
    } else if (!o.ca_pem.empty()) {
      BIO* bio = BIO_new_mem_buf(o.ca_pem.data(), static_cast<int>(o.ca_pem.size()));
      X509_STORE* store = SSL_CTX_get_cert_store(ctx);
      int n = 0;
      while (X509* x = PEM_read_bio_X509(bio, nullptr, nullptr, nullptr)) {
        X509_STORE_add_cert(store, x);
        X509_free(x);
        ++n;
      }
      BIO_free(bio);
      ERR_clear_error();  // the loop ends on a PEM "no start line"
      if (n == 0) throw std::runtime_error("CA data holds no certificate");
    } else {
      SSL_CTX_set_default_verify_paths(ctx);
    }
    if (!o.cert_file.empty()) {
      if (SSL_CTX_use_certificate_chain_file(ctx, o.cert_file.c_str()) != 1 ||
          SSL_CTX_use_PrivateKey_file(ctx, (o.key_file.empty() ? o.cert_file : o.key_file).c_str(), SSL_FILETYPE_PEM) != 1)
        throw std::runtime_error(ssl_error("loading client certificate"));
    } else if (!o.cert_pem.empty()) {
      BIO* cb = BIO_new_mem_buf(o.cert_pem.data(), static_cast<int>(o.cert_pem.size()));
      X509* cert = PEM_read_bio_X509(cb, nullptr, nullptr, nullptr);
      BIO_free(cb);
      const std::string& kp = o.key_pem.empty() ? o.cert_pem : o.key_pem;
      BIO* kb = BIO_new_mem_buf(kp.data(), static_cast<int>(kp.size()));
      EVP_PKEY* key = PEM_read_bio_PrivateKey(kb, nullptr, nullptr, nullptr);
      BIO_free(kb);
      bool ok = cert && key && SSL_CTX_use_certificate(ctx, cert) == 1 && SSL_CTX_use_PrivateKey(ctx, key) == 1;
      if (cert) X509_free(cert);
      if (key) EVP_PKEY_free(key);
      if (!ok) throw std::runtime_error(ssl_error("loading client certificate data"));
    }
    SSL_CTX_set_verify(ctx, insecure ? SSL_VERIFY_NONE : SSL_VERIFY_PEER, nullptr);
  }
  ~TlsContext() {
    if (ctx) SSL_CTX_free(ctx);
  }
  SSL_CTX* ctx = nullptr;
  bool insecure = false;
};

std::shared_ptr<TlsContext> make_tls_context(const TlsOptions& o) {
  return o.enabled ? std::make_shared<TlsContext>(o) : nullptr;
}

std::string url_segment(std::string_view s) {
  static const char* hex = "0123456789ABCDEF";
  std::string out;
  out.reserve(s.size());
  for (unsigned char c : s) {
    if (std::isalnum(c) || c == '-' || c == '_' || c == '.' || c == '~') {
      out.push_back(static_cast<char>(c));
    } else {
      out.push_back('%');
      out.push_back(hex[c >> 4]);
      out.push_back(hex[c & 15]);
    }
  }
  return out;
}

HttpConn::HttpConn(const Endpoint& ep, std::shared_ptr<TlsContext> tls, bool streaming) : ep_(ep), tls_(std::move(tls)) {
  addrinfo hints{};
  hints.ai_family = AF_UNSPEC;
  hints.ai_socktype = SOCK_STREAM;
  addrinfo* res = nullptr;
  std::string port = std::to_string(ep.port);
  if (int rc = getaddrinfo(ep.host.c_str(), port.c_str(), &hints, &res); rc != 0)
    throw std::runtime_error("resolve " + ep.host + ": " + gai_strerror(rc));
  std::string err = "connect " + ep.host + ":" + port + " failed";
  for (addrinfo* a = res; a; a = a->ai_next) {
    int fd = ::socket(a->ai_family, a->ai_socktype | SOCK_CLOEXEC, a->ai_protocol);
    if (fd < 0) continue;
    timeval tv{ep.timeout_ms / 1000, (ep.timeout_ms % 1000) * 1000};
    setsockopt(fd, SOL_SOCKET, SO_SNDTIMEO, &tv, sizeof(tv));
    if (!streaming) {
      setsockopt(fd, SOL_SOCKET, SO_RCVTIMEO, &tv, sizeof(tv));
    } else {
      // A watch idles between events until the server's timeoutSeconds
      // (300 s) ends it. A half-open connection (API server host lost, an
      // idle-dropping load balancer) would block recv forever: TCP keepalive
      // probes find a dead peer within ~1 min, and a receive timeout above
      // the watch timeout ends the stream regardless, so the mirror re-watches.
      timeval rtv{kWatchRecvTimeoutS, 0};
      setsockopt(fd, SOL_SOCKET, SO_RCVTIMEO, &rtv, sizeof(rtv));
      int on = 1, idle = 30, intvl = 10, cnt = 3;
      setsockopt(fd, SOL_SOCKET, SO_KEEPALIVE, &on, sizeof(on));
      setsockopt(fd, IPPROTO_TCP, TCP_KEEPIDLE, &idle, sizeof(idle));
      setsockopt(fd, IPPROTO_TCP, TCP_KEEPINTVL, &intvl, sizeof(intvl));
      setsockopt(fd, IPPROTO_TCP, TCP_KEEPCNT, &cnt, sizeof(cnt));
    }
    if (::connect(fd, a->ai_addr, a->ai_addrlen) == 0) {
      int one = 1;
      setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));  // small keep-alive requests
      fd_ = fd;
      break;
    }
    err += std::string(": ") + std::strerror(errno);
    ::close(fd);
  }
  freeaddrinfo(res);
  if (fd_ < 0) throw std::runtime_error(err);
  if (tls_) {
    SSL* ssl = SSL_new(tls_->ctx);
    ssl_ = ssl;
    SSL_set_fd(ssl, fd_);
    if (!is_ip_literal(ep.host)) SSL_set_tlsext_host_name(ssl, ep.host.c_str());
    if (!tls_->insecure) {
      X509_VERIFY_PARAM* param = SSL_get0_param(ssl);
      if (is_ip_literal(ep.host))
        X509_VERIFY_PARAM_set1_ip_asc(param, ep.host.c_str());
      else
        X509_VERIFY_PARAM_set1_host(param, ep.host.c_str(), 0);
    }
    if (SSL_connect(ssl) != 1) {
      std::string e = ssl_error("TLS handshake with " + ep.host);
      SSL_free(ssl);
      ssl_ = nullptr;
      ::close(fd_);
      fd_ = -1;
      throw std::runtime_error(e);
    }
  }
}

HttpConn::~HttpConn() {
  if (ssl_) {
    SSL_shutdown(static_cast<SSL*>(ssl_));
    SSL_free(static_cast<SSL*>(ssl_));
  }
  if (fd_ >= 0) ::close(fd_);
}

void HttpConn::shutdown() {
  if (fd_ >= 0) ::shutdown(fd_, SHUT_RDWR);
}

void HttpConn::send_request(std::string_view method, std::string_view path, std::string_view body,
                            std::string_view content_type) {
  std::string req;
  req.reserve(256 + body.size());
  req.append(method).append(" ").append(path).append(" HTTP/1.1\r\nHost: ");
  req.append(ep_.host).append(":").append(std::to_string(ep_.port));
  req.append("\r\nAccept: application/json\r\nUser-Agent: xsched-native/1\r\n");
  if (!ep_.token.empty()) req.append("Authorization: Bearer ").append(ep_.token).append("\r\n");
  if (!body.empty()) {
    req.append("Content-Type: ").append(content_type).append("\r\nContent-Length: ");
    req.append(std::to_string(body.size())).append("\r\n");
  }
  req.append("\r\n").append(body);  // one write: headers and body in one segment
  size_t off = 0;
  while (off < req.size()) {
    ssize_t n;
    if (ssl_) {
      n = SSL_write(static_cast<SSL*>(ssl_), req.data() + off, static_cast<int>(req.size() - off));
    } else {
      n = ::send(fd_, req.data() + off, req.size() - off, MSG_NOSIGNAL);
    }
    if (n <= 0) {
      if (!ssl_ && n < 0 && errno == EINTR) continue;
      reusable_ = false;
      note_io_failure(n);
      throw std::runtime_error(std::string("send: ") + (ssl_ ? "TLS write failed" : std::strerror(errno)));
    }
    off += static_cast<size_t>(n);
  }
}

bool HttpConn::fill() {
  if (pos_ > 0 && pos_ == buf_.size()) {
    buf_.clear();
    pos_ = 0;
  } else if (pos_ > 65536) {
    buf_.erase(0, pos_);
    pos_ = 0;
  }
  char tmp[16384];
  for (;;) {
    ssize_t n;
    if (ssl_) {
      n = SSL_read(static_cast<SSL*>(ssl_), tmp, sizeof(tmp));
    } else {
      n = ::recv(fd_, tmp, sizeof(tmp), 0);
    }
    if (n > 0) {
      buf_.append(tmp, static_cast<size_t>(n));
      rx_bytes_ += static_cast<size_t>(n);
      return true;
    }
    if (!ssl_ && n < 0 && errno == EINTR) continue;
    reusable_ = false;
    note_io_failure(n);
    return false;
  }
}

void HttpConn::note_io_failure(ssize_t n) {
  const int e = errno;
  if (e == EAGAIN || e == EWOULDBLOCK || e == ETIMEDOUT)
    fail_ = Fail::kTimeout;  // SO_RCVTIMEO/SO_SNDTIMEO expired: the server may be working on it
  else if (e == ECONNRESET || e == EPIPE || e == ECONNABORTED)
    fail_ = Fail::kReset;
  else if (n == 0)
    fail_ = Fail::kEof;
  else
    fail_ = Fail::kOther;
}

bool HttpConn::read_line_raw(std::string& out) {
  for (;;) {
    size_t nl = buf_.find('\n', pos_);
    if (nl != std::string::npos) {
      size_t end = nl;
      if (end > pos_ && buf_[end - 1] == '\r') --end;
      out.assign(buf_, pos_, end - pos_);
      pos_ = nl + 1;
      return true;
    }
    if (!fill()) return false;
  }
}

bool HttpConn::read_exact(size_t n, std::string& out) {
  while (buf_.size() - pos_ < n)
    if (!fill()) return false;
  out.append(buf_, pos_, n);
  pos_ += n;
  return true;
}

int HttpConn::read_head(bool* chunked, int64_t* content_length) {
  std::string line;
  if (!read_line_raw(line)) throw std::runtime_error("connection closed before the response");
  // "HTTP/1.1 200 OK"
  size_t sp = line.find(' ');
  if (sp == std::string::npos || line.compare(0, 5, "HTTP/") != 0) {
    reusable_ = false;
    throw std::runtime_error("malformed status line: " + line.substr(0, 80));
  }
  int status = std::atoi(line.c_str() + sp + 1);
  *chunked = false;
  *content_length = -1;
  bool close = line.compare(0, 8, "HTTP/1.0") == 0;
  for (;;) {
    if (!read_line_raw(line)) throw std::runtime_error("connection closed in the response headers");
    if (line.empty()) break;
    size_t colon = line.find(':');
    if (colon == std::string::npos) continue;
    std::string_view name(line.data(), colon);
    std::string_view value = trim(std::string_view(line).substr(colon + 1));
    if (ieq(name, "Content-Length")) {
      *content_length = std::strtoll(std::string(value).c_str(), nullptr, 10);
    } else if (ieq(name, "Transfer-Encoding")) {
      *chunked = value.find("chunked") != std::string_view::npos;
    } else if (ieq(name, "Connection")) {
      if (ieq(value, "close")) close = true;
    }
  }
  if (close) reusable_ = false;
  return status;
}

bool HttpConn::read_chunked_body(std::string& out) {
  std::string line;
  for (;;) {
    if (!read_line_raw(line)) return false;
    size_t len = std::strtoull(line.c_str(), nullptr, 16);
    if (len == 0) {
      // trailers until an empty line
      do {
        if (!read_line_raw(line)) return false;
      } while (!line.empty());
      return true;
    }
    if (!read_exact(len, out)) return false;
    if (!read_line_raw(line)) return false;  // CRLF after the chunk
  }
}

Response HttpConn::roundtrip(std::string_view method, std::string_view path, std::string_view body,
                             std::string_view content_type) {
  fail_ = Fail::kNone;
  rx_bytes_ = 0;
  errno = 0;
  send_request(method, path, body, content_type);
  bool chunked;
  int64_t len;
  Response r;
  r.status = read_head(&chunked, &len);
  bool ok;
  if (chunked) {
    ok = read_chunked_body(r.body);
  } else if (len >= 0) {
    ok = read_exact(static_cast<size_t>(len), r.body);
  } else if (method == "HEAD" || r.status == 204 || r.status == 304) {
    ok = true;
  } else {  // body until the server closes
    reusable_ = false;
    while (fill()) {
    }
    r.body.assign(buf_, pos_, std::string::npos);
    pos_ = buf_.size();
    ok = true;
  }
  if (!ok) {
    reusable_ = false;
    throw std::runtime_error("connection closed in the response body");
  }
  return r;
}

int HttpConn::open_stream(std::string_view path) {
  send_request("GET", path, {}, {});
  bool chunked;
  int64_t len;
  int status = read_head(&chunked, &len);
  stream_chunked_ = chunked;
  stream_left_ = chunked ? -1 : len;
  pending_.clear();
  reusable_ = false;  // a watch connection ends with its stream
  return status;
}

bool HttpConn::next_chunk() {
  if (stream_chunked_) {
    std::string line;
    if (!read_line_raw(line)) return false;
    size_t len = std::strtoull(line.c_str(), nullptr, 16);
    if (len == 0) return false;  // end of stream
    if (!read_exact(len, pending_)) return false;
    return read_line_raw(line);
  }
  if (stream_left_ == 0) return false;
  if (pos_ == buf_.size() && !fill()) return false;
  size_t avail = buf_.size() - pos_;
  size_t take = stream_left_ < 0 ? avail : std::min<size_t>(avail, static_cast<size_t>(stream_left_));
  pending_.append(buf_, pos_, take);
  pos_ += take;
  if (stream_left_ > 0) stream_left_ -= static_cast<int64_t>(take);
  return true;
}

bool HttpConn::next_line(std::string& line) {
  for (;;) {
    size_t nl = pending_.find('\n');
    if (nl != std::string::npos) {
      line.assign(pending_, 0, nl);
      pending_.erase(0, nl + 1);
      if (!line.empty() && line.back() == '\r') line.pop_back();
      if (line.empty()) continue;
      return true;
    }
    if (!next_chunk()) {
      if (pending_.empty()) return false;
      line.swap(pending_);  // a final line without a newline
      pending_.clear();
      return true;
    }
  }
}

}  // namespace xsched::rest
