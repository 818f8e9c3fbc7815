#include "apiserver/apiserver.h"

#include <arpa/inet.h>
#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <poll.h>
#include <sys/socket.h>
#include <openssl/err.h>
#include <openssl/ssl.h>
#include <unistd.h>

#include <algorithm>
#include <cctype>
#include <cerrno>
#include <chrono>
#include <cstring>
#include <map>
#include <set>
#include <stdexcept>

#include "rest/kube.h"

namespace xsched::apiserver {

namespace {

// An HTTP error with a Kubernetes Status body.
struct ApiError : std::runtime_error {
  ApiError(int c, std::string r, const std::string& m) : std::runtime_error(m), code(c), reason(std::move(r)) {}
  int code;
  std::string reason;
};

const char* phrase(int code) {
  switch (code) {
    case 200: return "OK";
    case 201: return "Created";
    case 400: return "Bad Request";
    case 401: return "Unauthorized";
    case 403: return "Forbidden";
    case 404: return "Not Found";
    case 405: return "Method Not Allowed";
    case 409: return "Conflict";
    case 410: return "Gone";
    case 413: return "Payload Too Large";
    case 415: return "Unsupported Media Type";
    case 422: return "Unprocessable Entity";
    case 429: return "Too Many Requests";
    case 431: return "Request Header Fields Too Large";
    case 500: return "Internal Server Error";
    case 503: return "Service Unavailable";
    default: return code < 400 ? "OK" : "Error";
  }
}

Json status_obj(int code, const std::string& reason, const std::string& message) {
  Json s = Json::object();
  s.set("kind", Json("Status"));
  s.set("apiVersion", Json("v1"));
  s.set("metadata", Json::object());
  s.set("status", Json(code >= 400 ? "Failure" : "Success"));
  s.set("message", Json(message));
  s.set("reason", Json(reason));
  s.set("code", Json(code));
  return s;
}

int hexval(char c) {
  if (c >= '0' && c <= '9') return c - '0';
  if (c >= 'a' && c <= 'f') return c - 'a' + 10;
  if (c >= 'A' && c <= 'F') return c - 'A' + 10;
  return -1;
}

std::string pct_decode(std::string_view s, bool plus_space) {
  std::string out;
  out.reserve(s.size());
  for (size_t i = 0; i < s.size(); ++i) {
    char c = s[i];
    if (c == '%' && i + 2 < s.size()) {
      int hi = hexval(s[i + 1]), lo = hexval(s[i + 2]);
      if (hi >= 0 && lo >= 0) {
        out.push_back(static_cast<char>(hi * 16 + lo));
        i += 2;
        continue;
      }
    }
    out.push_back(plus_space && c == '+' ? ' ' : c);
  }
  return out;
}

std::string_view trim(std::string_view s) {
  while (!s.empty() && std::isspace(static_cast<unsigned char>(s.front()))) s.remove_prefix(1);
  while (!s.empty() && std::isspace(static_cast<unsigned char>(s.back()))) s.remove_suffix(1);
  return s;
}

std::string lower(std::string_view s) {
  std::string o(s);
  for (auto& c : o) c = static_cast<char>(std::tolower(static_cast<unsigned char>(c)));
  return o;
}

// "<prefix>/<plural>" -> store kind, from the REST client's table (rest/kube.cc).
const std::unordered_map<std::string, std::string>& routes() {
  static const auto* m = [] {
    auto* r = new std::unordered_map<std::string, std::string>();
    for (const auto& [kind, rp] : rest::resource_table()) (*r)[rp.prefix + "/" + kind] = kind;
    return r;
  }();
  return *m;
}

bool valid_key_char(char c) {
  return std::isalnum(static_cast<unsigned char>(c)) || c == '_' || c == '.' || c == '/' || c == '-';
}

std::string field_string(const Json& obj, std::string_view path) {
  const Json* cur = &obj;
  size_t i = 0;
  while (i <= path.size()) {
    size_t j = path.find('.', i);
    if (j == std::string_view::npos) j = path.size();
    if (!cur->is_object()) return "";
    cur = cur->get(path.substr(i, j - i));
    if (!cur) return "";
    i = j + 1;
  }
  switch (cur->type()) {
    case Json::Type::Null: return "";
    case Json::Type::String: return cur->as_string();
    case Json::Type::Bool: return cur->as_bool() ? "true" : "false";
    case Json::Type::Int: return std::to_string(cur->as_int());
    default: return cur->dump();
  }
}

std::vector<std::string> split_pointer(const std::string& ptr) {
  std::vector<std::string> out;
  if (ptr.empty()) return out;
  if (ptr[0] != '/') throw ApiError(422, "Invalid", "bad JSON pointer \"" + ptr + "\"");
  size_t i = 1;
  for (;;) {
    size_t j = ptr.find('/', i);
    std::string seg = ptr.substr(i, j == std::string::npos ? std::string::npos : j - i);
    std::string d;
    for (size_t k = 0; k < seg.size(); ++k) {
      if (seg[k] == '~' && k + 1 < seg.size() && (seg[k + 1] == '0' || seg[k + 1] == '1')) {
        d.push_back(seg[k + 1] == '0' ? '~' : '/');
        ++k;
      } else {
        d.push_back(seg[k]);
      }
    }
    out.push_back(std::move(d));
    if (j == std::string::npos) break;
    i = j + 1;
  }
  return out;
}

size_t array_index(const std::string& s, size_t limit) {
  if (s.empty() || s.size() > 9 || !std::all_of(s.begin(), s.end(), [](char c) { return std::isdigit(c); }))
    throw std::out_of_range("bad array index " + s);
  size_t i = std::stoul(s);
  if (i > limit) throw std::out_of_range("array index " + s + " out of range");
  return i;
}

Json* child(Json* cur, const std::string& seg) {
  if (cur->is_array()) {
    auto& a = cur->items_mut();
    size_t i = array_index(seg, a.empty() ? 0 : a.size() - 1);
    if (i >= a.size()) throw std::out_of_range("array index out of range");
    return &a[i];
  }
  if (cur->is_object()) {
    Json* n = cur->get_mut(seg);
    if (!n) throw std::out_of_range("missing member " + seg);
    return n;
  }
  throw std::out_of_range("cannot descend into a scalar at " + seg);
}

Json* walk(Json& doc, const std::vector<std::string>& parts, size_t n) {
  Json* cur = &doc;
  for (size_t i = 0; i < n; ++i) cur = child(cur, parts[i]);
  return cur;
}

}  // namespace

// ----------------------------------------------------------- selectors ----
std::vector<Requirement> parse_selector(std::string_view s) {
  std::vector<Requirement> out;
  std::vector<std::string_view> terms;
  int depth = 0;
  size_t start = 0;
  for (size_t i = 0; i <= s.size(); ++i) {
    char c = i < s.size() ? s[i] : ',';
    if (c == '(') ++depth;
    if (c == ')') --depth;
    if (c == ',' && depth <= 0) {
      auto t = trim(s.substr(start, i - start));
      if (!t.empty()) terms.push_back(t);
      start = i + 1;
    }
  }
  for (auto term : terms) {
    Requirement r;
    size_t p;
    if ((p = term.find("!=")) != std::string_view::npos) {
      r.op = Requirement::Ne;
      r.key = std::string(trim(term.substr(0, p)));
      r.values = {std::string(trim(term.substr(p + 2)))};
    } else if ((p = term.find("==")) != std::string_view::npos) {
      r.op = Requirement::Eq;
      r.key = std::string(trim(term.substr(0, p)));
      r.values = {std::string(trim(term.substr(p + 2)))};
    } else if ((p = term.find('=')) != std::string_view::npos && term.find('(') == std::string_view::npos) {
      r.op = Requirement::Eq;
      r.key = std::string(trim(term.substr(0, p)));
      r.values = {std::string(trim(term.substr(p + 1)))};
    } else {
      std::string_view t = term;
      bool neg = false;
      if (!t.empty() && t[0] == '!') {
        neg = true;
        t = trim(t.substr(1));
      }
      size_t k = 0;
      while (k < t.size() && valid_key_char(t[k])) ++k;
      r.key = std::string(t.substr(0, k));
      std::string_view rest = trim(t.substr(k));
      if (rest.empty()) {
        r.op = neg ? Requirement::NotExists : Requirement::Exists;
      } else {
        bool notin = rest.substr(0, 5) == "notin", in = !notin && rest.substr(0, 2) == "in";
        if (neg || (!notin && !in) || k == t.size() || !std::isspace(static_cast<unsigned char>(t[k])))
          throw std::invalid_argument("invalid selector term \"" + std::string(term) + "\"");
        rest = trim(rest.substr(notin ? 5 : 2));
        if (rest.size() < 2 || rest.front() != '(' || rest.back() != ')')
          throw std::invalid_argument("invalid selector term \"" + std::string(term) + "\"");
        r.op = notin ? Requirement::NotIn : Requirement::In;
        std::string_view vals = rest.substr(1, rest.size() - 2);
        size_t a = 0;
        for (size_t i = 0; i <= vals.size(); ++i) {
          if (i == vals.size() || vals[i] == ',') {
            auto v = trim(vals.substr(a, i - a));
            if (!v.empty()) r.values.emplace_back(v);
            a = i + 1;
          }
        }
      }
    }
    if (r.key.empty()) throw std::invalid_argument("invalid selector term \"" + std::string(term) + "\"");
    out.push_back(std::move(r));
  }
  return out;
}

bool labels_match(const std::vector<Requirement>& reqs, const Json& obj) {
  const Json& labels = obj["metadata"]["labels"];
  for (const auto& r : reqs) {
    const Json* v = labels.get(r.key);
    bool has = v != nullptr;
    const std::string& val = has ? v->as_string() : json_null().as_string();
    bool in_values = has && std::find(r.values.begin(), r.values.end(), val) != r.values.end();
    bool ok;
    switch (r.op) {
      case Requirement::Exists: ok = has; break;
      case Requirement::NotExists: ok = !has; break;
      case Requirement::Eq:
      case Requirement::In: ok = in_values; break;
      default: ok = !in_values; break;  // != / notin: true when the key is absent
    }
    if (!ok) return false;
  }
  return true;
}

bool fields_match(const std::vector<Requirement>& reqs, const Json& obj) {
  for (const auto& r : reqs) {
    if (r.op != Requirement::Eq && r.op != Requirement::Ne)
      throw std::invalid_argument("field selector supports only = and !=");
    bool eq = field_string(obj, r.key) == r.values.at(0);
    if (eq != (r.op == Requirement::Eq)) return false;
  }
  return true;
}

// ----------------------------------------------------------- json patch ---
Json apply_json_patch(const Json& in, const Json& ops) {
  Json doc = in;
  if (!ops.is_array()) throw ApiError(422, "Invalid", "json patch body must be an array");
  for (const auto& op0 : ops.items()) {
    Json op = op0;
    std::string kind = op["op"].as_string();
    try {
      auto parts = split_pointer(op["path"].as_string());
      if (kind == "test") {
        const Json* cur = walk(doc, parts, parts.size());
        if (*cur != op["value"]) throw ApiError(422, "Invalid", "test failed at " + op["path"].as_string());
        continue;
      }
      if (kind == "move" || kind == "copy") {
        auto src = split_pointer(op["from"].as_string());
        if (src.empty()) throw std::out_of_range("cannot move/copy the document root");
        Json* sp = walk(doc, src, src.size() - 1);
        Json val = *child(sp, src.back());
        if (kind == "move") {
          if (sp->is_array()) {
            auto& a = sp->items_mut();
            a.erase(a.begin() + static_cast<long>(array_index(src.back(), a.size() - 1)));
          } else {
            sp->erase(src.back());
          }
        }
        kind = "add";
        op = Json::object();
        op.set("value", std::move(val));
      }
      if (parts.empty()) {
        doc = op["value"];
        continue;
      }
      Json* par = walk(doc, parts, parts.size() - 1);
      const std::string& last = parts.back();
      if (kind == "add") {
        if (par->is_array()) {
          auto& a = par->items_mut();
          size_t i = last == "-" ? a.size() : array_index(last, a.size());
          a.insert(a.begin() + static_cast<long>(i), op["value"]);
        } else if (par->is_object()) {
          par->set(last, op["value"]);
        } else {
          throw std::out_of_range("parent is not a container");
        }
      } else if (kind == "remove") {
        if (par->is_array()) {
          auto& a = par->items_mut();
          if (a.empty()) throw std::out_of_range("remove from an empty array");
          a.erase(a.begin() + static_cast<long>(array_index(last, a.size() - 1)));
        } else if (!par->is_object() || !par->erase(last)) {
          throw std::out_of_range("missing member " + last);
        }
      } else if (kind == "replace") {
        *child(par, last) = op["value"];
      } else {
        throw ApiError(422, "Invalid", "unknown json-patch op \"" + kind + "\"");
      }
    } catch (const std::out_of_range& e) {
      throw ApiError(422, "Invalid", "json patch " + op0.dump() + ": " + e.what());
    }
  }
  return doc;
}

// ------------------------------------------------------------- server -----
struct Server::Request {
  std::string method, path;
  std::unordered_map<std::string, std::string> query;
  std::string content_type, authorization, body;
  bool keep_alive = true;
  std::string q(const char* k) const {
    auto it = query.find(k);
    return it == query.end() ? std::string() : it->second;
  }
};

struct Server::Conn {
  int fd = -1;
  SSL* ssl = nullptr;  // HTTPS: every read and write goes through it
  std::string buf;
  size_t pos = 0;

  bool fill() {
    if (pos > 0 && pos == buf.size()) {
      buf.clear();
      pos = 0;
    } else if (pos > (1u << 16)) {
      buf.erase(0, pos);
      pos = 0;
    }
    char tmp[65536];
    for (;;) {
      ssize_t n = ssl ? SSL_read(ssl, tmp, sizeof tmp) : ::recv(fd, tmp, sizeof tmp, 0);
      if (n > 0) {
        buf.append(tmp, static_cast<size_t>(n));
        return true;
      }
      if (!ssl && n < 0 && errno == EINTR) continue;
      return false;
    }
  }
  bool send_all(std::string_view d) {
    while (!d.empty()) {
      ssize_t n;
      if (ssl) {
        n = SSL_write(ssl, d.data(), static_cast<int>(std::min<size_t>(d.size(), 1u << 30)));
        if (n <= 0) return false;
      } else {
        n = ::send(fd, d.data(), d.size(), MSG_NOSIGNAL);
        if (n < 0) {
          if (errno == EINTR) continue;
          return false;
        }
      }
      d.remove_prefix(static_cast<size_t>(n));
    }
    return true;
  }
  // Reads through the next CRLF (or LF); false on EOF.
  bool line(std::string& out) {
    for (;;) {
      size_t e = buf.find('\n', pos);
      if (e != std::string::npos) {
        size_t end = e > pos && buf[e - 1] == '\r' ? e - 1 : e;
        out.assign(buf, pos, end - pos);
        pos = e + 1;
        return true;
      }
      if (buf.size() - pos > (1u << 20) || !fill()) return false;
    }
  }
  bool exact(size_t n, std::string& out) {
    while (buf.size() - pos < n)
      if (!fill()) return false;
    out.append(buf, pos, n);
    pos += n;
    return true;
  }
};

namespace {

constexpr size_t kMaxBody = 256u << 20;

// Chunk-size line of a chunked body: 1-15 hex digits, optionally followed by
// ";extensions". False for anything else (an overlong or non-hex size is a
// malformed request, not a huge allocation).
bool parse_chunk_size(const std::string& line, size_t* out) {
  size_t v = 0, i = 0;
  for (; i < line.size() && i < 16; ++i) {
    char ch = line[i];
    int d = ch >= '0' && ch <= '9'   ? ch - '0'
            : ch >= 'a' && ch <= 'f' ? ch - 'a' + 10
            : ch >= 'A' && ch <= 'F' ? ch - 'A' + 10
                                     : -1;
    if (d < 0) break;
    v = v * 16 + static_cast<size_t>(d);
  }
  if (i == 0 || i > 15) return false;
  if (i < line.size() && line[i] != ';' && line[i] != ' ' && line[i] != '\t') return false;
  *out = v;
  return true;
}

bool open_path(const std::string& path) {
  return path == "/healthz" || path == "/readyz" || path == "/livez" || path == "/version";
}

// 0: ok, -1: connection closed, >0: HTTP error to send before closing. With
// a bearer `token`, a request without it is refused (401) before its body is
// read: an unauthenticated client cannot make the server buffer 256 MiB.
int read_request(Server::Conn& c, Server::Request& r, const std::string& token) {
  r.query.clear();
  r.content_type.clear();
  r.authorization.clear();
  std::string line;
  do {
    if (!c.line(line)) return -1;
  } while (line.empty());  // tolerate stray CRLFs between requests
  size_t a = line.find(' '), b = line.rfind(' ');
  if (a == std::string::npos || b == a) return 400;
  r.method = line.substr(0, a);
  std::string target = line.substr(a + 1, b - a - 1);
  std::string version = line.substr(b + 1);
  r.keep_alive = version != "HTTP/1.0";
  int64_t content_length = -1;
  bool chunked = false;
  for (size_t n = 0;; ++n) {
    if (n > 200 || !c.line(line)) return n > 200 ? 431 : -1;
    if (line.empty()) break;
    size_t col = line.find(':');
    if (col == std::string::npos) continue;
    std::string name = lower(trim(std::string_view(line).substr(0, col)));
    std::string value(trim(std::string_view(line).substr(col + 1)));
    if (name == "content-length") content_length = std::strtoll(value.c_str(), nullptr, 10);
    else if (name == "transfer-encoding") chunked = lower(value).find("chunked") != std::string::npos;
    else if (name == "content-type") r.content_type = value;
    else if (name == "authorization") r.authorization = value;
    else if (name == "connection") {
      std::string v = lower(value);
      if (v.find("close") != std::string::npos) r.keep_alive = false;
      else if (v.find("keep-alive") != std::string::npos) r.keep_alive = true;
    }
  }
  size_t qm = target.find('?');
  r.path = pct_decode(std::string_view(target).substr(0, qm), false);
  if (qm != std::string::npos) {
    std::string_view qs = std::string_view(target).substr(qm + 1);
    size_t i = 0;
    while (i <= qs.size()) {
      size_t j = qs.find('&', i);
      if (j == std::string_view::npos) j = qs.size();
      std::string_view kv = qs.substr(i, j - i);
      if (!kv.empty()) {
        size_t eq = kv.find('=');
        r.query[pct_decode(kv.substr(0, eq), true)] = eq == std::string_view::npos ? "" : pct_decode(kv.substr(eq + 1), true);
      }
      i = j + 1;
    }
  }
  r.body.clear();
  if (!token.empty() && !open_path(r.path) && r.authorization != "Bearer " + token) return 401;
  if (chunked) {
    for (;;) {
      if (!c.line(line)) return -1;
      size_t sz = 0;
      if (!parse_chunk_size(line, &sz)) return 400;
      if (sz == 0) {
        do {
          if (!c.line(line)) return -1;
        } while (!line.empty());
        break;
      }
      if (sz > kMaxBody - r.body.size()) return 413;
      if (!c.exact(sz, r.body) || !c.line(line)) return -1;
    }
  } else if (content_length > 0) {
    if (static_cast<size_t>(content_length) > kMaxBody) return 413;
    if (!c.exact(static_cast<size_t>(content_length), r.body)) return -1;
  }
  return 0;
}

bool respond(Server::Conn& c, int code, std::string_view body, bool keep_alive,
             std::string_view ctype = "application/json") {
  std::string out;
  out.reserve(body.size() + 160);
  out += "HTTP/1.1 ";
  out += std::to_string(code);
  out += ' ';
  out += phrase(code);
  out += "\r\nContent-Type: ";
  out += ctype;
  out += "\r\nContent-Length: ";
  out += std::to_string(body.size());
  if (!keep_alive) out += "\r\nConnection: close";
  out += "\r\n\r\n";
  out += body;
  return c.send_all(out);
}

bool respond_json(Server::Conn& c, int code, const Json& j, bool keep_alive) {
  std::string s;
  j.dump_to(s);
  return respond(c, code, s, keep_alive);
}

bool write_chunk(Server::Conn& c, std::string_view data) {
  char head[24];
  int n = std::snprintf(head, sizeof head, "%zx\r\n", data.size());
  std::string out;
  out.reserve(data.size() + 32);
  out.append(head, static_cast<size_t>(n));
  out += data;
  out += "\r\n";
  return c.send_all(out);
}

Json parse_body(const std::string& body) {
  if (body.empty()) return Json();
  try {
    return Json::parse(body);
  } catch (const JsonError& e) {
    throw ApiError(400, "BadRequest", std::string("invalid JSON body: ") + e.what());
  }
}

void type_meta(Json& obj, const rest::ResourcePath& rp) {
  if (!obj.get("apiVersion") || !obj.get("kind")) {
    if (!obj.get("apiVersion")) obj.set("apiVersion", Json(rp.api_version));
    if (!obj.get("kind")) obj.set("kind", Json(rp.kind));
  }
}

// The client went away (watch streams only write when events arrive).
bool peer_closed(int fd) {
  pollfd p{fd, POLLIN | POLLRDHUP, 0};
  if (::poll(&p, 1, 0) <= 0) return false;
  if (p.revents & (POLLRDHUP | POLLHUP | POLLERR)) return true;
  char b;
  ssize_t n = ::recv(fd, &b, 1, MSG_PEEK | MSG_DONTWAIT);
  return n == 0;
}

}  // namespace

namespace {
std::string ssl_error() {
  unsigned long e = ERR_get_error();
  char buf[256];
  ERR_error_string_n(e, buf, sizeof buf);
  return buf;
}
}  // namespace

Server::Server(std::shared_ptr<ObjectStore> store, Options o) : store_(std::move(store)), opts_(std::move(o)) {
  if (!opts_.tls_cert_file.empty()) {
    SSL_CTX* ctx = SSL_CTX_new(TLS_server_method());
    if (!ctx) throw std::runtime_error("apiserver: SSL_CTX_new: " + ssl_error());
    SSL_CTX_set_min_proto_version(ctx, TLS1_2_VERSION);
    const std::string& key = opts_.tls_key_file.empty() ? opts_.tls_cert_file : opts_.tls_key_file;
    if (SSL_CTX_use_certificate_chain_file(ctx, opts_.tls_cert_file.c_str()) != 1 ||
        SSL_CTX_use_PrivateKey_file(ctx, key.c_str(), SSL_FILETYPE_PEM) != 1 || SSL_CTX_check_private_key(ctx) != 1) {
      std::string err = ssl_error();
      SSL_CTX_free(ctx);
      throw std::runtime_error("apiserver: TLS certificate/key: " + err);
    }
    if (!opts_.client_ca_file.empty()) {
      if (SSL_CTX_load_verify_locations(ctx, opts_.client_ca_file.c_str(), nullptr) != 1) {
        std::string err = ssl_error();
        SSL_CTX_free(ctx);
        throw std::runtime_error("apiserver: client CA: " + err);
      }
      SSL_CTX_set_verify(ctx, SSL_VERIFY_PEER | SSL_VERIFY_FAIL_IF_NO_PEER_CERT, nullptr);
    }
    tls_ctx_ = ctx;
  }
  addrinfo hints{}, *res = nullptr;
  hints.ai_family = AF_UNSPEC;
  hints.ai_socktype = SOCK_STREAM;
  hints.ai_flags = AI_PASSIVE | AI_NUMERICSERV;
  std::string port = std::to_string(opts_.port);
  const char* host = opts_.host.empty() || opts_.host == "0.0.0.0" ? nullptr : opts_.host.c_str();
  if (int e = ::getaddrinfo(host, port.c_str(), &hints, &res); e != 0)
    throw std::runtime_error(std::string("apiserver: resolve ") + opts_.host + ": " + gai_strerror(e));
  std::string err;
  for (addrinfo* ai = res; ai; ai = ai->ai_next) {
    int fd = ::socket(ai->ai_family, ai->ai_socktype | SOCK_CLOEXEC, ai->ai_protocol);
    if (fd < 0) continue;
    int one = 1;
    ::setsockopt(fd, SOL_SOCKET, SO_REUSEADDR, &one, sizeof one);
    if (::bind(fd, ai->ai_addr, ai->ai_addrlen) == 0 && ::listen(fd, 1024) == 0) {
      listen_fd_ = fd;
      sockaddr_storage ss{};
      socklen_t len = sizeof ss;
      ::getsockname(fd, reinterpret_cast<sockaddr*>(&ss), &len);
      port_ = ss.ss_family == AF_INET6 ? ntohs(reinterpret_cast<sockaddr_in6*>(&ss)->sin6_port)
                                       : ntohs(reinterpret_cast<sockaddr_in*>(&ss)->sin_port);
      break;
    }
    err = std::strerror(errno);
    ::close(fd);
  }
  ::freeaddrinfo(res);
  if (listen_fd_ < 0) {
    if (tls_ctx_) SSL_CTX_free(static_cast<SSL_CTX*>(tls_ctx_));
    tls_ctx_ = nullptr;
    throw std::runtime_error("apiserver: cannot listen on " + opts_.host + ":" + port + ": " + err);
  }
}

Server::~Server() {
  stop();
  if (tls_ctx_) SSL_CTX_free(static_cast<SSL_CTX*>(tls_ctx_));
}

void Server::start() {
  if (acceptor_.joinable() || stopping_) return;
  acceptor_ = std::thread([this] { accept_loop(); });
}

size_t Server::connections() const {
  std::lock_guard<std::mutex> g(mu_);
  return conns_.size();
}

void Server::accept_loop() {
  while (!stopping_.load()) {
    pollfd p{listen_fd_, POLLIN, 0};
    int r = ::poll(&p, 1, 100);
    if (r <= 0) continue;
    int fd = ::accept4(listen_fd_, nullptr, nullptr, SOCK_CLOEXEC);
    if (fd < 0) continue;
    int one = 1;
    ::setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof one);
    {
      std::lock_guard<std::mutex> g(mu_);
      if (stopping_ || conns_.size() >= static_cast<size_t>(opts_.max_connections)) {
        ::close(fd);
        continue;
      }
      conns_.insert(fd);
      ++live_threads_;
    }
    std::thread([this, fd] { serve(fd); }).detach();
  }
}

void Server::stop() {
  if (stopping_.exchange(true)) {
    // Second call (destructor after an explicit stop): nothing left to do.
    return;
  }
  if (acceptor_.joinable()) acceptor_.join();
  if (listen_fd_ >= 0) {
    ::close(listen_fd_);
    listen_fd_ = -1;
  }
  std::unique_lock<std::mutex> g(mu_);
  for (int fd : conns_) ::shutdown(fd, SHUT_RDWR);
  for (const auto& w : watchers_) w->stop();
  idle_cv_.wait_for(g, std::chrono::seconds(10), [this] { return live_threads_ == 0; });
}

void Server::serve(int fd) {
  Conn c;
  c.fd = fd;
  Request r;
  if (tls_ctx_) {
    c.ssl = SSL_new(static_cast<SSL_CTX*>(tls_ctx_));
    if (!c.ssl || SSL_set_fd(c.ssl, fd) != 1 || SSL_accept(c.ssl) != 1) {
      if (c.ssl) SSL_free(c.ssl);
      ERR_clear_error();
      ::close(fd);
      std::lock_guard<std::mutex> g(mu_);
      conns_.erase(fd);
      if (--live_threads_ == 0) idle_cv_.notify_all();
      return;
    }
  }
  for (;;) {
    int rc = read_request(c, r, opts_.token);
    if (rc < 0) break;
    if (rc > 0) {
      const char* reason = rc == 401 ? "Unauthorized" : rc == 413 ? "RequestEntityTooLarge" : "BadRequest";
      const char* msg = rc == 401 ? "Unauthorized" : rc == 413 ? "request body too large" : "malformed request";
      respond_json(c, rc, status_obj(rc, reason, msg), false);
      break;
    }
    if (!handle(c, r) || stopping_) break;
  }
  if (c.ssl) {
    SSL_shutdown(c.ssl);
    SSL_free(c.ssl);
    ERR_clear_error();
  }
  ::close(fd);
  std::lock_guard<std::mutex> g(mu_);
  conns_.erase(fd);
  if (--live_threads_ == 0) idle_cv_.notify_all();
}

bool Server::handle(Conn& c, Request& r) {
  requests_.fetch_add(1, std::memory_order_relaxed);
  const bool ka = r.keep_alive;
  try {
    const std::string& path = r.path;
    if (path == "/healthz" || path == "/readyz" || path == "/livez") return respond(c, 200, "ok", ka, "text/plain") && ka;
    if (path == "/version") {
      return respond(c, 200,
                     R"({"major":"1","minor":"23","gitVersion":"v1.23.3-xsched","platform":"linux/amd64"})", ka) &&
             ka;
    }
    if (!opts_.token.empty() && r.authorization != "Bearer " + opts_.token)
      throw ApiError(401, "Unauthorized", "Unauthorized");
    if (path == "/api") return respond(c, 200, R"({"kind":"APIVersions","versions":["v1"]})", ka) && ka;
    if (path == "/apis") {
      std::map<std::string, std::set<std::string>> groups;
      for (const auto& [kind, rp] : rest::resource_table()) {
        size_t s = rp.api_version.find('/');
        if (s != std::string::npos) groups[rp.api_version.substr(0, s)].insert(rp.api_version.substr(s + 1));
      }
      Json list = Json::array();
      for (const auto& [g, vs] : groups) {
        Json gj = Json::object();
        gj.set("name", Json(g));
        Json versions = Json::array();
        for (const auto& v : vs) {
          Json vj = Json::object();
          vj.set("groupVersion", Json(g + "/" + v));
          vj.set("version", Json(v));
          versions.push_back(std::move(vj));
        }
        gj.set("versions", std::move(versions));
        list.push_back(std::move(gj));
      }
      Json out = Json::object();
      out.set("kind", Json("APIGroupList"));
      out.set("apiVersion", Json("v1"));
      out.set("groups", std::move(list));
      return respond_json(c, 200, out, ka) && ka;
    }
    // /api/<v>/... or /apis/<g>/<v>/...
    std::vector<std::string> parts;
    for (size_t i = 0; i < path.size();) {
      size_t j = path.find('/', i);
      if (j == std::string::npos) j = path.size();
      if (j > i) parts.push_back(path.substr(i, j - i));
      i = j + 1;
    }
    std::string prefix;
    size_t rest = 0;
    if (parts.size() >= 2 && parts[0] == "api") {
      prefix = "/api/" + parts[1];
      rest = 2;
    } else if (parts.size() >= 3 && parts[0] == "apis") {
      prefix = "/apis/" + parts[1] + "/" + parts[2];
      rest = 3;
    } else {
      throw ApiError(404, "NotFound", "the server could not find the requested resource (" + path + ")");
    }
    std::string ns;
    if (parts.size() - rest > 2 && parts[rest] == "namespaces") {
      ns = parts[rest + 1];
      rest += 2;
    }
    auto rit = rest < parts.size() ? routes().find(prefix + "/" + parts[rest]) : routes().end();
    if (rit == routes().end())
      throw ApiError(404, "NotFound", "the server could not find the requested resource (" + path + ")");
    const std::string& kind = rit->second;
    const rest::ResourcePath& rp = rest::resource_path(kind);
    std::string name = parts.size() > rest + 1 ? parts[rest + 1] : "";
    std::string sub = parts.size() > rest + 2 ? parts[rest + 2] : "";

    if (r.method == "GET") {
      if (!name.empty()) {
        JsonPtr obj = store_->get(kind, ns, name);
        if (!obj) throw ApiError(404, "NotFound", kind + " \"" + name + "\" not found");
        return respond_json(c, 200, *obj, ka) && ka;
      }
      std::string w = r.q("watch");
      if (w == "true" || w == "1") {
        watch(c, kind, ns, r);
        return false;  // the stream ended; clients reconnect for the next watch
      }
      std::vector<Requirement> ls, fs;
      try {
        ls = parse_selector(r.q("labelSelector"));
        fs = parse_selector(r.q("fieldSelector"));
        for (const auto& q : fs)
          if (q.op != Requirement::Eq && q.op != Requirement::Ne)
            throw std::invalid_argument("field selector supports only = and !=");
      } catch (const std::invalid_argument& e) {
        throw ApiError(400, "BadRequest", e.what());
      }
      int64_t rv = 0;
      auto items = store_->list(kind, ns, &rv);
      std::string out;
      out.reserve(items.size() * 512 + 128);
      out += R"({"kind":")" + rp.kind + R"(List","apiVersion":")" + rp.api_version +
             R"(","metadata":{"resourceVersion":")" + std::to_string(rv) + R"("},"items":[)";
      bool first = true;
      for (const auto& it : items) {
        if ((!ls.empty() && !labels_match(ls, *it)) || (!fs.empty() && !fields_match(fs, *it))) continue;
        if (!first) out += ',';
        first = false;
        it->dump_to(out);
      }
      out += "]}";
      return respond(c, 200, out, ka) && ka;
    }
    if (r.method == "POST") {
      Json body = parse_body(r.body);
      if (!body.is_object()) throw ApiError(400, "BadRequest", "request body must be a JSON object");
      if (kind == "pods" && !name.empty() && sub == "binding") {
        std::string target = body["target"]["name"].as_string();
        if (target.empty()) throw ApiError(422, "Invalid", "Binding.target.name: Required value");
        const Json& md = body["metadata"];
        const Json& ann = md["annotations"];
        store_->bind(ns.empty() ? "default" : ns, name, md["uid"].as_string(), target,
                     ann.is_object() ? ann : Json::object());
        Json ok = status_obj(201, "", "");
        ok.set("status", Json("Success"));
        return respond_json(c, 201, ok, ka) && ka;
      }
      if (!name.empty()) throw ApiError(405, "MethodNotAllowed", "POST to a named resource");
      if (rp.namespaced) {
        Json& md = body.at_or_create("metadata");
        if (!ns.empty()) {
          const Json* cur = md.get("namespace");
          if (cur && cur->is_string() && cur->as_string() != ns)
            throw ApiError(400, "BadRequest", "the namespace of the object does not match the request");
          md.set("namespace", Json(ns));
        }
      }
      type_meta(body, rp);
      return respond_json(c, 201, *store_->create(kind, std::move(body)), ka) && ka;
    }
    if (r.method == "PUT") {
      Json body = parse_body(r.body);
      if (!body.is_object()) throw ApiError(400, "BadRequest", "request body must be a JSON object");
      Json& md = body.at_or_create("metadata");
      const Json* n = md.get("name");
      if (n && n->is_string() && n->as_string() != name)
        throw ApiError(400, "BadRequest", "the name of the object does not match the request");
      md.set("name", Json(name));
      if (rp.namespaced) {
        std::string mns = ns.empty() ? md["namespace"].str_or("") : ns;
        md.set("namespace", Json(mns.empty() ? "default" : mns));
      }
      type_meta(body, rp);
      return respond_json(c, 200, *store_->update(kind, std::move(body), true), ka) && ka;
    }
    if (r.method == "PATCH") {
      std::string ct(trim(std::string_view(r.content_type).substr(0, r.content_type.find(';'))));
      if (ct.empty()) ct = "application/merge-patch+json";
      Json body = parse_body(r.body);
      if (ct == "application/json-patch+json") {
        JsonPtr cur = store_->get(kind, ns, name);
        if (!cur) throw ApiError(404, "NotFound", kind + " \"" + name + "\" not found");
        return respond_json(c, 200, *store_->update(kind, apply_json_patch(*cur, body), true), ka) && ka;
      }
      if (ct != "application/merge-patch+json" && ct != "application/strategic-merge-patch+json" &&
          ct != "application/apply-patch+yaml" && ct != "application/json")
        throw ApiError(415, "UnsupportedMediaType", "unsupported patch type " + ct);
      if (!body.is_object()) throw ApiError(400, "BadRequest", "merge patch body must be an object");
      return respond_json(c, 200, *store_->patch(kind, ns, name, body), ka) && ka;
    }
    if (r.method == "DELETE") {
      if (name.empty()) {
        size_t n = store_->delete_all(kind, ns);
        Json ok = status_obj(200, "", "deleted " + std::to_string(n));
        ok.set("status", Json("Success"));
        return respond_json(c, 200, ok, ka) && ka;
      }
      Json opts = parse_body(r.body);
      int64_t grace = 0;
      if (opts["gracePeriodSeconds"].is_number()) grace = opts["gracePeriodSeconds"].as_int();
      else if (!r.q("gracePeriodSeconds").empty()) grace = std::strtoll(r.q("gracePeriodSeconds").c_str(), nullptr, 10);
      std::string uid = opts["preconditions"]["uid"].as_string();
      JsonPtr old = store_->remove(kind, ns, name, grace, uid);
      return (old ? respond_json(c, 200, *old, ka) : respond(c, 200, "{}", ka)) && ka;
    }
    throw ApiError(405, "MethodNotAllowed", "method " + r.method + " not allowed");
  } catch (const ApiError& e) {
    return respond_json(c, e.code, status_obj(e.code, e.reason, e.what()), ka) && ka;
  } catch (const StoreError& e) {
    return respond_json(c, e.code(), status_obj(e.code(), e.reason(), e.what()), ka) && ka;
  } catch (const JsonError& e) {
    return respond_json(c, 400, status_obj(400, "BadRequest", e.what()), ka) && ka;
  } catch (const std::exception& e) {
    return respond_json(c, 500, status_obj(500, "InternalError", e.what()), ka) && ka;
  }
}

void Server::watch(Conn& c, const std::string& kind, const std::string& ns, Request& r) {
  const rest::ResourcePath& rp = rest::resource_path(kind);
  std::vector<Requirement> ls, fs;
  try {
    ls = parse_selector(r.q("labelSelector"));
    fs = parse_selector(r.q("fieldSelector"));
  } catch (const std::invalid_argument& e) {
    respond_json(c, 400, status_obj(400, "BadRequest", e.what()), false);
    return;
  }
  auto match = [&](const Json& o) {
    return (ls.empty() || labels_match(ls, o)) && (fs.empty() || fields_match(fs, o));
  };
  std::string rvp = r.q("resourceVersion");
  int64_t since = rvp.empty() || rvp == "0" ? 0 : std::strtoll(rvp.c_str(), nullptr, 10);
  double timeout_s = std::strtod(r.q("timeoutSeconds").c_str(), nullptr);
  std::string bm = r.q("allowWatchBookmarks");
  bool bookmarks = bm == "true" || bm == "1";

  WatcherPtr w;
  std::string expired;
  try {
    w = store_->watch({kind}, ns, since);
  } catch (const StoreError& e) {
    if (e.code() != 410) throw;
    expired = e.what();
  }
  if (w) {
    std::lock_guard<std::mutex> g(mu_);
    watchers_.insert(w);
    if (stopping_) w->stop();
  }
  struct Unregister {
    Server* s;
    WatcherPtr w;
    ~Unregister() {
      if (!w) return;
      s->store_->unwatch(w);
      std::lock_guard<std::mutex> g(s->mu_);
      s->watchers_.erase(w);
    }
  } unregister{this, w};

  if (!c.send_all("HTTP/1.1 200 OK\r\nContent-Type: application/json\r\nTransfer-Encoding: chunked\r\n\r\n")) return;
  if (!expired.empty()) {
    Json ev = Json::object();
    ev.set("type", Json("ERROR"));
    ev.set("object", status_obj(410, "Expired", expired));
    write_chunk(c, ev.dump() + "\n") && write_chunk(c, "");
    return;
  }
  int64_t floor = 0;
  if (since == 0) {
    auto items = store_->list(kind, ns, &floor);
    std::string out;
    for (const auto& it : items) {
      if (!match(*it)) continue;
      out += R"({"type":"ADDED","object":)";
      it->dump_to(out);
      out += "}\n";
      if (out.size() > (1u << 20)) {
        if (!write_chunk(c, out)) return;
        out.clear();
      }
    }
    if (!out.empty() && !write_chunk(c, out)) return;
  }
  using clock = std::chrono::steady_clock;
  auto deadline = timeout_s > 0 ? clock::now() + std::chrono::microseconds(static_cast<int64_t>(timeout_s * 1e6))
                                : clock::time_point::max();
  int64_t last_rv = floor;
  auto last_beat = clock::now();
  while (!stopping_ && !w->stopped()) {
    if (clock::now() >= deadline) break;
    auto evs = w->next(500, 1024);
    if (evs.empty()) {
      if (peer_closed(c.fd)) return;
      if (bookmarks && clock::now() - last_beat >= std::chrono::milliseconds(opts_.bookmark_interval_ms)) {
        std::string b = R"({"type":"BOOKMARK","object":{"kind":")" + rp.kind + R"(","apiVersion":")" + rp.api_version +
                        R"(","metadata":{"resourceVersion":")" + std::to_string(last_rv) + "\"}}}\n";
        if (!write_chunk(c, b)) return;
        last_beat = clock::now();
      }
      continue;
    }
    std::string out;
    for (const auto& ev : evs) {
      if (ev.rv <= floor || !ev.obj) continue;
      last_rv = ev.rv;
      if (!match(*ev.obj)) continue;
      out += R"({"type":")";
      out += event_type_name(ev.type);
      out += R"(","object":)";
      if (ev.type == EventType::Deleted) {
        Json o = *ev.obj;
        o.at_or_create("metadata").set("resourceVersion", Json(std::to_string(ev.rv)));
        o.dump_to(out);
      } else {
        ev.obj->dump_to(out);
      }
      out += "}\n";
    }
    if (!out.empty() && !write_chunk(c, out)) return;
    last_beat = clock::now();
  }
  write_chunk(c, "");
}

}  // namespace xsched::apiserver
